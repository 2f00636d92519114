// Replica mean-reduce and the fused DiLoCo outer step: HBM-streaming kernels
// over [K, ld] replica sets.  Roofline: HBM.
//
// Both kernels walk the arena in 4-element vectors (16 B per lane for f32,
// 8 B for bf16); workgroup b owns the contiguous vectors [b*kChunk,
// (b+1)*kChunk) (measured on MI355X: 5.1 TB/s for the K=8 DiLoCo stream vs
// 4.7 TB/s with a grid-stride loop; a plain float4 copy peaks at 5.2-5.5 TB/s
// on the same box, tools/ubench_stream.hip); every stream is loaded and stored
// non-temporally (stream_load / stream_store: 1.93 -> 1.88 ms for the K = 8 step
// on one box, profiles/r02z_ab_stream_nt.txt).  Each lane issues the K replica loads
// of one vector back to back (the k loop is unrolled so the loads are in
// flight together) and sums them in ascending k, so the result does not
// depend on the launch geometry.  dst may alias src (in-place average): each
// lane reads every replica of its vector before it writes any, and no two
// lanes touch the same vector, so the sources carry no __restrict__.
#include "ga_common.h"

namespace ga {

constexpr int kBlock = 256;
constexpr int64_t kChunk = 1024;  // vectors (or scalars) per workgroup

__device__ __forceinline__ void chunk_range(int64_t total, int64_t& lo, int64_t& hi) {
    lo = (int64_t)blockIdx.x * kChunk;
    hi = lo + kChunk < total ? lo + kChunk : total;
}

inline int chunk_grid(int64_t total) {
    const int64_t g = ceil_div(total, kChunk);
    return (int)(g < 1 ? 1 : g);
}

template <typename T>
__device__ __forceinline__ const T* replica_ptr(const T* base, const int32_t* rows, int64_t k,
                                                int64_t ld) {
    const int64_t r = rows ? (int64_t)rows[k] : k;
    return base + r * ld;
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kBlock) void replica_mean_kernel(
    const T* src, int64_t K, int64_t ld_src, const int32_t* __restrict__ rows,
    int64_t n, float divisor, T* dst, int64_t K_out, int64_t ld_dst) {
    const bool divide = divisor != 1.0f;
    int64_t lo, hi;
    if constexpr (VEC) {
        using V = typename Vec4<T>::type;
        chunk_range(n >> 2, lo, hi);
        for (int64_t v = lo + threadIdx.x; v < hi; v += kBlock) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
            for (int64_t k = 0; k < K; ++k) {
                const V raw = stream_load(reinterpret_cast<const V*>(replica_ptr(src, rows, k, ld_src)) + v);
                float f[4];
                Vec4<T>::unpack(raw, f);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] += f[e];
            }
            if (divide) {
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] = acc[e] / divisor;
            }
            const V out = Vec4<T>::pack(acc);
            for (int64_t j = 0; j < K_out; ++j) stream_store(reinterpret_cast<V*>(dst + j * ld_dst) + v, out);
        }
    } else {
        chunk_range(n, lo, hi);
        for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
            float acc = 0.f;
#pragma unroll 4
            for (int64_t k = 0; k < K; ++k) acc += Elem<T>::load(replica_ptr(src, rows, k, ld_src) + i);
            if (divide) acc = acc / divisor;
            for (int64_t j = 0; j < K_out; ++j) Elem<T>::store(dst + j * ld_dst + i, acc);
        }
    }
}

// One element of the DiLoCo outer update; mirrors torch.optim.SGD's
// single-tensor path (torch/optim/sgd.py) on the pseudo-gradient.
struct OuterParams {
    float divisor, lr, momentum, dampening, weight_decay;
    int first_step, nesterov;
};

__device__ __forceinline__ float outer_update(float sum, float& master, float& buf,
                                              const OuterParams& op) {
    const float avg = sum / op.divisor;
    float g = master - avg;
    if (op.weight_decay != 0.f) g = fmaf(op.weight_decay, master, g);
    if (op.momentum != 0.f) {
        if (op.first_step) buf = g;
        else buf = fmaf(1.f - op.dampening, g, buf * op.momentum);
        g = op.nesterov ? fmaf(op.momentum, buf, g) : buf;
    }
    master = fmaf(-op.lr, g, master);
    return master;
}

template <typename T, typename M, bool VEC>
__global__ __launch_bounds__(kBlock) void diloco_outer_kernel(
    const T* src, int64_t K, int64_t ld_src, int64_t n, M* master, M* mom,
    OuterParams op, T* dst, int64_t K_out, int64_t ld_dst) {
    const bool has_mom = op.momentum != 0.f;
    int64_t lo, hi;
    if constexpr (VEC) {
        using V = typename Vec4<T>::type;
        using VM = typename Vec4<M>::type;
        chunk_range(n >> 2, lo, hi);
        for (int64_t v = lo + threadIdx.x; v < hi; v += kBlock) {
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
            for (int64_t k = 0; k < K; ++k) {
                float f[4];
                Vec4<T>::unpack(stream_load(reinterpret_cast<const V*>(src + k * ld_src) + v), f);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] += f[e];
            }
            float m[4], b[4] = {0.f, 0.f, 0.f, 0.f};
            Vec4<M>::unpack(stream_load(reinterpret_cast<const VM*>(master) + v), m);
            if (has_mom && !op.first_step) Vec4<M>::unpack(stream_load(reinterpret_cast<const VM*>(mom) + v), b);
            float out[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) out[e] = outer_update(acc[e], m[e], b[e], op);
            const V o = Vec4<T>::pack(out);
            // device-scope (sc1) stores based at the workgroup's block of each stream
            const uint32_t i = (uint32_t)(v - lo);
            store_sc1(reinterpret_cast<VM*>(master) + lo, i, Vec4<M>::pack(m));
            if (has_mom) store_sc1(reinterpret_cast<VM*>(mom) + lo, i, Vec4<M>::pack(b));
            for (int64_t j = 0; j < K_out; ++j) store_sc1(reinterpret_cast<V*>(dst + j * ld_dst) + lo, i, o);
        }
    } else {
        chunk_range(n, lo, hi);
        for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
            float acc = 0.f;
#pragma unroll 4
            for (int64_t k = 0; k < K; ++k) acc += Elem<T>::load(src + k * ld_src + i);
            float m = Elem<M>::load(master + i);
            float b = (has_mom && !op.first_step) ? Elem<M>::load(mom + i) : 0.f;
            const float out = outer_update(acc, m, b, op);
            Elem<M>::store(master + i, m);
            if (has_mom) Elem<M>::store(mom + i, b);
            for (int64_t j = 0; j < K_out; ++j) Elem<T>::store(dst + j * ld_dst + i, out);
        }
    }
}

// Placement probe of the fused outer step (no reference counterpart): the exact
// access pattern of diloco_outer_kernel<float, float, true> -- workgroup b's block
// of K replica streams, master and momentum read, the same blocks written through
// the same stores -- with every value written back unchanged, so a caller can time
// candidate master/momentum buffers against a live replica set without side
// effects.  K <= kProbeK (the replicas are held in registers to be written back).
constexpr int kProbeK = 16;
__global__ __launch_bounds__(kBlock) void diloco_probe_kernel(float* src, int64_t K, int64_t ld_src, int64_t n,
                                                              float* master, float* mom) {
    int64_t lo, hi;
    chunk_range(n >> 2, lo, hi);
    for (int64_t v = lo + threadIdx.x; v < hi; v += kBlock) {
        float4 x[kProbeK];
#pragma unroll
        for (int k = 0; k < kProbeK; ++k)
            if (k < K) x[k] = stream_load(reinterpret_cast<const float4*>(src + k * ld_src) + v);
        const float4 m = stream_load(reinterpret_cast<const float4*>(master) + v);
        const float4 b = stream_load(reinterpret_cast<const float4*>(mom) + v);
        const uint32_t i = (uint32_t)(v - lo);
        store_sc1(reinterpret_cast<float4*>(master) + lo, i, m);
        store_sc1(reinterpret_cast<float4*>(mom) + lo, i, b);
#pragma unroll
        for (int k = 0; k < kProbeK; ++k)
            if (k < K) store_sc1(reinterpret_cast<float4*>(src + k * ld_src) + lo, i, x[k]);
    }
}

// Placement probe of the in-place replica mean (no reference counterpart): the access
// pattern of replica_mean_kernel<float, true> with dst == src -- workgroup b's block of
// the K replica streams loaded, then stored back non-temporally -- with every value
// written back unchanged.  K <= kProbeK.
__global__ __launch_bounds__(kBlock) void mean_probe_kernel(float* src, int64_t K, int64_t ld_src, int64_t n) {
    int64_t lo, hi;
    chunk_range(n >> 2, lo, hi);
    for (int64_t v = lo + threadIdx.x; v < hi; v += kBlock) {
        float4 x[kProbeK];
#pragma unroll
        for (int k = 0; k < kProbeK; ++k)
            if (k < K) x[k] = stream_load(reinterpret_cast<const float4*>(src + k * ld_src) + v);
#pragma unroll
        for (int k = 0; k < kProbeK; ++k)
            if (k < K) stream_store(reinterpret_cast<float4*>(src + k * ld_src) + v, x[k]);
    }
}

static bool aligned(const void* p, int bytes) { return p == nullptr || ((uintptr_t)p % bytes) == 0; }

template <typename T>
static int launch_replica_mean(const void* src, int64_t K, int64_t ld_src, const int32_t* rows,
                               int64_t n, float divisor, void* dst, int64_t K_out,
                               int64_t ld_dst, hipStream_t stream) {
    const int vb = 4 * (int)sizeof(T);
    const bool vec = (n % 4 == 0) && (ld_src % 4 == 0) && (ld_dst % 4 == 0) &&
                     aligned(src, vb) && aligned(dst, vb);
    if (vec) {
        hipLaunchKernelGGL((replica_mean_kernel<T, true>), dim3(chunk_grid(n / 4)),
                           dim3(kBlock), 0, stream, (const T*)src, K, ld_src, rows, n, divisor,
                           (T*)dst, K_out, ld_dst);
    } else {
        hipLaunchKernelGGL((replica_mean_kernel<T, false>), dim3(chunk_grid(n)),
                           dim3(kBlock), 0, stream, (const T*)src, K, ld_src, rows, n, divisor,
                           (T*)dst, K_out, ld_dst);
    }
    return check_launch("ga_replica_mean");
}

template <typename T, typename M>
static int launch_diloco(const void* src, int64_t K, int64_t ld_src, int64_t n, void* master,
                         void* mom, const OuterParams& op, void* dst, int64_t K_out,
                         int64_t ld_dst, hipStream_t stream) {
    const int vb = 4 * (int)sizeof(T);
    const int vm = 4 * (int)sizeof(M);
    const bool vec = (n % 4 == 0) && (ld_src % 4 == 0) && (ld_dst % 4 == 0) &&
                     aligned(src, vb) && aligned(dst, vb) && aligned(master, vm) &&
                     aligned(mom, vm);
    if (vec) {
        hipLaunchKernelGGL((diloco_outer_kernel<T, M, true>), dim3(chunk_grid(n / 4)),
                           dim3(kBlock), 0, stream, (const T*)src, K, ld_src, n, (M*)master,
                           (M*)mom, op, (T*)dst, K_out, ld_dst);
    } else {
        hipLaunchKernelGGL((diloco_outer_kernel<T, M, false>), dim3(chunk_grid(n)),
                           dim3(kBlock), 0, stream, (const T*)src, K, ld_src, n, (M*)master,
                           (M*)mom, op, (T*)dst, K_out, ld_dst);
    }
    return check_launch("ga_diloco_outer");
}

}  // namespace ga

using namespace ga;

extern "C" GA_API int ga_replica_mean(int dtype, const void* src, int64_t K, int64_t ld_src,
                                      const int32_t* rows, int64_t n, float divisor, void* dst,
                                      int64_t K_out, int64_t ld_dst, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && K >= 1 && K_out >= 0, "ga_replica_mean: bad sizes n=%lld K=%lld K_out=%lld",
               (long long)n, (long long)K, (long long)K_out);
    if (n == 0 || K_out == 0) return GA_OK;
    GA_REQUIRE(src && dst, "ga_replica_mean: null buffer");
    GA_REQUIRE(K == 1 || rows || ld_src >= n, "ga_replica_mean: ld_src %lld < n %lld", (long long)ld_src,
               (long long)n);
    GA_REQUIRE(K_out == 1 || ld_dst >= n, "ga_replica_mean: ld_dst %lld < n %lld", (long long)ld_dst,
               (long long)n);
    GA_REQUIRE(divisor != 0.0f, "ga_replica_mean: divisor is 0");
    switch (dtype) {
        case GA_F32:
            return launch_replica_mean<float>(src, K, ld_src, rows, n, divisor, dst, K_out, ld_dst, stream);
        case GA_BF16:
            return launch_replica_mean<__hip_bfloat16>(src, K, ld_src, rows, n, divisor, dst, K_out,
                                                       ld_dst, stream);
        default:
            set_error("ga_replica_mean: unknown dtype %d", dtype);
            return GA_EINVAL;
    }
}

extern "C" GA_API int ga_diloco_outer(int dtype, const void* src, int64_t K, int64_t ld_src,
                                      int64_t n, float divisor, void* master, void* mom,
                                      int master_f32, int first_step, float lr, float momentum,
                                      float dampening, float weight_decay, int nesterov,
                                      void* dst, int64_t K_out, int64_t ld_dst,
                                      hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && K >= 1 && K_out >= 0, "ga_diloco_outer: bad sizes n=%lld K=%lld K_out=%lld",
               (long long)n, (long long)K, (long long)K_out);
    if (n == 0) return GA_OK;
    GA_REQUIRE(src && master, "ga_diloco_outer: null src/master");
    GA_REQUIRE(K_out == 0 || dst, "ga_diloco_outer: null dst");
    GA_REQUIRE(momentum == 0.0f || mom, "ga_diloco_outer: momentum != 0 needs a momentum buffer");
    GA_REQUIRE(K == 1 || ld_src >= n, "ga_diloco_outer: ld_src < n");
    GA_REQUIRE(K_out <= 1 || ld_dst >= n, "ga_diloco_outer: ld_dst < n");
    GA_REQUIRE(divisor != 0.0f, "ga_diloco_outer: divisor is 0");
    GA_REQUIRE(!(nesterov && (momentum <= 0.0f || dampening != 0.0f)),
               "ga_diloco_outer: Nesterov momentum requires a momentum and zero dampening");
    OuterParams op{divisor, lr, momentum, dampening, weight_decay, first_step ? 1 : 0, nesterov ? 1 : 0};
    if (momentum == 0.0f) mom = nullptr;
    switch (dtype) {
        case GA_F32:
            return launch_diloco<float, float>(src, K, ld_src, n, master, mom, op, dst, K_out, ld_dst,
                                               stream);
        case GA_BF16:
            if (master_f32)
                return launch_diloco<__hip_bfloat16, float>(src, K, ld_src, n, master, mom, op, dst,
                                                            K_out, ld_dst, stream);
            return launch_diloco<__hip_bfloat16, __hip_bfloat16>(src, K, ld_src, n, master, mom, op,
                                                                 dst, K_out, ld_dst, stream);
        default:
            set_error("ga_diloco_outer: unknown dtype %d", dtype);
            return GA_EINVAL;
    }
}

extern "C" GA_API int ga_probe_diloco_placement(float* src, int64_t K, int64_t ld_src, int64_t n, float* master,
                                                float* mom, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && n % 4 == 0 && K >= 1 && K <= kProbeK, "ga_probe_diloco_placement: bad sizes n=%lld K=%lld "
               "(n a multiple of 4, K <= %d)", (long long)n, (long long)K, kProbeK);
    if (n == 0) return GA_OK;
    GA_REQUIRE(src && master && mom, "ga_probe_diloco_placement: null buffer");
    GA_REQUIRE(K == 1 || (ld_src >= n && ld_src % 4 == 0), "ga_probe_diloco_placement: bad ld_src");
    GA_REQUIRE(aligned(src, 16) && aligned(master, 16) && aligned(mom, 16), "ga_probe_diloco_placement: alignment");
    hipLaunchKernelGGL(diloco_probe_kernel, dim3(chunk_grid(n / 4)), dim3(kBlock), 0, stream, src, K, ld_src, n,
                       master, mom);
    return check_launch("ga_probe_diloco_placement");
}

extern "C" GA_API int ga_probe_mean_placement(float* src, int64_t K, int64_t ld_src, int64_t n, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && n % 4 == 0 && K >= 1 && K <= kProbeK, "ga_probe_mean_placement: bad sizes n=%lld K=%lld "
               "(n a multiple of 4, K <= %d)", (long long)n, (long long)K, kProbeK);
    if (n == 0) return GA_OK;
    GA_REQUIRE(src != nullptr, "ga_probe_mean_placement: null buffer");
    GA_REQUIRE(K == 1 || (ld_src >= n && ld_src % 4 == 0), "ga_probe_mean_placement: bad ld_src");
    GA_REQUIRE(aligned(src, 16), "ga_probe_mean_placement: alignment");
    hipLaunchKernelGGL(mean_probe_kernel, dim3(chunk_grid(n / 4)), dim3(kBlock), 0, stream, src, K, ld_src, n);
    return check_launch("ga_probe_mean_placement");
}
