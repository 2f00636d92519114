// Inner optimizer on the flat arena: fused Adam/AdamW step and gradient-norm
// clipping, one streaming pass each instead of torch's ~10 multi-tensor passes
// (torch/optim/adam.py _multi_tensor_adam) behind the reference's
// `clip_grad_norm_` + `self.optim.step()` (strategy.py:135-140,
// communicate_optimize_strategy.py:69-73, diloco.py:52-59).  Roofline: HBM.
//
// Per element (f32 arena, f32 state), in torch's op order:
//   g  = grad * clip_coef                       (clip_grad_norm_, if clipping)
//   p *= 1 - lr*wd                              (AdamW: decoupled decay)   | g += wd*p (Adam: L2)
//   m  = lerp(m, g, 1-b1)                       (torch's lerp: m + w*(g-m) for w < 0.5)
//   v  = b2*v + (1-b2)*g*g
//   p += step_size * m / (sqrt(v)/bc2_sqrt + eps),  step_size = -lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t)
// 28 bytes per element (read p, g, m, v; write p, m, v), +4 when the clipped
// gradient is written back.
#include "ga_common.h"
#include "adam_math.h"


namespace ga {

constexpr int kOptBlock = 256;
constexpr int64_t kOptChunk = 1024;  // float4 vectors per workgroup
constexpr int kSumsqBlocks = 1024;   // partials of the norm reduction

__global__ __launch_bounds__(kOptBlock) void adam_kernel(float* __restrict__ param, float* __restrict__ grad,
                                                         float* __restrict__ m_, float* __restrict__ v_, int64_t n,
                                                         int64_t ld, AdamParams ap,
                                                         const float* __restrict__ clip_coef) {
    const int64_t rep = blockIdx.y;  // replica (simulated node) of a [K, ld] set
    param += rep * ld;
    grad += rep * ld;
    m_ += rep * ld;
    v_ += rep * ld;
    const float coef = clip_coef ? clip_coef[2 * rep] : 1.f;
    const bool scale = coef < 1.f;
    const int64_t nv = n >> 2;
    const int64_t lo = (int64_t)blockIdx.x * kOptChunk;
    const int64_t hi = lo + kOptChunk < nv ? lo + kOptChunk : nv;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kOptBlock) {
        float4 p = stream_load(reinterpret_cast<const float4*>(param) + i);
        float4 g = stream_load(reinterpret_cast<const float4*>(grad) + i);
        float4 m = stream_load(reinterpret_cast<const float4*>(m_) + i);
        float4 v = stream_load(reinterpret_cast<const float4*>(v_) + i);
        if (scale) {
            g.x *= coef; g.y *= coef; g.z *= coef; g.w *= coef;
            stream_store(reinterpret_cast<float4*>(grad) + i, g);  // clip_grad_norm_ leaves the clipped grads
        }
        float gg[4] = {g.x, g.y, g.z, g.w};
        float pp[4] = {p.x, p.y, p.z, p.w}, mm[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) adam_elem(pp[e], gg[e], mm[e], vv[e], ap);
        const uint32_t o = (uint32_t)(i - lo);
        store_sc1(reinterpret_cast<float4*>(param) + lo, o, make_float4(pp[0], pp[1], pp[2], pp[3]));
        store_sc1(reinterpret_cast<float4*>(m_) + lo, o, make_float4(mm[0], mm[1], mm[2], mm[3]));
        store_sc1(reinterpret_cast<float4*>(v_) + lo, o, make_float4(vv[0], vv[1], vv[2], vv[3]));
    }
    // scalar tail (n % 4), handled by the last workgroup
    if (blockIdx.x == gridDim.x - 1) {
        for (int64_t j = (nv << 2) + threadIdx.x; j < n; j += kOptBlock) {
            float p = param[j], g = grad[j], m = m_[j], v = v_[j];
            if (scale) {
                g *= coef;
                grad[j] = g;
            }
            adam_elem(p, g, m, v, ap);
            param[j] = p;
            m_[j] = m;
            v_[j] = v;
        }
    }
}

// Placement probe of adam_kernel (no reference counterpart): its exact access pattern
// (replicas on grid.y, 1024 float4 per workgroup, p, g, m, v read, p, m, v written
// through the same stores) with every value written back unchanged, so ArenaAdam can
// time candidate physical buffers for the moments without side effects.
__global__ __launch_bounds__(kOptBlock) void adam_probe_kernel(float* __restrict__ param,
                                                               const float* __restrict__ grad,
                                                               float* __restrict__ m_, float* __restrict__ v_,
                                                               int64_t n, int64_t ld) {
    const int64_t rep = blockIdx.y;
    param += rep * ld;
    grad += rep * ld;
    m_ += rep * ld;
    v_ += rep * ld;
    const int64_t nv = n >> 2;
    const int64_t lo = (int64_t)blockIdx.x * kOptChunk;
    const int64_t hi = lo + kOptChunk < nv ? lo + kOptChunk : nv;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kOptBlock) {
        const float4 p = stream_load(reinterpret_cast<const float4*>(param) + i);
        const float4 g = stream_load(reinterpret_cast<const float4*>(grad) + i);
        const float4 m = stream_load(reinterpret_cast<const float4*>(m_) + i);
        const float4 v = stream_load(reinterpret_cast<const float4*>(v_) + i);
        const uint32_t o = (uint32_t)(i - lo);
        asm volatile("" ::"v"(g.x), "v"(g.y), "v"(g.z), "v"(g.w));  // the grad load stays live
        store_sc1(reinterpret_cast<float4*>(param) + lo, o, p);
        store_sc1(reinterpret_cast<float4*>(m_) + lo, o, m);
        store_sc1(reinterpret_cast<float4*>(v_) + lo, o, v);
    }
}

// partials[b] = sum of x^2 over a grid-stride share of the arena (fp32, fixed order)
template <typename T>
__global__ __launch_bounds__(kOptBlock) void sumsq_kernel(const T* __restrict__ x, int64_t n, int64_t ld,
                                                          float* __restrict__ partials) {
    __shared__ float red[kOptBlock / 64];
    x += (int64_t)blockIdx.y * ld;
    partials += (int64_t)blockIdx.y * gridDim.x;
    float acc = 0.f;
    const int64_t stride = (int64_t)gridDim.x * kOptBlock;
    const int64_t nv = ((uintptr_t)x % (4 * sizeof(T)) == 0) ? n / 4 : 0;  // 4-element vectors
    using V = typename Vec4<T>::type;
    for (int64_t i = (int64_t)blockIdx.x * kOptBlock + threadIdx.x; i < nv; i += stride) {
        float f[4];
        Vec4<T>::unpack(stream_load(reinterpret_cast<const V*>(x) + i), f);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = fmaf(f[e], f[e], acc);
    }
    for (int64_t i = 4 * nv + (int64_t)blockIdx.x * kOptBlock + threadIdx.x; i < n; i += stride) {
        const float f = Elem<T>::load(x + i);
        acc = fmaf(f, f, acc);
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) acc += __shfl_down(acc, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out[0] = min(1, max_norm / (sqrt(sum partials) + 1e-6)), out[1] = the total norm
// (torch.nn.utils.clip_grad_norm_ with norm_type 2)
__global__ __launch_bounds__(kOptBlock) void clip_coef_kernel(const float* __restrict__ partials, int np,
                                                              float max_norm, float* __restrict__ out) {
    __shared__ float red[kOptBlock / 64];
    partials += (int64_t)blockIdx.x * np;  // one workgroup per replica
    out += 2 * (int64_t)blockIdx.x;
    float acc = 0.f;
    for (int i = threadIdx.x; i < np; i += kOptBlock) acc += partials[i];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) acc += __shfl_down(acc, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float total = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
        const float c = max_norm / (total + 1e-6f);
        out[0] = c < 1.f ? c : 1.f;
        out[1] = total;
    }
}

}  // namespace ga

using namespace ga;

extern "C" GA_API int ga_sumsq_partials_count(void) { return kSumsqBlocks; }

extern "C" GA_API int ga_grad_clip_coef(int dtype, const void* grad, int64_t K, int64_t ld, int64_t n,
                                        float max_norm, float* partials, float* out, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && K >= 1 && K <= 65535, "ga_grad_clip_coef: bad sizes n=%lld K=%lld", (long long)n,
               (long long)K);
    GA_REQUIRE(K == 1 || ld >= n, "ga_grad_clip_coef: ld < n");
    GA_REQUIRE(grad && partials && out, "ga_grad_clip_coef: null buffer");
    GA_REQUIRE(max_norm > 0.f, "ga_grad_clip_coef: max_norm must be > 0");
    const int blocks = kSumsqBlocks;
    switch (dtype) {
        case GA_F32:
            hipLaunchKernelGGL(sumsq_kernel<float>, dim3(blocks, (unsigned)K), dim3(kOptBlock), 0, stream,
                               (const float*)grad, n, ld, partials);
            break;
        case GA_BF16:
            hipLaunchKernelGGL(sumsq_kernel<__hip_bfloat16>, dim3(blocks, (unsigned)K), dim3(kOptBlock), 0, stream,
                               (const __hip_bfloat16*)grad, n, ld, partials);
            break;
        default: set_error("ga_grad_clip_coef: unknown dtype %d", dtype); return GA_EINVAL;
    }
    if (int e = check_launch("ga_grad_clip_coef (sumsq)")) return e;
    hipLaunchKernelGGL(clip_coef_kernel, dim3((unsigned)K), dim3(kOptBlock), 0, stream, partials, blocks, max_norm,
                       out);
    return check_launch("ga_grad_clip_coef");
}

extern "C" GA_API int ga_adam_step(int dtype, void* param, void* grad, float* exp_avg, float* exp_avg_sq, int64_t K,
                                   int64_t ld, int64_t n, float lerp_w, float beta2, float one_m_beta2, float eps,
                                   float wd_factor, float l2_wd, float step_size, float bc2_sqrt,
                                   const float* clip_coef, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && K >= 1 && K <= 65535, "ga_adam_step: bad sizes n=%lld K=%lld", (long long)n, (long long)K);
    if (n == 0) return GA_OK;
    GA_REQUIRE(K == 1 || (ld >= n && ld % 4 == 0), "ga_adam_step: ld must be >= n and a multiple of 4");
    GA_REQUIRE(param && grad && exp_avg && exp_avg_sq, "ga_adam_step: null buffer");
    GA_REQUIRE(dtype == GA_F32, "ga_adam_step: only float32 arenas are fused (dtype %d)", dtype);
    GA_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
               "ga_adam_step: buffers must be 16-byte aligned");
    GA_REQUIRE(bc2_sqrt > 0.f, "ga_adam_step: bc2_sqrt must be > 0");
    const AdamParams ap{lerp_w, beta2, one_m_beta2, eps, wd_factor, l2_wd, step_size, bc2_sqrt};
    const int64_t nv = n / 4;
    int64_t grid = (nv + kOptChunk - 1) / kOptChunk;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)grid, (unsigned)K), dim3(kOptBlock), 0, stream, (float*)param,
                       (float*)grad, exp_avg, exp_avg_sq, n, ld, ap, clip_coef);
    return check_launch("ga_adam_step");
}

extern "C" GA_API int ga_probe_adam_placement(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                              int64_t K, int64_t ld, int64_t n, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && n % 4 == 0 && K >= 1 && K <= 65535, "ga_probe_adam_placement: bad sizes n=%lld K=%lld",
               (long long)n, (long long)K);
    if (n == 0) return GA_OK;
    GA_REQUIRE(K == 1 || (ld >= n && ld % 4 == 0), "ga_probe_adam_placement: ld must be >= n and a multiple of 4");
    GA_REQUIRE(param && grad && exp_avg && exp_avg_sq, "ga_probe_adam_placement: null buffer");
    GA_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
               "ga_probe_adam_placement: buffers must be 16-byte aligned");
    int64_t grid = (n / 4 + kOptChunk - 1) / kOptChunk;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(adam_probe_kernel, dim3((unsigned)grid, (unsigned)K), dim3(kOptBlock), 0, stream, param, grad,
                       exp_avg, exp_avg_sq, n, ld);
    return check_launch("ga_probe_adam_placement");
}
