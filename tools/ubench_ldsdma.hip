// Does an LDS-DMA read path (global_load_lds_dwordx4) stream HBM faster than
// register loads on MI355X, for the HBM-bound kernels of this repo (DiLoCo outer
// step, replica mean, AdamW)?  Standalone diagnostic, one GPU:
//   copy_reg   : 4 float4 nt loads per lane, then 4 nt stores (ga_stream_copy's shape)
//   copy_glds  : the same bytes, each wave's 4 KiB read by 4 global_load_lds_dwordx4 (aux
//                nt) into its own LDS slice, waited, read back to registers, nt stores
//   read_reg / read_glds : the read halves alone (sums kept by a never-taken store)
//   dl_reg / dl_glds     : the DiLoCo K = 8 pattern (10 read streams, 10 write streams)
// Each kernel moves every byte once; HIP-event mean over 10 launches after 2 warm-ups,
// three interleaved rounds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ntl(const f4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void nts(f4* p, f4 v) { __builtin_nontemporal_store(v, p); }

// one wave's 4 x 1 KiB from src (lane-linear) into its LDS slice
__device__ __forceinline__ void glds4(const f4* src, f4* slice, int lane) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + u * 64 + lane),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<uintptr_t>(slice + u * 64)),
                                         16, 0, 2);
}

__global__ __launch_bounds__(256) void copy_reg(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    const long base = (long)blockIdx.x * 1024 + threadIdx.x;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ntl(src + base + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) nts(dst + base + u * 256, v[u]);
}

__global__ __launch_bounds__(256) void copy_glds(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    __shared__ f4 buf[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long base = (long)blockIdx.x * 1024 + (long)w * 256;  // this wave's 4 KiB
    glds4(src + base, buf[w], lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = buf[w][u * 64 + lane];
#pragma unroll
    for (int u = 0; u < 4; ++u) nts(dst + base + u * 64 + lane, v[u]);
}

__global__ __launch_bounds__(256) void read_reg(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    const long base = (long)blockIdx.x * 1024 + threadIdx.x;
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) a += ntl(src + base + u * 256);
    if (a.x == 1234.5f) dst[0] = a;
}

__global__ __launch_bounds__(256) void read_glds(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    __shared__ f4 buf[4][256];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long base = (long)blockIdx.x * 1024 + (long)w * 256;
    glds4(src + base, buf[w], lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) a += buf[w][u * 64 + lane];
    if (a.x == 1234.5f) dst[0] = a;
}

// store policies: write-only streams and copies with mixed load/store hints
template <int ST>  // 0 plain, 1 nt, 2 sc0 sc1 (system scope write-through), 3 sc1
__device__ __forceinline__ void st(f4* p, f4 v) {
    if (ST == 0) *p = v;
    else if (ST == 1) nts(p, v);
    else if (ST == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
}
template <int ST>
__global__ __launch_bounds__(256) void write_only(f4* __restrict__ dst, long nvec) {
    const long base = (long)blockIdx.x * 1024 + threadIdx.x;
    const f4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
#pragma unroll
    for (int u = 0; u < 4; ++u) st<ST>(dst + base + u * 256, v);
}
template <int LDNT, int ST>
__global__ __launch_bounds__(256) void copy_mix(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    const long base = (long)blockIdx.x * 1024 + threadIdx.x;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = LDNT ? ntl(src + base + u * 256) : src[base + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u) st<ST>(dst + base + u * 256, v[u]);
}

// DiLoCo K = 8 shape: rows r[0..7] at stride ld, plus master m and momentum b; every
// vector: sum the 8 rows, update m and b, write m, b and the 8 rows (in place)
constexpr int K = 8;
__device__ __forceinline__ void dl_update(const f4* r, f4& m, f4& b, f4& out) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) acc += r[k];
    const f4 g = m - acc / 8.f;
    b = 0.9f * b + g;
    m = m - 0.7f * (g + 0.9f * b);
    out = m;
}

__global__ __launch_bounds__(256) void dl_reg(f4* __restrict__ reps, long ld, f4* __restrict__ mst, f4* __restrict__ mom,
                                              long nvec) {
    const long lo = (long)blockIdx.x * 1024;
    for (long v = lo + threadIdx.x; v < lo + 1024; v += 256) {
        f4 r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = ntl(reps + k * ld + v);
        f4 m = ntl(mst + v), b = ntl(mom + v), o;
        dl_update(r, m, b, o);
        nts(mst + v, m);
        nts(mom + v, b);
#pragma unroll
        for (int k = 0; k < K; ++k) nts(reps + k * ld + v, o);
    }
}

// the same, each wave's 10 streams x 1 KiB per step read by LDS-DMA into a 10 KiB slice
__global__ __launch_bounds__(256) void dl_glds(f4* __restrict__ reps, long ld, f4* __restrict__ mst, f4* __restrict__ mom,
                                               long nvec) {
    __shared__ f4 buf[4][K + 2][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long lo = (long)blockIdx.x * 1024;
    for (long v0 = lo + w * 64; v0 < lo + 1024; v0 += 256) {
#pragma unroll
        for (int k = 0; k < K + 2; ++k) {
            const f4* s = k < K ? reps + k * ld + v0 : (k == K ? mst + v0 : mom + v0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(s + lane),
                                             reinterpret_cast<__attribute__((address_space(3))) void*>(
                                                 reinterpret_cast<uintptr_t>(&buf[w][k][0])),
                                             16, 0, 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        f4 r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = buf[w][k][lane];
        f4 m = buf[w][K][lane], b = buf[w][K + 1][lane], o;
        dl_update(r, m, b, o);
        const long v = v0 + lane;
        nts(mst + v, m);
        nts(mom + v, b);
#pragma unroll
        for (int k = 0; k < K; ++k) nts(reps + k * ld + v, o);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slice reads done before the next DMA
    }
}

// sc1 (device-scope) stores through buffer_store_dwordx4 (__builtin_amdgcn_raw_buffer_store_b128,
// aux = 16), the workgroup's block as the descriptor base
__device__ __forceinline__ void st_sc1(f4* base, int idx, f4 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, idx * 16, 0, 16);
}
__global__ __launch_bounds__(256) void copy_buf_sc1(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    const long blk = (long)blockIdx.x * 1024;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ntl(src + blk + threadIdx.x + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) st_sc1(dst + blk, threadIdx.x + u * 256, v[u]);
}
template <int ST>  // 0 plain, 1 nt, 16 sc1 (buffer store)
__global__ __launch_bounds__(256) void dl_st(f4* __restrict__ reps, long ld, f4* __restrict__ mst, f4* __restrict__ mom,
                                             long nvec) {
    const long lo = (long)blockIdx.x * 1024;
    for (int i = threadIdx.x; i < 1024; i += 256) {
        const long v = lo + i;
        f4 r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = ntl(reps + k * ld + v);
        f4 m = ntl(mst + v), b = ntl(mom + v), o;
        dl_update(r, m, b, o);
        if (ST == 16) {
            st_sc1(mst + lo, i, m);
            st_sc1(mom + lo, i, b);
#pragma unroll
            for (int k = 0; k < K; ++k) st_sc1(reps + k * ld + lo, i, o);
        } else {
            st<ST>(mst + v, m);
            st<ST>(mom + v, b);
#pragma unroll
            for (int k = 0; k < K; ++k) st<ST>(reps + k * ld + v, o);
        }
    }
}

template <typename F> float time_ms(F f, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}

int main() {
    const long nvec = 1L << 28;  // 4 GiB per buffer (in float4)
    f4 *a, *b;
    CK(hipMalloc(&a, 16 * nvec)); CK(hipMalloc(&b, 16 * nvec));
    CK(hipMemset(a, 0, 16 * nvec)); CK(hipMemset(b, 0, 16 * nvec));
    const int grid = (int)(nvec / 1024);
    // DiLoCo arena: GPT-2 124M = 124,475,904 floats -> 31,118,976 float4 per row, rounded to 1024
    const long n4 = 31118976L / 1024 * 1024, ld = n4;
    f4 *reps, *mst, *mom;
    CK(hipMalloc(&reps, 16 * ld * K)); CK(hipMalloc(&mst, 16 * n4)); CK(hipMalloc(&mom, 16 * n4));
    CK(hipMemset(reps, 0, 16 * ld * K)); CK(hipMemset(mst, 0, 16 * n4)); CK(hipMemset(mom, 0, 16 * n4));
    const double dlb = (2.0 * K + 4) * 16 * n4;
    for (int r = 0; r < 3; ++r) {
        float t;
        t = time_ms([&] { copy_reg<<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy_reg   %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_glds<<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy_glds  %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { read_reg<<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d read_reg   %.3f ms %.0f GB/s\n", r, t, 16.0 * nvec / t / 1e6);
        t = time_ms([&] { read_glds<<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d read_glds  %.3f ms %.0f GB/s\n", r, t, 16.0 * nvec / t / 1e6);
        t = time_ms([&] { write_only<0><<<grid, 256>>>(b, nvec); }, 10);
        printf("round %d write_plain %.3f ms %.0f GB/s\n", r, t, 16.0 * nvec / t / 1e6);
        t = time_ms([&] { write_only<1><<<grid, 256>>>(b, nvec); }, 10);
        printf("round %d write_nt    %.3f ms %.0f GB/s\n", r, t, 16.0 * nvec / t / 1e6);
        t = time_ms([&] { write_only<2><<<grid, 256>>>(b, nvec); }, 10);
        printf("round %d write_sc01  %.3f ms %.0f GB/s\n", r, t, 16.0 * nvec / t / 1e6);
        t = time_ms([&] { write_only<3><<<grid, 256>>>(b, nvec); }, 10);
        printf("round %d write_sc1   %.3f ms %.0f GB/s\n", r, t, 16.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_mix<0, 0><<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy ld- st-   %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_mix<1, 0><<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy ldnt st-  %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_mix<0, 1><<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy ld- stnt  %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_mix<1, 2><<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy ldnt sc01 %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_mix<1, 3><<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy ldnt sc1  %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { copy_buf_sc1<<<grid, 256>>>(a, b, nvec); }, 10);
        printf("round %d copy ldnt bufsc1 %.3f ms %.0f GB/s\n", r, t, 32.0 * nvec / t / 1e6);
        t = time_ms([&] { dl_st<0><<<(int)(n4 / 1024), 256>>>(reps, ld, mst, mom, n4); }, 10);
        printf("round %d dl st plain %.3f ms %.0f GB/s\n", r, t, dlb / t / 1e6);
        t = time_ms([&] { dl_st<16><<<(int)(n4 / 1024), 256>>>(reps, ld, mst, mom, n4); }, 10);
        printf("round %d dl st bufsc1 %.3f ms %.0f GB/s\n", r, t, dlb / t / 1e6);
        t = time_ms([&] { dl_reg<<<(int)(n4 / 1024), 256>>>(reps, ld, mst, mom, n4); }, 10);
        printf("round %d dl_reg     %.3f ms %.0f GB/s\n", r, t, dlb / t / 1e6);
        t = time_ms([&] { dl_glds<<<(int)(n4 / 1024), 256>>>(reps, ld, mst, mom, n4); }, 10);
        printf("round %d dl_glds    %.3f ms %.0f GB/s\n", r, t, dlb / t / 1e6);
    }
    return 0;
}
