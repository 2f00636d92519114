// Would a 3-waves-per-SIMD DeMo encode that RE-READS delta and grad for its
// residual (no x tile kept: 8 KB of LDS per wave instead of 16.6 KB, ~161 VGPRs)
// beat today's 2-waves-per-SIMD kernel that keeps x in LDS?  Standalone
// diagnostic (round 5): the encode's memory pattern (64x64 chunks, one wave per
// chunk, coalesced 4-row loads of delta and grad, a delta store) with its
// compute emulated -- a dependent MFMA phase standing in for the two DCT
// products (NMF v_mfma_f32_32x32x2_f32 in 4 chains, chained on the loaded
// values), then a VALU phase standing in for the top-k (NV dependent fmaf per
// lane) -- at 2 waves per SIMD (8-wave workgroups, LDS-capped as today) and at
// 3 (4-wave workgroups, 3 per CU), the latter optionally re-loading delta and
// grad before the store.  GPT-2 350M sized arrays.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned coal(int i, int lane, int stride) {
    return (unsigned)(((lane >> 4) + 4 * i) * stride + 4 * (lane & 15));
}

// WAVES per workgroup; LDSB bytes of LDS per workgroup (occupancy cap); RELOAD: load
// delta and grad a second time before the store (the x tile not kept)
template <int WAVES, int LDSB, int NMF, int NV, bool RELOAD, bool HALVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(WAVES == 4 ? 3 : 2, WAVES == 4 ? 3 : 2)))
void enc_kernel(float* __restrict__ delta, const float* __restrict__ grad,
                                                         int R, int C, long njobs, float* sink) {
    __shared__ float pad[LDSB / 4];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gx = C / 64;
    const long stride = (long)gridDim.x * WAVES;
    float keep = 0.f;
    for (long job = (long)blockIdx.x * WAVES + wid; job < njobs; job += stride) {
        const int cy = (int)(job / gx), cx = (int)(job - (long)cy * gx);
        const long base = (long)cy * 64 * C + (long)cx * 64;
        f32x16 acc[4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
        float4 X[16];
        if (HALVES) {  // rows 0-31 then 32-63 (64 VGPRs of loads in flight at a time)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float4 D[8], G[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) D[i] = *reinterpret_cast<const float4*>(delta + base + coal(8 * h + i, lane, C));
#pragma unroll
                for (int i = 0; i < 8; ++i) G[i] = *reinterpret_cast<const float4*>(grad + base + coal(8 * h + i, lane, C));
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    X[8 * h + i].x = fmaf(1e-3f, G[i].x, D[i].x * 0.999f);
                    X[8 * h + i].y = fmaf(1e-3f, G[i].y, D[i].y * 0.999f);
                    X[8 * h + i].z = fmaf(1e-3f, G[i].z, D[i].z * 0.999f);
                    X[8 * h + i].w = fmaf(1e-3f, G[i].w, D[i].w * 0.999f);
                }
                // the half's row product (half of the first phase's MFMAs)
#pragma unroll
                for (int t = 0; t < NMF / 4; ++t) {
                    const float4 v = X[8 * h + (t & 7)];
                    acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.y, acc[t & 3], 0, 0, 0);
                }
            }
        } else {
            float4 D[16], G[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) D[i] = *reinterpret_cast<const float4*>(delta + base + coal(i, lane, C));
#pragma unroll
            for (int i = 0; i < 16; ++i) G[i] = *reinterpret_cast<const float4*>(grad + base + coal(i, lane, C));
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                X[i].x = fmaf(1e-3f, G[i].x, D[i].x * 0.999f);
                X[i].y = fmaf(1e-3f, G[i].y, D[i].y * 0.999f);
                X[i].z = fmaf(1e-3f, G[i].z, D[i].z * 0.999f);
                X[i].w = fmaf(1e-3f, G[i].w, D[i].w * 0.999f);
            }
#pragma unroll
            for (int t = 0; t < NMF / 2; ++t) {
                const float4 v = X[t & 15];
                acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.y, acc[t & 3], 0, 0, 0);
            }
        }
        // the x tile (today's kernel keeps it in LDS) -- here its share of LDS traffic
        if (!RELOAD) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                reinterpret_cast<float4*>(pad)[(wid * 1024 + i * 64 + lane) % (LDSB / 16)] = X[i];
        }
        // the column product: chained on the first
#pragma unroll
        for (int t = 0; t < NMF / 2; ++t) acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(acc[(t + 1) & 3][t & 15], acc[(t + 2) & 3][(t + 5) & 15], acc[t & 3], 0, 0, 0);
        // the top-k's VALU: a dependent chain per lane on the coefficients
        float v = acc[0][lane & 15] + acc[1][3] + acc[2][7] + acc[3][11];
#pragma unroll 16
        for (int s = 0; s < NV; ++s) v = fmaf(v, 0.999f, acc[s & 3][s & 15]);
        keep += v;
        if (RELOAD) {  // x again, from delta and grad (still unchanged in memory)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float4 D[8], G[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) D[i] = *reinterpret_cast<const float4*>(delta + base + coal(8 * h + i, lane, C));
#pragma unroll
                for (int i = 0; i < 8; ++i) G[i] = *reinterpret_cast<const float4*>(grad + base + coal(8 * h + i, lane, C));
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    float4 o;
                    o.x = fmaf(1e-3f, G[i].x, D[i].x * 0.999f) - v * 1e-30f;
                    o.y = fmaf(1e-3f, G[i].y, D[i].y * 0.999f);
                    o.z = fmaf(1e-3f, G[i].z, D[i].z * 0.999f);
                    o.w = fmaf(1e-3f, G[i].w, D[i].w * 0.999f);
                    *reinterpret_cast<float4*>(delta + base + coal(8 * h + i, lane, C)) = o;
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float4 o = reinterpret_cast<float4*>(pad)[(wid * 1024 + i * 64 + lane) % (LDSB / 16)];
                o.x -= v * 1e-30f;
                *reinterpret_cast<float4*>(delta + base + coal(i, lane, C)) = o;
            }
        }
    }
    if (keep == 1234.5f) sink[0] = keep;
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <typename K>
int occ(K k, int threads) {
    int n = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, threads, 0));
    return n;
}

int main() {
    const long N = 354871296L;  // GPT-2 350M
    float *d, *g, *sink;
    CK(hipMalloc(&d, 4 * N)); CK(hipMalloc(&g, 4 * N)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(d, 0, 4 * N)); CK(hipMemset(g, 0, 4 * N));
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int C = 1024, R = (int)(N / C / 64 * 64);
    const long nj = (long)(R / 64) * (C / 64);
    const double b = 12.0 * R * (double)C;
#define RUN(W, LDSB, NMF, NV, RL, HV, what) { auto k = enc_kernel<W, LDSB, NMF, NV, RL, HV>; const int per = occ(k, 64 * W); \
    for (int rep = 0; rep < 2; ++rep) { float ms = time_ms([&] { k<<<cus * per, 64 * W>>>(d, g, R, C, nj, sink); }, 10); \
    printf("%-34s waves/blk %2d blk/CU %d (%d waves/SIMD) mfma %3d valu %4d: %.3f ms  %.0f GB/s (12 B/elem)\n", what, W, per, W * per / 4, NMF, NV, ms, b / ms / 1e6); } }
    for (int NV : {0, 1}) {
        (void)NV;
    }
    // memory only
    RUN(8, 150000, 0, 0, false, false, "2 waves/SIMD, x kept, no compute")
    RUN(4, 50000, 0, 0, true, true, "3 waves/SIMD, reload, no compute")
    RUN(4, 50000, 0, 0, false, true, "3 waves/SIMD, x kept, no compute")
    // with the encode's compute stood in for
    RUN(8, 150000, 128, 500, false, false, "2 waves/SIMD, x kept, compute")
    RUN(8, 150000, 128, 500, false, true, "2 waves/SIMD, x kept, halves")
    RUN(4, 50000, 128, 500, true, true, "3 waves/SIMD, reload, compute")
    RUN(4, 50000, 128, 500, false, true, "3 waves/SIMD, x kept*, compute")
    RUN(8, 150000, 160, 1000, false, false, "2 waves/SIMD, x kept, more compute")
    RUN(4, 50000, 160, 1000, true, true, "3 waves/SIMD, reload, more compute")
    return 0;
}
