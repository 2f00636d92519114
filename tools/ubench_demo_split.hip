// Would the DeMo encode's two DCT products on bf16 MFMAs (each f32 operand split
// into three bf16 parts, six v_mfma_f32_32x32x16_bf16 per 32-deep f32 product:
// ~fp32 accuracy) beat the f32-input MFMAs it issues today?  Standalone
// diagnostic (round 5), on the encode emulation of tools/ubench_demo_occupancy.hip
// (2 waves per SIMD, the x tile kept in LDS, GPT-2 350M sized arrays): the
// memory pattern, then the products -- f32: NMF x v_mfma_f32_32x32x2_f32;
// split: the operands split 3 ways by VALU (NSPLIT values per lane) and NBF x
// v_mfma_f32_32x32x16_bf16 --, the residual's NRES f32 MFMAs, and the top-k's
// VALU (NV fmaf in 4 independent chains per lane).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned coal(int i, int lane, int stride) {
    return (unsigned)(((lane >> 4) + 4 * i) * stride + 4 * (lane & 15));
}

__device__ __forceinline__ unsigned hi16(float v) { return __float_as_uint(v) & 0xffff0000u; }

// v -> three bf16 parts (truncation splits, exact), packed pairwise
__device__ __forceinline__ void split3(float v0, float v1, unsigned& p0, unsigned& p1, unsigned& p2) {
    const unsigned a0 = hi16(v0), b0 = hi16(v1);
    const float r0 = v0 - __uint_as_float(a0), r1 = v1 - __uint_as_float(b0);
    const unsigned a1 = hi16(r0), b1 = hi16(r1);
    const float s0 = r0 - __uint_as_float(a1), s1 = r1 - __uint_as_float(b1);
    p0 = __builtin_amdgcn_perm(b0, a0, 0x07060302u);
    p1 = __builtin_amdgcn_perm(b1, a1, 0x07060302u);
    p2 = __builtin_amdgcn_perm(__float_as_uint(s1), __float_as_uint(s0), 0x07060302u);
}

template <int NMF, int NBF, int NSPLIT, int NRES, int NV>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void enc_kernel(float* __restrict__ delta, const float* __restrict__ grad, int C, long njobs, float* sink) {
    __shared__ float pad[150000 / 4];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gx = C / 64;
    const long stride = (long)gridDim.x * 8;
    float keep = 0.f;
    for (long job = (long)blockIdx.x * 8 + wid; job < njobs; job += stride) {
        const int cy = (int)(job / gx), cx = (int)(job - (long)cy * gx);
        const long base = (long)cy * 64 * C + (long)cx * 64;
        f32x16 acc[4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
        float4 X[16];
        {
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
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) reinterpret_cast<float4*>(pad)[(wid * 1024 + i * 64 + lane) % 9000] = X[i];
        if (NMF) {  // today's products: f32 MFMAs, operand = a loaded value / an accumulator element
#pragma unroll
            for (int t = 0; t < NMF / 2; ++t) {
                const float4 v = X[t & 15];
                acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.y, acc[t & 3], 0, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < NMF / 2; ++t)
                acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(acc[(t + 1) & 3][t & 15], acc[(t + 2) & 3][(t + 5) & 15],
                                                                  acc[t & 3], 0, 0, 0);
        }
        if (NBF) {  // split products: half the splits on the loaded values, half on the first product's accumulators
            unsigned P[3][NSPLIT / 4];
#pragma unroll
            for (int i = 0; i < NSPLIT / 4; ++i) {
                const float4 v = X[i & 15];
                split3(v.x + v.w, v.y - v.z, P[0][i], P[1][i], P[2][i]);
            }
#pragma unroll
            for (int t = 0; t < NBF / 2; ++t) {
                const int s = t % 6, j = (t / 6) * 4 % (NSPLIT / 4);
                bf16x8 a, b;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const unsigned w = P[s < 3 ? s : s - 3][(j + u) % (NSPLIT / 4)];
                    const unsigned w2 = P[s < 3 ? 0 : s - 2][(j + u + 1) % (NSPLIT / 4)];
                    a[2 * u] = (short)(w & 0xffff); a[2 * u + 1] = (short)(w >> 16);
                    b[2 * u] = (short)(w2 & 0xffff); b[2 * u + 1] = (short)(w2 >> 16);
                }
                acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t & 3], 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < NSPLIT / 4; ++i)
                split3(acc[i & 3][(2 * i) & 15], acc[(i + 1) & 3][(2 * i + 1) & 15], P[0][i], P[1][i], P[2][i]);
#pragma unroll
            for (int t = 0; t < NBF / 2; ++t) {
                const int s = t % 6, j = (t / 6) * 4 % (NSPLIT / 4);
                bf16x8 a, b;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const unsigned w = P[s < 3 ? s : s - 3][(j + u) % (NSPLIT / 4)];
                    const unsigned w2 = P[s < 3 ? 0 : s - 2][(j + u + 2) % (NSPLIT / 4)];
                    a[2 * u] = (short)(w & 0xffff); a[2 * u + 1] = (short)(w >> 16);
                    b[2 * u] = (short)(w2 & 0xffff); b[2 * u + 1] = (short)(w2 >> 16);
                }
                acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t & 3], 0, 0, 0);
            }
        }
        // the top-k's VALU: 4 independent chains per lane on the coefficients
        float v0 = acc[0][lane & 15], v1 = acc[1][3], v2 = acc[2][7], v3 = acc[3][11];
#pragma unroll 16
        for (int s = 0; s < NV / 4; ++s) {
            v0 = fmaf(v0, 0.999f, acc[s & 3][s & 15]);
            v1 = fmaf(v1, 0.998f, acc[(s + 1) & 3][s & 15]);
            v2 = fmaf(v2, 0.997f, acc[(s + 2) & 3][s & 15]);
            v3 = fmaf(v3, 0.996f, acc[(s + 3) & 3][s & 15]);
        }
        float v = v0 + v1 + v2 + v3;
        // the residual: f32 MFMAs on the selected values
#pragma unroll
        for (int t = 0; t < NRES; ++t) acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(v, acc[(t + 1) & 3][t & 15], acc[t & 3], 0, 0, 0);
        v += acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
        keep += v;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float4 o = reinterpret_cast<float4*>(pad)[(wid * 1024 + i * 64 + lane) % 9000];
            o.x -= v * 1e-30f;
            *reinterpret_cast<float4*>(delta + base + coal(i, lane, C)) = o;
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

int main() {
    const long N = 354871296L;  // GPT-2 350M
    float *d, *g, *sink;
    CK(hipMalloc(&d, 4 * N)); CK(hipMalloc(&g, 4 * N)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(d, 0, 4 * N)); CK(hipMemset(g, 0, 4 * N));
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int C = 1024, R = (int)(N / C / 64 * 64);
    const long nj = (long)(R / 64) * (C / 64);
    const double b = 12.0 * R * (double)C;
#define RUN(NMF, NBF, NSPLIT, NRES, NV, what) { auto k = enc_kernel<NMF, NBF, NSPLIT, NRES, NV>; \
    for (int rep = 0; rep < 3; ++rep) { float ms = time_ms([&] { k<<<cus, 512>>>(d, g, C, nj, sink); }, 10); \
    printf("%-26s f32 mfma %3d bf16 mfma %2d split %3d res %2d valu %4d: %.3f ms  %.0f GB/s (12 B/elem)\n", what, NMF, NBF, NSPLIT, NRES, NV, ms, b / ms / 1e6); } }
    RUN(0, 0, 0, 0, 0, "memory only")
    RUN(128, 0, 0, 34, 1500, "f32 products (today)")
    RUN(0, 48, 128, 34, 1500, "split bf16 products")
    RUN(128, 0, 0, 34, 2000, "f32 products, more valu")
    RUN(0, 48, 128, 34, 2000, "split, more valu")
    RUN(128, 0, 0, 0, 0, "f32 products only")
    RUN(0, 48, 128, 0, 0, "split products only")
    return 0;
}
