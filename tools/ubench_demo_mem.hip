// Memory-pattern ceiling of the DeMo wave encode (ga_demo_encode_sym) on MI355X.
// Standalone diagnostic: a [R, C] fp32 matrix cut in 64x64 chunks, one wavefront
// per chunk, persistent over the grid; read delta and grad in the coalesced
// 4-rows-per-instruction layout, x = decay*delta + lr*grad, optionally a chain of
// dummy MFMAs standing in for the transforms, store delta.  Compared against a
// plain float4 stream over the same three arrays.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ unsigned coal(int i, int lane, int stride) {
    return (unsigned)(((lane >> 4) + 4 * i) * stride + 4 * (lane & 15));
}

// NMF: MFMAs per chunk (4 independent chains); ROWMAJOR: job order row-band major
template <int NMF, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void chunk_kernel(float* __restrict__ delta, const float* __restrict__ grad,
                                                           int R, int C, long njobs, float* sink) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gx = C / 64;
    const long stride = (long)gridDim.x * WAVES;
    f32x16 acc[4];
    for (int a = 0; a < 4; ++a)
        for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
    for (long job = (long)blockIdx.x * WAVES + wid; job < njobs; job += stride) {
        const int cy = (int)(job / gx), cx = (int)(job - (long)cy * gx);
        const long base = (long)cy * 64 * C + (long)cx * 64;
        float4 D[16], G[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) D[i] = *reinterpret_cast<const float4*>(delta + base + coal(i, lane, C));
#pragma unroll
        for (int i = 0; i < 16; ++i) G[i] = *reinterpret_cast<const float4*>(grad + base + coal(i, lane, C));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            D[i].x = fmaf(1e-3f, G[i].x, D[i].x * 0.999f);
            D[i].y = fmaf(1e-3f, G[i].y, D[i].y * 0.999f);
            D[i].z = fmaf(1e-3f, G[i].z, D[i].z * 0.999f);
            D[i].w = fmaf(1e-3f, G[i].w, D[i].w * 0.999f);
        }
#pragma unroll
        for (int t = 0; t < NMF; ++t) {
            const float4 v = D[(t >> 2) & 15];
            acc[t & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(v.x, v.y, acc[t & 3], 0, 0, 0);
        }
        if (NMF) {
            const float s = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
            D[0].x += s * 1e-30f;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(delta + base + coal(i, lane, C)) = D[i];
    }
    if (acc[0][5] == 1234.5f) sink[0] = acc[1][3];
}

// Row-band form: a workgroup of W waves owns a band of W chunks side by side (64 rows x 64 W
// columns); every load/store instruction covers one contiguous 1-KB row segment (wave w: rows
// w, w + W, ..., 64 / W rows x W / 4 segments each = 16 instructions per array, as above).
template <int W>
__global__ __launch_bounds__(64 * W) void band_kernel(float* __restrict__ delta, const float* __restrict__ grad,
                                                      int R, int C, long nbands, float* sink) {
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gb = C / (64 * W);  // bands per 64-row strip
    constexpr int SEG = W / 4;    // 1-KB segments per band row
    for (long job = blockIdx.x; job < nbands; job += gridDim.x) {
        const int cy = (int)(job / gb), cx = (int)(job - (long)cy * gb);
        const long base = (long)cy * 64 * C + (long)cx * 64 * W;
        float4 D[16], G[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = wid + W * (i / SEG), seg = i % SEG;
            D[i] = *reinterpret_cast<const float4*>(delta + base + (long)row * C + 256 * seg + 4 * lane);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = wid + W * (i / SEG), seg = i % SEG;
            G[i] = *reinterpret_cast<const float4*>(grad + base + (long)row * C + 256 * seg + 4 * lane);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            D[i].x = fmaf(1e-3f, G[i].x, D[i].x * 0.999f);
            D[i].y = fmaf(1e-3f, G[i].y, D[i].y * 0.999f);
            D[i].z = fmaf(1e-3f, G[i].z, D[i].z * 0.999f);
            D[i].w = fmaf(1e-3f, G[i].w, D[i].w * 0.999f);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = wid + W * (i / SEG), seg = i % SEG;
            *reinterpret_cast<float4*>(delta + base + (long)row * C + 256 * seg + 4 * lane) = D[i];
        }
    }
    if (lane == 99) sink[0] = 0.f;
}

__global__ __launch_bounds__(256) void stream3(float4* __restrict__ d, const float4* __restrict__ g, long nv) {
    const long stride = (long)gridDim.x * 256;
    for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < nv; v += stride) {
        float4 a = d[v], b = g[v];
        a.x = fmaf(1e-3f, b.x, a.x * 0.999f);
        a.y = fmaf(1e-3f, b.y, a.y * 0.999f);
        a.z = fmaf(1e-3f, b.z, a.z * 0.999f);
        a.w = fmaf(1e-3f, b.w, a.w * 0.999f);
        d[v] = a;
    }
}

template <typename F> float time_ms(F f, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}

int main() {
    const long N = 354871296L;  // GPT-2 350M
    float *d, *g, *sink;
    CK(hipMalloc(&d, 4 * N)); CK(hipMalloc(&g, 4 * N)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(d, 0, 4 * N)); CK(hipMemset(g, 0, 4 * N));
    const double bytes = 12.0 * N;
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int grid : {1024, 4096, 16384}) {
        float ms = time_ms([&] { stream3<<<grid, 256>>>((float4*)d, (const float4*)g, N / 4); }, 10);
        printf("stream3 grid %5d                 : %.3f ms  %.0f GB/s\n", grid, ms, bytes / ms / 1e6);
    }
    for (int C : {1024, 4096}) {
        const int R = (int)(N / C / 64 * 64);
        const long nj = (long)(R / 64) * (C / 64);
        const double b = 12.0 * R * (double)C;
#define RUN(NMF, W, BPC) { float ms = time_ms([&] { chunk_kernel<NMF, W><<<cus * BPC, 64 * W>>>(d, g, R, C, nj, sink); }, 10); \
        printf("chunk C=%d mfma=%3d waves/blk=%2d blk/CU=%d: %.3f ms  %.0f GB/s\n", C, NMF, W, BPC, ms, b / ms / 1e6); }
        RUN(0, 8, 1) RUN(0, 8, 2) RUN(0, 16, 1)
        RUN(128, 8, 1) RUN(128, 8, 2) RUN(128, 16, 1)
        RUN(160, 8, 1) RUN(160, 8, 2)
#define BAND(W, BPC) { const long nb = (long)(R / 64) * (C / (64 * W)); \
        float ms = time_ms([&] { band_kernel<W><<<cus * BPC, 64 * W>>>(d, g, R, C, nb, sink); }, 10); \
        printf("band  C=%d waves/blk=%2d blk/CU=%d          : %.3f ms  %.0f GB/s\n", C, W, BPC, ms, b / ms / 1e6); }
        BAND(4, 2) BAND(4, 4) BAND(8, 1) BAND(8, 2) BAND(16, 1)
    }
    return 0;
}
