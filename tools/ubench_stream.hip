// Streaming-ceiling micro-benchmark on MI355X: float4 copy and the 20-stream
// DiLoCo pattern in several lane->address mappings.  Standalone tool.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_gs(const float4* __restrict__ a, float4* __restrict__ b, long nv) {
    long stride = (long)gridDim.x * 256 * U;
    for (long v0 = (long)blockIdx.x * 256 * U + threadIdx.x; v0 < nv; v0 += stride) {
        float4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { long v = v0 + u * 256; if (v < nv) x[u] = a[v]; }
#pragma unroll
        for (int u = 0; u < U; ++u) { long v = v0 + u * 256; if (v < nv) {
            if (NT) { __builtin_nontemporal_store(x[u].x, &b[v].x); __builtin_nontemporal_store(x[u].y, &b[v].y);
                      __builtin_nontemporal_store(x[u].z, &b[v].z); __builtin_nontemporal_store(x[u].w, &b[v].w); }
            else b[v] = x[u]; } }
    }
}

// contiguous chunk per block: block b owns [b*chunk, (b+1)*chunk)
template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const float4* __restrict__ a, float4* __restrict__ b, long nv, long chunk) {
    long lo = (long)blockIdx.x * chunk, hi = lo + chunk < nv ? lo + chunk : nv;
    for (long v0 = lo + threadIdx.x; v0 < hi; v0 += 256 * U) {
        float4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { long v = v0 + u * 256; if (v < hi) x[u] = a[v]; }
#pragma unroll
        for (int u = 0; u < U; ++u) { long v = v0 + u * 256; if (v < hi) b[v] = x[u]; }
    }
}

__global__ __launch_bounds__(256) void read_only(const float4* __restrict__ a, float* out, long nv) {
    long stride = (long)gridDim.x * 256 * 4;
    float4 acc = {0, 0, 0, 0};
    for (long v0 = (long)blockIdx.x * 256 * 4 + threadIdx.x; v0 < nv; v0 += stride) {
#pragma unroll
        for (int u = 0; u < 4; ++u) { long v = v0 + u * 256; if (v < nv) { float4 x = a[v]; acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w; } }
    }
    if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

__global__ __launch_bounds__(256) void write_only(float4* __restrict__ b, long nv) {
    long stride = (long)gridDim.x * 256;
    for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < nv; v += stride) b[v] = make_float4(1, 2, 3, 4);
}

template <int K, int U>
__global__ __launch_bounds__(256) void diloco_chunk(const float* src, long ld, long n, float* master, float* mom, float* dst, long chunk) {
    long nv = n >> 2;
    long lo = (long)blockIdx.x * chunk, hi = lo + chunk < nv ? lo + chunk : nv;
    for (long v0 = lo + threadIdx.x; v0 < hi; v0 += 256 * U) {
        float4 x[U][K], m[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { long v = v0 + u * 256; if (v < hi) {
#pragma unroll
            for (int k = 0; k < K; ++k) x[u][k] = reinterpret_cast<const float4*>(src + k * ld)[v];
            m[u] = reinterpret_cast<float4*>(master)[v]; b[u] = reinterpret_cast<float4*>(mom)[v]; } }
#pragma unroll
        for (int u = 0; u < U; ++u) { long v = v0 + u * 256; if (v < hi) {
            float4 a = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < K; ++k) { a.x += x[u][k].x; a.y += x[u][k].y; a.z += x[u][k].z; a.w += x[u][k].w; }
            float4 o; float* ap = &a.x; float* mp = &m[u].x; float* bp = &b[u].x; float* op = &o.x;
#pragma unroll
            for (int e = 0; e < 4; ++e) { float g = mp[e] - ap[e] / 8.f; bp[e] = fmaf(1.f, g, bp[e] * 0.9f); g = fmaf(0.9f, bp[e], g); mp[e] = fmaf(-0.7f, g, mp[e]); op[e] = mp[e]; }
            reinterpret_cast<float4*>(master)[v] = m[u]; reinterpret_cast<float4*>(mom)[v] = b[u];
#pragma unroll
            for (int k = 0; k < K; ++k) reinterpret_cast<float4*>(dst + k * ld)[v] = o; } }
    }
}

template <typename F> float time_ms(F f, int reps) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); return ms / reps;
}

int main() {
    const long n = 124475904, K = 8;
    float *src, *master, *mom, *big2, *out;
    CK(hipMalloc(&src, 4 * K * n)); CK(hipMalloc(&master, 4 * n)); CK(hipMalloc(&mom, 4 * n));
    CK(hipMalloc(&big2, 4 * 4 * n)); CK(hipMalloc(&out, 64));
    CK(hipMemset(src, 1, 4 * K * n)); CK(hipMemset(master, 1, 4 * n)); CK(hipMemset(mom, 1, 4 * n)); CK(hipMemset(big2, 1, 16 * n));
    const long nv = 4 * n / 4;  // copy 4*n floats = 2 GB read + 2 GB write
    int reps = 10;
    if (getenv("ONLY_DILOCO")) goto diloco;
    for (int g : {256, 512, 1024, 2048, 4096}) {
        float ms = time_ms([&] { read_only<<<g, 256>>>((const float4*)src, out, 2 * nv); }, reps);
        printf("read-only 4GB       grid %5d: %.0f GB/s\n", g, 8.0 * 2 * n / ms / 1e6 * 2);
    }
    for (int g : {512, 1024, 2048, 4096, 8192}) {
        float ms = time_ms([&] { write_only<<<g, 256>>>((float4*)big2, nv); }, reps);
        printf("write-only 2GB      grid %5d: %.0f GB/s\n", g, 16.0 * n / ms / 1e6);
    }
#define CG(U, NT) for (int g : {512, 1024, 2048, 4096}) { float ms = time_ms([&] { copy_gs<U, NT><<<g, 256>>>((const float4*)src, (float4*)big2, nv); }, reps); \
        printf("copy gs U=%d nt=%d 2+2GB grid %5d: %.0f GB/s\n", U, NT, g, 2 * 16.0 * n / ms / 1e6); }
    CG(1, false) CG(2, false) CG(4, false) CG(4, true)
    for (long chunk : {4096L, 16384L, 65536L}) {
        long g = (nv + chunk - 1) / chunk;
        float ms = time_ms([&] { copy_chunk<4><<<g, 256>>>((const float4*)src, (float4*)big2, nv, chunk); }, reps);
        printf("copy chunk %6ld (grid %ld): %.0f GB/s\n", chunk, g, 2 * 16.0 * n / ms / 1e6);
    }
diloco:
    const double bytes = (2.0 * K + 4.0) * 4.0 * n;
    for (long chunk : {128L, 256L, 512L, 1024L, 2048L}) {
        long g = (n / 4 + chunk - 1) / chunk;
        float ms = time_ms([&] { diloco_chunk<8, 1><<<g, 256>>>(src, n, n, master, mom, src, chunk); }, reps);
        float ms2 = time_ms([&] { diloco_chunk<8, 2><<<g, 256>>>(src, n, n, master, mom, src, chunk); }, reps);
        printf("diloco chunk %6ld (grid %ld): U1 %.3f ms %.0f GB/s | U2 %.3f ms %.0f GB/s\n", chunk, g, ms, bytes / ms / 1e6, ms2, bytes / ms2 / 1e6);
    }
    return 0;
}
