// A/B of traversals for the replica loop's fused AdamW + SPARTA average
// (ga_adam_sparta_step) at configs[3]'s size: K = 32 replicas of GPT-2 124M,
// p = 0.005 packed mask.  Standalone diagnostic, not part of the library:
//   hipcc -O3 --offload-arch=gfx950 -Igym_amd/csrc tools/ubench_adam_sparta.hip -o build/ubench_adam_sparta
// Kernels (all with the library's Adam arithmetic, adam_math.h):
//   adam      replica-major (the library's ga_adam_step: grid.y = replica, 16 KB per array per workgroup)
//   fusedU    element-major: a workgroup owns U float4 per lane of EVERY replica, k loop inside,
//             ascending-k sums, selected words written after the loop (U = 1: the library's form)
//   fusedUd   the same with the selected lanes' p stores deferred: their new p of every replica
//             parked in LDS (slot per selected lane), written once, averaged, after the loop
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ga_common.h"
#include "adam_math.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

using namespace ga;

__global__ __launch_bounds__(256) void adam_rows(float* param, float* grad, float* m_, float* v_, int64_t n, int64_t ld,
                                                 AdamParams ap) {
    const int64_t rep = blockIdx.y;
    param += rep * ld; grad += rep * ld; m_ += rep * ld; v_ += rep * ld;
    const int64_t nv = n >> 2, lo = (int64_t)blockIdx.x * 1024, hi = lo + 1024 < nv ? lo + 1024 : nv;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        float4 p = stream_load(reinterpret_cast<const float4*>(param) + i);
        float4 g = stream_load(reinterpret_cast<const float4*>(grad) + i);
        float4 m = stream_load(reinterpret_cast<const float4*>(m_) + i);
        float4 v = stream_load(reinterpret_cast<const float4*>(v_) + i);
        float gg[4] = {g.x, g.y, g.z, g.w}, pp[4] = {p.x, p.y, p.z, p.w}, mm[4] = {m.x, m.y, m.z, m.w},
              vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) adam_elem(pp[e], gg[e], mm[e], vv[e], ap);
        const uint32_t o = (uint32_t)(i - lo);
        store_sc1(reinterpret_cast<float4*>(param) + lo, o, make_float4(pp[0], pp[1], pp[2], pp[3]));
        store_sc1(reinterpret_cast<float4*>(m_) + lo, o, make_float4(mm[0], mm[1], mm[2], mm[3]));
        store_sc1(reinterpret_cast<float4*>(v_) + lo, o, make_float4(vv[0], vv[1], vv[2], vv[3]));
    }
}

// persistent form: a grid of G workgroups walks the chunks c = b, b + G, ...; all of
// them start their chunk's k loop together, so the grid streams ~one replica row at a time
__global__ __launch_bounds__(256) void fused_persist(const uint64_t* bits, int64_t n, float* param, float* grad,
                                                     float* m_, float* v_, int K, int64_t ld, AdamParams ap,
                                                     float divisor) {
    const int64_t nchunks = (n / 4 + 255) / 256;
    for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
        const int64_t blk = c * 256;
        const int64_t i = blk + threadIdx.x;
        const int64_t e0 = 4 * i;
        if (e0 >= n) continue;
        const uint32_t sel = (uint32_t)(bits[e0 >> 6] >> (e0 & 63)) & 0xFu;
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < K; ++k) {
            const int64_t rk = (int64_t)k * ld;
            float4 p = stream_load(reinterpret_cast<const float4*>(param + rk) + i);
            float4 g = stream_load(reinterpret_cast<const float4*>(grad + rk) + i);
            float4 m = stream_load(reinterpret_cast<const float4*>(m_ + rk) + i);
            float4 v = stream_load(reinterpret_cast<const float4*>(v_ + rk) + i);
            float gg[4] = {g.x, g.y, g.z, g.w}, pp[4] = {p.x, p.y, p.z, p.w}, mm[4] = {m.x, m.y, m.z, m.w},
                  vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                adam_elem(pp[e], gg[e], mm[e], vv[e], ap);
                s[e] += pp[e];
            }
            const uint32_t o = (uint32_t)threadIdx.x;
            *(reinterpret_cast<float4*>(param + rk) + i) = make_float4(pp[0], pp[1], pp[2], pp[3]);
            store_sc1(reinterpret_cast<float4*>(m_ + rk) + blk, o, make_float4(mm[0], mm[1], mm[2], mm[3]));
            store_sc1(reinterpret_cast<float4*>(v_ + rk) + blk, o, make_float4(vv[0], vv[1], vv[2], vv[3]));
        }
        if (sel) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!((sel >> e) & 1u)) continue;
                const float avg = s[e] / divisor;
                for (int k = 0; k < K; ++k) param[(int64_t)k * ld + e0 + e] = avg;
            }
        }
    }
}

template <int U, bool DEFER, bool PSC1>
__global__ __launch_bounds__(256) void fused(const uint64_t* bits, int64_t n, float* param, float* grad, float* m_,
                                             float* v_, int K, int64_t ld, AdamParams ap, float divisor) {
    constexpr int kSlots = 24;
    __shared__ float4 park[DEFER ? kSlots * 32 : 1];
    __shared__ int nslot;
    if (DEFER && threadIdx.x == 0) nslot = 0;
    if (DEFER) __syncthreads();
    const int64_t blk = (int64_t)blockIdx.x * 256 * U;
    uint32_t sel[U];
    int slot[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t e0 = 4 * (blk + threadIdx.x + 256 * u);
        sel[u] = e0 < n ? (uint32_t)(bits[e0 >> 6] >> (e0 & 63)) & 0xFu : 0u;
        slot[u] = -1;
        if (DEFER && sel[u] && K <= 32) {
            const int s = atomicAdd(&nslot, 1);
            slot[u] = s < kSlots ? s : -1;
        }
    }
    float s[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u][0] = s[u][1] = s[u][2] = s[u][3] = 0.f;
    for (int k = 0; k < K; ++k) {
        const int64_t rk = (int64_t)k * ld;
        float4 p[U], g[U], m[U], v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = blk + threadIdx.x + 256 * u;
            p[u] = stream_load(reinterpret_cast<const float4*>(param + rk) + i);
            g[u] = stream_load(reinterpret_cast<const float4*>(grad + rk) + i);
            m[u] = stream_load(reinterpret_cast<const float4*>(m_ + rk) + i);
            v[u] = stream_load(reinterpret_cast<const float4*>(v_ + rk) + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t o = (uint32_t)(threadIdx.x + 256 * u);
            float gg[4] = {g[u].x, g[u].y, g[u].z, g[u].w}, pp[4] = {p[u].x, p[u].y, p[u].z, p[u].w},
                  mm[4] = {m[u].x, m[u].y, m[u].z, m[u].w}, vv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                adam_elem(pp[e], gg[e], mm[e], vv[e], ap);
                s[u][e] += pp[e];
            }
            const float4 pn = make_float4(pp[0], pp[1], pp[2], pp[3]);
            if (DEFER && slot[u] >= 0) park[slot[u] * 32 + k] = pn;
            else if (PSC1) store_sc1(reinterpret_cast<float4*>(param + rk) + blk, o, pn);
            else *(reinterpret_cast<float4*>(param + rk) + blk + o) = pn;
            store_sc1(reinterpret_cast<float4*>(m_ + rk) + blk, o, make_float4(mm[0], mm[1], mm[2], mm[3]));
            store_sc1(reinterpret_cast<float4*>(v_ + rk) + blk, o, make_float4(vv[0], vv[1], vv[2], vv[3]));
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!sel[u]) continue;
        const int64_t i = blk + threadIdx.x + 256 * u;
        float avg[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) avg[e] = s[u][e] / divisor;
        if (DEFER && slot[u] >= 0) {
            for (int k = 0; k < K; ++k) {
                float4 q = park[slot[u] * 32 + k];
                if (sel[u] & 1u) q.x = avg[0];
                if (sel[u] & 2u) q.y = avg[1];
                if (sel[u] & 4u) q.z = avg[2];
                if (sel[u] & 8u) q.w = avg[3];
                *(reinterpret_cast<float4*>(param + (int64_t)k * ld) + i) = q;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (!((sel[u] >> e) & 1u)) continue;
                for (int k = 0; k < K; ++k) param[(int64_t)k * ld + 4 * i + e] = avg[e];
            }
        }
    }
}

template <typename F>
static float time_ms(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    const int K = 32;
    const int64_t n = 124475904, ld = n;
    float *P, *G, *M, *V;
    uint64_t* bits;
    CK(hipMalloc(&P, 4 * K * ld)); CK(hipMalloc(&G, 4 * K * ld)); CK(hipMalloc(&M, 4 * K * ld)); CK(hipMalloc(&V, 4 * K * ld));
    CK(hipMemset(P, 0, 4 * K * ld)); CK(hipMemset(G, 0, 4 * K * ld)); CK(hipMemset(M, 0, 4 * K * ld)); CK(hipMemset(V, 0, 4 * K * ld));
    const int64_t words = (n + 63) / 64;
    uint64_t* hb = (uint64_t*)malloc(8 * words);
    uint64_t st = 88172645463325252ull;
    int64_t nsel = 0;
    for (int64_t w = 0; w < words; ++w) {  // each bit set with probability ~0.005
        uint64_t b = 0;
        for (int j = 0; j < 64; ++j) {
            st ^= st << 13; st ^= st >> 7; st ^= st << 17;
            if ((st % 1000) < 5) { b |= 1ull << j; ++nsel; }
        }
        hb[w] = b;
    }
    CK(hipMalloc(&bits, 8 * words));
    CK(hipMemcpy(bits, hb, 8 * words, hipMemcpyHostToDevice));
    AdamParams ap{0.1f, 0.999f, 0.001f, 1e-8f, 1.f - 1e-5f, 0.f, -0.01f, 0.0316f};
    const double alg = 28.0 * K * n;
    printf("K=%d n=%lld selected=%lld\n", K, (long long)n, (long long)nsel);
    for (int r = 0; r < 3; ++r) {
        float t;
        t = time_ms([&] { adam_rows<<<dim3((unsigned)((n / 4 + 1023) / 1024), K), 256>>>(P, G, M, V, n, ld, ap); }, 5);
        printf("r%d adam (replica-major)     %.3f ms  %.0f GB/s\n", r, t, alg / t / 1e6);
#define F(U, D, S, name)                                                                                         \
        t = time_ms([&] { fused<U, D, S><<<(unsigned)((n / 4 + 256 * U - 1) / (256 * U)), 256>>>(bits, n, P, G, M, V, K, \
                                                                                          ld, ap, (float)K); }, 5); \
        printf("r%d %-24s %.3f ms  %.0f GB/s\n", r, name, t, alg / t / 1e6);
        F(1, false, false, "fused U=1")
        F(2, false, false, "fused U=2")
        F(4, false, false, "fused U=4")
        F(1, true, false, "fused U=1 deferred")
        F(4, true, false, "fused U=4 deferred")
        F(1, false, true, "fused U=1 p sc1")
        for (int gsz : {1024, 1536, 2048, 4096}) {
            t = time_ms([&] { fused_persist<<<gsz, 256>>>(bits, n, P, G, M, V, K, ld, ap, (float)K); }, 5);
            printf("r%d fused persistent G=%-5d   %.3f ms  %.0f GB/s\n", r, gsz, t, alg / t / 1e6);
        }
        fflush(stdout);
    }
    return 0;
}
