// Random-word ceiling for SPARTA's access pattern on MI355X: M ~ p*N selected
// positions (ascending) in each of K replicas of an N-element fp32 arena, read
// and written back (4-B words at random 64-B sectors).  Standalone tool:
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_gather.hip -o build/ubench_gather
// Orders: (a) element-major (lanes over replicas of one position), (b) replica-
// major over the whole list, (c) tile-grouped (a workgroup per 4096-element tile,
// replica-major inside it: what ga_sparta_average_local does, minus the mask).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void rmw_elem_major(float* a, long ld, const int* pos, long M, int K) {
    const long tot = M * K;
    for (long f = (long)blockIdx.x * blockDim.x + threadIdx.x; f < tot; f += (long)gridDim.x * blockDim.x) {
        const long j = f / K, k = f - j * K;
        float* p = a + k * ld + pos[j];
        *p = *p * 0.5f + 1.f;
    }
}

__global__ void rmw_rep_major(float* a, long ld, const int* pos, long M, int K) {
    const long tot = M * K;
    for (long f = (long)blockIdx.x * blockDim.x + threadIdx.x; f < tot; f += (long)gridDim.x * blockDim.x) {
        const long k = f / M, j = f - k * M;
        float* p = a + k * ld + pos[j];
        *p = *p * 0.5f + 1.f;
    }
}

// one workgroup per tile: tile_start[t] .. tile_start[t+1] positions, replica-major
__global__ __launch_bounds__(256) void rmw_tiles(float* a, long ld, const int* pos, const int* tile_start, int K) {
    const int b = tile_start[blockIdx.x], e = tile_start[blockIdx.x + 1], c = e - b;
    for (int f = threadIdx.x; f < c * K; f += 256) {
        const int k = f / c, j = f - k * c;
        float* p = a + (long)k * ld + pos[b + j];
        *p = *p * 0.5f + 1.f;
    }
}

// read-only variant of (c): per-position sums over the K replicas
__global__ __launch_bounds__(256) void read_tiles(const float* a, long ld, const int* pos, const int* tile_start,
                                                   int K, float* out) {
    __shared__ float acc[512];
    const int b = tile_start[blockIdx.x], e = tile_start[blockIdx.x + 1], c = e - b;
    for (int f = threadIdx.x; f < 512; f += 256) acc[f] = 0.f;
    __syncthreads();
    for (int f = threadIdx.x; f < c * K; f += 256) {
        const int k = f / c, j = f - k * c;
        atomicAdd(&acc[j & 511], a[(long)k * ld + pos[b + j]]);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < c; j += 256) out[b + j] = acc[j & 511];
}

// Line-granular forms for the element-major [n, 32] set (round 2): one selected
// element's 32 fp32 replicas are one 128-B line = 8 lanes x 16 B.  Flat over the
// M*8 quads (grid-stride) or one workgroup per 16384-element tile.  RMW reads and
// writes each line once; the read form sums the line (no write).
__global__ __launch_bounds__(256) void rmw_lines_flat(float4* a, const int* pos, long M) {
    const long tot = M * 8;
    for (long f = (long)blockIdx.x * 256 + threadIdx.x; f < tot; f += (long)gridDim.x * 256) {
        float4* q = a + (long)pos[f >> 3] * 8 + (f & 7);
        float4 v = *q;
        v.x = v.x * 0.5f + 1.f; v.y = v.y * 0.5f + 1.f; v.z = v.z * 0.5f + 1.f; v.w = v.w * 0.5f + 1.f;
        *q = v;
    }
}

__global__ __launch_bounds__(256) void rmw_lines_tiles(float4* a, const int* pos, const int* tile_start) {
    const int b = tile_start[blockIdx.x], c = tile_start[blockIdx.x + 1] - b;
    for (int f = threadIdx.x; f < c * 8; f += 256) {
        float4* q = a + (long)pos[b + (f >> 3)] * 8 + (f & 7);
        float4 v = *q;
        v.x = v.x * 0.5f + 1.f; v.y = v.y * 0.5f + 1.f; v.z = v.z * 0.5f + 1.f; v.w = v.w * 0.5f + 1.f;
        *q = v;
    }
}

__global__ __launch_bounds__(256) void read_lines_flat(const float4* a, const int* pos, long M, float* out) {
    const long tot = M * 8;
    float s = 0.f;
    for (long f = (long)blockIdx.x * 256 + threadIdx.x; f < tot; f += (long)gridDim.x * 256) {
        const float4 v = a[(long)pos[f >> 3] * 8 + (f & 7)];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    const int K = 32;
    const long n = 124475904, ld = n;
    const double p = 0.005;
    std::mt19937_64 rng(42);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<int> pos;
    const long tiles = (n + 4095) / 4096;
    std::vector<int> ts(tiles + 1, 0);
    for (long i = 0; i < n; ++i) {
        if (U(rng) < p) pos.push_back((int)i);
        if ((i & 4095) == 4095 || i == n - 1) ts[i / 4096 + 1] = (int)pos.size();
    }
    const long M = (long)pos.size();
    printf("n=%ld K=%d M=%ld pairs=%ld\n", n, K, M, M * K);
    float *a, *out;
    int *dpos, *dts;
    CK(hipMalloc(&a, sizeof(float) * K * ld));
    CK(hipMemset(a, 0, sizeof(float) * K * ld));
    CK(hipMalloc(&out, sizeof(float) * M));
    CK(hipMalloc(&dpos, sizeof(int) * M));
    CK(hipMalloc(&dts, sizeof(int) * (tiles + 1)));
    CK(hipMemcpy(dpos, pos.data(), sizeof(int) * M, hipMemcpyHostToDevice));
    CK(hipMemcpy(dts, ts.data(), sizeof(int) * (tiles + 1), hipMemcpyHostToDevice));
    const int reps = 10;
    const double pairs = (double)M * K;
    auto rep = [&](const char* name, float ms, int rw) {
        printf("%-28s %.3f ms  %.1f G words/s  %.0f GB/s at %d B per word\n", name, ms, pairs / ms / 1e6,
               pairs * (rw ? 96 : 64) / ms / 1e6, rw ? 96 : 64);
    };
    for (int g : {4096, 16384, 65536}) {
        char nm[64];
        snprintf(nm, sizeof nm, "rmw element-major g=%d", g);
        rep(nm, time_ms([&] { rmw_elem_major<<<g, 256>>>(a, ld, dpos, M, K); }, reps), 1);
        snprintf(nm, sizeof nm, "rmw replica-major g=%d", g);
        rep(nm, time_ms([&] { rmw_rep_major<<<g, 256>>>(a, ld, dpos, M, K); }, reps), 1);
    }
    rep("rmw tile-grouped", time_ms([&] { rmw_tiles<<<(unsigned)tiles, 256>>>(a, ld, dpos, dts, K); }, reps), 1);
    rep("read tile-grouped", time_ms([&] { read_tiles<<<(unsigned)tiles, 256>>>(a, ld, dpos, dts, K, out); }, reps), 0);
    // element-major [n, 32] lines (the same buffer viewed as n rows of 32 floats)
    std::vector<int> ts16((n + 16383) / 16384 + 1, 0);
    for (long j = 0, t = 0; t < (long)ts16.size() - 1; ++t) {
        while (j < M && pos[j] < (t + 1) * 16384) ++j;
        ts16[t + 1] = (int)j;
    }
    int* dts16;
    CK(hipMalloc(&dts16, sizeof(int) * ts16.size()));
    CK(hipMemcpy(dts16, ts16.data(), sizeof(int) * ts16.size(), hipMemcpyHostToDevice));
    const double line_bytes = (double)M * 128;
    auto repl = [&](const char* name, float ms, int rw) {
        printf("%-28s %.4f ms  %.0f GB/s of 128-B lines (%s)\n", name, ms, line_bytes * (rw ? 2 : 1) / ms / 1e6,
               rw ? "read + write" : "read");
    };
    float4* a4 = reinterpret_cast<float4*>(a);
    for (int g : {4096, 16384, 65536}) {
        char nm[64];
        snprintf(nm, sizeof nm, "lines rmw flat g=%d", g);
        repl(nm, time_ms([&] { rmw_lines_flat<<<g, 256>>>(a4, dpos, M); }, reps), 1);
        snprintf(nm, sizeof nm, "lines read flat g=%d", g);
        repl(nm, time_ms([&] { read_lines_flat<<<g, 256>>>(a4, dpos, M, out); }, reps), 0);
    }
    repl("lines rmw 16384-tiles", time_ms([&] { rmw_lines_tiles<<<(unsigned)ts16.size() - 1, 256>>>(a4, dpos, dts16); }, reps), 1);
    // The same kernel over NSETS independent position sets in rotation: a fixed
    // set (80 MB of lines) stays in the 256 MiB Infinity Cache from launch to
    // launch; four sets (320 MB) do not, as a SPARTA step whose mask changes
    // every iteration does not.
    const int NSETS = 4;
    std::vector<int*> rpos(NSETS), rts(NSETS);
    for (int s = 0; s < NSETS; ++s) {
        std::mt19937_64 r2(1000 + s);
        std::vector<int> ps;
        std::vector<int> tt((n + 16383) / 16384 + 1, 0);
        for (long i = 0; i < n; ++i) {
            if (U(r2) < p) ps.push_back((int)i);
            if ((i & 16383) == 16383 || i == n - 1) tt[i / 16384 + 1] = (int)ps.size();
        }
        CK(hipMalloc(&rpos[s], sizeof(int) * ps.size()));
        CK(hipMalloc(&rts[s], sizeof(int) * tt.size()));
        CK(hipMemcpy(rpos[s], ps.data(), sizeof(int) * ps.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(rts[s], tt.data(), sizeof(int) * tt.size(), hipMemcpyHostToDevice));
    }
    int cur = 0;
    const unsigned g16 = (unsigned)ts16.size() - 1;
    repl("lines rmw 16384-tiles 1 set", time_ms([&] { rmw_lines_tiles<<<g16, 256>>>(a4, rpos[0], rts[0]); }, 4 * reps), 1);
    repl("lines rmw 16384-tiles 4 sets", time_ms([&] {
        rmw_lines_tiles<<<g16, 256>>>(a4, rpos[cur], rts[cur]);
        cur = (cur + 1) % NSETS;
    }, 4 * reps), 1);
    CK(hipFree(a));
    return 0;
}
