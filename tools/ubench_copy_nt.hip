// Streaming-copy variants at the DiLoCo working-set scale: does a non-temporal
// hint on the loads and/or stores raise the float4 copy rate (the ceiling
// ga_diloco_outer is measured against)?  Sizes from 1 GiB to 4.6 GiB per side
// (the K = 8 DiLoCo step moves 10 GB).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy4(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    const long base = (long)blockIdx.x * 1024 + threadIdx.x;
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long i = base + u * 256;
        if (i < nvec) v[u] = NTL ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long i = base + u * 256;
        if (i < nvec) {
            if (NTS) __builtin_nontemporal_store(v[u], dst + i);
            else dst[i] = v[u];
        }
    }
}

// U float4 per lane, B threads per workgroup, both hints (shape sweep)
template <int U, int B>
__global__ __launch_bounds__(B) void copy_u(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    const long base = (long)blockIdx.x * (U * B) + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * B;
        if (i < nvec) v[u] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = base + (long)u * B;
        if (i < nvec) __builtin_nontemporal_store(v[u], dst + i);
    }
}

// grid-stride form with a fixed grid (8 workgroups per CU)
template <bool NTS>
__global__ __launch_bounds__(256) void copy_gs(const f4* __restrict__ src, f4* __restrict__ dst, long nvec) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (long)gridDim.x * 256) {
        const f4 v = src[i];
        if (NTS) __builtin_nontemporal_store(v, dst + i);
        else dst[i] = v;
    }
}

int main() {
    const long maxb = 4979036160L;  // = 10 GB / 2: the DiLoCo step's read (and write) bytes
    f4 *a, *b;
    CK(hipMalloc(&a, maxb));
    CK(hipMalloc(&b, maxb));
    CK(hipMemset(a, 1, maxb));
    CK(hipMemset(b, 0, maxb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (long bytes : {1L << 30, maxb}) {
        const long nvec = bytes / 16;
        const unsigned g = (unsigned)((nvec + 1023) / 1024);
        auto run = [&](const char* name, auto launch) {
            launch();
            CK(hipDeviceSynchronize());
            const int reps = 10;
            CK(hipEventRecord(e0));
            for (int r = 0; r < reps; ++r) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            printf("%-26s %5.2f GiB/side  %.4f ms  %.0f GB/s (read + write)\n", name, bytes / 1073741824.0, ms,
                   2.0 * bytes / ms / 1e6);
        };
        run("plain", [&] { copy4<false, false><<<g, 256>>>(a, b, nvec); });
        run("nt store", [&] { copy4<false, true><<<g, 256>>>(a, b, nvec); });
        run("nt load", [&] { copy4<true, false><<<g, 256>>>(a, b, nvec); });
        run("nt load + store", [&] { copy4<true, true><<<g, 256>>>(a, b, nvec); });
        run("grid-stride 2048 wg", [&] { copy_gs<false><<<2048, 256>>>(a, b, nvec); });
        run("grid-stride 2048 nt store", [&] { copy_gs<true><<<2048, 256>>>(a, b, nvec); });
        run("plain (again)", [&] { copy4<false, false><<<g, 256>>>(a, b, nvec); });
        run("nt U=2 B=256", [&] { copy_u<2, 256><<<(unsigned)((nvec + 511) / 512), 256>>>(a, b, nvec); });
        run("nt U=8 B=256", [&] { copy_u<8, 256><<<(unsigned)((nvec + 2047) / 2048), 256>>>(a, b, nvec); });
        run("nt U=4 B=512", [&] { copy_u<4, 512><<<(unsigned)((nvec + 2047) / 2048), 512>>>(a, b, nvec); });
        run("nt U=4 B=1024", [&] { copy_u<4, 1024><<<(unsigned)((nvec + 4095) / 4096), 1024>>>(a, b, nvec); });
        run("nt U=16 B=256", [&] { copy_u<16, 256><<<(unsigned)((nvec + 4095) / 4096), 256>>>(a, b, nvec); });
        run("nt U=4 B=256 (again)", [&] { copy_u<4, 256><<<g, 256>>>(a, b, nvec); });
    }
    return 0;
}
