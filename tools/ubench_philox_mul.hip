// r04 experiment: the Philox-4x32-10 round's two 32x32 products as mul_lo + mul_hi
// (what the compiler emits for lo = a * b, hi = __umulhi(a, b)) against one
// v_mad_u64_u32 per product (lo and hi from one instruction).  Each lane runs
// CALLS Philox calls; outputs xor-folded to one word per lane and compared.
// Not part of the library.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_philox_mul.hip -o build/ubench_philox_mul
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                           \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b) {
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b) : "vcc");
    return r;
}

template <int MODE>
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0, hi0, lo1, hi1;
        if (MODE == 0) {
            lo0 = M0 * c.x, hi0 = __umulhi(M0, c.x);
            lo1 = M1 * c.z, hi1 = __umulhi(M1, c.z);
        } else {
            const uint64_t p0 = mad64(M0, c.x), p1 = mad64(M1, c.z);
            lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
            lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        }
        c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k.x, 0x96), lo1,
                       __builtin_amdgcn_bitop3_b32(hi0, c.w, k.y, 0x96), lo0);
        k.x += W0;
        k.y += W1;
    }
    return c;
}

template <int MODE>
__global__ __launch_bounds__(256) void kern(uint32_t* out, int calls, uint2 key) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    for (int c0 = 0; c0 < calls; c0 += 4) {
        uint4 w[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) w[c] = philox<MODE>(make_uint4(t, 7u, (uint32_t)(c0 + c), 0u), key);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc ^= w[c].x ^ (w[c].y * 3u) ^ (w[c].z * 5u) ^ (w[c].w * 7u);
    }
    out[t] = acc;
}

int main() {
    const int blocks = 256 * 32, calls = 64;
    const size_t nt = (size_t)blocks * 256;
    uint32_t *a, *b;
    CK(hipMalloc(&a, nt * 4));
    CK(hipMalloc(&b, nt * 4));
    const uint2 key = make_uint2(0x1234567u, 0x89abcdefu);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 2; ++mode) {
            auto go = [&] {
                if (mode == 0) hipLaunchKernelGGL(kern<0>, dim3(blocks), dim3(256), 0, 0, a, calls, key);
                else hipLaunchKernelGGL(kern<1>, dim3(blocks), dim3(256), 0, 0, b, calls, key);
            };
            go();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) go();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double gcalls = (double)nt * calls / (ms / 10 * 1e-3) / 1e9;
            printf("mode %s: %.4f ms  %.1f G Philox calls/s\n", mode ? "mad_u64_u32" : "mul_lo+mul_hi", ms / 10,
                   gcalls);
        }
    }
    uint32_t *ha = (uint32_t*)malloc(nt * 4), *hb = (uint32_t*)malloc(nt * 4);
    CK(hipMemcpy(ha, a, nt * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb, b, nt * 4, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < nt; ++i) diff += ha[i] != hb[i];
    printf("outputs differing: %zu of %zu\n", diff, nt);
    return 0;
}
