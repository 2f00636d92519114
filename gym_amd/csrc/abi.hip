// Library-level entry points and the thread-local error string.
#include "ga_common.h"

#include <string.h>

namespace ga {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = 0; }

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
        return GA_EHIP;
    }
    return GA_OK;
}

}  // namespace ga

namespace ga {

// Streaming copy: each lane moves 4 float4 (loads issued back to back, then
// the stores); a workgroup covers 1024 contiguous float4 (16 KiB).
__global__ __launch_bounds__(256) void stream_copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                          int64_t nvec) {
    const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x;
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t i = base + u * 256;
        if (i < nvec) v[u] = stream_load(src + i);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t i = base + u * 256;
        if (i < nvec) stream_store(dst + i, v[u]);
    }
}

}  // namespace ga

extern "C" GA_API int ga_stream_copy(const void* src, void* dst, int64_t nbytes, hipStream_t stream) {
    ga::clear_error();
    GA_REQUIRE(nbytes >= 0 && nbytes % 16 == 0, "ga_stream_copy: nbytes must be a multiple of 16");
    GA_REQUIRE(((uintptr_t)src % 16) == 0 && ((uintptr_t)dst % 16) == 0, "ga_stream_copy: 16-byte alignment");
    if (nbytes == 0) return GA_OK;
    GA_REQUIRE(src && dst, "ga_stream_copy: null buffer");
    const int64_t nvec = nbytes / 16;
    const int64_t grid = ga::ceil_div(nvec, 1024);
    GA_REQUIRE(grid < (int64_t)INT32_MAX, "ga_stream_copy: too large");
    hipLaunchKernelGGL(ga::stream_copy_kernel, dim3((unsigned)grid), dim3(256), 0, stream, (const float4*)src,
                       (float4*)dst, nvec);
    return ga::check_launch("ga_stream_copy");
}

namespace ga {

// Random-word probe: lane f of the grid -> (position j, replica k), replica-major
// over the whole list (each replica's words of consecutive positions on adjacent
// lanes), read-modify-write or read + one sum store per 256 lanes.
__global__ __launch_bounds__(256) void probe_random_words_kernel(float* __restrict__ a, int64_t ld, int64_t K,
                                                                 const int32_t* __restrict__ pos, int64_t M,
                                                                 int write) {
    const int64_t tot = M * K;
    float acc = 0.f;
    for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < tot; f += (int64_t)gridDim.x * 256) {
        const int64_t k = f / M, j = f - k * M;
        float* p = a + k * ld + pos[j];
        if (write >= 2) {  // the whole aligned 64-B sector (2) or 128-B line (3) read and written back
            const int nv = write == 2 ? 4 : 8;
            float4* q = reinterpret_cast<float4*>(a + k * ld + (pos[j] & ~(4 * nv - 1)));
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (u < nv) v[u] = q[u];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (u < nv) q[u] = make_float4(v[u].x * 0.5f + 1.f, v[u].y, v[u].z, v[u].w);
            continue;
        }
        const float v = *p;
        if (write) *p = v * 0.5f + 1.f;
        else acc += v;
    }
    if (!write && acc == 12345.678f) a[0] = acc;  // keeps the reads (never true for the probe's data)
}

}  // namespace ga

extern "C" GA_API int ga_probe_random_words(float* a, int64_t ld, int64_t K, const int32_t* pos, int64_t M,
                                            int write, hipStream_t stream) {
    ga::clear_error();
    GA_REQUIRE(K >= 1 && M >= 0 && ld >= 1 && write >= 0 && write <= 3, "ga_probe_random_words: bad K/M/ld/write");
    GA_REQUIRE(write < 2 || (ld % 32 == 0 && ((uintptr_t)a % 128) == 0), "ga_probe_random_words: sector modes need 128-B aligned rows");
    if (M == 0) return GA_OK;
    GA_REQUIRE(a && pos, "ga_probe_random_words: null buffer");
    const int64_t tot = M * K;
    int64_t grid = ga::ceil_div(tot, 256);
    if (grid > 256 * 32) grid = 256 * 32;
    hipLaunchKernelGGL(ga::probe_random_words_kernel, dim3((unsigned)grid), dim3(256), 0, stream, a, ld, K, pos, M,
                       write);
    return ga::check_launch("ga_probe_random_words");
}

namespace ga {

// The DeMo codec's 64x64-chunk access pattern with no transform: one wavefront per
// chunk of a [rows, cols] fp32 matrix (persistent over the grid, 8 waves per
// workgroup, the chunk kernels' coalesced layout -- lane t holds rows (t >> 4) + 4i,
// i < 16, at column 4 (t & 15)).  mode 0 = the encode's traffic (read a and b,
// a <- 0.999 a + 1e-3 b), mode 1 = the decode's (read a, write a and b).
template <bool NT>
__device__ __forceinline__ float4 pld(const float* p) {
    if constexpr (NT) return stream_load(reinterpret_cast<const float4*>(p));
    else return *reinterpret_cast<const float4*>(p);
}
template <bool NT>
__device__ __forceinline__ void pst(float* p, const float4& v) {
    if constexpr (NT) stream_store(reinterpret_cast<float4*>(p), v);
    else *reinterpret_cast<float4*>(p) = v;
}

template <bool NT>
__global__ __launch_bounds__(512) void probe_chunk_stream_kernel(float* __restrict__ a, float* __restrict__ b,
                                                                 int64_t rows, int64_t cols, int mode) {
    const int lane = threadIdx.x & 63;
    const int64_t gx = cols / 64, nch = (rows / 64) * gx;
    for (int64_t c = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6); c < nch; c += (int64_t)gridDim.x * 8) {
        const int64_t cy = c / gx, cx = c - cy * gx;
        float* pa = a + cy * 64 * cols + cx * 64;
        float* pb = b + cy * 64 * cols + cx * 64;
        float4 x[16], y[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = pld<NT>(pa + ((lane >> 4) + 4 * i) * cols + 4 * (lane & 15));
        if (mode == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) y[i] = pld<NT>(pb + ((lane >> 4) + 4 * i) * cols + 4 * (lane & 15));
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                x[i].x = fmaf(1e-3f, y[i].x, 0.999f * x[i].x);
                x[i].y = fmaf(1e-3f, y[i].y, 0.999f * x[i].y);
                x[i].z = fmaf(1e-3f, y[i].z, 0.999f * x[i].z);
                x[i].w = fmaf(1e-3f, y[i].w, 0.999f * x[i].w);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                y[i] = make_float4(x[i].x > 0.f ? 1.f : -1.f, x[i].y > 0.f ? 1.f : -1.f, x[i].z > 0.f ? 1.f : -1.f,
                                   x[i].w > 0.f ? 1.f : -1.f);
                x[i].x -= 1e-3f * y[i].x;
                x[i].y -= 1e-3f * y[i].y;
                x[i].z -= 1e-3f * y[i].z;
                x[i].w -= 1e-3f * y[i].w;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) pst<NT>(pb + ((lane >> 4) + 4 * i) * cols + 4 * (lane & 15), y[i]);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) pst<NT>(pa + ((lane >> 4) + 4 * i) * cols + 4 * (lane & 15), x[i]);
    }
}

}  // namespace ga

extern "C" GA_API int ga_probe_chunk_stream(float* a, float* b, int64_t rows, int64_t cols, int mode,
                                            hipStream_t stream) {
    ga::clear_error();
    GA_REQUIRE(rows >= 0 && cols >= 0 && rows % 64 == 0 && cols % 64 == 0 && mode >= 0 && mode <= 3,
               "ga_probe_chunk_stream: rows, cols multiples of 64, mode 0..3");
    if (rows == 0 || cols == 0) return GA_OK;
    GA_REQUIRE(a && b && ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0, "ga_probe_chunk_stream: buffers");
    static const int cus = [] {
        int dev = 0, c = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        return c > 0 ? c : 256;
    }();
    const int64_t nch = (rows / 64) * (cols / 64);
    int64_t grid = ga::ceil_div(nch, 8);
    if (grid > cus) grid = cus;  // one 8-wave workgroup per CU, persistent (as ga_demo_encode_sym)
    if (mode & 2)
        hipLaunchKernelGGL(ga::probe_chunk_stream_kernel<true>, dim3((unsigned)grid), dim3(512), 0, stream, a, b,
                           rows, cols, mode & 1);
    else
        hipLaunchKernelGGL(ga::probe_chunk_stream_kernel<false>, dim3((unsigned)grid), dim3(512), 0, stream, a, b,
                           rows, cols, mode & 1);
    return ga::check_launch("ga_probe_chunk_stream");
}

extern "C" GA_API int ga_abi_version(void) { return 103; }

extern "C" GA_API const char* ga_last_error(void) { return ga::g_err; }
