// Micro-benchmark of streaming-kernel variants for the fused DiLoCo outer step
// ([K, n] replicas + master + momentum, fp32).  Standalone: hipcc -O3
// --offload-arch=gfx950 tools/ubench_diloco.hip -o build/ubench_diloco
// Prints GB/s of algorithmic bytes for each variant, and a float4 copy for
// calibration.  Not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

struct OP { float divisor, lr, mu; };

__device__ __forceinline__ float upd(float s, float& m, float& b, const OP& op) {
    float avg = s / op.divisor;
    float g = m - avg;
    b = fmaf(1.f, g, b * op.mu);
    g = fmaf(op.mu, b, g);
    m = fmaf(-op.lr, g, m);
    return m;
}

template <bool NT>
__device__ __forceinline__ float4 ld4(const float4* p) {
    if constexpr (NT) {
        float4 r;
        r.x = __builtin_nontemporal_load(&p->x);
        r.y = __builtin_nontemporal_load(&p->y);
        r.z = __builtin_nontemporal_load(&p->z);
        r.w = __builtin_nontemporal_load(&p->w);
        return r;
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ void st4(float4* p, float4 v) {
    if constexpr (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}

// runtime K (the library's current form)
__global__ __launch_bounds__(256) void v_runtime(const float* src, long K, long ld, long n, float* master, float* mom,
                                                 OP op, float* dst) {
    long stride = (long)gridDim.x * blockDim.x;
    long nv = n >> 2;
    for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
        float a[4] = {0, 0, 0, 0};
#pragma unroll 4
        for (long k = 0; k < K; ++k) {
            float4 x = reinterpret_cast<const float4*>(src + k * ld)[v];
            a[0] += x.x; a[1] += x.y; a[2] += x.z; a[3] += x.w;
        }
        float4 m = reinterpret_cast<float4*>(master)[v], b = reinterpret_cast<float4*>(mom)[v];
        float4 o;
        o.x = upd(a[0], m.x, b.x, op); o.y = upd(a[1], m.y, b.y, op);
        o.z = upd(a[2], m.z, b.z, op); o.w = upd(a[3], m.w, b.w, op);
        reinterpret_cast<float4*>(master)[v] = m;
        reinterpret_cast<float4*>(mom)[v] = b;
        for (long k = 0; k < K; ++k) reinterpret_cast<float4*>(dst + k * ld)[v] = o;
    }
}

// compile-time K, U vectors per lane per iteration, optional nontemporal loads/stores
template <int K, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void v_static(const float* src, long ld, long n, float* master, float* mom, OP op,
                                                float* dst) {
    long stride = (long)gridDim.x * blockDim.x * U;
    long nv = n >> 2;
    for (long v0 = ((long)blockIdx.x * blockDim.x) * U + threadIdx.x; v0 < nv; v0 += stride) {
        float4 x[U][K];
        float4 m[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long v = v0 + (long)u * blockDim.x;
            if (v < nv) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k] = ld4<NTL>(reinterpret_cast<const float4*>(src + k * ld) + v);
                m[u] = ld4<NTL>(reinterpret_cast<const float4*>(master) + v);
                b[u] = ld4<NTL>(reinterpret_cast<const float4*>(mom) + v);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long v = v0 + (long)u * blockDim.x;
            if (v < nv) {
                float a[4] = {0, 0, 0, 0};
#pragma unroll
                for (int k = 0; k < K; ++k) { a[0] += x[u][k].x; a[1] += x[u][k].y; a[2] += x[u][k].z; a[3] += x[u][k].w; }
                float4 o;
                o.x = upd(a[0], m[u].x, b[u].x, op); o.y = upd(a[1], m[u].y, b[u].y, op);
                o.z = upd(a[2], m[u].z, b[u].z, op); o.w = upd(a[3], m[u].w, b[u].w, op);
                st4<NTS>(reinterpret_cast<float4*>(master) + v, m[u]);
                st4<NTS>(reinterpret_cast<float4*>(mom) + v, b[u]);
#pragma unroll
                for (int k = 0; k < K; ++k) st4<NTS>(reinterpret_cast<float4*>(dst + k * ld) + v, o);
            }
        }
    }
}

// the library's mapping: workgroup b owns vectors [b*CH, (b+1)*CH); U vectors per lane in flight
template <int K, int CH, int U, bool NTS>
__global__ __launch_bounds__(256) void v_chunk(const float* src, long ld, long n, float* master, float* mom, OP op,
                                               float* dst) {
    const long nv = n >> 2;
    const long lo = (long)blockIdx.x * CH;
    const long hi = lo + CH < nv ? lo + CH : nv;
    for (long v0 = lo + threadIdx.x; v0 < hi; v0 += 256 * U) {
        float4 x[U][K], m[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long v = v0 + 256L * u;
            if (v < hi) {
#pragma unroll
                for (int k = 0; k < K; ++k) x[u][k] = reinterpret_cast<const float4*>(src + k * ld)[v];
                m[u] = reinterpret_cast<const float4*>(master)[v];
                b[u] = reinterpret_cast<const float4*>(mom)[v];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long v = v0 + 256L * u;
            if (v < hi) {
                float a[4] = {0, 0, 0, 0};
#pragma unroll
                for (int k = 0; k < K; ++k) { a[0] += x[u][k].x; a[1] += x[u][k].y; a[2] += x[u][k].z; a[3] += x[u][k].w; }
                float4 o;
                o.x = upd(a[0], m[u].x, b[u].x, op); o.y = upd(a[1], m[u].y, b[u].y, op);
                o.z = upd(a[2], m[u].z, b[u].z, op); o.w = upd(a[3], m[u].w, b[u].w, op);
                st4<NTS>(reinterpret_cast<float4*>(master) + v, m[u]);
                st4<NTS>(reinterpret_cast<float4*>(mom) + v, b[u]);
#pragma unroll
                for (int k = 0; k < K; ++k) st4<NTS>(reinterpret_cast<float4*>(dst + k * ld) + v, o);
            }
        }
    }
}

// v_chunk with an XCD-aware block order: blocks b and b+8 share an XCD (round-robin
// dispatch), so block b takes chunk (b % 8) * per + b / 8 and each XCD streams one
// contiguous eighth of the arena (fewer pages per XCD's TLB, longer DRAM runs)
template <int K, int CH>
__global__ __launch_bounds__(256) void v_chunk_xcd(const float* src, long ld, long n, float* master, float* mom, OP op,
                                                   float* dst) {
    const long nv = n >> 2;
    const long per = gridDim.x >> 3;
    const long cb = (long)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    const long lo = cb * CH;
    const long hi = lo + CH < nv ? lo + CH : nv;
    for (long v = lo + threadIdx.x; v < hi; v += 256) {
        float4 x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = reinterpret_cast<const float4*>(src + k * ld)[v];
        float4 m = reinterpret_cast<const float4*>(master)[v], b = reinterpret_cast<const float4*>(mom)[v];
        float a[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) { a[0] += x[k].x; a[1] += x[k].y; a[2] += x[k].z; a[3] += x[k].w; }
        float4 o;
        o.x = upd(a[0], m.x, b.x, op); o.y = upd(a[1], m.y, b.y, op);
        o.z = upd(a[2], m.z, b.z, op); o.w = upd(a[3], m.w, b.w, op);
        reinterpret_cast<float4*>(master)[v] = m;
        reinterpret_cast<float4*>(mom)[v] = b;
#pragma unroll
        for (int k = 0; k < K; ++k) reinterpret_cast<float4*>(dst + k * ld)[v] = o;
    }
}

// persistent contiguous ranges: workgroup b streams vectors [b*per, (b+1)*per)
template <int K, bool NTL>
__global__ __launch_bounds__(256) void v_persist(const float* src, long ld, long n, float* master, float* mom, OP op,
                                                 float* dst) {
    const long nv = n >> 2;
    const long per = (nv + gridDim.x - 1) / gridDim.x;
    const long lo = (long)blockIdx.x * per;
    const long hi = lo + per < nv ? lo + per : nv;
    for (long v = lo + threadIdx.x; v < hi; v += 256) {
        float4 x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = ld4<NTL>(reinterpret_cast<const float4*>(src + k * ld) + v);
        float4 m = reinterpret_cast<const float4*>(master)[v], b = reinterpret_cast<const float4*>(mom)[v];
        float a[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) { a[0] += x[k].x; a[1] += x[k].y; a[2] += x[k].z; a[3] += x[k].w; }
        float4 o;
        o.x = upd(a[0], m.x, b.x, op); o.y = upd(a[1], m.y, b.y, op);
        o.z = upd(a[2], m.z, b.z, op); o.w = upd(a[3], m.w, b.w, op);
        reinterpret_cast<float4*>(master)[v] = m;
        reinterpret_cast<float4*>(mom)[v] = b;
#pragma unroll
        for (int k = 0; k < K; ++k) reinterpret_cast<float4*>(dst + k * ld)[v] = o;
    }
}

__global__ void copy4(const float4* a, float4* b, long nv) {
    long stride = (long)gridDim.x * blockDim.x;
    for (long v = (long)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) b[v] = a[v];
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
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

// ALLOC=one|split|pad1g|contig: the [K, ld] replica set as one buffer, as K separate
// buffers (row pointers passed in a table), or one buffer with rows 1 GiB apart
template <int K>
__global__ __launch_bounds__(256) void v_rows(const float* const* rows, long n, float* master, float* mom, OP op) {
    const long nv = n >> 2;
    const long lo = (long)blockIdx.x * 1024;
    const long hi = lo + 1024 < nv ? lo + 1024 : nv;
    for (long v = lo + threadIdx.x; v < hi; v += 256) {
        float4 x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = reinterpret_cast<const float4*>(rows[k])[v];
        float4 m = reinterpret_cast<const float4*>(master)[v], b = reinterpret_cast<const float4*>(mom)[v];
        float a[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) { a[0] += x[k].x; a[1] += x[k].y; a[2] += x[k].z; a[3] += x[k].w; }
        float4 o;
        o.x = upd(a[0], m.x, b.x, op); o.y = upd(a[1], m.y, b.y, op);
        o.z = upd(a[2], m.z, b.z, op); o.w = upd(a[3], m.w, b.w, op);
        reinterpret_cast<float4*>(master)[v] = m;
        reinterpret_cast<float4*>(mom)[v] = b;
#pragma unroll
        for (int k = 0; k < K; ++k) reinterpret_cast<float4*>(const_cast<float*>(rows[k]))[v] = o;
    }
}

static int alloc_mode() {
    const char* mode = getenv("ALLOC");
    if (!mode) return -1;
    const int K = 8;
    const long n = 124475904;
    std::vector<float*> rows(K);
    float *master, *mom;
    CK(hipMalloc(&master, sizeof(float) * n));
    CK(hipMalloc(&mom, sizeof(float) * n));
    CK(hipMemset(master, 0, sizeof(float) * n));
    CK(hipMemset(mom, 0, sizeof(float) * n));
    const std::string m(mode);
    if (m == "contig") {  // one buffer, physically contiguous pages requested from the driver
        float* base;
        CK(hipExtMallocWithFlags((void**)&base, sizeof(float) * (K * n), hipDeviceMallocContiguous));
        for (int k = 0; k < K; ++k) rows[k] = base + k * n;
    } else if (m == "split") {
        for (int k = 0; k < K; ++k) CK(hipMalloc(&rows[k], sizeof(float) * n));
    } else {
        const long ld = m == "pad1g" ? (1L << 28) : n;  // 2^28 floats = 1 GiB
        float* base;
        CK(hipMalloc(&base, sizeof(float) * (K * ld)));
        for (int k = 0; k < K; ++k) rows[k] = base + k * ld;
    }
    for (int k = 0; k < K; ++k) CK(hipMemset(rows[k], 0, sizeof(float) * n));
    float** drows;
    CK(hipMalloc(&drows, sizeof(float*) * K));
    CK(hipMemcpy(drows, rows.data(), sizeof(float*) * K, hipMemcpyHostToDevice));
    OP op{8.f, 0.7f, 0.9f};
    const double bytes = (2.0 * K + 4.0) * 4.0 * n;
    const int g = (int)((n / 4 + 1023) / 1024);
    float ms = time_ms([&] { v_rows<K><<<g, 256>>>(drows, n, master, mom, op); }, 20);
    printf("alloc=%s %.3f ms %.0f GB/s\n", mode, ms, bytes / ms / 1e6);
    return 0;
}

int main() {
    if (alloc_mode() == 0) return 0;
    const int K = 8;
    const long n = 124475904;  // GPT-2 124M arena
    const long ld = n;
    float *src, *master, *mom;
    CK(hipMalloc(&src, sizeof(float) * K * ld));
    CK(hipMalloc(&master, sizeof(float) * n));
    CK(hipMalloc(&mom, sizeof(float) * n));
    CK(hipMemset(src, 0, sizeof(float) * K * ld));
    CK(hipMemset(master, 0, sizeof(float) * n));
    CK(hipMemset(mom, 0, sizeof(float) * n));
    OP op{8.f, 0.7f, 0.9f};
    const double bytes = (2.0 * K + 4.0) * 4.0 * n;
    const int reps = 20;
    {
        float* cdst;
        CK(hipMalloc(&cdst, sizeof(float) * 2 * n));
        for (int g : {1024, 2048, 4096, 8192}) {
            float ms = time_ms([&] { copy4<<<g, 256>>>((const float4*)src, (float4*)cdst, 2 * n / 4); }, reps);
            printf("copy float4 2x%.0fMB grid %5d: %.3f ms  %.0f GB/s\n", 4.0 * n / 1e6, g, ms, 2 * 8.0 * n / ms / 1e6);
        }
        CK(hipFree(cdst));
    }
    for (int g : {2048, 4096, 8192}) {
        float ms = time_ms([&] { v_runtime<<<g, 256>>>(src, K, ld, n, master, mom, op, src); }, reps);
        printf("runtime-K       grid %5d: %.3f ms  %.0f GB/s\n", g, ms, bytes / ms / 1e6);
    }
#define RUN(U, NTL, NTS)                                                                                  \
    for (int g : {1024, 2048, 4096, 8192, 16384}) {                                                     \
        float ms = time_ms([&] { v_static<K, U, NTL, NTS><<<g, 256>>>(src, ld, n, master, mom, op, src); }, reps); \
        printf("static U=%d ntl=%d nts=%d grid %5d: %.3f ms  %.0f GB/s\n", U, NTL, NTS, g, ms, bytes / ms / 1e6); \
    }
#define RUNC(CH, U, NTS)                                                                                   \
    {                                                                                                     \
        int g = (int)((n / 4 + CH - 1) / CH);                                                             \
        float ms = time_ms([&] { v_chunk<K, CH, U, NTS><<<g, 256>>>(src, ld, n, master, mom, op, src); }, reps); \
        printf("chunk CH=%d U=%d nts=%d grid %6d: %.3f ms  %.0f GB/s\n", CH, U, NTS, g, ms, bytes / ms / 1e6); \
    }
#define RUNP(G, NTL)                                                                                     \
    {                                                                                                     \
        float ms = time_ms([&] { v_persist<K, NTL><<<G, 256>>>(src, ld, n, master, mom, op, src); }, reps);  \
        printf("persist G=%d ntl=%d: %.3f ms  %.0f GB/s\n", G, NTL, ms, bytes / ms / 1e6);                 \
    }
#define RUNX(CH)                                                                                          \
    {                                                                                                     \
        int g = (int)(((n / 4 + CH - 1) / CH + 7) / 8 * 8);                                               \
        float ms = time_ms([&] { v_chunk_xcd<K, CH><<<g, 256>>>(src, ld, n, master, mom, op, src); }, reps); \
        printf("chunk-xcd CH=%d grid %6d: %.3f ms  %.0f GB/s\n", CH, g, ms, bytes / ms / 1e6);           \
    }
    if (getenv("XCD_AB")) {
        for (int rep = 0; rep < 3; ++rep) {
            RUNC(1024, 1, false)
            RUNX(1024)
            RUNX(2048)
            RUNX(512)
        }
        return 0;
    }
    RUNP(512, false)
    RUNP(1024, false)
    RUNP(2048, false)
    RUNP(4096, false)
    RUNP(1024, true)
    RUNP(2048, true)
    RUNC(1024, 1, false)
    RUNC(1024, 1, false)
    RUNC(512, 1, false)
    RUNC(2048, 1, false)
    RUNC(4096, 1, false)
    RUNC(1024, 2, false)
    RUNC(2048, 2, false)
    RUNC(1024, 1, true)
    RUNC(2048, 2, true)
    if (getenv("ONLY_CHUNK")) return 0;
    RUN(1, false, false)
    RUN(2, false, false)
    RUN(1, false, true)
    RUN(1, true, true)
    RUN(2, true, true)
    RUN(1, true, false)
    return 0;
}
