// Shared device helpers and error plumbing for libgym_amd (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/gym_amd.h"

namespace ga {

// ---- error string (thread local, set by the failing entry point) ----------
void set_error(const char* fmt, ...);
void clear_error();

#define GA_REQUIRE(cond, ...)                        \
    do {                                             \
        if (!(cond)) {                               \
            ::ga::set_error(__VA_ARGS__);            \
            return GA_EINVAL;                        \
        }                                            \
    } while (0)

// Checks the launch that was just enqueued.
int check_launch(const char* what);

// ---- element access: arenas are f32 or bf16, arithmetic is f32 ------------
template <typename T> struct Elem;
template <> struct Elem<float> {
    static __device__ __forceinline__ float load(const float* p) { return *p; }
    static __device__ __forceinline__ void store(float* p, float v) { *p = v; }
};
template <> struct Elem<__hip_bfloat16> {
    static __device__ __forceinline__ float load(const __hip_bfloat16* p) {
        return __bfloat162float(*p);
    }
    static __device__ __forceinline__ void store(__hip_bfloat16* p, float v) {
        *p = __float2bfloat16(v);  // round to nearest even; NaN stays NaN
    }
};

// 16-byte vector of 4 elements for f32, 8-byte for bf16.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
    using type = float4;
    static __device__ __forceinline__ void unpack(const float4& v, float (&f)[4]) {
        f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
    }
    static __device__ __forceinline__ float4 pack(const float (&f)[4]) {
        return make_float4(f[0], f[1], f[2], f[3]);
    }
};
template <> struct Vec4<__hip_bfloat16> {
    using type = uint2;  // 4 x bf16
    static __device__ __forceinline__ void unpack(const uint2& v, float (&f)[4]) {
        f[0] = __uint_as_float(v.x << 16);
        f[1] = __uint_as_float(v.x & 0xffff0000u);
        f[2] = __uint_as_float(v.y << 16);
        f[3] = __uint_as_float(v.y & 0xffff0000u);
    }
    static __device__ __forceinline__ uint2 pack(const float (&f)[4]) {
        __hip_bfloat16 b[4];
        for (int i = 0; i < 4; ++i) b[i] = __float2bfloat16(f[i]);
        uint2 r;
        r.x = (uint32_t)__bfloat16_as_ushort(b[0]) | ((uint32_t)__bfloat16_as_ushort(b[1]) << 16);
        r.y = (uint32_t)__bfloat16_as_ushort(b[2]) | ((uint32_t)__bfloat16_as_ushort(b[3]) << 16);
        return r;
    }
};

// Non-temporal (streaming) vector loads and stores for data touched once per
// launch: a float4 copy of 4.6 GiB runs 5.96 TB/s with both hinted against
// 5.67 TB/s plain (tools/ubench_copy_nt.hip, profiles/r02z_ubench_copy_nt.txt).
typedef float ga_f4 __attribute__((ext_vector_type(4)));
typedef unsigned int ga_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 stream_load(const float4* p) {
    const ga_f4 v = __builtin_nontemporal_load(reinterpret_cast<const ga_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 stream_load(const uint2* p) {
    const ga_u2 v = __builtin_nontemporal_load(reinterpret_cast<const ga_u2*>(p));
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void stream_store(float4* p, const float4& v) {
    ga_f4 w;
    w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
    __builtin_nontemporal_store(w, reinterpret_cast<ga_f4*>(p));
}
__device__ __forceinline__ void stream_store(uint2* p, const uint2& v) {
    ga_u2 w;
    w.x = v.x; w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<ga_u2*>(p));
}

// Device-scope (sc1) vector stores for streams written once per launch: the
// store goes out through buffer_store_dwordx4/x2 ... sc1 with the descriptor based
// at a WAVE-UNIFORM pointer (a workgroup's block of one row) and the lane's byte
// offset from it (< 2 GiB).  On MI355X a copy with nt loads and sc1 stores ran
// 5.91-5.93 TB/s against 5.64-5.68 TB/s with nt stores
// (tools/ubench_ldsdma.hip, profiles/r03k_ubench_store_policy.txt).
__device__ __forceinline__ void store_sc1(float4* wg_base, uint32_t idx, const float4& v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wg_base, 0, 0x7fffffff, 0x00020000);
    ga_f4 w;
    w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
    __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(idx * 16u), 0, 16);
}
__device__ __forceinline__ void store_sc1(uint2* wg_base, uint32_t idx, const uint2& v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wg_base, 0, 0x7fffffff, 0x00020000);
    ga_u2 w;
    w.x = v.x; w.y = v.y;
    __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)(idx * 8u), 0, 16);
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid size for a grid-stride streaming kernel: enough workgroups to fill
// 256 CUs several times over, capped so the tail stays short.
inline int stream_grid(int64_t work_items, int block) {
    int64_t g = ceil_div(work_items, block);
    if (g > 256 * 16) g = 256 * 16;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace ga
