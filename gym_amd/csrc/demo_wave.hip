// DeMo encode, register-resident wave-per-chunk form (ga_demo_encode_sym).
//
// Same contract and arithmetic as ga_demo_encode (demo.hip; demo.py:142-209),
// for plans whose chunks are all 64x64 or 1x64 with k <= 64 -- DeMo's
// compression_chunk = 64 on GPT-2-shaped models.  One wavefront owns a whole
// 64x64 chunk and keeps it in registers from the load to the delta store: no
// workgroup barrier in the chunk loop, and LDS only for the shared half basis
// and the top-k candidate list.  The 8 waves of a CU (2 per SIMD) interleave
// freely, one wave's MFMA chain running while another waits on its loads.
//
// Lane (l, h) = (lane & 31, lane >> 5) holds data rows l and 63 - l, columns
// S_h (eight 4-column blocks BL_h: h = 0 -> blocks 0-3, 12-15; h = 1 -> 4-11),
// a set closed under j -> 63 - j.  With the DCT symmetry
// F[63 - i][k] = (-1)^k F[i][k] every product is a 32-deep MFMA chain whose
// register operand is already in the right lane:
//   T  = X . F2   per row pair: A = x[j] +- x[63 - j] (own registers),
//                 B = F[j][2d' + qc] (LDS)               4 x 16 MFMAs
//   Y  = F1^T . T: B = T[i] +- T[63 - i] (own accumulators; rows l and 63 - l
//                 sit in the same register of the same lane), A = F[i][2b' + p]
//                                                        4 x 16 MFMAs
//   R^T = sum_e (v_e F[c][d_e]) (x) F[i][b_e] per parity of b_e, so that R
//                 lands in the load layout (column c = pi(m) of accumulator row
//                 m is the lane's own column); rows 63 - l by the symmetry
//                                                        ~k + 2 MFMAs
// 1x64 chunks (vectors) are processed 64 at a time (a "row group", rows =
// consecutive chunks): the same row product, then a per-lane exact top-k over
// the lane's own row through one LDS tile, and the residual as a dense
// R^T = F . Ymask^T product.
//
// Top-k (demo.py:315-328) is exact with ties to the lowest index; a chunk's
// entries are emitted in ascending coefficient index, as ga_demo_encode.
#include "ga_common.h"

namespace ga {
namespace dw {

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kLd = 65;     // LDS row stride (basis, row-group tile)
constexpr int kCand = 128;  // fast-path candidate capacity
static_assert(2 * (kCand + 64) >= 320, "the fallback top-k keeps its maps in lst[128..319]");

typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifdef GA_DEMO_STAMPS
extern __device__ unsigned long long* g_demo_stamps_w;
#define DW_PH_DECL unsigned long long ph_acc[16] = {}, ph_last = __builtin_amdgcn_s_memtime()
#define DW_PH(i)                                                    \
    do {                                                            \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph_acc[i] += t_ - ph_last;                                  \
        ph_last = t_;                                               \
    } while (0)
#define DW_CNT(i) (ph_acc[i] += 1)
#define DW_PH_FLUSH()                                                                                       \
    do {                                                                                                    \
        if ((threadIdx.x & 63) == 0) {                                                                      \
            unsigned long long* row_ = g_demo_stamps_w + ((size_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * 16; \
            for (int i_ = 0; i_ < 16; ++i_) row_[i_] = ph_acc[i_];                                          \
        }                                                                                                   \
    } while (0)
#else
#define DW_PH_DECL do {} while (0)
#define DW_PH(i) do {} while (0)
#define DW_CNT(i) do {} while (0)
#define DW_PH_FLUSH() do {} while (0)
#endif

// Lanes of one wave hand data to each other through LDS: keep the compiler
// from moving this lane's LDS accesses across the hand-off (the hardware runs
// a wave's LDS operations in order).
#define WAVE_LDS_SYNC() asm volatile("" ::: "memory")

__device__ __forceinline__ int lane_id() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));  // not hoisted out of the chunk loop (see demo.hip opaque_tid)
    return t & 63;
}

__device__ __forceinline__ f32x16 zero16() {
    f32x16 a;
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.f;
    return a;
}

__device__ __forceinline__ f32x16 mfma(float a, float b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// accumulator register r of lane half h: row (r & 3) + 8 (r >> 2) + 4 h of the 32x32 block
__device__ __forceinline__ constexpr int rowmap(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// column block q (0..7) of lane half h
__device__ __forceinline__ int blk(int h, int q) { return h ? 4 + q : (q < 4 ? q : 8 + q); }

// data column of residual accumulator half H, accumulator row m (the lane's own column, see header)
__device__ __forceinline__ int pi_col(int H, int m) { return 4 * blk((m >> 2) & 1, 4 * H + (m >> 3)) + (m & 3); }

// F[i][d] (0 <= i < 64) from the half table H = F[0..31][:]
__device__ __forceinline__ float basis64(const float* Hb, int i, int d) {
    const float v = Hb[(i < 32 ? i : 63 - i) * kLd + d];
    return (i >= 32 && (d & 1)) ? -v : v;
}

__device__ __forceinline__ uint32_t keyv(float v) { return (__float_as_uint(v) & 0x7fffffffu) + 1u; }

// exclusive prefix sum over the wave of a per-lane value 0 <= v < 128, bit-sliced:
// ballots and mbcnt only (no LDS round trips)
__device__ __forceinline__ int wave_excl_scan128(int v) {
    int r = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const uint64_t m = __ballot((v >> b) & 1);
        r += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    }
    return r;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Largest descriptor index t >= max(tix, 0) with chunk_start <= chunk (chunk_start
// increases): a uniform binary search on scalar loads (no vector memory operation)
__device__ __forceinline__ int find_tensor(const ga_demo_tensor* __restrict__ T, int ntens, int tix, int chunk) {
    int lo = tix < 0 ? 0 : tix, hi = ntens - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (T[mid].chunk_start <= chunk) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// The several-source decode's second half of waves (w >= 4: the partner of wave
// w - 4 on its SIMD, the arbitration loser by age) runs at static priority 1: at
// 350M in one process 8 sources 1.003 -> 0.958 ms, 2 sources 0.825 -> 0.817 ms, but
// one source 0.811 -> 0.844 ms, so only for S >= 2 (profiles/r06f_ab_demo_decode_prio.txt;
// MI355X_MICROARCH.md, two waves per SIMD, item 4).  The encode measured no gain
// from it, nor from a start stagger of the second half (profiles/r06e_ab_demo_wave_sched.txt).
// (one asm statement holding its own scalar branch: a branch in the kernel's control
// flow here made the register allocator spill 124 B/lane in the chunk loop)
__device__ __forceinline__ void decode_wave_priority() {
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    asm volatile("s_cmp_lt_u32 %0, 4\n\ts_cbranch_scc1 1f\n\ts_setprio 1\n1:" ::"s"(w) : "scc");
}

__device__ __forceinline__ uint32_t rdl(uint32_t v, int j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, j);
}

struct ListLDS {
    uint32_t lst[2 * (kCand + 64)];  // candidates (pos, bits); slots kCand + lane: discard
    uint32_t bm[128];                // 4096-bit position bitmap
    uint32_t sm[4];                  // 128-bit rank-space selection mask
};

struct WaveLDS : ListLDS {
    float tile[64 * kLd];  // 64x64 chunks: x, then delta (float4 t4 layout); row groups: T, then the masked coefficients
};

// ---- operands in registers --------------------------------------------------
// x[s][q][e]: row l (s = 0) or 63 - l (s = 1), column 4 blk(h, q) + e
// lane offset of x[s][q][0] from the chunk's (0, 0) element (32-bit: a chunk spans < 2^31 elements)
__device__ __forceinline__ uint32_t lane_off(int s, int q, int l, int h, int stride) {
    return (uint32_t)((s ? 63 - l : l) * stride + 4 * blk(h, q));
}

// uniform base + zero-extended 32-bit lane byte offset: global_load/store with an SGPR base
template <typename T>
__device__ __forceinline__ const T* at_off(const T* pb, uint32_t off) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(pb) + (uint64_t)(uint32_t)(off * (uint32_t)sizeof(T)));
}
template <typename T>
__device__ __forceinline__ T* at_off(T* pb, uint32_t off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(pb) + (uint64_t)(uint32_t)(off * (uint32_t)sizeof(T)));
}

template <typename T>
__device__ __forceinline__ void load_rows(const T* pb, int stride, int l, int h, bool vec, int nrows,
                                          float (&o)[2][8][4]) {
    if (vec && nrows == 64) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int q = 0; q < 8; ++q)
                Vec4<T>::unpack(*reinterpret_cast<const typename Vec4<T>::type*>(at_off(pb, lane_off(s, q, l, h, stride))),
                                o[s][q]);
        return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const bool live = (s ? 63 - l : l) < nrows;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const T* a = at_off(pb, lane_off(s, q, l, h, stride));
            if (live && vec) {
                Vec4<T>::unpack(*reinterpret_cast<const typename Vec4<T>::type*>(a), o[s][q]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) o[s][q][e] = live ? Elem<T>::load(a + e) : 0.f;
            }
        }
    }
}

template <typename T>
__device__ __forceinline__ void store_rows(T* pb, int stride, int l, int h, bool vec, int nrows,
                                           const float (&o)[2][8][4]) {
    if (vec && nrows == 64) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int q = 0; q < 8; ++q)
                *reinterpret_cast<typename Vec4<T>::type*>(at_off(pb, lane_off(s, q, l, h, stride))) = Vec4<T>::pack(o[s][q]);
        return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        if ((s ? 63 - l : l) >= nrows) continue;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            T* a = at_off(pb, lane_off(s, q, l, h, stride));
            if (vec) {
                *reinterpret_cast<typename Vec4<T>::type*>(a) = Vec4<T>::pack(o[s][q]);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) Elem<T>::store(a + e, o[s][q][e]);
            }
        }
    }
}

// x = decay*delta + lr*grad (+ p *= wd_factor): demo.py:159-167, same rounding as ga_demo_encode
template <typename T>
__device__ __forceinline__ void error_feedback(T* param, const T* grad, const T* delta, int stride, int l, int h,
                                               bool vec, int nrows, float lr, float decay, float wd_factor,
                                               float (&x)[2][8][4]) {
    if (wd_factor != 1.f) {  // its own pass: p is read and written before d, g are loaded
        load_rows(param, stride, l, h, vec, nrows, x);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) x[s][q][e] *= wd_factor;
        store_rows(param, stride, l, h, vec, nrows, x);
    }
    float g[2][8][4];
    load_rows(delta, stride, l, h, vec, nrows, x);
    load_rows(grad, stride, l, h, vec, nrows, g);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e)
                x[s][q][e] = fmaf(lr, g[s][q][e], decay != 1.f ? x[s][q][e] * decay : x[s][q][e]);
}

// T[s][qc] = rows of X (s = 0: rows l, 1: rows 63 - l) times F2, even (qc = 0) or
// odd (qc = 1) frequencies d = 2 col + qc; K index of step t, half h: column 16h + t
__device__ __forceinline__ void row_product_half(const float (&xs)[8][4], const float* Hb, int l, int h,
                                                 f32x16 (&Ts)[2]) {
#pragma unroll
    for (int qc = 0; qc < 2; ++qc) {
        f32x16 acc = zero16();
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int q = t >> 2, e = t & 3;
            const float u = xs[q][e], w = xs[7 - q][3 - e];
            const float a = qc ? u - w : u + w;
            acc = mfma(a, Hb[(16 * h + t) * kLd + 2 * l + qc], acc);
        }
        Ts[qc] = acc;
    }
}

__device__ __forceinline__ void row_product(const float (&x)[2][8][4], const float* Hb, int l, int h,
                                            f32x16 (&T)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int qc = 0; qc < 2; ++qc) {
            f32x16 acc = zero16();
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int q = t >> 2, e = t & 3;
                const float u = x[s][q][e], w = x[s][7 - q][3 - e];
                const float a = qc ? u - w : u + w;
                acc = mfma(a, Hb[(16 * h + t) * kLd + 2 * l + qc], acc);
            }
            T[s][qc] = acc;
        }
    }
}

// ---- sparse synthesis R = sum_e v_e F[:, b_e] (x) F[:, d_e] in the row-pair layout ----
// The entries (one per lane where `ent`) as per-parity-of-b lists lstp[par * 64 + i], each
// padded with a zero entry to whole pairs; np0 / np1 = entry pairs per list.
constexpr int kSynB = 4;  // entry pairs per synthesis batch (LDS reads issued ahead of the MFMAs)

__device__ __forceinline__ void parity_lists(uint32_t epos, uint32_t ebits, bool ent, int lane, uint2* lstp,
                                             int& np0, int& np1) {
    const int pl = (int)((epos >> 6) & 1u);
    const uint64_t m0 = __ballot(ent && pl == 0), m1 = __ballot(ent && pl == 1);
    const uint64_t mm = pl ? m1 : m0;
    const int ix = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
    const int E0 = __popcll(m0), E1 = __popcll(m1);
    const int P0 = (E0 + 1) & ~1, P1 = (E1 + 1) & ~1;  // <= 64
    WAVE_LDS_SYNC();
    if (ent) lstp[pl * 64 + ix] = make_uint2(epos, ebits);
    if (lane == 0 && E0 < P0) lstp[E0] = make_uint2(0u, 0u);  // zero partners
    if (lane == 1 && E1 < P1) lstp[64 + E1] = make_uint2(0u, 0u);
    WAVE_LDS_SYNC();
    np0 = P0 >> 1;
    np1 = P1 >> 1;
}

// B pairs of one parity list into acc: the entry and basis reads go out together,
// then the MFMAs (lane half h takes entry 2q + h)
template <int B>
__device__ __forceinline__ void synth_batch(const uint2* lst, int q, int cH, int l, int h, const float* Hb,
                                            f32x16& acc) {
    uint2 e[B];
#pragma unroll
    for (int u = 0; u < B; ++u) e[u] = lst[2 * (q + u) + h];
    float a[B], b[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
        const int bq = (int)(e[u].x >> 6), dq = (int)(e[u].x & 63);
        a[u] = __uint_as_float(e[u].y) * basis64(Hb, cH, dq);
        b[u] = Hb[l * kLd + bq];
    }
#pragma unroll
    for (int u = 0; u < B; ++u) acc = mfma(a[u], b[u], acc);
}

// one parity list's sum into acc: kSynB pairs per batch, then the 0..kSynB-1 left
// (whole pairs only: no MFMA spent on padding beyond one zero entry)
__device__ __forceinline__ void synth_list(const uint2* lst, int np, int cH, int l, int h, const float* Hb,
                                           f32x16& acc) {
    static_assert(kSynB == 2 || kSynB == 4 || kSynB == 8, "synthesis tail handles 4/2/1 pairs");
    int q = 0;
    for (; q + kSynB <= np; q += kSynB) synth_batch<kSynB>(lst, q, cH, l, h, Hb, acc);
    const int rem = np - q;  // < kSynB
    if (kSynB > 4 && (rem & 4)) {
        synth_batch<4>(lst, q, cH, l, h, Hb, acc);
        q += 4;
    }
    if (kSynB > 2 && (rem & 2)) {
        synth_batch<2>(lst, q, cH, l, h, Hb, acc);
        q += 2;
    }
    if (rem & 1) synth_batch<1>(lst, q, cH, l, h, Hb, acc);
}

// R^T of column half H per parity of b: lane (l, h) register 4qq + e holds the parity
// sums for rows l (Re + Ro) and 63 - l (Re - Ro), column 4 blk(h, 4H + qq) + e
__device__ __forceinline__ void synth_half(const uint2* lstp, int np0, int np1, int H, int l, int h,
                                           const float* Hb, f32x16& Re, f32x16& Ro) {
    const int cH = pi_col(H, l);
    Re = zero16();
    Ro = zero16();
    synth_list(lstp, np0, cH, l, h, Hb, Re);
    synth_list(lstp + 64, np1, cH, l, h, Hb, Ro);
}

// ---- 64x64 chunk ------------------------------------------------------------
// Global memory is read and written in the coalesced layout C -- lane t holds rows
// (t >> 4) + 4i (i < 16), 4 elements at column 4 (t & 15): each access covers 4
// whole 256-byte row segments -- and the chunk goes through the LDS tile into the
// row-pair layout of the products (a direct row-pair access touches 64 lines per
// instruction and runs ~20% slower).
__device__ __forceinline__ uint32_t coal_off(int i, int lane, int stride) {
    return (uint32_t)(((lane >> 4) + 4 * i) * stride + 4 * (lane & 15));
}

template <typename T, int I0 = 0, int NI = 16>
__device__ __forceinline__ void load_coal(const T* pb, int stride, bool vec, int lane, float (&o)[16][4]) {
    if (vec) {
#pragma unroll
        for (int i = I0; i < I0 + NI; ++i)
            Vec4<T>::unpack(*reinterpret_cast<const typename Vec4<T>::type*>(at_off(pb, coal_off(i, lane, stride))),
                            o[i]);
    } else {
#pragma unroll
        for (int i = I0; i < I0 + NI; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) o[i][e] = Elem<T>::load(at_off(pb, coal_off(i, lane, stride)) + e);
    }
}

template <typename T>
__device__ __forceinline__ void store_vec(T* pb, uint32_t off, const typename Vec4<T>::type& v) {
    *reinterpret_cast<typename Vec4<T>::type*>(at_off(pb, off)) = v;
}

template <typename T>
__device__ __forceinline__ void store_coal(T* pb, int stride, bool vec, int lane, const float (&o)[16][4]) {
    if (vec) {
#pragma unroll
        for (int i = 0; i < 16; ++i) store_vec(pb, coal_off(i, lane, stride), Vec4<T>::pack(o[i]));
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) Elem<T>::store(at_off(pb, coal_off(i, lane, stride)) + e, o[i][e]);
    }
}

// float4 index of (row, column block cb) in the chunk tile: row-major, blocks XOR-swizzled
// by row, so whole-row (layout C) and row-pair (l, h) accesses are both bank-conflict free
__device__ __forceinline__ int t4(int row, int cb) { return row * 16 + (cb ^ (row & 15)); }


// top-k of the chunk's coefficients Y (register t = 32 par + 16 qc + r: coefficient
// b = 2 rowmap(r, h) + par, d = 2 l + qc), the payload, the residual delta = x - R in
// the tile (x in the float4 t4 layout) and the coalesced delta store
template <typename T>
__device__ __forceinline__ void chunk64_tail(const f32x16 (&Y)[2][2], int k, T* delta, int cols, bool vec,
                                             int32_t* out_idx, float* out_val, const float* Hb, ListLDS& W,
                                             float4* tile
#ifdef GA_DEMO_STAMPS
                                             , unsigned long long (&ph_acc)[16], unsigned long long& ph_last
#endif
) {
    // ---- top-k: register t = 32 par + 16 qc + r holds coefficient
    //      b = 2 rowmap(r, h) + par, d = 2 l + qc
    const int lane = lane_id(), l = lane & 31, h = lane >> 5;
    // the top-k's chain of ballot rounds and LDS round trips at raised priority: the
    // partner wave's products fill its gaps, not the other way round (encode -0.8 to
    // -1.4% in 12 same-process pairs, profiles/r06ah_ab_demo_encode_topk_priority.txt)
    __builtin_amdgcn_s_setprio(1);
    auto posof = [&](int par, int qc, int r) -> uint32_t {
        return (uint32_t)((2 * rowmap(r, h) + par) * 64 + 2 * l + qc);
    };
    // |v| >= f(T) <=> keyv(v) >= T with f(T) = as_float(T - 1) (non-NaN v; abs is a free operand modifier)
    float mymaxf = 0.f;
#pragma unroll
    for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int qc = 0; qc < 2; ++qc)
#pragma unroll
            for (int r = 0; r < 16; ++r) mymaxf = fmaxf(mymaxf, fabsf(Y[par][qc][r]));
    const uint32_t mymax = keyv(mymaxf);
    uint32_t T0 = 0;
#pragma unroll
    for (int bit = 30; bit >= 19; --bit) {
        const uint32_t cnd = T0 | (1u << bit);
        if (__popcll(__ballot(mymax >= cnd)) >= k) T0 = cnd;
    }
    if (T0 == 0u) T0 = 1u;
    const float T0f = __uint_as_float(T0 - 1u);
    int mine = 0;
#pragma unroll
    for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int qc = 0; qc < 2; ++qc)
#pragma unroll
            for (int r = 0; r < 16; ++r) mine += fabsf(Y[par][qc][r]) >= T0f ? 1 : 0;
    const int excl = wave_excl_scan128(mine);  // mine <= 64
    const int incl = excl + mine;
    const int C = __builtin_amdgcn_readlane(incl, 63);
    DW_PH(10);
    W.bm[2 * lane] = 0u;
    W.bm[2 * lane + 1] = 0u;
    if (C <= kCand) {
        uint2* L2 = reinterpret_cast<uint2*>(W.lst);
        float T0c = T0f;  // an opaque copy: the 64 compares are redone here, not kept as 64 lane masks
        asm volatile("" : "+v"(T0c));
        // compact the candidates: (pos, bits) at the lane's next slot, others to its discard slot
        int at = excl;
#pragma unroll
        for (int par = 0; par < 2; ++par)
#pragma unroll
            for (int qc = 0; qc < 2; ++qc)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = Y[par][qc][r];
                    const bool cnd = fabsf(v) >= T0c;
                    L2[cnd ? at : kCand + lane] = make_uint2(posof(par, qc, r), __float_as_uint(v));
                    at += cnd ? 1 : 0;
                }
        WAVE_LDS_SYNC();
        DW_PH(11);
        uint32_t pos[2], bits[2], key[2];
        bool ok[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int g = e * 64 + lane;
            ok[e] = g < C;
            const uint2 pb = L2[ok[e] ? g : kCand + lane];
            pos[e] = ok[e] ? pb.x : 0u;
            bits[e] = pb.y;
            key[e] = ok[e] ? keyv(__uint_as_float(pb.y)) : 0u;
            if (ok[e]) atomicOr(&W.bm[pos[e] >> 5], 1u << (pos[e] & 31));
        }
        WAVE_LDS_SYNC();
        // rank of a candidate = candidates at lower positions (bitmap prefix counts)
        const uint32_t w0 = W.bm[2 * lane], w1 = W.bm[2 * lane + 1];
        const int cnt = __popc(w0) + __popc(w1);
        const int pre = wave_excl_scan128(cnt);  // cnt <= 64
        int rank[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int Lw = (int)(pos[e] >> 6);  // every lane takes part in the shuffles
            const uint64_t pair = ((uint64_t)(uint32_t)__shfl((int)w1, Lw, 64) << 32) |
                                  (uint32_t)__shfl((int)w0, Lw, 64);
            const int preL = __shfl(pre, Lw, 64);
            rank[e] = ok[e] ? preL + __popcll(pair & ((1ull << (pos[e] & 63)) - 1ull)) : 0x7fff;
        }
        DW_PH(12);
        // exact k-th key among the candidates
        uint32_t thr = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t cnd = thr | (1u << bit);
            if (__popcll(__ballot(key[0] >= cnd)) + __popcll(__ballot(key[1] >= cnd)) >= k) thr = cnd;
        }
        const int need = k - __popcll(__ballot(key[0] > thr)) - __popcll(__ballot(key[1] > thr));
        const uint64_t q0 = __ballot(key[0] == thr), q1 = __ballot(key[1] == thr);
        bool sel[2];
        if (__popcll(q0) + __popcll(q1) == need) {
            sel[0] = key[0] >= thr;
            sel[1] = key[1] >= thr;
        } else {  // ties at the k-th key: the lowest positions (ranks) win
            int tr[2] = {0, 0};
            for (uint64_t m = q0; m; m &= m - 1) {
                const int rj = __builtin_amdgcn_readlane(rank[0], __builtin_ctzll(m));
                tr[0] += rj < rank[0];
                tr[1] += rj < rank[1];
            }
            for (uint64_t m = q1; m; m &= m - 1) {
                const int rj = __builtin_amdgcn_readlane(rank[1], __builtin_ctzll(m));
                tr[0] += rj < rank[0];
                tr[1] += rj < rank[1];
            }
            sel[0] = key[0] > thr || (key[0] == thr && tr[0] < need);
            sel[1] = key[1] > thr || (key[1] == thr && tr[1] < need);
        }
        DW_PH(13);
        if (lane < 4) W.sm[lane] = 0u;
        WAVE_LDS_SYNC();
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (sel[e]) atomicOr(&W.sm[rank[e] >> 5], 1u << (rank[e] & 31));
        WAVE_LDS_SYNC();
        const uint64_t m0 = ((uint64_t)W.sm[1] << 32) | W.sm[0], m1 = ((uint64_t)W.sm[3] << 32) | W.sm[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            if (sel[e]) {
                const int r = rank[e];
                const int slot = r < 64 ? __popcll(m0 & ((1ull << r) - 1ull))
                                        : __popcll(m0) + __popcll(m1 & ((1ull << (r - 64)) - 1ull));
                W.lst[2 * slot] = pos[e];  // slots < k <= 64 <= the candidates' own range
                W.lst[2 * slot + 1] = bits[e];
                out_idx[slot] = (int32_t)pos[e];
                out_val[slot] = __uint_as_float(bits[e]);
            }
        }
        WAVE_LDS_SYNC();
    } else {
        // more than kCand keys >= T0 (flat spectra, all-zero chunks): exact k-th
        // key over all 4096 keys, ties to the lowest positions, slots in position order.
        // Rare, so written for registers, not speed: every loop re-reads Y through an
        // opaque copy and rebuilds positions from an opaque lane base (nothing derived
        // from the 64 coefficients stays live across loops), and the tie ranks come
        // from LDS (bitmap words + per-word prefix counts at lst[128..191]).
        DW_CNT(8);
        auto opq = [](float v) {
            asm volatile("" : "+v"(v));
            return v;
        };
        auto lane_pos = [&]() {  // p = lp + (2 ((r & 3) + 8 (r >> 2)) + par) * 64 + qc
            uint32_t lp = (uint32_t)(512 * h + 2 * l);
            asm volatile("" : "+v"(lp));
            return lp;
        };
        auto pos_c = [](int par, int qc, int r) -> uint32_t {
            return (uint32_t)((2 * ((r & 3) + 8 * (r >> 2)) + par) * 64 + qc);
        };
        uint32_t thr = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t cnd = thr | (1u << bit);
            const float f = __uint_as_float(cnd - 1u);
            int cl = 0;
#pragma unroll
            for (int par = 0; par < 2; ++par)
#pragma unroll
                for (int qc = 0; qc < 2; ++qc)
#pragma unroll
                    for (int r = 0; r < 16; ++r) cl += fabsf(opq(Y[par][qc][r])) >= f ? 1 : 0;
            if (wave_sum(cl) >= k) thr = cnd;
        }
        int gl = 0;
        {
            const uint32_t lp = lane_pos();
#pragma unroll
            for (int par = 0; par < 2; ++par)
#pragma unroll
                for (int qc = 0; qc < 2; ++qc)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t kv = keyv(opq(Y[par][qc][r]));
                        gl += kv > thr ? 1 : 0;
                        if (kv == thr) {
                            const uint32_t p = lp + pos_c(par, qc, r);
                            atomicOr(&W.bm[p >> 5], 1u << (p & 31));
                        }
                    }
        }
        const int need = k - wave_sum(gl);
        WAVE_LDS_SYNC();
        uint32_t* preL = W.lst + 128;  // per 64-position word pair: tied positions before it
        {
            const uint32_t w0 = W.bm[2 * lane], w1 = W.bm[2 * lane + 1];
            preL[lane] = (uint32_t)wave_excl_scan128(__popc(w0) + __popc(w1));
        }
        WAVE_LDS_SYNC();
        // a tied coefficient's tie rank = tied positions below it; the selection goes to
        // a second 4096-bit map at lst[192..319] (the entries written below use lst[0..2k))
        uint32_t* sel = W.lst + 192;
        sel[2 * lane] = 0u;
        sel[2 * lane + 1] = 0u;
        WAVE_LDS_SYNC();
        {
            const uint32_t lp = lane_pos();
#pragma unroll
            for (int par = 0; par < 2; ++par)
#pragma unroll
                for (int qc = 0; qc < 2; ++qc)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t kv = keyv(opq(Y[par][qc][r]));
                        const uint32_t p = lp + pos_c(par, qc, r);
                        bool s = kv > thr;
                        if (kv == thr) {
                            const uint32_t Lw = p >> 6;
                            const uint64_t pair = ((uint64_t)W.bm[2 * Lw + 1] << 32) | W.bm[2 * Lw];
                            const int tr = (int)preL[Lw] + __popcll(pair & ((1ull << (p & 63)) - 1ull));
                            s = tr < need;
                        }
                        if (s) atomicOr(&sel[p >> 5], 1u << (p & 31));
                    }
        }
        WAVE_LDS_SYNC();
        {
            const uint32_t w0 = sel[2 * lane], w1 = sel[2 * lane + 1];
            preL[lane] = (uint32_t)wave_excl_scan128(__popc(w0) + __popc(w1));
        }
        WAVE_LDS_SYNC();
        {
            const uint32_t lp = lane_pos();
#pragma unroll
            for (int par = 0; par < 2; ++par)
#pragma unroll
                for (int qc = 0; qc < 2; ++qc)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t p = lp + pos_c(par, qc, r);
                        const uint32_t Lw = p >> 6;
                        const uint64_t pair = ((uint64_t)sel[2 * Lw + 1] << 32) | sel[2 * Lw];
                        if ((pair >> (p & 63)) & 1ull) {
                            const int slot = (int)preL[Lw] + __popcll(pair & ((1ull << (p & 63)) - 1ull));
                            const float v = opq(Y[par][qc][r]);
                            W.lst[2 * slot] = p;  // slot < k <= 64: below lst[128]
                            W.lst[2 * slot + 1] = __float_as_uint(v);
                            out_idx[slot] = (int32_t)p;
                            out_val[slot] = v;
                        }
                    }
        }
        WAVE_LDS_SYNC();
    }
    DW_PH(3);
    __builtin_amdgcn_s_setprio(0);
    // ---- residual (demo.py:174-180) in the load layout: R^T per parity of b, one
    //      column half H at a time
    uint2* lstp = reinterpret_cast<uint2*>(W.lst);  // [parity][64] entries
    int np0, np1;
    parity_lists(lane < k ? W.lst[2 * lane] : 0u, lane < k ? W.lst[2 * lane + 1] : 0u, lane < k, lane, lstp, np0,
                 np1);
#pragma unroll
    for (int H = 0; H < 2; ++H) {
        f32x16 Re, Ro;
        synth_half(lstp, np0, np1, H, l, h, Hb, Re, Ro);
        // delta = x - R in the tile, at the lane's own blocks 4H .. 4H+3: row l gets
        // Re + Ro, row 63 - l gets Re - Ro
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                float4& v = tile[t4(s ? 63 - l : l, blk(h, 4 * H + qq))];
                float4 o = v;
                const int r = 4 * qq;
                o.x -= s ? Re[r] - Ro[r] : Re[r] + Ro[r];
                o.y -= s ? Re[r + 1] - Ro[r + 1] : Re[r + 1] + Ro[r + 1];
                o.z -= s ? Re[r + 2] - Ro[r + 2] : Re[r + 2] + Ro[r + 2];
                o.w -= s ? Re[r + 3] - Ro[r + 3] : Re[r + 3] + Ro[r + 3];
                v = o;
            }
        DW_PH(4);
    }
    WAVE_LDS_SYNC();
    {  // delta, coalesced
        float o[16][4];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
            o[i][0] = v.x;
            o[i][1] = v.y;
            o[i][2] = v.z;
            o[i][3] = v.w;
        }
        store_coal(delta, cols, vec, lane, o);
    }
    WAVE_LDS_SYNC();
    DW_PH(5);
}

template <typename T>
__device__ __forceinline__ void chunk64(const ga_demo_tensor& td, int c, T* param, const T* grad, T* delta,
                                        int32_t* out_idx, float* out_val, float lr, float decay, float wd_factor,
                                        int ptr_vec, const float* Hb, WaveLDS& W
#ifdef GA_DEMO_STAMPS
                                        , unsigned long long (&ph_acc)[16], unsigned long long& ph_last
#endif
) {
    const int cy = c / td.gx, cx = c - cy * td.gx;
    const int64_t base = td.offset + (int64_t)cy * 64 * td.cols + (int64_t)cx * 64;
    param += base;
    grad += base;
    delta += base;
    const bool vec = ptr_vec && (td.offset % 4 == 0) && (td.cols % 4 == 0);
    float4* tile = reinterpret_cast<float4*>(W.tile);  // x, then delta, in the swizzled row-major layout
    {
        const int lane = lane_id();
        if (wd_factor != 1.f) {  // decoupled weight decay of p (demo.py:159-160), its own pass
            float pv[16][4];
            load_coal(param, td.cols, vec, lane, pv);
#pragma unroll
            for (int i = 0; i < 16; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) pv[i][e] *= wd_factor;
            store_coal(param, td.cols, vec, lane, pv);
        }
    }
    f32x16 Y[2][2];  // [parity of b][qc]
    {
        // rows 0-31 (row-quads 0-7) are loaded ahead of rows 32-63, so the first
        // half's row product runs while the second half is still in flight (the
        // chunk's loads go out at raised priority, ahead of the partner wave's
        // transforms; the products themselves stay at priority 0)
        const int lane = lane_id(), l = lane & 31, h = lane >> 5;
        float Dv[16][4], Gv[16][4];
        __builtin_amdgcn_s_setprio(2);
        load_coal<T, 0, 8>(delta, td.cols, vec, lane, Dv);
        load_coal<T, 0, 8>(grad, td.cols, vec, lane, Gv);
        __builtin_amdgcn_sched_barrier(0);  // issue order = vmcnt order: first half first
        load_coal<T, 8, 8>(delta, td.cols, vec, lane, Dv);
        load_coal<T, 8, 8>(grad, td.cols, vec, lane, Gv);
#pragma unroll
        for (int i = 0; i < 8; ++i)  // the first half is consumed only after every load is out
            asm volatile("" : "+v"(Dv[i][0]), "+v"(Dv[i][1]), "+v"(Dv[i][2]), "+v"(Dv[i][3]), "+v"(Gv[i][0]),
                              "+v"(Gv[i][1]), "+v"(Gv[i][2]), "+v"(Gv[i][3])::"memory");
        __builtin_amdgcn_s_setprio(0);
        f32x16 Tm[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int i = 8 * s; i < 8 * s + 8; ++i) {
                if (s == 1)  // the second half's values materialise here, behind the first half's MFMAs
                    asm volatile("" : "+v"(Dv[i][0]), "+v"(Dv[i][1]), "+v"(Dv[i][2]), "+v"(Dv[i][3]),
                                      "+v"(Gv[i][0]), "+v"(Gv[i][1]), "+v"(Gv[i][2]), "+v"(Gv[i][3]));
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaf(lr, Gv[i][e], Dv[i][e] * decay);  // * 1.0f is exact
                tile[t4((lane >> 4) + 4 * i, lane & 15)] = make_float4(v[0], v[1], v[2], v[3]);
            }
            WAVE_LDS_SYNC();
            float xs[8][4];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float4 v = tile[t4(s ? 63 - l : l, blk(h, q))];
                xs[q][0] = v.x;
                xs[q][1] = v.y;
                xs[q][2] = v.z;
                xs[q][3] = v.w;
            }
            row_product_half(xs, Hb, l, h, Tm[s]);
            // keep the first half's MFMAs ahead of the second half's loads' uses
            if (s == 0) __builtin_amdgcn_sched_barrier(0);
        }
        DW_PH(1);
#pragma unroll
        for (int qc = 0; qc < 2; ++qc) {
#pragma unroll
            for (int par = 0; par < 2; ++par) {
                f32x16 acc = zero16();
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    const float u = Tm[0][qc][t], w = Tm[1][qc][t];
                    acc = mfma(Hb[rowmap(t, h) * kLd + 2 * l + par], par ? u - w : u + w, acc);
                }
                Y[par][qc] = acc;
            }
        }
    }
    DW_PH(2);
    chunk64_tail<T>(Y, td.k, delta, td.cols, vec, out_idx, out_val, Hb, W, tile
#ifdef GA_DEMO_STAMPS
                    , ph_acc, ph_last
#endif
    );
}

// ---- row group: up to 64 consecutive 1x64 chunks (F1 = [1]) ---------------
template <typename T>
__device__ __forceinline__ void rowgroup(const ga_demo_rowgroup& rg, T* param, const T* grad, T* delta,
                                         int32_t* pay_idx, float* pay_val, float lr, float decay,
                                         float wd_factor, int ptr_vec, const float* Hb, WaveLDS& W
#ifdef GA_DEMO_STAMPS
                                         , unsigned long long (&ph_acc)[16], unsigned long long& ph_last
#endif
) {
    const int rows = rg.rows, k = rg.k;
    const bool vec = ptr_vec && (rg.offset % 4 == 0);
    param += rg.offset;
    grad += rg.offset;
    delta += rg.offset;
    float x[2][8][4];
    {
        const int lane = lane_id(), l = lane & 31, h = lane >> 5;
        error_feedback(param, grad, delta, 64, l, h, vec, rows, lr, decay, wd_factor, x);
    }
    DW_PH(6);
    {
        const int lane = lane_id(), l = lane & 31, h = lane >> 5;
        f32x16 Tm[2][2];
        row_product(x, Hb, l, h, Tm);
        // T -> tile (row-major, natural frequency order)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int qc = 0; qc < 2; ++qc)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = rowmap(r, h);
                    W.tile[(s ? 63 - i : i) * kLd + 2 * l + qc] = Tm[s][qc][r];
                }
    }
    WAVE_LDS_SYNC();
    {
        // lane L: exact top-k of its row, ties to the lowest index, ascending emission
        const int L = lane_id();
        float* trow = W.tile + L * kLd;
        float yr[64];
#pragma unroll
        for (int t = 0; t < 64; ++t) yr[t] = trow[t];
        uint32_t thr = 0;
        for (int bit = 31; bit >= 0; --bit) {
            const uint32_t cnd = thr | (1u << bit);
            int cl = 0;
#pragma unroll
            for (int t = 0; t < 64; ++t) cl += fabsf(yr[t]) >= __uint_as_float(cnd - 1u) ? 1 : 0;
            if (cl >= k) thr = cnd;
        }
        int gl = 0;
#pragma unroll
        for (int t = 0; t < 64; ++t) gl += keyv(yr[t]) > thr ? 1 : 0;
        int need = k - gl;
        int slot = 0;
        const bool live = L < rows;
        int32_t* oi = pay_idx + (int64_t)L * k;
        float* ov = pay_val + (int64_t)L * k;
#pragma unroll
        for (int t = 0; t < 64; ++t) {
            const uint32_t kv = keyv(yr[t]);
            const bool tie = kv == thr && need > 0;
            const bool s = kv > thr || tie;
            need -= tie ? 1 : 0;
            if (s && live) {
                oi[slot] = t;
                ov[slot] = yr[t];
            }
            slot += s ? 1 : 0;
            trow[t] = s ? yr[t] : 0.f;  // the kept coefficients (Ymask)
        }
    }
    WAVE_LDS_SYNC();
    {
        // R^T[c][row] = sum_d F[c][d] Ymask[row][d]; rows l (s = 0) and 63 - l (s = 1)
        const int lane = lane_id(), l = lane & 31, h = lane >> 5;
        const int c0 = pi_col(0, l), c1 = pi_col(1, l);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const float* yrow = W.tile + (s ? 63 - l : l) * kLd;
            f32x16 r0 = zero16(), r1 = zero16();
#pragma unroll
            for (int t = 0; t < 32; ++t) {
                const int d = 2 * t + h;
                const float yv = yrow[d];
                r0 = mfma(basis64(Hb, c0, d), yv, r0);
                r1 = mfma(basis64(Hb, c1, d), yv, r1);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) x[s][q][e] -= (q < 4 ? r0 : r1)[4 * (q & 3) + e];
        }
        store_rows(delta, 64, l, h, vec, rows, x);
    }
    WAVE_LDS_SYNC();
    DW_PH(7);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void encode_kernel(
    const ga_demo_tensor* __restrict__ tens, int ntens, int nchunks, const ga_demo_rowgroup* __restrict__ groups,
    int ngroups, const float* __restrict__ F64, T* param0, const T* __restrict__ grad0, T* delta0, int64_t ld,
    int64_t K, float lr, float decay, float wd_factor, int32_t* payload0, int64_t pstride, int64_t M, int ptr_vec) {
    __shared__ float Hb[32 * kLd];
    __shared__ WaveLDS wl[kWaves];
    __shared__ int next_job;  // the workgroup's job counter
    for (int q = threadIdx.x; q < 32 * 64; q += kThreads) Hb[(q >> 6) * kLd + (q & 63)] = F64[q];
    next_job = 0;  // every lane stores the same 0 (no branch)
    __syncthreads();
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);  // wave-uniform: scalar job loop
    WaveLDS& W = wl[wid];
    DW_PH_DECL;
    const int64_t n64 = (int64_t)nchunks * K;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    // Job lists per workgroup b: its 64x64 chunks are the static b*8 + w + r*stride
    // (w < 8: index i -> chunk b*8 + (i & 7) + (i >> 3) * stride, increasing in i), and
    // its row groups g = b + r*grid (one per workgroup per round, spread over the
    // workgroups).  Its 8 waves draw from one LDS counter, row groups FIRST: a row group
    // costs ~2.5 chunks (0.058 ms for the groups alone, profiles/r06p_*), and drawn last
    // by a static order the ~194 of GPT-2 350M, packed 8 per workgroup into the last
    // ~25 workgroups, were the kernel's tail; now one workgroup's siblings take the
    // chunks its group-drawing wave would have had.
    const int64_t b8 = (int64_t)blockIdx.x * kWaves;
    const int64_t g_total = (int64_t)ngroups * K;
    const uint32_t st = (uint32_t)stride;  // 32-bit counts: the launch keeps the job space below 2^31
    uint32_t nc32 = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w)
        if (b8 + w < n64) nc32 += ((uint32_t)(n64 - (b8 + w)) + st - 1u) / st;
    const int64_t nc = nc32;
    const int64_t ng = (int64_t)blockIdx.x < g_total
                           ? ((uint32_t)(g_total - blockIdx.x) + gridDim.x - 1u) / gridDim.x : 0;
    const int64_t nt = nc + ng;
    int tix = -1;
    int64_t last_rep = -1;
    while (true) {
        // lane 0 draws (an LDS atomic at any LDS address; ds_append addresses only the
        // first 64 KB through M0[15:0], and this counter sits past the wave tiles)
        int tv = 0;
        if (lane_id() == 0) tv = atomicAdd(&next_job, 1);
        const int64_t t = __builtin_amdgcn_readfirstlane(tv);
        if (t >= nt) break;
        const int64_t job = t < ng ? n64 + (int64_t)blockIdx.x + t * gridDim.x  // a row group
                                   : b8 + ((t - ng) & 7) + ((t - ng) >> 3) * stride;
        if (job < n64) {  // a 64x64 chunk
            const int64_t rep = job / nchunks;
            const int chunk = (int)(job - rep * nchunks);
            if (rep != last_rep) {
                tix = -1;
                last_rep = rep;
            }
            tix = find_tensor(tens, ntens, tix, chunk);
            const ga_demo_tensor td = tens[tix];
            const int c = chunk - td.chunk_start;
            int32_t* pi = payload0 + rep * pstride + td.payload_off + (int64_t)c * td.k;
            float* pv = reinterpret_cast<float*>(payload0 + rep * pstride + M) + td.payload_off + (int64_t)c * td.k;
            chunk64<T>(td, c, param0 + rep * ld, grad0 + rep * ld, delta0 + rep * ld, pi, pv, lr, decay, wd_factor,
                       ptr_vec, Hb, W
#ifdef GA_DEMO_STAMPS
                       , ph_acc, ph_last
#endif
            );
            DW_CNT(9);
        } else {  // a row group
            const int64_t j = job - n64;
            const int64_t rep = j / ngroups;
            const int g = (int)(j - rep * ngroups);
            const ga_demo_rowgroup rg = groups[g];
            rowgroup<T>(rg, param0 + rep * ld, grad0 + rep * ld, delta0 + rep * ld,
                        payload0 + rep * pstride + rg.payload_off,
                        reinterpret_cast<float*>(payload0 + rep * pstride + M) + rg.payload_off, lr, decay,
                        wd_factor, ptr_vec, Hb, W
#ifdef GA_DEMO_STAMPS
                        , ph_acc, ph_last
#endif
            );
        }
    }
    DW_PH_FLUSH();
}

template <typename T>
static int launch(const ga_demo_tensor* tens, int32_t ntens, int32_t nchunks, const ga_demo_rowgroup* groups,
                  int32_t ngroups, const float* F64, void* param, const void* grad, void* delta, int64_t K,
                  int64_t ld, float lr, float decay, float wd_factor, int32_t* payload, int64_t pstride, int64_t M,
                  int ptr_vec, hipStream_t stream) {
    static const int cus = [] {
        int dev = 0, n = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n > 0 ? n : 256;
    }();
    auto kern = encode_kernel<T>;
    static const int resident = [&] {
        int per_cu = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kThreads, 0);
        return (per_cu > 0 ? per_cu : 1) * cus;
    }();
    const int64_t jobs = ((int64_t)nchunks + ngroups) * K;
    const int64_t want = (jobs + kWaves - 1) / kWaves;
    const int grid = (int)(want < resident ? want : resident);
    if (grid <= 0) return GA_OK;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, stream, tens, ntens, nchunks, groups, ngroups, F64,
                       (T*)param, (const T*)grad, (T*)delta, ld, K, lr, decay, wd_factor, payload, pstride, M,
                       ptr_vec);
    return GA_OK;
}

// ============================================================================
// Decode (ga_demo_decode_sym): the gathered payloads of S <= 15 sources,
// scatter-mean per chunk (demo.py:331-352), inverse DCT, sign, and the SGD step
// on every local replica (demo.py:192-209), one wavefront per chunk.
//   S == 1   the entries' sparse synthesis (synth_half, as the encode residual)
//   S >= 2   node-ordered scatter-add + 4-bit hit counts in LDS, the mean over
//            hitters, then g = F . X . F^T as two folded 64-deep MFMA products:
//            U = X . F^T (columns l and 63 - l from the even / odd-frequency
//            halves), g^T = U^T . F^T (rows l and 63 - l from the even / odd b)
// The signs go through the tile into the coalesced layout for the p update.
// ============================================================================
constexpr int kMaxSrc = 15;  // 4-bit hit counts

struct DecLDS {
    float tile[64 * 64];  // coefficients (swizzled row-major), then sign(g)
    uint32_t aux[512];    // 4-bit hit counts per coefficient | the S == 1 parity lists
};

// float index of (row, col) in the swizzled tile (see t4)
__device__ __forceinline__ int fidx(int row, int col) { return row * 64 + 4 * ((col >> 2) ^ (row & 15)) + (col & 3); }

// torch.sign with NaN -> 0: +-1 with g's sign bit where |g| > 0 (false for 0 and NaN), else 0
// (3 VALU: compare, bit-select, select; the (g > 0) - (g < 0) form issued 6)
__device__ __forceinline__ float sgnf(float g) {
    return fabsf(g) > 0.f ? __builtin_copysignf(1.f, g) : 0.f;
}

// the signs (layout C, read from the tile where used) -> p -= lr * sign, grad = sign,
// for each of K replicas; a full 64-row chunk's replica 0 comes in pre (loaded before
// the chunk's transform, so the load latency hides behind it)
// a chunk's parameters held as loaded (4 elements per Vec4<T>: 64 VGPRs for fp32, 32 for
// bf16), widened to fp32 only where the update consumes them
template <typename T>
using PRaw = typename Vec4<T>::type[16];

template <typename T>
__device__ __forceinline__ void load_coal_raw(const T* pb, int stride, bool vec, int lane, PRaw<T>& o) {
    if (vec) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            o[i] = *reinterpret_cast<const typename Vec4<T>::type*>(at_off(pb, coal_off(i, lane, stride)));
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            float f[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) f[e] = Elem<T>::load(at_off(pb, coal_off(i, lane, stride)) + e);
            o[i] = Vec4<T>::pack(f);  // exact: f holds T values
        }
    }
}

// NTS: the decode's grad stores non-temporal (the 2+-source decode: 1.19 -> 1.13 ms at 350M;
// the 1-source decode measured 5% slower with them, profiles/r03ac_ab_demo_nt.txt)
template <typename T, bool NTS = false>
__device__ __forceinline__ void store_quad(T* pb, int i, int stride, bool vec, int lane, const float (&f)[4]) {
    T* a = at_off(pb, coal_off(i, lane, stride));
    if (vec) {
        if constexpr (NTS) stream_store(reinterpret_cast<typename Vec4<T>::type*>(a), Vec4<T>::pack(f));
        else store_vec(pb, coal_off(i, lane, stride), Vec4<T>::pack(f));
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) Elem<T>::store(a + e, f[e]);
    }
}

template <typename T, bool NTS = false>
__device__ __forceinline__ void sign_update(const float4* tile, T* pr, T* gr, int stride, bool vec, float lr,
                                            int lane, PRaw<T>& raw) {
    if constexpr (sizeof(typename Vec4<T>::type) < 16) {
        // packed (bf16) rows: widen, update and store one row quad at a time, so the
        // fp32 copy of the chunk is never live whole (244 -> 116 B/lane of spill at 8 sources)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
            float f[4];
            Vec4<T>::unpack(raw[i], f);
            f[0] = fmaf(-lr, v.x, f[0]);
            f[1] = fmaf(-lr, v.y, f[1]);
            f[2] = fmaf(-lr, v.z, f[2]);
            f[3] = fmaf(-lr, v.w, f[3]);
            store_quad(pr, i, stride, vec, lane, f);
        }
        if (gr) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
                const float f[4] = {v.x, v.y, v.z, v.w};
                store_quad<T, NTS>(gr, i, stride, vec, lane, f);
            }
        }
    } else {
        // fp32: every fused update first (in place, in the registers the parameters were
        // loaded into), then the 16 stores back to back (measured: the per-quad form
        // above costs fp32 ~20% here)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
            raw[i].x = fmaf(-lr, v.x, raw[i].x);
            raw[i].y = fmaf(-lr, v.y, raw[i].y);
            raw[i].z = fmaf(-lr, v.z, raw[i].z);
            raw[i].w = fmaf(-lr, v.w, raw[i].w);
        }
        if (vec) {
#pragma unroll
            for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(at_off(pr, coal_off(i, lane, stride))) = raw[i];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float f[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
                store_quad(pr, i, stride, vec, lane, f);
            }
        }
        if (gr) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
                const float f[4] = {v.x, v.y, v.z, v.w};
                store_quad<T, NTS>(gr, i, stride, vec, lane, f);
            }
        }
    }
}

template <typename T, bool NTS = false>
__device__ __forceinline__ void apply_signs(const float4* tile, T* param, T* grad, int64_t K, int64_t ld, int stride,
                                            bool vec, int nrows, float lr, int lane, PRaw<T>& pre, bool lean = false) {
    if (nrows == 64) {
        sign_update<T, NTS>(tile, param, grad, stride, vec, lr, lane, pre);
        if (lean) {  // replicas 1.. a row quad at a time (the updater waves' register budget)
            for (int64_t r = 1; r < K; ++r) {
#pragma unroll 4
                for (int i = 0; i < 16; ++i) {
                    const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
                    T* a = at_off(param + r * ld, coal_off(i, lane, stride));
                    float f[4];
                    if (vec) {
                        Vec4<T>::unpack(*reinterpret_cast<const typename Vec4<T>::type*>(a), f);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) f[e] = Elem<T>::load(a + e);
                    }
                    f[0] = fmaf(-lr, v.x, f[0]);
                    f[1] = fmaf(-lr, v.y, f[1]);
                    f[2] = fmaf(-lr, v.z, f[2]);
                    f[3] = fmaf(-lr, v.w, f[3]);
                    store_quad(param + r * ld, i, stride, vec, lane, f);
                    if (grad) {
                        const float g4[4] = {v.x, v.y, v.z, v.w};
                        store_quad(grad + r * ld, i, stride, vec, lane, g4);
                    }
                }
            }
            return;
        }
        for (int64_t r = 1; r < K; ++r) {
            PRaw<T> p;
            load_coal_raw(param + r * ld, stride, vec, lane, p);
            sign_update<T, NTS>(tile, param + r * ld, grad ? grad + r * ld : nullptr, stride, vec, lr, lane, p);
        }
        return;
    }
    for (int64_t r = 0; r < K; ++r) {  // a partial row group: 8 row quads' loads, then their stores
#pragma unroll
        for (int i0 = 0; i0 < 16; i0 += 8) {
            float f[8][4];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const bool live = (lane >> 4) + 4 * (i0 + i) < nrows;
                const T* a = at_off(param + r * ld, coal_off(i0 + i, lane, stride));
#pragma unroll
                for (int e = 0; e < 4; ++e) f[i][e] = live ? Elem<T>::load(a + e) : 0.f;
            }
#pragma unroll
            for (int ii = 0; ii < 8; ++ii) {
                const int i = i0 + ii;
                if ((lane >> 4) + 4 * i >= nrows) continue;
                const float4 v = tile[t4((lane >> 4) + 4 * i, lane & 15)];
                const float sg[4] = {v.x, v.y, v.z, v.w};
                T* a = at_off(param + r * ld, coal_off(i, lane, stride));
#pragma unroll
                for (int e = 0; e < 4; ++e) Elem<T>::store(a + e, fmaf(-lr, sg[e], f[ii][e]));
                if (grad) {
                    T* gq = at_off(grad + r * ld, coal_off(i, lane, stride));
#pragma unroll
                    for (int e = 0; e < 4; ++e) Elem<T>::store(gq + e, sg[e]);
                }
            }
        }
    }
}

// node-ordered scatter-add of S sources' entries (n per source, entry j -> tile row
// row_of(j)) and the 4-bit hit counts, sources in order (a source's indices are
// distinct, so its adds never collide; one wave's LDS adds run in issue order, so
// the per-coefficient sums accumulate in node order).  A row group holds up to
// 64 x k entries per source: each lane loads kGrpBatch of them before any add, so
// the scatter costs one memory latency per batch instead of one per entry (S x 32
// dependent round trips per row group at k = 32, which made the row groups the
// decode's tail)
constexpr int kGrpBatch = 16;

template <typename RowOf>
__device__ __forceinline__ void scatter_sources(DecLDS& W, const int32_t* __restrict__ payload, int64_t pstride,
                                                int64_t M, int64_t e0, int S, int n, int nvalid, RowOf row_of,
                                                int lane) {
    for (int s = 0; s < S; ++s) {
        const int32_t* pi = payload + (int64_t)s * pstride + e0;
        const float* pv = reinterpret_cast<const float*>(payload + (int64_t)s * pstride + M) + e0;
        for (int j0 = 0; j0 < n; j0 += 64 * kGrpBatch) {
            int xb[kGrpBatch];
            float vb[kGrpBatch];
#pragma unroll
            for (int u = 0; u < kGrpBatch; ++u) {
                const int j = j0 + 64 * u + lane;
                xb[u] = j < n ? pi[j] : -1;
                vb[u] = j < n ? pv[j] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < kGrpBatch; ++u) {
                const int x = xb[u];
                if ((unsigned)x < (unsigned)nvalid) {
                    const int j = j0 + 64 * u + lane;
                    const int row = row_of(j, x), col = nvalid == 64 ? x : (x & 63);
                    atomicAdd(&W.tile[fidx(row, col)], vb[u]);
                    const int cid = row * 64 + col;
                    atomicAdd(&W.aux[cid >> 3], 1u << (4 * (cid & 7)));
                }
            }
        }
        WAVE_LDS_SYNC();
    }
}

// sum / (hit count in the low nibble of cw), true division as scatter_reduce_(mean)
__device__ __forceinline__ float mean_of(float sum, uint32_t cw) {
    const uint32_t n = cw & 15u;
    return n > 1u ? sum / (float)n : sum;
}

// a 64x64 chunk's global inputs: each source's entry `lane` (k <= 64), MS >= S register
// slots (the kernel is built for MS = 8 and 15: at most 8 sources it holds no spill)
template <int MS>
struct DecIn {
    int xs[MS];
    float vs[MS];
};

__device__ __forceinline__ int64_t chunk_base(const ga_demo_tensor& td, int c) {
    const int cy = c / td.gx, cx = c - cy * td.gx;
    return td.offset + (int64_t)cy * 64 * td.cols + (int64_t)cx * 64;
}

__device__ __forceinline__ bool chunk_vec(const ga_demo_tensor& td, int ptr_vec) {
    return ptr_vec && (td.offset % 4 == 0) && (td.cols % 4 == 0);
}

// issue the loads of chunk c's entries, all sources at once
template <int MS>
__device__ __forceinline__ void dchunk_entries(const ga_demo_tensor& td, int c, const int32_t* __restrict__ payload,
                                               int64_t pstride, int64_t M, int S, DecIn<MS>& in) {
    const int k = td.k, lane = lane_id();
    const int64_t e0 = td.payload_off + (int64_t)c * k;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
        in.xs[s] = -1;
        in.vs[s] = 0.f;
        if (s < S && lane < k) {
            in.xs[s] = payload[(int64_t)s * pstride + e0 + lane];
            in.vs[s] = reinterpret_cast<const float*>(payload + (int64_t)s * pstride + M)[e0 + lane];
        }
    }
}

template <typename T>
__device__ __forceinline__ void dchunk_params(const ga_demo_tensor& td, int c, const T* param, int ptr_vec,
                                              PRaw<T>& p0) {
    load_coal_raw(param + chunk_base(td, c), td.cols, chunk_vec(td, ptr_vec), lane_id(), p0);
}

// sign(g) of chunk c into the tile (swizzled row-major) from the entries in `in`;
// `consumed()` runs as soon as the entries are in LDS (the caller loads the next
// chunk's entries into `in` there, a whole transform ahead of their use)
template <int MS, typename Consumed>
__device__ __forceinline__ void dchunk_signs(int k, int S, DecIn<MS>& in, const float* Hb, DecLDS& W,
                                             Consumed consumed) {
    float4* tile = reinterpret_cast<float4*>(W.tile);
    const int lane = lane_id(), l = lane & 31, h = lane >> 5;
    const int (&xs)[MS] = in.xs;
    const float (&vs)[MS] = in.vs;
    if (S == 1) {
        uint32_t epos = 0u, ebits = 0u;
        bool ent = false;
        if (lane < k) {
            const int x = xs[0];
            const float v = vs[0];
            ent = (unsigned)x < 4096u;
            epos = ent ? (uint32_t)x : 0u;
            ebits = ent ? __float_as_uint(v) : 0u;
        }
        uint2* lstp = reinterpret_cast<uint2*>(W.aux);
        int np0, np1;
        parity_lists(epos, ebits, ent, lane, lstp, np0, np1);
        consumed();
#pragma unroll
        for (int H = 0; H < 2; ++H) {
            f32x16 Re, Ro;
            synth_half(lstp, np0, np1, H, l, h, Hb, Re, Ro);
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int r = 4 * qq;
                tile[t4(l, blk(h, 4 * H + qq))] = make_float4(sgnf(Re[r] + Ro[r]), sgnf(Re[r + 1] + Ro[r + 1]),
                                                              sgnf(Re[r + 2] + Ro[r + 2]), sgnf(Re[r + 3] + Ro[r + 3]));
                tile[t4(63 - l, blk(h, 4 * H + qq))] =
                    make_float4(sgnf(Re[r] - Ro[r]), sgnf(Re[r + 1] - Ro[r + 1]), sgnf(Re[r + 2] - Ro[r + 2]),
                                sgnf(Re[r + 3] - Ro[r + 3]));
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) tile[i * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
        reinterpret_cast<uint4*>(W.aux)[lane] = make_uint4(0u, 0u, 0u, 0u);
        reinterpret_cast<uint4*>(W.aux)[64 + lane] = make_uint4(0u, 0u, 0u, 0u);
        WAVE_LDS_SYNC();
        // node-ordered scatter-add with 4-bit hit counts, one source per pass (a
        // source's indices are distinct: the adds of one pass never collide)
#pragma unroll
        for (int s = 0; s < MS; ++s) {
            const int x = xs[s];  // -1 past S
            if ((unsigned)x < 4096u) {
                atomicAdd(&W.tile[fidx(x >> 6, x & 63)], vs[s]);
                atomicAdd(&W.aux[x >> 3], 1u << (4 * (x & 7)));
            }
            WAVE_LDS_SYNC();
        }
        consumed();
        // U = X . F^T: U[b][l] = ue + uo, U[b][63 - l] = ue - uo (even / odd frequency d)
        f32x16 U[2][2];  // [b block][column set]
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            f32x16 ue = zero16(), uo = zero16();
            const int row = 32 * bb + l;
#pragma unroll
            for (int t = 0; t < 8; ++t) {  // lane half h: frequencies 32h + 4t .. +3
                // the mean over the hitters (demo.py:331-352), applied as the sums are read
                float4 xv = tile[t4(row, 8 * h + t)];
                const uint32_t cw = W.aux[(row * 64 + 32 * h + 4 * t) >> 3] >> (16 * (t & 1));
                // the true divisions only where some lane's four coefficients had two or more
                // hitters (wave-uniform branch: ~12 VALU per division, 64 per chunk otherwise)
                const bool multi = ((cw & 0xeu) | ((cw >> 4) & 0xeu) | ((cw >> 8) & 0xeu) | ((cw >> 12) & 0xeu)) != 0u;
                if (__builtin_amdgcn_ballot_w64(multi)) {
                    xv.x = mean_of(xv.x, cw);
                    xv.y = mean_of(xv.y, cw >> 4);
                    xv.z = mean_of(xv.z, cw >> 8);
                    xv.w = mean_of(xv.w, cw >> 12);
                }
                const float* fr = Hb + l * kLd + 32 * h + 4 * t;
                ue = mfma(xv.x, fr[0], ue);
                uo = mfma(xv.y, fr[1], uo);
                ue = mfma(xv.z, fr[2], ue);
                uo = mfma(xv.w, fr[3], uo);
            }
            U[bb][0] = ue + uo;
            U[bb][1] = ue - uo;
        }
        WAVE_LDS_SYNC();
        // g^T = U^T . F^T per column set: row l gets ge + go, row 63 - l gets ge - go
#pragma unroll
        for (int cs = 0; cs < 2; ++cs) {
            f32x16 ge = zero16(), go = zero16();
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int bb = s >> 3, r2 = 2 * (s & 7);
                ge = mfma(U[bb][cs][r2], Hb[l * kLd + 32 * bb + rowmap(r2, h)], ge);
                go = mfma(U[bb][cs][r2 + 1], Hb[l * kLd + 32 * bb + rowmap(r2 + 1, h)], go);
            }
            // register 4q' + e: column m = 8q' + 4h + e (cs = 0) or 63 - m (cs = 1)
#pragma unroll
            for (int qp = 0; qp < 4; ++qp) {
                float a[4], b[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    a[e] = sgnf(ge[4 * qp + e] + go[4 * qp + e]);
                    b[e] = sgnf(ge[4 * qp + e] - go[4 * qp + e]);
                }
                const int cb = cs ? 15 - (2 * qp + h) : 2 * qp + h;
                tile[t4(l, cb)] = cs ? make_float4(a[3], a[2], a[1], a[0]) : make_float4(a[0], a[1], a[2], a[3]);
                tile[t4(63 - l, cb)] = cs ? make_float4(b[3], b[2], b[1], b[0]) : make_float4(b[0], b[1], b[2], b[3]);
            }
        }
    }
    WAVE_LDS_SYNC();
}

// row group: rows = consecutive 1x64 chunks (contiguous, stride 64); g[row] = X[row] . F^T
template <typename T>
__device__ __forceinline__ void dgroup(const ga_demo_rowgroup& rg, const int32_t* __restrict__ payload,
                                       int64_t pstride, int64_t M, int S, T* param, T* grad, int64_t K, int64_t ld,
                                       float lr, int ptr_vec, const float* Hb, DecLDS& W) {
    const int rows = rg.rows, k = rg.k;
    const bool vec = ptr_vec && (rg.offset % 4 == 0);
    float4* tile = reinterpret_cast<float4*>(W.tile);
    const int lane = lane_id(), l = lane & 31, h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; ++i) tile[i * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<uint4*>(W.aux)[lane] = make_uint4(0u, 0u, 0u, 0u);
    reinterpret_cast<uint4*>(W.aux)[64 + lane] = make_uint4(0u, 0u, 0u, 0u);
    WAVE_LDS_SYNC();
    scatter_sources(W, payload, pstride, M, rg.payload_off, S, rows * k, 64, [k](int j, int) { return j / k; }, lane);
    if (S > 1) {  // mean over the hitters: a pass over the whole tile (row groups are few)
#pragma unroll 4
        for (int i = 0; i < 64; ++i) {
            const int cid = i * 64 + lane;
            const int n = (int)((W.aux[cid >> 3] >> (4 * (cid & 7))) & 15u);
            if (n > 1) W.tile[fidx(i, lane)] /= (float)n;
        }
        WAVE_LDS_SYNC();
    }
    PRaw<T> pre;  // a full group's replica 0, in flight behind the transform (after the scatter,
                  // whose double-buffered entry batches need the registers)
    if (rows == 64) load_coal_raw(param + rg.offset, 64, vec, lane, pre);
    // R^T[c][row] = sum_d F[c][d] X[row][d] for rows l (s = 0) and 63 - l (s = 1)
    const int c0 = pi_col(0, l), c1 = pi_col(1, l);
    f32x16 r[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int row = s ? 63 - l : l;
        r[s][0] = zero16();
        r[s][1] = zero16();
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int d = 2 * t + h;
            const float xv = W.tile[fidx(row, d)];
            r[s][0] = mfma(basis64(Hb, c0, d), xv, r[s][0]);
            r[s][1] = mfma(basis64(Hb, c1, d), xv, r[s][1]);
        }
    }
    WAVE_LDS_SYNC();
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f32x16& a = r[s][q >> 2];
            const int o = 4 * (q & 3);
            tile[t4(s ? 63 - l : l, blk(h, q))] =
                make_float4(sgnf(a[o]), sgnf(a[o + 1]), sgnf(a[o + 2]), sgnf(a[o + 3]));
        }
    WAVE_LDS_SYNC();
    apply_signs(tile, param + rg.offset, grad ? grad + rg.offset : nullptr, K, ld, 64, vec, rows, lr, lane, pre);
    WAVE_LDS_SYNC();
}

template <typename T, int MS, bool NTS = false>
__global__ __launch_bounds__(kThreads) void decode_kernel(
    const ga_demo_tensor* __restrict__ tens, int ntens, int nchunks, const ga_demo_rowgroup* __restrict__ groups,
    int ngroups, const float* __restrict__ F64, const int32_t* __restrict__ payload, int64_t pstride, int64_t M,
    int S, T* param, T* grad, int64_t K, int64_t ld, float lr, int ptr_vec) {
    __shared__ float Hb[32 * kLd];
    __shared__ DecLDS wl[kWaves];
    if constexpr (NTS) decode_wave_priority();  // NTS: the launch's S >= 2 instantiation
    for (int q = threadIdx.x; q < 32 * 64; q += kThreads) Hb[(q >> 6) * kLd + (q & 63)] = F64[q];
    __syncthreads();
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    DecLDS& W = wl[wid];
    const int64_t total = (int64_t)nchunks + ngroups;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int tix = -1;
    int64_t job = (int64_t)blockIdx.x * kWaves + wid;
    // 64x64 chunks, software-pipelined: chunk j+1's entries are loaded as soon as chunk
    // j's are in LDS (before chunk j's transform and stores: vmcnt retires in order, so a
    // load issued behind the stores would wait for them) and its parameters right after
    // chunk j's stores, a whole transform ahead of their use
    if (job < nchunks) {
        DecIn<MS> cur;
        PRaw<T> p0;
        tix = find_tensor(tens, ntens, tix, (int)job);
        ga_demo_tensor td = tens[tix];
        dchunk_entries(td, (int)job - td.chunk_start, payload, pstride, M, S, cur);
        dchunk_params<T>(td, (int)job - td.chunk_start, param, ptr_vec, p0);
        while (true) {
            const int c = (int)job - td.chunk_start;
            const int64_t base = chunk_base(td, c);
            const bool vec = chunk_vec(td, ptr_vec);
            const int cols = td.cols, kc = td.k;
            job += stride;
            if (job < nchunks) {
                tix = find_tensor(tens, ntens, tix, (int)job);
                td = tens[tix];
            }
            // the next chunk's entries are issued once this chunk's are in LDS: in flight
            // behind this chunk's transform and stores (vmcnt retires in order: older than
            // the stores, so waiting for them never waits for the stores)
            dchunk_signs(kc, S, cur, Hb, W, [&] {
                if (job < nchunks) dchunk_entries(td, (int)job - td.chunk_start, payload, pstride, M, S, cur);
            });
            apply_signs<T, NTS>(reinterpret_cast<const float4*>(W.tile), param + base, grad ? grad + base : nullptr,
                                K, ld, cols, vec, 64, lr, lane_id(), p0);
            WAVE_LDS_SYNC();
            if (job >= nchunks) break;
            dchunk_params<T>(td, (int)job - td.chunk_start, param, ptr_vec, p0);
        }
    }
    for (; job < total; job += stride) {
        const ga_demo_rowgroup rg = groups[(int)(job - nchunks)];
        dgroup<T>(rg, payload, pstride, M, S, param, grad, K, ld, lr, ptr_vec, Hb, W);
    }
}

template <typename T, int MS>
static void launch_decode_ms(const ga_demo_tensor* tens, int32_t ntens, int32_t nchunks,
                             const ga_demo_rowgroup* groups, int32_t ngroups, const float* F64,
                             const int32_t* payload, int64_t pstride, int64_t M, int S, void* param, void* grad,
                             int64_t K, int64_t ld, float lr, int ptr_vec, hipStream_t stream) {
    auto kern = decode_kernel<T, MS>;
    static const int resident = [&] {
        int per_cu = 0, dev = 0, cus = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kThreads, 0);
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 256);
    }();
    // Workgroups: not one persistent workgroup per CU but m workgroups per CU, m chosen
    // for ~1.75 jobs per wave at S >= 2 and ~5.3 at S = 1: the dispatcher then balances
    // the CUs (a persistent grid waits for its slowest CU) while each wave still
    // pipelines a few chunks.  A whole number of workgroups per CU matters as much: the
    // static job order gives the LAST-dispatched workgroups the fewer jobs, and no
    // partial last round of workgroups runs alone (5418 workgroups for GPT-2 350M's
    // 86.7k 8-source jobs ran 0.936 ms, 6144 = 24 per CU 0.838 ms).  GPT-2 350M, one
    // process (profiles/r06t_ab_demo_decode_grid.txt): 8 sources 0.94-0.97 ms persistent,
    // 0.838-0.846 ms at 24 per CU, 0.94-0.99 ms at one job per wave; one source
    // 0.857-0.867 ms persistent, 0.841-0.844 ms at 8 per CU.
    const int64_t jobs = (int64_t)nchunks + ngroups;
    const int64_t want = (jobs + kWaves - 1) / kWaves;
    const int64_t wr = (int64_t)kWaves * resident;  // waves resident at once
    int64_t m = S >= 2 ? (8 * jobs + 7 * wr) / (14 * wr)    // round(jobs / (1.75 wr))
                       : (6 * jobs + 16 * wr) / (32 * wr);  // round(jobs / (5.33 wr))
    if (m < 1) m = 1;
    const int64_t g = resident * m;
    const int grid = (int)(g < want ? g : want);
    if (grid <= 0) return;
    if (S >= 2)  // several sources: non-temporal grad stores
        hipLaunchKernelGGL((decode_kernel<T, MS, true>), dim3(grid), dim3(kThreads), 0, stream, tens, ntens, nchunks,
                           groups, ngroups, F64, payload, pstride, M, S, (T*)param, (T*)grad, K, ld, lr, ptr_vec);
    else
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, stream, tens, ntens, nchunks, groups, ngroups, F64,
                           payload, pstride, M, S, (T*)param, (T*)grad, K, ld, lr, ptr_vec);
}

template <typename T>
static void launch_decode(const ga_demo_tensor* tens, int32_t ntens, int32_t nchunks, const ga_demo_rowgroup* groups,
                          int32_t ngroups, const float* F64, const int32_t* payload, int64_t pstride, int64_t M,
                          int S, void* param, void* grad, int64_t K, int64_t ld, float lr, int ptr_vec,
                          hipStream_t stream) {
    if (S <= 8)
        launch_decode_ms<T, 8>(tens, ntens, nchunks, groups, ngroups, F64, payload, pstride, M, S, param, grad, K, ld,
                               lr, ptr_vec, stream);
    else
        launch_decode_ms<T, kMaxSrc>(tens, ntens, nchunks, groups, ngroups, F64, payload, pstride, M, S, param, grad,
                                     K, ld, lr, ptr_vec, stream);
}

#ifdef GA_DEMO_STAMPS
__device__ unsigned long long* g_demo_stamps_w;
#endif

}  // namespace dw
}  // namespace ga

using namespace ga;

#ifdef GA_DEMO_STAMPS
extern "C" GA_API int ga_demo_stamps_set_wave(unsigned long long* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(ga::dw::g_demo_stamps_w), &buf, sizeof(buf)) == hipSuccess ? 0 : 2;
}
#endif

extern "C" GA_API int ga_demo_encode_sym(int dtype, const ga_demo_tensor* tensors, int32_t ntensors,
                                         int32_t nchunks, const ga_demo_rowgroup* groups, int32_t ngroups,
                                         const float* F64, void* param, const void* grad, void* delta, int64_t K,
                                         int64_t ld, float lr, float decay, float wd_factor, int32_t* payload,
                                         int64_t payload_stride, int64_t M, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(ntensors >= 0 && nchunks >= 0 && ngroups >= 0 && (nchunks > 0 || ngroups > 0),
               "ga_demo_encode_sym: empty plan (ntensors=%d nchunks=%d ngroups=%d)", ntensors, nchunks, ngroups);
    GA_REQUIRE(nchunks == 0 || (tensors && ntensors >= 1), "ga_demo_encode_sym: no descriptors");
    GA_REQUIRE(ngroups == 0 || groups, "ga_demo_encode_sym: no row groups");
    GA_REQUIRE(F64 && param && grad && delta && payload, "ga_demo_encode_sym: null buffer");
    GA_REQUIRE(K >= 1 && ((int64_t)nchunks + ngroups) * K < (1ll << 31), "ga_demo_encode_sym: K=%lld out of range",
               (long long)K);
    GA_REQUIRE(K == 1 || (ld > 0 && payload_stride >= 2 * M), "ga_demo_encode_sym: bad replica strides");
    const int vb = dtype == GA_F32 ? 16 : 8;
    const int ptr_vec = ((uintptr_t)param % vb == 0) && ((uintptr_t)grad % vb == 0) &&
                        ((uintptr_t)delta % vb == 0) && (K == 1 || ld % 4 == 0);
    switch (dtype) {
        case GA_F32:
            dw::launch<float>(tensors, ntensors, nchunks, groups, ngroups, F64, param, grad, delta, K, ld, lr, decay,
                              wd_factor, payload, payload_stride, M, ptr_vec, stream);
            break;
        case GA_BF16:
            dw::launch<__hip_bfloat16>(tensors, ntensors, nchunks, groups, ngroups, F64, param, grad, delta, K, ld,
                                       lr, decay, wd_factor, payload, payload_stride, M, ptr_vec, stream);
            break;
        default: set_error("ga_demo_encode_sym: unknown dtype %d", dtype); return GA_EINVAL;
    }
    return check_launch("ga_demo_encode_sym");
}

extern "C" GA_API int ga_demo_decode_sym(int dtype, const ga_demo_tensor* tensors, int32_t ntensors,
                                         int32_t nchunks, const ga_demo_rowgroup* groups, int32_t ngroups,
                                         const float* F64, const int32_t* payload, int64_t payload_stride, int64_t M,
                                         int64_t S, void* param, void* grad, int64_t K, int64_t ld, float lr,
                                         hipStream_t stream) {
    clear_error();
    GA_REQUIRE(ntensors >= 0 && nchunks >= 0 && ngroups >= 0 && (nchunks > 0 || ngroups > 0),
               "ga_demo_decode_sym: empty plan (ntensors=%d nchunks=%d ngroups=%d)", ntensors, nchunks, ngroups);
    GA_REQUIRE(nchunks == 0 || (tensors && ntensors >= 1), "ga_demo_decode_sym: no descriptors");
    GA_REQUIRE(ngroups == 0 || groups, "ga_demo_decode_sym: no row groups");
    GA_REQUIRE(F64 && payload && param, "ga_demo_decode_sym: null buffer");
    GA_REQUIRE(S >= 1 && S <= dw::kMaxSrc, "ga_demo_decode_sym: S=%lld sources (1..%d; use ga_demo_decode)",
               (long long)S, dw::kMaxSrc);
    GA_REQUIRE(S == 1 || payload_stride >= 2 * M, "ga_demo_decode_sym: payload_stride < 2*M");
    GA_REQUIRE(K >= 1 && (K == 1 || ld > 0), "ga_demo_decode_sym: bad K=%lld / ld", (long long)K);
    const int vb = dtype == GA_F32 ? 16 : 8;
    const int ptr_vec = ((uintptr_t)param % vb == 0) && (grad == nullptr || (uintptr_t)grad % vb == 0) &&
                        (K == 1 || ld % 4 == 0);
    switch (dtype) {
        case GA_F32:
            dw::launch_decode<float>(tensors, ntensors, nchunks, groups, ngroups, F64, payload, payload_stride, M,
                                     (int)S, param, grad, K, ld, lr, ptr_vec, stream);
            break;
        case GA_BF16:
            dw::launch_decode<__hip_bfloat16>(tensors, ntensors, nchunks, groups, ngroups, F64, payload,
                                              payload_stride, M, (int)S, param, grad, K, ld, lr, ptr_vec, stream);
            break;
        default: set_error("ga_demo_decode_sym: unknown dtype %d", dtype); return GA_EINVAL;
    }
    return check_launch("ga_demo_decode_sym");
}
