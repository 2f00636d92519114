// DeMo DCT codec on gfx950: chunked DCT-II encode + per-chunk top-k + residual
// update (ga_demo_encode) and the gathered scatter-mean + inverse DCT + sign-SGD
// apply (ga_demo_decode).
//
// Persistent workgroups (256 lanes = 4 waves; as many as fit the chip, 3-4 per CU)
// walk the chunks of every tensor with a stride of the grid size; the next
// chunk's operands are loaded into registers while the current one is being
// transformed (the barriers inside a chunk wait for LDS only, so those loads stay
// in flight), and a chunk's DCT basis is staged into LDS only when it changes.
//
// Transforms run on the matrix cores (v_mfma_f32_32x32x2_f32: exact f32 FMA
// chains in k order; each wave owns one 32x32 quadrant of the 64x64 tile):
//   dense   64x64x64 products for the forward DCT (encode) and the gathered
//           inverse DCT of several sources (decode);
//   sparse  sum_e v_e * F1[:, b_e] (x) F2[:, d_e] over an entry list, as
//           ceil(E/2) MFMAs whose operands are read straight from the entry list
//           and the LDS basis: the encode residual (k entries) and the decode of
//           a single source.
// Chunks with n1, n2 < 64 are computed zero padded: the basis tables are zero
// outside n x n, so padded rows/columns are exactly 0.
//
// LDS per workgroup (~40 KB): one 64x65 working tile, the chunk's basis F
// (spatial row i, frequency column k) with the same 65-float row stride (every
// operand orientation reads 32 consecutive lanes from 32 banks), the 256 lane
// maxima and a 512-entry list.
//
// Top-k (demo.py:315-328, torch.topk(|x|, k, sorted=False)) is exact; among
// coefficients tied with the k-th magnitude the lowest index wins, and a
// chunk's entries are emitted in ascending index order (the reference's order
// is unspecified; only the set matters).  Keys come straight from the MFMA
// accumulators: T0 = a lower bound of the k-th largest key from the 256
// per-lane maxima, the keys >= T0 (about k of them on DCT coefficients) are
// compacted into LDS and one wave bitonic-sorts them (key desc, index asc),
// then re-sorts the first k by index.  A radix select handles the rest
// (more than 256 candidates, e.g. an all-zero chunk where every key ties, or
// k > 256).
#include "ga_common.h"

namespace ga {

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its outstanding global loads (the register prefetch of
// the next chunk stays in flight; __syncthreads() would drain it).
#define LDS_BARRIER()                                                    \
    do {                                                                 \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  \
        __builtin_amdgcn_s_barrier();                                    \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");  \
    } while (0)

// Diagnostic build only (tools/demo_stamps.py, -DGA_DEMO_STAMPS): per-phase
// s_memtime sums per workgroup, one row of 16 per workgroup, written at exit
// into a buffer nothing else reads.
#ifdef GA_DEMO_STAMPS
__device__ unsigned long long* g_demo_stamps;
#define GA_PH_DECL unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ph_last = __builtin_amdgcn_s_memtime()
#define GA_PH(i)                                            \
    do {                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph_acc[i] += t_ - ph_last;                          \
        ph_last = t_;                                       \
    } while (0)
#define GA_PH_FLUSH(nch)                                                                              \
    do {                                                                                              \
        if (threadIdx.x == 0) {                                                                       \
            unsigned long long* row_ = g_demo_stamps + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16; \
            for (int i_ = 0; i_ < 8; ++i_) row_[i_] = ph_acc[i_];                                     \
            row_[8] = (nch);                                                                          \
        }                                                                                             \
    } while (0)
#else
#define GA_PH_DECL do {} while (0)
#define GA_PH(i) do {} while (0)
#define GA_PH_FLUSH(nch) do {} while (0)
#endif

constexpr int kDmBlock = 256;
constexpr int kLd = 65;
constexpr int kTile = 64 * kLd;
constexpr int kEntMax = 512;  // entries per chunk (topk <= 512)
constexpr int kSortMax = 128; // fast-path candidates (2 per lane of one wave)

typedef float f32x16 __attribute__((ext_vector_type(16)));

// opaque_tid() behind an empty volatile asm: lane-dependent addresses derived from
// it are recomputed where they are used instead of being hoisted out of the
// persistent chunk loop (where dozens of them would stay live in VGPRs).
__device__ __forceinline__ int opaque_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

__device__ __forceinline__ f32x16 zero16() {
    f32x16 a;
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.f;
    return a;
}

// Quadrant of C = A . B (64x64x64) for this wave, operands addressed by
// compile-time strides: A[i][k] = A[i*ASI + k*ASK], B[k][j] = B[k*BSK + j*BSJ].
template <int ASI, int ASK, int BSK, int BSJ>
__device__ __forceinline__ f32x16 mm64(const float* A, const float* Bm, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int i = 32 * (w >> 1) + (lane & 31);
    const int j = 32 * (w & 1) + (lane & 31);
    const int h = lane >> 5;
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 32; ++s) {
        const int k = 2 * s + h;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[i * ASI + k * ASK], Bm[k * BSK + j * BSJ], acc, 0, 0, 0);
    }
    return acc;
}

// operand addressing modes
#define TILE_ROW kLd, 1      // a 64x65 LDS tile, or the LDS basis F, read by rows
#define TILE_COL 1, kLd      // the same, transposed (F^T)
#define GTAB_COL 1, 64       // a 64x64 global table, transposed
#define GTAB_ROW 64, 1       // a 64x64 global table, by rows

// GA_BF16_REF: the reference's bf16 arithmetic (demo.py:235-236, 238-252 as torch
// runs it): every stage of a transform rounds to bf16 (nearest even)
__device__ __forceinline__ float bf16r(float v) { return __bfloat162float(__float2bfloat16(v)); }
__device__ __forceinline__ void round16(f32x16& a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = bf16r(a[r]);
}

// Row / column of accumulator register r for this lane (C/D layout of the 32x32 MFMA).
__device__ __forceinline__ int acc_row(int r, int tid) {
    const int w = tid >> 6, lane = tid & 63;
    return 32 * (w >> 1) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col(int tid) {
    const int w = tid >> 6, lane = tid & 63;
    return 32 * (w & 1) + (lane & 31);
}

__device__ __forceinline__ void store_acc(float* tile, const f32x16& acc, int tid) {
    const int c = acc_col(tid);
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[acc_row(r, tid) * kLd + c] = acc[r];
}

// The reference's decode of a coefficient tile S (natural layout, LDS) in bf16
// stages: Z = bf16(F1 . S) (einsum_2d_t contracts the coefficient rows first,
// B1[k][b] = F1[b][k]), then R = bf16(Z . F2^T); n1 == 1: one stage (the 1-D
// einsum_2d_t).  F1 from the LDS basis (f1 = 0: F1 == F2), the global DCT table
// (f1 = 1: tab1 = F1, row-major) or the inverse table (f1 = 2: tab1 = B1 = F1^T).
// Leaves R in S (natural layout); barriers inside.
__device__ __forceinline__ void ref_inverse(float* S, const float* FT, const float* tab1, int f1, int n1, int tid) {
    f32x16 acc;
    if (n1 > 1) {
        acc = f1 == 0 ? mm64<TILE_ROW, TILE_ROW>(FT, S, tid)
                      : (f1 == 1 ? mm64<GTAB_ROW, TILE_ROW>(tab1, S, tid) : mm64<GTAB_COL, TILE_ROW>(tab1, S, tid));
        round16(acc);
        LDS_BARRIER();
        store_acc(S, acc, tid);
        LDS_BARRIER();
    }
    acc = mm64<TILE_ROW, TILE_COL>(S, FT, tid);  // . F2^T
    round16(acc);
    LDS_BARRIER();
    store_acc(S, acc, tid);
    LDS_BARRIER();
}

// ---- DCT symmetry (64-point bases): F[63-i][k] = (-1)^k F[i][k] ----
// The forward products then need half the MFMAs: with Xe = X[:, i] + X[:, 63-i]
// and Xo = X[:, i] - X[:, 63-i] (i < 32), T[:, k] = Xe . F[:32, k] for even k and
// Xo . F[:32, k] for odd k (K = 32 instead of 64).  Outputs come in a permuted
// order: wave quadrant column j' of half qc is frequency 2j' + qc (and, for the
// second product, row i' of half qr is frequency 2i' + qr).

// T'[r][32qc + j'] = sum_{k<32} X[r][32qc + k] . F[k][2j' + qc]; the tile holds
// [Xe | Xo] in its two column halves (put_tile_sym).
__device__ __forceinline__ f32x16 mm_sym1(const float* X, const float* FT, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int qr = w >> 1, qc = w & 1, h = lane >> 5, l = lane & 31;
    const float* A = X + (32 * qr + l) * kLd + 32 * qc;
    const float* Bm = FT + 2 * l + qc;
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int k = 2 * s + h;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[k], Bm[k * kLd], acc, 0, 0, 0);
    }
    return acc;
}

// Y'[32qr + i'][c] = sum_{r<32} F1[r][2i' + qr] . (T'[r][c] +- T'[63-r][c])
// (+ for even output frequencies, - for odd).
__device__ __forceinline__ f32x16 mm_sym2(const float* T, const float* FT, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int qr = w >> 1, qc = w & 1, h = lane >> 5, l = lane & 31;
    const float* A = FT + 2 * l + qr;
    const float* Bt = T + 32 * qc + l;
    const float sg = qr ? -1.f : 1.f;
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int k = 2 * s + h;
        const float b = fmaf(sg, Bt[(63 - k) * kLd], Bt[k * kLd]);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[k * kLd], b, acc, 0, 0, 0);
    }
    return acc;
}

// Inverse transforms with the same symmetry (decode, several sources):
// U = S . F2^T with U[b][j] = Ue + Uo, U[b][63-j] = Ue - Uo (j < 32), where
// Ue/Uo sum over the even/odd columns d of S.  Wave (qr, par) computes rows
// 32qr.. of U' = [Ue | Uo] (K = 32), stored back as that quadrant.
__device__ __forceinline__ f32x16 mm_isym1(const float* S, const float* FT, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int qr = w >> 1, par = w & 1, h = lane >> 5, l = lane & 31;
    const float* A = S + (32 * qr + l) * kLd + par;
    const float* Bm = FT + l * kLd + par;
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int k = 2 * (2 * s + h);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[k], Bm[k], acc, 0, 0, 0);
    }
    return acc;
}

// g = F1 . U with g[i] = ge + go, g[63-i] = ge - go (i < 32), ge/go summing over
// the even/odd rows b of U, U read from U' (mm_isym1).  Wave (par, qc) computes
// rows i < 32 of ge (par 0) / go (par 1) for natural columns 32qc.., stored at
// tile rows 32*par + i: the [ge ; go] layout the split read combines.
__device__ __forceinline__ f32x16 mm_isym2(const float* U, const float* FT, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int par = w >> 1, qc = w & 1, h = lane >> 5, l = lane & 31;
    const float* A = FT + l * kLd + par;
    // U[b][32qc + l]: qc 0 -> U'[b][l] + U'[b][32 + l]; qc 1 -> U'[b][31 - l] - U'[b][63 - l]
    const float* U0 = U + (qc ? 31 - l : l);
    const float sg = qc ? -1.f : 1.f;
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int k = 2 * (2 * s + h);  // b = k + par
        const float* row = U0 + (k + par) * kLd;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[k], fmaf(sg, row[32], row[0]), acc, 0, 0, 0);
    }
    return acc;
}

// Natural (row, column) of this lane's accumulators and the tile position of a
// natural coefficient, for the plain and the permuted (symmetric) layouts.
struct Perm {
    bool rowp, colp;
    int tid;
    __device__ __forceinline__ int row(int r) const {
        const int lane = tid & 63, w = tid >> 6;
        const int ip = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        return rowp ? 2 * ip + (w >> 1) : 32 * (w >> 1) + ip;
    }
    __device__ __forceinline__ int col() const {
        const int lane = tid & 63, w = tid >> 6;
        return colp ? 2 * (lane & 31) + (w & 1) : 32 * (w & 1) + (lane & 31);
    }
    __device__ __forceinline__ int tile(int b, int d) const {
        const int tr = rowp ? 32 * (b & 1) + (b >> 1) : b;
        const int tc = colp ? 32 * (d & 1) + (d >> 1) : d;
        return tr * kLd + tc;
    }
};

// Largest descriptor index t >= tix with chunk_start <= chunk (chunk_start is
// strictly increasing).  Wave-level (ballot), no LDS, no barrier; uniform.
__device__ __forceinline__ int advance_tensor(const ga_demo_tensor* T, int ntens, int tix, int chunk, int tid) {
    const int lane = tid & 63;
    for (;;) {
        const int t = tix + 1 + lane;
        const bool le = t < ntens && T[t].chunk_start <= chunk;
        const uint64_t m = __ballot(le);
        tix += __popcll(m);
        if (m != ~0ull) return tix;
    }
}

// ---- chunk I/O: lane t owns rows (t>>4) + 16i (i < 4), columns 4(t&15) .. +3 ----
struct ChunkIO {
    int64_t base;  // element offset of the chunk's (0, 0)
    int cols, n1, n2;
    int r0, c0;    // this lane's first row / column
    bool vec;      // 4-element vector accesses are legal for this tensor
    __device__ __forceinline__ int row(int i) const { return r0 + 16 * i; }
    __device__ __forceinline__ int col0() const { return c0; }
    __device__ __forceinline__ bool live(int i) const { return row(i) < n1 && col0() < n2; }
    __device__ __forceinline__ int64_t addr(int i) const { return base + (int64_t)row(i) * cols + col0(); }
};

template <typename T>
__device__ __forceinline__ void load4(const T* p, const ChunkIO& io, int i, float (&v)[4]) {
    if (io.vec) {
        Vec4<T>::unpack(*reinterpret_cast<const typename Vec4<T>::type*>(p + io.addr(i)), v);
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (io.col0() + c < io.n2) ? Elem<T>::load(p + io.addr(i) + c) : 0.f;
    }
}

template <typename T>
__device__ __forceinline__ void store4(T* p, const ChunkIO& io, int i, const float (&v)[4]) {
    if (io.vec) {
        *reinterpret_cast<typename Vec4<T>::type*>(p + io.addr(i)) = Vec4<T>::pack(v);
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (io.col0() + c < io.n2) Elem<T>::store(p + io.addr(i) + c, v[c]);
    }
}

// a whole chunk (this lane's 16 elements; zeros outside the tensor)
template <typename T>
__device__ __forceinline__ void load_chunk(const T* p, const ChunkIO& io, float (&v)[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (io.live(i)) load4(p, io, i, v[i]);
        else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[i][e] = 0.f;
        }
    }
}

template <typename T>
__device__ __forceinline__ ChunkIO chunk_io(const ga_demo_tensor& td, int c, bool ptr_vec, int tid) {
    ChunkIO io;
    const int cy = c / td.gx, cx = c - cy * td.gx;
    io.base = td.offset + (int64_t)cy * td.n1 * td.cols + (int64_t)cx * td.n2;
    io.cols = td.cols;
    io.n1 = td.n1;
    io.n2 = td.n2;
    io.r0 = tid >> 4;
    io.c0 = 4 * (tid & 15);
    io.vec = ptr_vec && (td.offset % 4 == 0) && (td.cols % 4 == 0) && (td.n2 % 4 == 0);
    return io;
}

// tile row(i), columns col0..+3 <- v (zero outside n2)
__device__ __forceinline__ void put_tile(float* X, const ChunkIO& io, const float (&v)[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) X[io.row(i) * kLd + io.col0() + e] = (io.col0() + e < io.n2) ? v[i][e] : 0.f;
}

// The tile as [Xe | Xo] (see mm_sym1): column c < 32 holds x[c] + x[63-c],
// column 32 + c holds x[c] - x[63-c].  The mirror column of a lane's 4 columns
// belongs to lane ^ 15 of the same row (DPP row_mirror), element 3 - e.
__device__ __forceinline__ void put_tile_sym(float* X, const ChunkIO& io, const float (&v)[4][4]) {
    const bool lo = io.col0() < 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float m = __int_as_float(
                __builtin_amdgcn_mov_dpp(__float_as_int(v[i][3 - e]), 0x140, 0xf, 0xf, false));  // row_mirror
            const int c = io.col0() + e;
            if (lo) X[io.row(i) * kLd + c] = v[i][e] + m;
            else X[io.row(i) * kLd + 95 - c] = m - v[i][e];
        }
    }
}

// Stage a chunk's basis into LDS as F[i*kLd + k] (spatial i, frequency k).
// From the DCT table F (row-major 64x64): a straight copy; from the inverse
// table B = F^T: the transpose.  Global reads are row-major (coalesced); the
// LDS writes of consecutive lanes land in different banks either way.
template <bool FROM_B>
__device__ __forceinline__ void stage_basis(float* FT, const float* tab, int tid) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int q = tid + 256 * r;  // float4 index of the global table
        const float4 v = reinterpret_cast<const float4*>(tab)[q];
        const int row = q >> 4, c0 = 4 * (q & 15);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (FROM_B) FT[(c0 + c) * kLd + row] = vv[c];  // B[row][c0+c] = F[c0+c][row]
            else FT[row * kLd + c0 + c] = vv[c];
        }
    }
}

// How the first factor F1 of a chunk is read: the 1x1 identity (n1 == 1), the
// LDS basis (F1 == F2), or a global 64x64 table (row-major F, or B = F^T).
struct Basis1 {
    int mode;           // 0 identity, 1 LDS, 2 global
    const float* tab;   // mode 2
    bool transposed;    // mode 2: tab is B1 = F1^T
    __device__ __forceinline__ float at(const float* FT, int i, int b) const {
        if (mode == 0) return i == b ? 1.f : 0.f;
        if (mode == 1) return FT[i * kLd + b];
        return transposed ? tab[b * 64 + i] : tab[i * 64 + b];
    }
};

__device__ __forceinline__ Basis1 basis1_of(const ga_demo_tensor& td, const float* tabs, bool transposed) {
    Basis1 b;
    b.mode = td.n1 == 1 ? 0 : (td.basis1 == td.basis2 ? 1 : 2);
    b.tab = tabs + (int64_t)td.basis1 * 4096;
    b.transposed = transposed;
    return b;
}

// R = sum_{e<E} v_e * F1[:, b_e] (x) F2[:, d_e] (this wave's quadrant), entries
// lst[2e] = b_e*64 + d_e, lst[2e+1] = bits of v_e.  The sparse form of
// F1 . S . F2^T = B1^T . S . B2 (demo.py:279-299 with B = F^T): one MFMA per
// pair of entries, the A operand v_e*F1[i][b_e] and the B operand F2[j][d_e]
// read straight from LDS.
__device__ __forceinline__ f32x16 sparse_synth(const uint32_t* lst, int E, const float* FT, const Basis1& b1,
                                               int rowbase, int tid) {
    const int lane = tid & 63, w = tid >> 6;
    const int i = (rowbase < 0 ? 32 * (w >> 1) : rowbase) + (lane & 31);
    const int j = 32 * (w & 1) + (lane & 31);
    const int h = lane >> 5;
    f32x16 acc = zero16();
    for (int e0 = 0; e0 < E; e0 += 8) {
        uint32_t pos[4];
        float v[4], a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + 2 * u + h;
            const bool ok = e < E;
            pos[u] = ok ? lst[2 * e] : 0u;
            v[u] = ok ? __uint_as_float(lst[2 * e + 1]) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = v[u] * b1.at(FT, i, (int)(pos[u] >> 6));
            b[u] = FT[j * kLd + (int)(pos[u] & 63)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
    }
    return acc;
}

// Per-chunk top-k of |y| (y: the MFMA accumulators, coordinates via P) over the
// valid n1 x n2 coefficients.  Output: k entries in ascending coefficient order
// in out_idx/out_val (global), and the entry list (b*64 + d, value bits) in LDS,
// returned: the calling wave's own copy (fast path) or the shared lst (radix
// path).  On entry bm (128 words) is zero and misc[0] == 0 (both published by
// an earlier barrier); tmax: 256 words; cand: 2*kSortMax words; lst: 1024 words
// (per-wave residual lists of 256 words); selm: 4 words; scratch:
// >= 1024 words of LDS free here (the tile).
//
// Fast path (k <= C <= kSortMax): every wave derives T0 from the 256 lane maxima
// (>= k lane maxima, each a key, are >= T0, so T0 <= the k-th largest key) and
// appends its keys >= T0 to a shared candidate list (C of them, about k on DCT
// coefficients) and to a 4096-bit position bitmap.  Then each wave on its own,
// no further barrier: the candidates' coefficient ranks from the bitmap's prefix
// counts, the exact k-th largest key by a bitwise search over ballot counts,
// ties at the k-th key to the lowest coefficients, and each selected entry's
// output slot from a rank-space selection mask.  The radix path handles the
// rest (k > kSortMax, or more than kSortMax candidates, e.g. all-zero chunks
// where every key ties).
__device__ __forceinline__ const uint32_t* topk_emit(const f32x16& y, const Perm& P, int n1, int n2, int k,
                                                     int32_t* out_idx, float* out_val, uint32_t* tmax, uint32_t* bm,
                                                     uint32_t* cand, uint32_t* lst, uint32_t* selm, int* misc,
                                                     float* scratch) {
    const int t = P.tid, lane = t & 63, wid = t >> 6;
    const int col = P.col();
    // key of accumulator r: order-preserving |y| + 1; 0 marks padding
    auto keyof = [&](int r) -> uint32_t {
        return (P.row(r) < n1 && col < n2) ? (__float_as_uint(y[r]) & 0x7fffffffu) + 1u : 0u;
    };
    // append this lane's flagged accumulators to dst as (first(r), second(r)) pairs:
    // wave scan of the per-lane counts, one LDS atomic per wave on misc[slot]
    auto append = [&](uint32_t* dst, int cap, auto flag, auto first, auto second, int slot) {
        int mine = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) mine += flag(r) ? 1 : 0;
        int incl = mine;
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const int yv = __shfl_up(incl, dd, 64);
            if (lane >= dd) incl += yv;
        }
        const int wtot = __shfl(incl, 63, 64);
        int wbase = 0;
        if (lane == 63 && wtot) wbase = atomicAdd(&misc[slot], wtot);
        wbase = __shfl(wbase, 63, 64);
        int at = wbase + incl - mine;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (flag(r)) {
                if (at < cap) {
                    dst[2 * at] = first(r);
                    dst[2 * at + 1] = second(r);
                }
                ++at;
            }
        }
    };
    auto posof = [&](int r) { return (uint32_t)(P.row(r) * 64 + col); };
    auto bitsof = [&](int r) { return __float_as_uint(y[r]); };
    uint32_t mymax = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t kr = keyof(r);
        mymax = kr > mymax ? kr : mymax;
    }
    tmax[t] = mymax;
    LDS_BARRIER();
    if (k <= kSortMax) {
        // T0: the largest 12-bit-granular threshold with >= k lane maxima above it
        uint32_t mx[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) mx[r] = tmax[r * 64 + lane];
        uint32_t T0 = 0;
#pragma unroll
        for (int bit = 30; bit >= 19; --bit) {
            const uint32_t c = T0 | (1u << bit);
            int cnt = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) cnt += __popcll(__ballot(mx[r] >= c));
            if (cnt >= k) T0 = c;
        }
        if (T0 == 0u) T0 = 1u;  // key 0 marks padding; small chunks rank all their keys
        auto is_cand = [&](int r) { return keyof(r) >= T0; };
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (is_cand(r)) {
                const uint32_t pos = posof(r);
                atomicOr(&bm[pos >> 5], 1u << (pos & 31));
            }
        append(cand, kSortMax, is_cand, posof, bitsof, 0);
        LDS_BARRIER();
        const int C = misc[0];
        if (C <= kSortMax) {
            if (wid == 0) {
                // coefficient rank of a position = set bits of the bitmap below it
                const uint32_t w0 = bm[2 * lane], w1 = bm[2 * lane + 1];
                const int cnt = __popc(w0) + __popc(w1);
                int incl = cnt;
#pragma unroll
                for (int dd = 1; dd < 64; dd <<= 1) {
                    const int yv = __shfl_up(incl, dd, 64);
                    if (lane >= dd) incl += yv;
                }
                const int pre = incl - cnt;
                uint32_t pos[2], bits[2], key[2];
                int rank[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int g = e * 64 + lane;
                    const bool ok = g < C;
                    pos[e] = ok ? cand[2 * g] : 0u;
                    bits[e] = ok ? cand[2 * g + 1] : 0u;
                    key[e] = ok ? (bits[e] & 0x7fffffffu) + 1u : 0u;
                    const int L = (int)(pos[e] >> 6);
                    const uint64_t pair = ((uint64_t)(uint32_t)__shfl((int)w1, L, 64) << 32) |
                                          (uint32_t)__shfl((int)w0, L, 64);
                    const int lp = __shfl(pre, L, 64);
                    rank[e] = ok ? lp + __popcll(pair & ((1ull << (pos[e] & 63)) - 1ull)) : 0x7fff;
                }
                // exact k-th largest key
                uint32_t thr = 0;
                for (int bit = 31; bit >= 0; --bit) {
                    const uint32_t c = thr | (1u << bit);
                    if (__popcll(__ballot(key[0] >= c)) + __popcll(__ballot(key[1] >= c)) >= k) thr = c;
                }
                const int need = k - __popcll(__ballot(key[0] > thr)) - __popcll(__ballot(key[1] > thr));
                const uint64_t q0 = __ballot(key[0] == thr), q1 = __ballot(key[1] == thr);
                bool sel[2];
                if (__popcll(q0) + __popcll(q1) == need) {  // every tie is in
                    sel[0] = key[0] >= thr;
                    sel[1] = key[1] >= thr;
                } else {  // ties at the k-th key: the lowest coefficients win
                    int tr[2] = {0, 0};
                    for (uint64_t m = q0; m; m &= m - 1) {
                        const int rj = __shfl(rank[0], __builtin_ctzll(m), 64);
                        tr[0] += rj < rank[0];
                        tr[1] += rj < rank[1];
                    }
                    for (uint64_t m = q1; m; m &= m - 1) {
                        const int rj = __shfl(rank[1], __builtin_ctzll(m), 64);
                        tr[0] += rj < rank[0];
                        tr[1] += rj < rank[1];
                    }
                    sel[0] = key[0] > thr || (key[0] == thr && tr[0] < need);
                    sel[1] = key[1] > thr || (key[1] == thr && tr[1] < need);
                }
                // output slot = selected candidates of lower rank (rank-space mask)
                if (lane < 4) selm[lane] = 0u;
#pragma unroll
                for (int e = 0; e < 2; ++e)
                    if (sel[e]) atomicOr(&selm[rank[e] >> 5], 1u << (rank[e] & 31));
                const uint64_t m0 = ((uint64_t)selm[1] << 32) | selm[0], m1 = ((uint64_t)selm[3] << 32) | selm[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    if (sel[e]) {
                        const int r = rank[e];
                        const int slot = r < 64 ? __popcll(m0 & ((1ull << r) - 1ull))
                                                : __popcll(m0) + __popcll(m1 & ((1ull << (r - 64)) - 1ull));
                        cand[2 * slot] = pos[e];  // the candidates are in registers: reuse the list
                        cand[2 * slot + 1] = bits[e];
                        out_idx[slot] = (int32_t)((pos[e] >> 6) * n2 + (pos[e] & 63));
                        out_val[slot] = __uint_as_float(bits[e]);
                    }
                }
            }
            LDS_BARRIER();
            return cand;
        }
    }
    // radix select of the k-th largest key (4 rounds of 8 bits); hist = tmax
    int* hist = reinterpret_cast<int*>(tmax);
    uint32_t prefix = 0, pmask = 0;
    int kk = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        hist[t] = 0;
        LDS_BARRIER();
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t kr = keyof(r);
            if ((kr & pmask) == prefix) atomicAdd(&hist[(kr >> shift) & 255u], 1);
        }
        LDS_BARRIER();
        if (t < 64) {
            int hb[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) hb[b] = hist[4 * t + b];
            const int lsum = hb[0] + hb[1] + hb[2] + hb[3];
            int x = lsum;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int yv = __shfl_down(x, d, 64);
                if (t + d < 64) x += yv;
            }
            int cum = x - lsum;  // keys in higher buckets
#pragma unroll
            for (int b = 3; b >= 0; --b) {
                if (cum < kk && cum + hb[b] >= kk) {
                    misc[1] = 4 * t + b;
                    misc[2] = kk - cum;
                }
                cum += hb[b];
            }
        }
        LDS_BARRIER();
        prefix |= (uint32_t)misc[1] << shift;
        pmask |= 0xffu << shift;
        kk = misc[2];
        LDS_BARRIER();
    }
    // keys > prefix are in; of the keys == prefix the kk lowest positions are:
    // bitmap of the tied positions (128 words) + per-word prefix counts
    uint32_t* bpre = tmax;  // [128]
    if (t < 128) bm[t] = 0u;
    if (t == 0) misc[3] = 0;
    LDS_BARRIER();
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (keyof(r) == prefix) {
            const int pos = P.row(r) * 64 + col;
            atomicOr(&bm[pos >> 5], 1u << (pos & 31));
        }
    LDS_BARRIER();
    if (t < 64) {
        const int c0 = __popc(bm[2 * t]), c1 = __popc(bm[2 * t + 1]);
        int x = c0 + c1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int yv = __shfl_up(x, d, 64);
            if (lane >= d) x += yv;
        }
        bpre[2 * t] = x - c0 - c1;
        bpre[2 * t + 1] = x - c1;
    }
    LDS_BARRIER();
    // append the selected (pos, bits) in any order, then one wave sorts them by pos
    auto chosen = [&](int r) {
        const uint32_t kr = keyof(r);
        if (kr != prefix) return kr > prefix;
        const int pos = P.row(r) * 64 + col;
        const int rank = (int)bpre[pos >> 5] + __popc(bm[pos >> 5] & ((1u << (pos & 31)) - 1u));
        return rank < kk;
    };
    append(lst, kEntMax, chosen, posof, bitsof, 3);
    LDS_BARRIER();
    // rank each entry by position (k <= 512, at most 2 per lane; rare path), emit,
    // and stage the sorted list in the tile (free here), then copy it to lst
    uint32_t* srt = reinterpret_cast<uint32_t*>(scratch);
    for (int g = t; g < k; g += kDmBlock) {
        const uint32_t pos = lst[2 * g], bits = lst[2 * g + 1];
        int rank = 0;
        for (int e = 0; e < k; ++e) rank += lst[2 * e] < pos;
        out_idx[rank] = (int32_t)((pos >> 6) * n2 + (pos & 63));
        out_val[rank] = __uint_as_float(bits);
        srt[2 * rank] = pos;
        srt[2 * rank + 1] = bits;
    }
    LDS_BARRIER();
    for (int g = t; g < 2 * k; g += kDmBlock) lst[g] = srt[g];
    LDS_BARRIER();
    return lst;
}


constexpr int kDmEncWaves = 3;  // workgroups per CU the encode is compiled for (register budget ~168 VGPRs, no spills)
// REF (T = bf16): the reference's bf16 arithmetic (GA_BF16_REF): delta rounded after
// the decay and after the gradient add, Y = bf16(bf16(F1^T X) F2) (rows first, as the
// reference's einsum contracts), the residual as its bf16 two-stage decode
// (ref_inverse), bf16 bases from the caller's table; no symmetric folding.
template <typename T, bool REF = false>
__global__ __launch_bounds__(kDmBlock, kDmEncWaves) void demo_encode_kernel(
    const ga_demo_tensor* __restrict__ tens, int ntens, int nchunks, const float* __restrict__ F, T* param,
    const T* __restrict__ grad, T* delta, int64_t ld, float lr, float decay, float wd_factor, int32_t* payload,
    int64_t pstride, int64_t M, int ptr_vec) {
    __shared__ float X[kTile];   // delta -> T -> (Y) -> the residual
    __shared__ float FT[kTile];  // basis F (row stride kLd)
    __shared__ uint32_t tmax[kDmBlock];
    __shared__ uint32_t lst[2 * kEntMax];   // entry lists (per wave, or shared on the radix path)
    __shared__ uint32_t cand[2 * kSortMax]; // top-k candidates
    __shared__ uint32_t bm[128];            // top-k position bitmap
    __shared__ uint32_t selm[16];           // per-wave selection masks
    __shared__ int misc[4];

    int chunk = blockIdx.x;
    if (chunk >= nchunks) return;
    const int64_t rep = blockIdx.y;
    param += rep * ld;
    grad += rep * ld;
    delta += rep * ld;
    payload += rep * pstride;
    float* vals = reinterpret_cast<float*>(payload + M);
    GA_PH_DECL;

    const int tid0 = opaque_tid();
    int tix = advance_tensor(tens, ntens, -1, chunk, tid0);
    ga_demo_tensor td = tens[tix];
    ChunkIO io = chunk_io<T>(td, chunk - td.chunk_start, ptr_vec != 0, tid0);
    float d[4][4], g[4][4];
    load_chunk(delta, io, d);
    load_chunk(grad, io, g);
    int staged = -1;
    int done = 0;
    (void)done;
    for (;;) {
        // this iteration's lane id: everything lane-dependent is derived from it here,
        // not hoisted out of the loop into long-lived registers
        const int tid = opaque_tid();
        const int c = chunk - td.chunk_start;
        const int n1 = td.n1, n2 = td.n2, k = td.k;
        if (td.basis2 != staged) {  // uniform; the barrier below publishes it
            stage_basis<false>(FT, F + (int64_t)td.basis2 * 4096, tid);
            staged = td.basis2;
        }
        // 1. error feedback in registers: x = decay*delta + lr*grad (+ decoupled weight decay on p)
        if (wd_factor != 1.f) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (io.live(i)) {
                    float p[4];
                    load4(param, io, i, p);
#pragma unroll
                    for (int e = 0; e < 4; ++e) p[e] *= wd_factor;
                    store4(param, io, i, p);
                }
            }
        }
        {
            const int tq = tid;
            if (tq < 128) bm[tq] = 0u;  // top-k state of this chunk, published by the barriers below
            if (tq == 0) misc[0] = 0;
        }
        float x[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (REF) {  // delta.mul_(decay) then delta.add_(grad, alpha=lr), each a bf16 tensor op
                    const float d1 = decay != 1.f ? bf16r(d[i][e] * decay) : d[i][e];
                    x[i][e] = bf16r(fmaf(lr, g[i][e], d1));
                } else {
                    x[i][e] = fmaf(lr, g[i][e], decay != 1.f ? d[i][e] * decay : d[i][e]);
                }
            }
        const bool sym = !REF && n2 == 64 && (n1 == 64 || n1 == 1);  // uniform
        if (sym) put_tile_sym(X, io, x);
        else put_tile(X, io, x);
        // prefetch the next chunk's delta and grad (in flight until the next iteration)
        const int next = chunk + (int)gridDim.x;
        const bool more = next < nchunks;
        int tixn = tix;
        ga_demo_tensor tdn = td;
        ChunkIO ion = io;
        if (more) {
            tixn = advance_tensor(tens, ntens, tix, next, tid);
            tdn = tens[tixn];
            ion = chunk_io<T>(tdn, next - tdn.chunk_start, ptr_vec != 0, tid);
            load_chunk(delta, ion, d);
            load_chunk(grad, ion, g);
        }
        LDS_BARRIER();
        GA_PH(0);

        // 2. Y = F1^T . X . F2 on the matrix cores (half the MFMAs for 64-point bases)
        f32x16 acc;
        if (REF) {  // U = bf16(F1^T . X) (the chunk rows first), Y = bf16(U . F2)
            const int tid = opaque_tid();
            if (n1 > 1) {
                acc = td.basis1 == td.basis2 ? mm64<TILE_COL, TILE_ROW>(FT, X, tid)
                                             : mm64<GTAB_COL, TILE_ROW>(F + (int64_t)td.basis1 * 4096, X, tid);
                round16(acc);
                LDS_BARRIER();
                store_acc(X, acc, tid);
                LDS_BARRIER();
            }
            acc = mm64<TILE_ROW, TILE_ROW>(X, FT, tid);
            round16(acc);
            GA_PH(1);
        } else {
        {
            const int tid = opaque_tid();  // a fresh lane id per phase keeps its derived values short-lived
        if (sym) {
            acc = mm_sym1(X, FT, tid);  // reads only this wave's quadrant of X: T' goes back in place
        } else {
            acc = mm64<TILE_ROW, TILE_ROW>(X, FT, tid);  // T = X . F2
            LDS_BARRIER();
        }
        store_acc(X, acc, tid);
        LDS_BARRIER();
        GA_PH(1);
        }
        {
            const int tid = opaque_tid();
        if (n1 > 1) {
            if (sym) acc = mm_sym2(X, FT, tid);  // F1^T . T
            else if (td.basis1 == td.basis2) acc = mm64<TILE_COL, TILE_ROW>(FT, X, tid);
            else acc = mm64<GTAB_COL, TILE_ROW>(F + (int64_t)td.basis1 * 4096, X, tid);
        }  // n1 == 1: F1 = [1], Y = T
        }
        }
        GA_PH(2);
        Perm P;
        P.tid = opaque_tid();
        P.colp = sym;
        P.rowp = sym && n1 > 1;

        // 3. top-k of |Y| -> payload entries (ascending index) + LDS entry list
        const int64_t e0 = td.payload_off + (int64_t)c * k;
        const uint32_t* ent = topk_emit(acc, P, n1, n2, k, payload + e0, vals + e0, tmax, bm, cand, lst, selm,
                                        misc, X);
        GA_PH(3);

        // 4. residual: delta = x - sum_e v_e * F1[:, b_e] (x) F2[:, d_e]  (demo.py:174-180).
        //    Per-wave list with 64-point row bases: waves of row half 0 sum the even-b
        //    entries (Re), of half 1 the odd-b ones (Ro), over rows i < 32 only; then
        //    R[i] = Re[i] + Ro[i] and R[63-i] = Re[i] - Ro[i].
        const bool split = P.rowp && ent == cand;  // uniform
        f32x16 R;
        const int tid4 = opaque_tid();
        if (REF) {
            // the reference's transmit_grad: decompress (the k entries into a zero tile), then
            // its bf16 two-stage decode (demo.py:174-180); R is left in X
            LDS_BARRIER();  // every wave is done with its top-k reads of X
            for (int q = tid4; q < kTile; q += kDmBlock) X[q] = 0.f;
            LDS_BARRIER();
            for (int j = tid4; j < k; j += kDmBlock) {
                const uint32_t pos = ent[2 * j];
                X[(pos >> 6) * kLd + (pos & 63)] = __uint_as_float(ent[2 * j + 1]);
            }
            LDS_BARRIER();
            ref_inverse(X, FT, F + (int64_t)td.basis1 * 4096, td.basis1 == td.basis2 ? 0 : 1, n1, tid4);
        } else if (split) {
            const int tid = tid4;
            const int lane = tid & 63, par = tid >> 7;
            uint32_t* own = lst + 256 * (tid >> 6);
            uint32_t ep[2], ev[2];
            bool mine[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int gq = e * 64 + lane;
                ep[e] = gq < k ? ent[2 * gq] : 0u;
                ev[e] = gq < k ? ent[2 * gq + 1] : 0u;
                mine[e] = gq < k && (int)((ep[e] >> 6) & 1u) == par;
            }
            const uint64_t b0 = __ballot(mine[0]), b1 = __ballot(mine[1]);
            const uint64_t blw = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                if (mine[e]) {
                    const int at = e == 0 ? __popcll(b0 & blw) : __popcll(b0) + __popcll(b1 & blw);
                    own[2 * at] = ep[e];
                    own[2 * at + 1] = ev[e];
                }
            }
            R = sparse_synth(own, __popcll(b0) + __popcll(b1), FT, basis1_of(td, F, false), 0, tid);
        } else {
            R = sparse_synth(ent, k, FT, basis1_of(td, F, false), -1, tid4);
        }
        if (!REF) {
            store_acc(X, R, tid4);  // X is free: every wave is past its last read of T (top-k barriers)
            LDS_BARRIER();
        }
        GA_PH(4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (io.live(i)) {
                float o[4];
                const int rr = io.row(i);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int cc = io.col0() + e;
                    float rv;
                    if (!split) rv = X[rr * kLd + cc];
                    else if (i < 2) rv = X[rr * kLd + cc] + X[(32 + rr) * kLd + cc];  // rows < 32
                    else rv = X[(63 - rr) * kLd + cc] - X[(95 - rr) * kLd + cc];
                    o[e] = x[i][e] - rv;
                }
                store4(delta, io, i, o);
            }
        }
        ++done;
        GA_PH(5);
        if (!more) break;
        chunk = next;
        tix = tixn;
        td = tdn;
        io = ion;
        LDS_BARRIER();  // every lane has read the residual out of X
    }
    GA_PH_FLUSH(done);
}

// Decode.  nsrc == 1: the single source's entries are distinct, the mean is the
// value itself, and the inverse DCT is the sparse synthesis of those entries.
// nsrc > 1: node-ordered scatter-mean into the tile, then two dense products.
constexpr int kPfSrc = 8;  // sources whose entries are prefetched into registers (k <= 256)

// REF (T = bf16): the reference's bf16 decode (GA_BF16_REF): the scatter-mean
// rounded to bf16, then its two-stage bf16 inverse (ref_inverse), also for one source.
template <typename T, typename CntT, bool REF = false>
__global__ __launch_bounds__(kDmBlock, sizeof(CntT) == 1 ? 4 : 3) void demo_decode_kernel(
    const ga_demo_tensor* __restrict__ tens, int ntens, int nchunks, const float* __restrict__ B,
    const int32_t* __restrict__ payload, int64_t pstride, int64_t M, int nsrc, T* param, T* grad, int64_t K,
    int64_t ld, float lr, int ptr_vec) {
    __shared__ float S[kTile];   // scatter-mean tile -> U -> g (in place)
    __shared__ float FT[kTile];  // basis F (row stride kLd), staged from B = F^T
    constexpr int kCntWords = (4096 * (int)sizeof(CntT) + 3) / 4;
    constexpr int kAuxWords = kCntWords > 2 * kEntMax ? kCntWords : 2 * kEntMax;
    __shared__ uint32_t aux[kAuxWords];  // hit counts (nsrc > 1) | entry list (nsrc == 1)
    CntT* cnt = reinterpret_cast<CntT*>(aux);
    uint32_t* lst = aux;

    int chunk = blockIdx.x;
    if (chunk >= nchunks) return;
    const bool pf = nsrc <= kPfSrc;  // k <= 256 is checked per tensor below
    const int t = opaque_tid();

    int tix = advance_tensor(tens, ntens, -1, chunk, t);
    ga_demo_tensor td = tens[tix];
    ChunkIO io = chunk_io<T>(td, chunk - td.chunk_start, ptr_vec != 0, t);
    int32_t pidx[kPfSrc];
    float pval[kPfSrc];
    auto fetch_entries = [&](const ga_demo_tensor& tq, int cq, int t) {
        const int64_t eo = tq.payload_off + (int64_t)cq * tq.k;
#pragma unroll
        for (int s = 0; s < kPfSrc; ++s) {
            pidx[s] = -1;
            pval[s] = 0.f;
            if (s < nsrc && t < tq.k) {
                pidx[s] = payload[s * pstride + eo + t];
                pval[s] = reinterpret_cast<const float*>(payload + s * pstride + M)[eo + t];
            }
        }
    };
    float p0[4][4];
    if (pf && td.k <= kDmBlock) fetch_entries(td, chunk - td.chunk_start, t);
    load_chunk(param, io, p0);
    int staged = -1;
    for (;;) {
        const int tid = opaque_tid();  // this iteration's lane id (see encode)
        const int c = chunk - td.chunk_start;
        const int n1 = td.n1, n2 = td.n2, nk = td.k, nvalid = n1 * n2;
        const bool use_pf = pf && nk <= kDmBlock;
        if (td.basis2 != staged) {
            stage_basis<true>(FT, B + (int64_t)td.basis2 * 4096, tid);
            staged = td.basis2;
        }
        const int64_t eoff = td.payload_off + (int64_t)c * nk;
        f32x16 acc;
        // the dense (several-source) inverse uses the DCT symmetry for 64-point bases
        const bool dsym = !REF && nsrc > 1 && n2 == 64 && (n1 == 64 || n1 == 1);  // uniform
        const int next = chunk + (int)gridDim.x;
        const bool more = next < nchunks;
        int tixn = tix;
        ga_demo_tensor tdn = td;
        if (more) {
            tixn = advance_tensor(tens, ntens, tix, next, tid);
            tdn = tens[tixn];
        }
        if (nsrc == 1 && !REF) {
            // entry list (b*64 + d, value) straight from the payload
            for (int j = tid; j < nk; j += kDmBlock) {
                const int x = use_pf ? pidx[0] : payload[eoff + j];
                const float v = use_pf ? pval[0] : reinterpret_cast<const float*>(payload + M)[eoff + j];
                const bool ok = x >= 0 && x < nvalid;
                const int b = ok ? x / n2 : 0, dd = ok ? x - b * n2 : 0;
                lst[2 * j] = (uint32_t)(b * 64 + dd);
                lst[2 * j + 1] = __float_as_uint(ok ? v : 0.f);
            }
            if (more && pf && tdn.k <= kDmBlock) fetch_entries(tdn, next - tdn.chunk_start, tid);
            LDS_BARRIER();
            acc = sparse_synth(lst, nk, FT, basis1_of(td, B, true), -1, tid);
        } else {
            for (int e = tid; e < kTile; e += kDmBlock) S[e] = 0.f;
            for (int e = tid; e < kCntWords; e += kDmBlock) aux[e] = 0u;
            LDS_BARRIER();
            // scatter-mean (demo.py:331-352): sources in node order; one source's
            // indices are distinct, so each source is one conflict-free pass and the
            // per-coefficient sums accumulate in node order.
            // REF: the running sum rounded to bf16 after every source's add, in node order
            // (torch's bf16 scatter_reduce adds with bf16 rounding per add; its GPU atomics
            // add in an unspecified order, which matters only at 3+ hitters of a position)
            auto hit = [&](int x, float v) {
                if (x >= 0 && x < nvalid) {
                    const int b = x / n2, dd = x - b * n2;
                    const float sum = S[b * kLd + dd] + v;
                    S[b * kLd + dd] = REF ? bf16r(sum) : sum;
                    cnt[b * 64 + dd] += 1;
                }
            };
            if (use_pf) {
#pragma unroll
                for (int s = 0; s < kPfSrc; ++s) {
                    if (s < nsrc) {  // uniform
                        if (tid < nk) hit(pidx[s], pval[s]);
                        LDS_BARRIER();
                    }
                }
            } else {
                for (int s = 0; s < nsrc; ++s) {
                    for (int j = tid; j < nk; j += kDmBlock)
                        hit(payload[(int64_t)s * pstride + eoff + j],
                            reinterpret_cast<const float*>(payload + (int64_t)s * pstride + M)[eoff + j]);
                    LDS_BARRIER();
                }
            }
            if (more && pf && tdn.k <= kDmBlock) fetch_entries(tdn, next - tdn.chunk_start, tid);
            for (int e = tid; e < 4096; e += kDmBlock) {
                const int n = cnt[e];
                if (n > 1) S[(e >> 6) * kLd + (e & 63)] /= (float)n;
                if (REF) S[(e >> 6) * kLd + (e & 63)] = bf16r(S[(e >> 6) * kLd + (e & 63)]);
            }
            LDS_BARRIER();
            if (REF) ref_inverse(S, FT, B + (int64_t)td.basis1 * 4096, td.basis1 == td.basis2 ? 0 : 2, n1, tid);
            if (!REF) {
            // g = B1^T . S . B2 = F1 . S . F2^T on the matrix cores, in place in S
            // (half the MFMAs for 64-point bases: mm_isym1 / mm_isym2)
            acc = dsym ? mm_isym1(S, FT, tid) : mm64<TILE_ROW, TILE_COL>(S, FT, tid);  // U = S . F2^T
            LDS_BARRIER();
            store_acc(S, acc, tid);
            LDS_BARRIER();
            if (n1 > 1) {
                if (dsym) acc = mm_isym2(S, FT, tid);  // F1 . U
                else if (td.basis1 == td.basis2) acc = mm64<TILE_ROW, TILE_ROW>(FT, S, tid);
                else acc = mm64<GTAB_COL, TILE_ROW>(B + (int64_t)td.basis1 * 4096, S, tid);  // F1[i][k] = B1[k][i]
                LDS_BARRIER();
            }
            }  // !REF
        }
        if (!REF) {  // REF: ref_inverse left g in S
            store_acc(S, acc, tid);
            LDS_BARRIER();
        }
        // grad = sign(g) (torch.sign: NaN -> 0);  p -= lr * grad   (demo.py:200-209)
        float p1[4][4];
        ChunkIO ion = io;
        if (more) ion = chunk_io<T>(tdn, next - tdn.chunk_start, ptr_vec != 0, tid);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float sg[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int rr = io.row(i), cc = io.col0() + e;
                float gv;
                if (!dsym) gv = S[rr * kLd + cc];
                else if (n1 == 1) gv = cc < 32 ? S[rr * kLd + cc] + S[rr * kLd + 32 + cc]  // [Ue | Uo] of row 0
                                               : S[rr * kLd + 63 - cc] - S[rr * kLd + 95 - cc];
                else if (i < 2) gv = S[rr * kLd + cc] + S[(32 + rr) * kLd + cc];  // [ge ; go], rows < 32
                else gv = S[(63 - rr) * kLd + cc] - S[(95 - rr) * kLd + cc];
                sg[e] = (float)((gv > 0.f) - (gv < 0.f));
            }
            if (io.live(i)) {
                float p[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) p[e] = fmaf(-lr, sg[e], p0[i][e]);
                store4(param, io, i, p);
                if (grad) store4(grad, io, i, sg);
                for (int64_t kr = 1; kr < K; ++kr) {
                    load4(param + kr * ld, io, i, p);
#pragma unroll
                    for (int e = 0; e < 4; ++e) p[e] = fmaf(-lr, sg[e], p[e]);
                    store4(param + kr * ld, io, i, p);
                    if (grad) store4(grad + kr * ld, io, i, sg);
                }
            }
        }
        if (!more) break;
        load_chunk(param, ion, p1);  // the next chunk's replica-0 parameters
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) p0[i][e] = p1[i][e];
        chunk = next;
        tix = tixn;
        td = tdn;
        io = ion;
        LDS_BARRIER();  // every lane has read g out of S
    }
}

// Persistent grid: as many workgroups per replica as are resident at once.
template <typename K>
static int resident_blocks(K kernel) {
    int dev = 0, cus = 256, per = 4;
    if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kernel, kDmBlock, 0) == hipSuccess && v > 0) per = v;
    }
    return cus * per;
}

static dim3 persistent_grid(int resident, int nchunks, int64_t reps) {
    int64_t per_rep = (resident + reps - 1) / reps;
    if (per_rep > nchunks) per_rep = nchunks;
    if (per_rep < 1) per_rep = 1;
    return dim3((unsigned)per_rep, (unsigned)reps);
}

static int check_tensors_host(int32_t ntensors, int32_t nchunks) {
    GA_REQUIRE(ntensors >= 1 && nchunks >= 1, "demo: empty descriptor table (ntensors=%d nchunks=%d)", ntensors,
               nchunks);
    return GA_OK;
}

template <typename T, bool REF = false>
static void launch_encode(const ga_demo_tensor* tensors, int32_t ntensors, int32_t nchunks, const float* F,
                          void* param, const void* grad, void* delta, int64_t K, int64_t ld, float lr, float decay,
                          float wd_factor, int32_t* payload, int64_t pstride, int64_t M, int ptr_vec,
                          hipStream_t stream) {
    auto kern = demo_encode_kernel<T, REF>;
    static const int resident = resident_blocks(kern);
    hipLaunchKernelGGL(kern, persistent_grid(resident, nchunks, K), dim3(kDmBlock), 0, stream, tensors, ntensors,
                       nchunks, F, (T*)param, (const T*)grad, (T*)delta, ld, lr, decay, wd_factor, payload, pstride,
                       M, ptr_vec);
}

template <typename T, typename CntT, bool REF = false>
static void launch_decode(const ga_demo_tensor* tensors, int32_t ntensors, int32_t nchunks, const float* B,
                          const int32_t* payload, int64_t pstride, int64_t M, int64_t S, void* param, void* grad,
                          int64_t K, int64_t ld, float lr, int ptr_vec, hipStream_t stream) {
    auto kern = demo_decode_kernel<T, CntT, REF>;
    static const int resident = resident_blocks(kern);
    hipLaunchKernelGGL(kern, persistent_grid(resident, nchunks, 1), dim3(kDmBlock), 0, stream, tensors, ntensors,
                       nchunks, B, payload, pstride, M, (int)S, (T*)param, (T*)grad, K, ld, lr, ptr_vec);
}

}  // namespace ga

using namespace ga;

extern "C" GA_API int ga_demo_tensor_bytes(void) { return (int)sizeof(ga_demo_tensor); }

#ifdef GA_DEMO_STAMPS
extern "C" GA_API int ga_demo_stamps_set(unsigned long long* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(ga::g_demo_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : 2;
}
#endif

extern "C" GA_API int ga_demo_encode(int dtype, const ga_demo_tensor* tensors, int32_t ntensors, int32_t nchunks,
                                     const float* F, const float* B, void* param, const void* grad, void* delta,
                                     int64_t K, int64_t ld, float lr, float decay, float wd_factor,
                                     int32_t* payload, int64_t payload_stride, int64_t M, hipStream_t stream) {
    clear_error();
    if (int e = check_tensors_host(ntensors, nchunks)) return e;
    GA_REQUIRE(tensors && F && B && param && grad && delta && payload, "ga_demo_encode: null buffer");
    GA_REQUIRE(K >= 1 && K <= 65535, "ga_demo_encode: K=%lld out of range", (long long)K);
    GA_REQUIRE(K == 1 || (ld > 0 && payload_stride >= 2 * M), "ga_demo_encode: bad replica strides");
    const int vb = dtype == GA_F32 ? 16 : 8;
    const int ptr_vec = ((uintptr_t)param % vb == 0) && ((uintptr_t)grad % vb == 0) &&
                        ((uintptr_t)delta % vb == 0) && (K == 1 || ld % 4 == 0);
    switch (dtype) {
        case GA_F32:
            launch_encode<float>(tensors, ntensors, nchunks, F, param, grad, delta, K, ld, lr, decay, wd_factor,
                                 payload, payload_stride, M, ptr_vec, stream);
            break;
        case GA_BF16:
            launch_encode<__hip_bfloat16>(tensors, ntensors, nchunks, F, param, grad, delta, K, ld, lr, decay,
                                          wd_factor, payload, payload_stride, M, ptr_vec, stream);
            break;
        case GA_BF16_REF:
            launch_encode<__hip_bfloat16, true>(tensors, ntensors, nchunks, F, param, grad, delta, K, ld, lr, decay,
                                                wd_factor, payload, payload_stride, M, ptr_vec, stream);
            break;
        default: set_error("ga_demo_encode: unknown dtype %d", dtype); return GA_EINVAL;
    }
    return check_launch("ga_demo_encode");
}

extern "C" GA_API int ga_demo_decode(int dtype, const ga_demo_tensor* tensors, int32_t ntensors, int32_t nchunks,
                                     const float* B, const int32_t* payload, int64_t payload_stride, int64_t M,
                                     int64_t S, void* param, void* grad, int64_t K, int64_t ld, float lr,
                                     hipStream_t stream) {
    clear_error();
    if (int e = check_tensors_host(ntensors, nchunks)) return e;
    GA_REQUIRE(tensors && B && payload && param, "ga_demo_decode: null buffer");
    GA_REQUIRE(S >= 1 && K >= 1, "ga_demo_decode: bad S=%lld K=%lld", (long long)S, (long long)K);
    GA_REQUIRE(S == 1 || payload_stride >= 2 * M, "ga_demo_decode: payload_stride < 2*M");
    GA_REQUIRE(S <= 65535, "ga_demo_decode: more than 65535 sources");
    GA_REQUIRE(K == 1 || ld > 0, "ga_demo_decode: bad ld");
    const int vb = dtype == GA_F32 ? 16 : 8;
    const int ptr_vec = ((uintptr_t)param % vb == 0) && (grad == nullptr || (uintptr_t)grad % vb == 0) &&
                        (K == 1 || ld % 4 == 0);
    switch (dtype) {
        case GA_F32:
            if (S <= 255)
                launch_decode<float, uint8_t>(tensors, ntensors, nchunks, B, payload, payload_stride, M, S, param,
                                              grad, K, ld, lr, ptr_vec, stream);
            else
                launch_decode<float, uint16_t>(tensors, ntensors, nchunks, B, payload, payload_stride, M, S, param,
                                               grad, K, ld, lr, ptr_vec, stream);
            break;
        case GA_BF16:
            if (S <= 255)
                launch_decode<__hip_bfloat16, uint8_t>(tensors, ntensors, nchunks, B, payload, payload_stride, M, S,
                                                       param, grad, K, ld, lr, ptr_vec, stream);
            else
                launch_decode<__hip_bfloat16, uint16_t>(tensors, ntensors, nchunks, B, payload, payload_stride, M,
                                                        S, param, grad, K, ld, lr, ptr_vec, stream);
            break;
        case GA_BF16_REF:
            if (S <= 255)
                launch_decode<__hip_bfloat16, uint8_t, true>(tensors, ntensors, nchunks, B, payload, payload_stride,
                                                             M, S, param, grad, K, ld, lr, ptr_vec, stream);
            else
                launch_decode<__hip_bfloat16, uint16_t, true>(tensors, ntensors, nchunks, B, payload, payload_stride,
                                                              M, S, param, grad, K, ld, lr, ptr_vec, stream);
            break;
        default: set_error("ga_demo_decode: unknown dtype %d", dtype); return GA_EINVAL;
    }
    return check_launch("ga_demo_decode");
}
