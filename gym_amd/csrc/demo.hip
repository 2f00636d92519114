// DeMo DCT codec on gfx950: chunked DCT-II encode + per-chunk top-k + residual
// update (ga_demo_encode) and the gathered scatter-mean + inverse DCT + sign-SGD
// apply (ga_demo_decode).  One 256-lane workgroup (4 waves) per chunk.
//
// Transforms run on the matrix cores as 64x64x64 fp32 products
// (v_mfma_f32_32x32x2_f32: exact f32 FMA chains in k order; each wave owns one
// 32x32 quadrant).  Chunks with n1, n2 < 64 are computed zero padded: the basis
// tables are zero outside n x n, so padded rows/columns are exactly 0.
//
// LDS layout (per workgroup): ONE 64x65 working tile, products computed in
// place (accumulate in registers, barrier, store back), and ONE copy of the
// chunk's DCT basis F (spatial row i, frequency column k) with the same
// 65-float row stride: every operand orientation the transforms need (F, F^T,
// as A or B operand) then reads 32 consecutive lanes from 32 different banks.
// Encode ~40 KB (4 workgroups per CU), decode ~37 KB.
//
// Top-k (demo.py:315-328, torch.topk(|x|, k, sorted=False)): exact; among
// coefficients tied with the k-th magnitude the lowest index wins, and a
// chunk's entries are emitted in ascending index order (the reference's order
// is unspecified; only the set matters).
#include "ga_common.h"

namespace ga {

// Diagnostic build only (tools/demo_stamps.py, -DGA_DEMO_STAMPS): s_memtime at
// phase boundaries, one row of 16 per workgroup, into a buffer nothing else reads.
#ifdef GA_DEMO_STAMPS
__device__ unsigned long long* g_demo_stamps;
#define GA_STAMP(i)                                                                              \
    do {                                                                                         \
        if (threadIdx.x == 0)                                                                    \
            g_demo_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define GA_STAMP(i) \
    do {            \
    } while (0)
#endif

constexpr int kDmBlock = 256;
constexpr int kLd = 65;
constexpr int kTile = 64 * kLd;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Quadrant of C = A . B (64x64x64) for this wave, operands addressed by
// compile-time strides: A[i][k] = A[i*ASI + k*ASK], B[k][j] = B[k*BSK + j*BSJ].
template <int ASI, int ASK, int BSK, int BSJ>
__device__ __forceinline__ f32x16 mm64(const float* A, const float* Bm) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = 32 * (w >> 1) + (lane & 31);
    const int j = 32 * (w & 1) + (lane & 31);
    const int h = lane >> 5;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
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

// Row of accumulator register r for this lane (C/D layout of the 32x32 MFMA).
__device__ __forceinline__ int acc_row(int r) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    return 32 * (w >> 1) + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col() {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    return 32 * (w & 1) + (lane & 31);
}

__device__ __forceinline__ void store_acc(float* tile, const f32x16& acc) {
    const int c = acc_col();
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[acc_row(r) * kLd + c] = acc[r];
}

// Chunk -> tensor descriptor by a parallel scan of chunk_start (no serial
// dependent loads): returns the descriptor index, identical in every lane.
__device__ __forceinline__ int find_tensor(const ga_demo_tensor* T, int ntens, int chunk, int* slot) {
    for (int t = threadIdx.x; t < ntens; t += kDmBlock) {
        const int s0 = T[t].chunk_start;
        const int s1 = (t + 1 < ntens) ? T[t + 1].chunk_start : 0x7fffffff;
        if (s0 <= chunk && chunk < s1) *slot = t;
    }
    __syncthreads();
    return *slot;
}

// Exclusive scan of one int per lane over the 256-lane workgroup (optionally
// the total).
__device__ __forceinline__ int scan256(int v, int* wave_tot, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wave_tot[wid] = x;
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        pre += (w < wid) ? wave_tot[w] : 0;
        tot += wave_tot[w];
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + x - v;
}

// ---- chunk I/O: lane t owns rows (t>>4) + 16i (i < 4), columns 4(t&15) .. +3 ----
struct ChunkIO {
    int64_t base;  // element offset of the chunk's (0, 0)
    int cols, n1, n2;
    bool vec;      // 4-element vector accesses are legal for this tensor
    __device__ __forceinline__ int row(int i) const { return (threadIdx.x >> 4) + 16 * i; }
    __device__ __forceinline__ int col0() const { return 4 * (threadIdx.x & 15); }
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

template <typename T>
__device__ __forceinline__ ChunkIO chunk_io(const ga_demo_tensor& td, int c, int64_t ld, bool ptr_vec) {
    ChunkIO io;
    const int cy = c / td.gx, cx = c - cy * td.gx;
    io.base = td.offset + (int64_t)cy * td.n1 * td.cols + (int64_t)cx * td.n2;
    io.cols = td.cols;
    io.n1 = td.n1;
    io.n2 = td.n2;
    io.vec = ptr_vec && (td.offset % 4 == 0) && (td.cols % 4 == 0) && (td.n2 % 4 == 0) && (ld % 4 == 0);
    return io;
}

constexpr int kCandMax = 1024;   // candidate list of the threshold top-k
constexpr int kEntMax = 512;     // entries per chunk (topk <= 512; the list lives in the candidate buffer)
constexpr int kUBatch = 32;      // residual entries staged per pass

// Stage a chunk's basis into LDS as F[i*kLd + k] (spatial i, frequency k).
// From the DCT table F (row-major 64x64): a straight copy; from the inverse
// table B = F^T: the transpose.  Global reads are row-major (coalesced); the
// LDS writes of consecutive lanes land in different banks either way.
template <bool FROM_B>
__device__ __forceinline__ void stage_basis(float* FT, const float* tab) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int q = threadIdx.x + 256 * r;  // float4 index of the global table
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

// r[i][c] -= sum_e v_e * B1[b_e, row(i)] * B2[d_e, col0 + c] over an entry list
// (the sparse form of B1^T . S . B2, B = F^T).  Per batch of 32 entries,
// U[e][h] = v_e * F1[h, b_e] and W[e][w] = F2[w, d_e] are staged in `scratch`
// (2 x 32 x 64 floats); every lane then accumulates its 16 outputs from
// broadcast and 16-byte LDS reads.  F1 is the identity (n1 == 1), the LDS
// basis, or the global inverse table B1 (b1mode 0 / 1 / 2).
__device__ __forceinline__ void sparse_rank_update(float (&r)[4][4], const int* ent_bd, const float* ent_v, int E,
                                                   const float* FT, const float* B1g, int b1mode, const ChunkIO& io,
                                                   float* scratch) {
    float* U = scratch;
    float* W = scratch + kUBatch * 64;
    for (int e0 = 0; e0 < E; e0 += kUBatch) {
        const int ne = (E - e0) < kUBatch ? (E - e0) : kUBatch;
        __syncthreads();  // previous batch consumed
        for (int f = threadIdx.x; f < ne * 128; f += kDmBlock) {
            const int e = f >> 7, x = f & 127;
            const int bd = ent_bd[e0 + e];
            if (x < 64) {
                const int b = bd >> 8;
                float b1;
                if (b1mode == 0) b1 = (x == b) ? 1.f : 0.f;
                else if (b1mode == 1) b1 = FT[x * kLd + b];
                else b1 = B1g[b * 64 + x];
                U[e * 64 + x] = ent_v[e0 + e] * b1;
            } else {
                W[e * 64 + x - 64] = FT[(x - 64) * kLd + (bd & 255)];
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int e = 0; e < ne; ++e) {
            const float4 wv = *reinterpret_cast<const float4*>(W + e * 64 + io.col0());
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float u = U[e * 64 + io.row(i)];
                r[i][0] = fmaf(-u, wv.x, r[i][0]);
                r[i][1] = fmaf(-u, wv.y, r[i][1]);
                r[i][2] = fmaf(-u, wv.z, r[i][2]);
                r[i][3] = fmaf(-u, wv.w, r[i][3]);
            }
        }
    }
}

__device__ __forceinline__ int b1_mode(const ga_demo_tensor& td) {
    return td.n1 == 1 ? 0 : (td.basis1 == td.basis2 ? 1 : 2);
}

// Selection bits (T-map: lane t owns coefficients 16t .. 16t+15 of the padded
// row-major grid) of the k largest keys; ties at the k-th key -> lowest index.
// Fast path (k <= 256): T0 = the k-th largest of the 256 per-lane maxima is a
// lower bound on the k-th largest key (>= k lanes hold a key >= T0), found by
// every wave redundantly with a 31-step bitwise search over the maxima
// (ballot + popcount per step, no LDS traffic, no barrier).  The keys >= T0
// (about k of them on DCT coefficients) are appended to an LDS list and ranked
// exactly (key, then coefficient position).  Falls back to a 4-round 8-bit
// radix select if the candidates overflow (e.g. an all-zero chunk, where every
// key ties) or k > 256.
__device__ uint32_t select_topk(const uint32_t (&key)[16], int k, uint32_t* tmax, uint32_t* cand_key,
                                uint8_t* cand_sel, int* hist, int* misc) {
    const int t = threadIdx.x, lane = t & 63;
    constexpr int kCap = kCandMax / 2;                       // candidates: key[kCap], 16-bit position[kCap]
    uint16_t* cpos = reinterpret_cast<uint16_t*>(cand_sel);  // cand_sel is kCandMax bytes
    uint32_t* selw = tmax;                                   // selection words, reusing the maxima slots
    uint32_t mymax = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) mymax = key[j] > mymax ? key[j] : mymax;
    if (k <= kDmBlock) {
        if (t == 0) misc[3] = 0;  // candidate counter
        tmax[t] = mymax;
        __syncthreads();
        GA_STAMP(8);
        uint32_t v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tmax[r * 64 + lane];
        // bitwise search over the top 12 key bits (the exponent and 4 mantissa bits):
        // any threshold <= the exact k-th largest maximum keeps the >= k guarantee
        uint32_t T0 = 0;
#pragma unroll
        for (int bit = 30; bit >= 19; --bit) {
            const uint32_t cand = T0 | (1u << bit);
            int cnt = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) cnt += __popcll(__ballot(v[r] >= cand));
            if (cnt >= k) T0 = cand;
        }
        if (T0 == 0u) T0 = 1u;  // key 0 marks padding; small chunks rank all their keys
        GA_STAMP(9);
        __syncthreads();        // every wave has read the maxima: tmax becomes selw
        selw[t] = 0u;
        // append the candidates: per-wave ballot compaction, one LDS atomic per wave
        uint64_t m[16];
        int wcount = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            m[j] = __ballot(key[j] >= T0);
            wcount += __popcll(m[j]);
        }
        int wbase = 0;
        if (lane == 0 && wcount) wbase = atomicAdd(&misc[3], wcount);
        wbase = __shfl(wbase, 0, 64);
        const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if ((m[j] >> lane) & 1ull) {
                const int at = wbase + __popcll(m[j] & below);
                if (at < kCap) {
                    cand_key[at] = key[j];
                    cpos[at] = (uint16_t)(16 * t + j);
                }
            }
            wbase += __popcll(m[j]);
        }
        __syncthreads();
        const int C = misc[3];
        GA_STAMP(10);
#ifdef GA_DEMO_STAMPS
        if (threadIdx.x == 0) g_demo_stamps[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + 12] = C;
#endif
        if (C <= kCap) {
            for (int i = t; i < C; i += kDmBlock) {
                const uint32_t ki = cand_key[i];
                const int pi = cpos[i];
                int rank = 0;
                for (int j = 0; j < C; ++j) {
                    const uint32_t kj = cand_key[j];
                    rank += (kj > ki) | ((kj == ki) & (cpos[j] < pi));
                }
                if (rank < k) atomicOr(&selw[pi >> 4], 1u << (pi & 15));
            }
            __syncthreads();
            GA_STAMP(11);
            return selw[t];
        }
        __syncthreads();  // overflow: fall back to the radix select below
    }
    uint32_t sel = 0;
    // radix select of the k-th largest key
    uint32_t prefix = 0, pmask = 0;
    int kk = k;
    for (int shift = 24; shift >= 0; shift -= 8) {
        hist[t] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if ((key[j] & pmask) == prefix) atomicAdd(&hist[(key[j] >> shift) & 255u], 1);
        __syncthreads();
        if (t < 64) {
            int hb[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) hb[b] = hist[4 * t + b];
            const int lsum = hb[0] + hb[1] + hb[2] + hb[3];
            int x = lsum;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_down(x, d, 64);
                if (t + d < 64) x += y;
            }
            int cum = x - lsum;
#pragma unroll
            for (int b = 3; b >= 0; --b) {
                if (cum < kk && cum + hb[b] >= kk) {
                    misc[1] = 4 * t + b;
                    misc[2] = kk - cum;
                }
                cum += hb[b];
            }
        }
        __syncthreads();
        prefix |= (uint32_t)misc[1] << shift;
        pmask |= 0xffu << shift;
        kk = misc[2];
        __syncthreads();
    }
    int eq = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) eq += key[j] == prefix;
    int eq_run = scan256(eq, misc + 4, nullptr);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (key[j] > prefix) sel |= 1u << j;
        else if (key[j] == prefix) {
            if (eq_run < kk) sel |= 1u << j;
            ++eq_run;
        }
    }
    return sel;
}

template <typename T>
__global__ __launch_bounds__(kDmBlock) void demo_encode_kernel(
    const ga_demo_tensor* __restrict__ tens, int ntens, const float* __restrict__ F,
    const float* __restrict__ B, T* param, const T* __restrict__ grad, T* delta, int64_t ld, float lr,
    float decay, float wd_factor, int32_t* payload, int64_t pstride, int64_t M, int ptr_vec) {
    __shared__ __attribute__((aligned(16))) float X[kTile];  // delta -> T -> Y (in place); then residual staging
    __shared__ float FT[kTile];                               // basis F (row stride kLd)
    __shared__ uint32_t tmax[kDmBlock];
    __shared__ uint32_t cand_key[kCandMax];  // candidates; then the entry list
    __shared__ uint8_t cand_sel[kCandMax];
    __shared__ int hist[256];
    __shared__ int misc[8];

    const int chunk = blockIdx.x;
    const int tix = find_tensor(tens, ntens, chunk, &misc[0]);
    const ga_demo_tensor td = tens[tix];
    const int c = chunk - td.chunk_start;
    const int64_t rep = blockIdx.y;
    param += rep * ld;
    grad += rep * ld;
    delta += rep * ld;
    payload += rep * pstride;
    const ChunkIO io = chunk_io<T>(td, c, ld, ptr_vec != 0);
    const int n1 = td.n1, n2 = td.n2, k = td.k;
    GA_STAMP(0);
    stage_basis<false>(FT, F + (int64_t)td.basis2 * 4096);

    // 1. error feedback in registers: x = decay*delta + lr*grad (+ decoupled weight decay on p)
    float x[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (io.live(i)) {
            float d[4], g[4];
            load4(delta, io, i, d);
            load4(grad, io, i, g);
            if (wd_factor != 1.f) {
                float p[4];
                load4(param, io, i, p);
#pragma unroll
                for (int e = 0; e < 4; ++e) p[e] *= wd_factor;
                store4(param, io, i, p);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) x[i][e] = fmaf(lr, g[e], decay != 1.f ? d[e] * decay : d[e]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[i][e] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) X[io.row(i) * kLd + io.col0() + e] = (io.col0() + e < n2) ? x[i][e] : 0.f;
    }
    __syncthreads();
    GA_STAMP(1);

    // 2. Y = F1^T . X . F2 on the matrix cores, in place in X
    f32x16 acc = mm64<TILE_ROW, TILE_ROW>(X, FT);  // T = X . F2
    __syncthreads();
    store_acc(X, acc);
    __syncthreads();
    GA_STAMP(2);
    if (n1 > 1) {
        if (td.basis1 == td.basis2) acc = mm64<TILE_COL, TILE_ROW>(FT, X);  // F1^T . T
        else acc = mm64<GTAB_COL, TILE_ROW>(F + (int64_t)td.basis1 * 4096, X);
        __syncthreads();
        store_acc(X, acc);
        __syncthreads();
    }  // n1 == 1: F1 = [1], Y = T
    GA_STAMP(3);

    // 3. top-k of |Y| over the valid n1 x n2 coefficients
    const int row = threadIdx.x >> 2, col0 = 16 * (threadIdx.x & 3);
    uint32_t key[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const bool valid = row < n1 && (col0 + j) < n2;
        key[j] = valid ? (__float_as_uint(X[row * kLd + col0 + j]) & 0x7fffffffu) + 1u : 0u;
    }
    const uint32_t sel = select_topk(key, k, tmax, cand_key, cand_sel, hist, misc);
    GA_STAMP(4);

    // 4. emit the entries in ascending coefficient order; keep (b, d, v) in LDS
    int* ent_bd = reinterpret_cast<int*>(cand_key);
    float* ent_v = reinterpret_cast<float*>(cand_key + kEntMax);
    int slot = scan256(__popc(sel), misc + 4, nullptr);
    int32_t* out_idx = payload + td.payload_off + (int64_t)c * k;
    float* out_val = reinterpret_cast<float*>(payload + M) + td.payload_off + (int64_t)c * k;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (sel & (1u << j)) {
            const float y = X[row * kLd + col0 + j];
            out_idx[slot] = row * n2 + col0 + j;
            out_val[slot] = y;
            ent_bd[slot] = (row << 8) | (col0 + j);
            ent_v[slot] = y;
            ++slot;
        }
    }
    GA_STAMP(5);

    // 5. residual: delta = x - sum_e v_e * outer(B1[b_e, :], B2[d_e, :])  (the sparse
    //    form of B1^T . S . B2: k rank-1 terms instead of two dense products)
    sparse_rank_update(x, ent_bd, ent_v, k, FT, B + (int64_t)td.basis1 * 4096, b1_mode(td), io, X);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (io.live(i)) store4(delta, io, i, x[i]);
    GA_STAMP(6);
}

template <typename T, typename CntT>
__global__ __launch_bounds__(kDmBlock) void demo_decode_kernel(
    const ga_demo_tensor* __restrict__ tens, int ntens, const float* __restrict__ B,
    const int32_t* __restrict__ payload, int64_t pstride, int64_t M, int64_t nsrc, T* param, T* grad,
    int64_t K, int64_t ld, float lr, int ptr_vec) {
    __shared__ float S[kTile];   // scatter-mean tile -> U -> g (in place)
    __shared__ float FT[kTile];  // basis F (row stride kLd), staged from B = F^T
    __shared__ CntT cnt[4096];   // hits per coefficient
    __shared__ int misc[4];

    const int chunk = blockIdx.x;
    const int tix = find_tensor(tens, ntens, chunk, &misc[0]);
    const ga_demo_tensor td = tens[tix];
    const int c = chunk - td.chunk_start;
    const int n2 = td.n2, nk = td.k, nvalid = td.n1 * td.n2;
    const ChunkIO io = chunk_io<T>(td, c, ld, ptr_vec != 0);

    stage_basis<true>(FT, B + (int64_t)td.basis2 * 4096);
    for (int e = threadIdx.x; e < kTile; e += kDmBlock) S[e] = 0.f;
    for (int e = threadIdx.x; e < 4096; e += kDmBlock) cnt[e] = 0;
    __syncthreads();

    // scatter-mean (demo.py:331-352): sources in node order; one source's
    // indices are distinct, so each source is one conflict-free pass and the
    // per-coefficient sums accumulate in node order.
    const int64_t eoff = td.payload_off + (int64_t)c * nk;
    for (int64_t s = 0; s < nsrc; ++s) {
        const int32_t* pi = payload + s * pstride + eoff;
        const float* pv = reinterpret_cast<const float*>(payload + s * pstride + M) + eoff;
        for (int j = threadIdx.x; j < nk; j += kDmBlock) {
            const int x = pi[j];
            if (x >= 0 && x < nvalid) {
                const int b = x / n2, d = x - b * n2;
                S[b * kLd + d] += pv[j];
                cnt[b * 64 + d] += 1;
            }
        }
        __syncthreads();
    }
    if (nsrc > 1) {
        for (int e = threadIdx.x; e < 4096; e += kDmBlock) {
            const int n = cnt[e];
            if (n > 1) S[(e >> 6) * kLd + (e & 63)] /= (float)n;
        }
        __syncthreads();
    }

    // g = B1^T . S . B2 = F1 . S . F2^T on the matrix cores, in place in S
    f32x16 acc = mm64<TILE_ROW, TILE_COL>(S, FT);  // U = S . F2^T
    __syncthreads();
    store_acc(S, acc);
    __syncthreads();
    if (td.n1 > 1) {
        if (td.basis1 == td.basis2) acc = mm64<TILE_ROW, TILE_ROW>(FT, S);  // F1 . U
        else acc = mm64<GTAB_COL, TILE_ROW>(B + (int64_t)td.basis1 * 4096, S);  // F1[i][k] = B1[k][i]
        __syncthreads();
        store_acc(S, acc);
        __syncthreads();
    }

    // grad = sign(g) (torch.sign: NaN -> 0);  p -= lr * grad   (demo.py:200-209)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!io.live(i)) continue;
        float sg[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float g = S[io.row(i) * kLd + io.col0() + e];
            sg[e] = (float)((g > 0.f) - (g < 0.f));
        }
        for (int64_t k = 0; k < K; ++k) {
            float p[4];
            load4(param + k * ld, io, i, p);
#pragma unroll
            for (int e = 0; e < 4; ++e) p[e] = fmaf(-lr, sg[e], p[e]);
            store4(param + k * ld, io, i, p);
            if (grad) store4(grad + k * ld, io, i, sg);
        }
    }
}

static int check_tensors_host(int32_t ntensors, int32_t nchunks) {
    GA_REQUIRE(ntensors >= 1 && nchunks >= 1, "demo: empty descriptor table (ntensors=%d nchunks=%d)", ntensors,
               nchunks);
    return GA_OK;
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
    const int ptr_vec = ((uintptr_t)param % vb == 0) && ((uintptr_t)grad % vb == 0) && ((uintptr_t)delta % vb == 0);
    dim3 grid((unsigned)nchunks, (unsigned)K);
    switch (dtype) {
        case GA_F32:
            hipLaunchKernelGGL((demo_encode_kernel<float>), grid, dim3(kDmBlock), 0, stream, tensors, ntensors, F, B,
                               (float*)param, (const float*)grad, (float*)delta, ld, lr, decay, wd_factor, payload,
                               payload_stride, M, ptr_vec);
            break;
        case GA_BF16:
            hipLaunchKernelGGL((demo_encode_kernel<__hip_bfloat16>), grid, dim3(kDmBlock), 0, stream, tensors,
                               ntensors, F, B, (__hip_bfloat16*)param, (const __hip_bfloat16*)grad,
                               (__hip_bfloat16*)delta, ld, lr, decay, wd_factor, payload, payload_stride, M, ptr_vec);
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
    const int ptr_vec = ((uintptr_t)param % vb == 0) && (grad == nullptr || (uintptr_t)grad % vb == 0);
    switch (dtype) {
        case GA_F32:
            if (S <= 255)
                hipLaunchKernelGGL((demo_decode_kernel<float, uint8_t>), dim3((unsigned)nchunks), dim3(kDmBlock), 0,
                                   stream, tensors, ntensors, B, payload, payload_stride, M, S, (float*)param,
                                   (float*)grad, K, ld, lr, ptr_vec);
            else
                hipLaunchKernelGGL((demo_decode_kernel<float, uint16_t>), dim3((unsigned)nchunks), dim3(kDmBlock),
                                   0, stream, tensors, ntensors, B, payload, payload_stride, M, S, (float*)param,
                                   (float*)grad, K, ld, lr, ptr_vec);
            break;
        case GA_BF16:
            if (S <= 255)
                hipLaunchKernelGGL((demo_decode_kernel<__hip_bfloat16, uint8_t>), dim3((unsigned)nchunks),
                                   dim3(kDmBlock), 0, stream, tensors, ntensors, B, payload, payload_stride, M, S,
                                   (__hip_bfloat16*)param, (__hip_bfloat16*)grad, K, ld, lr, ptr_vec);
            else
                hipLaunchKernelGGL((demo_decode_kernel<__hip_bfloat16, uint16_t>), dim3((unsigned)nchunks),
                                   dim3(kDmBlock), 0, stream, tensors, ntensors, B, payload, payload_stride, M, S,
                                   (__hip_bfloat16*)param, (__hip_bfloat16*)grad, K, ld, lr, ptr_vec);
            break;
        default: set_error("ga_demo_decode: unknown dtype %d", dtype); return GA_EINVAL;
    }
    return check_launch("ga_demo_decode");
}
