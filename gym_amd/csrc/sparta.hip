// SPARTA sparse parameter averaging over a flat arena (one launch covers every
// tensor): select -> gather(sum over local replicas) -> [RCCL all-reduce of
// the packed values, host side] -> scatter(/divisor) into every replica.
//
// Selection is a stream compaction in ascending element order, so the packed
// order equals `param.data[mask]` over the concatenated parameters
// (sparta.py:38).  The mask is either a uint8 arena (rank 0's mask, exactly
// the reference semantics), the same mask packed to one bit per element
// (ga_sparta_pack_mask: what crosses the wire at N > 1, n/8 bytes instead of
// n) or generated in-kernel from Philox4x32-10 keyed by
// (seed, iteration) -- then every rank derives the same mask and nothing is
// broadcast.  Three passes: per-tile count, one-block scan of tile counts,
// select+gather (the predicate is recomputed).
//
// The Philox stream draws i.i.d. Bernoulli(p) selections as geometric gaps:
// each 64-element group g takes the 32-bit words of
// philox(key = seed, ctr = {g, r, iteration}) (r = 0, 1, ... as needed) in
// order; a word u gives the gap t = #{j : T[j] <= u} to the next selected
// element, where T[j] = round(2^32 (1 - (1 - p)^(j + 1))) (so P(gap = t) =
// (1 - p)^t p up to the 2^-32 rounding), and u >= T[63] ends the group.  At
// p = 0.005 a group costs one Philox call (~1.3 words) instead of sixteen
// (one 24-bit draw per element): the mask no longer bounds the kernel.
#include <math.h>


#include "ga_common.h"

namespace ga {

constexpr int kSpBlock = 256;
constexpr int kSpPerThread = 64;                       // elements per lane: one Philox group
constexpr int kSpTile = kSpBlock * kSpPerThread;       // 16384 elements per workgroup
constexpr int kSelCap = 4096;                  // selected positions listed per window
constexpr int kScanBlock = 1024;
constexpr int kGapTable = 64;

// a * b as one v_mad_u64_u32 (low and high words from one instruction); the
// compiler's v_mul_lo_u32 + v_mul_hi_u32 pair runs Philox 20% slower
// (tools/ubench_philox_mul.hip, profiles/r04n_philox_mul.txt: 0.218 -> 0.175 ms,
// identical outputs); in the library the reference draw alone 0.068 -> 0.051 ms and
// the reference-draw elem step 0.088 -> 0.071 ms (same-box A/B, r04n_ab_philox_mad.txt)
__device__ __forceinline__ uint64_t mul_wide(uint32_t a, uint32_t b) {
    uint64_t r;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "s"(a), "v"(b) : "vcc");
    return r;
}

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = mul_wide(M0, c.x), p1 = mul_wide(M1, c.z);
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        // 3-input XORs as one gfx950 v_bitop3_b32 each (LUT 0x96 = a ^ b ^ c)
        c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k.x, 0x96), lo1,
                       __builtin_amdgcn_bitop3_b32(hi0, c.w, k.y, 0x96), lo0);
        k.x += W0;
        k.y += W1;
    }
    return c;
}

// torch's stream calls Philox with counter {ctr, t}: the 16 calls t = t0 .. t0 + 15 of
// one 64-element word (t0 % 16 == 0) share ctr and t >> 32, so round 1's ctr product
// and round 2's second product are the same for all of them: computed once per word
// (TorchCtr), each call then issues 18 products instead of 20 (bit-identical words)
struct TorchCtr {
    uint32_t A, B, C, D;  // ctr_hi ^ k0.x; hi(P) ^ k1.x; lo(P); lo(M0 ctr_lo) ^ k1.y (P: round 2's second product)
};

__device__ __forceinline__ TorchCtr torch_ctr(uint2 k, uint64_t ctr, uint32_t t_hi) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    const uint64_t p0 = mul_wide(M0, (uint32_t)ctr);                           // round 1: M0 * c.x
    const uint32_t z1 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), t_hi, k.y, 0x96);  // round 1's c.z
    const uint64_t p1 = mul_wide(M1, z1);                                      // round 2: M1 * c.z
    TorchCtr T;
    T.A = (uint32_t)(ctr >> 32) ^ k.x;
    T.B = (uint32_t)(p1 >> 32) ^ (k.x + W0);
    T.C = (uint32_t)p1;
    T.D = (uint32_t)p0 ^ (k.y + W1);
    return T;
}

// philox4x32_10({ctr, t}, k) for t_lo = (uint32_t)t, given torch_ctr(k, ctr, t >> 32)
__device__ __forceinline__ uint4 torch_philox(const TorchCtr& T, uint32_t t_lo, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    const uint64_t a = mul_wide(M1, t_lo);                                     // round 1: M1 * c.z
    const uint64_t b = mul_wide(M0, (uint32_t)(a >> 32) ^ T.A);                 // round 2: M0 * c.x
    uint4 c = make_uint4((uint32_t)a ^ T.B, T.C, (uint32_t)(b >> 32) ^ T.D, (uint32_t)b);
    k.x += 2u * W0;
    k.y += 2u * W1;
#pragma unroll
    for (int r = 2; r < 10; ++r) {
        const uint64_t p0 = mul_wide(M0, c.x), p1 = mul_wide(M1, c.z);
        c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k.x, 0x96), (uint32_t)p1,
                       __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k.y, 0x96), (uint32_t)p0);
        k.x += W0;
        k.y += W1;
    }
    return c;
}

struct Pred {
    const uint8_t* mask;  // uint8 mask arena, or null
    const uint64_t* bits; // packed mask (bit j of word w = element 64 w + j), or null; both null -> Philox
    const int64_t* ttab;  // GA_MASK_TORCH: the reference draw in-kernel (ga_sparta_torch_draw), or null
    int32_t tn;
    uint32_t tthr;  // select a 32-bit Philox word w iff tany && w <= tthr (tb_threshold)
    int32_t tany;
    uint64_t toff0, tstep;
    const uint64_t* tseedoff;
    uint2 tkey;
    uint2 key;
    uint32_t it_lo, it_hi;
    const int64_t* skip;  // Philox: sorted disjoint [lo, hi) element ranges never selected
    int32_t nskip;
    uint64_t gap[kGapTable];  // T[j] (<= 2^32), nondecreasing
};

// Clear the bits of the 64 elements at e0 that fall in a skipped range
// (tensors without a gradient, sparta.py:29-30).  Binary search for the first
// range ending after e0; a 64-element group meets at most a few ranges.
__device__ __forceinline__ uint64_t clear_skipped(const Pred& P, int64_t e0, uint64_t bits) {
    int lo = 0, hi = P.nskip;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (P.skip[2 * mid + 1] <= e0) lo = mid + 1;
        else hi = mid;
    }
    for (int r = lo; r < P.nskip && bits; ++r) {
        const int64_t a = P.skip[2 * r], b = P.skip[2 * r + 1];
        if (a >= e0 + 64) break;
        const int s = a > e0 ? (int)(a - e0) : 0;
        const int t = b < e0 + 64 ? (int)(b - e0) : 64;
        const uint64_t hi_m = t >= 64 ? ~0ull : ((1ull << t) - 1ull);
        bits &= ~(hi_m & ~((1ull << s) - 1ull));
    }
    return bits;
}

// gap of word u (< T[63]): the number of table entries <= u, by binary search
__device__ __forceinline__ int gap_of(const uint64_t* tab, uint32_t u) {
    int t = 0;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
        if (tab[t + s - 1] <= (uint64_t)u) t += s;
    return t;
}

// The 64-element word of torch's bernoulli stream at 4-element group t0 (t0 %
// 16 == 0): 16 Philox calls with counter {ctr, t}, four independent chains at
// a time; element 4t + j is selected iff word j of call t is <= thr (the exact
// integer form of rocrand's uniform 2^-32 + w 2^-32 <= p, see tb_threshold),
// and only the first `rem` elements exist.
__device__ __forceinline__ uint64_t torch_word(uint2 key, uint64_t ctr, uint64_t t0, int64_t rem, uint32_t thr,
                                               int32_t any) {
    uint32_t half[2] = {0u, 0u};
    // chunks from the top down; each word shifts its NOT-selected bit (the
    // borrow of thr - w) in from the bottom: acc = 2 acc + borrow, two VALU per
    // element against three for compare + select + or (torch_draw 0.069 ->
    // 0.067 ms, profiles/r02z_ab_torch_asmpack.txt)
    const uint32_t vthr = thr;
    const TorchCtr T = torch_ctr(key, ctr, (uint32_t)(t0 >> 32));
#pragma unroll
    for (int c0 = 12; c0 >= 0; c0 -= 4) {
        uint4 w[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) w[c] = torch_philox(T, (uint32_t)t0 + (uint32_t)(c0 + c), key);
        uint32_t& acc = half[c0 >> 3];
#pragma unroll
        for (int c = 3; c >= 0; --c) {
            const uint32_t ws[4] = {w[c].x, w[c].y, w[c].z, w[c].w};
#pragma unroll
            for (int j = 3; j >= 0; --j) {
                uint32_t tmp;
                asm("v_sub_co_u32 %1, vcc, %2, %3\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
                    : "+v"(acc), "=&v"(tmp)
                    : "v"(vthr), "v"(ws[j])
                    : "vcc");
            }
        }
    }
    half[0] = ~half[0];
    half[1] = ~half[1];
    const uint64_t bits = ((uint64_t)half[1] << 32) | half[0];
    if (!any || rem <= 0) return 0ull;
    return rem >= 64 ? bits : bits & ((1ull << rem) - 1ull);
}

// GA_MASK_TORCH: the 64 elements at e0 as ga_sparta_torch_bernoulli draws them
// (tensor offsets are multiples of 64, so the group lies in one tensor or in
// padding / a tensor not drawn): 16 Philox calls, four chains at a time
__device__ __forceinline__ uint64_t torch_bits64(const Pred& P, int64_t e0) {
    // last drawn tensor starting at or before e0: a wave-uniform (scalar) search
    // for the wave's first active lane, then each lane walks forward (lanes hold
    // increasing e0 in every caller; a 64-group tile spans few tensors)
    const int64_t ef = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(e0 >> 32)) << 32) |
                                 (uint32_t)__builtin_amdgcn_readfirstlane((int)e0));
    int lo = 0, hi = P.tn - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (P.ttab[3 * mid] <= ef) lo = mid;
        else hi = mid - 1;
    }
    while (lo + 1 < P.tn && P.ttab[3 * (lo + 1)] <= e0) ++lo;
    const int64_t base = P.ttab[3 * lo], numel = P.ttab[3 * lo + 1];
    if (e0 < base || e0 >= base + numel) return 0ull;
    uint2 key = P.tkey;
    uint64_t off0 = P.toff0;
    if (P.tseedoff) {
        const uint64_t sd = P.tseedoff[0];
        key = make_uint2((uint32_t)sd, (uint32_t)(sd >> 32));
        off0 = P.tseedoff[1];
    }
    const uint64_t ctr = (off0 + (uint64_t)lo * P.tstep) >> 2;
    const int64_t rel = e0 - base;
    return torch_word(key, ctr, (uint64_t)rel >> 2, numel - rel, P.tthr, P.tany);
}

// Selection bits of the 64 elements starting at element `e0` (e0 % 64 == 0);
// tab: the gap table in LDS.
// SRC: 0 = whichever source P names; 1 = the in-kernel reference draw only;
// 2 = anything but it (per-source instantiations keep each kernel's registers
// to what its source needs)
template <int SRC = 0>
__device__ __forceinline__ uint64_t pred_bits64(const Pred& P, const uint64_t* tab, int64_t e0, int64_t n) {
    uint64_t bits = 0;
    if (SRC == 1 || (SRC == 0 && P.ttab)) {
        bits = torch_bits64(P, e0);
        return e0 + 64 <= n ? bits : bits & ((1ull << (n - e0)) - 1ull);
    }
    if (P.bits) {
        bits = P.bits[e0 >> 6];
        return e0 + 64 <= n ? bits : bits & ((1ull << (n - e0)) - 1ull);
    }
    if (P.mask) {
        if (e0 + 64 <= n) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint4 m = *reinterpret_cast<const uint4*>(P.mask + e0 + 16 * v);
                const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        bits |= (uint64_t)(((w[q] >> (8 * b)) & 0xffu) != 0u) << (16 * v + 4 * q + b);
            }
        } else {
            for (int j = 0; j < 64 && e0 + j < n; ++j) bits |= (uint64_t)(P.mask[e0 + j] != 0) << j;
        }
        return bits;
    }
    const uint64_t t63 = tab[kGapTable - 1];
    const uint32_t g = (uint32_t)(e0 >> 6);  // n < 2^31: g < 2^25
    int pos = 0;
    bool live = true;
    for (uint32_t r = 0; live; ++r) {
        const uint4 w4 = philox4x32_10(make_uint4(g, r, P.it_lo, P.it_hi), P.key);
        const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (live) {
                if ((uint64_t)w[j] >= t63) {
                    live = false;
                } else {
                    pos += gap_of(tab, w[j]);
                    if (pos < 64) bits |= 1ull << pos;
                    ++pos;
                    live = pos < 64;
                }
            }
        }
    }
    if (e0 + 64 > n) bits &= (n - e0) >= 64 ? ~0ull : ((1ull << (uint32_t)(n - e0)) - 1ull);
    if (P.nskip) bits = clear_skipped(P, e0, bits);
    return bits;
}

__device__ __forceinline__ void load_gap_table(const Pred& P, uint64_t* tab) {
    if (threadIdx.x < kGapTable) tab[threadIdx.x] = P.gap[threadIdx.x];
    __syncthreads();
}

// Exclusive scan of one int per lane over a 256-lane workgroup.
__device__ __forceinline__ int block_excl_scan_256(int v, int* wave_tot, int* total) {
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
        const int t = wave_tot[w];
        pre += (w < wid) ? t : 0;
        tot += t;
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + x - v;
}

__global__ __launch_bounds__(kSpBlock) void sparta_count_kernel(Pred P, int64_t n, int32_t* tile_counts) {
    __shared__ int wave_tot[4];
    __shared__ uint64_t tab[kGapTable];
    load_gap_table(P, tab);
    const int64_t e0 = (int64_t)blockIdx.x * kSpTile + (int64_t)threadIdx.x * kSpPerThread;
    const int c = e0 < n ? __popcll(pred_bits64(P, tab, e0, n)) : 0;
    int total;
    block_excl_scan_256(c, wave_tot, &total);
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

// One workgroup: exclusive scan of the tile counts -> tile offsets, total and
// the overflow flag.  The counts are staged through LDS in coalesced passes of
// kScanChunk tiles (all loads in flight at once), then each lane scans a
// contiguous run of its pass from LDS.
constexpr int kScanChunk = 16384;

__global__ __launch_bounds__(kScanBlock) void sparta_scan_kernel(const int32_t* tile_counts, int64_t ntiles,
                                                                 int32_t* tile_offsets, int64_t cap,
                                                                 int64_t* count) {
    __shared__ int32_t buf[kScanChunk];
    __shared__ int64_t wave_tot[kScanBlock / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int per = kScanChunk / kScanBlock;  // 16 tiles per lane per pass
    int64_t carry = 0;
    for (int64_t base = 0; base < ntiles; base += kScanChunk) {
        const int64_t m = (ntiles - base) < kScanChunk ? (ntiles - base) : kScanChunk;
        for (int i = threadIdx.x; i < kScanChunk; i += kScanBlock) buf[i] = i < m ? tile_counts[base + i] : 0;
        __syncthreads();
        int32_t v[per];
        int64_t s = 0;
#pragma unroll
        for (int i = 0; i < per; ++i) {
            v[i] = buf[threadIdx.x * per + i];
            s += v[i];
        }
        int64_t x = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) wave_tot[wid] = x;
        __syncthreads();
        int64_t pre = carry, tot = 0;
        for (int w = 0; w < kScanBlock / 64; ++w) {
            pre += (w < wid) ? wave_tot[w] : 0;
            tot += wave_tot[w];
        }
        int64_t run = pre + x - s;
#pragma unroll
        for (int i = 0; i < per; ++i) {
            buf[threadIdx.x * per + i] = (int32_t)run;
            run += v[i];
        }
        __syncthreads();
        for (int i = threadIdx.x; i < m; i += kScanBlock) tile_offsets[base + i] = buf[i];
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        count[0] = carry;
        count[1] = carry > cap ? 1 : 0;
    }
}

// Exact unsigned division of small numerators (f * d < 2^32) by a uniform d.
struct FastDiv {
    uint64_t m;  // ceil(2^32 / d)
    uint32_t d;
    __device__ __forceinline__ explicit FastDiv(uint32_t dd) : m(((1ull << 32) + dd - 1) / dd), d(dd) {}
    __device__ __forceinline__ uint32_t div(uint32_t f) const { return (uint32_t)(((uint64_t)f * m) >> 32); }
};

// Select + gather.  The workgroup recomputes its tile's predicate, scans it
// to output positions, lists its selected elements in LDS, then all 256 lanes
// load the (element, replica) pairs densely (one load per lane, no idle lanes
// on sparse tiles) into LDS, and one lane per element sums its K values in
// ascending replica order.
//
// Replica-set layouts (Rep): replica k of element i is at i*ei + k*ek.
//   [K, ld] rows (ek = ld, ei = 1): consecutive lanes read consecutive selected
//     elements of ONE replica (same 16 KB of a row -> few DRAM pages), but every
//     (element, replica) is a separate random 4-B word;
//   [n, ld] element-major (ei = ld >= K, ek = 1): consecutive lanes read the K
//     replicas of ONE element, i.e. one element's K=32 fp32 values are one
//     128-B line -- the gather/write-back moves whole lines.
constexpr int kGatherSlots = 2048;  // floats of LDS for the (element, replica) values
constexpr int kGatherSlotsV4 = 3072;  // the same for the 4-replica vector form
// (measured, K = 32: 2048 slots 0.058-0.060 ms, 3072 0.053-0.056 ms, 4096 0.055-0.056 ms)
// (measured, K = 32 element-major: 2048 slots 0.075 ms, 4096 slots 0.090 ms -- the
// 16 loads in flight per lane cost 95 VGPRs and occupancy; 3072: 0.097-0.107 ms)

struct Rep {
    int64_t ek, ei;  // strides of replica and element
    bool em;         // element-major
    __device__ __forceinline__ int64_t at(int64_t i, int64_t k) const { return i * ei + k * ek; }
};

// With divisor > 0 the kernel also finishes the step for a single process
// (ga_sparta_average_local): each selected element's average is written back
// to every replica right after its gather, while its lines are still in L2
// (full-line write-backs instead of partial writes from a later scatter pass).
// V4: element-major set whose rows are 4-replica aligned (K % 4 == 0, ld % 4 == 0,
// base aligned to 4 elements): each lane moves one 4-replica vector, so an element's
// K = 32 fp32 replicas are 8 lanes x 16 B and the gather issues a quarter of the
// loads and address computations.
template <typename T, bool V4>
__global__ __launch_bounds__(kSpBlock) void sparta_select_kernel(Pred P, int64_t n, const int32_t* tile_offsets,
                                                                 T* src, int64_t K, Rep R,
                                                                 int64_t cap, int32_t* __restrict__ idx,
                                                                 T* __restrict__ vals, float divisor) {
    __shared__ int wave_tot[4];
    __shared__ uint64_t tab[kGapTable];
    __shared__ uint16_t sel_list[kSelCap];  // tile-local positions (< 16384) of one window
    constexpr int kSlots = V4 ? kGatherSlotsV4 : kGatherSlots;
    __shared__ float gv[kSlots];
    __shared__ float gavg[kSpBlock];
    load_gap_table(P, tab);
    const int64_t tile0 = (int64_t)blockIdx.x * kSpTile;
    const int64_t e0 = tile0 + (int64_t)threadIdx.x * kSpPerThread;
    const uint64_t bits0 = e0 < n ? pred_bits64(P, tab, e0, n) : 0ull;
    int total;
    const int local0 = block_excl_scan_256(__popcll(bits0), wave_tot, &total);
    const int64_t out0 = tile_offsets ? tile_offsets[blockIdx.x] : 0;
    // entries per pass: as many as fit K values each in the LDS slots.  An
    // entry's K values sit at an odd LDS stride Kp (K, or K + 1 for even K), so
    // lanes of consecutive entries (the rows layout's stores, every layout's
    // per-entry sums) hit distinct banks instead of one bank at K = 32.
    const int Ki = (int)(K < kSlots ? K : kSlots);
    const int Kp = (Ki & 1) || Ki + 1 > kSlots ? Ki : Ki + 1;
    const int per_pass = K >= kSlots ? 1 : (kSlots / Kp < kSpBlock ? kSlots / Kp : kSpBlock);
    const FastDiv divK((uint32_t)Ki);
    // the tile's selected elements in windows of kSelCap list slots (one window
    // unless p is large)
    for (int w0 = 0; w0 < total; w0 += kSelCap) {
        {
            uint64_t bits = bits0;
            int local = local0;
            while (bits) {
                const int j = __builtin_ctzll(bits);
                bits &= bits - 1;
                const int32_t i = (int32_t)(threadIdx.x * kSpPerThread + j);
                if (local >= w0 && local < w0 + kSelCap) sel_list[local - w0] = (uint16_t)i;
                const int64_t pos = out0 + local;
                if (w0 == 0 && idx && pos < cap) idx[pos] = (int32_t)(tile0 + i);
                ++local;
            }
        }
        __syncthreads();
        const int wtot = (total - w0) < kSelCap ? (total - w0) : kSelCap;
        for (int c0 = 0; c0 < wtot; c0 += per_pass) {
            const int ce = (wtot - c0) < per_pass ? (wtot - c0) : per_pass;
            if constexpr (V4) {
                // lane f -> (element e, replica quad q); staged into LDS per element at
                // the odd stride Kp, summed in ascending replica order as below
                using V = typename Vec4<T>::type;
                const int Kq = Ki >> 2;
                const FastDiv divQ((uint32_t)Kq);
                constexpr int kLoads4 = kSlots / 4 / kSpBlock;
                const int nf = ce * Kq;
                float v[kLoads4][4];
#pragma unroll
                for (int u = 0; u < kLoads4; ++u) {
                    const int f = threadIdx.x + u * kSpBlock;
                    if (f < nf) {
                        const int e = (int)divQ.div(f), q = f - e * Kq;
                        Vec4<T>::unpack(*reinterpret_cast<const V*>(src + R.at(tile0 + sel_list[c0 + e], 4 * q)), v[u]);
                    }
                }
#pragma unroll
                for (int u = 0; u < kLoads4; ++u) {
                    const int f = threadIdx.x + u * kSpBlock;
                    if (f < nf) {
                        const int e = (int)divQ.div(f), q = f - e * Kq;
#pragma unroll
                        for (int r = 0; r < 4; ++r) gv[e * Kp + 4 * q + r] = v[u][r];
                    }
                }
                __syncthreads();
                if (threadIdx.x < ce) {
                    float acc = 0.f;
                    for (int k = 0; k < Ki; ++k) acc += gv[threadIdx.x * Kp + k];
                    const int64_t pos = out0 + w0 + c0 + threadIdx.x;
                    if (vals && pos < cap) Elem<T>::store(vals + pos, acc);
                    if (divisor > 0.f) gavg[threadIdx.x] = acc / divisor;
                }
                __syncthreads();
                if (divisor > 0.f) {
#pragma unroll
                    for (int u = 0; u < kLoads4; ++u) {
                        const int f = threadIdx.x + u * kSpBlock;
                        if (f < nf) {
                            const int e = (int)divQ.div(f), q = f - e * Kq;
                            const float a = gavg[e];
                            const float w[4] = {a, a, a, a};
                            *reinterpret_cast<V*>(src + R.at(tile0 + sel_list[c0 + e], 4 * q)) = Vec4<T>::pack(w);
                        }
                    }
                    __syncthreads();
                }
            } else {
            if (K <= kSlots) {
                // lane f -> (element e, replica k): replica-major for [K, ld] rows,
                // element-major for [n, ld] (one element's replicas on adjacent lanes)
                // every lane's loads of the pass issued back to back (one HBM latency
                // per pass instead of one per load), then staged into LDS
                const FastDiv divC((uint32_t)ce);
                constexpr int kLoads = kGatherSlots / kSpBlock;
                float v[kLoads];
#pragma unroll
                for (int u = 0; u < kLoads; ++u) {
                    const int f = threadIdx.x + u * kSpBlock;
                    if (f < ce * Ki) {
                        const int k = R.em ? f - (int)divK.div(f) * Ki : (int)divC.div(f);
                        const int e = R.em ? (int)divK.div(f) : f - k * ce;
                        v[u] = Elem<T>::load(src + R.at(tile0 + sel_list[c0 + e], k));
                    }
                }
#pragma unroll
                for (int u = 0; u < kLoads; ++u) {
                    const int f = threadIdx.x + u * kSpBlock;
                    if (f < ce * Ki) {
                        const int k = R.em ? f - (int)divK.div(f) * Ki : (int)divC.div(f);
                        const int e = R.em ? (int)divK.div(f) : f - k * ce;
                        gv[e * Kp + k] = v[u];
                    }
                }
                __syncthreads();
                if (threadIdx.x < ce) {
                    float acc = 0.f;
                    for (int k = 0; k < Ki; ++k) acc += gv[threadIdx.x * Kp + k];
                    const int64_t pos = out0 + w0 + c0 + threadIdx.x;
                    if (vals && pos < cap) Elem<T>::store(vals + pos, acc);
                    if (divisor > 0.f) gavg[threadIdx.x] = acc / divisor;
                }
                __syncthreads();
                if (divisor > 0.f) {
                    for (int f = threadIdx.x; f < ce * Ki; f += kSpBlock) {
                        const int k = R.em ? f - (int)divK.div(f) * Ki : (int)divC.div(f);
                        const int e = R.em ? (int)divK.div(f) : f - k * ce;
                        Elem<T>::store(src + R.at(tile0 + sel_list[c0 + e], k), gavg[e]);
                    }
                    __syncthreads();
                }
            } else {  // very many replicas: one element at a time, lanes over replicas
                const int64_t i = tile0 + sel_list[c0];
                float acc = 0.f;
                if (threadIdx.x == 0)
                    for (int64_t k = 0; k < K; ++k) acc += Elem<T>::load(src + R.at(i, k));
                const int64_t pos = out0 + w0 + c0;
                if (threadIdx.x == 0 && vals && pos < cap) Elem<T>::store(vals + pos, acc);
                if (threadIdx.x == 0 && divisor > 0.f) {
                    const float a = acc / divisor;
                    for (int64_t k = 0; k < K; ++k) Elem<T>::store(src + R.at(i, k), a);
                }
            }
            }
        }
        __syncthreads();
    }
}

// Single-process average without the packed list (ga_sparta_average_local with
// no idx/vals/count) on an element-major set with 4-aligned rows and K = 4*KQ
// replicas, KQ | 64: one WAVEFRONT per 4096-element tile, waves synchronised
// only with themselves (no workgroup barrier after the gap table), so a SIMD
// mixes waves drawing their mask with waves whose gathers are in flight.  The
// wave scans its lanes' selection counts with shuffles, lists the selected
// positions in its own LDS, then moves each element's K values as KQ lanes x
// one 4-replica vector (whole 128-B lines at K = 32 fp32), up to 8 passes of
// loads in flight per lane, sums each element in ascending replica order across
// its lanes in registers and divides (the tile-gather kernel's fp32 order:
// bit-identical), and writes the average back to every replica.
// Measured (K = 32, 124M, p = 0.005): 0.049-0.053 ms (0.047-0.052 with the
// register-only batch) against 0.054-0.063 ms for
// the 16384-element tile-gather kernel; a persistent form that draws tile t+1's
// mask while tile t's loads are in flight ran 0.062 / 0.065 / 0.074 ms at 2 / 4 /
// 8 tiles per wave (fewer waves in flight), and builds of the kernel with only
// its mask (0.015 ms) or only its gather (0.034 ms) add up to the whole.
constexpr int kWGroups = 1;  // 64-element groups per lane (2: no faster, profiles/r02x_ab_sparta_groups.txt)
constexpr int kWTile = 64 * kSpPerThread * kWGroups;  // elements per wavefront tile
constexpr int kWList = 256;                // listed positions per window
constexpr int kSpWaves = 4;  // wavefronts (independent tiles) per workgroup

// x / d as torch's true division; a power-of-two d (K = 4, 8, 16, 32, 64 nodes) is
// an exact scaling, so the reciprocal multiply gives the same bits in one VALU
// instead of the ~10 of the IEEE division sequence (uniform branch)
__device__ __forceinline__ float div_nodes(float x, float d) {
    if ((__float_as_uint(d) & 0x807fffffu) == 0u && d != 0.f) return x * (1.f / d);
    return x / d;
}

// orders this wave's LDS accesses (the wave is the only writer of its slices)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One batch (<= EB listed elements from list[b0]) in registers: each element's K
// values stay in its KQ lanes (4 per lane) and the ascending-replica sum walks
// the lanes with DPP row shifts (lane q adds its four values to lane q - 1's
// running sum: the oracle's sequential order exactly), then the last lane's
// average is broadcast back.  No LDS staging, no wave_sync; NP passes (8
// elements each at K = 32) in flight; the lines are loaded and stored
// non-temporally (0.045 -> 0.041 ms, profiles/r02z_ab_sparta_nt.txt).  An LDS-staged form (values written at an
// odd stride, summed by one lane per element) measured 5% slower
// (profiles/r02x_ab_sparta_batch.txt).
template <typename T, int KQ>
struct WaveBatchDpp {
    static constexpr int K = 4 * KQ, EPP = 64 / KQ, NP = 8, EB = NP * EPP;
    using V = typename Vec4<T>::type;
    __device__ __forceinline__ static float shr1(float a) {  // lane i <- lane i - 1 within each 16-lane row
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x111, 0xf, 0xf, true));
    }
    // select form: the ascending-replica sum of each listed element goes to
    // vals[pos0 + e] (pos < cap), nothing is written back
    __device__ __forceinline__ static void sums(const T* src, int64_t ld, int64_t tile0, const uint16_t* list,
                                                int b0, int ne, int lane, T* vals, int64_t pos0, int64_t cap) {
        const int q = lane % KQ, el = lane / KQ;
        V v[NP];
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int e = u * EPP + el;
            if (e < ne) v[u] = stream_load(reinterpret_cast<const V*>(src + (tile0 + list[b0 + e]) * ld + 4 * q));
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            if (u * EPP >= ne) break;  // wave-uniform
            const int e = u * EPP + el;
            float f[4] = {0.f, 0.f, 0.f, 0.f};
            if (e < ne) Vec4<T>::unpack(v[u], f);
            float a = 0.f;
#pragma unroll
            for (int s = 0; s < KQ; ++s) {
                float left = KQ > 1 ? shr1(a) : 0.f;
                if (q == 0) left = 0.f;
                const float c = (((left + f[0]) + f[1]) + f[2]) + f[3];
                a = q == s ? c : a;
            }
            const int64_t pos = pos0 + b0 + e;
            if (q == KQ - 1 && e < ne && pos < cap) Elem<T>::store(vals + pos, a);
        }
    }
    __device__ __forceinline__ static void run(T* src, int64_t ld, int64_t tile0, const uint16_t* list, int b0,
                                               int ne, int lane, float divisor) {
        const int q = lane % KQ, el = lane / KQ;
        V v[NP];
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int e = u * EPP + el;
            if (e < ne) v[u] = stream_load(reinterpret_cast<const V*>(src + (tile0 + list[b0 + e]) * ld + 4 * q));
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            if (u * EPP >= ne) break;  // wave-uniform
            const int e = u * EPP + el;
            float f[4] = {0.f, 0.f, 0.f, 0.f};
            if (e < ne) Vec4<T>::unpack(v[u], f);
            float a = 0.f;
#pragma unroll
            for (int s = 0; s < KQ; ++s) {
                float left = KQ > 1 ? shr1(a) : 0.f;
                if (q == 0) left = 0.f;
                const float c = (((left + f[0]) + f[1]) + f[2]) + f[3];
                a = q == s ? c : a;
            }
            const float avg = __shfl(a / divisor, (lane & ~(KQ - 1)) | (KQ - 1), 64);
            if (e < ne) {
                const float w[4] = {avg, avg, avg, avg};
                stream_store(reinterpret_cast<V*>(src + (tile0 + list[b0 + e]) * ld + 4 * q), Vec4<T>::pack(w));
            }
        }
    }
};

// WaveBatchDpp with each lane holding VPL 4-replica vectors (16 VPL contiguous
// bytes of the element's line): KQ / VPL lanes per element, 64 VPL / KQ elements
// per pass, the ascending-replica walk KQ / VPL steps of 4 VPL adds.  Same sum
// order as WaveBatchDpp (bit-identical); 1 / VPL of the walk steps per element,
// so ~20 listed elements take two passes of 4 steps instead of three of 8 at
// VPL = 2.
constexpr int kSpVpl = 2;  // 4 vectors per lane: 0.0667 -> 0.072 ms (profiles/r04ad_ab_sparta_vpl4.txt)
template <typename T, int KQ, int VPL = kSpVpl>
struct WaveBatchDpp2 {
    static constexpr int LQ = KQ / VPL, K = 4 * KQ, EPP = 64 / LQ, NP = 8 / VPL, EB = NP * EPP;
    using V = typename Vec4<T>::type;
    __device__ __forceinline__ static float shr1(float a) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x111, 0xf, 0xf, true));
    }
    __device__ __forceinline__ static void run(T* src, int64_t ld, int64_t tile0, const uint16_t* list, int b0,
                                               int ne, int lane, float divisor) {
        const int q = lane % LQ, el = lane / LQ;
        V v[NP][VPL];
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int e = u * EPP + el;
            if (e < ne) {
                const V* p = reinterpret_cast<const V*>(src + (tile0 + list[b0 + e]) * ld + 4 * VPL * q);
#pragma unroll
                for (int j = 0; j < VPL; ++j) v[u][j] = stream_load(p + j);
            }
        }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            if (u * EPP >= ne) break;  // wave-uniform
            const int e = u * EPP + el;
            float f[VPL][4];
#pragma unroll
            for (int j = 0; j < VPL; ++j) {
                f[j][0] = f[j][1] = f[j][2] = f[j][3] = 0.f;
                if (e < ne) Vec4<T>::unpack(v[u][j], f[j]);
            }
            float a = 0.f;
#pragma unroll
            for (int s = 0; s < LQ; ++s) {
                float c = LQ > 1 ? shr1(a) : 0.f;
                if (q == 0) c = 0.f;
#pragma unroll
                for (int j = 0; j < VPL; ++j) c = (((c + f[j][0]) + f[j][1]) + f[j][2]) + f[j][3];
                a = q == s ? c : a;
            }
            const float avg = __shfl(div_nodes(a, divisor), (lane & ~(LQ - 1)) | (LQ - 1), 64);
            if (e < ne) {
                const float w[4] = {avg, avg, avg, avg};
                V* p = reinterpret_cast<V*>(src + (tile0 + list[b0 + e]) * ld + 4 * VPL * q);
#pragma unroll
                for (int j = 0; j < VPL; ++j) stream_store(p + j, Vec4<T>::pack(w));
            }
        }
    }
};

// 8 waves per SIMD: the per-source instantiations fit 64 VGPRs without spills
// (67 / 63 unconstrained); Philox mode 0.048 -> 0.045 ms, reference draw
// unchanged (profiles/r02z_ab_sparta_split_wpe.txt)
#define GA_SP_WPE_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
template <typename T, int KQ, int SRC>
__global__ __launch_bounds__(64 * kSpWaves) GA_SP_WPE_ATTR void sparta_average_wave_kernel(Pred P, int64_t n, T* __restrict__ src,
                                                                               int64_t ld, float divisor) {
    using B = WaveBatchDpp<T, KQ>;
    __shared__ uint64_t tab[kGapTable];
    __shared__ uint16_t lists[kSpWaves][kWList];
    if (SRC != 1) load_gap_table(P, tab);  // the reference draw has no gap table
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint16_t* list = lists[wid];
    const int64_t t = (int64_t)blockIdx.x * kSpWaves + wid;
    const int64_t tile0 = t * kWTile;
    // lane owns the kWGroups consecutive 64-element groups from e0 (ascending over lanes)
    const int64_t e0 = tile0 + (int64_t)lane * kSpPerThread * kWGroups;
    uint64_t bits[kWGroups];
    int c = 0;
#pragma unroll
    for (int g = 0; g < kWGroups; ++g) {
        const int64_t eg = e0 + (int64_t)g * kSpPerThread;
        bits[g] = eg < n ? pred_bits64<SRC>(P, tab, eg, n) : 0ull;
        c += __popcll(bits[g]);
    }
    int x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    const int total = __shfl(x, 63, 64);
    const int local0 = x - c;
    for (int w0 = 0; w0 < total; w0 += kWList) {  // one window unless p is large
        {
            int l = local0;
#pragma unroll
            for (int g = 0; g < kWGroups; ++g) {
                uint64_t b = bits[g];
                while (b) {
                    const int j = __builtin_ctzll(b);
                    b &= b - 1;
                    if (l >= w0 && l < w0 + kWList)
                        list[l - w0] = (uint16_t)((lane * kWGroups + g) * kSpPerThread + j);
                    ++l;
                }
            }
        }
        wave_sync();
        const int wtot = (total - w0) < kWList ? (total - w0) : kWList;
        // the reference draw leaves the kernel VALU-bound: the two-vector batch's shorter
        // walk takes it 0.0717 -> 0.0664 ms; the Philox stream's memory-bound step runs
        // 0.042 -> 0.048 ms with it, so that keeps the one-vector batch
        // (profiles/r04ac_ab_sparta_dpp2.txt)
        if (KQ >= kSpVpl && SRC == 1) {
            using B2 = WaveBatchDpp2<T, (KQ >= kSpVpl ? KQ : kSpVpl)>;
            for (int b0 = 0; b0 < wtot; b0 += B2::EB)
                B2::run(src, ld, tile0, list, b0, (wtot - b0) < B2::EB ? (wtot - b0) : B2::EB, lane, divisor);
        } else {
            for (int b0 = 0; b0 < wtot; b0 += B::EB)
                B::run(src, ld, tile0, list, b0, (wtot - b0) < B::EB ? (wtot - b0) : B::EB, lane, divisor);
        }
        wave_sync();  // the list is rewritten by the next window
    }
}

// Single-process average on the [K, ld] ROWS set (the replica training loop's
// layout: each node's parameters contiguous), without the packed list.  Every
// selected (element, replica) is its own random word here, so the step is the
// latency of ~K x pN scattered reads and writes; the kernel's job is to keep as
// many of them in flight as the wave slots allow.  One wavefront per 4096-element
// tile (mask, shuffle scan and LDS list as the element-major wave kernel); then
// ONE LANE PER LISTED ELEMENT issues all its replicas' loads back to back
// (up to kRowsKB in flight per lane, 64-bit row offsets), sums them in ascending
// replica order in the lane (the oracle's sequential fp32 order: bit-identical
// to the tile-gather kernel), divides, and writes the average to every replica.
// At p = 0.005 a tile lists ~20 elements: 20 x K words per wave, with no workgroup
// barrier between the mask draw and the gathers.
constexpr int kRowsKB = 32;
constexpr int kRTile = 64 * kSpPerThread;  // one 64-element group per lane, whatever kWGroups is
template <typename T, int SRC>
__global__ __launch_bounds__(64 * kSpWaves) void sparta_average_rows_wave_kernel(Pred P, int64_t n, T* src,
                                                                                    int64_t ld, int K, float divisor) {
    __shared__ uint64_t tab[kGapTable];
    __shared__ uint16_t lists[kSpWaves][kWList];
    if (SRC != 1) load_gap_table(P, tab);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint16_t* list = lists[wid];
    const int64_t tile0 = ((int64_t)blockIdx.x * kSpWaves + wid) * kRTile;
    const int64_t e0 = tile0 + (int64_t)lane * kSpPerThread;
    const uint64_t bits = e0 < n ? pred_bits64<SRC>(P, tab, e0, n) : 0ull;
    const int c = __popcll(bits);
    int x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    const int total = __shfl(x, 63, 64);
    const int local0 = x - c;
    for (int w0 = 0; w0 < total; w0 += kWList) {  // one window unless p is large
        {
            int l = local0;
            uint64_t b = bits;
            while (b) {
                const int j = __builtin_ctzll(b);
                b &= b - 1;
                if (l >= w0 && l < w0 + kWList) list[l - w0] = (uint16_t)(lane * kSpPerThread + j);
                ++l;
            }
        }
        wave_sync();
        const int wtot = (total - w0) < kWList ? (total - w0) : kWList;
        for (int b0 = 0; b0 < wtot; b0 += 64) {
            const bool on = b0 + lane < wtot;
            T* p = src + tile0 + (on ? list[b0 + lane] : 0);
            float acc = 0.f;
            for (int k0 = 0; k0 < K; k0 += kRowsKB) {
                float v[kRowsKB];
#pragma unroll
                for (int u = 0; u < kRowsKB; ++u) v[u] = on && k0 + u < K ? Elem<T>::load(p + (int64_t)(k0 + u) * ld) : 0.f;
#pragma unroll
                for (int u = 0; u < kRowsKB; ++u)
                    if (k0 + u < K) acc += v[u];
            }
            const float avg = acc / divisor;
            if (on)
                for (int k = 0; k < K; ++k) Elem<T>::store(p + (int64_t)k * ld, avg);
        }
        wave_sync();  // the list is rewritten by the next window
    }
}

template <typename T>
static bool launch_average_rows_wave(hipStream_t stream, const Pred& P, int64_t n, void* src, int64_t ld, int64_t K,
                                     float divisor) {
    if (K < 1 || K > 4 * kRowsKB) return false;
    const dim3 grid((unsigned)ceil_div(ceil_div(n, kRTile), kSpWaves)), block(64 * kSpWaves);
    if (P.ttab)
        hipLaunchKernelGGL((sparta_average_rows_wave_kernel<T, 1>), grid, block, 0, stream, P, n, (T*)src, ld, (int)K,
                           divisor);
    else
        hipLaunchKernelGGL((sparta_average_rows_wave_kernel<T, 2>), grid, block, 0, stream, P, n, (T*)src, ld, (int)K,
                           divisor);
    return true;
}

// The exchange path's select on the [n, K] layout in the wave form: a
// workgroup of kSpWaves wave tiles is exactly one count/scan tile (kSpTile),
// so its packed-list base comes from tile_offsets and each wave adds the
// totals of the waves before it.  Every selected element's index goes to idx,
// its K-replica sum (ascending replica order, the DPP lane walk) to vals.
static_assert(kSpWaves * kWTile == kSpTile, "select wave kernel: a workgroup is one count/scan tile");
template <typename T, int KQ, int SRC>
__global__ __launch_bounds__(64 * kSpWaves) GA_SP_WPE_ATTR void sparta_select_wave_kernel(
    Pred P, int64_t n, const int32_t* __restrict__ tile_offsets, const T* __restrict__ src, int64_t ld, int64_t cap,
    int32_t* __restrict__ idx, T* __restrict__ vals) {
    using B = WaveBatchDpp<T, KQ>;
    __shared__ uint64_t tab[kGapTable];
    __shared__ uint16_t lists[kSpWaves][kWList];
    __shared__ int wave_tot[kSpWaves];
    if (SRC != 1) load_gap_table(P, tab);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint16_t* list = lists[wid];
    const int64_t tile0 = ((int64_t)blockIdx.x * kSpWaves + wid) * kWTile;
    const int64_t e0 = tile0 + (int64_t)lane * kSpPerThread;
    const uint64_t bits = e0 < n ? pred_bits64<SRC>(P, tab, e0, n) : 0ull;
    const int c = __popcll(bits);
    int x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    const int total = __shfl(x, 63, 64);
    const int local0 = x - c;
    if (lane == 0) wave_tot[wid] = total;
    __syncthreads();
    int64_t pos0 = tile_offsets[blockIdx.x];
    for (int w = 0; w < wid; ++w) pos0 += wave_tot[w];
    {
        int l = local0;
        uint64_t b = bits;
        while (b) {
            const int j = __builtin_ctzll(b);
            b &= b - 1;
            const int64_t pos = pos0 + l;
            if (idx && pos < cap) idx[pos] = (int32_t)(e0 + j);
            ++l;
        }
    }
    if (!vals) return;
    for (int w0 = 0; w0 < total; w0 += kWList) {  // one window unless p is large
        {
            int l = local0;
            uint64_t b = bits;
            while (b) {
                const int j = __builtin_ctzll(b);
                b &= b - 1;
                if (l >= w0 && l < w0 + kWList) list[l - w0] = (uint16_t)(lane * kSpPerThread + j);
                ++l;
            }
        }
        wave_sync();
        const int wtot = (total - w0) < kWList ? (total - w0) : kWList;
        for (int b0 = 0; b0 < wtot; b0 += B::EB)
            B::sums(src, ld, tile0, list, b0, (wtot - b0) < B::EB ? (wtot - b0) : B::EB, lane, vals, pos0 + w0, cap);
    }
}

template <typename T>
static bool launch_select_wave(hipStream_t stream, const Pred& P, int64_t n, const int32_t* tile_offsets,
                               const void* src, int64_t ld, int64_t K, int64_t cap, int32_t* idx, void* vals) {
    const dim3 grid((unsigned)ceil_div(n, (int64_t)kSpTile)), block(64 * kSpWaves);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, block, 0, stream, P, n, tile_offsets, (const T*)src, ld, cap, idx, (T*)vals);
    };
    switch (K) {
        case 4: P.ttab ? go(sparta_select_wave_kernel<T, 1, 1>) : go(sparta_select_wave_kernel<T, 1, 2>); return true;
        case 8: P.ttab ? go(sparta_select_wave_kernel<T, 2, 1>) : go(sparta_select_wave_kernel<T, 2, 2>); return true;
        case 16: P.ttab ? go(sparta_select_wave_kernel<T, 4, 1>) : go(sparta_select_wave_kernel<T, 4, 2>); return true;
        case 32: P.ttab ? go(sparta_select_wave_kernel<T, 8, 1>) : go(sparta_select_wave_kernel<T, 8, 2>); return true;
        case 64: P.ttab ? go(sparta_select_wave_kernel<T, 16, 1>) : go(sparta_select_wave_kernel<T, 16, 2>); return true;
        default: return false;
    }
}

template <typename T>
static bool launch_average_wave(hipStream_t stream, const Pred& P, int64_t n, void* src, int64_t ld, int64_t K,
                                float divisor) {
    const dim3 grid((unsigned)ceil_div(ceil_div(n, kWTile), kSpWaves)), block(64 * kSpWaves);
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, 0, stream, P, n, (T*)src, ld, divisor); };
    switch (K) {
        case 4: P.ttab ? go(sparta_average_wave_kernel<T, 1, 1>) : go(sparta_average_wave_kernel<T, 1, 2>); return true;
        case 8: P.ttab ? go(sparta_average_wave_kernel<T, 2, 1>) : go(sparta_average_wave_kernel<T, 2, 2>); return true;
        case 16: P.ttab ? go(sparta_average_wave_kernel<T, 4, 1>) : go(sparta_average_wave_kernel<T, 4, 2>); return true;
        case 32: P.ttab ? go(sparta_average_wave_kernel<T, 8, 1>) : go(sparta_average_wave_kernel<T, 8, 2>); return true;
        case 64: P.ttab ? go(sparta_average_wave_kernel<T, 16, 1>) : go(sparta_average_wave_kernel<T, 16, 2>); return true;
        default: return false;
    }
}

// Scatter: one lane per (element, replica) pair, so every lane stores.
// [K, ld] rows: replicas on the grid's y dimension (no per-lane division);
// element-major: consecutive lanes store the K replicas of one element (one
// line per element at K = 32 fp32), as 4-replica vectors (V4) when the rows
// are 4-aligned; pair indices in 32-bit arithmetic when cap * K < 2^31 (W32).
template <typename T, bool V4, bool W32>
__global__ __launch_bounds__(kSpBlock) void sparta_scatter_kernel(const T* __restrict__ vals,
                                                                  const int32_t* __restrict__ idx,
                                                                  const int64_t* __restrict__ count, int64_t cap,
                                                                  float divisor, T* dst, int64_t K, Rep R) {
    const int64_t m = count[0] < cap ? count[0] : cap;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (R.em) {
        const int64_t Kv = V4 ? K / 4 : K;  // lanes per element
        const int64_t tot = m * Kv;
        for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += stride) {
            int64_t j, q;
            if (W32) {
                j = (int64_t)((uint32_t)t / (uint32_t)Kv);
                q = t - j * Kv;
            } else {
                j = t / Kv;
                q = t - j * Kv;
            }
            const float a = Elem<T>::load(vals + j) / divisor;
            if (V4) {
                const float w[4] = {a, a, a, a};
                *reinterpret_cast<typename Vec4<T>::type*>(dst + R.at(idx[j], 4 * q)) = Vec4<T>::pack(w);
            } else {
                Elem<T>::store(dst + R.at(idx[j], q), a);
            }
        }
        return;
    }
    for (int64_t k = blockIdx.y; k < K; k += gridDim.y) {
        T* d = dst + k * R.ek;
        for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride)
            Elem<T>::store(d + idx[j], Elem<T>::load(vals + j) / divisor);
    }
}

template <typename T>
static void launch_scatter(dim3 grid, hipStream_t stream, const void* vals, const int32_t* idx,
                           const int64_t* count, int64_t cap, float divisor, void* dst, int64_t K, Rep R) {
    const bool v4 = R.em && K % 4 == 0 && R.ei % 4 == 0 && ((uintptr_t)dst % (4 * sizeof(T))) == 0;
    const bool w32 = cap * K < ((int64_t)1 << 31);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kSpBlock), 0, stream, (const T*)vals, idx, count, cap, divisor, (T*)dst,
                           K, R);
    };
    if (v4) {
        if (w32) go(sparta_scatter_kernel<T, true, true>);
        else go(sparta_scatter_kernel<T, true, false>);
    } else {
        if (w32) go(sparta_scatter_kernel<T, false, true>);
        else go(sparta_scatter_kernel<T, false, false>);
    }
}

// uint8 mask arena -> one bit per element (bit j of word w = mask[64 w + j] != 0;
// bits past n are 0): one lane per 64-element word, the mask read as 4 x 16 B
__global__ __launch_bounds__(kSpBlock) void sparta_pack_mask_kernel(const uint8_t* __restrict__ mask, int64_t n,
                                                                    uint64_t* __restrict__ bits) {
    const int64_t w = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
    const int64_t e0 = w * 64;
    if (e0 >= n) return;
    uint64_t b = 0;
    if (e0 + 64 <= n) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint4 m = *reinterpret_cast<const uint4*>(mask + e0 + 16 * v);
            const uint32_t q[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) b |= (uint64_t)(((q[i] >> (8 * j)) & 0xffu) != 0u) << (16 * v + 4 * i + j);
        }
    } else {
        for (int j = 0; e0 + j < n; ++j) b |= (uint64_t)(mask[e0 + j] != 0) << j;
    }
    bits[w] = b;
}

// The reference's mask draw on the GPU, all tensors in one launch: for every
// drawn tensor i, torch.bernoulli(torch.full(shape_i, p)) on a CUDA/HIP device
// runs ATen's bernoulli_tensor_cuda_kernel through CUDA_tensor_apply2<.., 4>
// (block 512, grid ceil(numel / 2048): one pass, no grid-stride reuse below
// 2^31 blocks): thread t initialises Philox4x32-10 with (seed, subsequence t,
// offset O_i) -- counter {O_i/4 lo, O_i/4 hi, t lo, t hi}, key seed (O_i % 4 ==
// 0) -- takes one uniform4 (u = 2^-32 + w * 2^-32 per 32-bit word w, float)
// and selects element 4t + j iff u_j <= p (float).  O_i = O_0 + i * step, the
// generator offset torch hands out per bernoulli_ call.  One lane per
// 4-element group; a workgroup stays inside one tensor (table rows: arena
// offset, numel, first workgroup), so the lookup is a uniform binary search.
constexpr int kTbCalls = 4;                 // Philox calls (4-element groups) per lane
constexpr int64_t kTbSpan = 4 * kSpBlock * kTbCalls;  // elements per workgroup

// Packed output: one wavefront per workgroup span, each lane the 16 calls of
// one 64-element word (no cross-lane assembly).
constexpr int kTbWordLanes = (int)(kTbSpan / 64);

template <bool BITS>
__global__ __launch_bounds__(BITS ? kTbWordLanes : kSpBlock) void sparta_torch_bernoulli_kernel(
    const int64_t* __restrict__ tab, int ntens, uint32_t thr, int32_t any, uint2 key, uint64_t off0, uint64_t step,
    const uint64_t* seedoff, void* __restrict__ mask) {
    if (seedoff) {  // the generator state as rank 0 broadcast it (device memory)
        const uint64_t sd = seedoff[0];
        key = make_uint2((uint32_t)sd, (uint32_t)(sd >> 32));
        off0 = seedoff[1];
    }
    const int b = (int)blockIdx.x;
    int lo = 0, hi = ntens - 1;
    while (lo < hi) {  // last row whose first workgroup <= b
        const int mid = (lo + hi + 1) >> 1;
        if (tab[3 * mid + 2] <= b) lo = mid;
        else hi = mid - 1;
    }
    const int64_t base = tab[3 * lo], numel = tab[3 * lo + 1];
    const uint64_t ctr = (off0 + (uint64_t)lo * step) >> 2;
    if constexpr (BITS) {
        const int64_t rel = (int64_t)(b - tab[3 * lo + 2]) * kTbSpan + 64 * (int64_t)threadIdx.x;
        if (rel < numel)
            reinterpret_cast<uint64_t*>(mask)[(base + rel) >> 6] =
                torch_word(key, ctr, (uint64_t)rel >> 2, numel - rel, thr, any);
        return;
    }
    const uint64_t t0 = (uint64_t)(b - tab[3 * lo + 2]) * kSpBlock * kTbCalls + threadIdx.x;
    uint4 w[kTbCalls];
#pragma unroll
    for (int c = 0; c < kTbCalls; ++c) {  // independent chains: the calls interleave
        const uint64_t t = t0 + (uint64_t)c * kSpBlock;
        w[c] = philox4x32_10(make_uint4((uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)t, (uint32_t)(t >> 32)), key);
    }
#pragma unroll
    for (int c = 0; c < kTbCalls; ++c) {
        const int64_t e0 = (int64_t)(t0 + (uint64_t)c * kSpBlock) * 4;
        const uint32_t ws[4] = {w[c].x, w[c].y, w[c].z, w[c].w};
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (any && ws[j] <= thr) ? 1u : 0u;
        if (e0 < numel) {
            uint8_t* m = reinterpret_cast<uint8_t*>(mask) + base + e0;
            if (e0 + 4 <= numel) {
                *reinterpret_cast<uchar4*>(m) = make_uchar4(v[0], v[1], v[2], v[3]);
            } else {
                for (int j = 0; e0 + j < numel; ++j) m[j] = (uint8_t)v[j];
            }
        }
    }
}

static int64_t sparta_tiles(int64_t n) { return ceil_div(n, kSpTile); }

static Rep make_rep(int64_t ld, int layout) {
    Rep R;
    R.em = layout == GA_LAYOUT_ELEM_MAJOR;
    R.ek = R.em ? 1 : ld;
    R.ei = R.em ? ld : 1;
    return R;
}

template <typename T>
static int launch_select(const void* src, int64_t K, Rep R, int64_t n, const Pred& P, int64_t cap,
                         int32_t* idx, void* vals, int64_t* count, void* work, float divisor, hipStream_t stream) {
    const int64_t ntiles = sparta_tiles(n);
    const bool v4 = R.em && K % 4 == 0 && K <= kGatherSlotsV4 && R.ei % 4 == 0 &&
                    ((uintptr_t)src % (4 * sizeof(T))) == 0;
    int32_t* tile_offsets = nullptr;
    if (idx || vals || count) {  // positions of the packed list: count + scan passes
        int32_t* tile_counts = (int32_t*)work;
        tile_offsets = tile_counts + ntiles;
        hipLaunchKernelGGL(sparta_count_kernel, dim3((unsigned)ntiles), dim3(kSpBlock), 0, stream, P, n,
                           tile_counts);
        if (int e = check_launch("ga_sparta_select(count)")) return e;
        hipLaunchKernelGGL(sparta_scan_kernel, dim3(1), dim3(kScanBlock), 0, stream, tile_counts, ntiles,
                           tile_offsets, cap, count);
        if (int e = check_launch("ga_sparta_select(scan)")) return e;
    }
    if (v4 && !tile_offsets && !vals && divisor > 0.f && launch_average_wave<T>(stream, P, n, (void*)src, R.ei, K,
                                                                                divisor))
        return check_launch("ga_sparta_average_local(wave)");
    if (!R.em && !tile_offsets && !vals && divisor > 0.f &&
        launch_average_rows_wave<T>(stream, P, n, (void*)src, R.ek, K, divisor))
        return check_launch("ga_sparta_average_local(rows wave)");
    if (v4 && tile_offsets && divisor == 0.f &&
        launch_select_wave<T>(stream, P, n, tile_offsets, src, R.ei, K, cap, idx, vals))
        return check_launch("ga_sparta_select(wave)");
    if (v4)
        hipLaunchKernelGGL((sparta_select_kernel<T, true>), dim3((unsigned)ntiles), dim3(kSpBlock), 0, stream, P, n,
                           tile_offsets, (T*)src, K, R, cap, idx, (T*)vals, divisor);
    else
        hipLaunchKernelGGL((sparta_select_kernel<T, false>), dim3((unsigned)ntiles), dim3(kSpBlock), 0, stream, P, n,
                           tile_offsets, (T*)src, K, R, cap, idx, (T*)vals, divisor);
    return check_launch("ga_sparta_select(gather)");
}

// Calibration (no reference counterpart): the Philox4x32-10 issue ceiling of the
// reference draw.  One lane per 64-element word runs the 16 calls of torch_word
// (four independent chains at a time, same counters), XOR-folds the words instead
// of comparing and packing them and stores nothing: the draw's arithmetic alone.
__global__ __launch_bounds__(kTbWordLanes) void probe_philox_kernel(int64_t nwords, uint2 key, uint64_t ctr,
                                                                   uint32_t* sink) {
    const int64_t wd = (int64_t)blockIdx.x * kTbWordLanes + threadIdx.x;
    if (wd >= nwords) return;
    uint32_t acc = 0u;
    const uint64_t t0 = (uint64_t)wd * 16;
    const TorchCtr T = torch_ctr(key, ctr, (uint32_t)(t0 >> 32));
#pragma unroll
    for (int c0 = 0; c0 < 16; c0 += 4) {
        uint4 w[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) w[c] = torch_philox(T, (uint32_t)t0 + (uint32_t)(c0 + c), key);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            acc = __builtin_amdgcn_bitop3_b32(acc, __builtin_amdgcn_bitop3_b32(w[c].x, w[c].y, w[c].z, 0x96), w[c].w,
                                              0x96);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the calls
}

}  // namespace ga

using namespace ga;

extern "C" GA_API int64_t ga_sparta_workspace_bytes(int64_t n) {
    // tile counts + tile offsets, one int32 each per count tile
    return 2 * sparta_tiles(n < 0 ? 0 : n) * (int64_t)sizeof(int32_t);
}

extern "C" GA_API void ga_sparta_gap_table(double p, uint64_t* table) {
    // T[j] = round(2^32 * P(gap <= j)), P(gap <= j) = 1 - (1 - p)^(j + 1) = -expm1((j + 1) log1p(-p))
    for (int j = 0; j < kGapTable; ++j) {
        double v;
        if (!(p > 0.0)) v = 0.0;
        else if (p >= 1.0) v = 4294967296.0;
        else v = floor(-expm1((double)(j + 1) * log1p(-p)) * 4294967296.0 + 0.5);
        if (v > 4294967296.0) v = 4294967296.0;
        table[j] = (uint64_t)v;
    }
}

// rocrand's uniform of a 32-bit word w is RN(2^-32 + w * 2^-32) (float; the
// product is exact, so fused or not it rounds once) and is nondecreasing in w,
// so {w : uniform(w) <= p} is [0, thr]: the largest such w, found by bisection
// with the same float arithmetic; false when no word qualifies (p < 2^-32 or
// NaN).  The kernels then compare integers.
static bool tb_threshold(float p, uint32_t* thr) {
    const float inv = ldexpf(1.f, -32);
    auto sel = [&](uint32_t w) {
        volatile float x = (float)w * inv;
        volatile float u = x + inv;
        return u <= p;
    };
    *thr = 0u;
    if (!sel(0u)) return false;
    uint32_t lo = 0u, hi = 0xFFFFFFFFu;
    if (sel(hi)) {
        *thr = hi;
        return true;
    }
    while (hi - lo > 1u) {  // sel(lo) && !sel(hi)
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (sel(mid)) lo = mid;
        else hi = mid;
    }
    *thr = lo;
    return true;
}

static Pred make_pred(const void* mask, int mask_format, uint64_t seed, uint64_t iteration, double p,
                      const int64_t* skip, int64_t nskip) {
    Pred P;
    P.mask = mask_format == GA_MASK_BYTES ? (const uint8_t*)mask : nullptr;
    P.bits = mask_format == GA_MASK_BITS ? (const uint64_t*)mask : nullptr;
    P.ttab = nullptr;
    P.tn = 0;
    P.tthr = 0u;
    P.tany = 0;
    P.toff0 = P.tstep = 0;
    P.tseedoff = nullptr;
    P.tkey = make_uint2(0u, 0u);
    if (mask_format == GA_MASK_TORCH && mask) {
        const ga_sparta_torch_draw* d = (const ga_sparta_torch_draw*)mask;
        P.ttab = d->table;
        P.tn = d->ntens;
        P.tany = tb_threshold(d->p, &P.tthr) ? 1 : 0;
        P.toff0 = d->offset0;
        P.tstep = d->offset_step;
        P.tseedoff = d->seedoff;
        P.tkey = make_uint2((uint32_t)d->seed, (uint32_t)(d->seed >> 32));
    }
    P.key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    P.it_lo = (uint32_t)iteration;
    P.it_hi = (uint32_t)(iteration >> 32);
    P.skip = skip;
    P.nskip = (int32_t)nskip;
    ga_sparta_gap_table(mask ? 0.0 : p, P.gap);
    return P;
}

extern "C" GA_API int ga_sparta_select(int dtype, const void* src, int64_t K, int64_t ld, int layout, int64_t n,
                                       const void* mask, int mask_format, uint64_t seed, uint64_t iteration,
                                       double p, const int64_t* skip, int64_t nskip,
                                       int64_t cap, int32_t* idx, void* vals,
                                       int64_t* count, void* work, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "ga_sparta_select: n=%lld out of int32 index range", (long long)n);
    GA_REQUIRE(K >= 1 && cap >= 0, "ga_sparta_select: bad K=%lld cap=%lld", (long long)K, (long long)cap);
    GA_REQUIRE(count && work, "ga_sparta_select: null count/work");
    GA_REQUIRE(layout == GA_LAYOUT_ROWS || layout == GA_LAYOUT_ELEM_MAJOR, "ga_sparta_select: bad layout %d", layout);
    GA_REQUIRE(layout == GA_LAYOUT_ELEM_MAJOR ? ld >= K : (K == 1 || ld >= n), "ga_sparta_select: ld too small");
    GA_REQUIRE(p >= 0.0 && p <= 1.0, "ga_sparta_select: p=%g outside [0, 1]", p);
    GA_REQUIRE(mask_format == GA_MASK_BYTES || mask_format == GA_MASK_BITS || mask_format == GA_MASK_TORCH,
               "ga_sparta_select: bad mask_format %d", mask_format);
    GA_REQUIRE(mask == nullptr || mask_format == GA_MASK_TORCH || ((uintptr_t)mask % 16) == 0,
               "ga_sparta_select: mask must be 16-byte aligned");
    GA_REQUIRE(mask_format != GA_MASK_TORCH || (mask && ((const ga_sparta_torch_draw*)mask)->table &&
                                                ((const ga_sparta_torch_draw*)mask)->ntens > 0 &&
                                                ((const ga_sparta_torch_draw*)mask)->offset0 % 4 == 0),
               "ga_sparta_select: bad ga_sparta_torch_draw");
    GA_REQUIRE(nskip >= 0 && nskip < (1 << 24) && (nskip == 0 || skip), "ga_sparta_select: bad skip table");
    if (n == 0) return hipMemsetAsync(count, 0, 2 * sizeof(int64_t), stream) == hipSuccess ? GA_OK : GA_EHIP;
    GA_REQUIRE(src && idx && vals, "ga_sparta_select: null src/idx/vals");
    const Pred P = make_pred(mask, mask_format, seed, iteration, p, skip, nskip);
    switch (dtype) {
        case GA_F32:
            return launch_select<float>(src, K, make_rep(ld, layout), n, P, cap, idx, vals, count, work, 0.f, stream);
        case GA_BF16:
            return launch_select<__hip_bfloat16>(src, K, make_rep(ld, layout), n, P, cap, idx, vals, count, work, 0.f,
                                                 stream);
        default: set_error("ga_sparta_select: unknown dtype %d", dtype); return GA_EINVAL;
    }
}

extern "C" GA_API int ga_sparta_average_local(int dtype, void* reps, int64_t K, int64_t ld, int layout, int64_t n,
                                              const void* mask, int mask_format, uint64_t seed,
                                              uint64_t iteration, double p, const int64_t* skip, int64_t nskip,
                                              float divisor, int32_t* idx, void* vals,
                                              int64_t cap, int64_t* count, void* work, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && n < (int64_t)INT32_MAX, "ga_sparta_average_local: n=%lld out of range", (long long)n);
    GA_REQUIRE(K >= 1 && cap >= 0, "ga_sparta_average_local: bad K/cap");
    GA_REQUIRE(divisor > 0.0f, "ga_sparta_average_local: divisor must be > 0");
    GA_REQUIRE(layout == GA_LAYOUT_ROWS || layout == GA_LAYOUT_ELEM_MAJOR, "ga_sparta_average_local: bad layout");
    GA_REQUIRE(layout == GA_LAYOUT_ELEM_MAJOR ? ld >= K : (K == 1 || ld >= n), "ga_sparta_average_local: ld too small");
    GA_REQUIRE(p >= 0.0 && p <= 1.0, "ga_sparta_average_local: p=%g outside [0, 1]", p);
    GA_REQUIRE(mask_format == GA_MASK_BYTES || mask_format == GA_MASK_BITS || mask_format == GA_MASK_TORCH,
               "ga_sparta_average_local: bad mask_format %d", mask_format);
    GA_REQUIRE(mask == nullptr || mask_format == GA_MASK_TORCH || ((uintptr_t)mask % 16) == 0,
               "ga_sparta_average_local: mask alignment");
    GA_REQUIRE(mask_format != GA_MASK_TORCH || (mask && ((const ga_sparta_torch_draw*)mask)->table &&
                                                ((const ga_sparta_torch_draw*)mask)->ntens > 0 &&
                                                ((const ga_sparta_torch_draw*)mask)->offset0 % 4 == 0),
               "ga_sparta_average_local: bad ga_sparta_torch_draw");
    GA_REQUIRE(nskip >= 0 && nskip < (1 << 24) && (nskip == 0 || skip), "ga_sparta_average_local: bad skip table");
    GA_REQUIRE((idx == nullptr && vals == nullptr && count == nullptr) || (idx && vals && count && work),
               "ga_sparta_average_local: idx, vals, count and work go together");
    if (n == 0) return GA_OK;
    GA_REQUIRE(reps, "ga_sparta_average_local: null replicas");
    const Pred P = make_pred(mask, mask_format, seed, iteration, p, skip, nskip);
    switch (dtype) {
        case GA_F32:
            return launch_select<float>(reps, K, make_rep(ld, layout), n, P, cap, idx, vals, count, work, divisor,
                                        stream);
        case GA_BF16:
            return launch_select<__hip_bfloat16>(reps, K, make_rep(ld, layout), n, P, cap, idx, vals, count, work,
                                                 divisor, stream);
        default: set_error("ga_sparta_average_local: unknown dtype %d", dtype); return GA_EINVAL;
    }
}

extern "C" GA_API int ga_sparta_pack_mask(const uint8_t* mask, int64_t n, uint64_t* bits, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0, "ga_sparta_pack_mask: n=%lld", (long long)n);
    if (n == 0) return GA_OK;
    GA_REQUIRE(mask && bits, "ga_sparta_pack_mask: null mask/bits");
    GA_REQUIRE(((uintptr_t)mask % 16) == 0 && ((uintptr_t)bits % 8) == 0, "ga_sparta_pack_mask: alignment");
    const int64_t words = ceil_div(n, (int64_t)64);
    hipLaunchKernelGGL(sparta_pack_mask_kernel, dim3((unsigned)ceil_div(words, (int64_t)kSpBlock)), dim3(kSpBlock), 0,
                       stream, mask, n, bits);
    return check_launch("ga_sparta_pack_mask");
}

extern "C" GA_API int64_t ga_sparta_torch_bernoulli_span(void) { return kTbSpan; }

extern "C" GA_API int ga_probe_philox(int64_t n, uint32_t* sink, hipStream_t stream) {
    clear_error();
    GA_REQUIRE(n >= 0 && sink, "ga_probe_philox: bad n or null sink");
    const int64_t nwords = ceil_div(n, (int64_t)64);
    if (nwords == 0) return GA_OK;
    hipLaunchKernelGGL(probe_philox_kernel, dim3((unsigned)ceil_div(nwords, (int64_t)kTbWordLanes)),
                       dim3(kTbWordLanes), 0, stream, nwords, make_uint2(0x1234u, 0x5678u), (uint64_t)48, sink);
    return check_launch("ga_probe_philox");
}

extern "C" GA_API int ga_sparta_torch_draw_bytes(void) { return (int)sizeof(ga_sparta_torch_draw); }

extern "C" GA_API int ga_sparta_torch_bernoulli(const int64_t* table, int32_t ntens, int64_t nblocks, float p,
                                                uint64_t seed, uint64_t offset0, uint64_t offset_step,
                                                const uint64_t* seedoff, void* mask, int mask_format,
                                                hipStream_t stream) {
    clear_error();
    GA_REQUIRE(mask_format == GA_MASK_BYTES || mask_format == GA_MASK_BITS,
               "ga_sparta_torch_bernoulli: bad mask_format %d", mask_format);
    GA_REQUIRE(ntens >= 0 && nblocks >= 0 && nblocks < (int64_t)INT32_MAX, "ga_sparta_torch_bernoulli: bad sizes");
    GA_REQUIRE(p >= 0.f && p <= 1.f, "ga_sparta_torch_bernoulli: p=%g outside [0, 1]", (double)p);
    GA_REQUIRE(offset0 % 4 == 0 && offset_step % 4 == 0, "ga_sparta_torch_bernoulli: offsets must be multiples of 4");
    if (ntens == 0 || nblocks == 0) return GA_OK;
    GA_REQUIRE(table && mask && ((uintptr_t)mask % 8) == 0, "ga_sparta_torch_bernoulli: null table/mask or mask alignment");
    uint32_t thr;
    const int32_t any = tb_threshold(p, &thr) ? 1 : 0;
    auto go = [&](auto kern, int block) {
        hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(block), 0, stream, table, (int)ntens, thr, any,
                           make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)), offset0, offset_step, seedoff, mask);
    };
    if (mask_format == GA_MASK_BITS) go(sparta_torch_bernoulli_kernel<true>, kTbWordLanes);
    else go(sparta_torch_bernoulli_kernel<false>, kSpBlock);
    return check_launch("ga_sparta_torch_bernoulli");
}

extern "C" GA_API int ga_sparta_scatter(int dtype, const void* vals, const int32_t* idx, const int64_t* count,
                                        int64_t cap, float divisor, void* dst, int64_t K, int64_t ld, int layout,
                                        hipStream_t stream) {
    clear_error();
    GA_REQUIRE(K >= 1 && cap >= 0, "ga_sparta_scatter: bad K/cap");
    GA_REQUIRE(layout == GA_LAYOUT_ROWS || layout == GA_LAYOUT_ELEM_MAJOR, "ga_sparta_scatter: bad layout");
    GA_REQUIRE(layout == GA_LAYOUT_ROWS || ld >= K, "ga_sparta_scatter: element stride < K");
    if (cap == 0) return GA_OK;
    GA_REQUIRE(vals && idx && count && dst, "ga_sparta_scatter: null buffer");
    GA_REQUIRE(divisor != 0.0f, "ga_sparta_scatter: divisor is 0");
    const int gx = stream_grid(cap, kSpBlock);
    const Rep R = make_rep(ld, layout);
    const dim3 grid = R.em ? dim3((unsigned)stream_grid(cap * K, kSpBlock)) :
                             dim3(gx > 64 ? 64 : gx, (unsigned)(K < 65535 ? K : 65535));
    switch (dtype) {
        case GA_F32: launch_scatter<float>(grid, stream, vals, idx, count, cap, divisor, dst, K, R); break;
        case GA_BF16: launch_scatter<__hip_bfloat16>(grid, stream, vals, idx, count, cap, divisor, dst, K, R); break;
        default: set_error("ga_sparta_scatter: unknown dtype %d", dtype); return GA_EINVAL;
    }
    return check_launch("ga_sparta_scatter");
}
