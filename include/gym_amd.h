/*
 * gym_amd.h — C ABI of the MI355X (gfx950) strategy-communication-step kernels.
 *
 * This is the drop-in boundary under EXO Gym's Strategy API (reference:
 * satoutahhaithem/gym @ 2025-07-11).  Every entry point replaces the per-tensor
 * torch op loop of one reference function; the replaced interface is cited on
 * each declaration as `file:line` relative to the reference root.
 *
 * Conventions:
 *   - plain pointers + element counts; no torch types cross this boundary;
 *   - the caller (PyTorch) owns every buffer: the library never allocates or
 *     frees device memory and keeps no mutable global state other than a
 *     thread-local error string;
 *   - all work is enqueued asynchronously on the given hipStream_t (pass the
 *     torch current stream); nothing synchronises the host;
 *   - every function returns 0 on success or a GA_E* code; the message for the
 *     last failure on the calling thread is available from ga_last_error().
 *
 * A "replica set" is K simulated-node copies of one flat parameter arena laid
 * out as [K, ld] (replica k starts at element k*ld).  K = 1 is the ordinary
 * one-node-per-GPU case; K > 1 is batched-replica mode.
 */
#ifndef GYM_AMD_H
#define GYM_AMD_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GA_API __attribute__((visibility("default")))

/* error codes */
#define GA_OK 0
#define GA_EINVAL 1   /* bad argument (null pointer, bad size, unknown dtype) */
#define GA_EHIP 2     /* a HIP runtime call or kernel launch failed */
#define GA_EUNSUP 3   /* unsupported configuration */

/* element types of arena buffers */
#define GA_F32 0
#define GA_BF16 1
/* DeMo only (ga_demo_encode / ga_demo_decode): bf16 arenas with the reference's
 * bf16 arithmetic -- bf16 DCT bases (the caller's F / B tables hold
 * bf16-representable values), every stage of each transform rounded to bf16 in
 * the reference's contraction order (chunk rows first), the delta rounded after
 * the decay and after the gradient add (exogym/strategy/demo_impl/demo.py:
 * 159-180, 235-252 as torch runs it); the decode's scatter-mean adds the sources
 * in node order with the sum rounded to bf16 after every add, then divides
 * (demo.py:339-341: torch's bf16 scatter_reduce; on the GPU its atomic adds run
 * in an unspecified order, so at 3+ hitters of one position node order is one
 * of the orders the reference can produce). */
#define GA_BF16_REF 2

/* replica-set layouts (SPARTA entry points):
 *   GA_LAYOUT_ROWS        [K, ld]: replica k of element i at k*ld + i (every other kernel's layout)
 *   GA_LAYOUT_ELEM_MAJOR  [n, ld]: replica k of element i at i*ld + k (ld >= K): the K replicas of
 *                         one element are adjacent, so a sparse gather moves whole lines */
#define GA_LAYOUT_ROWS 0
#define GA_LAYOUT_ELEM_MAJOR 1

/* SPARTA mask formats:
 *   GA_MASK_BYTES  uint8 per element (selected iff != 0), 16-byte aligned
 *   GA_MASK_BITS   uint64 words, bit j of word w = element 64 w + j (ga_sparta_pack_mask) */
#define GA_MASK_BYTES 0
#define GA_MASK_BITS 1
#define GA_MASK_TORCH 2

/* GA_MASK_TORCH: the mask argument points to this HOST struct, and the select /
 * average kernels draw the reference's masks themselves, exactly as
 * ga_sparta_torch_bernoulli would write them (no mask in memory). */
typedef struct ga_sparta_torch_draw {
    const int64_t* table;     /* device rows {arena offset (multiple of 64), numel, -} per drawn tensor, ascending */
    int32_t ntens;            /* rows */
    float p;                  /* selection probability as torch.full(shape, p) holds it (fp32) */
    uint64_t seed, offset0;   /* torch generator state for the first drawn tensor */
    uint64_t offset_step;     /* generator offset per tensor (12) */
    const uint64_t* seedoff;  /* device {seed, offset0} overriding the two above, or null */
} ga_sparta_torch_draw;

/* ---- library ---------------------------------------------------------- */

/* ABI version (major*100 + minor). */
GA_API int ga_abi_version(void);

/* Message describing the last failure on the calling thread ("" if none). */
GA_API const char* ga_last_error(void);

/*
 * Calibration helper (no reference counterpart): dst <- src, nbytes (a multiple
 * of 16, 16-byte aligned buffers) as a float4 streaming copy.  bench.py times
 * it in the same process as the step kernels, so a roofline fraction can be
 * read against what the box actually streams.
 */
GA_API int ga_stream_copy(const void* src, void* dst, int64_t nbytes, hipStream_t stream);

/*
 * Calibration helper (no reference counterpart): the random-word floor of the
 * [K, ld] rows layout.  For each of the M positions pos[j] (int32, ascending)
 * and each replica k < K, the fp32 word at a[k * ld + pos[j]] is read and
 * (write != 0) written back as x * 0.5 + 1, one lane per (position, replica),
 * replica-major within 16384-element tiles as the SPARTA rows kernel walks
 * them -- the same 4-B words at random 64-B sectors, without the mask.  bench.py
 * times it on the positions a SPARTA step selected, in the same process.
 * write = 2 / 3: the whole aligned 64-B sector / 128-B line holding the word is
 * read and written back instead (ld a multiple of 32, a 128-B aligned): what a
 * full-sector write-back would cost against the word's partial write.
 */
GA_API int ga_probe_random_words(float* a, int64_t ld, int64_t K, const int32_t* pos, int64_t M, int write,
                                 hipStream_t stream);

/*
 * Calibration helper (no reference counterpart): the Philox4x32-10 issue
 * ceiling of the reference's SPARTA mask draw (sparta.py:80-85 through
 * ga_sparta_torch_bernoulli).  The n / 4 calls an n-element draw makes, in
 * ga_sparta_torch_bernoulli's packed-word launch shape (one lane per 64
 * elements, four independent chains), with the words XOR-folded instead of
 * compared and packed and nothing stored (sink: one device uint32, written only
 * in the never-taken case).  bench.py times it to give the draw a VALU roofline.
 */
GA_API int ga_probe_philox(int64_t n, uint32_t* sink, hipStream_t stream);

/*
 * Calibration helper (no reference counterpart): the memory floor of the DeMo
 * codec's access pattern (demo_impl/demo.py:142-209 through ga_demo_encode_sym /
 * ga_demo_decode_sym).  One wavefront per 64x64 chunk of a [rows, cols] fp32
 * matrix (rows, cols multiples of 64), the chunk kernels' grid and coalesced
 * layout, no transform: mode 0 reads a and b and writes a (the encode's 12 B per
 * element), mode 1 reads a and writes a and b (the decode's).  bench.py prices
 * the codec kernels against it on a matrix of the model's size.
 */
GA_API int ga_probe_chunk_stream(float* a, float* b, int64_t rows, int64_t cols, int mode, hipStream_t stream);

/*
 * Placement probe (no reference counterpart) for the fused DiLoCo outer step:
 * ga_diloco_outer's access pattern over an fp32 [K, ld_src] replica set (K <= 16)
 * and a master / momentum pair -- every stream read and written back through the
 * kernel's own loads and stores -- with every value unchanged.  On MI355X the
 * step's rate depends on where master / momentum sit physically relative to the
 * replicas (1.65 vs 1.88 ms at GPT-2 124M x 8 for the same virtual layout,
 * profiles/r04b_placement_search_p*.txt); DiLoCoOuter times candidate buffers with
 * this probe once and keeps the fastest (gym_amd/engine.py).
 */
GA_API int ga_probe_diloco_placement(float* src, int64_t K, int64_t ld_src, int64_t n, float* master, float* mom,
                                     hipStream_t stream);

/*
 * Placement probe (no reference counterpart) for the in-place replica mean
 * (ga_replica_mean with dst == src, the SimpleReduce / FedAvg step over K local
 * replicas): its access pattern over an fp32 [K, ld_src] set (K <= 16, n a
 * multiple of 4) with every value written back unchanged.  The in-place mean over
 * GPT-2 124M x 8 runs 1.49 ms in an ordinary allocation and 1.26 ms in the
 * fastest of 12 fresh ones (profiles/r05y_mean_placement.txt); MeanReduce times
 * candidate sets with this probe once and moves the caller's set to the fastest.
 */
GA_API int ga_probe_mean_placement(float* src, int64_t K, int64_t ld_src, int64_t n, hipStream_t stream);

/*
 * Placement probe (no reference counterpart) for the fused Adam/AdamW step:
 * ga_adam_step's access pattern over fp32 [K, ld] param / grad / exp_avg /
 * exp_avg_sq sets (n a multiple of 4, 16-byte aligned) -- p, g, m, v read, p, m,
 * v written back unchanged.  ArenaAdam times candidate physical buffers for the
 * moments with it once (the step ran 0.553-0.625 ms at GPT-2 124M by where they
 * sit, profiles/r04k_adam_placement.txt).
 */
GA_API int ga_probe_adam_placement(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t K,
                                   int64_t ld, int64_t n, hipStream_t stream);

/* ---- mean reduce: SimpleReduce / FedAvg / DiLoCo averaging ------------- */

/*
 * dst_j[i] = (sum_{k<K} src[k*ld_src + i]) / divisor   for j < K_out, i < n
 * (dst_j = dst + j*ld_dst).  Sum in ascending k, fp32 accumulation, then a
 * correctly rounded true division (reference quirk Q2: division, not *1/K).
 * If `rows` is non-null it is a device array of K int32 replica indices and
 * replica rows[k] is read instead of replica k (FedAvg islands).
 * dst may alias src (in-place all-replica average).  divisor == 1 gives a sum.
 *
 * Replaces: exogym/strategy/strategy.py:130-133 (per-param all_reduce + div_),
 *           exogym/strategy/diloco.py:34-37, exogym/strategy/federated_averaging.py:53-69,
 *           exogym/trainer.py:95-119 (final state averaging).
 */
GA_API int ga_replica_mean(int dtype, const void* src, int64_t K, int64_t ld_src,
                           const int32_t* rows, int64_t n, float divisor,
                           void* dst, int64_t K_out, int64_t ld_dst, hipStream_t stream);

/* ---- DiLoCo outer step -------------------------------------------------- */

/*
 * Fused DiLoCo outer step over n elements (one arena or one shard of it):
 *   avg  = (sum_{k<K} src_k[i]) / divisor                 (diloco.py:34-37)
 *   g    = master[i] - avg                                (diloco.py:43-45)
 *   g   += weight_decay * master[i]          if weight_decay != 0
 *   buf  = first_step ? g : momentum*buf + (1-dampening)*g   if momentum != 0
 *   g    = nesterov ? g + momentum*buf : buf                  if momentum != 0
 *   master[i] -= lr * g                                   (torch SGD, diloco.py:70)
 *   dst_j[i] = master[i]  for j < K_out                   (diloco.py:47-49 + 39-41)
 * `mom` may be null when momentum == 0.  master and mom are fp32 when
 * master_f32 != 0, otherwise they share `dtype` with src/dst.
 *
 * Replaces: exogym/strategy/diloco.py:51-76 (the outer-step branch) and the
 * CPU torch.optim.SGD it drives (diloco.py:26-28,86).
 */
GA_API int ga_diloco_outer(int dtype, const void* src, int64_t K, int64_t ld_src,
                           int64_t n, float divisor, void* master, void* mom,
                           int master_f32, int first_step, float lr, float momentum,
                           float dampening, float weight_decay, int nesterov,
                           void* dst, int64_t K_out, int64_t ld_dst, hipStream_t stream);

/* ---- SPARTA sparse averaging ------------------------------------------- */

/* Workspace bytes needed by ga_sparta_select for an arena of n elements. */
GA_API int64_t ga_sparta_workspace_bytes(int64_t n);

/*
 * Gap table of the Philox mask stream for selection rate p (64 entries):
 * table[j] = round(2^32 * (1 - (1 - p)^(j + 1))) (0 for p <= 0, 2^32 for
 * p >= 1), nondecreasing.  Each 64-element group g of the arena reads the
 * 32-bit words of philox4x32_10(key = seed, ctr = {g, r, iteration_lo,
 * iteration_hi}), r = 0, 1, ..., in order (x, y, z, w); starting at pos = 0,
 * a word u >= table[63] ends the group, otherwise pos += #{j : table[j] <= u},
 * element 64 g + pos is selected if pos < 64, and pos += 1 (the group ends at
 * pos >= 64).  The gaps are Geometric(p): every element is selected
 * independently with probability p (up to the 2^-32 rounding of the table).
 */
GA_API void ga_sparta_gap_table(double p, uint64_t* table);

/*
 * bits[w] = OR_j (mask[64 w + j] != 0) << j over the n-element uint8 mask
 * arena, ceil(n/64) words, bits past n zero: rank 0's selector masks in the
 * form they are broadcast at N > 1 (n/8 bytes on the wire instead of the
 * reference's n bool bytes per step, sparta.py:32-37).
 */
GA_API int ga_sparta_pack_mask(const uint8_t* mask, int64_t n, uint64_t* bits, hipStream_t stream);

/*
 * The reference's per-tensor mask draw, RandomIndexSelector.get_indices =
 * torch.bernoulli(torch.full(shape, p, device=cuda)) (sparta.py:80-85), for
 * every drawn tensor in one launch, bit-identical to ATen's HIP kernel for it:
 * tensor i (table row i = {arena offset (a multiple of 64), numel, first
 * workgroup}, each workgroup ga_sparta_torch_bernoulli_span() elements of one
 * tensor, nblocks in total) uses generator offset offset0 + i * offset_step; element
 * 4t + j of the tensor is selected iff the j-th uniform of Philox4x32-10
 * (key seed, counter {offset/4, t}) is <= p.  GA_MASK_BYTES: mask[offset + e]
 * <- 0/1; GA_MASK_BITS (arena offsets multiples of 64): the tensor's bits of
 * the packed words (ga_sparta_pack_mask layout; words of tensors not drawn
 * are left as they are).  If seedoff != null (device memory, {seed,
 * offset0}) those replace the seed/offset0 arguments: the generator state rank
 * 0 broadcast (16 bytes), so every rank draws rank 0's masks (the reference
 * broadcasts the masks themselves, sparta.py:32-37).  The caller advances its
 * torch generator by ntens * offset_step.
 */
/* sizeof(ga_sparta_torch_draw) (binding layout check). */
GA_API int ga_sparta_torch_draw_bytes(void);

/* Elements per workgroup of ga_sparta_torch_bernoulli (the table's first-workgroup unit). */
GA_API int64_t ga_sparta_torch_bernoulli_span(void);

GA_API int ga_sparta_torch_bernoulli(const int64_t* table, int32_t ntens, int64_t nblocks, float p,
                                     uint64_t seed, uint64_t offset0, uint64_t offset_step,
                                     const uint64_t* seedoff, void* mask, int mask_format,
                                     hipStream_t stream);

/*
 * Select the SPARTA index set over an arena of n elements and gather the
 * selected values summed over the K local replicas (replica set in `layout`,
 * GA_LAYOUT_*).
 *   mask source: if mask != null, element i is selected iff its mask entry is
 *   set (mask_format GA_MASK_BYTES: uint8 mask arena, GA_MASK_BITS: the packed
 *   words of ga_sparta_pack_mask -- rank 0's per-tensor index_selector masks,
 *   broadcast, sparta.py:32-37; GA_MASK_TORCH: mask -> a host
 *   ga_sparta_torch_draw, the reference's draw computed in-kernel); otherwise
 *   the in-kernel Philox4x32-10 stream decides
 *   with selection rate p (see ga_sparta_gap_table), except inside the `nskip` element ranges skip[2r] <= i < skip[2r+1]
 *   (sorted, disjoint: the tensors without a gradient, which the reference
 *   skips, sparta.py:29-30; skip may be null when nskip == 0).
 * Outputs (device): idx[j] = j-th selected element index in ascending order
 * (row-major over the arena, == param.data[mask] order, sparta.py:38),
 * vals[j] = sum_k src_k[idx[j]], count[0] = number selected (int64),
 * count[1] = 1 if that exceeded `cap` (only the first cap are written).
 * `work` must hold ga_sparta_workspace_bytes(n) bytes.
 *
 * Replaces: RandomIndexSelector.get_indices (sparta.py:80-85), the mask
 * broadcast and gather of SparseCommunicator.communicate (sparta.py:24-38).
 */
GA_API int ga_sparta_select(int dtype, const void* src, int64_t K, int64_t ld,
                            int layout, int64_t n, const void* mask, int mask_format,
                            uint64_t seed, uint64_t iteration, double p,
                            const int64_t* skip, int64_t nskip, int64_t cap,
                            int32_t* idx, void* vals, int64_t* count, void* work,
                            hipStream_t stream);

/*
 * dst_k[idx[j]] = vals[j] / divisor for j < min(count[0], cap), k < K
 * (replica set in `layout`, GA_LAYOUT_*).
 * Replaces: `sparse_data /= num_nodes; param.masked_scatter_(mask, sparse_data)`
 * (sparta.py:40-42).
 */
GA_API int ga_sparta_scatter(int dtype, const void* vals, const int32_t* idx,
                             const int64_t* count, int64_t cap, float divisor,
                             void* dst, int64_t K, int64_t ld, int layout, hipStream_t stream);

/*
 * Single-process SPARTA step (every node is a local replica, no exchange):
 * select as ga_sparta_select, then each selected element of every replica
 * <- (sum over the K replicas) / divisor, in the same pass (the gathered lines
 * are written back while still in L2).  idx/vals/count/work may all be null
 * (no packed list, no count/scan pass); if given they are filled as by
 * ga_sparta_select.  Replaces sparta.py:24-44 for batched replicas.
 */
GA_API int ga_sparta_average_local(int dtype, void* reps, int64_t K, int64_t ld, int layout, int64_t n,
                                   const void* mask, int mask_format, uint64_t seed,
                                   uint64_t iteration, double p, const int64_t* skip, int64_t nskip,
                                   float divisor, int32_t* idx, void* vals,
                                   int64_t cap, int64_t* count, void* work, hipStream_t stream);

/* ---- DeMo DCT codec ------------------------------------------------------ */

/*
 * One parameter tensor as the DeMo codec sees it: a 2-D [rows, cols] view of
 * the arena at `offset` (1-D [L] -> [1, L] with n1 = 1; 4-D [b,c,h,w] ->
 * [b*c*h, w] with n1 = h, n2 = w), cut into gy x gx chunks of n1 x n2
 * (demo_impl/demo.py:255-276).  Each chunk sends k entries
 * (k = clamp(topk, 1, n1*n2), demo.py:307-323) stored at payload entry
 * payload_off + chunk*k.  basis1/basis2 index the 64x64 basis tables
 * (zero padded; n = 1 is the identity).  chunk_start is the prefix sum of
 * gy*gx over the descriptor table.
 */
typedef struct ga_demo_tensor {
    int64_t offset;
    int64_t payload_off;
    int32_t rows, cols;
    int32_t n1, n2;
    int32_t gy, gx;
    int32_t k;
    int32_t basis1, basis2;
    int32_t chunk_start;
} ga_demo_tensor;

/* sizeof(ga_demo_tensor) as compiled into the library (ABI check for bindings). */
GA_API int ga_demo_tensor_bytes(void);

/*
 * Encode + compress + residual for every chunk of every tensor, for each of
 * K replicas (replica r: param/grad/delta at + r*ld, payload at + r*payload_stride):
 *   p     *= wd_factor                      if wd_factor != 1 (demo.py:159-160; the
 *                                           caller passes 1 - lr*weight_decay computed
 *                                           in double, as the reference's Python scalar)
 *   delta  = decay*delta + lr*grad          (demo.py:163-167)
 *   Y      = F1^T . delta_chunk . F2        (DCT-II, demo.py:255-276; fp32 MFMA)
 *   top-k of |Y| per chunk                   (demo.py:315-328; ties: lowest index)
 *   delta -= B1^T . S . B2                  (S = the k kept coefficients, demo.py:174-180)
 * Payload per replica: idx int32[M] then val f32[M] (M = total entries), entries
 * of one chunk in ascending coefficient index.  F/B tables: [nbasis][64][64] fp32.
 */
GA_API int ga_demo_encode(int dtype, const ga_demo_tensor* tensors, int32_t ntensors,
                          int32_t nchunks, const float* F, const float* B,
                          void* param, const void* grad, void* delta, int64_t K,
                          int64_t ld, float lr, float decay, float wd_factor,
                          int32_t* payload, int64_t payload_stride, int64_t M,
                          hipStream_t stream);

/*
 * Up to 64 consecutive 1x64 chunks of one tensor (rows of a vector's chunk
 * view): element offset of the first chunk, payload entry offset of its
 * entries, number of chunks, entries per chunk.
 */
typedef struct ga_demo_rowgroup {
    int64_t offset;
    int64_t payload_off;
    int32_t rows;
    int32_t k;
} ga_demo_rowgroup;

/*
 * ga_demo_encode (demo.py:142-209 encode + compress + residual) for plans whose
 * chunks are all 64x64 or 1x64 with k <= 64 -- compression_chunk = 64 on
 * GPT-2-shaped models: same arithmetic, payload layout and tie rule.  The
 * 64x64 chunks are described by `tensors` (only 64x64 tensors, chunk_start
 * counting those chunks, payload_off as in the full plan), the 1x64 chunks by
 * `groups`; F64 is the 64-point basis F[i][k] (64x64 fp32).  One wavefront per
 * chunk (or row group), operands register-resident, the DCT products folded by
 * the symmetry F[63-i][k] = (-1)^k F[i][k].
 */
GA_API int ga_demo_encode_sym(int dtype, const ga_demo_tensor* tensors, int32_t ntensors,
                              int32_t nchunks, const ga_demo_rowgroup* groups, int32_t ngroups,
                              const float* F64, void* param, const void* grad, void* delta,
                              int64_t K, int64_t ld, float lr, float decay, float wd_factor,
                              int32_t* payload, int64_t payload_stride, int64_t M,
                              hipStream_t stream);

/*
 * Decode the gathered payloads of S sources (source s at payload + s*payload_stride,
 * in node order), scatter-mean them per chunk (mean over the entries that hit a
 * coefficient, demo.py:331-352), inverse DCT (B1^T . X . B2), sign, and apply the
 * SGD step to each of K local replicas:  grad = sign(g);  p -= lr*grad
 * (demo.py:192-209).  grad may be null (then only p is written).
 */
GA_API int ga_demo_decode(int dtype, const ga_demo_tensor* tensors, int32_t ntensors,
                          int32_t nchunks, const float* B, const int32_t* payload,
                          int64_t payload_stride, int64_t M, int64_t S, void* param,
                          void* grad, int64_t K, int64_t ld, float lr,
                          hipStream_t stream);

/*
 * ga_demo_decode for the plans ga_demo_encode_sym takes (64x64 chunks in
 * `tensors`, 1x64 chunks in `groups`, F64 the 64-point basis) and S <= 15
 * sources: same arithmetic and replica update as ga_demo_decode
 * (demo.py:192-209, 331-352), one wavefront per chunk or row group.  S == 1 is
 * a sparse synthesis of the k entries; S >= 2 scatter-adds the sources in node
 * order into an LDS tile with 4-bit hit counts, takes the mean over hitters and
 * runs the inverse transform as two folded 64-deep MFMA products.
 */
GA_API int ga_demo_decode_sym(int dtype, const ga_demo_tensor* tensors, int32_t ntensors,
                              int32_t nchunks, const ga_demo_rowgroup* groups, int32_t ngroups,
                              const float* F64, const int32_t* payload, int64_t payload_stride,
                              int64_t M, int64_t S, void* param, void* grad, int64_t K, int64_t ld,
                              float lr, hipStream_t stream);

/* ---- inner optimizer on the arena --------------------------------------- */

/* Number of fp32 partials ga_grad_clip_coef needs in its `partials` buffer. */
GA_API int ga_sumsq_partials_count(void);

/*
 * Gradient-norm clipping coefficient per replica k < K of a gradient replica set
 * (replica k: n elements at grad + k*ld):
 *   out[2k+1] = ||grad_k||_2 (fp32 partial sums in a fixed order), and
 *   out[2k]   = min(1, max_norm / (out[2k+1] + 1e-6)).
 * `partials` holds K * ga_sumsq_partials_count() floats.  Device side only
 * (nothing synchronises); ga_adam_step applies out[2k] to replica k.
 * Replaces: torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm) at
 * exogym/strategy/strategy.py:135-138, communicate_optimize_strategy.py:69-71,
 * diloco.py:52-56 (the per-tensor norms + stack + norm + per-tensor mul_).
 */
GA_API int ga_grad_clip_coef(int dtype, const void* grad, int64_t K, int64_t ld, int64_t n, float max_norm,
                             float* partials, float* out, hipStream_t stream);

/*
 * One fused Adam/AdamW step over K replicas of an fp32 arena (param, grad,
 * exp_avg, exp_avg_sq: [K, ld] sets, n elements per replica, 16-byte aligned),
 * every replica with the same hyper-parameters, in torch's op order
 * (torch/optim/adam.py, _multi_tensor_adam):
 *   g = grad * clip_coef[2k]  (and written back) if clip_coef != null and < 1
 *   p *= wd_factor            (AdamW: 1 - lr*weight_decay, computed by the caller in double)
 *   g += l2_wd * p            (Adam with weight_decay)
 *   m = lerp(m, g, lerp_w)    (lerp_w = 1 - beta1)
 *   v = beta2*v + one_m_beta2*g*g
 *   p += step_size * m / (sqrt(v)/bc2_sqrt + eps)   (step_size = -lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t))
 * Replaces: `self.optim.step()` with the default inner optimizer
 * torch.optim.AdamW (exogym/strategy/strategy.py:140, diloco.py:59,
 * communicate_optimize_strategy.py:74; OptimSpec default optim.py:11).
 */
GA_API int ga_adam_step(int dtype, void* param, void* grad, float* exp_avg, float* exp_avg_sq, int64_t K,
                        int64_t ld, int64_t n, float lerp_w, float beta2, float one_m_beta2, float eps,
                        float wd_factor, float l2_wd, float step_size, float bc2_sqrt, const float* clip_coef,
                        hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GYM_AMD_H */
