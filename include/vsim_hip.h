/* include/vsim_hip.h — C-ABI of libvsim_hip.so, the MI355X (gfx950) replacement for the
 * reference's imax.c / emax7lib.c offload layer.
 *
 * Three layers, all plain C types (no torch / HIP types in any signature):
 *
 *  1. Drop-in entry points with the reference's own symbol names and signatures, so a
 *     reference build links libvsim_hip.so where it linked imax.o:
 *       init_xmax()                                   replaces imax.c:52-142
 *       imax_ggml_compute_forward_mul_mat_q4_0_f32()  replaces imax.c:1133-2292
 *                                                     (called from ggml.c:5115)
 *     plus vsim_ggml_* hooks for the ops that have no offload boundary in the reference
 *     (RoPE ggml.c:6086/5919, soft_max ggml.c:5825, KQ/KQV mul_mat ggml.c:4355).
 *  2. Op-level device API (vsim_op_*): every hot op on device pointers, in the exact
 *     (reference-bit-identical) or fast numeric mode.  Used by the parity tests.
 *  3. Model-level executor (vsim_model_*): device-resident GPT-NeoX (vsim.cpp:470-747)
 *     and GPT-J graphs, whole decode step captured in a hipGraph; host<->device traffic
 *     per token is the token ids in and one logits row out (vsim.cpp:736-737).
 *
 * Device weight layout ("W4T32"): a Q4_0 matrix of M rows x K weights keeps the
 * reference's 0.625 B/weight but splits the 20-byte blocks (ggml.c:204-251) into a
 * 16-byte nibble plane followed by an fp32 scale plane, with rows grouped in tiles of 32
 * and, inside a tile, block b of all 32 rows stored contiguously (512 B of nibbles,
 * 128 B of scales) so row-per-lane waves read whole cache lines.  M is padded to a
 * multiple of 32: vsim_q4_bytes(M, K) = ceil(M/32)*32 * K/32 * 20 bytes.
 * Activation rows (vsim_op_q4_quantize output, "Q4 SoA"): nibble plane [n][K/32][16] then
 * scale plane [n][K/32], n*K/32*20 bytes.
 *
 * Every function returns 0 on success or a negative VSIM_E* code; vsim_last_error()
 * describes the last failure of the calling thread.
 */
#ifndef VSIM_HIP_H
#define VSIM_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "ggml_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VSIM_OK 0
#define VSIM_EINVAL (-1)
#define VSIM_EHIP (-2)
#define VSIM_ENOMEM (-3)
#define VSIM_EFILE (-4)
#define VSIM_ENODEV (-5)
#define VSIM_ESPIN (-6) /* a bounded cross-workgroup wait inside a fused kernel gave up: the
                           call's results are not valid (vsim_spin_timeouts counts them)  */

/* numeric modes */
#define VSIM_MODE_EXACT 0 /* bit-identical to the reference at --threads 1            */
#define VSIM_MODE_FAST 1  /* split-K integer-dot GEMV: same math, different rounding  */

/* architectures */
#define VSIM_ARCH_GPTNEOX 0 /* vsim.cpp:470-747                                      */
#define VSIM_ARCH_GPTJ 1    /* ggml GPT-J graph composed from the same ops           */
#define VSIM_ARCH_BLOOM 2   /* BLOOM graph (ALiBi, fused QKV) composed from the same ops
                               + ggml_alibi (ggml.c:6184-6244); convert_bloom_to_ggml.py */

const char *vsim_last_error(void);
int vsim_device_count(void);
size_t vsim_q4_bytes(int rows, int k);

/* ---------------------------------------------------------------- 1. drop-in ----- */
void init_xmax(void);
void imax_ggml_compute_forward_mul_mat_q4_0_f32(int THREAD, int LANE, const struct ggml_compute_params *params,
                                                const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                                                struct ggml_tensor *dst);
/* New hooks (same (params, src0, src1, dst) shape as the static ggml.c kernels they
 * replace; host tensors in, host tensors out, exact mode).  Called by every thread of the
 * reference's pool in every phase: the checks read metadata only, so all threads agree -
 * either every call returns VSIM_EINVAL (each thread runs its own CPU slice) or thread 0's
 * COMPUTE call runs the whole op and every call returns 0 (handled; INIT / FINALIZE have
 * nothing left to do).  mul_mat_f32 takes any strided F32 views; its transposed-src0 branch
 * (KQV) groups the partial sums by params->nth as ggml.c:4535-4581 + 4469-4493 does.  A
 * device failure after the checks exits, as the offload layer does (imax.c:2042-2049). */
int vsim_ggml_gptneox_rope_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                               const struct ggml_tensor *src1, struct ggml_tensor *dst);
int vsim_ggml_rope_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                       const struct ggml_tensor *src1, struct ggml_tensor *dst);
int vsim_ggml_soft_max_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                           struct ggml_tensor *dst);
int vsim_ggml_mul_mat_f32(const struct ggml_compute_params *params, const struct ggml_tensor *src0,
                          const struct ggml_tensor *src1, struct ggml_tensor *dst);
/* Device executor for the reference's graph: the drop-in for ggml_graph_compute
 * (ggml.c:8245-8700, called at vsim.cpp:725 as ggml_graph_compute(ctx0, &gf)).  Walks
 * cgraph->nodes[] in order on the GPU with the exact-mode kernels; the eval context's arena
 * (ctx's mem_buffer) and every leaf outside it (model weights, KV cache: mirrored once, then
 * device-resident) are mirrored at the same offsets, and the last node's bytes are copied
 * back to its host address.  The KQV product's thread-partial grouping follows
 * cgraph->n_threads, so the logits equal the reference's at any --threads.
 * vsim_graph_compute prints the error and exits (as the reference's offload layer does,
 * imax.c:2042-2049); vsim_graph_compute_rc returns VSIM_E* instead and leaves host memory
 * untouched when a node is not supported (all nodes are checked before any runs). */
void vsim_graph_compute(struct ggml_context *ctx, struct ggml_cgraph *cgraph);
int vsim_graph_compute_rc(struct ggml_context *ctx, struct ggml_cgraph *cgraph);
/* copy one tensor of the last computed graph back to its host address */
int vsim_graph_sync_tensor(const struct ggml_tensor *t);
/* forget every mirror (weights, KV cache, arena) */
void vsim_graph_reset(void);
void vsim_graph_stats(uint64_t *computes, uint64_t *nodes, uint64_t *h2d_bytes, uint64_t *d2h_bytes);
/* per-op device time (event pair per node; also VSIM_GRAPH_PROFILE=1): enable resets the
 * totals; the report is a text table with the reference's monitor.c row names
 * (monitor.c:182-262, show_time_sep).  Returns the report's full length. */
int vsim_graph_set_profile(int enable);
int vsim_graph_profile_report(char *buf, size_t cap);
/* Decode fast path of vsim_graph_compute.  A single-token eval of gptneox_eval
 * (vsim.cpp:470-747, use_parallel_residual = 1) is recognised node by node (42 nodes per
 * layer in ggml_build_forward_expand order, plus get_rows and the final norm + lm_head) and
 * runs as the model executor's fused decode step -- 2 launches per layer (since r06), replayed as one
 * hipGraph -- on the weights and KV cache the per-node path mirrored, with the KQV grouping of
 * cgraph->n_threads.  Every other graph (prompt batches, the serial residual) runs per node.
 * VSIM_GRAPH_FAST=0 turns the fast path off.
 * vsim_graph_match checks a graph on the host only (no device needed): 0 and the recognised
 * shape in `info`, or VSIM_EINVAL with the first mismatch in vsim_last_error(). */
typedef struct {
  int32_t n_layer, n_embd, n_head, n_rot, n_vocab, n_ctx, n_past, token;
} vsim_graph_match_info;
int vsim_graph_match(const struct ggml_cgraph *cgraph, vsim_graph_match_info *info);
/* evals that took the fast path, and fast-path plans built (one per set of weight tensors) */
void vsim_graph_fast_stats(uint64_t *fast_evals, uint64_t *plans);
/* drop-in statistics: calls, bytes moved host<->device, device weight-cache size */
void vsim_dropin_stats(uint64_t *calls, uint64_t *h2d_bytes, uint64_t *d2h_bytes, uint64_t *cached_bytes);
void vsim_dropin_reset(void);

/* ------------------------------------------------------- 2. op-level (device ptrs) -- */
/* `stream` is a hipStream_t passed as void* (NULL = default stream). */
/* weights: ggml AoS blocks <-> W4T32 */
int vsim_op_q4_repack(const void *aos, void *w, int rows, int k, void *stream);
int vsim_op_q4_unpack(const void *w, void *aos, int rows, int k, void *stream);
/* activation rows: ggml AoS blocks <-> Q4 SoA */
int vsim_op_act_repack(const void *aos, void *xq, int n, int k, void *stream);
int vsim_op_act_unpack(const void *xq, void *aos, int n, int k, void *stream);
/* quantize_row_q4_0 (ggml.c:209-251) of n rows of k floats: xq in Q4 SoA, xd = the
 * dequantized values d*(q-8) the exact GEMV multiplies with (ggml.c:497-498). */
int vsim_op_q4_quantize(const float *x, int k, int n, void *xq, float *xd, void *stream);
/* y[n][M] = W[M][K] . q4_0(x)[n][K] (+ bias[M] if bias != NULL, added after the dot
 * as ggml_add does, vsim.cpp:545-547) */
int vsim_op_q4_gemv(const void *w, int M, int K, const void *xq, const float *xd, int n, const float *bias,
                    float *y, int mode, void *stream);
/* Long-prompt GEMM pieces (fast mode, N >= 256 inside the model): the fp16 image [M][K] of a
 * W4T32 weight (values d*(q-8) rounded to fp16), and Y[n][m] (+bias[m]) = sum_k W16[m][k] *
 * X16[n][k] on the 256 x 256-tile fp16 MFMA GEMM (K % 64 == 0; X16 [n][K] fp16). */
int vsim_op_q4_expand_f16(const void *w, int M, int K, void *w16, void *stream);
int vsim_op_gemm_f16(const void *w16, int M, int K, const void *x16, int n, const float *bias, float *y,
                     void *stream);
/* The activation step between two prompt GEMMs: x [n][K] f32 -> (x + bias, GELU table: when
 * gelu != 0) -> quantize_row_q4_0 per 32-block -> the values d*(q-8) as fp16 [n][K].  And the
 * fc_in GEMM with that step in its epilogue (q16 [n][M] instead of y; M % 32 == 0). */
int vsim_op_act_quant_f16(const float *x, int K, int n, const float *bias, int gelu, void *x16, void *stream);
int vsim_op_gemm_f16_gelu_q(const void *w16, int M, int K, const void *x16, int n, const float *bias, void *q16,
                            void *stream);
/* The same GEMM with the prompt layer's next step in its f32 epilogue:
 *  _rope: GPT-J rotary pairs (rows m, m+1 with m % d < n_rot, even m) at position p0 + n, as
 *    the rope + KV-write step of vsim.cpp:553-580 computes them (double cos/sin table cs
 *    [pos][n_rot/2][2], the products and differences in double, rounded to float);
 *  _join: the residual, res = res + (res_a + y) (vsim.cpp:694-695), or y + res when res_a is
 *    NULL (vsim.cpp:657), in place.  M % 4 == 0. */
int vsim_op_gemm_f16_rope(const void *w16, int M, int K, const void *x16, int n, const float *bias, float *y,
                          const double *cs, int d, int n_rot, int p0, void *stream);
int vsim_op_gemm_f16_join(const void *w16, int M, int K, const void *x16, int n, const float *bias, float *res,
                          const float *res_a, void *stream);
/* The model's long-prompt GEMM: the products of vsim_op_gemm_f16* straight from the W4T32
 * weight w, dequantized in LDS to the same fp16 halves (no image).  Epilogue, one at a time:
 * q16 != NULL the GELU-quantize one (y unused, bias required), cs != NULL the RoPE one into y,
 * join != 0 the residual join in place (y = res, res_a as in vsim_op_gemm_f16_join); else the
 * plain store (+ bias). */
int vsim_op_gemm_q4_256(const void *w, int M, int K, const void *x16, int n, const float *bias, float *y, void *q16,
                        const double *cs, int d, int n_rot, int p0, int join, const float *res_a, void *stream);
int vsim_op_get_rows(const void *w, int K, int V, const int32_t *rows, int n, float *y, void *stream);
/* ggml_norm (ggml.c:4246-4304); optional affine y = w*y + b (w, b may be NULL) */
int vsim_op_norm(const float *x, float *y, int k, int rows, const float *w, const float *b, void *stream);
/* cumulative counts of exact-LayerNorm rows that needed the sequential fallback:
 * out[0] = mean not certified, out[1] = variance scale not certified (summed over devices) */
int vsim_norm_fallbacks(unsigned out[2]);
/* cumulative count of bounded cross-workgroup waits that gave up, summed over devices and models:
 * the fused layer tail's waits (its attention heads, the in-tail LayerNorm's granules), the
 * barrier-free chain GEMV's ring hand-off, the prompt GEMM's stream-K finisher.  0 in every healthy
 * run; the model calls (eval, eval_argmax, generate, sync) count their own launches' timeouts and
 * return VSIM_ESPIN when that model's count grew. */
int vsim_spin_timeouts(unsigned *out);
int vsim_op_gelu(const float *x, float *y, int n, void *stream);
/* Greedy token of a logit row: *out = numpy.argmax(x[0:n]) (first index among equal maxima, -0.0 ==
 * +0.0, the first NaN if any); x and out device pointers; enqueued on stream, not synchronized.
 * The model's greedy step (vsim_model_eval_argmax / vsim_model_generate) runs the same kernel in
 * place of the reference's host-side greedy pick (sample_top_k with top_k = 1, utils.cpp:339-371,
 * called from vsim.cpp's main loop).  Ties differ: the reference orders equal logits by
 * std::partial_sort over (logit, id) pairs, whose order among equal keys the standard leaves
 * unspecified; this kernel returns the first index, as numpy does.  Distinct maxima agree. */
int vsim_op_argmax(const float *x, int n, int32_t *out, void *stream);
/* scale -> diag_mask_inf(n_past) -> soft_max over p[nz][nr][nc], in place */
int vsim_op_attn_softmax(float *p, int nc, int nr, int nz, int n_past, float scale, void *stream);
/* style 0 = GPT-NeoX rotate-half (ggml.c:6086), 1 = GPT-J pairs (ggml.c:5919);
 * x[T][H][d] in place; mode 0: p = n_past+i2, mode 1: i2 >= n_past only, p = i2 */
int vsim_op_rope(int style, float *x, int d, int H, int T, int n_past, int n_dims, int mode, void *stream);
int vsim_op_kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int n, float *kq,
               void *stream);
int vsim_op_kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int n, float *out, void *stream);
/* the same with the prompt's causal mask (query j sees keys <= n_past + j, ggml.c:5764-5798):
 * KQ leaves fully masked 64 x 64 tiles unwritten (diag_mask_inf overwrites them), KQV stops each
 * query tile's chains at its last unmasked key (every later probability is +0) - the model's
 * exact prompt path (run_layer) */
int vsim_op_kq_causal(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int n, int n_past,
                      float *kq, void *stream);
int vsim_op_kqv_causal(const float *V, int ldv, const float *S, int d, int H, int nk, int n, int n_past, float *out,
                       void *stream);
/* Fast-mode prompt attention (fp16 MFMA, one pass with an online softmax): for N queries
 * Q [N][d*H] at positions n_past.., keys/values kc/vc [n_past+N][d*H] (post-RoPE K),
 * out[q][h*d + dd] = softmax_k(scale * K.Q, causal) . V.  d in {64, 96, 128, 256}. */
int vsim_op_attn_prefill(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                         float scale, float *out, void *stream);
/* The same attention (d = 256 only) written as the next GEMM's fp16 operand out16 [N][d*H]:
 * quantize_row_q4_0 (ggml.c:209-251) of each 32-value block of the output row, the values
 * d*(q-8) as fp16 -- what vsim_op_act_quant_f16 makes of vsim_op_attn_prefill's out. */
int vsim_op_attn_prefill_q16(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                             float scale, void *out16, void *stream);
/* The long-prompt GEMM (vsim_op_gemm_q4_256, the model's N >= 256 path) splits the K range of
 * grids with fewer 256 x 256 tiles than CUs between two workgroups (stream-K: every CU busy, the
 * two partial sums added once; a different summation order than one pass, same per-element
 * bound).  enable = 0 keeps one pass per tile.  Process-wide; returns the previous setting. */
int vsim_gemm_set_streamk(int enable);
/* Two long-prompt GEMMs of one shape with the RoPE epilogue (the GPT-J prompt's Q and K
 * projections, vsim.cpp:540-580: ggml_mul_mat (ggml.c:4891-5165) then ggml_rope mode 0) in one
 * launch: y0 = RoPE(w0 x), y1 = RoPE(w1 x), M % 256 == 0, K % 128 == 0, positions p0 + n.  The
 * tile grid covers both; a remainder beyond whole rounds of the CUs is split as above.  Same
 * per-element bound as vsim_op_gemm_q4_256 with cs. */
int vsim_op_gemm_q4_256_pair(const void *w0, const void *w1, int M, int K, const void *x16, int n, float *y0, float *y1,
                             const double *cs, int d, int n_rot, int p0, void *stream);
/* mode 0: the model runs its prompt Q and K projections as two launches; 1 (default): one
 * paired launch, its remainder past whole rounds of the CUs split as above; 2: paired, whole
 * tiles only.  Process-wide; returns the previous setting. */
int vsim_gemm_set_qk_pair(int mode);
/* Order of the long-prompt GEMM's 256 x 256 tiles over the grid: groups of `cols` tile-columns
 * (256 tokens each), each group walked row by row, so the tiles one XCD runs together share
 * fewer activation slices; 0 = one group (row-major).  Used only when it divides the tile
 * columns.  Outputs do not depend on the order, except that a stream-K split then falls at other
 * tiles (same per-element bound).  Process-wide; returns the previous setting. */
int vsim_gemm_set_tile_order(int cols);
/* Fast-mode prompt LayerNorm (ggml_norm + affine, ggml.c:4246-4304, double sums in any order)
 * straight to the next GEMM's fp16 operand: quantize_row_q4_0 per 32-value block, d*(q-8) as
 * fp16 -- what vsim_op_act_quant_f16 makes of the normalized rows. */
int vsim_op_norm_f16q(const float *x, int k, int rows, const float *w, const float *b, void *x16, void *stream);
/* device fp16 tables (exp, gelu) as built by ggml_init (ggml.c:1240-1251) */
int vsim_op_tables(uint16_t *exp_f16_host, uint16_t *gelu_f16_host);

/* ------------------------------------------------------ 3. model-level executor ---- */
typedef struct vsim_model vsim_model;

typedef struct {
  int32_t n_vocab, n_embd, n_head, n_layer, n_rot, use_parallel_residual;
} vsim_hparams;

/* Layers [layer_begin, layer_end) live on `device`; the first stage also owns the
 * embedding, the last stage ln_f + lm_head. */
int vsim_model_create(int arch, const vsim_hparams *hp, int n_ctx, int device, int layer_begin, int layer_end,
                      vsim_model **out);
/* Load a ggml model file of `arch` (vsim.cpp:108-458 / convert_gptj_to_ggml.py format);
 * creates the model, uploads every tensor this stage owns. */
int vsim_model_load_file(const char *path, int arch, int n_ctx, int device, int layer_begin, int layer_end,
                         vsim_model **out);
/* Upload one tensor by its ggml-file name (Q4_0 tensors in the on-disk AoS format). */
int vsim_model_set_tensor(vsim_model *m, const char *name, const void *host, size_t nbytes);
/* Read one tensor back in the same file format (Q4_0 as AoS blocks, F32 as floats). */
int vsim_model_get_tensor(vsim_model *m, const char *name, void *host, size_t nbytes);
/* Synthetic weights drawn on the device (N(0,std), LN gains 1+N(0,std)), quantized with
 * quantize_row_q4_0 semantics; for throughput runs of full-size configs. */
int vsim_model_randomize(vsim_model *m, uint64_t seed, float std);
int vsim_model_set_mode(vsim_model *m, int mode);
/* Allocates ahead what a prompt of up to n_tokens sets up on its first eval (the N-token
 * scratch, the fp16 key copies of the prompt attention, the GEMMs' stream-K workspace) and
 * loads the prompt kernels, so that the first prompt runs at the steady-state rate.  Optional:
 * an eval allocates whatever is missing itself.  VSIM_EINVAL if n_tokens is not in 1..n_ctx. */
int vsim_model_reserve(vsim_model *m, int n_tokens);
int vsim_model_hparams(const vsim_model *m, vsim_hparams *hp, int *n_ctx, int *layer_begin, int *layer_end);
/* One eval of N tokens at n_past (vsim.cpp:470-747).  First stage reads `tokens`;
 * non-first stages read the residual from `resid_in` (device, [N][n_embd] f32);
 * non-last stages write their residual to `resid_out` (device); the last stage copies
 * the last row of logits to `logits` (host, n_vocab floats) if non-NULL. */
int vsim_model_eval(vsim_model *m, int n_past, const int32_t *tokens, int N, const float *resid_in,
                    float *resid_out, float *logits);
/* Greedy single-token decode step of a whole-model stage: eval of `token` at n_past, then
 * the argmax of the logits on the device (numpy.argmax conventions: first maximum, first
 * NaN); only the token id leaves the device.  The reference's loop samples on the host
 * from the logits (vsim.cpp:860-891); this is its greedy case without the logits copy. */
int vsim_model_eval_argmax(vsim_model *m, int n_past, int32_t token, int32_t *next_token);
/* Device-resident greedy generation: n_steps single-token steps from (n_past, token), each
 * step's argmax feeding the next on the device (no host round trip per token); the
 * n_steps generated tokens are copied to tokens_out at the end.  Same tokens as calling
 * vsim_model_eval_argmax n_steps times. */
int vsim_model_generate(vsim_model *m, int n_past, int32_t token, int n_steps, int32_t *tokens_out);
/* Pipeline stage step: the single-token step of this stage's layers between
 * device buffers the caller binds once -- tok_in (first stage: the token to embed), resid_in
 * (other stages: the [n_embd] residual from the previous stage), resid_out (non-last stages:
 * this stage's residual for the next), tok_out (last stage: the greedy token, device argmax,
 * numpy.argmax conventions).  stage_begin sets n_past on the device; every stage_step
 * enqueues one step on the model's stream without waiting (captured as a hipGraph when the
 * graph is on) and advances the device n_past, so a caller can queue steps and the
 * collective sends / receives between them on that stream without a host round trip.
 * vsim_model_sync waits for the model's stream. */
int vsim_model_stage_bind(vsim_model *m, const int32_t *tok_in, const float *resid_in, float *resid_out,
                          int32_t *tok_out);
int vsim_model_stage_begin(vsim_model *m, int n_past);
int vsim_model_stage_step(vsim_model *m);
int vsim_model_sync(vsim_model *m);
/* Test support: size the scratch for n_tokens and fill every scratch buffer and the whole KV
 * cache with NaN, so that a kernel reading bytes no earlier kernel wrote shows up as a
 * changed (NaN) result.  Results of later evals must not depend on it. */
int vsim_model_debug_poison(vsim_model *m, int n_tokens);
/* Decode-step timing helpers for bench.py: the stream the executor launches on, and
 * device pointers of the last logits / residual buffers. */
void *vsim_model_stream(vsim_model *m);
const float *vsim_model_logits_dev(vsim_model *m);
/* Number of kernels one eval launches; whether the decode step replays a hipGraph. */
int vsim_model_info(vsim_model *m, int *kernels_per_eval, int *graph_enabled, size_t *weight_bytes);
int vsim_model_set_graph(vsim_model *m, int enable);
/* Per-kernel profiling for the live roofline: when enabled (this resets the totals), the
 * decode step runs without its hipGraph and an event pair on the model's stream brackets
 * every launch, tagged with the kernel's name and the algorithmic bytes it moves (Q4_0
 * weights at 0.625 B/weight, KV rows read and written, LayerNorm rows).
 * profile_kernel(i): totals of the i-th kernel name seen (VSIM_EINVAL past the last);
 * profile_stats: the sums over all of them. */
int vsim_model_set_profile(vsim_model *m, int enable);
int vsim_model_profile_kernel(vsim_model *m, int i, char *name, int name_cap, double *ms, long *launches,
                              double *bytes);
int vsim_model_profile_stats(vsim_model *m, double *gemv_ms, long *gemv_launches, double *gemv_bytes);
void vsim_model_free(vsim_model *m);

#ifdef __cplusplus
}
#endif

#endif /* VSIM_HIP_H */
