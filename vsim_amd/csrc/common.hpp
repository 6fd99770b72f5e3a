// vsim_amd/csrc/common.hpp — shared device helpers and launch declarations.
//
// Every translation unit is compiled with -ffp-contract=off: the reference's x86 build
// (-O2 -msse3, Makefile-ubuntu:5-6) never fuses a multiply into an add, and the exact
// kernels must round every product and sum exactly where the reference does.  Fast
// kernels that want FMA call __builtin_fmaf explicitly.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>

#include "../../include/vsim_hip.h"

namespace vsim {

constexpr int QK = 32;       // weights per Q4_0 block (ggml.c:204)
constexpr int QBYTES = 20;   // fp32 d + 16 nibble bytes (ggml.c:907-909)

// ---------------------------------------------------------------- weight layout W4T32
// Q4_0 weight matrix of `rows` x `k`: rows padded to tiles of T32; inside a tile block b
// of its 32 rows is contiguous.  Nibble plane qs (16 B per block) first, then the fp32
// scale plane d: block (r, b) lives at index ((r/32)*nb + b)*32 + r%32 of both.
constexpr int T32 = 32;

// clang vector types for register arrays: arrays of HIP's float4/uint4 classes that are
// copied or conditionally assigned are not promoted to registers (they land in scratch)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct W4 {
  const uint8_t *qs;
  const float *d;
  int rows, k, tiles;
  __host__ __device__ int nb() const { return k / QK; }
  __host__ __device__ size_t off(int r, int b) const {
    return ((size_t)(r / T32) * nb() + b) * T32 + (r & (T32 - 1));
  }
};

inline size_t w4_bytes(int rows, int k) { return (size_t)((rows + T32 - 1) / T32) * T32 * (k / QK) * QBYTES; }

inline W4 w4_view(const void *base, int rows, int k) {
  W4 v;
  v.rows = rows;
  v.k = k;
  v.tiles = (rows + T32 - 1) / T32;
  const size_t nblk = (size_t)v.tiles * T32 * (k / QK);
  v.qs = (const uint8_t *)base;
  v.d = (const float *)((const uint8_t *)base + nblk * 16);
  return v;
}

// A batch of up to 4 independent GEMVs (same token) in one launch; workgroups take the
// tiles of job 0, then job 1, ...  Activation operands: xd = dequantized factors (exact
// mode), xqs/xdd = Q4_0 nibbles and scales of the activation row (fast mode).
// Epilogues: EPI_STORE y[row] = dot (+ bias[row]); EPI_GELU_Q: g = gelu_lut(dot + bias)
// (vsim.cpp:680-683), y[row] = g if y != NULL, and the tile's 32 values — block `tile` of
// the next product's activation row — are quantized with quantize_row_q4_0 semantics into
// (oq_qs, oq_d, oxd) (the INIT-phase quantization of the following mul_mat, ggml.c:5024).
enum { EPI_STORE = 0, EPI_GELU_Q = 1 };
struct GemvJob {
  W4 w;
  const float *xd;
  const uint8_t *xqs;
  const float *xdd;
  const float *bias;
  float *y;
  int epi;
  const uint16_t *gelu_tab;
  uint8_t *oq_qs;
  float *oq_d;
  float *oxd;
};
struct GemvBatch {
  GemvJob j[4];
  int nj;
};

// ---------------------------------------------------------------- fused decode kernels
// (layer.hip)
struct LnQuantJob {
  const float *x;      // [n] input row
  const float *w, *b;  // affine (non-null)
  uint8_t *qs;         // [n/32][16]
  float *d;            // [n/32]
  float *xd;           // [n]
  // optional residual join of the previous layer before the norm (ja == null: none):
  // row = x + ((ja + jab) + (jf + jfb)), stored to jout when non-null
  const float *ja, *jab, *jf, *jfb;
  float *jout;
  unsigned *ep;  // non-null: the decode step's epoch, advanced by one (the layer tails' tags, TailSync / TailLn)
};

// The next LayerNorm inside the layer tail (r06, k_layer_tail with TailJob::ln): the join
// v = x + ((a + ab) + (f + fb)) of the layer's two branches (vsim.cpp:694-695), the norm
// (ggml.c:4246-4304) from one round of per-tile partial sums, and the affine + Q4_0 quantize of
// one 32-block per tile (ggml.c:5024-5041), for norm 1 and optionally norm 2 (GPT-NeoX parallel
// residual: the post-attention norm of the same row).  Hand-offs inside the launch are data-
// tagged granules (tag = epoch << 8 | layer + 1): out-projection tile t's outputs (og, 8-byte
// {value, tag}), each tile's joined values (jg, for the fallback path) and partial sums (rec, two
// 16-byte granules), all sc1 stores polled with sc1 loads.
struct TailLn {
  const float *x;            // residual in [E]
  const float *ab, *fb;      // attention-output and MLP-output biases (ab may be null)
  float *jout;               // joined residual out [E]
  const float *w1, *b1;      // norm 1 affine
  uint8_t *q1;               // norm 1 output, Q4 SoA: nibbles [E/32][16], then d
  float *d1, *xd1;
  const float *w2, *b2;      // norm 2 (null: one norm)
  uint8_t *q2;
  float *d2, *xd2;
  unsigned long long *og, *jg;  // [E] granules
  uint4 *rec;                // [2 * E/32] granules
  const unsigned *ep;        // the step's epoch (written by the step's first k_ln_quant)
  unsigned *stats;           // LayerNorm fallback counters (dev_stats)
  int il;                    // layer index (tag)
};
constexpr int LNT_MAX_TILES = 256;  // E <= 8192

struct AttnJob {
  const float *q, *k, *v;  // new rows [E] (Q, K, V after bias)
  float *kc, *vc;          // this layer's cache, [n_ctx][E]
  const int *npast;        // device scalar
  const double2 *cs;       // RoPE cos/sin table [n_ctx][n_rot/2]
  const uint16_t *etab;    // table_exp_f16
  int d, H, n_rot, style;  // style 0 = GPT-NeoX rotate-half, 1 = GPT-J pairs
  int n_ctx;               // cache rows (sizes the LDS score array, attn_lds_floats)
  int nsplit;              // workgroups per head (column parts of KQV, attn.hpp); 0/1 = one
  int kqv_nth;             // KQV key grouping of the reference's pool (ggml.c:4535-4581, FINALIZE
                           // 4469-4493): keys in kqv_nth runs of ceil(nk/nth), each chained from 0,
                           // run sums added in order; 0/1 = one chain (--threads 1)
  float scale;
  const float *alibi;      // BLOOM: per-head ALiBi slopes (null: none); the single query row
                           // j = 0 gets (j + 1) * m_h added after the scale (ggml.c:6184-6244)
  uint8_t *oq_qs;          // output activation, Q4 SoA (E/32 blocks)
  float *oq_d, *oxd;
  float *out;              // optional float copy [E]
};

// exact decode attention (attn.hpp): LDS floats for q, k, the scores and two V tiles
constexpr int ATT_VTF = 8192;  // floats per V tile (32 KB)
__host__ __device__ constexpr int attn_lds_floats(int d, int n_ctx) {
  return ((2 * d + n_ctx + 3) & ~3) + 2 * ATT_VTF;
}

int launch_ln_quant(const LnQuantJob &j0, const LnQuantJob *j1, int n, hipStream_t s);
// out[i] = x[i] + ((a[i] + ab[i]) + (f[i] + fb[i]))  (ab may be null; a null: x[i] + (f[i] + fb[i]),
// the serial-residual graphs): the residual join alone
int launch_residual_join(const float *x, const float *a, const float *ab, const float *f, const float *fb, float *out,
                         int n, hipStream_t s);
int launch_gemv_epi(const GemvBatch &B, int mode, hipStream_t s);
int launch_attn_decode(const AttnJob &A, int n_ctx, hipStream_t s);
// exact-mode chain GEMV (gemv_chain.hip): a batch of jobs with the GemvBatch epilogues
int launch_gemv_chain_batch(const GemvBatch &B, hipStream_t s);
// true when launch_gemv_chain_batch runs B as k_gemv_solo (else k_gemv_chain32)
bool gemv_chain_solo(const GemvBatch &B);

// ---------------------------------------------------------------- fp16 (ggml.c:95-142)
__device__ __forceinline__ float bits_f(uint32_t w) { return __uint_as_float(w); }
__device__ __forceinline__ uint32_t f_bits(float f) { return __float_as_uint(f); }

__device__ __forceinline__ float h2f(uint16_t h) {
  const uint32_t w = (uint32_t)h << 16;
  const uint32_t sign = w & 0x80000000u;
  const uint32_t two_w = w + w;
  const float normalized = bits_f((two_w >> 4) + (0xE0u << 23)) * 0x1.0p-112f;
  const float denormalized = bits_f((two_w >> 17) | (126u << 23)) - 0.5f;
  return bits_f(sign | (two_w < (1u << 27) ? f_bits(denormalized) : f_bits(normalized)));
}

__device__ __forceinline__ uint16_t f2h(float f) {
  float base = (fabsf(f) * 0x1.0p+112f) * 0x1.0p-110f;
  const uint32_t w = f_bits(f);
  const uint32_t shl1_w = w + w;
  const uint32_t sign = w & 0x80000000u;
  uint32_t bias = shl1_w & 0xFF000000u;
  if (bias < 0x71000000u) bias = 0x71000000u;
  base = bits_f((bias >> 1) + 0x07800000u) + base;
  const uint32_t bits = f_bits(base);
  const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
  const uint32_t mantissa_bits = bits & 0x00000FFFu;
  const uint32_t nonsign = exp_bits + mantissa_bits;
  return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

// (int8_t)round(v) as the reference's x86 build evaluates it (ggml.c:239-240): round to
// nearest, ties away from zero, then cvttsd2si — whose out-of-range / NaN result is
// INT_MIN (low byte 0) where the GPU's v_cvt_i32_f32 would saturate.  Matters only for
// the degenerate blocks whose id = 1/d overflows (subnormal amax).
__device__ __forceinline__ int x86_round_i8(float v) {
  const float r = roundf(v);
  const int i = fabsf(r) < 2147483648.0f ? (int)r : (int)0x80000000u;
  return (int)(int8_t)i;
}

// The prompt GEMMs' fp16 activation value d*(q-8): the exact f32 x f32 product rounded once to
// fp16 (v_fma_mix with addend +0; d >= 0, so the product is never -0).  Spelled out because the
// compiler folds fptrunc(fmul) into this instruction in some kernels and rounds twice (f32,
// then fp16) in others -- and every producer of that operand must give the same bits.
__device__ __forceinline__ _Float16 f16_of_product(float a, float b) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return __builtin_bit_cast(_Float16, (uint16_t)r);
}

// ---------------------------------------------------------------- wave reductions
// Butterfly/broadcast steps in DPP (a few cycles each instead of an LDS permute round trip):
// quad_perm xor 1 and 2, row_half_mirror (8), row_mirror (16), row_bcast15 and row_bcast31
// (upper rows only), which leaves the full reduction in lane 63; readlane broadcasts it.
// Every caller combines values whose result is independent of the order (exact sums,
// min/max, or a sum whose rounding is bounded by a certificate).
namespace dpp {
constexpr int QP_XOR1 = 0xB1, QP_XOR2 = 0x4E, HALF_MIRROR = 0x141, MIRROR = 0x140, BCAST15 = 0x142, BCAST31 = 0x143;
template <int CTRL, int ROWS>
__device__ __forceinline__ int mov(int v, int identity) {
  return __builtin_amdgcn_update_dpp(identity, v, CTRL, ROWS, 0xF, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double mov(double v, double identity) {
  const long long b = __double_as_longlong(v), ib = __double_as_longlong(identity);
  const int lo = mov<CTRL, ROWS>((int)(b & 0xFFFFFFFF), (int)(ib & 0xFFFFFFFF));
  const int hi = mov<CTRL, ROWS>((int)(b >> 32), (int)(ib >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ float mov(float v, float identity) {
  return __int_as_float(mov<CTRL, ROWS>(__float_as_int(v), __float_as_int(identity)));
}
template <typename T, typename Op>
__device__ __forceinline__ T reduce(T v, T identity, Op op) {
  v = op(v, mov<QP_XOR1, 0xF>(v, identity));
  v = op(v, mov<QP_XOR2, 0xF>(v, identity));
  v = op(v, mov<HALF_MIRROR, 0xF>(v, identity));
  v = op(v, mov<MIRROR, 0xF>(v, identity));
  v = op(v, mov<BCAST15, 0xA>(v, identity));
  v = op(v, mov<BCAST31, 0xC>(v, identity));
  return v;  // lane 63 holds the reduction
}
__device__ __forceinline__ int lane63(int v) { return __builtin_amdgcn_readlane(v, 63); }
__device__ __forceinline__ float lane63(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63)); }
__device__ __forceinline__ double lane63(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFF), 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
}  // namespace dpp

__device__ __forceinline__ float wave_sum_f(float v) {
  return dpp::lane63(dpp::reduce(v, 0.0f, [](float a, float b) { return a + b; }));
}
__device__ __forceinline__ double wave_sum_d(double v) {
  return dpp::lane63(dpp::reduce(v, 0.0, [](double a, double b) { return a + b; }));
}
__device__ __forceinline__ float wave_max_f(float v) {
  return dpp::lane63(dpp::reduce(v, -INFINITY, [](float a, float b) { return fmaxf(a, b); }));
}
__device__ __forceinline__ int wave_min_i(int v) {
  return dpp::lane63(dpp::reduce(v, 0x7FFFFFFF, [](int a, int b) { return min(a, b); }));
}

// ---------------------------------------------------------------- errors
void set_error(const std::string &msg);
int hip_fail(hipError_t e, const char *what);
#define VSIM_HIP(call)                                          \
  do {                                                          \
    hipError_t e_ = (call);                                     \
    if (e_ != hipSuccess) return ::vsim::hip_fail(e_, #call);   \
  } while (0)

// ---------------------------------------------------------------- launchers (ops_*.hip)
// All return 0 / negative VSIM_E*; all enqueue on `s` and never synchronise.
struct DevTables {
  const uint16_t *exp_f16;   // table_exp_f16 (ggml.c:1249)
  const uint16_t *gelu_f16;  // table_gelu_f16 (ggml.c:1247)
};
int tables_get(DevTables *t);  // lazily uploads host-built tables for the current device
// Health counters of the current device (ops_elt.hip; null before tables_get on that device):
// LayerNorm fallbacks, and the bounded cross-workgroup waits that gave up
unsigned *dev_stats();
unsigned *spin_error_counter();  // the calling thread's target (set_spin_error_target) or the device's
// the word the bounded waits of the launches this thread enqueues count into (null: the current
// device's own counter); returns the previous target
unsigned *set_spin_error_target(unsigned *p);
void add_model_spin_timeouts(unsigned n);  // a model's timeouts, for vsim_spin_timeouts' total
int norm_stats(unsigned *out2);              // LayerNorm fallbacks, summed over devices
int spin_timeouts(unsigned *out);            // waits that gave up, summed over devices

int launch_q4_repack(const void *aos, void *soa, int rows, int k, hipStream_t s);
int launch_q4_unpack(const void *soa, void *aos, int rows, int k, hipStream_t s);
int launch_q4_quantize(const float *x, int k, int n, void *xq, float *xd, hipStream_t s);
int launch_q4_gemv(const void *w, int M, int K, const void *xq, const float *xd, int n, const float *bias,
                   float *y, int mode, hipStream_t s);
int launch_gemv_batch(const GemvBatch &B, int mode, hipStream_t s);
// exact mode, N > 1 tokens: every (row, token) the reference's fp32 chain (gemm_exact.hip)
int launch_gemm_exact(const W4 &W, const float *xd, int n, const float *bias, float *y, hipStream_t s);
int launch_act_repack(const void *aos, void *xq, int n, int k, hipStream_t s);
int launch_act_unpack(const void *xq, void *aos, int n, int k, hipStream_t s);
int launch_q4_dequant(const void *xq, int rows, int k, float *y, hipStream_t s);
int launch_get_rows(const void *w, int K, int V, const int32_t *rows, int n, float *y, hipStream_t s);
int launch_norm(const float *x, float *y, int k, int rows, const float *w, const float *b, hipStream_t s);
// prompt batches: the norm + affine of each row straight to the GEMM's fp16 operand
// (launch_act_quant_f16 of launch_norm's output, in one kernel)
int launch_norm_f16q(const float *x, void *x16, int k, int rows, const float *w, const float *b, hipStream_t s);
// ws: 16 bytes of zeroed device memory per concurrent caller (the kernel leaves it zeroed)
int launch_argmax(const float *x, int n, int *out, unsigned long long *ws, hipStream_t s);
int launch_gemm_q4_f16(const W4 &W, const void *xq, int n, const float *bias, float *y, hipStream_t s);
// fast-mode prompt batches (n >= GEMM_MIN_N): activation rows quantized (optionally after
// bias + GELU) straight to the GEMM's fp16 operand x16 [n][K], and the GEMM on it
constexpr int GEMM_MIN_N = 8;
int launch_act_quant_f16(const float *x, int K, int n, const float *bias, bool gelu, void *x16, hipStream_t s);
int launch_gemm_f16x(const W4 &W, const void *x16, int n, const float *bias, float *y, hipStream_t s);
// long prompts: fp16 weight images (launch_w4_expand_f16: [M][K], 2 bytes per weight) and the
// 256 x 256-tile GEMM on them (K % 64 == 0), same operand values as launch_gemm_f16x
constexpr int EXACT_GEMV_MAX_N = 32;  // exact prompt batches up to this many tokens run as batched decode GEMVs (ops_q4.hip)
constexpr int G2_MIN_N = 256;
int launch_w4_expand_f16(const W4 &W, void *out, hipStream_t s);
// q16 non-null: y is not written; bias + GELU + Q4_0 quantize of the result into q16 ([n][M]
// fp16 values d*(q-8), the next GEMM's operand, as launch_act_quant_f16(y, ..., gelu) makes)
// Extra work of its f32 epilogue (v = product + bias, per output row m and column n):
//  * cs != null: GPT-J RoPE of the row pairs (m, m+1) with m % d < n_rot, at position p0 + n
//    (k_rope_kv_write's arithmetic, ops_attn.hip), so Q and K leave the GEMM rotated;
//  * res != null: y = res + (res_a + v), or v + res without res_a (k_add_residual's orders;
//    y may be res);
//  * h16 != null (with or without RoPE): the result also as fp16 for the prompt attention,
//    row-major at h16[(p0 + n) * M + m] (its K copy), or with h16_t, transposed at
//    h16[m * h16_ld + vt_pos(p0 + n)] (its V^T copy) -- what k_kv_f16 makes of the cache rows.
// Key order of the prompt attention's V^T copy within each 16-key group: keys 0-3, 8-11,
// 4-7, 12-15 (the middle quads swapped), so the 8 keys one lane of the P^T MFMA operand needs
// (4 hl .. 4 hl + 3 and 8 + 4 hl .. 11 + 4 hl, the S^T accumulator's row order) are 16
// contiguous bytes: one ds_read_b128 per V fragment, conflict-free under the tile's swizzle.
__host__ __device__ constexpr int vt_pos(int k) { return (k & ~12) | ((k & 4) << 1) | ((k & 8) >> 1); }

struct G2Epi {
  const double2 *cs = nullptr;
  int d = 0, n_rot = 0, p0 = 0;
  const float *res = nullptr, *res_a = nullptr;
  _Float16 *h16 = nullptr;
  int h16_ld = 0, h16_t = 0;
};
// the same GEMM straight from the W4T32 weight (dequantized to the same fp16 halves in LDS, no
// image): what the model runs for N >= G2_MIN_N
int launch_gemm_q4_256(const W4 &W, const void *x16, int n, const float *bias, float *y, hipStream_t s,
                       void *q16 = nullptr, const G2Epi *epi = nullptr);
int launch_gemm_f16_256(const void *A16, int M, int K, const void *x16, int n, const float *bias, float *y,
                        hipStream_t s, void *q16 = nullptr, const G2Epi *epi = nullptr);
// the Q and K projections of a long GPT-J prompt (same M x K, RoPE epilogues) in one launch;
// gemm_pair_enabled: the model takes it for this shape (else two launch_gemm_q4_256 calls)
int launch_gemm_q4_256_pair(const W4 &W0, const W4 &W1, const void *x16, int n, float *y0, float *y1, const G2Epi &e0,
                            const G2Epi &e1, hipStream_t s);
bool gemm_pair_enabled(int M, int K);
int gemm_set_qk_pair(int mode);  // vsim_gemm_set_qk_pair (0 off, 1 default, 2 no split); returns the old setting
int gemm_set_tile_order(int cols);  // vsim_gemm_set_tile_order; returns the old setting
int gemm_set_streamk(int on);  // stream-K split of the register-dequant GEMM (default on); returns the old setting
int gemm_release_stream(hipStream_t s);  // frees the stream-K workspace of (current device, s)
int gemm_reserve_stream(hipStream_t s);  // the split workspace and kernel attributes, ahead of a prompt
int attn_prefill_prepare();              // the prompt attention's kernel attributes
bool attn_prefill_supported(int d);
// scratch: attn_prefill_scratch(E, n_past + N) bytes for the fp16 K / V^T copies (null or
// smaller: allocated stream-ordered per call); fresh: the new keys [n_past, n_past + N) are
// already there (written by the K and V GEMM epilogues, attn_prefill_k16/_vt16 give where)
// out16 (head dim 256 only, attn_prefill_quantizes): instead of out, the next GEMM's fp16
// operand -- quantize_row_q4_0 of each 32-value block, d*(q-8) as fp16 (k_act_quant_f16's values)
int launch_attn_prefill_f16(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                            float scale, float *out, hipStream_t s, void *scratch = nullptr, size_t scratch_bytes = 0,
                            bool fresh = false, void *out16 = nullptr);
bool attn_prefill_quantizes(int d);
int attn_prefill_ldt(int nk);  // V^T row length (keys padded to the key tile)
_Float16 *attn_prefill_k16(void *scratch, int E, int nk);
_Float16 *attn_prefill_vt16(void *scratch, int E, int nk);
size_t attn_prefill_scratch(int E, int nk);
// The heads' completion flags of the layer tail (r06): one 8-byte {unused, tag} sc1 granule per head
// workgroup, tag = epoch << 8 | layer + 1 (the epoch advanced by the step's first k_ln_quant), so
// no counter has to be zeroed between layers or steps
struct TailSync {
  unsigned long long *hflag;  // [TAIL_MAX_HEADS]
  const unsigned *ep;
  int il;
};
constexpr int TAIL_MAX_HEADS = 128;
// ln non-null (f and o one job each, both E rows): the tail also joins the residual and runs the
// next LayerNorm(s) (TailLn); neither job's y is written (the joined row goes to ln->jout)
int launch_layer_tail(const GemvBatch &f, const GemvBatch &o, const AttnJob &a, const TailSync &sy, int n_ctx,
                      hipStream_t s, const TailLn *ln = nullptr);
// true when the tail LayerNorm can run for a model of width E on the current device (every
// out-projection tile resident at once: E/32 tiles, one workgroup per CU)
bool tail_ln_ok(int E);
int launch_argmax_gen(const float *x, int n, int *out, unsigned long long *ws, int *tok, int *npast, int *hist,
                      hipStream_t s);
int launch_gelu(const float *x, float *y, int n, const float *bias, int bias_len, hipStream_t s);
int launch_attn_softmax(float *p, int nc, int nr, int nz, int n_past, float scale, hipStream_t s,
                        const float *alibi = nullptr);
// ggml_alibi head slopes (ggml.c:6217-6232), computed on the host with the reference's
// double pow and float rounding
void alibi_slopes_host(float *m, int n_head);
int launch_rope(int style, float *x, int d, int H, int T, int n_past, int n_dims, int mode,
                const double2 *cs, hipStream_t s);
// exact KQ / KQV of a batch of n queries over nk keys (attn_exact.hip); n_past >= 0: the causal
// mask of the prompt follows (query j sees keys <= n_past + j): fully masked KQ tiles are left
// unwritten, KQV stops at the last unmasked key.  merged = 1: out [n][H d], else [H][n][d]
int launch_kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int n, float *kq,
              hipStream_t s, int n_past = -1);
int launch_kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int n, float *out, int merged,
               hipStream_t s, int n_past = -1);
int launch_rope_kv_write(int style, float *Q, const float *K, const float *V, float *kcache, float *vcache,
                         int d, int H, int N, int n_past, int n_dims, const double2 *cs, hipStream_t s);
int launch_add_residual(float *inpL, const float *attn, const float *ff, int n, int order_ff_first,
                        hipStream_t s);
int launch_add_bias(float *x, const float *b, int k, int n, hipStream_t s);
int launch_randn_q4(void *soa, int rows, int k, uint64_t seed, float stddev, hipStream_t s);
int launch_randn_f32(float *x, int n, uint64_t seed, float stddev, float mean, hipStream_t s);

// host-side: cos/sin table of the reference RoPE angles (ggml.c:6117-6120 / 5952-5955),
// cs[p*(n_dims/2) + j] = {cos(p*theta_j), sin(p*theta_j)}, theta_j = 10000^(-2j/n_dims)
void rope_table_host(double2 *cs, int n_pos, int n_dims);

// model.cpp: a whole-model executor on borrowed device buffers (graph.cpp's fast path) and its
// per-call attention settings
int model_create_impl(int arch, const vsim_hparams *hp, int n_ctx, int device, int layer_begin, int layer_end,
                      const std::map<std::string, void *> *borrow, float *kc, float *vc, vsim_model **out);
int model_set_attn(vsim_model *m, int kqv_nth, float scale);

}  // namespace vsim
