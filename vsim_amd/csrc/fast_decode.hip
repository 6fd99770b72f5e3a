// vsim_amd/csrc/fast_decode.hip — fast-mode single-token decode step (VSIM_MODE_FAST).
//
// The fast mode keeps the reference's graph (vsim.cpp:521-696 for GPT-NeoX with the
// parallel residual; the same ops composed for GPT-J) and its Q4_0 x Q4_0 operands
// (activations re-quantized with quantize_row_q4_0 semantics, ggml.c:209-251), but sums
// each Q4_0 block with the integer dot v_dot8_i32_i4 and accumulates in any order, so it is
// HBM-bound rather than bound by the reference's sequential fp32 chain.  It is not
// bit-exact.  One layer = 4 launches:
//
//   k_fast_ln          LayerNorm(s) of the joined residual (ggml.c:4246-4304 + the affine,
//                      vsim.cpp:525-532), quantized (ggml.c:209-251)
//   k_fast_gemv        32-row tiles of {fc_in (+bias, GELU, quantize into fc_out's
//                      activation), Q, K, V}
//   k_fast_tail        fc_out split over K (FD_SF partial rows, summed in a fixed order by
//                      the next kernel) beside flash-decoding attention: each (head,
//                      64-position chunk) workgroup does RoPE (ggml.c:6086-6153 /
//                      5919-5974), the KV write, KQ, a chunk softmax and KQV
//   k_fast_oproj_join  merges the attention chunks and quantizes the attention output in
//                      every workgroup, then the out-projection and the residual join
//                      inpL + ((attn + b_o) + (ff + b_proj)) (vsim.cpp:694-695)
//
// The head (final LayerNorm + lm_head) is k_fast_ln + k_fast_gemv.  n_past is read from
// device memory, so the step is captured once in a hipGraph and replayed for every position.
#include <cstdlib>

#include "fast.hpp"
#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

// ------------------------------------------------------------------ helpers
// quantize_row_q4_0 (ggml.c:209-251) of one 32-value block held by a half-wave (lanes
// 0-31 or 32-63, element = lane & 31); writes the 4 nibble words and d (no xd factors).
__device__ __forceinline__ void fq_half(float v, int lane, bool ok, uint32_t *qw, float *dout, uint32_t xr = 0u) {
  auto mx = [](float a, float b) { return a > b ? a : b; };
  float a = fabsf(v);
  a = mx(a, dpp::mov<dpp::QP_XOR1, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::QP_XOR2, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::HALF_MIRROR, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::MIRROR, 0xF>(a, 0.0f));
  a = mx(a, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(a), 0x401F)));
  const float d = a / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  const int q = x86_round_i8(v * id) + 8;
  const int l = lane & 31;
  const int qn = dpp::mov<dpp::QP_XOR1, 0xF>(q, 0);
  const uint32_t byte = (l & 1) ? (uint32_t)((qn & 0xF) | ((q & 0xF) << 4)) : (uint32_t)((q & 0xF) | ((qn & 0xF) << 4));
  uint32_t word = byte << (8 * ((l >> 1) & 3));
  word |= (uint32_t)dpp::mov<dpp::QP_XOR2, 0xF>((int)word, 0);
  word |= (uint32_t)dpp::mov<dpp::HALF_MIRROR, 0xF>((int)word, 0);
  if (ok && (l & 7) == 0) qw[l >> 3] = word ^ xr;
  if (ok && l == 0) *dout = d;
}

// The same for a block held as 4 consecutive values in each of 8 consecutive lanes (lane
// group = lane / 8); writes this lane's 2 nibble bytes (XOR-ed with xr) and, from the
// group's first lane, d.
__device__ __forceinline__ void fq_oct(float4 v, int lane, bool ok, uint8_t *blk, float *dout, uint16_t xr = 0) {
  auto mx = [](float a, float b) { return a > b ? a : b; };
  float a = mx(mx(fabsf(v.x), fabsf(v.y)), mx(fabsf(v.z), fabsf(v.w)));
  a = mx(a, dpp::mov<dpp::QP_XOR1, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::QP_XOR2, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::HALF_MIRROR, 0xF>(a, 0.0f));
  const float d = a / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  const int q0 = x86_round_i8(v.x * id) + 8, q1 = x86_round_i8(v.y * id) + 8;
  const int q2 = x86_round_i8(v.z * id) + 8, q3 = x86_round_i8(v.w * id) + 8;
  const uint16_t w = (uint16_t)((q0 & 0xF) | ((q1 & 0xF) << 4) | ((q2 & 0xF) << 8) | ((q3 & 0xF) << 12));
  if (ok) {
    ((uint16_t *)blk)[lane & 7] = w ^ xr;
    if ((lane & 7) == 0) *dout = d;
  }
}

template <int NT>
__device__ __forceinline__ double block_sum_d(double v, double *red) {
  v = wave_sum_d(v);
  const int wid = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) s += red[w];
  return s;
}

// Signed 4-bit dot of a weight block and an activation block (nibble n encodes n - 8; the
// XOR with 8 turns it into the two's-complement nibble v_dot8_i32_i4 reads).
__device__ __forceinline__ int dot_q4(uint4 q, uint4 x) {
  int s = __builtin_amdgcn_sdot8((int)(q.x ^ 0x88888888u), (int)(x.x ^ 0x88888888u), 0, false);
  s = __builtin_amdgcn_sdot8((int)(q.y ^ 0x88888888u), (int)(x.y ^ 0x88888888u), s, false);
  s = __builtin_amdgcn_sdot8((int)(q.z ^ 0x88888888u), (int)(x.z ^ 0x88888888u), s, false);
  s = __builtin_amdgcn_sdot8((int)(q.w ^ 0x88888888u), (int)(x.w ^ 0x88888888u), s, false);
  return s;
}

// One wave's share of a 32-row tile: blocks b = b0 + h + 2i < b1 (h = lane >> 5, row =
// lane & 31), U loads per lane in flight, the next batch issued before the current one
// is consumed.  The activation (nibbles + scales) is read from LDS.  `pre` tells whether
// batch 0 was already issued by the caller (into qa/da).
template <int U = FD_U>
struct TileStream {
  const uint8_t *qs;  // tile's nibble plane: block b row r at (b*32 + r)*16
  const float *dd;    // tile's scale plane: (b*32 + r)
  int b0, b1, lane;
  int xoff = 0;  // first block of the activation slice staged in LDS
  uint4 qa[U];
  float da[U];

  // Slots past the wave's range still load (a neighbour's blocks, or the arena's FD_PAD
  // slack past the last tensor) and get a zero scale: constant offsets, no per-slot branch.
  __device__ __forceinline__ void load(uint4 *q, float *dw, int it) {
    const int r = lane & 31, h = lane >> 5;
    const int bs = b0 + h + 2 * it * U;
    const uint8_t *qp = qs + ((size_t)bs * T32 + r) * 16;  // slot u at + u * 1 KB
    const float *dp = dd + (size_t)bs * T32 + r;           // slot u at + u * 64 floats
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(qp + u * 2 * T32 * 16));
      q[u] = make_uint4(v.x, v.y, v.z, v.w);
      dw[u] = __builtin_nontemporal_load(dp + u * 2 * T32);  // zeroed past b1 in consume
    }
  }
  // xq holds the activation nibbles already XOR-ed with 8 (see act_xor)
  __device__ __forceinline__ float consume(const uint4 *q, const float *dw, int it, const uint4 *xq,
                                           const float *xd, float acc) {
    const int h = lane >> 5;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int bu = b0 + h + 2 * (it * U + u);
      const int b = min(bu, b1 - 1) - xoff;  // activation slot in LDS
      const uint4 x = xq[b];
      int s = __builtin_amdgcn_sdot8((int)(q[u].x ^ 0x88888888u), (int)x.x, 0, false);
      s = __builtin_amdgcn_sdot8((int)(q[u].y ^ 0x88888888u), (int)x.y, s, false);
      s = __builtin_amdgcn_sdot8((int)(q[u].z ^ 0x88888888u), (int)x.z, s, false);
      s = __builtin_amdgcn_sdot8((int)(q[u].w ^ 0x88888888u), (int)x.w, s, false);
      acc = __builtin_fmaf((bu < b1 ? dw[u] : 0.0f) * xd[b], (float)s, acc);
    }
    return acc;
  }
  __device__ __forceinline__ int iters() const { return (b1 - b0 + 2 * U - 1) / (2 * U); }
  __device__ __forceinline__ void prefetch() { load(qa, da, 0); }
  // runs all batches; batch 0 must have been prefetched.  One register set: with 8 waves
  // per workgroup a K = 4096 tile is one batch per wave, and the other resident workgroups
  // keep the CU's loads in flight between batches.
  __device__ __forceinline__ float run(const uint4 *xq, const float *xd) {
    const int n = iters();
    float acc = 0.0f;
    if (n <= 0) return acc;  // (small K: some waves own no block)
#pragma unroll 1
    for (int it = 0;;) {
      acc = consume(qa, da, it, xq, xd, acc);
      if (++it >= n) break;
      load(qa, da, it);
    }
    return acc;
  }
};

// Sum the per-(wave, half) partials of a tile; returns the row sum in lanes 0..31 of wave 0.
template <int NW>
__device__ __forceinline__ float tile_reduce(float acc, float (*part)[T32]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  part[2 * wave + (lane >> 5)][lane & 31] = acc;
  __syncthreads();
  float s = 0.0f;
  if (wave == 0 && lane < T32) {
#pragma unroll
    for (int i = 0; i < 2 * NW; ++i) s += part[i][lane];
  }
  return s;
}

// Stage a Q4 SoA activation slice (blocks [b0, b1)) into LDS.
// Stage a Q4 SoA activation slice (blocks [b0, b1), at most NT of them, one per thread) into
// LDS, nibbles XOR-ed with 8 (the two's-complement nibble n - 8 that v_dot8_i32_i4 reads).
// The loads are issued before the caller's weight prefetch and stored after it, so the
// vmcnt wait for them does not also wait for the weights (the counter retires in order).
struct ActStage {
  uint4 v;
  float d;
  int b;
  int b0;
  __device__ __forceinline__ void load(const uint8_t *qs, const float *dp, int b0_, int b1) {
    b0 = b0_;
    b = b0 + (int)threadIdx.x;
    if (b < b1) {
      v = *(const uint4 *)(qs + (size_t)b * 16);
      d = dp[b];
    }
  }
  __device__ __forceinline__ void store(int b1, uint4 *xq, float *xd) const {
    if (b < b1) {  // LDS slot b - b0
      xq[b - b0] = make_uint4(v.x ^ 0x88888888u, v.y ^ 0x88888888u, v.z ^ 0x88888888u, v.w ^ 0x88888888u);
      xd[b - b0] = d;
    }
  }
};

// ------------------------------------------------------------------ LayerNorm + quantize
// ggml_compute_forward_norm_f32 (ggml.c:4246-4304): mean and variance in double,
// y = (float)(x - mean) * (float)(1/sqrt(var + eps)), then w*y + b in float
// (vsim.cpp:525-532), then quantize_row_q4_0.  Fast mode takes both moments in one pass
// (var = E[x^2] - mean^2 in double: one block reduction).  LN_SPLIT workgroups per
// LayerNorm: each reads the whole row for the moments (16 KB from L2 for E = 4096) and
// normalizes and quantizes one slice of it, so the per-element phase runs on LN_SPLIT CUs.
constexpr int LN_NT = 256, LN_SPLIT = 8;
__global__ void __launch_bounds__(LN_NT) k_fast_ln(FastLn P) {
  constexpr int MAXPER = FD_MAXE / (4 * LN_NT);  // float4 per thread
  __shared__ double red[2 * (LN_NT / 64)];
  const int tid = threadIdx.x, wid = tid >> 6, E = P.E;
  const int l = blockIdx.x / LN_SPLIT, part = blockIdx.x % LN_SPLIT;
  const float *__restrict__ w = P.w[l];
  const float *__restrict__ bb = P.b[l];
  const int nb = E / QK;
  const int b0 = part * nb / LN_SPLIT, b1 = (part + 1) * nb / LN_SPLIT;  // this slice's blocks
  constexpr int MAXS = FD_MAXE / LN_SPLIT / LN_NT;  // slice elements per thread
  float xi[MAXS], wi[MAXS], bi[MAXS];
#pragma unroll
  for (int k = 0; k < MAXS; ++k) {
    const int i = b0 * QK + tid + LN_NT * k;
    const bool mine = i < b1 * QK;
    xi[k] = mine ? P.x[i] : 0.0f;
    wi[k] = mine ? w[i] : 0.0f;
    bi[k] = mine ? bb[i] : 0.0f;
  }
  double s = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < MAXPER; ++k) {
    const int e = 4 * (tid + LN_NT * k);
    if (e < E) {
      const float4 v = *(const float4 *)(P.x + e);
      s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
      s2 += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
    }
  }
  s = wave_sum_d(s);
  s2 = wave_sum_d(s2);
  if ((tid & 63) == 0) {
    red[2 * wid] = s;
    red[2 * wid + 1] = s2;
  }
  __syncthreads();
  s = 0.0;
  s2 = 0.0;
#pragma unroll
  for (int k = 0; k < LN_NT / 64; ++k) {
    s += red[2 * k];
    s2 += red[2 * k + 1];
  }
  const double mean = s / E;
  const double var = s2 / E - mean * mean;
  const float scale = (float)(1.0 / sqrt(var + (double)1e-5f));
#pragma unroll
  for (int k = 0; k < MAXS; ++k) {
    const int i0 = b0 * QK + LN_NT * k;
    if (i0 >= b1 * QK) break;
    const int i = i0 + tid;
    const bool ok = i0 + (tid & ~31) < b1 * QK;  // half-wave uniform
    const float y = ok ? wi[k] * ((float)((double)xi[k] - mean) * scale) + bi[k] : 0.0f;
    const int blk = ok ? i / QK : 0;
    fq_half(y, tid & 63, ok, (uint32_t *)(P.qs[l] + (size_t)blk * 16), P.d[l] + blk);
  }
}

// The LayerNorm of k_fast_ln in a GEMV workgroup's prologue: the residual row and the
// affine are loaded (PER float4 of each per thread) before the workgroup's first weight
// batch, the moments reduced while that batch is in flight, and the normalized row
// quantized straight into the LDS activation slots (8 lanes per 32-value block, fq_oct).
template <int NT, int PER>
struct LnStage {
  f32x4 x[PER], w[PER], b[PER];
  __device__ __forceinline__ void load(const float *lx, const float *lw, const float *lb, int E) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      int e = 4 * ((int)threadIdx.x + NT * k);
      e = e < E ? e : 0;  // (the tail's elements are masked in finish)
      x[k] = *(const f32x4 *)(lx + e);
      w[k] = *(const f32x4 *)(lw + e);
      b[k] = *(const f32x4 *)(lb + e);
    }
  }
  __device__ __forceinline__ void finish(int E, uint4 *xq, float *xd, double *red) {
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    double s = 0.0, s2 = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const f32x4 v = 4 * (tid + NT * k) < E ? x[k] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      s += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
      s2 += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
    }
    s = wave_sum_d(s);
    s2 = wave_sum_d(s2);
    if (lane == 0) {
      red[2 * wid] = s;
      red[2 * wid + 1] = s2;
    }
    __syncthreads();
    s = 0.0;
    s2 = 0.0;
#pragma unroll
    for (int k = 0; k < NT / 64; ++k) {
      s += red[2 * k];
      s2 += red[2 * k + 1];
    }
    const double mean = s / E;
    const double var = s2 / E - mean * mean;
    const float scale = (float)(1.0 / sqrt(var + (double)1e-5f));
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int f = tid + NT * k;  // float4 index; lanes 8g..8g+7 hold block f / 8
      const bool ok = 4 * f < E;   // uniform over the 8 lanes (E % 32 == 0)
      float4 y;
      y.x = w[k].x * ((float)((double)x[k].x - mean) * scale) + b[k].x;
      y.y = w[k].y * ((float)((double)x[k].y - mean) * scale) + b[k].y;
      y.z = w[k].z * ((float)((double)x[k].z - mean) * scale) + b[k].z;
      y.w = w[k].w * ((float)((double)x[k].w - mean) * scale) + b[k].w;
      const int blk = ok ? f >> 3 : 0;
      fq_oct(y, lane, ok, (uint8_t *)&xq[blk], &xd[blk], (uint16_t)0x8888);
    }
  }
};

// ------------------------------------------------------------------ GEMV batch (K1, head)
// LNP = 0: activations staged from global Q4 rows; LNP > 0: LayerNorm prologue (LnStage
// with LNP float4 per thread).
template <int NW, int LNP>
__global__ void __launch_bounds__(64 * NW, LNP > 2 ? 5 : 6) k_fast_gemv(FastGemv P) {
  __shared__ uint4 xq[FD_MAXE / QK];
  __shared__ float xd[FD_MAXE / QK];
  __shared__ float part[2 * NW][T32];
  __shared__ double red[2 * NW];
  int t = blockIdx.x, ji = 0;
  while (ji + 1 < P.nj && t >= P.j[ji].w.tiles) { t -= P.j[ji].w.tiles; ++ji; }
  const FastJob &J = P.j[ji];
  const int nb = J.w.nb();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  TileStream<> ts;
  ts.qs = J.w.qs + (size_t)t * nb * T32 * 16;
  ts.dd = J.w.d + (size_t)t * nb * T32;
  ts.b0 = wave * nb / NW;
  ts.b1 = (wave + 1) * nb / NW;
  ts.lane = lane;
  ActStage st;
  LnStage<64 * NW, LNP> ln;
  if constexpr (LNP > 0) ln.load(P.lnx, P.lnw[J.act], P.lnb[J.act], nb * QK);
  else st.load(P.xq[J.act], P.xd[J.act], 0, nb);
  const int n_past = J.epi >= FE_ROPE_Q ? *P.npast : 0;
  if (P.clear && blockIdx.x == 0)
    for (int i = threadIdx.x; i < P.nclear; i += 64 * NW) P.clear[i] = 0u;
  ts.prefetch();
  if constexpr (LNP > 0) ln.finish(nb * QK, xq, xd, red);
  else st.store(nb, xq, xd);
  __syncthreads();
  const float acc = ts.run(xq, xd);
  const float s = tile_reduce<NW>(acc, part);
  if (wave != 0) return;
  const int row = t * T32 + lane;
  if (J.epi == FE_GELU_Q) {  // fc_in rows of this tile = one 32-block of fc_out's input
    const float g = lane < T32 ? h2f(P.gelu_tab[f2h(s + J.bias[row])]) : 0.0f;
    fq_half(g, lane, lane < T32, (uint32_t *)(P.oq_qs + (size_t)t * 16), P.oq_d + t);
    return;
  }
  const float v = lane < T32 && J.bias ? s + J.bias[row] : s;
  if (J.epi == FE_STORE) {
    if (lane < T32 && row < J.w.rows) J.y[row] = v;
    return;
  }
  const size_t E = (size_t)J.w.rows;
  if (J.epi == FE_V) {
    if (lane < T32) J.y[(size_t)n_past * E + row] = v;
    return;
  }
  // RoPE at position n_past: the pair partner of head dim i is i +- n_rot/2 (style 0,
  // rotate-half; n_rot <= 32 keeps both in this tile) or i ^ 1 (style 1, GPT-J pairs)
  const int i = row % P.d, half = P.n_rot / 2;
  const bool rot = lane < T32 && i < P.n_rot;
  const int j = P.style == 0 ? (i < half ? i : i - half) : i >> 1;
  const bool first = P.style == 0 ? i < half : (i & 1) == 0;
  const int partner = P.style == 0 ? (first ? lane + half : lane - half) : lane ^ 1;
  const float pv = __shfl(v, partner & 63, 64);
  float y = v;
  if (rot) {
    const double2 c = P.cs[(size_t)n_past * half + j];
    const double x0 = first ? v : pv, x1 = first ? pv : v;
    if (P.style == 0) y = first ? (float)(c.x * x0 - c.y * x1) : (float)(c.x * x1 + c.y * x0);
    else y = first ? (float)(x0 * c.x - x1 * c.y) : (float)(x0 * c.y + x1 * c.x);
  }
  if (lane < T32) {
    if (J.epi == FE_ROPE_Q) J.y[row] = y;
    else J.y[(size_t)n_past * E + row] = y;
  }
}

// ------------------------------------------------------------------ K2: fc_out | attention
constexpr int FT_NT = 64 * FD_WAVES;
// fc_out's stream: K / sf blocks per tile over 8 waves, several batches per wave, and only
// H * nchunk + tiles * sf workgroups (about 1.5 per CU for GPT-J): more loads in flight per
// lane than K1 (which has 3 workgroups on every CU)
// (A/B on GPT-J, 64 tokens: U = 4 at 4 workgroups per CU 973 tok/s, U = 8 923)
constexpr int FT_U = 4;
constexpr int FT_OCC = 4;

// One (head, chunk) of flash-decoding attention.  Wave w takes positions p0 + 8w .. +7 of
// the chunk: its K and V rows and q are loaded at once (one round trip), one float4 of the
// head dimension per lane (d <= 256).  q is already rotated and the new position's K/V
// row already written by k_fast_gemv's epilogues.  A chunk past n_past writes m = -inf,
// l = 0, which the merge weighs by zero.
constexpr int FD_PPW = FD_CHUNK / FD_WAVES;  // positions per wave
__device__ void fast_attn_chunk(const FastTail &A, int h, int c, float *ored) {  // (partials stored sc1)
  __shared__ float pr[FD_CHUNK];
  const int d = A.d, E = A.d * A.H, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int e0 = 4 * lane;
  const bool act = e0 < d;
  const float4 q4 = act ? *(const float4 *)(A.q + h * d + e0) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int n_past = *A.npast, nk = n_past + 1;
  const int p0 = c * FD_CHUNK, p1 = min(p0 + FD_CHUNK, nk);
  float *mine = A.part + ((size_t)h * A.nchunk + c) * (d + 2);
  if (p0 >= nk) {
    if (tid == 0) {
      st_out<true>(mine, -INFINITY);
      st_out<true>(mine + 1, 0.0f);
    }
    return;
  }
  const int pw = p0 + wid * FD_PPW;
  f32x4 kv4[FD_PPW], vv4[FD_PPW];  // (clang vectors: kept in registers)
#pragma unroll
  for (int j = 0; j < FD_PPW; ++j) {
    const int p = min(pw + j, p1 - 1);
    kv4[j] = act ? *(const f32x4 *)(A.kc + (size_t)p * E + h * d + e0) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float t[FD_PPW];
#pragma unroll
  for (int j = 0; j < FD_PPW; ++j) {
    t[j] = kv4[j].x * q4.x;
    t[j] = __builtin_fmaf(kv4[j].y, q4.y, t[j]);
    t[j] = __builtin_fmaf(kv4[j].z, q4.z, t[j]);
    t[j] = __builtin_fmaf(kv4[j].w, q4.w, t[j]);
  }
  // V rows: issued once the K rows are consumed (their registers free), in flight during
  // the score reductions and the softmax
#pragma unroll
  for (int j = 0; j < FD_PPW; ++j) {
    const int p = min(pw + j, p1 - 1);
    vv4[j] = act ? *(const f32x4 *)(A.vc + (size_t)p * E + h * d + e0) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < FD_PPW; ++j) {
    const float sj = wave_sum_f(t[j]);
    if (lane == 0 && pw + j < p1) pr[pw + j - p0] = sj * A.scale;
  }
  __syncthreads();
  if (wid == 0) {  // chunk softmax: one position per lane
    const int n = p1 - p0;
    const float sc = lane < n ? pr[lane] : -INFINITY;
    const float m = wave_max_f(sc);
    const float e = lane < n ? __expf(sc - m) : 0.0f;
    const float l = wave_sum_f(e);
    pr[lane] = e;
    if (lane == 0) {
      st_out<true>(mine, m);
      st_out<true>(mine + 1, l);
    }
  }
  __syncthreads();
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < FD_PPW; ++j) {
    const float pj = pw + j < p1 ? pr[pw + j - p0] : 0.0f;
    o.x = __builtin_fmaf(pj, vv4[j].x, o.x);
    o.y = __builtin_fmaf(pj, vv4[j].y, o.y);
    o.z = __builtin_fmaf(pj, vv4[j].z, o.z);
    o.w = __builtin_fmaf(pj, vv4[j].w, o.w);
  }
  if (act) *(float4 *)(ored + wid * 256 + e0) = o;
  __syncthreads();
  for (int i = tid; i < d; i += FT_NT) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < FD_WAVES; ++w) v += ored[w * 256 + i];
    st_out<true>(mine + 2 + i, v);
  }
}

__device__ __forceinline__ void fast_fcout_part(const FastTail &A, int idx, uint4 *xq, float *xd,
                                                float (*part)[T32]);
__device__ void fast_merge_head(const FastTail &A, int h, int lane);

__global__ void __launch_bounds__(FT_NT, FT_OCC) k_fast_tail(FastTail A) {
  __shared__ uint4 xq[FD_MAXE / QK];
  __shared__ float xd[FD_MAXE / QK];
  __shared__ float part[2 * FD_WAVES][T32];
  __shared__ float ored[FD_WAVES * 256];
  __shared__ int last;
  const int na = A.H * A.nchunk;
  if ((int)blockIdx.x < na) {
    const int h = blockIdx.x / A.nchunk;
    fast_attn_chunk(A, h, blockIdx.x % A.nchunk, ored);
    // counter hand-off (cdna_hip_programming.md §6 Guideline 16): every wave drains its sc1
    // partial stores, one lane counts; the head's last chunk workgroup acquires and merges
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(A.hcnt + 4 * h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (unsigned)A.nchunk - 1;
    __syncthreads();
    if (last && threadIdx.x < 64) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      fast_merge_head(A, h, threadIdx.x);
    }
    return;
  }
  fast_fcout_part(A, blockIdx.x - na, xq, xd, part);
}

// One (tile, K split) of fc_out: partial rows into ffp[split].
__device__ __forceinline__ void fast_fcout_part(const FastTail &A, int idx, uint4 *xq, float *xd,
                                                float (*part)[T32]) {
  const int t = idx / A.sf, sp = idx % A.sf;
  const int nb = A.wf.nb();
  const int kb0 = sp * nb / A.sf, kb1 = (sp + 1) * nb / A.sf;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  TileStream<FT_U> ts;
  ts.qs = A.wf.qs + (size_t)t * nb * T32 * 16;
  ts.dd = A.wf.d + (size_t)t * nb * T32;
  ts.b0 = kb0 + wave * (kb1 - kb0) / FD_WAVES;
  ts.b1 = kb0 + (wave + 1) * (kb1 - kb0) / FD_WAVES;
  ts.lane = lane;
  ts.xoff = kb0;
  ActStage st;
  st.load(A.xf_qs, A.xf_d, kb0, kb1);
  ts.prefetch();
  st.store(kb1, xq, xd);
  __syncthreads();
  const float acc = ts.run(xq, xd);
  const float s = tile_reduce<FD_WAVES>(acc, part);
  if (wave == 0 && lane < T32) A.ffp[(size_t)sp * A.wf.rows + t * T32 + lane] = s;
}

// ------------------------------------------------------------------ attention merge
// Head h's chunks (chunk c: m = max score, l = sum e^(s - m), o = sum e^(s - m) v) into the
// attention output sum_c o_c e^(m_c - M) / sum_c l_c e^(m_c - M), quantized into the
// out-projection's Q4 input.  Run by wave 0 of the chunk workgroup that counts last for the
// head, behind one agent acquire (the partials were stored sc1).  Four consecutive outputs
// per lane, a 32-block = 8 lanes; chunks past n_past weigh zero.
constexpr int FD_MAXCH = 64;  // chunks per head (n_ctx <= 4096)
__device__ void fast_merge_head(const FastTail &A, int h, int lane) {
  const int d = A.d, nch = A.nchunk;
  const int nv = min(*A.npast / FD_CHUNK + 1, nch);  // chunks holding positions 0 .. n_past
  const float *ph = A.part + (size_t)h * nch * (d + 2);
  float M = -INFINITY;
  for (int c = 0; c < nch; ++c) M = fmaxf(M, ph[(size_t)c * (d + 2)]);
  float L = 0.0f;
  for (int c = 0; c < nch; ++c) {
    const float e = __expf(ph[(size_t)c * (d + 2)] - M);
    L = __builtin_fmaf(ph[(size_t)c * (d + 2) + 1], e, L);
  }
  const float inv = 1.0f / L;
  const int i = 4 * lane;
  const bool ok = i < d;  // 8-lane uniform (d % 32 == 0)
  float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; c < nv; ++c) {
    const float w = __expf(ph[(size_t)c * (d + 2)] - M) * inv;
    const float4 o = ok ? *(const float4 *)(ph + (size_t)c * (d + 2) + 2 + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    y.x = __builtin_fmaf(o.x, w, y.x);
    y.y = __builtin_fmaf(o.y, w, y.y);
    y.z = __builtin_fmaf(o.z, w, y.z);
    y.w = __builtin_fmaf(o.w, w, y.w);
  }
  const int blk = (h * d + (ok ? i : 0)) / QK;
  fq_oct(y, lane, ok, A.oq_qs + (size_t)blk * 16, A.oq_d + blk);
}

// Out-projection tile t and the residual join (K3).
template <int NW>
__device__ __forceinline__ void fast_oproj_tile(const FastOproj &P, int t, uint4 *xq, float *xd, float (*part)[T32]) {
  const int nb = P.w.nb(), E = P.w.rows;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  TileStream<> ts;
  ts.qs = P.w.qs + (size_t)t * nb * T32 * 16;
  ts.dd = P.w.d + (size_t)t * nb * T32;
  ts.b0 = wave * nb / NW;
  ts.b1 = (wave + 1) * nb / NW;
  ts.lane = lane;
  ActStage st;
  st.load(P.xq, P.xd, 0, nb);
  ts.prefetch();
  st.store(nb, xq, xd);
  __syncthreads();
  const float acc = ts.run(xq, xd);
  const float s = tile_reduce<NW>(acc, part);
  if (wave == 0 && lane < T32) {
    const int row = t * T32 + lane;
    float f = 0.0f;
    for (int i = 0; i < P.sf; ++i) f += P.ffp[(size_t)i * E + row];
    const float attn = P.bo ? s + P.bo[row] : s;
    P.out[row] = P.x[row] + (attn + (f + P.bproj[row]));
  }
}

__global__ void __launch_bounds__(64 * FD_OWAVES) k_fast_oproj_join(FastOproj P) {
  __shared__ uint4 xq[FD_MAXE / QK];
  __shared__ float xd[FD_MAXE / QK];
  __shared__ float part[2 * FD_OWAVES][T32];
  fast_oproj_tile<FD_OWAVES>(P, blockIdx.x, xq, xd, part);
}

// ------------------------------------------------------------------ launchers
int launch_fast_ln(const FastLn &P, hipStream_t s) {
  if (P.E > FD_MAXE || P.E % (4 * QK) != 0 || P.n < 1 || P.n > 2) {
    set_error("fast decode: n_embd must be a multiple of 128, at most 8192");
    return VSIM_EINVAL;
  }
  hipLaunchKernelGGL(k_fast_ln, dim3(P.n * LN_SPLIT), dim3(LN_NT), 0, s, P);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_fast_gemv(const FastGemv &P, int E, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < P.nj; ++i) {
    if (P.j[i].w.k != E || E > FD_MAXE || E / QK > 64 * FD_WAVES) {
      set_error("fast decode: GEMV batch K must equal n_embd (at most 8192)");
      return VSIM_EINVAL;
    }
    tiles += P.j[i].w.tiles;
  }
  const dim3 g(tiles), b(64 * FD_WAVES);
  if (!P.lnx) {
    hipLaunchKernelGGL((k_fast_gemv<FD_WAVES, 0>), g, b, 0, s, P);
  } else {
    switch ((E / 4 + 64 * FD_WAVES - 1) / (64 * FD_WAVES)) {  // float4 per thread
      case 1: hipLaunchKernelGGL((k_fast_gemv<FD_WAVES, 1>), g, b, 0, s, P); break;
      case 2: hipLaunchKernelGGL((k_fast_gemv<FD_WAVES, 2>), g, b, 0, s, P); break;
      case 3: hipLaunchKernelGGL((k_fast_gemv<FD_WAVES, 3>), g, b, 0, s, P); break;
      default: hipLaunchKernelGGL((k_fast_gemv<FD_WAVES, 4>), g, b, 0, s, P); break;
    }
  }
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_fast_tail(const FastTail &A, hipStream_t s) {
  if (A.d > 256 || A.d % QK != 0 || A.wf.k / A.sf > FD_MAXE || A.wf.nb() % A.sf != 0 ||
      A.wf.nb() / A.sf > FT_NT || A.nchunk > FD_MAXCH || !A.hcnt) {
    set_error("fast decode: unsupported head dim, fc_out split or context length");
    return VSIM_EINVAL;
  }
  const int grid = A.H * A.nchunk + A.wf.tiles * A.sf;
  hipLaunchKernelGGL(k_fast_tail, dim3(grid), dim3(FT_NT), 0, s, A);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_fast_oproj_join(const FastOproj &P, hipStream_t s) {
  if (P.w.k > FD_MAXE || P.w.nb() > 64 * FD_OWAVES || P.w.rows != P.w.k) {
    set_error("fast decode: out-projection K too large");
    return VSIM_EINVAL;
  }
  hipLaunchKernelGGL(k_fast_oproj_join, dim3(P.w.tiles), dim3(64 * FD_OWAVES), 0, s, P);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
