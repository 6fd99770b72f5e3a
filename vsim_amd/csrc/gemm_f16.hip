// vsim_amd/csrc/gemm_f16.hip — prompt (prefill) GEMM on fp16 MFMA after in-LDS dequant.
//
// Y[n][m] (+ bias[m]) = sum_k W[m][k] * X[n][k] for N prompt tokens at once, the shape of
// ggml_compute_forward_mul_mat_q4_0_f32 (ggml.c:4891-5165) with N > 1: W is the Q4_0
// weight in the W4T32 layout, X the Q4_0-quantized activation rows the reference's INIT
// phase produces (ggml.c:5024-5041; Q4 SoA here).  Both are dequantized to fp16 while
// they are staged into LDS (d*(q-8) rounded once to fp16), multiplied on
// v_mfma_f32_32x32x16_f16 and accumulated in fp32.
//
// Numerics: this is the throughput path for long prompts (codegen-16B, N = 2048); it is
// not the reference's sequential fp32 chain per (row, token), so it belongs to the fast
// mode.  Exact mode keeps the per-chain kernel for prompt batches.
//
// Tiling: one workgroup = 128 weight rows x 128 tokens, 4 waves of 64 x 64 (2 x 2 MFMA
// tiles of 32 x 32); K in steps of 64 (two Q4_0 blocks).  Staging: each of the 256 threads
// dequantizes one (row, block) unit of W and one of X per step -- 16 bytes of nibbles and
// a scale into 32 halves -- with the fp8 nibble conversion of the exact GEMV (an e4m3 byte
// n in 0..15 is n * 2^-9).  The next step's units are loaded into registers before the
// MFMAs of the current step, so their global latency hides behind the matrix work.
#include <map>
#include <mutex>

#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GM_BM = 128, GM_BN = 128, GM_BK = 64, GM_THREADS = 256;
constexpr int GM_LD = GM_BK + 8;  // halves per LDS row: 16-byte pad against bank conflicts

// 8 fp16 values d * (q - 8) of one word of a Q4_0 block (elements 8w .. 8w+7: lo b0, hi b0,
// lo b1, hi b1, ...): the nibble n as n 2^-9 from the fp8 conversion, then one fused multiply-add
// that rounds the exact d (n - 8) once, straight to fp16 (v_fma_mix_f16; the file is built
// without SLP vectorization so the scalar FMAs are not re-packed into v_pk_fma_f32 + a separate
// conversion, which would round twice).  Every fp16 weight operand of the prompt GEMMs comes
// from here: the fp16 image (k_w4_expand_f16), the in-LDS dequant, the 128-tile kernel.
__device__ __forceinline__ half8 deq_word_f16(uint32_t qw, float d) {
  const float d512 = 512.0f * d, m8 = -8.0f * d;
  const int lo = (int)(qw & 0x0F0F0F0Fu), hi = (int)((qw >> 4) & 0x0F0F0F0Fu);
  const f32x2 nl01 = __builtin_amdgcn_cvt_pk_f32_fp8(lo, false), nh01 = __builtin_amdgcn_cvt_pk_f32_fp8(hi, false);
  const f32x2 nl23 = __builtin_amdgcn_cvt_pk_f32_fp8(lo, true), nh23 = __builtin_amdgcn_cvt_pk_f32_fp8(hi, true);
  half8 h;
  h[0] = (_Float16)__builtin_fmaf(nl01.x, d512, m8);
  h[1] = (_Float16)__builtin_fmaf(nh01.x, d512, m8);
  h[2] = (_Float16)__builtin_fmaf(nl01.y, d512, m8);
  h[3] = (_Float16)__builtin_fmaf(nh01.y, d512, m8);
  h[4] = (_Float16)__builtin_fmaf(nl23.x, d512, m8);
  h[5] = (_Float16)__builtin_fmaf(nh23.x, d512, m8);
  h[6] = (_Float16)__builtin_fmaf(nl23.y, d512, m8);
  h[7] = (_Float16)__builtin_fmaf(nh23.y, d512, m8);
  return h;
}

// 32 fp16 values d * (q - 8) of one Q4_0 block (byte j: element 2j low nibble, 2j+1 high)
__device__ __forceinline__ void deq_block_f16(uint4 q, float d, half8 out[4]) {
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int w = 0; w < 4; ++w) out[w] = deq_word_f16(qw[w], d);
}

// The activation rows dequantized once per GEMM call: X16[token][K], block i = token * nb + b
// at X16 + 32 i, each value d * (q - 8) rounded once to fp16 (f16_of_product) -- the halves
// k_act_quant_f16 writes.
__global__ void __launch_bounds__(256) k_act_deq_f16(const uint8_t *__restrict__ xqs, const float *__restrict__ xdd,
                                                      size_t nblk, half8 *__restrict__ X16) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nblk) return;
  const uint4 q = *(const uint4 *)(xqs + i * 16);
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
  const float d = xdd[i];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    half8 h;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h[2 * j] = f16_of_product(d, (float)((int)((qw[w] >> (8 * j)) & 15u) - 8));
      h[2 * j + 1] = f16_of_product(d, (float)((int)((qw[w] >> (8 * j + 4)) & 15u) - 8));
    }
    X16[4 * i + w] = h;
  }
}

// Prompt activation rows straight to the GEMM's fp16 operand: (bias + GELU table,
// ggml.c:4113-4152, optional) then quantize_row_q4_0 per 32-block and the dequantized
// values d*(q-8) as fp16 — what k_q4_quantize + k_act_deq_f16 give, in one pass over the
// f32 row (which k_gelu would otherwise have read and written once more).  One value per
// lane, a half-wave per block (q4_half): coalesced 128-byte reads and 64-byte writes; each
// wave takes AQ_U block pairs with all their loads issued first (one load per lane at a time
// left the kernel latency-bound at ~1.8 TB/s).
constexpr int AQ_U = 8;
__global__ void __launch_bounds__(256) k_act_quant_f16(const float *__restrict__ x, size_t nblk, int nb,
                                                       const float *__restrict__ bias,
                                                       const uint16_t *__restrict__ gelu_tab, _Float16 *__restrict__ X16) {
  const int lane = threadIdx.x & 63;
  const size_t pair0 = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * AQ_U;
  float v[AQ_U];
#pragma unroll
  for (int u = 0; u < AQ_U; ++u) {
    const size_t blk = (pair0 + u) * 2 + (lane >> 5);
    v[u] = blk < nblk ? x[blk * QK + (lane & 31)] : 0.0f;
  }
#pragma unroll
  for (int u = 0; u < AQ_U; ++u) {
    const size_t blk = (pair0 + u) * 2 + (lane >> 5);
    const bool ok = blk < nblk;  // (uniform per half-wave)
    float t = v[u];
    if (gelu_tab && ok) {
      if (bias) t = t + bias[(int)(blk % (size_t)nb) * QK + (lane & 31)];
      t = h2f(gelu_tab[f2h(t)]);
    }
    float d;
    const int q = q4_half(t, d);
    if (ok) X16[blk * QK + (lane & 31)] = f16_of_product(d, (float)(q - 8));
  }
}

__global__ void __launch_bounds__(GM_THREADS) k_gemm_q4_f16(W4 W, const _Float16 *__restrict__ X16, int N,
                                                             const float *__restrict__ bias, float *__restrict__ Y) {
  __shared__ __attribute__((aligned(16))) _Float16 As[GM_BM * GM_LD];
  __shared__ __attribute__((aligned(16))) _Float16 Bs[GM_BN * GM_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = W.rows, nb = W.k / QK;
  const int m0 = blockIdx.x * GM_BM, n0 = blockIdx.y * GM_BN;
  // staging unit of this thread: row (of W) / token (of X) u, block ub of the K step
  const int u = tid & 127, ub = tid >> 7;
  const int mrow = m0 + u, ntok = n0 + u;
  const bool mok = mrow < M, nok = ntok < N;
  const size_t wbase = mok ? ((size_t)(mrow / T32) * nb * T32 + (mrow & (T32 - 1))) : 0;
  auto ldW = [&](int kb, uint4 &q, float &d) {  // block kb of row mrow
    const int b = kb + ub;
    if (mok && b < nb) {
      const size_t o = wbase + (size_t)b * T32;
      q = *(const uint4 *)(W.qs + o * 16);
      d = W.d[o];
    } else {
      q = make_uint4(0x88888888u, 0x88888888u, 0x88888888u, 0x88888888u);  // q = 8: value 0
      d = 0.0f;
    }
  };
  auto ldX = [&](int kb, u32x4 *xv) {  // the 32 halves of block kb + ub of token ntok
    const int b = kb + ub;
    const bool ok = nok && b < nb;
    const u32x4 *src = (const u32x4 *)(X16 + ((size_t)(ok ? ntok : 0) * nb + (ok ? b : 0)) * 32);
#pragma unroll
    for (int w = 0; w < 4; ++w) xv[w] = ok ? src[w] : u32x4{0u, 0u, 0u, 0u};
  };
  const int wm = wave & 1, wn = wave >> 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};
  uint4 qa;
  float da;
  u32x4 xb[4];
  ldW(0, qa, da);
  ldX(0, xb);
  const int r = lane & 31, h = lane >> 5;
  for (int kb = 0; kb < nb; kb += 2) {
    // dequantize this step's units into LDS
    half8 ha[4];
    deq_block_f16(qa, da, ha);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      *(half8 *)&As[u * GM_LD + ub * 32 + 8 * w] = ha[w];
      *(u32x4 *)&Bs[u * GM_LD + ub * 32 + 8 * w] = xb[w];
    }
    __syncthreads();
    // next step's units in flight during the MFMAs
    if (kb + 2 < nb) {
      ldW(kb + 2, qa, da);
      ldX(kb + 2, xb);
    }
#pragma unroll
    for (int kk = 0; kk < GM_BK / 16; ++kk) {
      half8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *(const half8 *)&As[(wm * 64 + i * 32 + r) * GM_LD + kk * 16 + 8 * h];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = *(const half8 *)&Bs[(wn * 64 + j * 32 + r) * GM_LD + kk * 16 + 8 * h];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map of 32x32 MFMA: column (token) = lane & 31, row (weight row) =
  // (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + r;
      if (n >= N) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m = m0 + wm * 64 + i * 32 + 8 * g + 4 * h;
        float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
        if (bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (m + e < M) v[e] = v[e] + bias[m + e];
        }
        float *dst = Y + (size_t)n * M + m;
        if (m + 3 < M && (M & 3) == 0) {
          *(float4 *)dst = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (m + e < M) dst[e] = v[e];
        }
      }
    }
}

// ================================================================== fp16 weight image GEMM
// Long prompts (N >= G2_MIN_N): the Q4_0 weight is expanded once into an fp16 image [M][K]
// (k_w4_expand_f16: the same halves deq_block_f16 gives), kept by the model per weight, so the
// GEMM stages both operands by LDS-DMA straight from HBM/L2 and the K loop carries no dequant.
//
// k_gemm_f16_256: one 512-thread workgroup per BM x 256 output tile, BM = 64 * AP (AP = 4:
// 256 rows, AP = 3: 192 rows, chosen per shape so the tiles fill the 256 CUs: M = 6144 at
// N = 2048 is 192 tiles of 256 rows but 256 tiles of 192), 8 waves: 2 along M x 4 along N,
// (BM/2) x 64 each, v_mfma_f32_16x16x32_f16, K in tiles of 64.  LDS: two buffers x {AP A
// pieces, 4 B pieces} of 8 KB ([64 rows][64 halves], 16-byte chunks XOR-swizzled by
// row & 7 so the 16 lanes of a ds_read_b128 group hit 16 different bank slots (and the 8 lanes
// of a ds_write_b128 group of the Q4A dequant 8 different 16-byte slots of the 32 banks); the DMA
// is lane-linear, the swizzle is on its source address).  Each K-tile is 4 phases, one output
// quadrant ((BM/4) x 32 per wave) per phase; a phase is {LDS reads, DMA issue} barrier {MFMAs}
// barrier.  The two wave groups (A rows [0, BM/2) and [BM/2, BM); one wave of each per SIMD)
// run one barrier apart, so on every SIMD one wave's MFMAs overlap the other's LDS reads
// (group 1 takes one extra barrier first, group 0 one last):
//   P1: read A rows 0..BM/4-1 of the wave's half + B cols 0-31, stage A pieces [0, AP/2) of t+1
//   P2: read B cols 32-63,                                     stage A pieces [AP/2, AP) of t+1
//   P3: read A rows BM/4..BM/2-1,                              wait for all of tile t+1 (vmcnt(0))
//   P4: (B cols 0-31 still held),                              stage the 4 B pieces of tile t+2
// With the groups a barrier apart, a piece is restaged >= 2 phases after its last read (A:
// read up to P3, restaged in P1/P2 of the next tile; B: read up to P2, restaged in P4) and read
// >= 2 phases after the wait that retires it (tile t+1 waited in P3 of tile t, first read in P1
// of tile t+1) -- cdna_hip_programming.md §5 ("read a staged buffer one phase after the wait",
// "one barrier more when two wave groups run staggered").  The DMA stays in flight across the
// raw s_barriers.  Workgroups are remapped so each XCD takes a contiguous range of tiles
// (neighbours share A rows in that XCD's L2).
constexpr int G2_BN = 256, G2_BK = 64, G2_THREADS = 512;
constexpr int G2_PIECE = 64 * G2_BK;  // halves per staged piece (8 KB)
__host__ __device__ constexpr int g2_lds_bytes(int ap) { return 2 * (ap + 4) * G2_PIECE * 2; }

__global__ void __launch_bounds__(256) k_w4_expand_f16(W4 W, half8 *__restrict__ out) {
  const int nb = W.k / QK;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // (row, block), blocks of a row adjacent
  if (i >= (size_t)W.rows * nb) return;
  const int row = (int)(i / nb), b = (int)(i % nb);
  const size_t o = ((size_t)(row / T32) * nb + b) * T32 + (row & (T32 - 1));
  half8 h[4];
  deq_block_f16(*(const uint4 *)(W.qs + o * 16), W.d[o], h);
#pragma unroll
  for (int w = 0; w < 4; ++w) out[4 * i + w] = h[w];
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// GQ: the fc_in epilogue of the next GEMM's operand instead of Y: bias + GELU table
// (ggml.c:4113-4152) + quantize_row_q4_0 per 32 consecutive rows m + the values d*(q-8) as
// fp16 into Q16[n][m] -- what k_act_quant_f16 makes of Y + bias, without Y's round trip.  A
// 32-row block of one column n sits in 4 lanes (fk = 0..3) x 8 registers of two accumulators.
// EM: the f32 epilogue's extra work (G2Epi): 0 none, 1 RoPE (+ the fp16 row copy), 2 residual
// join, 3 the fp16 transposed copy.
// Q4A: the weight operand is the W4T32 Q4_0 weight WQ itself (0.625 B per weight from HBM, no
// fp16 image): each K-tile's raw blocks are loaded into registers in P2 two tiles ahead (one
// Q4_0 block of one row per thread: 16 nibble bytes + the scale, a wave = one 32-row tile's two
// blocks, 1 KB + 256 B contiguous) and in P2 of the tile before their use dequantized with
// deq_word_f16 -- the same fp16 halves k_w4_expand_f16 writes -- into the A pieces of the LDS
// buffer, where the DMA of the image path would have put them (same swizzle, same reads).
// The epilogue of one wave's region of the prompt GEMM: MW rows from mw x 64 columns from nc0,
// acc in the 16x16 MFMA C/D map (column (token) = lane & 15, rows 4 * (lane >> 4) + reg of each
// 16 x 16 fragment).  GQ: bias + GELU + quantize into Q16 (fp16); else the f32 tile Y through
// this wave's LDS area (LDSB: the workgroup's LDS bytes, 8 waves), with the EM extra work.
// The caller has passed a barrier after its last LDS operand read; a wave may call it again
// for its next region (its own LDS writes and reads are ordered).
template <bool GQ, int EM, int MW, int LDSB, int NC = 64>
__device__ __forceinline__ void g2_epilogue(const f32x4 (&acc)[MW / 16][NC / 16], int mw, int nc0, int M, int N,
                                            const float *__restrict__ bias, float *__restrict__ Y,
                                            const uint16_t *__restrict__ gelu_tab, _Float16 *__restrict__ Q16,
                                            const G2Epi &epi, _Float16 *lds, int wave, int lane) {
  const int fr = lane & 15, fk = lane >> 4;
  if constexpr (GQ) {
    // quantized fp16 values go through LDS too (as the f32 tile below): direct stores would
    // write 32-byte pieces of 16 columns per instruction
    constexpr int LDH = MW + 8;  // LDS row stride (halves, padded)
    _Float16 *eh = lds + wave * 32 * LDH;
#pragma unroll
    for (int pass = 0; pass < NC / 32; ++pass) {
#pragma unroll
    for (int p = 0; p < MW / 32; ++p) {
      const int mb = mw + 32 * p;  // the block's first row
      float bv[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bv[e] = mb + 4 * fk + e < M ? bias[mb + 4 * fk + e] : 0.0f;
        bv[4 + e] = mb + 16 + 4 * fk + e < M ? bias[mb + 16 + 4 * fk + e] : 0.0f;
      }
#pragma unroll
      for (int j = 2 * pass; j < 2 * pass + 2; ++j) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = h2f(gelu_tab[f2h(acc[2 * p][j][e] + bv[e])]);
          v[4 + e] = h2f(gelu_tab[f2h(acc[2 * p + 1][j][e] + bv[4 + e])]);
        }
        float amax = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = amax > fabsf(v[e]) ? amax : fabsf(v[e]);
        float o = __shfl_xor(amax, 16, 64);
        amax = amax > o ? amax : o;
        o = __shfl_xor(amax, 32, 64);
        amax = amax > o ? amax : o;
        const float d = amax / 7.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        _Float16 h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = f16_of_product(d, (float)x86_round_i8(v[e] * id));
        _Float16 *row = eh + ((j & 1) * 16 + fr) * LDH + 32 * p + 4 * fk;
        *(uint2 *)row = *(const uint2 *)&h[0];
        *(uint2 *)(row + 16) = *(const uint2 *)&h[4];
      }
    }
    // (M % 32 == 0: a chunk of 8 rows is wholly in or out)
    for (int idx = lane; idx < 32 * (MW / 8); idx += 64) {
      const int nl = idx / (MW / 8), c = idx % (MW / 8);
      const int n = nc0 + 32 * pass + nl, m = mw + 8 * c;
      const uint4 v = *(const uint4 *)(eh + nl * LDH + 8 * c);
      if (n < N && m < M) *(uint4 *)(Q16 + (size_t)n * M + m) = v;
    }
    }
    return;
  }
  // The f32 tile leaves through LDS: a lane's accumulator holds 4 consecutive rows m of one
  // column n, so direct stores write 16 columns x 64 bytes per instruction; each wave instead
  // writes its (BM/2) x 64 region into its own LDS area, CP columns at a time, and stores
  // whole runs of (BM/2) floats per column (the direct stores cost 8-10 % of the GEMM).
  constexpr int LDW = MW + 4;  // LDS row stride (floats, padded)
  constexpr int CP = 8 * 32 * LDW * 4 <= LDSB ? 32 : 16;  // columns per pass
  float *ep = (float *)lds + wave * CP * LDW;
  const bool vec = (M & 3) == 0;
  constexpr int RW = MW / 4, NIT = CP * RW / 64;  // float4 chunks per column run; per lane
  static_assert(CP * RW % 64 == 0, "whole chunks per lane");
  // the epilogue's extra inputs, software-pipelined one pass ahead: pass p+1's are issued
  // before pass p's stores (Y may be epi.res, and a load behind a store it may alias waits for
  // it; pass p+1's columns are not pass p's), so only the first pass's latency is exposed
  [[maybe_unused]] f32x4 xr[2][EM == 2 ? NIT : 1], xa[2][EM == 2 ? NIT : 1];
  [[maybe_unused]] double2 cq[2][EM == 1 ? NIT : 1][2];
  auto extra = [&](int pass, int slot) {
    if constexpr (EM != 0) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int idx = lane + 64 * it, nl = idx / RW, c = idx % RW;
        const int n = nc0 + CP * pass + nl, m = mw + 4 * c;
        if (n >= N || m >= M) continue;
        if constexpr (EM == 2) {
          xr[slot][it] = *(const f32x4 *)(epi.res + (size_t)n * M + m);
          if (epi.res_a) xa[slot][it] = *(const f32x4 *)(epi.res_a + (size_t)n * M + m);
        } else {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int dd = (m + 2 * q) % epi.d;
            cq[slot][it][q] =
                dd < epi.n_rot ? epi.cs[(size_t)(epi.p0 + n) * (epi.n_rot / 2) + dd / 2] : make_double2(1.0, 0.0);
          }
        }
      }
    }
  };
  extra(0, 0);
#pragma unroll
  for (int pass = 0; pass < NC / CP; ++pass) {
    const int sl = pass & 1;
    if (pass + 1 < NC / CP) extra(pass + 1, sl ^ 1);
#pragma unroll
    for (int i = 0; i < MW / 16; ++i)
#pragma unroll
      for (int jj = 0; jj < CP / 16; ++jj)
        *(f32x4 *)(ep + (16 * jj + fr) * LDW + 16 * i + 4 * fk) = acc[i][(CP / 16) * pass + jj];
    // (a wave's own LDS writes and reads are ordered)
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = lane + 64 * it, nl = idx / RW, c = idx % RW;
      const int n = nc0 + CP * pass + nl, m = mw + 4 * c;
      f32x4 v = *(const f32x4 *)(ep + nl * LDW + 4 * c);
      if (n >= N || m >= M) continue;
      if (bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += m + e < M ? bias[m + e] : 0.0f;
      }
      if constexpr (EM == 1) {  // (the launcher guarantees M % 4 == 0 and an even d: pairs stay in the run)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          if ((m + 2 * q) % epi.d < epi.n_rot) {
            const double2 cs = cq[sl][it][q];
            const double x0 = v[2 * q], x1 = v[2 * q + 1];
            v[2 * q] = (float)(x0 * cs.x - x1 * cs.y);
            v[2 * q + 1] = (float)(x0 * cs.y + x1 * cs.x);
          }
        }
        if (epi.h16) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          *(h4 *)(epi.h16 + (size_t)(epi.p0 + n) * M + m) = (h4){(_Float16)v[0], (_Float16)v[1], (_Float16)v[2],
                                                                 (_Float16)v[3]};
        }
      }
      if constexpr (EM == 2) {
        if (epi.res_a) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = xr[sl][it][e] + (xa[sl][it][e] + v[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] + xr[sl][it][e];
        }
      }
      float *dst = Y + (size_t)n * M + m;
      if (vec && m + 3 < M) {
        *(f32x4 *)dst = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (m + e < M) dst[e] = v[e];
      }
    }
    if constexpr (EM == 3) {
      // the pass's columns again, read down the LDS region: runs of 8 columns of one row m,
      // as fp16, into row m of the transposed copy (4 lanes cover a row's 32 columns)
      constexpr int C8 = CP / 8, NT2 = MW * C8 / 64;
      static_assert(MW * C8 % 64 == 0, "whole runs per lane");
#pragma unroll
      for (int it = 0; it < NT2; ++it) {
        const int idx = lane + 64 * it, c8 = idx % C8, ml = idx / C8;
        const int m = mw + ml, nb = nc0 + CP * pass + 8 * c8;
        if (m >= M || nb >= N) continue;
        const float bm = bias ? bias[m] : 0.0f;
        half8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (_Float16)(ep[(8 * c8 + j) * LDW + ml] + bm);
        _Float16 *dst = epi.h16 + (size_t)m * epi.h16_ld;
        const int k = epi.p0 + nb;  // (keys in vt_pos order: an aligned run of 8 is two quads)
        if (nb + 8 <= N && (k & 7) == 0) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          *(h4 *)(dst + vt_pos(k)) = (h4){h[0], h[1], h[2], h[3]};
          *(h4 *)(dst + vt_pos(k + 4)) = (h4){h[4], h[5], h[6], h[7]};
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (nb + j < N) dst[vt_pos(k + j)] = h[j];
        }
      }
    }
  }
}

template <bool GQ, int AP, int EM, bool Q4A = false>
__global__ void __launch_bounds__(G2_THREADS, 1) k_gemm_f16_256(const _Float16 *__restrict__ A, int M, int K,
                                                                 const _Float16 *__restrict__ B, int N,
                                                                 const float *__restrict__ bias, float *__restrict__ Y,
                                                                 const uint16_t *__restrict__ gelu_tab,
                                                                 _Float16 *__restrict__ Q16, const G2Epi epi,
                                                                 const W4 WQ) {
  constexpr int BM = 64 * AP, MR = 2 * AP;  // tile rows; 16-row M-reps per wave
  constexpr int NPC = AP + 4;               // pieces per buffer
  extern __shared__ __attribute__((aligned(16))) _Float16 g2lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wr = wave >> 2, wc = wave & 3;
  const int tm = (M + BM - 1) / BM, tn = (N + G2_BN - 1) / G2_BN, nwg = tm * tn;
  // XCD remap (bijective): the blocks dispatched to one XCD (bid % 8) take consecutive tiles
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int m0 = (wg / tn) * BM, n0 = (wg % tn) * G2_BN;
  const int nk = K / G2_BK;
  const uint32_t lbase = lds_addr(g2lds);
  // stage piece p (A: p < AP, rows 64p..; B: p - AP) of K-tile kt into buffer kt & 1; the
  // source tile is clamped to the last one (the loads past the end fill a buffer that is not
  // read again, and keep the per-wave DMA count of every phase the same)
  auto stage = [&](int kt, int p) {
    const int kc = min(kt, nk - 1);
    const bool isA = p < AP;
    const int r = wave * 8 + (lane >> 3);        // this lane's row within the piece
    const int c = (lane & 7) ^ (r & 7);  // logical chunk stored at LDS chunk lane & 7
    const int grow = min((isA ? m0 + p * 64 : n0 + (p - AP) * 64) + r, (isA ? M : N) - 1);
    const _Float16 *g = (isA ? A : B) + (size_t)grow * K + (size_t)kc * G2_BK + 8 * c;
    glds16<false>(g, lbase + (uint32_t)((((kt & 1) * NPC + p) * G2_PIECE + wave * 8 * G2_BK) * 2));
  };
  // Q4A: this thread's unit of a K-tile: 32-row tile ut of the BM rows (its wave), block ub of
  // the tile's two, row ur of the 32 (the lane); waves past the tile's 32-row tiles take none
  const int ut = wave, ub = lane >> 5, ur = lane & 31;
  const bool qown = Q4A && ut < BM / T32;
  const int qnb = K / QK, qtiles = (M + T32 - 1) / T32;
  const int qtile = min(m0 / T32 + ut, qtiles - 1);  // clamped: the rows past M are not stored
  [[maybe_unused]] u32x4 qraw = {0u, 0u, 0u, 0u}, qraw_n = {0u, 0u, 0u, 0u};  // tile t+1's unit, tile t+2's
  [[maybe_unused]] float qd = 0.0f, qd_n = 0.0f;
  // (inline asm, like the DMA: the compiler's wait-count bookkeeping would put a vmcnt(0) in
  // front of the first use, which also waits for the B pieces staged after these loads; they
  // are retired by the explicit vmcnt(0) of P4 in the tile before their use)
  auto qload = [&](int kt, u32x4 &r, float &rd) {  // raw block (2 kt + ub) of row ur of tile qtile
    if (!qown) return;
    const size_t o = ((size_t)qtile * qnb + 2 * min(kt, nk - 1) + ub) * T32 + ur;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(WQ.qs + o * 16) : "memory");
    asm volatile("global_load_dword %0, %1, off" : "=v"(rd) : "v"(WQ.d + o) : "memory");
  };
  auto qstore = [&](int buf) {  // dequantize the unit into the A pieces of `buf`
    if (!qown) return;
    half8 h[4];
    deq_block_f16(make_uint4(qraw[0], qraw[1], qraw[2], qraw[3]), qd, h);
    const int row = ut * T32 + ur;
    _Float16 *base = g2lds + buf * NPC * G2_PIECE + row * G2_BK;
#pragma unroll
    for (int j = 0; j < 4; ++j) *(half8 *)(base + 8 * ((4 * ub + j) ^ (row & 7))) = h[j];
  };
  // one word (8 values) of the unit, stored to its chunk
  auto qstore_word = [&](int buf, int w) {
    if (!qown) return;
    const half8 h = deq_word_f16(qraw[w], qd);
    const int row = ut * T32 + ur;
    *(half8 *)(g2lds + buf * NPC * G2_PIECE + row * G2_BK + 8 * ((4 * ub + w) ^ (row & 7))) = h;
  };
  f32x4 acc[MR][4];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  half8 a[AP][2], b0[2][2], b1[2][2];
  const int fr = lane & 15, fk = lane >> 4;
  auto rd = [&](const _Float16 *base, int row, int kk) {  // fragment: 8 halves of `row` at k 8*fk + 32*kk
    const int c = kk * 4 + fk;
    return *(const half8 *)(base + row * G2_BK + 8 * (c ^ (row & 7)));
  };
  auto rdA = [&](int buf, int mh) {  // rows of the tile: wave half wr, quarter mh
    const _Float16 *bp = g2lds + buf * NPC * G2_PIECE;
#pragma unroll
    for (int i = 0; i < AP; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) a[i][kk] = rd(bp, wr * (BM / 2) + mh * (BM / 4) + i * 16 + fr, kk);
  };
  auto rdB = [&](half8 (&bb)[2][2], int buf, int nh) {
    const _Float16 *bp = g2lds + (buf * NPC + AP) * G2_PIECE;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bb[j][kk] = rd(bp, wc * 64 + (2 * nh + j) * 16 + fr, kk);
  };
  auto mma = [&](int mh, int nh, const half8 (&bb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < AP; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[AP * mh + i][2 * nh + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][kk], bb[j][kk], acc[AP * mh + i][2 * nh + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
#define G2_SYNC_MMA(MH, NH, BB)                        \
  __builtin_amdgcn_sched_barrier(0);                   \
  __builtin_amdgcn_s_barrier();                        \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
  mma(MH, NH, BB);                                     \
  __builtin_amdgcn_sched_barrier(0);
  // prologue: tile 0 whole, tile 1's B pieces in flight (as if staged in P4 of tile -1); Q4A:
  // tile 0's A dequantized, tile 1's raw blocks in registers
#pragma unroll
  for (int p = AP; p < NPC; ++p) stage(0, p);
  if constexpr (Q4A) {
    qload(0, qraw, qd);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);  // the dequant reads the loaded registers after the wait
    qstore(0);
    qload(1, qraw_n, qd_n);  // waited in P2 of tile 0
  } else {
#pragma unroll
    for (int p = 0; p < AP; ++p) stage(0, p);
  }
#pragma unroll
  for (int p = AP; p < NPC; ++p) stage(1, p);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 landed (Q4A: and tile 1's raw blocks)
  if constexpr (Q4A) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tile 0's A stores
  __builtin_amdgcn_s_barrier();
  if (wr) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
  for (int t = 0; t < nk; ++t) {
    const int cb = t & 1;
    rdA(cb, 0);
    rdB(b0, cb, 0);
    if constexpr (Q4A) {
      G2_SYNC_MMA(0, 0, b0)
    } else {
#pragma unroll
      for (int p = 0; p < AP / 2; ++p) stage(t + 1, p);
      G2_SYNC_MMA(0, 0, b0)
    }
    __builtin_amdgcn_s_barrier();
    rdB(b1, cb, 1);
    if constexpr (Q4A) {
      // tile t+1's A from its raw blocks (loaded in P2 of tile t-1), dequantized in P2 (the
      // phase with the fewest LDS reads) into buffer cb^1: writable from P1 on (its last reads
      // were P3 of tile t-1), the writes complete by the lgkmcnt(0) ending P3, before either
      // wave group's first read of it in P1 of tile t+1.  Counted wait: the oldest loads in
      // flight are tile t+1's raw blocks (2 per wave), then tile t+1's B pieces (4, P4 of tile
      // t-1), which stay in flight.  The wait names the registers, so no use of them moves above it.
      if (qown) asm volatile("s_waitcnt vmcnt(4)" : "+v"(qraw_n), "+v"(qd_n)::"memory");
      qraw = qraw_n;
      qd = qd_n;
      qload(t + 2, qraw_n, qd_n);  // waited in P2 of tile t+1
#pragma unroll
      for (int w = 0; w < 4; ++w) qstore_word(cb ^ 1, w);
      G2_SYNC_MMA(0, 1, b1)
    } else {
#pragma unroll
      for (int p = AP / 2; p < AP; ++p) stage(t + 1, p);
      G2_SYNC_MMA(0, 1, b1)
    }
    __builtin_amdgcn_s_barrier();
    rdA(cb, 1);
    if constexpr (Q4A) {
      G2_SYNC_MMA(1, 1, b1)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's A writes of tile t+1 landed
      // tile t+1's B pieces landed; tile t+2's raw blocks (the 2 newest) stay in flight
      if (qown)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      G2_SYNC_MMA(1, 1, b1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 (and tile t+1's B pieces) landed
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int p = AP; p < NPC; ++p) stage(t + 2, p);
    G2_SYNC_MMA(1, 0, b0)
    __builtin_amdgcn_s_barrier();
  }
#undef G2_SYNC_MMA
  if (!wr) __builtin_amdgcn_s_barrier();  // (pairs with group 1's last barrier)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped DMAs past the end have landed
  // C/D map of the 16x16 MFMA: column (token) = lane & 15, rows (weight rows) 4 * (lane >> 4) + reg
  __syncthreads();  // (every wave is past its last LDS operand read)
  g2_epilogue<GQ, EM, BM / 2, g2_lds_bytes(AP)>(acc, m0 + wr * (BM / 2), n0 + wc * 64, M, N, bias, Y, gelu_tab, Q16, epi,
                                              g2lds, wave, lane);
}

// ================================================================== register-dequant prompt GEMM
// k_gemm_q4r: the long-prompt GEMM with the weight operand dequantized straight into MFMA
// registers, no LDS for A.  One 512-thread workgroup per 256 x 256 output tile; wave w owns
// rows [32 w, 32 w + 32) -- one W4T32 tile, whose rows no other wave reads, so each weight
// value is dequantized once per workgroup, as in the in-LDS variant, but without its LDS
// stores (13 cycles per ds_write_b128) and the A fragment reads -- and all 256 columns.
// A fragment (16 rows x 32 K of v_mfma_f32_16x16x32_f16): lane (fr, fk) holds 8 values of row
// 16 i + fr at K offset 8 fk of block kk = word fk of that row's Q4_0 block, so a fragment is
// one dword of nibbles and one scale per lane (16 rows x 16 bytes contiguous per load).
// B (the fp16 activations): 4 pieces of 64 columns per K-tile, LDS-DMA into two buffers
// (64 KB), XOR-swizzled as in k_gemm_f16_256.  Phase p of K-tile t (4 per K-tile): read
// B piece p (8 fragments), dequantize fragment p of tile t+1, issue one B piece (piece p+2 of
// tile t+1 for p < 2, piece p-2 of tile t+2 otherwise: restaged 2 phases after its last read)
// and the raw loads of fragment p of tile t+3; barrier; 16 MFMAs (rows 2 x 16, columns of
// piece p 4 x 16, K 2 x 32); wait; barrier.  Per wave and phase: 1 DMA then 2 raw loads, so
// vmcnt(14) at the end of phase f retires the DMA of phase f-4 (read in phase f+2: one phase
// after the wait, and one barrier more for the two staggered wave groups) and every raw load
// up to phase f-5 (fragment loads are used 8 phases after their issue).  Raw loads ride in
// two register sets by tile parity (the loop takes K-tiles in pairs: K % 128 == 0).
constexpr int R_BM = 256;
constexpr int r_lds_bytes() { return 2 * 4 * G2_PIECE * 2; }

// Stream-K (sk.upw > 0, for grids of fewer tiles than CUs: the 192 tiles of every 6144-row
// codegen-16B GEMM): the grid is one workgroup per CU and workgroup b takes the K-tile pairs
// ("units") [b upw, (b + 1) upw) of the tiles laid end to end, so every CU does the same work.
// A tile split between two workgroups: the one holding its start (the lower index) computes that
// part first thing and publishes its accumulators (write-through sc1 stores in the register
// layout, drained, then an sc1 flag holding this launch's epoch); the one holding its end
// computes that part last, polls the flag (sc1), adds the partial with sc1 loads (one rounded
// add per value: partial + own, the same in every run) and runs the epilogue.  The launcher
// checks no tile has 3 pieces and sizes the grid to the device's CUs (at most one workgroup per
// CU is needed for all of them to be resident at once).  The publisher publishes before it waits
// on anything, so whatever order the workgroups are dispatched in, a waiter's publisher runs as
// soon as it has a CU.  Liveness therefore needs every workgroup of the grid resident at once:
// with the XCD remap (xcd_index, r04) a tile's publisher can have a HIGHER blockIdx than its
// finisher, so "waits only on lower-indexed, already dispatched workgroups" no longer holds, and
// the grid (hipDeviceAttributeMultiprocessorCount workgroups, one per CU by launch bounds and LDS)
// relies on the whole device being available to this process.  On a CU-masked or shared device a
// finisher can wait on an undispatched publisher; the wait is bounded (SK_SPIN_MAX sleeps, ~1 s),
// past it the per-device error counter (vsim_spin_timeouts) is bumped and the model call that
// ran the prompt fails with VSIM_ESPIN.  r04 tried a wait-free variant (the second of
// the two pieces to arrive finishes the tile, from an atomic counter): with two epilogue sites
// the kernel spilled 100-350 VGPRs (scratch traffic beside the counted vmcnt waits) and ran
// 0.5 ms slower per codegen-16B prompt (61.7 vs 61.1-61.2 ms); not kept.
// Hybrid split (PAIR launches, wg0 > 0): workgroups [0, wg0) take the whole tiles [0, wg0) (a
// full round of the CUs), the rest run the split above over the tiles from t0 = wg0 on.
struct RSk {
  int cg = 0;           // tile order: column groups of cg tile-columns (0: one group, row-major)
  int upw = 0;          // units (K-tile pairs) per workgroup; 0: one tile per workgroup
  float *ws = nullptr;  // partials: [tile - t0][wave][32 f32x4][64 lanes]
  unsigned *flags = nullptr;
  unsigned epoch = 0;
  unsigned *err = nullptr;  // bounded-wait timeouts (vsim_spin_timeouts)
  int wg0 = 0, t0 = 0;
};
constexpr unsigned SK_SPIN_MAX = 1u << 23;

// PAIR: two GEMMs of the same shape (M rows each: the Q and K projections of a long GPT-J
// prompt, both with the RoPE epilogue) in one launch.  The tile grid covers 2M rows; tiles of
// rows >= M are the second GEMM's (pr: its weight, output and epilogue).  One launch of 2x the
// tiles fills the CUs where each alone leaves some idle or needs the split.
struct RPair {
  W4 w{};
  float *y = nullptr;
  G2Epi epi{};
};

template <bool GQ, int EM, bool SK = false, bool PAIR = false>
__global__ void __launch_bounds__(G2_THREADS, 1) k_gemm_q4r(const W4 WQ, int M, int K, const _Float16 *__restrict__ B,
                                                             int N, const float *__restrict__ bias, float *__restrict__ Y,
                                                             const uint16_t *__restrict__ gelu_tab,
                                                             _Float16 *__restrict__ Q16, const G2Epi epi, const RSk sk,
                                                             const RPair pr) {
  extern __shared__ __attribute__((aligned(16))) _Float16 g2lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), wr = wave >> 2;
  const int tm = (PAIR ? 2 : 1) * ((M + R_BM - 1) / R_BM), tn = (N + G2_BN - 1) / G2_BN, nwg = tm * tn;
  const int nk = K / G2_BK, nb = K / QK;
  const uint32_t lbase = lds_addr(g2lds);
  const int fr = lane & 15, fk = lane >> 4;
  f32x4 acc[2][16];
  // K-tiles [kt0, kt0 + nkt) of the tile at (m0, n0) into acc (nkt even, >= 2)
  auto run = [&](int m0, int n0, int kt0, int nkt) __attribute__((always_inline)) {
    const bool j2 = PAIR && m0 >= M;
    const W4 WJ = j2 ? pr.w : WQ;
    if (j2) m0 -= M;
    // (the K range's offset folded into the base pointers: the loop's addressing is the whole-K one)
    const _Float16 *Bk = B + (size_t)kt0 * G2_BK;
    auto stage = [&](int kt, int q) {  // B piece q of K-tile kt into buffer kt & 1 (clamped source tile)
      const int kc = min(kt, nkt - 1);
      const int r = wave * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      const int grow = min(n0 + q * 64 + r, N - 1);
      glds16<false>(Bk + (size_t)grow * K + (size_t)kc * G2_BK + 8 * c,
                    lbase + (uint32_t)((((kt & 1) * 4 + q) * G2_PIECE + wave * 8 * G2_BK) * 2));
    };
    const int qt = min(m0 / T32 + wave, (M + T32 - 1) / T32 - 1);  // (clamped: rows past M are not stored)
    const uint8_t *qbase = WJ.qs + ((size_t)qt * nb * T32 + fr) * 16 + 4 * fk + (size_t)2 * kt0 * T32 * 16;
    const float *dbase = WJ.d + (size_t)qt * nb * T32 + fr + (size_t)2 * kt0 * T32;
    // raw fragment f = 2 i + kk of K-tile kt: word fk of block 2 kt + kk of row 16 i + fr, its scale
    auto rload = [&](int kt, int f, uint32_t &w, float &d) {
      const size_t o = (size_t)(2 * min(kt, nkt - 1) + (f & 1)) * T32 + 16 * (f >> 1);
      asm volatile("global_load_dword %0, %1, off" : "=v"(w) : "v"(qbase + o * 16) : "memory");
      asm volatile("global_load_dword %0, %1, off" : "=v"(d) : "v"(dbase + o) : "memory");
    };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    uint32_t rw[2][4];
    float rd[2][4];
    half8 a[2][4], bq[4][2];
    auto rdB = [&](int buf, int q) {
      const _Float16 *bp = g2lds + (buf * 4 + q) * G2_PIECE;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int row = 16 * jj + fr, c = kk * 4 + fk;
          bq[jj][kk] = *(const half8 *)(bp + row * G2_BK + 8 * (c ^ (row & 7)));
        }
    };
    // prologue: raw tile 0 and fragments 0-1 of tile 1, then the ops of phases -6 and -5 of the
    // loop's order; tile 0 dequantized; then phases -4 .. -1 (their raw loads reuse tile 0's set)
#pragma unroll
    for (int f = 0; f < 4; ++f) rload(0, f, rw[0][f], rd[0][f]);
    rload(1, 0, rw[1][0], rd[1][0]);
    rload(1, 1, rw[1][1], rd[1][1]);
    stage(0, 0);
    rload(1, 2, rw[1][2], rd[1][2]);
    stage(0, 1);
    rload(1, 3, rw[1][3], rd[1][3]);
    asm volatile("s_waitcnt vmcnt(10)" : "+v"(rw[0][0]), "+v"(rw[0][1]), "+v"(rw[0][2]), "+v"(rw[0][3]), "+v"(rd[0][0]),
                 "+v"(rd[0][1]), "+v"(rd[0][2]), "+v"(rd[0][3])::"memory");
#pragma unroll
    for (int f = 0; f < 4; ++f) a[0][f] = deq_word_f16(rw[0][f], rd[0][f]);
    stage(0, 2);
    rload(2, 0, rw[0][0], rd[0][0]);
    stage(0, 3);
    rload(2, 1, rw[0][1], rd[0][1]);
    stage(1, 0);
    rload(2, 2, rw[0][2], rd[0][2]);
    stage(1, 1);
    rload(2, 3, rw[0][3], rd[0][3]);
    asm volatile("s_waitcnt vmcnt(14)" : "+v"(rw[1][0])::"memory");  // B pieces 0, 1 of tile 0
    __builtin_amdgcn_s_barrier();
    if (wr) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
    // one phase: P = t & 1 (the parity of K-tile t), p = 0..3
#define R_PHASE(t, P, p)                                                                                       \
  {                                                                                                            \
    rdB(P, p);                                                                                                 \
    a[(P) ^ 1][p] = deq_word_f16(rw[(P) ^ 1][p], rd[(P) ^ 1][p]);                                              \
    stage((p) < 2 ? (t) + 1 : (t) + 2, ((p) + 2) & 3);                                                         \
    rload((t) + 3, p, rw[(P) ^ 1][p], rd[(P) ^ 1][p]);                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                                         \
    __builtin_amdgcn_s_barrier();                                                                              \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                         \
    __builtin_amdgcn_s_setprio(1);                                                                             \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                                           \
      _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                            \
        _Pragma("unroll") for (int jj = 0; jj < 4; ++jj)                                                       \
          acc[i][4 * (p) + jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[P][2 * i + kk], bq[jj][kk],          \
                                                                        acc[i][4 * (p) + jj], 0, 0, 0);        \
    __builtin_amdgcn_s_setprio(0);                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                                         \
    if ((p) < 3)                                                                                               \
      asm volatile("s_waitcnt vmcnt(14)" : "+v"(rw[(P) ^ 1][((p) + 1) & 3]), "+v"(rd[(P) ^ 1][((p) + 1) & 3])::"memory"); \
    else                                                                                                       \
      asm volatile("s_waitcnt vmcnt(14)" : "+v"(rw[P][0]), "+v"(rd[P][0])::"memory");                          \
    __builtin_amdgcn_s_barrier();                                                                              \
  }
    for (int t = 0; t < nkt; t += 2) {
      R_PHASE(t, 0, 0)
      R_PHASE(t, 0, 1)
      R_PHASE(t, 0, 2)
      R_PHASE(t, 0, 3)
      R_PHASE(t + 1, 1, 0)
      R_PHASE(t + 1, 1, 1)
      R_PHASE(t + 1, 1, 2)
      R_PHASE(t + 1, 1, 3)
    }
#undef R_PHASE
    if (!wr) __builtin_amdgcn_s_barrier();  // (pairs with group 1's last barrier)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped loads past the end have landed
    __syncthreads();
  };
  // tile t of the launch order -> its first row and column.  Column groups of sk.cg tile-columns,
  // each walked row by row, so that the tiles an XCD runs at once (a contiguous range of t, below)
  // span fewer columns: fewer activation slices streamed past the XCD's L2 per tile
  // (PAIR: every tile of the first GEMM before the second's -- M % 256 == 0 -- so the hybrid
  // split's remainder stays in the second weight)
  auto tile_at = [&](int t, int &m0, int &n0) __attribute__((always_inline)) {
    const int tmj = PAIR ? tm / 2 : tm, j = PAIR ? t / (tmj * tn) : 0;
    t -= j * tmj * tn;
    const int cg = sk.cg > 0 ? sk.cg : tn, per = tmj * cg, g = t / per, i = t - g * per;
    m0 = j * M + (i / cg) * R_BM;
    n0 = (g * cg + i % cg) * G2_BN;
  };
  // a contiguous range of `count` indices per XCD (workgroup b runs on XCD b % 8), in dispatch order
  auto xcd_index = [&](int bid, int count) __attribute__((always_inline)) {
    const int xcd = bid & 7, q8 = count >> 3, r8 = count & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  };
  auto epilogue = [&](int m0, int n0) __attribute__((always_inline)) {  // the wave's 32 rows x 256 columns
    if (PAIR && m0 >= M) {
      g2_epilogue<GQ, EM, 32, r_lds_bytes(), 256>(acc, m0 - M + 32 * wave, n0, M, N, bias, pr.y, gelu_tab, Q16, pr.epi,
                                                  g2lds, wave, lane);
    } else {
      g2_epilogue<GQ, EM, 32, r_lds_bytes(), 256>(acc, m0 + 32 * wave, n0, M, N, bias, Y, gelu_tab, Q16, epi, g2lds,
                                                  wave, lane);
    }
  };
  // one whole tile per workgroup, the first `count` tiles, XCD-remapped
  auto whole = [&](int count) __attribute__((always_inline)) {
    int m0, n0;
    tile_at(xcd_index(blockIdx.x, count), m0, n0);
    run(m0, n0, 0, nk);
    epilogue(m0, n0);
  };
  if constexpr (!SK) {
    whole(nwg);
  } else {
    if (PAIR && (int)blockIdx.x < sk.wg0) {
      whole(sk.wg0);
      return;
    }
    // [u0, u1) meets at most two tiles (the launcher checks): the end of tA (from unit aA) and
    // the start of tA + 1.  Straight-line code, no loop over pieces: values of the second piece
    // must not be hoisted above the first's K loop (the counted waits allow no spill traffic).
    const int nu = nk / 2;
    const int t0 = PAIR ? sk.t0 : 0;  // (tile indices below count from t0)
    // (split workgroups XCD-remapped like whole tiles: a tile's pieces run on one XCD; wg0 % 8 == 0)
    const int nsp = (int)gridDim.x - (PAIR ? sk.wg0 : 0);
    const int u0 = xcd_index((int)blockIdx.x - (PAIR ? sk.wg0 : 0), nsp) * sk.upw, u1 = min(u0 + sk.upw, (nwg - t0) * nu);
    const int tA = u0 / nu, aA = u0 - tA * nu, eA = min(u1 - tA * nu, nu);
    const int eB = max(u1 - (tA + 1) * nu, 0);  // units of tA + 1 from its start
    // first: the piece that starts a tile and is finished by the next workgroup (published)
    const bool pubA = aA == 0 && eA < nu, pubB = eB > 0 && eB < nu;
    if (pubA || pubB) {
      const int t = pubA ? tA : tA + 1, e = pubA ? eA : eB;
      int m0, n0;
      tile_at(t + t0, m0, n0);
      run(m0, n0, 0, 2 * e);
      float *wp = sk.ws + ((size_t)(t * 8 + wave) * 32 * 64 + lane) * 4;
      // (4 stores per base address, offsets 0-3 KB)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 16; j += 4) {
          asm volatile(
              "global_store_dwordx4 %0, %1, off sc1\n\t"
              "global_store_dwordx4 %0, %2, off offset:1024 sc1\n\t"
              "global_store_dwordx4 %0, %3, off offset:2048 sc1\n\t"
              "global_store_dwordx4 %0, %4, off offset:3072 sc1" ::"v"(wp),
              "v"(acc[i][j]), "v"(acc[i][j + 1]), "v"(acc[i][j + 2]), "v"(acc[i][j + 3])
              : "memory");
          wp += 4 * 256;
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(sk.flags + t, sk.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (pubA) return;  // (tA's start was the whole range)
    }
    // then the piece this workgroup finishes: tA from aA (after a published tA + 1 start), or
    // tA + 1 whole / tA whole
    const bool finA = !pubA;
    const int t = finA ? tA : tA + 1, a = finA ? aA : 0, e = finA ? eA : eB;
    if (!finA && e < nu) return;
    int m0, n0;
    tile_at(t + t0, m0, n0);
    run(m0, n0, 2 * a, 2 * (e - a));
    if (a > 0) {  // the earlier part's partial
      if (tid == 0) {
        unsigned spins = 0;
        while (__hip_atomic_load(sk.flags + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != sk.epoch) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins == SK_SPIN_MAX) {
            if (sk.err) __hip_atomic_fetch_add(sk.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __syncthreads();
      const float *wp = sk.ws + ((size_t)(t * 8 + wave) * 32 * 64 + lane) * 4;
#pragma unroll
      for (int g = 0; g < 8; ++g) {  // 4 registers' worth at a time (acc holds 128 VGPRs)
        f32x4 pv[4];
        asm volatile(
            "global_load_dwordx4 %0, %4, off sc1\n\t"
            "global_load_dwordx4 %1, %4, off offset:1024 sc1\n\t"
            "global_load_dwordx4 %2, %4, off offset:2048 sc1\n\t"
            "global_load_dwordx4 %3, %4, off offset:3072 sc1\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(pv[0]), "=&v"(pv[1]), "=&v"(pv[2]), "=&v"(pv[3])
            : "v"(wp)
            : "memory");
        wp += 4 * 256;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[g >> 2][4 * (g & 3) + q] = pv[q] + acc[g >> 2][4 * (g & 3) + q];
      }
    }
    epilogue(m0, n0);
  }
}

// Stream-K workspace per stream (partials + flags), grown on demand; the epoch tells one
// launch's flags from the last one's, so the flags are never cleared.
struct SkWs {
  float *ws = nullptr;
  unsigned *flags = nullptr;
  int tiles = 0;
  unsigned epoch = 0;
};
static int g_streamk = 1;  // vsim_gemm_set_streamk
int gemm_set_streamk(int on) {
  const int was = g_streamk;
  g_streamk = on ? 1 : 0;
  return was;
}

static int g_tile_cols = 4;  // vsim_gemm_set_tile_order
int gemm_set_tile_order(int cols) {
  const int was = g_tile_cols;
  g_tile_cols = cols < 0 ? 0 : cols;
  return was;
}
static int tile_cg(int tn) { return g_tile_cols > 0 && tn % g_tile_cols == 0 ? g_tile_cols : 0; }

static std::mutex g_sk_mu;
static std::map<std::pair<int, hipStream_t>, SkWs> g_sk_ws;  // (device, stream): a null stream is per device

static int device_cus();

// (a split never covers a full round of CUs: sized for one, the workspace is allocated once per
// stream and a prompt's later, larger split does not synchronize the stream to grow it)
static int sk_grow(SkWs &w, int tiles, hipStream_t s) {
  tiles = std::max(tiles, device_cus());
  if (w.tiles >= tiles) return VSIM_OK;
  if (w.ws) {
    VSIM_HIP(hipStreamSynchronize(s));
    VSIM_HIP(hipFree(w.ws));
    VSIM_HIP(hipFree(w.flags));
  }
  VSIM_HIP(hipMalloc((void **)&w.ws, (size_t)tiles * 8 * 32 * 64 * 16));
  VSIM_HIP(hipMalloc((void **)&w.flags, (size_t)tiles * sizeof(unsigned)));
  VSIM_HIP(hipMemset(w.flags, 0, (size_t)tiles * sizeof(unsigned)));
  w.tiles = tiles;
  w.epoch = 0;
  return VSIM_OK;
}

// the stream's split workspace for `tiles` split tiles (partials, flags, this launch's epoch)
static int sk_workspace(int tiles, hipStream_t s, RSk &sk) {
  int dev = 0;
  VSIM_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(g_sk_mu);
  SkWs &w = g_sk_ws[{dev, s}];
  if (int rc = sk_grow(w, tiles, s)) return rc;
  if (++w.epoch == 0) ++w.epoch;  // (0 is the cleared flag)
  sk.ws = w.ws;
  sk.flags = w.flags;
  sk.epoch = w.epoch;
  sk.err = spin_error_counter();
  return VSIM_OK;
}

static int r_attrs();

// everything a long prompt's GEMMs set up on first use, done ahead (vsim_model_reserve): the
// split workspace of (current device, s) and the kernels' LDS attributes (which also loads
// their code object)
int gemm_reserve_stream(hipStream_t s) {
  int dev = 0;
  VSIM_HIP(hipGetDevice(&dev));
  {
    std::lock_guard<std::mutex> lock(g_sk_mu);
    if (int rc = sk_grow(g_sk_ws[{dev, s}], 0, s)) return rc;
  }
  return r_attrs();
}

// frees the split workspace of (current device, s) after the stream's work (vsim_model_free)
int gemm_release_stream(hipStream_t s) {
  int dev = 0;
  VSIM_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(g_sk_mu);
  auto it = g_sk_ws.find({dev, s});
  if (it == g_sk_ws.end()) return VSIM_OK;
  VSIM_HIP(hipStreamSynchronize(s));
  VSIM_HIP(hipFree(it->second.ws));
  VSIM_HIP(hipFree(it->second.flags));
  g_sk_ws.erase(it);
  return VSIM_OK;
}

// CUs of the current device (the stream-K grid is one workgroup per CU)
static int device_cus() {
  static std::mutex mu;
  static std::map<int, int> cus;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cus.find(dev);
  if (it != cus.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cus[dev] = n;
  return n;
}

// every split tile in at most two pieces (a piece strictly inside a tile would need a third)
static bool sk_two_pieces(int tiles, int nu, int upw) {
  for (int t = 0; t < tiles; ++t) {
    const int b0 = t * nu / upw, b1 = ((t + 1) * nu - 1) / upw;
    if (b1 - b0 > 1) return false;
  }
  return true;
}

template <bool GQ, int EM>
static int r_go(const W4 &WQ, int M, int K, const void *x16, int n, const float *bias, float *y, const uint16_t *tab,
                void *q16, const G2Epi &epi, hipStream_t s) {
  const int nwg = ((M + R_BM - 1) / R_BM) * ((n + G2_BN - 1) / G2_BN);
  RSk sk;
  sk.cg = tile_cg((n + G2_BN - 1) / G2_BN);
  int grid = nwg;
  const int nu = K / G2_BK / 2;
  // (grids of at least half the CUs: each tile in at most two pieces.  GPT-J-6B's 128-tile
  // GEMMs at N = 2048: prompt 32.5 -> 28.5 ms, profiles/r03_streamk_half_grid_ab.jsonl)
  // (the V^T-copy epilogue only below 3/4: at codegen-16B's 192 tiles 167.0 vs 160.9 us with the split)
  const int cus = device_cus();
  if (g_streamk && !GQ && (EM != 3 || nwg * 4 < cus * 3) && nwg < cus && nwg * 2 >= cus && nu >= 2) {
    const int upw = (nwg * nu + cus - 1) / cus;
    if (sk_two_pieces(nwg, nu, upw)) {
      if (int rc = sk_workspace(nwg, s, sk)) return rc;
      sk.upw = upw;
      grid = (nwg * nu + upw - 1) / upw;
    }
  }
  if constexpr (!GQ) {
    if (sk.upw) {
      hipLaunchKernelGGL((k_gemm_q4r<GQ, EM, true>), dim3(grid), dim3(G2_THREADS), r_lds_bytes(), s, WQ, M, K,
                         (const _Float16 *)x16, n, bias, y, tab, (_Float16 *)q16, epi, sk, RPair{});
      return VSIM_OK;
    }
  }
  hipLaunchKernelGGL((k_gemm_q4r<GQ, EM>), dim3(grid), dim3(G2_THREADS), r_lds_bytes(), s, WQ, M, K, (const _Float16 *)x16,
                     n, bias, y, tab, (_Float16 *)q16, epi, sk, RPair{});
  return VSIM_OK;
}

// the LDS attribute of every k_gemm_q4r instance, once per process
static int r_attrs() {
  static std::once_flag once;
  static int rc = VSIM_OK;
  std::call_once(once, [] {
    const void *fns[] = {(const void *)k_gemm_q4r<false, 0>,          (const void *)k_gemm_q4r<false, 1>,
                         (const void *)k_gemm_q4r<false, 2>,          (const void *)k_gemm_q4r<false, 3>,
                         (const void *)k_gemm_q4r<true, 0>,           (const void *)k_gemm_q4r<false, 0, true>,
                         (const void *)k_gemm_q4r<false, 1, true>,    (const void *)k_gemm_q4r<false, 2, true>,
                         (const void *)k_gemm_q4r<false, 3, true>,    (const void *)k_gemm_q4r<false, 1, false, true>,
                         (const void *)k_gemm_q4r<false, 1, true, true>};
    for (const void *f : fns)
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, r_lds_bytes()) != hipSuccess) {
        set_error("k_gemm_q4r: LDS attribute refused");
        rc = VSIM_EHIP;
      }
  });
  return rc;
}

static int r_launch(const W4 &WQ, int M, int K, const void *x16, int n, const float *bias, float *y, hipStream_t s,
                    const uint16_t *tab, void *q16, const G2Epi &epi) {
  if (int rc = r_attrs()) return rc;
  int rc;
  if (q16) rc = r_go<true, 0>(WQ, M, K, x16, n, bias, y, tab, q16, epi, s);
  else if (epi.cs) rc = r_go<false, 1>(WQ, M, K, x16, n, bias, y, tab, q16, epi, s);
  else if (epi.res) rc = r_go<false, 2>(WQ, M, K, x16, n, bias, y, tab, q16, epi, s);
  else if (epi.h16) rc = r_go<false, 3>(WQ, M, K, x16, n, bias, y, tab, q16, epi, s);
  else rc = r_go<false, 0>(WQ, M, K, x16, n, bias, y, tab, q16, epi, s);
  if (rc) return rc;
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_w4_expand_f16(const W4 &W, void *out, hipStream_t s) {
  const size_t n = (size_t)W.rows * (W.k / QK);
  hipLaunchKernelGGL(k_w4_expand_f16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, (half8 *)out);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// The Q and K projections of a long GPT-J prompt in one launch (RPair): two W4 weights of the
// same M x K, both with the RoPE epilogue, no bias.  2 x 192 tiles for codegen-16B (E = 6144,
// N = 2048): one full round of 256 whole tiles, then the other 128 split in halves over 256
// workgroups (hybrid split); 2 x 128 for GPT-J-6B: exactly one round.
static bool r_use(int K);
static int g_qk_pair = 1;  // vsim_gemm_set_qk_pair: 0 off, 1 with the hybrid split, 2 whole tiles only
int gemm_set_qk_pair(int mode) {
  const int was = g_qk_pair;
  g_qk_pair = mode < 0 || mode > 2 ? 1 : mode;
  return was;
}

bool gemm_pair_enabled(int M, int K) { return g_qk_pair && M % R_BM == 0 && r_use(K); }

int launch_gemm_q4_256_pair(const W4 &W0, const W4 &W1, const void *x16, int n, float *y0, float *y1, const G2Epi &e0,
                            const G2Epi &e1, hipStream_t s) {
  const int M = W0.rows, K = W0.k;
  if (W1.rows != M || W1.k != K || M % R_BM || !r_use(K) || n <= 0 || !e0.cs || !e1.cs || e0.res || e1.res ||
      (e0.h16 && e0.h16_t) || (e1.h16 && e1.h16_t) || e0.d <= 0 || e0.d % 2 || e0.n_rot % 2 || e0.n_rot > e0.d ||
      e1.d != e0.d || e1.n_rot != e0.n_rot) {
    set_error("gemm pair: two M x K weights (M % 256 == 0, K % 128 == 0) with RoPE epilogues of one head shape");
    return VSIM_EINVAL;
  }
  if (int rc = r_attrs()) return rc;
  RPair pr;
  pr.w = W1;
  pr.y = y1;
  pr.epi = e1;
  const int nwg = 2 * (M / R_BM) * ((n + G2_BN - 1) / G2_BN), nu = K / G2_BK / 2;
  RSk sk;
  sk.cg = tile_cg((n + G2_BN - 1) / G2_BN);
  // hybrid split: the whole rounds as whole tiles, the remainder split over one round of CUs
  const int cus = device_cus();
  const int wg0 = nwg / cus * cus, rest = nwg - wg0;
  if (g_streamk && g_qk_pair == 1 && wg0 > 0 && rest > 0 && nu >= 2) {
    const int upw = (rest * nu + cus - 1) / cus;
    if (upw < nu && sk_two_pieces(rest, nu, upw)) {
      if (int rc = sk_workspace(rest, s, sk)) return rc;
      sk.upw = upw;
      sk.wg0 = wg0;
      sk.t0 = wg0;
      const int grid = wg0 + (rest * nu + upw - 1) / upw;
      hipLaunchKernelGGL((k_gemm_q4r<false, 1, true, true>), dim3(grid), dim3(G2_THREADS), r_lds_bytes(), s, W0, M, K,
                         (const _Float16 *)x16, n, nullptr, y0, nullptr, nullptr, e0, sk, pr);
      VSIM_HIP(hipGetLastError());
      return VSIM_OK;
    }
  }
  hipLaunchKernelGGL((k_gemm_q4r<false, 1, false, true>), dim3(nwg), dim3(G2_THREADS), r_lds_bytes(), s, W0, M, K,
                     (const _Float16 *)x16, n, nullptr, y0, nullptr, nullptr, e0, sk, pr);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// AP (tile height 64 * AP): the one of 3 and 4 whose tiles fill the CUs in fewer
// tile-height-weighted rounds (ties: 4)
static int g2_ap(int M, int n) {
  const int cus = 256;
  auto cost = [&](int ap) {
    const long tiles = (long)((M + 64 * ap - 1) / (64 * ap)) * ((n + G2_BN - 1) / G2_BN);
    return ((tiles + cus - 1) / cus) * ap;
  };
  return cost(3) < cost(4) ? 3 : 4;
}

template <int AP, bool Q4A>
static int g2_launch(const void *A16, const W4 &WQ, int M, int K, const void *x16, int n, const float *bias, float *y,
                     hipStream_t s, const uint16_t *tab, void *q16, const G2Epi &epi) {
  static bool attr = false;
  if (!attr) {
    const void *fns[] = {(const void *)k_gemm_f16_256<false, AP, 0, Q4A>, (const void *)k_gemm_f16_256<false, AP, 1, Q4A>,
                         (const void *)k_gemm_f16_256<false, AP, 2, Q4A>, (const void *)k_gemm_f16_256<false, AP, 3, Q4A>,
                         (const void *)k_gemm_f16_256<true, AP, 0, Q4A>};
    for (const void *f : fns)
      VSIM_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, g2_lds_bytes(AP)));
    attr = true;
  }
  const int nwg = ((M + 64 * AP - 1) / (64 * AP)) * ((n + G2_BN - 1) / G2_BN);
#define G2_GO(GQ, EM, TAB, Q)                                                                              \
  hipLaunchKernelGGL((k_gemm_f16_256<GQ, AP, EM, Q4A>), dim3(nwg), dim3(G2_THREADS), g2_lds_bytes(AP), s, \
                     (const _Float16 *)A16, M, K, (const _Float16 *)x16, n, bias, y, TAB, (_Float16 *)Q, epi, WQ)
  if (q16) G2_GO(true, 0, tab, q16);
  else if (epi.cs) G2_GO(false, 1, nullptr, nullptr);
  else if (epi.res) G2_GO(false, 2, nullptr, nullptr);
  else if (epi.h16) G2_GO(false, 3, nullptr, nullptr);
  else G2_GO(false, 0, nullptr, nullptr);
#undef G2_GO
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

static int g2_checked(const void *A16, const W4 *WQ, int M, int K, const void *x16, int n, const float *bias, float *y,
                      hipStream_t s, void *q16, const G2Epi *epi);

int launch_gemm_f16_256(const void *A16, int M, int K, const void *x16, int n, const float *bias, float *y,
                        hipStream_t s, void *q16, const G2Epi *epi) {
  return g2_checked(A16, nullptr, M, K, x16, n, bias, y, s, q16, epi);
}

int launch_gemm_q4_256(const W4 &W, const void *x16, int n, const float *bias, float *y, hipStream_t s, void *q16,
                       const G2Epi *epi) {
  return g2_checked(nullptr, &W, W.rows, W.k, x16, n, bias, y, s, q16, epi);
}

// the register-dequant kernel for every Q4_0 weight with K % 128 == 0 (the in-LDS dequant
// kernel for the rest).  Measured at the codegen-16B shapes (N = 2048,
// tools/gemm_bench.py): 24576 x 6144 941 -> 964-972 TFLOP/s, 6144 x 24576 893-898 -> 916,
// 6144 x 6144 803 -> 811-824 even though its 192 tiles of 256 rows leave 64 CUs idle (the
// in-LDS kernel's 256 tiles of 192 rows fill them).
static bool r_use(int K) { return K % (2 * G2_BK) == 0; }

static int g2_checked(const void *A16, const W4 *WQ, int M, int K, const void *x16, int n, const float *bias, float *y,
                      hipStream_t s, void *q16, const G2Epi *epi) {
  if (K % G2_BK || K <= 0 || M <= 0 || n <= 0 || (q16 && (M % QK || !bias))) {
    set_error("f16 gemm: K must be a positive multiple of 64 (and M of 32, with a bias, for the GELU epilogue)");
    return VSIM_EINVAL;
  }
  const G2Epi e = epi ? *epi : G2Epi{};
  if ((e.cs || e.res || e.h16) && (q16 || M % 4 || (e.cs && (e.d <= 0 || e.d % 2 || e.n_rot % 2 || e.n_rot > e.d)))) {
    set_error("f16 gemm: RoPE / residual / copy epilogue needs M % 4 == 0, even d >= n_rot, no GELU epilogue");
    return VSIM_EINVAL;
  }
  if (e.h16 && (e.res || (e.cs ? e.h16_t != 0 : (e.h16_t == 0 || e.h16_ld < e.p0 + n)))) {
    set_error("f16 gemm: the fp16 copy is row-major with RoPE, transposed (h16_ld >= p0 + n) without");
    return VSIM_EINVAL;
  }
  const uint16_t *tab = nullptr;
  if (q16) {
    DevTables t;
    if (int rc = tables_get(&t)) return rc;
    tab = t.gelu_f16;
  }
  if (WQ && r_use(K)) return r_launch(*WQ, M, K, x16, n, bias, y, s, tab, q16, e);
  if (WQ) {
    return g2_ap(M, n) == 3 ? g2_launch<3, true>(nullptr, *WQ, M, K, x16, n, bias, y, s, tab, q16, e)
                            : g2_launch<4, true>(nullptr, *WQ, M, K, x16, n, bias, y, s, tab, q16, e);
  }
  const W4 none{};
  return g2_ap(M, n) == 3 ? g2_launch<3, false>(A16, none, M, K, x16, n, bias, y, s, tab, q16, e)
                          : g2_launch<4, false>(A16, none, M, K, x16, n, bias, y, s, tab, q16, e);
}

int launch_act_quant_f16(const float *x, int K, int n, const float *bias, bool gelu, void *x16, hipStream_t s) {
  if (K % QK || n <= 0) {
    set_error("act_quant_f16: K must be a multiple of 32");
    return VSIM_EINVAL;
  }
  const uint16_t *tab = nullptr;
  if (gelu) {
    DevTables t;
    if (int rc = tables_get(&t)) return rc;
    tab = t.gelu_f16;
  }
  const size_t nblk = (size_t)n * (K / QK);
  const size_t per_wg = 4 * 2 * AQ_U;  // blocks per workgroup
  hipLaunchKernelGGL(k_act_quant_f16, dim3((unsigned)((nblk + per_wg - 1) / per_wg)), dim3(256), 0, s, x, nblk, K / QK, bias, tab,
                     (_Float16 *)x16);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_gemm_f16x(const W4 &W, const void *x16, int n, const float *bias, float *y, hipStream_t s) {
  if (W.k % QK) {
    set_error("q4 gemm: K must be a multiple of 32");
    return VSIM_EINVAL;
  }
  const dim3 grid((W.rows + GM_BM - 1) / GM_BM, (n + GM_BN - 1) / GM_BN);
  hipLaunchKernelGGL(k_gemm_q4_f16, grid, dim3(GM_THREADS), 0, s, W, (const _Float16 *)x16, n, bias, y);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_gemm_q4_f16(const W4 &W, const void *xq, int n, const float *bias, float *y, hipStream_t s) {
  if (W.k % QK) {
    set_error("q4 gemm: K must be a multiple of 32");
    return VSIM_EINVAL;
  }
  const size_t nbk = (size_t)n * (W.k / QK);
  const uint8_t *xqs = (const uint8_t *)xq;
  const float *xdd = (const float *)(xqs + nbk * 16);
  _Float16 *x16 = nullptr;
  VSIM_HIP(hipMallocAsync((void **)&x16, nbk * QK * sizeof(_Float16), s));
  hipLaunchKernelGGL(k_act_deq_f16, dim3((unsigned)((nbk + 255) / 256)), dim3(256), 0, s, xqs, xdd, nbk, (half8 *)x16);
  const dim3 grid((W.rows + GM_BM - 1) / GM_BM, (n + GM_BN - 1) / GM_BN);
  hipLaunchKernelGGL(k_gemm_q4_f16, grid, dim3(GM_THREADS), 0, s, W, x16, n, bias, y);
  VSIM_HIP(hipGetLastError());
  VSIM_HIP(hipFreeAsync(x16, s));
  return VSIM_OK;
}

}  // namespace vsim
