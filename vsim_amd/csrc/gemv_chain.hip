// vsim_amd/csrc/gemv_chain.hip — exact-mode Q4_0 GEMV (decode, one activation row).
//
// The reference dot (imax.c:1182-1230 / ggml.c:472-511) is one sequential fp32 chain per
// output row: sumf += f0*f2 + f1*f3 over the K/2 bytes of the row, every product and sum
// rounded separately.  The chain cannot be re-associated without changing the result, so
// the kernel is bounded by the dependent-add latency of the chain (one chain per lane), not
// by HBM: K = 16384 is 8192 dependent adds.  Every other cost is arranged to hide behind
// that chain.  Producer / consumer split inside a workgroup:
//
//  * the consumer wave runs the chains, one per lane: a lane reads its row's pair terms
//    from LDS (16-byte reads, a window ahead of the adds) and adds them in order;
//  * producer waves compute the pair terms of one Q4_0 block each (16 pairs, one per byte)
//    for the workgroup's rows into a 3-slot LDS ring, one s_barrier per chunk: in iteration
//    k producers fill chunk k while the consumer adds chunk k-2 (and reads ahead into k-1).
//
// Shapes: k_gemv_solo (64 rows per workgroup, the consumer alone on SIMD0, six producers on
// SIMD1-3, for batches with many rows), chain32_body (k_gemv_chain32: one 32-row tile per
// workgroup, for batches with few rows) and chain32_nb_body (the GEMV roles of k_layer_tail:
// 32-row tiles with a barrier-free hand-off and a pair-lane consumer, r05).
// Epilogues: plain store (+bias), and fc_in's bias + GELU table + re-quantization of the
// outputs into the next product's Q4_0 activation blocks (ggml.c:5024-5041).
#include <cstdlib>
#include <cstring>

// VSIM_NB_STAMPS (a diagnostic build, tools/build_variant.sh): per-workgroup s_memtime sums of
// where the barrier-free GEMVs' waves wait, an s_memrealtime timeline of the layer tail's roles
// and the attention heads' phases, read back by vsim_debug_nb_stamps (tools/nb_stamps.py)
#ifdef VSIM_NB_STAMPS
namespace vsim {
__device__ unsigned long long g_nb_stamps[2048][32];
}
#define ATT_STAMP(i) \
  if (threadIdx.x == 0) g_nb_stamps[1536 + blockIdx.x][4 + (i)] = __builtin_amdgcn_s_memrealtime()
#endif
#include "attn.hpp"
#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

typedef const __attribute__((address_space(4))) float sfloat;  // scalar-loaded
typedef const __attribute__((address_space(1))) u32x4 gu32x4;  // global, for nontemporal loads
typedef const __attribute__((address_space(1))) float gfloat;

// Producer-side barrier without the lgkmcnt(0) of __syncthreads: it would also wait for the
// scalar loads of the next chunk's activation factors still in flight.  The pair terms
// written before it are first read by the consumer one whole chunk later (it reads chunk
// k-1 near the end of iteration k), and the slot reuse is guarded by the consumer's own
// full wait before its barrier.  The "memory" clobber keeps the compiler from moving the
// stores across.
__device__ __forceinline__ void producer_barrier() { asm volatile("s_barrier" ::: "memory"); }


// ================================================================== 32-row variant
// Same chain and producer/consumer protocol for one W4T32 tile (32 rows) per workgroup, so a
// job with few rows spreads over more CUs (fc_out: 128 workgroups instead of 64) and each
// CU's producers carry half the work.  Producer waves take 2 blocks of the chunk each (lanes
// 0-31: rows of block 2p, lanes 32-63: rows of block 2p+1); the activation factors then differ
// between the two half-waves, so they come through the LDS ring as well (LDS-DMA of 1 KB pieces
// per chunk by the first producers, read with per-half broadcast loads) instead of scalar loads.
// Shapes (C2Shape): k_gemv_chain32: 8-block chunks, 4 producers, the fourth (wave 4) on the
// consumer's SIMD, LDS-DMA depth 4; k_layer_tail: 16-block chunks, 8 producers, FILL (the
// consumer's SIMD left to the consumer: waves 4, 8 only join the barriers), depth 4.  r04 per-chunk s_memtime stamps of the
// tail's fc_out tiles (tools/variants/mk_tail_stamps.py, profiles/r04_tail_stamps*.txt): a step of
// ~1,600 cycles, the consumer's 128 adds 1,308 of them (10.2 cycles per add against the 4.63 of a
// dependent add alone); with 12-block chunks, 6 producers and the consumer alone on SIMD0 still
// 9.4 per add (the producers then waited 830-880 cycles a step at the barrier) and the tail 41.4
// vs 38.8 us: the consumer loop itself, not the producer beside it, set the step.  Its LDS reads
// issued one per 4 adds cost that; issued in groups of 4 after 16 adds (one lgkmcnt wait per
// group), the tail took 36.3 vs 39.0 us (574-576 vs 550-551 tok/s; groups of 8 the same).
// s_waitcnt vmcnt(n) alone (expcnt, lgkmcnt at their maxima): n's low 4 bits in [3:0], high 2 in [15:14]
constexpr int waitcnt_vm(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }
// waves for NPW producers when the waves on the consumer's SIMD (4, 8, ...) are left idle
constexpr int c2_waves(int npw, bool fill) {
  int w = 1, p = 0;
  while (p < npw) p += (!fill || w % 4 != 0) ? 1 : 0, ++w;
  return w;
}
template <int CB_, int DEPTH_, bool FILL_, int PAD_ = 4>
struct C2Shape {
  // PAD: row pad of the pair-term ring in floats (LD = CP + PAD); 8 for the pair-lane consumer
  // (chain32_nb_body): rows 8 banks apart, so the 32-byte row pieces of one 16-byte read per lane
  // pair and the producers' 16-byte stores are both conflict-free
  static constexpr int CB = CB_, CP = CB * 16, LD = CP + PAD_, NPW = CB / 2, DEPTH = DEPTH_;
  static constexpr bool FILL = FILL_;
  static constexpr int THREADS = 64 * c2_waves(NPW, FILL);
  static constexpr int XP = (CB + 7) / 8;  // 1 KB factor pieces per chunk (8 blocks each)
  static_assert(CB % 2 == 0 && XP <= NPW && CP / 4 % 16 == 0, "chunk shape");
};
constexpr int C2_RING = 3, C2_WIN = 16;
// DEPTH: chunks of weights and factors in flight by LDS-DMA (and raw LDS slots).  r04 A/B of the
// 8-block tail (tools/tail_ab.sh): tail 38.9-39.0 us at 8 vs 39.7-39.8 at 4, 40.1-40.2 at 6,
// 40.3-40.4 at 10.  k_gemv_chain32 keeps 4, so two workgroups still fit a CU.
// The tail (r04, after the fence-free hand-off and the grouped consumer reads): 16-block chunks,
// eight producers on SIMD1-3 (11 waves), the consumer alone on SIMD0, 4 chunks ahead: 33.8-34.2
// us per tail, 601.2-604.6 tok/s at 248 tokens, against 12-block chunks 35.1 (591.8-592.8) and
// the 8-block shape with wave 4 producing beside the consumer 36.0-36.3 (581.4-582.7); 3 chunks
// ahead 34.8-34.9 (profiles/r04_tail_consumer_ab.txt)
// r05, the barrier-free tail (chain32_nb_body only): rows padded to 8 banks for the pair-lane
// consumer, four pair-term slots (NB_RING) and the LDS-DMA two chunks ahead, which is what the
// LDS holds beside them (profiles/r05_tail_consumer_pairlane.txt)
using C2Gemv = C2Shape<8, 4, false>;
using C2Tail = C2Shape<16, 2, true, 8>;

template <class S>
struct C2Lds {
  float P[C2_RING][32 * S::LD];
  uint4 RQ[S::DEPTH][S::NPW][64];
  float RD[S::DEPTH][S::NPW][64];
  float RX[S::DEPTH][S::XP * 8 * QK];
};

// tile t of the batch's jobs (blockIdx.x in k_gemv_chain32, a role offset in k_layer_tail)
template <class S>
__device__ __forceinline__ void chain32_body(const GemvBatch &B, int t, C2Lds<S> &L) {
  constexpr int DEPTH = S::DEPTH, CB = S::CB, CP = S::CP, LD = S::LD;
  constexpr int C2_RAW = DEPTH;  // raw slot reuse: see below
  constexpr int C2_WAIT_VM3 = waitcnt_vm(3 * (DEPTH - 2));  // factor-piece producers: nibbles, scales, factors
  constexpr int C2_WAIT_VM2 = waitcnt_vm(2 * (DEPTH - 2));  // other producers: nibbles, scales
  static_assert(3 * (DEPTH - 2) < 64, "vmcnt immediate");
  auto &P = L.P;
  auto &RQ = L.RQ;
  auto &RD = L.RD;
  auto &RX = L.RX;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int ji = 0;
  while (ji < B.nj) {
    if (t < B.j[ji].w.tiles) break;
    t -= B.j[ji].w.tiles;
    ++ji;
  }
  if (ji >= B.nj) return;
  ji = __builtin_amdgcn_readfirstlane(ji);
  const int nb = B.j[ji].w.k / QK, nch = (nb + CB - 1) / CB;
  const int nit = (nch + 2 + 1) & ~1;
  const uint8_t *tqs = B.j[ji].w.qs + (size_t)t * nb * T32 * 16;
  const float *td = B.j[ji].w.d + (size_t)t * nb * T32;
  const float *x = B.j[ji].xd;

  if (S::FILL && wave > 0 && wave % 4 == 0) {  // the consumer's SIMD: barriers only
    for (int k = 0; k < nit + 2; ++k) __syncthreads();
    return;
  }
  if (wave > 0) {
    // ------------------------------------------------------------- producer
    // Step k: read chunk k+1's raw block and factors (landed before the
    // previous barrier) into registers, LDS-DMA of chunk k+DEPTH, pair terms of chunk k from
    // the registers filled in step k-1, wait for this wave's DMA of chunk k+2, barrier.
    // Raw slot reuse: chunk c lives in slot c % RAW; the DMA of chunk k+DEPTH (step k) reuses
    // the slot of chunk k, whose registers were read in step k-1 (retired at that barrier).
    const int p = S::FILL ? wave - 1 - wave / 4 : wave - 1, r = lane & 31, hb = lane >> 5;
    const int o = 2 * p + hb;  // this lane's block within the chunk
    const bool xp = p < S::XP;  // this wave also brings a 1 KB piece of the chunk's factors
    const uint8_t *qs = tqs + (size_t)r * 16;
    const float *dd = td + r;
    auto dma = [&](int c) {
      const int slot = c % C2_RAW;
      const int b = min(c * CB + o, nb - 1);
      glds16(qs + (size_t)b * (T32 * 16), lds_addr(&RQ[slot][p][0]));
      glds4(dd + (size_t)b * T32, lds_addr(&RD[slot][p][0]));
      if (xp) {  // 8 blocks x 32 factors, 16 bytes per lane (clamped block)
        const int bx = min(c * CB + 8 * p + (lane >> 3), nb - 1);
        glds16_sc1(x + (size_t)bx * QK + 4 * (lane & 7), lds_addr(&RX[slot][256 * p]));
      }
    };
    auto ldraw = [&](int c, uint4 &q, float &dq, f32x2 *xv) {
      const int slot = c % C2_RAW;
      q = RQ[slot][p][lane];
      dq = RD[slot][p][lane];
      const float4 *xq = (const float4 *)&RX[slot][o * QK];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 v = xq[i];
        xv[2 * i].x = v.x;
        xv[2 * i].y = v.y;
        xv[2 * i + 1].x = v.z;
        xv[2 * i + 1].y = v.w;
      }
    };
    int ps = 0;
    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const uint4 &qc, float dqc, uint4 &qn, float &dqn) {
      ldraw(k + 1, qn, dqn, xn);
      dma(k + DEPTH);
      {
        const float dv = k * CB + o < nb ? dqc : 0.0f;
        const f32x2 d2 = {512.0f * dv, 512.0f * dv}, m2 = {-8.0f * dv, -8.0f * dv};
        float *dst = &P[ps][r * LD + o * 16];
        const uint32_t qw[4] = {qc.x, qc.y, qc.z, qc.w};
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          float p4[4];
          pair_terms4_x(qw[wv], d2, m2, xc + 4 * wv, p4);
          *(float4 *)(dst + 4 * wv) = make_float4(p4[0], p4[1], p4[2], p4[3]);
        }
      }
      ps = ps == C2_RING - 1 ? 0 : ps + 1;
      if (xp)  // this wave's DMA of chunk k+2 landed
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM3);
      else
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM2);
      __syncthreads();
    };
#pragma unroll
    for (int c = 0; c < DEPTH; ++c) dma(c);
    f32x2 xa[16], xb[16];
    uint4 qa, qb;
    float da, db;
    if (xp)  // chunks 0 and 1 landed
      __builtin_amdgcn_s_waitcnt(C2_WAIT_VM3);
    else
      __builtin_amdgcn_s_waitcnt(C2_WAIT_VM2);
    __syncthreads();
    ldraw(0, qa, da, xa);
    __syncthreads();
    for (int k = 0; k < nit; k += 2) {
      step(k, xa, xb, qa, da, qb, db);
      step(k + 1, xb, xa, qb, db, qa, da);
    }
    return;
  }

  // --------------------------------------------------------------- consumer (lanes 0-31)
  float acc = 0.0f;
  float4 win[C2_WIN];
  const int lr = lane & 31;
  auto src = [&](int c) { return &P[c % C2_RING][lr * LD]; };
  __builtin_amdgcn_s_setprio(3);
  __syncthreads();
  __syncthreads();
  for (int k = 0; k < nit; ++k) {
    const int c = k - 2;
    if (c == -1 && nch > 0) {
      const float *p0 = src(0);
#pragma unroll
      for (int j = 0; j < C2_WIN; ++j) win[j] = *(const float4 *)(p0 + 4 * j);
    } else if (c >= 0 && c < nch) {
      const float *pc = src(c), *pn = src(c + 1);
#pragma unroll
      for (int j0 = 0; j0 < CP / 4; j0 += 4) {
#pragma unroll
        for (int j = j0; j < j0 + 4; ++j) {
          const float4 v = win[j % C2_WIN];
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }
#pragma unroll
        for (int j = j0; j < j0 + 4; ++j) {
          const int jn = j + C2_WIN;
          win[j % C2_WIN] = jn < CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - CP / 4));
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      }
    }
    __syncthreads();
  }

  // ----------------------------------------------------------------- epilogue
  const int row = t * T32 + lr;
  const int rows = B.j[ji].w.rows;
  const float *bias = B.j[ji].bias;
  float *y = B.j[ji].y;
  if (B.j[ji].epi == EPI_GELU_Q) {
    const bool ok = lane < 32 && row < rows;
    float g = 0.0f;
    if (ok) {
      g = h2f(B.j[ji].gelu_tab[f2h(acc + bias[row])]);
      if (y) y[row] = g;
    }
    quantize_half(g, lane, ok, B.j[ji].oq_qs + (size_t)t * 16, B.j[ji].oq_d + t, B.j[ji].oxd + (size_t)t * QK);
  } else if (lane < 32 && row < rows) {
    y[row] = bias ? acc + bias[row] : acc;
  }
}

__global__ void __launch_bounds__(C2Gemv::THREADS, 2) k_gemv_chain32(GemvBatch B) {
  __shared__ C2Lds<C2Gemv> L;
  chain32_body(B, blockIdx.x, L);
}

// ================================================================== 32-row, barrier-free
// The same chains and pair terms as chain32_body with no workgroup barrier in the loop: the
// consumer and each producer hand the pair-term ring over through LDS counters instead.
//  * ready[s]: producers add 1 after their terms of a chunk in slot s landed (lgkmcnt(0));
//    chunk c is complete when ready[c % NB_RING] reaches NPW * (c / NB_RING + 1);
//  * cons: chunks the consumer has read into registers; a producer writes chunk k into its slot
//    once cons >= k - NB_RING + 1.
// Each producer brings its own weights, scales and activation factors by LDS-DMA (DEPTH chunks
// ahead, retired by its own counted vmcnt), so no wave waits for another's loads.  The consumer
// reads its 256 pair terms per chunk in batches of 8 16-byte reads issued one batch ahead of the
// 32 adds they feed; the next chunk's ready count is read with the last batch.  Why: the
// barrier version's per-chunk s_barrier and lgkmcnt(0) drain cost the chain 8.5 cycles per add
// against the 4.3 the batched loop reaches alone (profiles/r04_cons_lat3.txt).
// The chain adds of one consumer batch as volatile asm statements of 32 adds (8 float4 in
// registers) with a memory clobber: the compiler keeps each batch's LDS reads in front of the adds
// they overlap (left to itself it issued all of a chunk's reads first and spilled them), waits only
// for the batch being added, and puts no s_nop inside a statement (it does between statements).
#define NB_A4(i) "v_add_f32 %0, %0, %" #i "\n\t"
#define NB_ADDS8(acc, a, o)                                                                                      \
  asm volatile(NB_A4(1) NB_A4(2) NB_A4(3) NB_A4(4) NB_A4(5) NB_A4(6) NB_A4(7) NB_A4(8) NB_A4(9) NB_A4(10) NB_A4(11) \
                   NB_A4(12) NB_A4(13) NB_A4(14) NB_A4(15) NB_A4(16) NB_A4(17) NB_A4(18) NB_A4(19) NB_A4(20)      \
                       NB_A4(21) NB_A4(22) NB_A4(23) NB_A4(24) NB_A4(25) NB_A4(26) NB_A4(27) NB_A4(28) NB_A4(29)  \
                           NB_A4(30) NB_A4(31) NB_A4(32)                                                         \
               : "+v"(acc)                                                                                       \
               : "v"(a[o].x), "v"(a[o].y), "v"(a[o].z), "v"(a[o].w), "v"(a[o + 1].x), "v"(a[o + 1].y),           \
                 "v"(a[o + 1].z), "v"(a[o + 1].w), "v"(a[o + 2].x), "v"(a[o + 2].y), "v"(a[o + 2].z),            \
                 "v"(a[o + 2].w), "v"(a[o + 3].x), "v"(a[o + 3].y), "v"(a[o + 3].z), "v"(a[o + 3].w),            \
                 "v"(a[o + 4].x), "v"(a[o + 4].y), "v"(a[o + 4].z), "v"(a[o + 4].w), "v"(a[o + 5].x),            \
                 "v"(a[o + 5].y), "v"(a[o + 5].z), "v"(a[o + 5].w), "v"(a[o + 6].x), "v"(a[o + 6].y),            \
                 "v"(a[o + 6].z), "v"(a[o + 6].w), "v"(a[o + 7].x), "v"(a[o + 7].y), "v"(a[o + 7].z),            \
                 "v"(a[o + 7].w)                                                                                 \
               : "memory")
#define NB_ADDS4(acc, a, o)                                                                                      \
  asm volatile(NB_A4(1) NB_A4(2) NB_A4(3) NB_A4(4) NB_A4(5) NB_A4(6) NB_A4(7) NB_A4(8) NB_A4(9) NB_A4(10) NB_A4(11) \
                   NB_A4(12) NB_A4(13) NB_A4(14) NB_A4(15) NB_A4(16)                                             \
               : "+v"(acc)                                                                                       \
               : "v"(a[o].x), "v"(a[o].y), "v"(a[o].z), "v"(a[o].w), "v"(a[o + 1].x), "v"(a[o + 1].y),           \
                 "v"(a[o + 1].z), "v"(a[o + 1].w), "v"(a[o + 2].x), "v"(a[o + 2].y), "v"(a[o + 2].z),            \
                 "v"(a[o + 2].w), "v"(a[o + 3].x), "v"(a[o + 3].y), "v"(a[o + 3].z), "v"(a[o + 3].w)             \
               : "memory")
// The pair-lane form (chain32_nb_body's consumer): lanes 2r and 2r+1 hold terms 8i..8i+3 and
// 8i+4..8i+7 of row r in float4 a[o+i]; lane 2r adds its own four, then its partner's four through
// a DPP quad_perm source (lane 2r+1 runs a chain of no use).  One 16-byte read then brings 8 terms
// of a row instead of 4 (r05: tools/cons_lat5.hip, the dependent DPP add costs what the plain one
// does, 4.63 cycles; a consumer loop with 4x fewer reads ran 4.96 vs 5.53 cycles per add alone
// and 5.48 vs 8.14 beside eight busy producers).
#define NB_DP(i) "v_add_f32_dpp %0, %" #i ", %0 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf\n\t"
#define NB_PAIR(a, b, c, d) NB_A4(a) NB_A4(b) NB_A4(c) NB_A4(d) NB_DP(a) NB_DP(b) NB_DP(c) NB_DP(d)
#define NB_ADDS4P(acc, a, o)                                                                                     \
  asm volatile(NB_PAIR(1, 2, 3, 4) NB_PAIR(5, 6, 7, 8) NB_PAIR(9, 10, 11, 12) NB_PAIR(13, 14, 15, 16)              \
               : "+v"(acc)                                                                                       \
               : "v"(a[o].x), "v"(a[o].y), "v"(a[o].z), "v"(a[o].w), "v"(a[o + 1].x), "v"(a[o + 1].y),           \
                 "v"(a[o + 1].z), "v"(a[o + 1].w), "v"(a[o + 2].x), "v"(a[o + 2].y), "v"(a[o + 2].z),            \
                 "v"(a[o + 2].w), "v"(a[o + 3].x), "v"(a[o + 3].y), "v"(a[o + 3].z), "v"(a[o + 3].w)             \
               : "memory")
#ifdef VSIM_NB_STAMPS
#define NBS(...) __VA_ARGS__
#else
#define NBS(...)
#endif
#ifndef NB_RING_N  // pair-term ring slots of the barrier-free GEMVs (A/B builds override)
#define NB_RING_N 4
#endif
constexpr int NB_RING = NB_RING_N;
constexpr unsigned NB_SPIN_MAX = 1u << 24;
template <class S>
struct NbLds {
  float P[NB_RING][32 * S::LD];
  uint4 RQ[S::DEPTH][S::NPW][64];
  float RD[S::DEPTH][S::NPW][64];
  float RX[S::DEPTH][S::NPW][64];
  unsigned ready[NB_RING];
  unsigned cons;
};

__device__ __forceinline__ unsigned lds_load(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ================================================================== the tail's LayerNorm (r06)
// TailLn (common.hpp): the next layer's LayerNorm(s) computed inside the layer tail, so no
// k_ln_quant launch (5.5 us) and no launch boundary sit between the tail and the next layer's
// GEMV batch.  Per output tile t (32 rows):
//  1. out-projection tile t stores its 32 sums as 8-byte granules {value, tag} (sc1), and is done;
//  2. fc_out tile t (the tile's "owner": its K = 4E chain usually ends last, and it loads the
//     out-projection's granules one chunk before its chain ends) joins the residual
//     v = x + ((a + ab) + (f + fb)) (vsim.cpp:694-695, the order k_ln_quant's join keeps), stores
//     v, and publishes the tile's partial sums as two 16-byte granules: sum v and min ulp (the
//     exact-mean certificate's operands, ggml.c:4264-4270 summed in double), sum v^2 and an
//     upper bound of sum |v|;
//  3. every owner polls all tiles' partials (one round, no counter: the tags say which are in;
//     r06: a drained store + agent counter polled by one lane, then one read of the partials,
//     took the tail 36.5 vs 34.0 us, 639.4-639.8 vs 669.7-669.8 tok/s, profiles/r06_lnt_ab.txt),
//     reduces them in one fixed order, so every owner derives the same mean and scale, then
//     normalizes, applies the affine and quantizes its own 32-block (one Q4_0 block per tile).
// fc_out tiles wait for higher-indexed workgroups here (the out-projection tiles): they hold at
// most E/32 CUs, and the out-projection tiles wait for nothing but the heads, so they always get
// the other CUs (tail_ln_ok: E/32 below the CU count).
// The variance needs the mean, which a single round of partials cannot give exactly; it is
// taken from the moments, s2 = (Q - 2 m S) + n m^2, and accepted when both ends of an error
// interval covering this formula and the reference's sequential sum (ggml.c:4285-4293) give
// the same float scale (the map S2 -> (float)(1/sqrt(S2/n + eps)) is monotone): the
// certificate idea of ln_exact_lds_t with a wider interval.  Otherwise (an uncertified mean
// or an ambiguous scale) the owners read the whole joined row back from its granules and run
// ln_exact_lds_t's statistics on it: the sequential mean, the tree s2, the sequential s2.
// Tags: epoch << 8 | layer + 1; the epoch is advanced by the step's first k_ln_quant, so a
// granule left by an earlier step or layer never matches.
constexpr unsigned LNT_SPIN_MAX = 1u << 22;
typedef __attribute__((address_space(1))) unsigned long long gu64;
__device__ __forceinline__ unsigned lnt_tag(const TailLn &N) { return (*N.ep << 8) | (unsigned)(N.il + 1); }
__device__ __forceinline__ void st_granule(unsigned long long *p, float v, unsigned tag) {
  const unsigned long long g = (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
  __hip_atomic_store((gu64 *)p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store_dwordx2 sc1
}
__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load_dwordx2 sc1
}
__device__ __forceinline__ void st16_sc1(uint4 *p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ double dbl_of(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ void lnt_spin(unsigned &spins, unsigned *err, int lane) {
  __builtin_amdgcn_s_sleep(1);
  if (++spins == LNT_SPIN_MAX && err && lane == 0) __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// out-projection tile t, wave 0 (row t*32 + lane in lanes 0-31)
__device__ __forceinline__ void lnt_oproj(const TailLn &N, int row, int rows, float acc, int lane) {
  if (lane < 32 && row < rows) st_granule(N.og + row, acc, lnt_tag(N));
  NBS(if (lane == 0) g_nb_stamps[1536 + blockIdx.x][8] = __builtin_amdgcn_s_memrealtime();)
}

// What the owner loads before its chain ends (a chunk early, so the loads land behind the last
// adds): the out-projection's granule of the lane's row, the join's operands (the residual, the
// two biases) and the affine of the lane's norm (lanes 0-31 norm 1, 32-63 norm 2)
struct LntPre {
  unsigned long long g;
  float x, ab, fb, w, b;
};
__device__ __forceinline__ LntPre lnt_prefetch(const TailLn &N, int t) {
  const int lane = threadIdx.x & 63, i = t * T32 + (lane & 31);
  const bool hi = lane >= 32, mine = !hi || N.w2 != nullptr;
  LntPre p;
  p.g = ld_granule(N.og + i);
  p.x = N.x[i];
  p.ab = N.ab ? N.ab[i] : 0.0f;
  p.fb = N.fb ? N.fb[i] : 0.0f;
  p.w = mine ? (hi ? N.w2 : N.w1)[i] : 0.0f;
  p.b = mine ? (hi ? N.b2 : N.b1)[i] : 0.0f;
  return p;
}
// a double summed over each half-wave (lanes 0-31, 32-63), the sum in every lane of the half
__device__ __forceinline__ double half_sum_d(double v) {
  v = v + dpp::mov<dpp::QP_XOR1, 0xF>(v, 0.0);
  v = v + dpp::mov<dpp::QP_XOR2, 0xF>(v, 0.0);
  v = v + dpp::mov<dpp::HALF_MIRROR, 0xF>(v, 0.0);
  v = v + dpp::mov<dpp::MIRROR, 0xF>(v, 0.0);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xFFFFFFFF), 0x401F), hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), 0x401F);
  return v + __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int half_min_i(int v) {
  v = min(v, dpp::mov<dpp::QP_XOR1, 0xF>(v, 0x7FFFFFFF));
  v = min(v, dpp::mov<dpp::QP_XOR2, 0xF>(v, 0x7FFFFFFF));
  v = min(v, dpp::mov<dpp::HALF_MIRROR, 0xF>(v, 0x7FFFFFFF));
  v = min(v, dpp::mov<dpp::MIRROR, 0xF>(v, 0x7FFFFFFF));
  return min(v, __builtin_amdgcn_ds_swizzle(v, 0x401F));
}

// fc_out tile t, wave 0: acc = row t*32 + (lane & 31) of fc_out (lanes 32-63 hold copies); pre:
// lnt_prefetch's loads, issued a chunk before the chain ended; scr: LDS for E floats (the
// fallback's copy of the joined row)
__device__ __forceinline__ void lnt_owner(const TailLn &N, int t, int ntile, float acc, const LntPre &pre,
                                          float *scr, unsigned *err) {
  const int lane = threadIdx.x & 63, i = t * T32 + (lane & 31), n = ntile * T32;
  const unsigned tag = lnt_tag(N);
  NBS(unsigned long long *ls = g_nb_stamps[1536 + blockIdx.x] + 8;
      if (lane == 0) ls[0] = __builtin_amdgcn_s_memrealtime();)
  const bool hi = lane >= 32, two = N.w2 != nullptr, mine = !hi || two;
  const float xv = pre.x, abv = pre.ab, fbv = pre.fb, wv = pre.w, bv = pre.b;
  unsigned spins = 0;
  // 1. the out-projection's value of row i
  unsigned long long ga = pre.g;
  while (!__all((unsigned)(ga >> 32) == tag) && spins < LNT_SPIN_MAX) {
    lnt_spin(spins, err, lane);
    ga = ld_granule(N.og + i);
  }
  NBS(if (lane == 0) {
    ls[1] = __builtin_amdgcn_s_memrealtime();
    ls[5] = spins;  // (the granule's re-polls)
  })
  // 2. the join (ja + jab) + (jf + jfb), then x + that (kern.hpp ln_exact_lds_t's join)
  const float a = N.ab ? __uint_as_float((unsigned)ga) + abv : __uint_as_float((unsigned)ga);
  const float ff = N.fb ? acc + fbv : acc;
  const float v = xv + (a + ff);
  {
    // (every lane holds a row of the tile: the half-wave sums are the tile's)
    const double s = half_sum_d((double)v), sa = half_sum_d((double)fabsf(v));
    const double q = half_sum_d((double)v * (double)v);  // exact squares: 48-bit products
    const int um = half_min_i(ulp_exp(v));
    if (lane == 0) {
      float au = (float)sa;  // rounded up: an upper bound of sum |v| is all the certificate needs
      if ((double)au < sa) au = __uint_as_float(__float_as_uint(au) + 1u);
      const unsigned long long sb = (unsigned long long)__double_as_longlong(s), qb = (unsigned long long)__double_as_longlong(q);
      st16_sc1(N.rec + 2 * t, u32x4{(unsigned)sb, (unsigned)(sb >> 32), (unsigned)um, tag});
      st16_sc1(N.rec + 2 * t + 1, u32x4{(unsigned)qb, (unsigned)(qb >> 32), __float_as_uint(au), tag});
    }
  }
  if (lane < 32) {  // the joined row: the next layer's residual, and the fallback's granules
    N.jout[i] = v;
    st_granule(N.jg + i, v, tag);
  }
  NBS(if (lane == 0) ls[2] = __builtin_amdgcn_s_memrealtime();)
  // 3. every tile's partials: granule g = lane + 64 k (even g: {sum, umin}, odd g: {sum v^2, sum |v|})
  const int ng = 2 * ntile;
  double S = 0.0, Q = 0.0, A = 0.0;
  int U = 1 << 30;
  spins = 0;
  for (;;) {
    u32x4 g[8];
    const uint4 *p[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = N.rec + min(lane + 64 * k, ng - 1);
    // (one statement: the loads and their wait, so no use of a result can move above the wait)
    asm volatile(
        "global_load_dwordx4 %0, %8, off sc1\n\t"
        "global_load_dwordx4 %1, %9, off sc1\n\t"
        "global_load_dwordx4 %2, %10, off sc1\n\t"
        "global_load_dwordx4 %3, %11, off sc1\n\t"
        "global_load_dwordx4 %4, %12, off sc1\n\t"
        "global_load_dwordx4 %5, %13, off sc1\n\t"
        "global_load_dwordx4 %6, %14, off sc1\n\t"
        "global_load_dwordx4 %7, %15, off sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(g[0]), "=&v"(g[1]), "=&v"(g[2]), "=&v"(g[3]), "=&v"(g[4]), "=&v"(g[5]), "=&v"(g[6]), "=&v"(g[7])
        : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
        : "memory");
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (lane + 64 * k < ng) ok = ok && g[k].w == tag;
    if (__all(ok) || spins >= LNT_SPIN_MAX) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (lane + 64 * k >= ng) continue;
        if ((lane & 1) == 0) {
          S += dbl_of(g[k].x, g[k].y);
          U = min(U, (int)g[k].z);
        } else {
          Q += dbl_of(g[k].x, g[k].y);
          A += (double)__uint_as_float(g[k].z);
        }
      }
      break;
    }
    lnt_spin(spins, err, lane);
  }
  NBS(if (lane == 0) {
    ls[3] = __builtin_amdgcn_s_memrealtime();
    ls[6] = spins;  // (the partials' re-polls)
  })
  S = wave_sum_d(S);
  Q = wave_sum_d(Q);
  A = wave_sum_d(A);
  U = wave_min_i(U);
  const double eps = 1e-5f;
  double mean = 0.0;
  float scale = 0.0f;
  const bool mean_ok = U == (1 << 30) || A * (1.0 + 0x1.0p-30) < ldexp(1.0, 53 + U);
  bool fallback = !mean_ok;
  if (mean_ok) {
    // S is exact (every partial sum of the row is, under the certificate): the reference's mean
    mean = S / n;
    const double t1 = mean * S, t3 = (mean * mean) * n;
    const double s2 = (Q - 2.0 * t1) + t3, M = Q + 2.0 * fabs(t1) + t3;
    // |s2 - exact| <= ~20 u M (Q's tree, the three rounded terms); the reference's sequential
    // s2 lies within (n + 5) u of the exact value (ggml.c:4287-4291): both inside B
    const double s2c = s2 > 0.0 ? s2 : 0.0;
    const double B = ((2.0 * n + 64.0) * s2c + 64.0 * M) * 0x1.0p-53 * (1.0 + 0x1.0p-20);
    // r(S2) = 1/sqrt(S2/n + eps) is decreasing and convex, so over [s2 - B, s2 + B] it moves by at
    // most B |r'(s2 - B)| <= r * B / (2 (s2 - B + n eps)) * sqrt(1 + d), d = B / (s2 - B + n eps);
    // for d <= 1 that is below r * B / (s2 - B + n eps), and for d > 1 the widening below exceeds r
    // and the check fails.  The reference's and this evaluation of the double expression each round
    // a few times (<= 2^-50 relative, four times covered): when r widened by both still rounds to
    // one float, that float is the reference's scale.  (One sqrt and one division, not one per end.)
    const double r = 1.0 / sqrt(s2 / n + eps);
    const double dr = r * (B / ((s2c - B > 0.0 ? s2c - B : 0.0) + n * eps) + 0x1.0p-48);
    const float sc = (float)r;
    if ((float)(r - dr) == sc && (float)(r + dr) == sc)
      scale = sc;
    else
      fallback = true;
  }
  if (fallback) {
    // the whole joined row from its granules, then ln_exact_lds_t's statistics in one wave
    for (int k = lane; k < n; k += 64) {
      unsigned sp = 0;
      unsigned long long g;
      do {
        g = ld_granule(N.jg + k);
        if ((unsigned)(g >> 32) == tag) break;
        __builtin_amdgcn_s_sleep(1);
      } while (++sp < LNT_SPIN_MAX);
      scr[k] = __uint_as_float((unsigned)g);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const double m = mean_ok ? S : seq_sum_exact_inl(scr, n, lane);
    mean = m / n;
    double s2 = 0.0;
    for (int k = lane; k < n; k += 64) {
      const double d = (double)scr[k] - mean;
      s2 += d * d;
    }
    s2 = wave_sum_d(s2);
    const double B = (2.0 * n + 64.0) * 0x1.0p-53 * s2;
    const float sc_lo = (float)(1.0 / sqrt((s2 + B) / n + eps));
    const float sc_hi = (float)(1.0 / sqrt((s2 - B > 0.0 ? s2 - B : 0.0) / n + eps));
    scale = sc_lo;
    if (sc_lo != sc_hi) {  // the reference's order, in lane 0
      float sq = 0.0f;
      if (lane == 0) {
        double qq = 0.0;
        for (int k = 0; k < n; ++k) {
          const double d = (double)scr[k] - mean;
          qq += d * d;
        }
        sq = (float)(1.0 / sqrt(qq / n + eps));
      }
      scale = __shfl(sq, 0);
      if (t == 0 && lane == 0 && N.stats) atomicAdd(&N.stats[1], 1u);
    }
    if (!mean_ok && t == 0 && lane == 0 && N.stats) atomicAdd(&N.stats[0], 1u);
  }
  // 4. this tile's block: norm 1 in lanes 0-31, norm 2 in lanes 32-63 (same row values)
  float y = (float)((double)v - mean);
  y = y * scale;
  const float z = mine ? (wv * y) + bv : 0.0f;
  uint8_t *qs = hi ? N.q2 : N.q1;
  float *dq = hi ? N.d2 : N.d1, *xd = hi ? N.xd2 : N.xd1;
  quantize_half(z, lane, mine, mine ? qs + (size_t)t * 16 : nullptr, mine ? dq + t : nullptr,
                mine ? xd + (size_t)t * QK : nullptr);
  NBS(if (lane == 0) ls[4] = __builtin_amdgcn_s_memrealtime();)
}

// SC1: the activation factors were written write-through by other workgroups of this launch
// ONE: B holds a single job (the tail's fc_out and out-projection): its arguments are read at
// constant offsets with no job probe, so they load in one round trip at the workgroup's start
// (the probe loop and the chosen job's fields behind it were three dependent kernarg round trips,
// ~1.1 us from a tail workgroup's start to its first weight DMA, r05 stamps)
// LNR (the tail's LayerNorm, TailLn): 0 the job's own epilogue, 1 fc_out: the tile's owner, 2 the
// out-projection's granules
template <class S, bool SC1, bool ONE = false, int LNR = 0>
__device__ __forceinline__ void chain32_nb_body(const GemvBatch &B, int t, NbLds<S> &L, unsigned *err,
                                                const TailLn *N = nullptr) {
  constexpr int DEPTH = S::DEPTH, CB = S::CB, LD = S::LD, NPW = S::NPW;
  constexpr int WAIT_VM = waitcnt_vm(3 * (DEPTH - 1));  // chunk c landed, c+1 .. c+DEPTH-1 in flight
  static_assert(3 * (DEPTH - 1) < 64, "vmcnt immediate");
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int ji = 0;
  if constexpr (ONE) {
    if (t >= B.j[0].w.tiles) return;
  } else {
    while (ji < B.nj) {
      if (t < B.j[ji].w.tiles) break;
      t -= B.j[ji].w.tiles;
      ++ji;
    }
    if (ji >= B.nj) return;
    ji = __builtin_amdgcn_readfirstlane(ji);
  }
  const GemvJob &J = B.j[ONE ? 0 : ji];
  const int nb = J.w.k / QK, nch = (nb + CB - 1) / CB;
  if (threadIdx.x < NB_RING) L.ready[threadIdx.x] = 0;
  if (threadIdx.x == 0) L.cons = 0;
  __syncthreads();
  if (S::FILL && wave > 0 && wave % 4 == 0) return;  // the consumer's SIMD is left to it

  if (wave > 0) {
    // ------------------------------------------------------------- producer
    const int p = S::FILL ? wave - 1 - wave / 4 : wave - 1, r = lane & 31, hb = lane >> 5;
    if (p >= NPW) return;  // (a launch wider than this shape needs)
    const int o = 2 * p + hb;  // this lane's block within the chunk
    const uint8_t *qs = J.w.qs + (size_t)t * nb * T32 * 16 + (size_t)r * 16;
    const float *dd = J.w.d + (size_t)t * nb * T32 + r;
    const float *xr = J.xd + r;
    // every chunk up to nch + DEPTH is loaded (block clamped), so the counted waits hold
    auto dma = [&](int c) {
      const int slot = c % DEPTH;
      const int b = min(c * CB + o, nb - 1);
      glds16(qs + (size_t)b * (T32 * 16), lds_addr(&L.RQ[slot][p][0]));
      glds4(dd + (size_t)b * T32, lds_addr(&L.RD[slot][p][0]));
      if constexpr (SC1)
        glds4_sc1(xr + (size_t)b * QK, lds_addr(&L.RX[slot][p][0]));
      else
        glds4<false>(xr + (size_t)b * QK, lds_addr(&L.RX[slot][p][0]));
    };
    NBS(unsigned long long sw_dma = 0, sw_slot = 0, sw_comp = 0;)
    // chunk c's raw block and factors from its DMA slot into registers (issued, not waited for:
    // the reads complete behind the next chunk's pair terms)
    // (factors: F0 / F1 = slots 0-15 / 16-31 of the half's block in every 16-lane row, for the
    // DPP broadcast of pair_terms4_dpp: two 4-byte reads instead of eight 16-byte broadcasts)
    const int fx = (lane & 32) + (lane & 15);
    auto issue_raw = [&](int c, uint4 &q, float &dq, float &f0, float &f1) {
      const int slot = c % DEPTH;
      NBS(const unsigned long long t0 = __builtin_amdgcn_s_memtime();)
      __builtin_amdgcn_s_waitcnt(WAIT_VM);  // this wave's DMA of chunk c landed
      NBS(sw_dma += __builtin_amdgcn_s_memtime() - t0;)
      q = L.RQ[slot][p][lane];
      dq = L.RD[slot][p][lane];
      f0 = L.RX[slot][p][fx];
      f1 = L.RX[slot][p][fx + 16];
    };
    // chunk k's pair terms into ring slot k % NB_RING, then (lgkmcnt(0): the terms and the raw
    // reads of chunk k+1 landed) the count, and the DMA of chunk k+1+DEPTH into the raw slot just read
    auto compute = [&](int k, float f0, float f1, const uint4 &qc, float dqc) {
      const int slot = k % NB_RING;
      NBS(const unsigned long long t0 = __builtin_amdgcn_s_memtime();)
      if (k >= NB_RING) {
        unsigned spins = 0;
        while ((int)lds_load(&L.cons) < k - NB_RING + 1) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins == NB_SPIN_MAX) {
            if (err && lane == 0) __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        asm volatile("" ::: "memory");
      }
      NBS(const unsigned long long t1 = __builtin_amdgcn_s_memtime(); sw_slot += t1 - t0;)
      const float dv = k * CB + o < nb ? dqc : 0.0f;
      const f32x2 d2 = {512.0f * dv, 512.0f * dv}, m2 = {-8.0f * dv, -8.0f * dv};
      float *dst = &L.P[slot][r * LD + o * 16];
      float p4[4];
      pair_terms4_dpp<0>(qc.x, d2, m2, f0, f1, p4);
      *(float4 *)(dst + 0) = make_float4(p4[0], p4[1], p4[2], p4[3]);
      pair_terms4_dpp<1>(qc.y, d2, m2, f0, f1, p4);
      *(float4 *)(dst + 4) = make_float4(p4[0], p4[1], p4[2], p4[3]);
      pair_terms4_dpp<2>(qc.z, d2, m2, f0, f1, p4);
      *(float4 *)(dst + 8) = make_float4(p4[0], p4[1], p4[2], p4[3]);
      pair_terms4_dpp<3>(qc.w, d2, m2, f0, f1, p4);
      *(float4 *)(dst + 12) = make_float4(p4[0], p4[1], p4[2], p4[3]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      NBS(sw_comp += __builtin_amdgcn_s_memtime() - t1;)
      if (lane == 0) __hip_atomic_fetch_add(&L.ready[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // (stamps: fc_out tiles' startup, producer 0: chunk 0 counted)
      NBS(if (ONE && LNR == 1 && p == 0 && k == 0 && lane == 0) g_nb_stamps[1536 + blockIdx.x][7] = __builtin_amdgcn_s_memrealtime();)
      dma(k + 1 + DEPTH);
    };
#pragma unroll
    for (int c = 0; c < DEPTH; ++c) dma(c);
    NBS(if (ONE && LNR == 1 && p == 0 && lane == 0) g_nb_stamps[1536 + blockIdx.x][4] = __builtin_amdgcn_s_memrealtime();)
    uint4 qa, qb;
    float da, db, fa0, fa1, fb0, fb1;
    issue_raw(0, qa, da, fa0, fa1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    NBS(if (ONE && LNR == 1 && p == 0 && lane == 0) g_nb_stamps[1536 + blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();)
    dma(DEPTH);
    for (int k = 0; k < nch; k += 2) {
      issue_raw(k + 1, qb, db, fb0, fb1);
      compute(k, fa0, fa1, qa, da);
      issue_raw(k + 2, qa, da, fa0, fa1);
      if (k + 1 < nch) compute(k + 1, fb0, fb1, qb, db);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup ends
    NBS(if (lane == 0 && p < 8) {
      g_nb_stamps[blockIdx.x][4 + p] = sw_dma;
      g_nb_stamps[blockIdx.x][12 + p] = sw_slot;
      g_nb_stamps[blockIdx.x][20 + p] = sw_comp;
      if (p < 4) g_nb_stamps[blockIdx.x][28 + p] = __builtin_amdgcn_s_memtime();
    })
    return;
  }

  // --------------------------------------------------------------- consumer (row r: lane 2r)
  // Batches of 4 reads (32 terms of each row, NB_ADDS4P) in four register sets: the reads of batch
  // q+3 go out with the adds of batch q, so a read has three batches (~100 adds) to land, and at
  // most 13 LDS reads are in flight (lgkmcnt counts 15: every wait is exact).  Batch q of a chunk
  // always sits in set q % 4 (8 batches per chunk), so the sets need no copies across chunks.
  float acc = 0.0f;
  const int lr = lane >> 1, lk = lane & 1;
  constexpr int NV = S::CP / 8, BQ = 4, NBQ = NV / BQ;  // 8-term reads per chunk and row, per batch, batches
  static_assert(NV % BQ == 0 && NBQ % 4 == 0, "batches tile the chunk in whole rounds of four sets");
  auto need = [](int c) { return (unsigned)(NPW * (c / NB_RING + 1)); };
  NBS(unsigned long long cw = 0;)
  // (the re-poll is asm: a C++ loop of LDS loads made the compiler drain every read in flight
  // where its path joins the fast one, once per chunk)
  auto wait_ready = [&](int c, unsigned have) {
    NBS(const unsigned long long t0 = __builtin_amdgcn_s_memtime();)
    if (have < need(c)) {
      unsigned spins = 0, h;
      asm volatile(
          "1:\n\t"
          "ds_read_b32 %0, %2\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "v_cmp_lt_u32 vcc, %0, %3\n\t"
          "s_cbranch_vccz 2f\n\t"
          "s_add_u32 %1, %1, 1\n\t"
          "s_cmp_lt_u32 %1, %4\n\t"
          "s_cbranch_scc1 1b\n\t"
          "2:"
          : "=&v"(h), "+s"(spins)
          : "v"(lds_addr(&L.ready[c % NB_RING])), "s"(need(c)), "s"(NB_SPIN_MAX)
          : "vcc", "scc", "memory");
      if (spins >= NB_SPIN_MAX && err && lane == 0) __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    NBS(const unsigned long long dw = __builtin_amdgcn_s_memtime() - t0; cw += dw;
        if (ONE && blockIdx.x < 128 && c < 32 && lane == 0) {
          g_nb_stamps[960 + blockIdx.x][c] = dw;
          g_nb_stamps[1088 + blockIdx.x][c] = t0;
        })
  };
  __builtin_amdgcn_s_setprio(3);
  NBS(const unsigned long long c_t0 = __builtin_amdgcn_s_memtime();)
  wait_ready(0, 0u);
  NBS(if (ONE && LNR == 1 && lane == 0) g_nb_stamps[1536 + blockIdx.x][3] = __builtin_amdgcn_s_memrealtime();)
  f32x4 b0[BQ], b1[BQ], b2[BQ], b3[BQ];
  auto rd = [&](f32x4 (&d)[BQ], int c, int q) {  // batch q of chunk c (past the last chunk: harmless)
    const f32x4 *src = (const f32x4 *)&L.P[c % NB_RING][lr * LD] + 2 * q * BQ + lk;
#pragma unroll
    for (int j = 0; j < BQ; ++j) d[j] = src[2 * j];
  };
  rd(b0, 0, 0);
  rd(b1, 0, 1);
  rd(b2, 0, 2);
  // (LNR 1: the LayerNorm epilogue's operands, loaded a chunk before the chain ends)
  LntPre pre{};
  const int c_pre = nch > 1 ? nch - 2 : 0;
  for (int c = 0; c < nch; ++c) {
    if constexpr (LNR == 1)
      if (c == c_pre) pre = lnt_prefetch(*N, t);
    // the next chunk's count is read after batch NBQ-6's adds (behind the reads of batch NBQ-3,
    // so it lands with them) and compared at batch NBQ-3, before that chunk's first read; r05: read
    // at the chunk's top instead, it was often short by the chunk's last producers, and the
    // re-poll cost ~180 cycles a chunk (a poll at the chunk's end drained the read pipeline)
    unsigned rdy = 0;
#pragma unroll
    for (int q = 0; q < NBQ; ++q) {
      const int qn = q + 3, cn = qn < NBQ ? c : c + 1, qr = qn < NBQ ? qn : qn - NBQ;
      if (q == NBQ - 5) rdy = lds_load(&L.ready[(c + 1) % NB_RING]);
      if (qn == NBQ && c + 1 < nch) {
        unsigned r = rdy;
        asm volatile("" : "+v"(r));  // compared here, not where it was read
        wait_ready(c + 1, r);
      }
      asm volatile("" ::: "memory");
      f32x4(&dst)[BQ] = (qn % 4 == 0) ? b0 : (qn % 4 == 1) ? b1 : (qn % 4 == 2) ? b2 : b3;
      rd(dst, cn, qr);
      f32x4(&cur)[BQ] = (q % 4 == 0) ? b0 : (q % 4 == 1) ? b1 : (q % 4 == 2) ? b2 : b3;
      NB_ADDS4P(acc, cur, 0);
      if (q == NBQ - 1)  // the chunk's last reads landed (the adds waited for them): refill its slot
        __hip_atomic_store(&L.cons, (unsigned)(c + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __builtin_amdgcn_s_setprio(0);
  NBS(if (lane == 0) {
    g_nb_stamps[blockIdx.x][0] = c_t0;
    g_nb_stamps[blockIdx.x][1] = __builtin_amdgcn_s_memtime();
    g_nb_stamps[blockIdx.x][2] = cw;
    g_nb_stamps[blockIdx.x][3] = nch;
  })
  acc = __shfl(acc, (2 * lane) & 63);  // row r's sum from lane 2r to lane r (lanes 32-63: copies)

  // ----------------------------------------------------------------- epilogue
  const int row = t * T32 + (lane & 31);
  const int rows = J.w.rows;
  const float *bias = J.bias;
  float *y = J.y;
  if constexpr (LNR == 1) {
    lnt_owner(*N, t, J.w.tiles, acc, pre, &L.P[0][0], err);
    return;
  }
  if constexpr (LNR == 2) {
    lnt_oproj(*N, row, rows, acc, lane);
    return;
  }
  if (J.epi == EPI_GELU_Q) {
    const bool ok = lane < 32 && row < rows;
    float g = 0.0f;
    if (ok) {
      g = h2f(J.gelu_tab[f2h(acc + bias[row])]);
      if (y) y[row] = g;
    }
    quantize_half(g, lane, ok, J.oq_qs + (size_t)t * 16, J.oq_d + t, J.oxd + (size_t)t * QK);
  } else if (lane < 32 && row < rows) {
    y[row] = bias ? acc + bias[row] : acc;
  }
}

// ================================================================== fused layer tail
// fc_out, the attention heads and the out-projection of one layer in one launch, so the
// attention and the out-projection run beside fc_out, whose K = 4E chain is the layer's
// longest dependency, instead of before it.  Roles by workgroup index:
//   [0, nf)          fc_out tiles (chain32_nb_body: 32 rows, 16-block chunks, eight producers,
//                    the consumer alone on SIMD0)
//   [nf, nf + na)    attention heads (attn.hpp; each head over nsplit workgroups, KQV columns
//                    split); each stores the out-projection's operand write-through (sc1,
//                    CO = true), drains it (vmcnt) and counts itself in *done (agent scope)
//   [nf + na, ...)   out-projection tiles; wait until every head's flag carries this step's tag
//                    (r06: an 8-byte sc1 granule per head instead of one agent counter, which the
//                    tiles saw ~3 us after the last head's add, profiles/r06_nb_stamps.txt); their factor loads are sc1
//                    (device-coherent: they read past stale lines in the XCD's L2), so neither
//                    side needs a fence.  r04: the release fence (an L2 write-back per head)
//                    and the acquire (an L2 invalidate, which also dropped fc_out's lines)
//                    cost 38.9 vs 35.8-36.0 us per tail at the bench's 248 positions
//                    (profiles/r04_tail_headpath_ab.txt)
// Waiting workgroups only wait for lower-indexed ones, which the dispatcher places first on
// this part (and fc_out's tiles never wait, so the CUs they hold always come free); the wait
// is bounded all the same (TAIL_SPIN_MAX sleeps, ~1 s): past it the error counter is bumped, the
// tile goes on, and the executor fails the call (VSIM_ESPIN).  r05 A/B of the barrier-free hand-off against r04's per-chunk
// barrier (chain32_body): 31.4 vs 33.7 us per tail (profiles/r05_tail_nb_ab.txt); the barrier
// tail is no longer built.
constexpr unsigned TAIL_SPIN_MAX = 1u << 22;
struct TailJob {
  GemvBatch f, o;
  AttnJob a;
  TailSync sy;  // the heads' flags
  unsigned *err;
  int nf;
  int lnon;  // the next LayerNorm in this launch (TailLn)
  TailLn ln;
};

__global__ void __launch_bounds__(C2Tail::THREADS, 1) k_layer_tail(TailJob T) {
  __shared__ union {
    NbLds<C2Tail> n;
    float a[sizeof(NbLds<C2Tail>) / sizeof(float)];
  } L;
  int b = blockIdx.x;
  // fc_out's producer arguments and the role bound in one kernel-argument round trip
  asm volatile("" ::"s"(T.nf), "s"(T.f.j[0].w.qs), "s"(T.f.j[0].w.d), "s"(T.f.j[0].w.k), "s"(T.f.j[0].w.tiles),
               "s"(T.f.j[0].xd));
  // (VSIM_NB_STAMPS: s_memrealtime timeline per workgroup in rows 1536.. : start, the role's
  // marks, end; tools/nb_stamps.py)
  NBS(unsigned long long *tl = g_nb_stamps[1536 + blockIdx.x];
      if (threadIdx.x == 0) tl[0] = __builtin_amdgcn_s_memrealtime();)
  if (b < T.nf) {
    if (T.lnon)
      chain32_nb_body<C2Tail, false, true, 1>(T.f, b, L.n, T.err, &T.ln);
    else
      chain32_nb_body<C2Tail, false, true>(T.f, b, L.n, T.err);
    NBS(if (threadIdx.x == 0) tl[2] = __builtin_amdgcn_s_memrealtime();)
    return;
  }
  b -= T.nf;
  const int na = T.a.H * (T.a.nsplit > 1 ? T.a.nsplit : 1);
  const unsigned htag = (*T.sy.ep << 8) | (unsigned)(T.sy.il + 1);
  if (b < na) {
    attn_body<C2Tail::THREADS, true>(T.a, b, L.a);
    NBS(if (threadIdx.x == 0) tl[1] = __builtin_amdgcn_s_memrealtime();)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the write-through output stores landed
    __syncthreads();
    if (threadIdx.x == 0) st_granule(T.sy.hflag + b, 0.0f, htag);  // (r06: was one agent counter)
    NBS(if (threadIdx.x == 0) tl[2] = __builtin_amdgcn_s_memrealtime();)
    return;
  }
  b -= na;
  // wave 0 polls every head's flag (one or two per lane), the other waves wait at the barrier
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    unsigned spins = 0;
    for (;;) {
      const bool ok = (lane >= na || (unsigned)(ld_granule(T.sy.hflag + lane) >> 32) == htag) &&
                      (lane + 64 >= na || (unsigned)(ld_granule(T.sy.hflag + lane + 64) >> 32) == htag);
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(2);
      if (++spins == TAIL_SPIN_MAX) {
        if (T.err && lane == 0) __hip_atomic_fetch_add(T.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  NBS(if (threadIdx.x == 0) tl[1] = __builtin_amdgcn_s_memrealtime();)
  if (T.lnon)
    chain32_nb_body<C2Tail, true, true, 2>(T.o, b, L.n, T.err, &T.ln);
  else
    chain32_nb_body<C2Tail, true, true>(T.o, b, L.n, T.err);
  NBS(if (threadIdx.x == 0) tl[2] = __builtin_amdgcn_s_memrealtime();)
}

bool tail_ln_ok(int E) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  // every owner waits for every other owner's partials: all E/32 out-projection tiles must be
  // resident at once (one workgroup per CU), beside at least one CU for the rest
  return E % T32 == 0 && E / T32 <= LNT_MAX_TILES && E / T32 < cus;
}

int launch_layer_tail(const GemvBatch &f, const GemvBatch &o, const AttnJob &a, const TailSync &sy, int n_ctx,
                      hipStream_t s, const TailLn *ln) {
  const int S = a.nsplit > 1 ? a.nsplit : 1;
  if (a.d % 32 != 0 || a.d > 256 || a.n_ctx != n_ctx || a.d % S != 0 || (a.d / S) % QK != 0 ||
      (size_t)attn_lds_floats(a.d, n_ctx) * sizeof(float) > sizeof(NbLds<C2Tail>)) {
    set_error("layer tail: attention shape (head dim, n_ctx) outside the fused kernel's range");
    return VSIM_EINVAL;
  }
  if (f.nj > 1 || o.nj > 1) {
    set_error("layer tail: fc_out and the out-projection are one job each");
    return VSIM_EINVAL;
  }
  TailJob T{};
  T.f = f;
  T.o = o;
  T.a = a;
  T.sy = sy;
  if (!sy.hflag || !sy.ep || sy.il < 0 || sy.il > 254 || a.H * S > TAIL_MAX_HEADS) {
    set_error("layer tail: the heads' flags need a flag buffer, the step epoch, a layer below 255, at most 128 heads");
    return VSIM_EINVAL;
  }
  T.err = spin_error_counter();
  T.nf = 0;
  if (ln) {
    const int E = o.nj == 1 ? o.j[0].w.rows : 0;
    if (f.nj != 1 || o.nj != 1 || f.j[0].w.rows != E || a.d * a.H != E || !tail_ln_ok(E) || ln->il < 0 ||
        ln->il > 254 || !ln->x || !ln->jout || !ln->w1 || !ln->b1 || !ln->q1 || !ln->d1 || !ln->xd1 || !ln->og ||
        !ln->jg || !ln->rec || !ln->ep || (ln->w2 && (!ln->b2 || !ln->q2 || !ln->d2 || !ln->xd2))) {
      set_error("layer tail: the in-tail LayerNorm needs fc_out and the out-projection over E rows, E/32 below the CU count");
      return VSIM_EINVAL;
    }
    T.lnon = 1;
    T.ln = *ln;
  }
  for (int i = 0; i < f.nj; ++i) T.nf += f.j[i].w.tiles;
  int no = 0;
  for (int i = 0; i < o.nj; ++i) no += o.j[i].w.tiles;
  // one workgroup per CU (fc_out's consumer keeps its SIMD): the static LDS is above half the
  // CU's (a dynamic pad would keep it so for a smaller shape); the workgroups that find no CU
  // start as attention heads end
  const dim3 grid(T.nf + a.H * S + no), blk(C2Tail::THREADS);
  constexpr size_t pad = sizeof(NbLds<C2Tail>) > 80 * 1024 ? 0 : 81 * 1024 - sizeof(NbLds<C2Tail>);
  hipLaunchKernelGGL(k_layer_tail, grid, blk, pad, s, T);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ================================================================== 64-row, SIMD0 solo
// For jobs whose chains are the whole cost (fc_out: K = 16384 over only 4096 rows): the
// consumer wave alone on SIMD0 (producers sharing its SIMD stretch each dependent add by a
// VALU slot), CB producer waves on SIMD1-3, one Q4_0 block of the chunk for the 64 rows
// each, so the activation factors are wave-uniform scalar loads and the LDS carries
// nothing but pair terms.  Waves the hardware places on the consumer's SIMD (4, 8, ...) only
// join the barriers.  Weights: register ring as k_gemv_chain2.
// Placement as measured (r05, tools/solo_placement.py, HW_ID stamps): waves w and w + 4 always
// share a SIMD, but which SIMD wave 0 gets rotates per workgroup, and the two workgroups of a CU
// always put their consumers on different SIMDs, each beside two of the other workgroup's
// producers (SIMD loads 4 / 4 / 2 + consumer / 2 + consumer producers).  Roles re-assigned from
// HW_ID so both consumers share one SIMD (4 / 4 / 4 producers) ran slower, 22.47 vs 21.96 us
// (profiles/r05_solo_nb2_ab.txt).
// CONS = 2: 128 rows per workgroup, two consumer waves (0 and 4: the waves of a workgroup go
// to the SIMDs cyclically, so these two share one SIMD, where two independent chains
// interleave without stretching each other) and 2 CB producers on the other three SIMDs
// (wave 8 and 12 join the barriers only), the LDS ring for 128 rows (153.6 KB at CB = 6:
// one workgroup per CU by construction, so no other workgroup's producers land on the
// consumers' SIMD).
template <int CB, int CONS = 1>
struct SoloShape {
  static constexpr int CP = CB * 16, LD = CP + 4;
  static constexpr int PRODUCERS = CB * CONS;
  // waves with index = 0 mod 4 share the consumers' SIMD: the first CONS are the consumers,
  // the rest only join the barriers; the others are the producers
  static constexpr int WAVES = PRODUCERS + (PRODUCERS + 2) / 3;  // a 0-mod-4 slot per 3 producers
  static constexpr int ROWS = 64 * CONS;
  // (r04: 12 and chain32's 16 read deeper than r03's 8: tail -1.1 us.  The reads go in groups of
  // 6 after 24 adds, as chain32's in groups of 4: batch 21.9 vs 22.4 us, lm_head 37.6-37.8 vs 38.6)
  static constexpr int WIN = 12;
  static_assert(CP / 4 % WIN == 0, "the read window must tile the chunk");
  static_assert(WAVES <= 16, "workgroup size");
  static_assert((WAVES + 3) / 4 >= CONS, "consumer waves on one SIMD");
};
constexpr int C5_RING = 3;

// PF: prefetch distance of the weight loads in chunks (register ring of PF+1 sets)
// One ROWS-row group g of batch B (groups numbered job by job); P: the pair-term ring.
// Every wave returns from here (producers and fillers early); all take nit barriers.
template <int CB, int PF, int CONS>
__device__ __forceinline__ void solo_body(const GemvBatch &B, int g, float (*P)[SoloShape<CB, CONS>::ROWS * SoloShape<CB, CONS>::LD]) {
  using S = SoloShape<CB, CONS>;
  constexpr int TPG = 2 * CONS;  // 32-row tiles per group
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int ji = 0;
  while (ji < B.nj) {
    const int ng = (B.j[ji].w.tiles + TPG - 1) / TPG;
    if (g < ng) break;
    g -= ng;
    ++ji;
  }
  if (ji >= B.nj) return;
  ji = __builtin_amdgcn_readfirstlane(ji);
  g = __builtin_amdgcn_readfirstlane(g);
  const int tiles = B.j[ji].w.tiles, nb = B.j[ji].w.k / QK, nch = (nb + CB - 1) / CB;
  const int nit = (nch + 2 + PF) / (PF + 1) * (PF + 1);
  // (VSIM_NB_STAMPS: where each wave runs, HW_ID | XCC_ID << 32, rows 512 + workgroup)
  NBS(if (lane == 0 && gridDim.x < 512 && wave < 32) g_nb_stamps[512 + blockIdx.x][wave] =
          (unsigned long long)__builtin_amdgcn_s_getreg(0xF804) | (unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32;)

  if ((wave & 3) == 0 && (wave >> 2) >= CONS) {  // filler on the consumers' SIMD
    for (int k = 0; k < nit; ++k) __syncthreads();
    return;
  }
  if ((wave & 3) != 0) {
    // ------------------------------------------------------------- producer
    const int pi = wave - 1 - (wave >> 2);  // 1,2,3,5,6,7,9,... -> 0,1,2,...
    const int o = pi % CB, c = pi / CB;     // block of the chunk, consumer (64-row half) served
    const int h = lane >> 5, r = lane & 31;
    const int tile = TPG * g + 2 * c + h;
    const bool tile_ok = tile < tiles;
    const int tl = tile_ok ? tile : tiles - 1;
    const uint8_t *qs = B.j[ji].w.qs + ((size_t)tl * nb * T32 + r) * 16;
    const float *dd = B.j[ji].w.d + (size_t)tl * nb * T32 + r;
    const float *xg = B.j[ji].xd;
    auto ld = [&](int c, u32x4 &qv, float &dv) {
      const int b = min(c * CB + o, nb - 1);
      qv = __builtin_nontemporal_load((gu32x4 *)(qs + (size_t)b * (T32 * 16)));
      dv = __builtin_nontemporal_load((gfloat *)(dd + (size_t)b * T32));
    };
    auto ldx = [&](int c, f32x2 *xv) {
      const int b = min(c * CB + o, nb - 1);
      const sfloat *xp = (const sfloat *)(xg + (size_t)b * QK);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        xv[i].x = xp[2 * i];
        xv[i].y = xp[2 * i + 1];
      }
    };
    int ps = 0;
    // (VSIM_NB_STAMPS: per producer wave, shader cycles summed over its steps: waiting for the
    // factors and LDS stores (lgkmcnt(0)), computing, at the barrier -- rows 512 + workgroup,
    // columns 12 + 3 pi ..; s_getreg of the 20-bit SHADER_CYCLES counter: no lgkmcnt)
    NBS(unsigned long long st_fw = 0, st_comp = 0, st_bar = 0, pa = 0, pb = 0, pc = 0, pd = 0;
        auto cyc = []() { return __builtin_amdgcn_s_memtime(); };)
    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const u32x4 &qc, float dqc, u32x4 &qn, float &dqn) {
      ld(k + PF, qn, dqn);
      // (stamps: s_memtime is a scalar-memory read; the previous step's four stamps are summed
      // after this step's lgkmcnt(0), which they ride along, so no extra wait is added)
      NBS(const unsigned long long c0 = cyc();)
      // this chunk's factors (loaded a whole step ago) before the next chunk's loads go out:
      // scalar loads return out of order, so any later wait for them would be lgkmcnt(0)
      // and would also wait for the loads just issued
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      NBS(if (pa) { st_fw += pb - pa; st_comp += pc - pb; st_bar += pd - pc; }
          pa = c0; pb = cyc();)
      __builtin_amdgcn_sched_barrier(0);
      ldx(k + 1, xn);
      __builtin_amdgcn_sched_barrier(0);
      {
        const float dv = tile_ok && k * CB + o < nb ? dqc : 0.0f;
        const float dl = 512.0f * dv, ml = -8.0f * dv;
        float dh, mh;
        asm("v_mov_b32 %0, %1" : "=v"(dh) : "v"(dl));  // see k_gemv_chain2
        asm("v_mov_b32 %0, %1" : "=v"(mh) : "v"(ml));
        const f32x2 d2 = {dl, dh}, m2 = {ml, mh};
        float *dst = &P[ps][(64 * c + lane) * S::LD + o * 16];
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          float p4[4];
          pair_terms4_x(qc[wv], d2, m2, xc + 4 * wv, p4);
          *(float4 *)(dst + 4 * wv) = make_float4(p4[0], p4[1], p4[2], p4[3]);
        }
      }
      ps = ps == C5_RING - 1 ? 0 : ps + 1;
      __builtin_amdgcn_sched_barrier(0);
      NBS(pc = cyc();)
      producer_barrier();
      NBS(pd = cyc();)
    };
    u32x4 q[PF + 1];
    float e[PF + 1];
#pragma unroll
    for (int c = 0; c < PF; ++c) ld(c, q[c], e[c]);
    f32x2 xa[16], xb[16];
    ldx(0, xa);
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" ::"s"(xa[i].x), "s"(xa[i].y));
    static_assert((PF + 1) % 2 == 0, "two factor sets alternate");
    for (int k = 0; k < nit; k += PF + 1) {
#pragma unroll
      for (int u = 0; u < PF + 1; u += 2) {
        step(k + u, xa, xb, q[u], e[u], q[(u + PF) % (PF + 1)], e[(u + PF) % (PF + 1)]);
        step(k + u + 1, xb, xa, q[u + 1], e[u + 1], q[u % (PF + 1)], e[u % (PF + 1)]);
      }
    }
    NBS(if (lane == 0 && gridDim.x < 512 && pi < 6) {
      unsigned long long *st = g_nb_stamps[512 + blockIdx.x] + 12 + 3 * pi;
      st[0] = st_fw;
      st[1] = st_comp;
      st[2] = st_bar;
    })
    return;
  }

  // --------------------------------------------------------------- consumer
  float acc = 0.0f;
  float4 win[S::WIN];
  NBS(unsigned long long sc_bar = 0;
      auto ccyc = []() { return __builtin_amdgcn_s_memtime(); };)
  const int crow = 64 * wave / 4 + lane;  // this consumer's row within the group
  auto src = [&](int c) { return &P[c % C5_RING][crow * S::LD]; };
  __builtin_amdgcn_s_setprio(3);
  // (VSIM_NB_STAMPS: the consumer's shader-clock and 100 MHz real-time stamps at its start and end)
  NBS(const unsigned long long c_m0 = __builtin_amdgcn_s_memtime(), c_r0 = __builtin_amdgcn_s_memrealtime();)
  for (int k = 0; k < nit; ++k) {
    const int c = k - 2;
    if (c == -1 && nch > 0) {
      const float *p0 = src(0);
#pragma unroll
      for (int j = 0; j < S::WIN; ++j) win[j] = *(const float4 *)(p0 + 4 * j);
    } else if (c >= 0 && c < nch) {
      const float *pc = src(c), *pn = src(c + 1);
#pragma unroll
      for (int j0 = 0; j0 < S::CP / 4; j0 += 6) {
#pragma unroll
        for (int j = j0; j < j0 + 6; ++j) {
          const float4 v = win[j % S::WIN];
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }
#pragma unroll
        for (int j = j0; j < j0 + 6; ++j) {
          const int jn = j + S::WIN;
          win[j % S::WIN] = jn < S::CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - S::CP / 4));
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 24, 0);  // VALU x24
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);  // DS read x6
      }
    }
    NBS(const unsigned long long b0 = ccyc();)
    __syncthreads();
    NBS(sc_bar += ccyc() - b0;)
  }
  NBS(if (lane == 0 && wave == 0 && gridDim.x < 512) {
    g_nb_stamps[512 + blockIdx.x][30] = sc_bar;
    g_nb_stamps[512 + blockIdx.x][31] = nit;
  })
  NBS(if (lane == 0 && wave == 0 && gridDim.x < 512) {
    unsigned long long *st = g_nb_stamps[512 + blockIdx.x];
    st[8] = c_m0;
    st[9] = __builtin_amdgcn_s_memtime();
    st[10] = c_r0;
    st[11] = __builtin_amdgcn_s_memrealtime();
  })

  // ----------------------------------------------------------------- epilogue
  const int row = g * S::ROWS + crow;
  const int rows = B.j[ji].w.rows;
  const float *bias = B.j[ji].bias;
  float *y = B.j[ji].y;
  if (B.j[ji].epi == EPI_GELU_Q) {
    const bool ok = row < rows;
    float gv = 0.0f;
    if (ok) {
      gv = h2f(B.j[ji].gelu_tab[f2h(acc + bias[row])]);
      if (y) y[row] = gv;
    }
    const int blk = row / QK;
    quantize_half(gv, lane, ok, B.j[ji].oq_qs + (size_t)blk * 16, B.j[ji].oq_d + blk,
                  B.j[ji].oxd + (size_t)blk * QK);
  } else if (row < rows) {
    y[row] = bias ? acc + bias[row] : acc;
  }
  __builtin_amdgcn_s_setprio(0);
}

template <int CB, int PF, int CONS>
__global__ void __launch_bounds__((64 * SoloShape<CB, CONS>::WAVES), 1) k_gemv_solo(GemvBatch B) {
  __shared__ __attribute__((aligned(16))) float P[C5_RING][SoloShape<CB, CONS>::ROWS * SoloShape<CB, CONS>::LD];
  solo_body<CB, PF, CONS>(B, blockIdx.x, P);
}

static int solo_groups(const GemvBatch &B, int cons = 1) {
  int g = 0;
  for (int i = 0; i < B.nj; ++i) g += (B.j[i].w.tiles + 2 * cons - 1) / (2 * cons);
  return g;
}

// The exact GEMV of a batch: 64-row SIMD0-solo workgroups (k_gemv_solo: six producers of one
// block each, CB = 6, weights 3 chunks ahead in a register ring) when there are enough of
// them to cover the CUs, else 32-row workgroups (k_gemv_chain32: more CUs per row, for
// fc_out and the out-projection, whose K = 4E chains are the whole cost).
constexpr int SOLO_CB = 6, SOLO_PF = 3, SOLO_MIN_GROUPS = 192;

bool gemv_chain_solo(const GemvBatch &B) { return solo_groups(B) >= SOLO_MIN_GROUPS; }

int launch_gemv_chain_batch(const GemvBatch &B, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < B.nj; ++i) {
    if (B.j[i].w.k % QK != 0 || B.j[i].w.k <= 0) {
      set_error("gemv: K must be a positive multiple of 32");
      return VSIM_EINVAL;
    }
    if (!B.j[i].xd) { set_error("gemv: exact mode needs the activation factors xd"); return VSIM_EINVAL; }
    tiles += B.j[i].w.tiles;
  }
  if (tiles == 0) return VSIM_OK;
  if (gemv_chain_solo(B)) {
    hipLaunchKernelGGL((k_gemv_solo<SOLO_CB, SOLO_PF, 1>), dim3(solo_groups(B)), dim3(64 * SoloShape<SOLO_CB, 1>::WAVES),
                       0, s, B);
  } else {
    hipLaunchKernelGGL(k_gemv_chain32, dim3(tiles), dim3(C2Gemv::THREADS), 0, s, B);
  }
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim

#ifdef VSIM_NB_STAMPS
extern "C" int vsim_debug_nb_stamps(void *dst, size_t bytes) {
  if (bytes > sizeof(vsim::g_nb_stamps)) bytes = sizeof(vsim::g_nb_stamps);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(vsim::g_nb_stamps), bytes) == hipSuccess ? 0 : -2;
}
#endif
