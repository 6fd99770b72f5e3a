// vsim_amd/csrc/gemv_chain.hip — exact-mode Q4_0 GEMV (decode, one activation row).
//
// The reference dot (imax.c:1182-1230 / ggml.c:1471-1500) is one sequential fp32 chain per
// output row: sumf += f0*f2 + f1*f3 over the K/2 bytes of the row, every product and sum
// rounded separately.  The chain cannot be re-associated without changing the result, so
// the kernel is bounded by the dependent-add latency of the chain (≈7.8 cycles per add on
// gfx950, one chain per lane), not by HBM: K = 16384 is 8192 dependent adds ≈ 27 µs.  Every
// other cost is arranged to hide behind that chain.  One workgroup = 64 rows (two W4T32
// tiles) of one job:
//
//  * the consumer wave runs the 64 chains, one per lane: a lane reads its row's pair terms
//    from LDS (16-byte reads, a few ahead of the adds) and adds them in order;
//  * CH_NPW producer waves compute the pair terms, one block of the chunk each: 16 pairs
//    of one Q4_0 block for the 64 rows.  Nibbles and scales stream into an
//    LDS ring by LDS-DMA (global_load_lds), CH_DEPTH chunks ahead, and are read into
//    registers one chunk before use; the item's activation factors are wave-uniform and
//    come into SGPRs by scalar loads one chunk ahead.
//    Two producer waves share each SIMD (one wave alone issues VALU at ≈5 cycles per
//    instruction; a second wave nearly doubles the SIMD's rate), and a 128-pair chunk
//    amortizes the per-chunk barrier and wait latencies;
//  * a 3-slot LDS ring of pair terms, one s_barrier per chunk: in iteration k producers
//    fill chunk k while the consumer adds chunk k-2 (and reads ahead into chunk k-1).
//
// Epilogues: plain store (+bias), and fc_in's bias + GELU table + re-quantization of the
// 64 outputs into two blocks of the next product's Q4_0 activation (ggml.c:5024-5041).
#include <cstdlib>
#include <cstring>

#include "attn.hpp"
#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

// template CB: Q4_0 blocks per chunk = producer waves (one per block); a chunk is CB*16
// pairs per row, its LDS row stride CB*16+4 floats (conflict-free 16-byte access).  CB = 8
// (152 KB LDS, one workgroup per CU) for few rows, CB = 4 (77 KB, two per CU) for many.
constexpr int CH_RING = 3;               // pair-term ring slots
constexpr int CH_WIN = 8;                // consumer read-ahead (16-byte reads)
constexpr int CH_DEPTH = 4;              // LDS-DMA prefetch depth (chunks)
constexpr int CH_RAW = CH_DEPTH + 1;     // raw weight ring slots
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int WAIT_VM_DEPTH = 0x0F70 | (2 * (CH_DEPTH - 2));  // two DMA ops per chunk per wave

static_assert(CH_DEPTH >= 3 && 2 * (CH_DEPTH - 2) < 16, "vmcnt immediate");

typedef const __attribute__((address_space(4))) float sfloat;  // scalar-loaded

__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }

// Producer-side barrier without the lgkmcnt(0) of __syncthreads: it would also wait for the
// scalar loads of the next chunk's activation factors still in flight.  The pair terms
// written before it are first read by the consumer one whole chunk later (it reads chunk
// k-1 near the end of iteration k), and the slot reuse is guarded by the consumer's own
// full wait before its barrier.  The "memory" clobber keeps the compiler from moving the
// stores across.
__device__ __forceinline__ void producer_barrier() { asm volatile("s_barrier" ::: "memory"); }

// LDS-DMA: each lane's 16 (4) bytes from its own global address land lane-linearly at the
// wave-uniform LDS address.  Inline asm keeps the load out of the compiler's wait-count
// bookkeeping: completion is retired by the explicit vmcnt waits.  nt: streamed once.
__device__ __forceinline__ void glds16(const void *g, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void *g, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

struct ChainRows {
  const uint8_t *qs0, *qs1;  // nibble planes of the two 32-row tiles (qs1 null: absent)
  const float *d0, *d1;
  const float *x;            // dequantized activation factors, K floats
  int nb;                    // K/32
  int job, g;                // batch job (-1: grid tail), 64-row group within it
};

// Field-wise reads of the kernel arguments with wave-uniform indices (whole-struct copies
// make the compiler spill the argument block to private memory).
__device__ __forceinline__ void chain_rows(const GemvBatch &B, ChainRows &S) {
  S.nb = 0;
  S.job = -1;
  S.qs1 = nullptr;
  S.d1 = nullptr;
  int g = blockIdx.x, ji = 0;
  while (ji < B.nj) {
    const int ng = (B.j[ji].w.tiles + 1) / 2;
    if (g < ng) break;
    g -= ng;
    ++ji;
  }
  if (ji >= B.nj) return;
  ji = __builtin_amdgcn_readfirstlane(ji);
  const uint8_t *wqs = B.j[ji].w.qs;
  const float *wd = B.j[ji].w.d;
  const int tiles = B.j[ji].w.tiles, nb = B.j[ji].w.k / QK;
  S.x = B.j[ji].xd;
  S.job = ji;
  S.nb = nb;
  S.g = g;
  S.qs0 = wqs + (size_t)(2 * g) * nb * T32 * 16;
  S.d0 = wd + (size_t)(2 * g) * nb * T32;
  if (2 * g + 1 < tiles) {
    S.qs1 = wqs + (size_t)(2 * g + 1) * nb * T32 * 16;
    S.d1 = wd + (size_t)(2 * g + 1) * nb * T32;
  }
}

// timing experiment output (DBG & 8): [0..3] producer wave 0 of block 0, [4] iterations,
// [8..9] consumer of block 0 (cycles summed over iterations)
__device__ unsigned long long g_chain_prof[64];

// DBG (timing experiments only; results are wrong unless 0 or 8): bit0 = the consumer skips
// the adds, bit1 = producers skip the pair terms, bit2 = producers skip the LDS-DMA
template <int DBG, int CB>
__global__ void __launch_bounds__(64 * (1 + CB), 2) k_gemv_chain(GemvBatch B) {
  constexpr int CP = CB * 16, LD = CP + 4;
  __shared__ __attribute__((aligned(16))) float P[CH_RING][64 * LD];
  __shared__ __attribute__((aligned(16))) uint4 RQ[CH_RAW][CB][64];
  __shared__ __attribute__((aligned(16))) float RD[CH_RAW][CB][64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  ChainRows S;
  chain_rows(B, S);
  if (S.job < 0) return;  // whole workgroup: no barrier is reached
  const int nb = S.nb, nch = (nb + CB - 1) / CB;
  // iterations (one barrier each, after a prologue barrier): chunk k is produced in
  // iteration k and added in k+2; even count for the producers' two x register sets
  const int nit = (nch + 2 + 1) & ~1;

  if (wave > 0) {
    // ------------------------------------------------------------- producer
    // Step k issues everything for later chunks first and then computes: scalar loads of
    // the activation factors of chunk k+1, LDS reads of chunk k+1's raw block (landed before
    // the previous barrier), LDS-DMA of chunk k+DEPTH; then chunk k's pair terms from the
    // registers filled in step k-1 -> P; wait until this wave's DMA of chunk k+2 landed;
    // barrier (its lgkmcnt(0) retires this step's reads).
    const int p = wave - 1, o = p;
    const int r = lane & 31, h = lane >> 5;
    const bool tile_ok = h == 0 || S.qs1 != nullptr;
    const uint8_t *qs = (tile_ok && h ? S.qs1 : S.qs0) + (size_t)r * 16;
    const float *dd = (tile_ok && h ? S.d1 : S.d0) + r;
    int dslot = 0;  // raw slot of chunk k+DEPTH (advanced per step)
    auto dma = [&](int c, int slot) {  // chunk c, block clamped so every load stays in bounds
      const int b = min(c * CB + o, nb - 1);
      glds16(qs + (size_t)b * (T32 * 16), lds_addr(&RQ[slot][o][0]));
      glds4(dd + (size_t)b * T32, lds_addr(&RD[slot][o][0]));
    };
    auto ldx = [&](int c, f32x2 *xv) {  // this item's 32 activation factors (16 pairs)
      const int b = min(c * CB + o, nb - 1);
      const sfloat *xp = (const sfloat *)(S.x + (size_t)b * QK);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        xv[i].x = xp[2 * i];
        xv[i].y = xp[2 * i + 1];
      }
    };
    int rslot = 0;  // raw slot of chunk k+1
    auto ldraw = [&](int slot, uint4 &q, float &dq) {
      q = RQ[slot][o][lane];
      dq = RD[slot][o][lane];
    };
    const bool prof = (DBG & 8) && blockIdx.x == 0;
    unsigned long long pt[4] = {0, 0, 0, 0}, tp = 0;
    auto stamp = [&](int i) {
      if (DBG & 8) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (i >= 0) pt[i] += t - tp;
        tp = t;
      }
    };
    int ps = 0;  // P ring slot of chunk k
    // two sets of 32 SGPRs for the factors: chunk k+1's load at the top of step k, so their
    // latency falls into chunk k's compute instead of the barrier
    auto step = [&](int k, const f32x2 *x, const uint4 &qc, float dqc, uint4 &qn, float &dqn, f32x2 *xn) {
      stamp(-1);
      rslot = rslot == CH_RAW - 1 ? 0 : rslot + 1;
      ldraw(rslot, qn, dqn);
      ldx(k + 1, xn);
      if (!(DBG & 4)) dma(k + CH_DEPTH, dslot);
      dslot = dslot == CH_RAW - 1 ? 0 : dslot + 1;
      __builtin_amdgcn_sched_barrier(0);
      stamp(0);
      if (!(DBG & 2)) {
        const float dv = tile_ok && k * CB + o < nb ? dqc : 0.0f;
        const f32x2 d2 = {512.0f * dv, 512.0f * dv}, m2 = {-8.0f * dv, -8.0f * dv};
        float *dst = &P[ps][lane * LD + o * 16];
        const uint32_t qw[4] = {qc.x, qc.y, qc.z, qc.w};
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          float p4[4];
          pair_terms4_x(qw[wv], d2, m2, x + 4 * wv, p4);
          *(float4 *)(dst + 4 * wv) = make_float4(p4[0], p4[1], p4[2], p4[3]);
        }
      }
      ps = ps == CH_RING - 1 ? 0 : ps + 1;
      __builtin_amdgcn_sched_barrier(0);
      stamp(1);
      __builtin_amdgcn_s_waitcnt(WAIT_VM_DEPTH);  // this wave's DMA of chunk k+2 landed
      stamp(2);
      __syncthreads();
      stamp(3);
    };
#pragma unroll
    for (int c = 0; c < CH_DEPTH; ++c) dma(c, c);
    dslot = CH_DEPTH % CH_RAW;
    f32x2 xa[16], xb[16];
    uint4 qa, qb;
    float da, db;
    ldx(0, xa);
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" ::"s"(xa[i].x), "s"(xa[i].y));  // loaded before the loop
    __builtin_amdgcn_s_waitcnt(WAIT_VM_DEPTH);  // chunks 0 and 1 landed
    __syncthreads();
    ldraw(0, qa, da);
    __syncthreads();  // (second prologue barrier: the reads above are retired here)
    for (int k = 0; k < nit; k += 2) {
      step(k, xa, qa, da, qb, db, xb);
      step(k + 1, xb, qb, db, qa, da, xa);
    }
    if (prof && lane == 0) {
      for (int i = 0; i < 4; ++i) g_chain_prof[16 + 4 * p + i] = pt[i];
      if (p == 0) {
        for (int i = 0; i < 4; ++i) g_chain_prof[i] = pt[i];
        g_chain_prof[4] = nit;
      }
    }
    return;
  }

  // --------------------------------------------------------------- consumer
  // Rolling window of CH_WIN 16-byte LDS reads ahead of the chain (few registers, so two
  // workgroups fit per CU): iteration k adds chunk k-2 and, near its end, reads the first
  // window of chunk k-1 (published one barrier earlier; the 3-slot ring keeps both alive).
  float acc = 0.0f;
  float4 win[CH_WIN];
  auto src = [&](int c) { return &P[c % CH_RING][lane * LD]; };
  __builtin_amdgcn_s_setprio(3);  // the chain issues first whenever it is ready
  __syncthreads();  // prologue (producers: chunks 0 and 1 landed)
  __syncthreads();  // prologue (producers: raw chunk 0 in registers)
  unsigned long long ct[2] = {0, 0}, tc = 0;
  auto cstamp = [&](int i) {
    if (DBG & 8) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (i >= 0) ct[i] += t - tc;
      tc = t;
    }
  };
  for (int k = 0; k < nit; ++k) {
    cstamp(-1);
    const int c = k - 2;
    if (c == -1 && nch > 0) {
      const float *p0 = src(0);
#pragma unroll
      for (int j = 0; j < CH_WIN; ++j) win[j] = *(const float4 *)(p0 + 4 * j);
    } else if (c >= 0 && c < nch) {
      // groups pinned in order (4 adds, then the next read) so the scheduler cannot hoist the
      // reads into one burst with a full wait in front of the adds; the reads past the
      // chunk's end come from chunk c+1's slot (stale when c+1 == nch, never added)
      const float *pc = src(c), *pn = src(c + 1);
#pragma unroll
      for (int j = 0; j < CP / 4; ++j) {
        const float4 v = win[j % CH_WIN];
        if (!(DBG & 1)) {
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }
        const int jn = j + CH_WIN;
        win[j % CH_WIN] = jn < CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU x4
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read x1
      }
    }
    cstamp(0);
    __syncthreads();
    cstamp(1);
  }
  if ((DBG & 8) && blockIdx.x == 0 && lane == 0) {
    g_chain_prof[8] = ct[0];
    g_chain_prof[9] = ct[1];
  }

  // ----------------------------------------------------------------- epilogue
  const int ji = S.job;
  const int row = S.g * 64 + lane;
  const int rows = B.j[ji].w.rows;
  const float *bias = B.j[ji].bias;
  float *y = B.j[ji].y;
  if (B.j[ji].epi == EPI_GELU_Q) {
    const bool ok = row < rows;
    float g = 0.0f;
    if (ok) {
      g = h2f(B.j[ji].gelu_tab[f2h(acc + bias[row])]);
      if (y) y[row] = g;
    }
    const int blk = row / QK;
    quantize_half(g, lane, ok, B.j[ji].oq_qs + (size_t)blk * 16, B.j[ji].oq_d + blk,
                  B.j[ji].oxd + (size_t)blk * QK);
  } else if (row < rows) {
    y[row] = bias ? acc + bias[row] : acc;
  }
}

// ================================================================== 32-row variant
// Same chain and producer/consumer protocol for one W4T32 tile (32 rows) per workgroup, so a
// job with few rows spreads over more CUs (fc_out: 128 workgroups instead of 64) and each
// CU's producers carry half the work.  4 producer waves, each 2 blocks of the 8-block chunk
// (lanes 0-31: rows of block 2p, lanes 32-63: rows of block 2p+1); the activation factors
// then differ between the two half-waves, so they come through the LDS ring as well (one
// LDS-DMA per chunk by the first producer, read with per-half broadcast loads) instead of
// scalar loads.
constexpr int C2_CB = 8, C2_CP = C2_CB * 16, C2_LD = C2_CP + 4, C2_NPW = C2_CB / 2;
constexpr int C2_THREADS = 64 * (1 + C2_NPW);
constexpr int C2_RING = 3, C2_WIN = 8, C2_DEPTH = 4, C2_RAW = C2_DEPTH;  // raw slot reuse: see below
constexpr int C2_WAIT_VM3 = 0x0F70 | (3 * (C2_DEPTH - 2));  // wave 1: nibbles, scales, factors
constexpr int C2_WAIT_VM2 = 0x0F70 | (2 * (C2_DEPTH - 2));  // other producers: nibbles, scales
static_assert(3 * (C2_DEPTH - 2) < 16, "vmcnt immediate");

struct C2Lds {
  float P[C2_RING][32 * C2_LD];
  uint4 RQ[C2_RAW][C2_NPW][64];
  float RD[C2_RAW][C2_NPW][64];
  float RX[C2_RAW][C2_CB * QK];
};

// tile t of the batch's jobs (blockIdx.x in k_gemv_chain32, a role offset in k_layer_tail)
template <int DBG>
__device__ __forceinline__ void chain32_body(const GemvBatch &B, int t, C2Lds &L) {
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
  const int nb = B.j[ji].w.k / QK, nch = (nb + C2_CB - 1) / C2_CB;
  const int nit = (nch + 2 + 1) & ~1;
  const uint8_t *tqs = B.j[ji].w.qs + (size_t)t * nb * T32 * 16;
  const float *td = B.j[ji].w.d + (size_t)t * nb * T32;
  const float *x = B.j[ji].xd;

  if (wave > 0) {
    // ------------------------------------------------------------- producer
    // Step k (as in k_gemv_chain): read chunk k+1's raw block and factors (landed before the
    // previous barrier) into registers, LDS-DMA of chunk k+DEPTH, pair terms of chunk k from
    // the registers filled in step k-1, wait for this wave's DMA of chunk k+2, barrier.
    // Raw slot reuse: chunk c lives in slot c % RAW; the DMA of chunk k+DEPTH (step k) reuses
    // the slot of chunk k, whose registers were read in step k-1 (retired at that barrier).
    const int p = wave - 1, r = lane & 31, hb = lane >> 5;
    const int o = 2 * p + hb;  // this lane's block within the chunk
    const uint8_t *qs = tqs + (size_t)r * 16;
    const float *dd = td + r;
    auto dma = [&](int c) {
      const int slot = c % C2_RAW;
      const int b = min(c * C2_CB + o, nb - 1);
      glds16(qs + (size_t)b * (T32 * 16), lds_addr(&RQ[slot][p][0]));
      glds4(dd + (size_t)b * T32, lds_addr(&RD[slot][p][0]));
      if (p == 0) {  // the chunk's 8 x 32 activation factors, 16 bytes per lane (clamped block)
        const int bx = min(c * C2_CB + (lane >> 3), nb - 1);
        glds16(x + (size_t)bx * QK + 4 * (lane & 7), lds_addr(&RX[slot][0]));
      }
    };
    auto ldraw = [&](int c, uint4 &q, float &dq, f32x2 *xv) {
      const int slot = c % C2_RAW;
      q = RQ[slot][p][lane];
      dq = RD[slot][p][lane];
      const float4 *xp = (const float4 *)&RX[slot][o * QK];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 v = xp[i];
        xv[2 * i].x = v.x;
        xv[2 * i].y = v.y;
        xv[2 * i + 1].x = v.z;
        xv[2 * i + 1].y = v.w;
      }
    };
    int ps = 0;
    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const uint4 &qc, float dqc, uint4 &qn, float &dqn) {
      ldraw(k + 1, qn, dqn, xn);
      if (!(DBG & 4)) dma(k + C2_DEPTH);
      if (!(DBG & 2)) {
        const float dv = k * C2_CB + o < nb ? dqc : 0.0f;
        const f32x2 d2 = {512.0f * dv, 512.0f * dv}, m2 = {-8.0f * dv, -8.0f * dv};
        float *dst = &P[ps][r * C2_LD + o * 16];
        const uint32_t qw[4] = {qc.x, qc.y, qc.z, qc.w};
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          float p4[4];
          pair_terms4_x(qw[wv], d2, m2, xc + 4 * wv, p4);
          *(float4 *)(dst + 4 * wv) = make_float4(p4[0], p4[1], p4[2], p4[3]);
        }
      }
      ps = ps == C2_RING - 1 ? 0 : ps + 1;
      if (p == 0)  // this wave's DMA of chunk k+2 landed
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM3);
      else
        __builtin_amdgcn_s_waitcnt(C2_WAIT_VM2);
      __syncthreads();
    };
#pragma unroll
    for (int c = 0; c < C2_DEPTH; ++c) dma(c);
    f32x2 xa[16], xb[16];
    uint4 qa, qb;
    float da, db;
    if (p == 0)  // chunks 0 and 1 landed
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
  auto src = [&](int c) { return &P[c % C2_RING][lr * C2_LD]; };
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
      for (int j = 0; j < C2_CP / 4; ++j) {
        const float4 v = win[j % C2_WIN];
        if (!(DBG & 1)) {
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }
        const int jn = j + C2_WIN;
        win[j % C2_WIN] = jn < C2_CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - C2_CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
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

// ================================================================== 128-row variant
// Two consumer waves (rows 0-63 and 64-127 of the workgroup, on SIMD0 and SIMD1) and 12
// producer waves (three per SIMD: one wave alone issues VALU at ~1 per 5 cycles, three
// share a SIMD at ~1 per 2).  A chunk is C3_CB = 6 blocks; producer p computes block p % 6
// of row group p / 6.  With 128 rows in flight per CU a K = 4096 batch of up to 32768 rows
// (Q, K, V and fc_in of GPT-J: 28672) is a single round of workgroups, each CU running two
// chains at once instead of one.  The pair-term ring takes the whole LDS (3 x 128 rows x
// 100 floats), so nibbles and scales come straight from global memory into a register ring
// C3_PF chunks ahead (the compiler's own loads: its vmcnt bookkeeping waits only for the
// oldest set) and the activation factors by scalar loads one chunk ahead, as in
// k_gemv_chain.
constexpr int C3_CB = 6, C3_CP = C3_CB * 16, C3_LD = C3_CP + 4, C3_NP = 2 * C3_CB;
constexpr int C3_THREADS = 64 * (2 + C3_NP);
constexpr int C3_RING = 3, C3_WIN = 8, C3_PF = 3;  // register ring: C3_PF + 1 sets
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
typedef const __attribute__((address_space(1))) float gfloat;

template <int DBG>
__global__ void __launch_bounds__(C3_THREADS, 1) k_gemv_chain2(GemvBatch B) {
  __shared__ __attribute__((aligned(16))) float P[C3_RING][128 * C3_LD];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int g = blockIdx.x, ji = 0;
  while (ji < B.nj) {
    const int ng = (B.j[ji].w.tiles + 3) / 4;
    if (g < ng) break;
    g -= ng;
    ++ji;
  }
  if (ji >= B.nj) return;
  ji = __builtin_amdgcn_readfirstlane(ji);
  g = __builtin_amdgcn_readfirstlane(g);
  const int tiles = B.j[ji].w.tiles, nb = B.j[ji].w.k / QK, nch = (nb + C3_CB - 1) / C3_CB;
  // chunk k is produced in iteration k and added in k+2; a multiple of 4 for the producers'
  // unrolled register rings
  const int nit = (nch + 2 + 3) & ~3;

  if (wave >= 2) {
    // ------------------------------------------------------------- producer
    const int p = wave - 2, o = p % C3_CB, rg = p / C3_CB;
    const int h = lane >> 5, r = lane & 31;
    const int tile = 4 * g + 2 * rg + h;
    const bool tile_ok = tile < tiles;
    const int tl = tile_ok ? tile : tiles - 1;  // absent tile: in-bounds loads, zero terms
    const uint8_t *qs = B.j[ji].w.qs + ((size_t)tl * nb * T32 + r) * 16;
    const float *dd = B.j[ji].w.d + (size_t)tl * nb * T32 + r;
    const float *xg = B.j[ji].xd;
    auto ld = [&](int c, u32x4 &qv, float &dv) {
      const int b = min(c * C3_CB + o, nb - 1);
      qv = __builtin_nontemporal_load((gu32x4 *)(qs + (size_t)b * (T32 * 16)));
      dv = __builtin_nontemporal_load((gfloat *)(dd + (size_t)b * T32));
    };
    auto ldx = [&](int c, f32x2 *xv) {
      const int b = min(c * C3_CB + o, nb - 1);
      const sfloat *xp = (const sfloat *)(xg + (size_t)b * QK);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        xv[i].x = xp[2 * i];
        xv[i].y = xp[2 * i + 1];
      }
    };
    int ps = 0;
    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const u32x4 &qc, float dqc, u32x4 &qn, float &dqn) {
      ld(k + C3_PF, qn, dqn);  // the set of chunk k-1, used in the previous step
      ldx(k + 1, xn);
      __builtin_amdgcn_sched_barrier(0);
      if (!(DBG & 2)) {
        const float dv = tile_ok && k * C3_CB + o < nb ? dqc : 0.0f;
        // both halves of the broadcast pairs as real registers: with one half left undefined
        // the allocator may overlay it on a register whose global load is still in flight,
        // and the read of the pair then waits for that load
        const float dl = 512.0f * dv, ml = -8.0f * dv;
        float dh, mh;
        asm("v_mov_b32 %0, %1" : "=v"(dh) : "v"(dl));
        asm("v_mov_b32 %0, %1" : "=v"(mh) : "v"(ml));
        const f32x2 d2 = {dl, dh}, m2 = {ml, mh};
        float *dst = &P[ps][(rg * 64 + lane) * C3_LD + o * 16];
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          float p4[4];
          pair_terms4_x(qc[wv], d2, m2, xc + 4 * wv, p4);
          *(float4 *)(dst + 4 * wv) = make_float4(p4[0], p4[1], p4[2], p4[3]);
        }
      }
      ps = ps == C3_RING - 1 ? 0 : ps + 1;
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
    };
    u32x4 q0, q1, q2, q3;
    float e0, e1, e2, e3;
    ld(0, q0, e0);
    ld(1, q1, e1);
    ld(2, q2, e2);
    f32x2 xa[16], xb[16];
    ldx(0, xa);
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" ::"s"(xa[i].x), "s"(xa[i].y));  // loaded before the loop
    static_assert(C3_PF == 3, "register ring unrolled for 4 sets");
    for (int k = 0; k < nit; k += 4) {
      step(k, xa, xb, q0, e0, q3, e3);
      step(k + 1, xb, xa, q1, e1, q0, e0);
      step(k + 2, xa, xb, q2, e2, q1, e1);
      step(k + 3, xb, xa, q3, e3, q2, e2);
    }
    return;
  }

  // --------------------------------------------------------------- consumers
  const int rg = wave;
  float acc = 0.0f;
  float4 win[C3_WIN];
  auto src = [&](int c) { return &P[c % C3_RING][(rg * 64 + lane) * C3_LD]; };
  __builtin_amdgcn_s_setprio(3);
  for (int k = 0; k < nit; ++k) {
    const int c = k - 2;
    if (c == -1 && nch > 0) {
      const float *p0 = src(0);
#pragma unroll
      for (int j = 0; j < C3_WIN; ++j) win[j] = *(const float4 *)(p0 + 4 * j);
    } else if (c >= 0 && c < nch) {
      const float *pc = src(c), *pn = src(c + 1);
#pragma unroll
      for (int j = 0; j < C3_CP / 4; ++j) {
        const float4 v = win[j % C3_WIN];
        if (!(DBG & 1)) {
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }
        const int jn = j + C3_WIN;
        win[j % C3_WIN] = jn < C3_CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - C3_CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU x4
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read x1
      }
    }
    __syncthreads();
  }

  // ----------------------------------------------------------------- epilogue
  const int row = (4 * g + 2 * rg) * T32 + lane;
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
}

template <int DBG>
__global__ void __launch_bounds__(C2_THREADS, 2) k_gemv_chain32(GemvBatch B) {
  __shared__ C2Lds L;
  chain32_body<DBG>(B, blockIdx.x, L);
}

// ================================================================== fused layer tail
// fc_out, the attention heads and the out-projection of one layer in one launch, so the
// attention and the out-projection run beside fc_out, whose K = 4E chain is the layer's
// longest dependency, instead of before it.  Roles by workgroup index:
//   [0, nf)          fc_out tiles (32-row chain GEMV)
//   [nf, nf + H)     attention heads (attn.hpp with this kernel's 5 waves); each head
//                    releases its output and counts itself in *done (agent scope)
//   [nf + H, ...)    out-projection tiles; wait until *done == H, then acquire
// Waiting workgroups only wait for lower-indexed ones, which the dispatcher has already
// placed, so the wait always ends.  *done is zeroed by the layer's LayerNorm kernel.
struct TailJob {
  GemvBatch f, o;
  AttnJob a;
  unsigned *done;
  int nf;
};

__global__ void __launch_bounds__(C2_THREADS, 1) k_layer_tail(TailJob T) {
  __shared__ union {
    C2Lds g;
    float a[sizeof(C2Lds) / sizeof(float)];
  } L;
  int b = blockIdx.x;
  if (b < T.nf) {
    chain32_body<0>(T.f, b, L.g);
    return;
  }
  b -= T.nf;
  const int na = T.a.H * (T.a.nsplit > 1 ? T.a.nsplit : 1);
  if (b < na) {
    attn_body<C2_THREADS>(T.a, b, L.a);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every wave's output stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(T.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  b -= na;
  if (threadIdx.x == 0)
    while (__hip_atomic_load(T.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)na)
      __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  chain32_body<0>(T.o, b, L.g);
}

int launch_layer_tail(const GemvBatch &f, const GemvBatch &o, const AttnJob &a, unsigned *done, int n_ctx,
                      hipStream_t s) {
  const int S = a.nsplit > 1 ? a.nsplit : 1;
  if (a.d % 32 != 0 || a.d > 256 || a.n_ctx != n_ctx || a.d % S != 0 || (a.d / S) % QK != 0 ||
      (size_t)attn_lds_floats(a.d, n_ctx) * sizeof(float) > sizeof(C2Lds)) {
    set_error("layer tail: attention shape (head dim, n_ctx) outside the fused kernel's range");
    return VSIM_EINVAL;
  }
  TailJob T;
  T.f = f;
  T.o = o;
  T.a = a;
  T.done = done;
  T.nf = 0;
  for (int i = 0; i < f.nj; ++i) T.nf += f.j[i].w.tiles;
  int no = 0;
  for (int i = 0; i < o.nj; ++i) no += o.j[i].w.tiles;
  // dynamic LDS pad: above half the CU's LDS, so one workgroup per CU (fc_out's consumer
  // keeps its SIMD); the out-projection tiles that find no CU start as attention heads end
  hipLaunchKernelGGL(k_layer_tail, dim3(T.nf + a.H * S + no), dim3(C2_THREADS), 8192, s, T);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// ================================================================== 64-row, SIMD0 solo
// For jobs whose chains are the whole cost (fc_out: K = 16384 over only 4096 rows): the
// consumer wave alone on SIMD0 (producers sharing its SIMD stretch each dependent add by a
// VALU slot), CB producer waves on SIMD1-3, one Q4_0 block of the chunk for the 64 rows
// each, so the activation factors are wave-uniform scalar loads and the LDS carries
// nothing but pair terms.  Waves the hardware would place on SIMD0 (4, 8, ...) only join
// the barriers.  Weights: register ring as k_gemv_chain2.
template <int CB>
struct SoloShape {
  static constexpr int CP = CB * 16, LD = CP + 4;
  static constexpr int WAVES = 1 + CB + (CB - 1) / 3;  // consumer, producers, SIMD0 fillers
  static constexpr int WIN = CP / 4 % 8 == 0 ? 8 : 12;
  static_assert(CP / 4 % WIN == 0, "the read window must tile the chunk");
  static_assert(WAVES <= 16, "workgroup size");
};
constexpr int C5_RING = 3;

// PF: prefetch distance of the weight loads in chunks (register ring of PF+1 sets)
// One 64-row group g of batch B (groups numbered job by job); P: the pair-term ring.
// Every wave returns from here (producers and fillers early); all take nit barriers.
template <int DBG, int CB, int PF, bool CO = false>
__device__ __forceinline__ void solo_body(const GemvBatch &B, int g, float (*P)[64 * SoloShape<CB>::LD]) {
  using S = SoloShape<CB>;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  int ji = 0;
  while (ji < B.nj) {
    const int ng = (B.j[ji].w.tiles + 1) / 2;
    if (g < ng) break;
    g -= ng;
    ++ji;
  }
  if (ji >= B.nj) return;
  ji = __builtin_amdgcn_readfirstlane(ji);
  g = __builtin_amdgcn_readfirstlane(g);
  const int tiles = B.j[ji].w.tiles, nb = B.j[ji].w.k / QK, nch = (nb + CB - 1) / CB;
  const int nit = (nch + 2 + PF) / (PF + 1) * (PF + 1);

  if (wave != 0 && (wave & 3) == 0) {  // SIMD0 filler
    for (int k = 0; k < nit; ++k) __syncthreads();
    return;
  }
  if (wave > 0) {
    // ------------------------------------------------------------- producer
    const int o = wave - 1 - (wave >> 2);  // 1,2,3,5,6,7,9,... -> 0,1,2,...
    const int h = lane >> 5, r = lane & 31;
    const int tile = 2 * g + h;
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
    unsigned long long pt[4] = {0, 0, 0, 0}, tp = 0;
    auto stamp = [&](int i) {
      if (DBG & 8) {
        const unsigned long long tt = __builtin_amdgcn_s_memtime();
        if (i >= 0) pt[i] += tt - tp;
        tp = tt;
      }
    };
    auto step = [&](int k, const f32x2 *xc, f32x2 *xn, const u32x4 &qc, float dqc, u32x4 &qn, float &dqn) {
      stamp(-1);
      ld(k + PF, qn, dqn);
      // this chunk's factors (loaded a whole step ago) before the next chunk's loads go out:
      // scalar loads return out of order, so any later wait for them would be lgkmcnt(0)
      // and would also wait for the loads just issued
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
      stamp(0);
      ldx(k + 1, xn);
      __builtin_amdgcn_sched_barrier(0);
      if (!(DBG & 2)) {
        const float dv = tile_ok && k * CB + o < nb ? dqc : 0.0f;
        const float dl = 512.0f * dv, ml = -8.0f * dv;
        float dh, mh;
        asm("v_mov_b32 %0, %1" : "=v"(dh) : "v"(dl));  // see k_gemv_chain2
        asm("v_mov_b32 %0, %1" : "=v"(mh) : "v"(ml));
        const f32x2 d2 = {dl, dh}, m2 = {ml, mh};
        float *dst = &P[ps][lane * S::LD + o * 16];
#pragma unroll
        for (int wv = 0; wv < 4; ++wv) {
          float p4[4];
          pair_terms4_x(qc[wv], d2, m2, xc + 4 * wv, p4);
          *(float4 *)(dst + 4 * wv) = make_float4(p4[0], p4[1], p4[2], p4[3]);
        }
      }
      ps = ps == C5_RING - 1 ? 0 : ps + 1;
      __builtin_amdgcn_sched_barrier(0);
      stamp(1);
      if (DBG & 4)
        __syncthreads();
      else
        producer_barrier();
      stamp(2);
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
    if ((DBG & 8) && blockIdx.x == 0 && lane == 0) {
      for (int i = 0; i < 3; ++i) g_chain_prof[16 + 4 * o + i] = pt[i];
      if (o == 0) g_chain_prof[4] = nit;
    }
    return;
  }

  // --------------------------------------------------------------- consumer
  float acc = 0.0f;
  float4 win[S::WIN];
  auto src = [&](int c) { return &P[c % C5_RING][lane * S::LD]; };
  __builtin_amdgcn_s_setprio(3);
  unsigned long long ct[2] = {0, 0}, tc = 0;
  auto cstamp = [&](int i) {
    if (DBG & 8) {
      const unsigned long long tt = __builtin_amdgcn_s_memtime();
      if (i >= 0) ct[i] += tt - tc;
      tc = tt;
    }
  };
  for (int k = 0; k < nit; ++k) {
    cstamp(-1);
    const int c = k - 2;
    if (c == -1 && nch > 0) {
      const float *p0 = src(0);
#pragma unroll
      for (int j = 0; j < S::WIN; ++j) win[j] = *(const float4 *)(p0 + 4 * j);
    } else if (c >= 0 && c < nch) {
      const float *pc = src(c), *pn = src(c + 1);
#pragma unroll
      for (int j = 0; j < S::CP / 4; ++j) {
        const float4 v = win[j % S::WIN];
        if (!(DBG & 1)) {
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
        }
        const int jn = j + S::WIN;
        win[j % S::WIN] = jn < S::CP / 4 ? *(const float4 *)(pc + 4 * jn) : *(const float4 *)(pn + 4 * (jn - S::CP / 4));
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU x4
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read x1
      }
    }
    cstamp(0);
    __syncthreads();
    cstamp(1);
  }
  if ((DBG & 8) && blockIdx.x == 0 && lane == 0) {
    g_chain_prof[8] = ct[0];
    g_chain_prof[9] = ct[1];
  }

  // ----------------------------------------------------------------- epilogue
  const int row = g * 64 + lane;
  const int rows = B.j[ji].w.rows;
  const float *bias = B.j[ji].bias;
  float *y = B.j[ji].y;
  if (B.j[ji].epi == EPI_GELU_Q) {
    const bool ok = row < rows;
    float gv = 0.0f;
    if (ok) {
      gv = h2f(B.j[ji].gelu_tab[f2h(acc + bias[row])]);
      if (y) st_out<CO>(y + row, gv);
    }
    const int blk = row / QK;
    quantize_half<CO>(gv, lane, ok, B.j[ji].oq_qs + (size_t)blk * 16, B.j[ji].oq_d + blk,
                  B.j[ji].oxd + (size_t)blk * QK);
  } else if (row < rows) {
    st_out<CO>(y + row, bias ? acc + bias[row] : acc);
  }
  __builtin_amdgcn_s_setprio(0);
}

template <int DBG, int CB, int PF>
__global__ void __launch_bounds__(64 * SoloShape<CB>::WAVES, 1) k_gemv_solo(GemvBatch B) {
  __shared__ __attribute__((aligned(16))) float P[C5_RING][64 * SoloShape<CB>::LD];
  // (timing experiments: DBG 16 / 32 raise the kernel's VGPR count to 144 / 104)
  if (DBG & 16) asm volatile("v_mov_b32 v143, 0" ::: "v143");
  if (DBG & 32) asm volatile("v_mov_b32 v103, 0" ::: "v103");
  solo_body<DBG & 15, CB, PF>(B, blockIdx.x, P);
}

// ================================================================== one launch per layer
// An exact decode layer in one grid, so that fc_out's K = 4E chain (the layer's longest
// dependency) starts as soon as fc_in's chains end and the attention branch fills the CUs
// beside it.  Segments in grid order:
//   ln  (join of the previous layer +) LayerNorm(s) + quantize, 8 workgroups per norm
//                                                                   -> counts cnt[192]
//   in  fc_in (+ bias, GELU, requantize), 64-row solo groups: wait cnt[192] == n_ln
//                                                                   -> counts cnt[0]
//   f   fc_out: waits cnt[0] == n_in; solo groups or 32-row tiles
//   q   Q, K, V, 64-row solo groups: wait cnt[192] == n_ln          -> counts cnt[64]
//   a   attention heads: wait cnt[64] == n_q                        -> count cnt[128]
//   o   out-projection, 32-row tiles: waits cnt[128] == n_a
// (qfirst: q before f; n_ln == 0: the LayerNorm ran as its own launch.)  A segment waits
// only on lower-indexed workgroups, which the dispatcher has placed before it, so every
// wait ends.  The counters are zeroed before the launch (a memset node per token).  Segments of 32-row tiles and heads use
// the first C2_THREADS threads; the other waves leave at once (s_barrier then counts only
// the waves still running).  A producer segment releases its stores at agent scope before
// it counts; a waiting one acquires after its wait.  The activation factors read by a
// waiting solo segment's scalar loads were written in this launch, but no workgroup reads
// them before its wait, so the scalar cache holds no stale copy.
extern unsigned *g_norm_stats;
constexpr int LX_CB = 6, LX_PF = 3;
constexpr int LX_THREADS = 64 * SoloShape<LX_CB>::WAVES;
static_assert(LX_THREADS >= C2_THREADS, "tile segments run on the first C2_THREADS threads");
struct LayerExactJob {
  GemvBatch in, f, q, o;
  AttnJob a;
  LnQuantJob ln[2];  // the layer's LayerNorm(s) (+ the previous layer's join), n_ln > 0
  unsigned *stats;   // LayerNorm fallback counters (g_norm_stats)
  unsigned *cnt;
  int n_ln, ln_n, n_in, n_f, n_q, n_a, fsolo, qfirst;
  int dbg;  // VSIM_LX_DBG (timing experiments): skip the work of in 1, f 2, q 4, a 8, o 16
};
union LxLds {
  float s[C5_RING][64 * SoloShape<LX_CB>::LD];
  C2Lds g;
};

// Hand-offs (cdna_hip_programming.md §6 Guideline 16, counter form): producers store their
// outputs sc1 (st_out<true>), every wave drains its stores, one lane adds to the counter; a
// consumer polls relaxed in one lane, then ONE agent acquire (this CU's L1) before the barrier.
// (A release fence per producer workgroup, i.e. an L2 write-back each, made this launch 2x
// slower than the three-launch layer.)  Consumer loads of handed-off bytes: vector loads
// behind the acquire, and fc_out's scalar factor loads, which no workgroup issues before
// its wait in this launch (the scalar cache starts the launch empty).
// acq = false: the segment reads the handed-off bytes only by scalar loads (the solo
// producers' activation factors), which the L1 acquire does not concern.
__device__ __forceinline__ void lx_wait(const unsigned *c, unsigned target, bool acq = true) {
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0)
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(4);
    if (acq) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
}
__device__ __forceinline__ void lx_count(unsigned *c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 output stores
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(LX_THREADS, 1) k_layer_exact(LayerExactJob T) {
  __shared__ __attribute__((aligned(16))) LxLds L;
  const int wave = threadIdx.x >> 6;
  int b = blockIdx.x;
  if (b < T.n_ln) {  // k_ln_quant's body (layer.hip), outputs stored sc1
    const int part = b % 8;
    const LnQuantJob &J = T.ln[b / 8];
    const int n = T.ln_n, nb = n / QK, lane = threadIdx.x & 63;
    const int b0 = part * nb / 8, b1 = (part + 1) * nb / 8;
    float *row = (float *)&L;
    ln_exact_lds_t<LX_THREADS>(J.x, row, n, J.w, J.b, part == 0 ? T.stats : nullptr, J.ja, J.jab, J.jf, J.jfb,
                               J.jout, nullptr, b0 * QK / 4, b1 * QK / 4);
    for (int b2 = wave; b0 + 2 * b2 < b1; b2 += LX_THREADS / 64) {
      const int bb = b0 + 2 * b2 + (lane >> 5);
      const bool ok = bb < b1;
      const float v = ok ? row[bb * QK + (lane & 31)] : 0.0f;
      quantize_half<true>(v, lane, ok, J.qs + (size_t)bb * 16, J.d + bb, J.xd + (size_t)bb * QK);
    }
    lx_count(T.cnt + 192);
    return;
  }
  b -= T.n_ln;
  if (b < T.n_in) {
    if (T.n_ln) lx_wait(T.cnt + 192, (unsigned)T.n_ln, false);
    if (!(T.dbg & 1)) solo_body<0, LX_CB, LX_PF, true>(T.in, b, L.s);
    lx_count(T.cnt);
    return;
  }
  b -= T.n_in;
  const int nf = T.n_f, nq = T.n_q;
  const bool is_f = T.qfirst ? (b >= nq && b < nq + nf) : b < nf;
  const bool is_q = T.qfirst ? b < nq : (b >= nf && b < nf + nq);
  if (is_f) {
    b -= T.qfirst ? nq : 0;
    if (T.n_in > 0) lx_wait(T.cnt, (unsigned)T.n_in, !T.fsolo);
    if (T.dbg & 2) {
    } else if (T.fsolo) {
      solo_body<0, LX_CB, LX_PF>(T.f, b, L.s);
    } else if (wave < C2_THREADS / 64) {
      chain32_body<0>(T.f, b, L.g);
    }
    return;
  }
  if (is_q) {
    b -= T.qfirst ? 0 : nf;
    if (T.n_ln) lx_wait(T.cnt + 192, (unsigned)T.n_ln, false);
    if (!(T.dbg & 4)) solo_body<0, LX_CB, LX_PF, true>(T.q, b, L.s);
    lx_count(T.cnt + 64);
    return;
  }
  b -= nf + nq;
  if (wave >= C2_THREADS / 64) return;
  if (b < T.n_a) {
    lx_wait(T.cnt + 64, (unsigned)nq);
    if (!(T.dbg & 8)) attn_body<C2_THREADS, true>(T.a, b, (float *)&L);
    lx_count(T.cnt + 128);
    return;
  }
  b -= T.n_a;
  lx_wait(T.cnt + 128, (unsigned)T.n_a);
  if (!(T.dbg & 16)) chain32_body<0>(T.o, b, L.g);
}

static int solo_groups(const GemvBatch &B) {
  int g = 0;
  for (int i = 0; i < B.nj; ++i) g += (B.j[i].w.tiles + 1) / 2;
  return g;
}
static int batch_tiles(const GemvBatch &B) {
  int t = 0;
  for (int i = 0; i < B.nj; ++i) t += B.j[i].w.tiles;
  return t;
}

int launch_layer_exact(const LnQuantJob *ln, int n_ln, const GemvBatch &in, const GemvBatch &f, const GemvBatch &q,
                       const GemvBatch &o, const AttnJob &a, unsigned *cnt, int n_ctx, int fsolo, int qfirst,
                       hipStream_t s) {
  const int S = a.nsplit > 1 ? a.nsplit : 1;
  if (a.d % 32 != 0 || a.d > 256 || a.n_ctx != n_ctx || a.d % S != 0 || (a.d / S) % QK != 0 ||
      (size_t)attn_lds_floats(a.d, n_ctx) * sizeof(float) > sizeof(LxLds)) {
    set_error("layer kernel: attention shape (head dim, n_ctx) outside the fused kernel's range");
    return VSIM_EINVAL;
  }
  for (const GemvBatch *B : {&in, &f, &q, &o})
    for (int i = 0; i < B->nj; ++i)
      if (B->j[i].w.k % QK != 0 || B->j[i].w.k <= 0 || !B->j[i].xd) {
        set_error("layer kernel: K must be a positive multiple of 32 and the activation factors set");
        return VSIM_EINVAL;
      }
  LayerExactJob T;
  T.n_ln = 8 * n_ln;
  T.ln_n = n_ln ? in.j[0].w.k : 0;
  for (int i = 0; i < 2; ++i) T.ln[i] = n_ln ? ln[i < n_ln ? i : 0] : LnQuantJob{};
  T.stats = g_norm_stats;
  if (n_ln && (in.nj != 1 || (size_t)T.ln_n * sizeof(float) > sizeof(LxLds) || T.ln_n % QK != 0)) {
    set_error("layer kernel: the LayerNorm segment needs fc_in in the launch and E within the LDS row");
    return VSIM_EINVAL;
  }
  T.in = in;
  T.f = f;
  T.q = q;
  T.o = o;
  T.a = a;
  T.cnt = cnt;
  T.n_in = solo_groups(in);
  T.n_f = fsolo ? solo_groups(f) : batch_tiles(f);
  T.n_q = solo_groups(q);
  T.n_a = a.H * S;
  T.fsolo = fsolo;
  T.qfirst = qfirst;
  static const int dbg = [] {
    const char *e = getenv("VSIM_LX_DBG");
    return e ? atoi(e) : 0;
  }();
  T.dbg = dbg;
  const int grid = T.n_ln + T.n_in + T.n_f + T.n_q + T.n_a + batch_tiles(o);
  hipLaunchKernelGGL(k_layer_exact, dim3(grid), dim3(LX_THREADS), 0, s, T);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

template <int DBG>
static void chain_launch_t(int grid, const GemvBatch &B, hipStream_t s) {
  // (CB = 4 at two workgroups per CU measured slower than CB = 8 at one: the producers'
  // VALU issue per CU, not the grid's rounds, bounds the large batches.  Replacing the
  // per-chunk barriers by LDS full/free counters was bit-exact but 10-20% slower.)
  hipLaunchKernelGGL((k_gemv_chain<DBG, 8>), dim3(grid), dim3(64 * 9), 0, s, B);
}

int launch_gemv_chain_batch(const GemvBatch &B, hipStream_t s) {
  int groups = 0;
  for (int i = 0; i < B.nj; ++i) {
    if (B.j[i].w.k % QK != 0 || B.j[i].w.k <= 0) {
      set_error("gemv: K must be a positive multiple of 32");
      return VSIM_EINVAL;
    }
    if (!B.j[i].xd) { set_error("gemv: exact mode needs the activation factors xd"); return VSIM_EINVAL; }
    groups += (B.j[i].w.tiles + 1) / 2;
  }
  if (groups == 0) return VSIM_OK;
  static const int variant = [] {
    const char *e = getenv("VSIM_CHAIN_ROWS");
    return e ? atoi(e) : 0;
  }();
  int tiles = 0, g128 = 0;
  for (int i = 0; i < B.nj; ++i) {
    tiles += B.j[i].w.tiles;
    g128 += (B.j[i].w.tiles + 3) / 4;
  }
  // The widest variant whose grid still covers most of the 256 CUs: 128-row workgroups
  // (two chains per CU) for large batches, 64-row, else 32-row (more CUs per row).
  // VSIM_CHAIN_ROWS=32|64|128 forces one.
  // default: 64-row SIMD0-solo workgroups when there are enough of them to cover the CUs,
  // else 32-row ones (more CUs per row: fc_out and the out-projection)
  const int rows_per_wg = variant ? variant : groups >= 192 ? 640 : 32;
  const bool narrow = rows_per_wg == 32;
  static const int dbg = [] {
    const char *e = getenv("VSIM_CHAIN_DBG");
    return e ? atoi(e) : 0;
  }();
  static const int solo_env = [] {  // VSIM_SOLO=6|9: the 64-row SIMD0-solo kernel for every batch
    const char *e = getenv("VSIM_SOLO");
    return e ? atoi(e) : 0;
  }();
  const int solo_cb = solo_env ? solo_env : rows_per_wg == 640 ? 6 : 0;
  if (solo_cb) {
    static const int pf = [] {
      const char *e = getenv("VSIM_SOLO_PF");
      return e ? atoi(e) : 3;
    }();
    static const size_t solo_pad = [] {  // VSIM_SOLO_PAD=bytes: dynamic LDS pad (occupancy experiments)
      const char *e = getenv("VSIM_SOLO_PAD");
      return e ? (size_t)atol(e) : (size_t)0;
    }();
#define C5L(D, CB, PF) \
  hipLaunchKernelGGL((k_gemv_solo<D, CB, PF>), dim3(groups), dim3(64 * SoloShape<CB>::WAVES), solo_pad, s, B)
    if (solo_cb == 9) {
      if (pf == 7) C5L(0, 9, 7); else C5L(0, 9, 3);
    } else {
      if (pf == 7) {
        if (dbg == 1) C5L(1, 6, 7); else if (dbg == 2) C5L(2, 6, 7); else C5L(0, 6, 7);
      } else if (pf == 5) {
        C5L(0, 6, 5);
      } else {
        if (dbg == 1) C5L(1, 6, 3); else if (dbg == 2) C5L(2, 6, 3); else if (dbg == 4) C5L(4, 6, 3);
        else if (dbg == 8) C5L(8, 6, 3); else if (dbg == 9) C5L(9, 6, 3);
        else if (dbg == 16) C5L(16, 6, 3); else if (dbg == 32) C5L(32, 6, 3); else C5L(0, 6, 3);
      }
    }
#undef C5L
    VSIM_HIP(hipGetLastError());
    return VSIM_OK;
  }
  if (narrow) {
    switch (dbg) {
      case 1: hipLaunchKernelGGL(k_gemv_chain32<1>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
      case 2: hipLaunchKernelGGL(k_gemv_chain32<2>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
      case 4: hipLaunchKernelGGL(k_gemv_chain32<4>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
      case 5: hipLaunchKernelGGL(k_gemv_chain32<5>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
      case 6: hipLaunchKernelGGL(k_gemv_chain32<6>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
      case 7: hipLaunchKernelGGL(k_gemv_chain32<7>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
      default: hipLaunchKernelGGL(k_gemv_chain32<0>, dim3(tiles), dim3(C2_THREADS), 0, s, B); break;
    }
    VSIM_HIP(hipGetLastError());
    return VSIM_OK;
  }
  if (rows_per_wg == 128) {
    switch (dbg) {
      case 1: hipLaunchKernelGGL(k_gemv_chain2<1>, dim3(g128), dim3(C3_THREADS), 0, s, B); break;
      case 2: hipLaunchKernelGGL(k_gemv_chain2<2>, dim3(g128), dim3(C3_THREADS), 0, s, B); break;
      default: hipLaunchKernelGGL(k_gemv_chain2<0>, dim3(g128), dim3(C3_THREADS), 0, s, B); break;
    }
    VSIM_HIP(hipGetLastError());
    return VSIM_OK;
  }
  switch (dbg) {
    case 1: chain_launch_t<1>(groups, B, s); break;
    case 2: chain_launch_t<2>(groups, B, s); break;
    case 3: chain_launch_t<3>(groups, B, s); break;
    case 4: chain_launch_t<4>(groups, B, s); break;
    case 5: chain_launch_t<5>(groups, B, s); break;
    case 7: chain_launch_t<7>(groups, B, s); break;
    case 10: chain_launch_t<10>(groups, B, s); break;
    case 12: chain_launch_t<12>(groups, B, s); break;
    case 8: chain_launch_t<8>(groups, B, s); break;
    default: chain_launch_t<0>(groups, B, s); break;
  }
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim

// timing-experiment readout (tools/gemv_bench.py); not part of include/vsim_hip.h
extern "C" int vsim_debug_chain_prof(unsigned long long *out64) {
  return hipMemcpyFromSymbol(out64, HIP_SYMBOL(vsim::g_chain_prof), 64 * sizeof(unsigned long long)) == hipSuccess
             ? 0 : -1;
}
