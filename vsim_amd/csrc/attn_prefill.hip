// vsim_amd/csrc/attn_prefill.hip — prompt (prefill) attention on fp16 MFMA, fast mode.
//
// For N > 1 tokens at n_past, the reference computes KQ = K·Q (ggml.c:4495-4534), scale,
// causal mask (key > n_past + query -> -inf), softmax over the keys (5825-5893) and
// KQV = V·softmax (4535-4581) per head.  This kernel does the same in one pass with an
// online softmax (flash attention): no [H][N][n_past+N] score tensor, K and V read once
// per 128 queries.  It is the throughput path for long prompts (codegen-16B, N = 2048),
// in the fast mode with the fp16 MFMA GEMM (gemm_f16.hip); exact mode keeps the
// reference-order kernels of ops_attn.hip.
//
// One workgroup = one head x 128 queries, 4 waves of 32 queries; keys in blocks of 64.
//  * S^T = K·Q^T on v_mfma_f32_32x32x16_f16: keys are the tile's rows (in registers),
//    queries its columns (one per lane), so each query's softmax statistics are a
//    reduction over the lane's own registers plus one exchange with lane ^ 32.  Q comes
//    pre-scaled by scale * log2(e) (fp16 fragments in registers for the whole loop), so
//    p = exp2(s - max).
//  * O^T += V^T·P^T: P^T is the S^T accumulator itself, converted to fp16 in place -- the
//    MFMA operand that sums over the accumulator's row index needs no lane movement
//    (cdna_hip_programming.md §3); V is staged transposed in LDS with the matching k
//    order.  O^T (head dim x 32 queries) lives in the accumulator registers.
#include <mutex>

#include "kern.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

typedef _Float16 ahalf8 __attribute__((ext_vector_type(8)));
typedef _Float16 ahalf4 __attribute__((ext_vector_type(4)));
typedef float af32x16 __attribute__((ext_vector_type(16)));

constexpr int AP_BQ = 128, AP_BK = 64, AP_THREADS = 256;

// Keys [0, nk) of this layer's F32 cache as fp16, once per prompt eval: K16[key][E]
// (row-major, as the cache) and Vt16[h][dim][ldt] (each head's V transposed, keys padded
// with zeros to ldt, a multiple of AP_BK), so the attention workgroups stage both operand
// tiles with 16-byte loads and stores.  64 keys x 64 columns per workgroup; V goes through
// an LDS tile for the transpose.
// Keys [f0, f1) are skipped (already written by the K / V GEMM epilogues).
__global__ void __launch_bounds__(256) k_kv_f16(const float *__restrict__ kc, const float *__restrict__ vc, int E,
                                                 int d, int nk, int ldt, _Float16 *__restrict__ k16,
                                                 _Float16 *__restrict__ vt16, int f0, int f1) {
  __shared__ float tv[64][65];
  const int key0 = blockIdx.x * 64, col0 = blockIdx.y * 64;
  if (key0 >= f0 && key0 + 64 <= f1) return;  // (a block of fresh keys only)
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * 16; e += 256) {  // 64 keys x 16 float4 columns
    const int kk = e / 16, c4 = (e % 16) * 4, key = key0 + kk;
    float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
    if (key < nk && (key < f0 || key >= f1)) {
      kv = *(const float4 *)(kc + (size_t)key * E + col0 + c4);
      vv = *(const float4 *)(vc + (size_t)key * E + col0 + c4);
      ahalf4 hk = {(_Float16)kv.x, (_Float16)kv.y, (_Float16)kv.z, (_Float16)kv.w};
      *(ahalf4 *)(k16 + (size_t)key * E + col0 + c4) = hk;
    }
    tv[kk][c4] = vv.x;
    tv[kk][c4 + 1] = vv.y;
    tv[kk][c4 + 2] = vv.z;
    tv[kk][c4 + 3] = vv.w;
  }
  __syncthreads();
  for (int e = tid; e < 64 * 16; e += 256) {  // 64 columns x 16 groups of 4 keys
    const int cc = e / 16, k4 = (e % 16) * 4;
    const int col = col0 + cc, h = col / d, dim = col % d;
    ahalf4 hv = {(_Float16)tv[k4][cc], (_Float16)tv[k4 + 1][cc], (_Float16)tv[k4 + 2][cc], (_Float16)tv[k4 + 3][cc]};
    _Float16 *dst = vt16 + ((size_t)h * d + dim) * ldt;  // (keys in vt_pos order: a quad stays whole)
    const int k = key0 + k4;
    if (k + 4 <= f0 || k >= f1) {
      if (k < ldt) *(ahalf4 *)(dst + vt_pos(k)) = hv;
    } else {  // (a group that straddles the fresh range)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((k + j < f0 || k + j >= f1) && k + j < ldt) dst[vt_pos(k + j)] = hv[j];
    }
  }
}

// One workgroup = one head x 128 queries (4 waves of 32), keys in tiles of 64 through two
// LDS buffers: the next tile's fp16 K rows and V^T rows load into registers (16-byte
// chunks) while the current tile's MFMAs run.  Workgroups are ordered longest causal range
// first (query block descending, heads interleaved) so the long ones do not start last.
template <int D>
__global__ void __launch_bounds__(AP_THREADS) k_attn_prefill_f16(const float *__restrict__ Q,
                                                                  const _Float16 *__restrict__ k16,
                                                                  const _Float16 *__restrict__ vt16, int E, int H,
                                                                  int N, int n_past, int ldt, float qscale,
                                                                  float *__restrict__ out) {
  constexpr int KLD = D + 8;      // K tile [key][dim], halves
  constexpr int VLD = AP_BK + 8;  // V^T tile [dim][key], halves
  constexpr int NT = D / 32;      // O^T tiles (32 dims each)
  constexpr int KCH = AP_BK * D / 8 / AP_THREADS;  // 16-byte chunks per thread per operand tile
  extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
  // buffer b: K tile at lds + b * AP_BK * KLD, V^T tile at lds + 2 * AP_BK * KLD + b * D * VLD
  const int nqb = (N + AP_BQ - 1) / AP_BQ;
  const int h = blockIdx.x % H, q0 = (nqb - 1 - (int)blockIdx.x / H) * AP_BQ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hl = lane >> 5;
  const int qw = q0 + wave * 32;  // this wave's first query
  const int myq = qw + r;         // this lane's query (column of S^T / O^T)
  const _Float16 *kbase = k16 + (size_t)h * D, *vbase = vt16 + (size_t)h * D * ldt;

  // Q^T fragments: lane (query r, half hl) holds Q[q][16s + 8hl + j], j < 8, for every s
  ahalf8 qf[D / 16];
  {
    const float *qr = Q + (size_t)min(myq, N - 1) * E + h * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const float4 a = *(const float4 *)(qr + 16 * s + 8 * hl), b = *(const float4 *)(qr + 16 * s + 8 * hl + 4);
      ahalf8 f;
      f[0] = (_Float16)(a.x * qscale);
      f[1] = (_Float16)(a.y * qscale);
      f[2] = (_Float16)(a.z * qscale);
      f[3] = (_Float16)(a.w * qscale);
      f[4] = (_Float16)(b.x * qscale);
      f[5] = (_Float16)(b.y * qscale);
      f[6] = (_Float16)(b.z * qscale);
      f[7] = (_Float16)(b.w * qscale);
      qf[s] = f;
    }
  }
  af32x16 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = (af32x16){};
  float mrow = -INFINITY, lrow = 0.0f;

  const int klast = n_past + min(q0 + AP_BQ, N) - 1;  // last key any query of the block sees
  const int nkb = klast / AP_BK + 1;
  // tile staging: chunk c of thread t = 16 bytes; K: key c8 / (D/8), dims 8 * (c8 % (D/8));
  // V^T: dim c8 / 8, keys 8 * (c8 % 8)
  u32x4 rk[KCH], rv[KCH];
  auto kload = [&](int kb) __attribute__((always_inline)) {
    const int k0 = kb * AP_BK;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      const int c8 = tid + AP_THREADS * c;
      const int key = k0 + c8 / (D / 8), col = 8 * (c8 % (D / 8));
      rk[c] = *(const u32x4 *)(kbase + (size_t)min(key, klast) * E + col);
    }
  };
  auto vload = [&](int kb) __attribute__((always_inline)) {
    const int k0 = kb * AP_BK;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      const int c8 = tid + AP_THREADS * c;
      rv[c] = *(const u32x4 *)(vbase + (size_t)(c8 / 8) * ldt + k0 + 8 * (c8 % 8));
    }
  };
  auto kstore = [&](int buf) __attribute__((always_inline)) {
    _Float16 *Ks = lds + buf * AP_BK * KLD;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      const int c8 = tid + AP_THREADS * c;
      *(u32x4 *)&Ks[(c8 / (D / 8)) * KLD + 8 * (c8 % (D / 8))] = rk[c];
    }
  };
  auto vstore = [&](int buf) __attribute__((always_inline)) {
    _Float16 *Vt = lds + 2 * AP_BK * KLD + buf * D * VLD;
#pragma unroll
    for (int c = 0; c < KCH; ++c) {
      const int c8 = tid + AP_THREADS * c;
      *(u32x4 *)&Vt[(c8 / 8) * VLD + 8 * (c8 % 8)] = rv[c];
    }
  };
  kload(0);
  vload(0);
  kstore(0);
  vstore(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * AP_BK, buf = kb & 1;
    const bool next = kb + 1 < nkb;
    // next tile: K rows load during this tile's S^T, V^T rows during its P·V
    if (next) kload(kb + 1);
    const _Float16 *Ks = lds + buf * AP_BK * KLD;
    const _Float16 *Vt = lds + 2 * AP_BK * KLD + buf * D * VLD;
    const bool vis = k0 <= n_past + min(qw + 31, N - 1);  // wave-uniform: some key of the block is visible
    af32x16 st[2];
    if (vis) {
      // S^T tiles t = 0, 1 (keys k0 + 32t + row)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        st[t] = (af32x16){};
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          const int krow = 32 * t + r;
          const ahalf8 kf = *(const ahalf8 *)&Ks[krow * KLD + 16 * s + 8 * hl];
          st[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[s], st[t], 0, 0, 0);
        }
      }
    }
    if (next) {
      kstore(buf ^ 1);
      vload(kb + 1);
    }
    if (vis) {
      // causal mask and the block maximum of this lane's query
      float bm = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int key = k0 + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * hl;
          if (key > n_past + myq) st[t][g] = -INFINITY;
          bm = fmaxf(bm, st[t][g]);
        }
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mnew = fmaxf(mrow, bm);
      const float alpha = mnew == -INFINITY ? 1.0f : exp2f(mrow - mnew);
      float ls = 0.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const float p = st[t][g] == -INFINITY ? 0.0f : exp2f(st[t][g] - mnew);
          st[t][g] = p;
          ls += p;
        }
      ls += __shfl_xor(ls, 32, 64);
      lrow = lrow * alpha + ls;
      mrow = mnew;
#pragma unroll
      for (int i = 0; i < NT; ++i) o[i] = o[i] * alpha;
      // O^T += V^T · P^T: k-step s2 of tile t covers keys 32t + 16s2 + 8(j>>2) + 4hl + (j&3)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          ahalf8 pf;
#pragma unroll
          for (int j = 0; j < 8; ++j) pf[j] = (_Float16)st[t][8 * s2 + j];
          const int kbase2 = 32 * t + 16 * s2 + 4 * hl;
#pragma unroll
          for (int i = 0; i < NT; ++i) {
            const int vrow = 32 * i + r, vc = kbase2 >> 3;  // (kbase2 & 7 == 4 hl: within the chunk)
            // (vt_pos order: the lane's keys kbase2 .. +3 and kbase2 + 8 .. +11 are chunk vc + hl)
            const ahalf8 vf = *(const ahalf8 *)&Vt[vrow * VLD + 8 * (vc + hl)];
            o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf, o[i], 0, 0, 0);
          }
        }
    }
    if (next) vstore(buf ^ 1);
    __syncthreads();
  }
  // O^T / l: lane = query, rows = dims (reg & 3) + 8 (reg >> 2) + 4 hl of tile i
  if (myq < N) {
    const float inv = 1.0f / lrow;
    float *orow = out + (size_t)myq * E + h * D;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * i + 8 * g + 4 * hl;
        *(float4 *)(orow + dd) = make_float4(o[i][4 * g] * inv, o[i][4 * g + 1] * inv, o[i][4 * g + 2] * inv,
                                             o[i][4 * g + 3] * inv);
      }
  }
}

// D = 256, two waves per query group: k_attn_prefill_f16 at D = 256 holds a 32-query group's
// Q fragments (64 VGPRs), its 256 x 32 O^T accumulators (128) and both S^T tiles in one wave,
// 472 registers: one wave per SIMD, every latency exposed.  Here a workgroup is 8 waves for
// the same 128 queries; waves g and g + 4 share query group g and split each 64-key block:
//  * S^T: wave half c computes keys 32 c .. 32 c + 31 (one 32 x 32 tile, 16 MFMAs over D);
//  * the block maximum of each query goes through LDS to the partner, so both take the same
//    new running maximum and rescale factor (the same operations on the same values);
//  * each wave turns its tile into P^T (the next MFMA's B operand, as above) and stores it
//    for the partner (lane-linear: the partner's lane l needs exactly lane l's values);
//  * O^T: wave half c accumulates dims 128 c .. 128 c + 127 over all 64 keys (4 tiles x 4
//    K-steps: its own P^T for its keys, the partner's for the others).
// Each wave keeps the running sum of its own keys' probabilities; the two partial sums are
// added (half 0's first) at the end.  ≈190 registers: two waves per SIMD.  Barriers per key
// block: after the maxima, after the P^T stores, after the next tile's DMA (as above).
constexpr int AP_KPF = 4;  // K fragments in flight in the S^T chain
constexpr int AP2_THREADS = 512;
constexpr size_t ap2_lds() { return (size_t)2 * 2 * AP_BK * 256 * sizeof(_Float16) + 4 * 2 * 2 * 64 * 16 + 4 * 2 * 64 * 4; }

__global__ void __launch_bounds__(AP2_THREADS, 1) k_attn_prefill_pair(const float *__restrict__ Q,
                                                                       const _Float16 *__restrict__ k16,
                                                                       const _Float16 *__restrict__ vt16, int E, int H,
                                                                       int N, int n_past, int ldt, float qscale,
                                                                       float *__restrict__ out,
                                                                       _Float16 *__restrict__ out16) {
  constexpr int D = 256;
  extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
  // [0, 128 KB): K and V^T tiles, two buffers each (as k_attn_prefill_f16's D = 256 path);
  // then the P^T exchange [group][half][s2][lane] (16 B) and the maxima / sums [group][half][lane]
  u32x4 *pex = (u32x4 *)(lds + 2 * 2 * AP_BK * D);
  float *mex = (float *)(pex + 4 * 2 * 2 * 64);
  const int nqb = (N + AP_BQ - 1) / AP_BQ;
  const int h = blockIdx.x % H, q0 = (nqb - 1 - (int)blockIdx.x / H) * AP_BQ;
  const int tid = threadIdx.x, lane = tid & 63;
  // pair (2 g, 2 g + 1) takes query group g; groups 0, 1 (waves 0-3, one per SIMD) lead, groups
  // 2, 3 (waves 4-7) run one barrier behind, so the two waves on a SIMD are
  // in different phases: one's softmax beside the other's MFMAs
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), grp = wv >> 1, half = wv & 1;
  const bool lag = wv >= 4;
  const int r = lane & 31, hl = lane >> 5;
  const int qw = q0 + grp * 32;
  const int myq = qw + r;
  const _Float16 *kbase = k16 + (size_t)h * D, *vbase = vt16 + (size_t)h * D * ldt;
  ahalf8 qf[D / 16];
  {
    const float *qr = Q + (size_t)min(myq, N - 1) * E + h * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const float4 a = *(const float4 *)(qr + 16 * s + 8 * hl), b = *(const float4 *)(qr + 16 * s + 8 * hl + 4);
      ahalf8 f;
      f[0] = (_Float16)(a.x * qscale);
      f[1] = (_Float16)(a.y * qscale);
      f[2] = (_Float16)(a.z * qscale);
      f[3] = (_Float16)(a.w * qscale);
      f[4] = (_Float16)(b.x * qscale);
      f[5] = (_Float16)(b.y * qscale);
      f[6] = (_Float16)(b.z * qscale);
      f[7] = (_Float16)(b.w * qscale);
      qf[s] = f;
    }
  }
  af32x16 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (af32x16){};
  float mrow = -INFINITY, lrow = 0.0f;
  const int klast = n_past + min(q0 + AP_BQ, N) - 1;
  const int nkb = klast / AP_BK + 1;
  const uint32_t lb = lds_addr(lds);
  // K(kb) into K buffer kb & 1, V^T(kb) into V buffer kb & 1: each wave 4 LDS-DMAs per tile
  auto stage_k = [&](int kb) __attribute__((always_inline)) {
    const int k0 = kb * AP_BK, buf = kb & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // 2 rows (keys) per wave instruction
      const int row0 = (j * 8 + wv) * 2, row = row0 + (lane >> 5);
      const int c = (lane & 31) ^ (row & 15);
      glds16<false>(kbase + (size_t)min(k0 + row, klast) * E + 8 * c,
                    lb + (uint32_t)((buf * AP_BK * D + row0 * D) * 2));
    }
  };
  auto stage_v = [&](int kb) __attribute__((always_inline)) {
    const int k0 = kb * AP_BK, buf = kb & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // 8 rows (dims) per wave instruction
      const int row0 = (j * 8 + wv) * 8, row = row0 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      glds16<false>(vbase + (size_t)row * ldt + k0 + 8 * c,
                    lb + (uint32_t)((2 * AP_BK * D + buf * D * AP_BK + row0 * AP_BK) * 2));
    }
  };
  // Tiles 0 and 1 up front; then K(kb+2) is issued at the start of PV(kb) (its buffer's last
  // reader is S(kb), one phase earlier even for the lagging group) and waited for at the end of
  // SM(kb+1); V(kb+1) at the start of SM(kb) (last reader PV(kb-1)), waited for at the end of
  // S(kb+1).  In issue order V(kb+1) follows K(kb+1) and K(kb+2) follows V(kb+1), so each wait
  // leaves the one later tile (4 DMAs) in flight.
  stage_k(0);
  stage_v(0);
  if (nkb > 1) {
    stage_k(1);
    stage_v(1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (lag) __builtin_amdgcn_s_barrier();
  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * AP_BK, buf = kb & 1;
    const _Float16 *Ks = lds + buf * AP_BK * D;
    const _Float16 *Vt = lds + 2 * AP_BK * D + buf * D * AP_BK;
    const bool vis = k0 <= n_past + min(qw + 31, N - 1);  // uniform over the pair
    // ---- S(kb): S^T of this wave's 32 keys, the block maximum to the partner
    af32x16 st = (af32x16){};
    if (vis) {
      // K fragments AP_KPF steps ahead of their MFMA (LDS latency behind the chain)
      const int krow = 32 * half + r;
      auto kfrag = [&](int s) { return *(const ahalf8 *)&Ks[krow * D + 8 * ((2 * s + hl) ^ (krow & 15))]; };
      ahalf8 kf[AP_KPF];
#pragma unroll
      for (int s = 0; s < AP_KPF; ++s) kf[s] = kfrag(s);
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        st = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[s % AP_KPF], qf[s], st, 0, 0, 0);
        if (s + AP_KPF < D / 16) kf[s % AP_KPF] = kfrag(s + AP_KPF);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      }
      float bm = -INFINITY;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int key = k0 + 32 * half + (g & 3) + 8 * (g >> 2) + 4 * hl;
        if (key > n_past + myq) st[g] = -INFINITY;
        bm = fmaxf(bm, st[g]);
      }
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      mex[(grp * 2 + half) * 64 + lane] = bm;
    }
    if (kb >= 2) {  // this wave's V(kb) DMAs
      if (kb + 1 < nkb)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // ---- SM(kb): the pair's common maximum, P^T of this wave's keys to the partner
    if (kb >= 1 && kb + 1 < nkb) stage_v(kb + 1);
    if (vis) {
      const float mnew = fmaxf(mrow, fmaxf(mex[(grp * 2) * 64 + lane], mex[(grp * 2 + 1) * 64 + lane]));
      const float alpha = mnew == -INFINITY ? 1.0f : exp2f(mrow - mnew);
      float ls = 0.0f;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float pv = st[g] == -INFINITY ? 0.0f : exp2f(st[g] - mnew);
        st[g] = pv;
        ls += pv;
      }
      ls += __shfl_xor(ls, 32, 64);
      lrow = lrow * alpha + ls;
      mrow = mnew;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = o[i] * alpha;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        ahalf8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (_Float16)st[8 * s2 + j];
        pex[((grp * 2 + half) * 2 + s2) * 64 + lane] = *(const u32x4 *)&pf;
      }
    }
    if (kb >= 1 && kb + 1 < nkb) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // this wave's K(kb+1) DMAs
    __syncthreads();
    // ---- PV(kb): O^T dims 128 half + 32 i, keys 32 t + 16 s2 + ...: P^T of tile t from wave half t
    if (kb + 2 < nkb) stage_k(kb + 2);
    if (vis) {
      // step u = 2 t + s2 (16 keys): P^T from wave half t, V fragments of the 4 dim tiles;
      // step u + 1's operands load while step u's 4 MFMAs run
      auto pfrag = [&](int u) {
        const u32x4 pw = pex[((grp * 2 + (u >> 1)) * 2 + (u & 1)) * 64 + lane];
        return *(const ahalf8 *)&pw;
      };
      auto vfrag = [&](int u, int i) {  // (vt_pos order: the lane's 8 keys are chunk 2 u + hl)
        const int vrow = 128 * half + 32 * i + r;
        return *(const ahalf8 *)&Vt[vrow * AP_BK + 8 * ((2 * u + hl) ^ ((vrow >> 1) & 7))];
      };
      ahalf8 pf[2], vf[2][4];
      pf[0] = pfrag(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) vf[0][i] = vfrag(0, i);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u + 1 < 4) {
          pf[(u + 1) & 1] = pfrag(u + 1);
#pragma unroll
          for (int i = 0; i < 4; ++i) vf[(u + 1) & 1][i] = vfrag(u + 1, i);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf[u & 1][i], pf[u & 1], o[i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
  }
  if (!lag) __builtin_amdgcn_s_barrier();  // (pairs with the lagging group's last)
  // the running sums of both halves (half 0's + half 1's, in that order, in both waves)
  mex[(grp * 2 + half) * 64 + lane] = lrow;
  __syncthreads();
  const float lt = mex[(grp * 2) * 64 + lane] + mex[(grp * 2 + 1) * 64 + lane];
  const float inv = 1.0f / lt;
  if (out16) {
    // the wo GEMM's fp16 operand straight from here: quantize_row_q4_0 per 32 dims of the
    // query's row, the values d*(q-8) as fp16 -- k_act_quant_f16's arithmetic on the same f32
    // values (dims 32 i .. 32 i + 31 of this half: 16 in this lane, 16 in lane ^ 32)
    _Float16 *qrow = out16 + (size_t)min(myq, N - 1) * E + h * D + 128 * half;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[16], amax = 0.0f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        v[k] = o[i][k] * inv;
        amax = amax > fabsf(v[k]) ? amax : fabsf(v[k]);
      }
      const float ao = __shfl_xor(amax, 32, 64);
      amax = amax > ao ? amax : ao;
      const float d = amax / 7.0f;
      const float id = d != 0.0f ? 1.0f / d : 0.0f;
      if (myq < N) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          ahalf4 hq;
#pragma unroll
          for (int e = 0; e < 4; ++e) hq[e] = f16_of_product(d, (float)x86_round_i8(v[4 * g + e] * id));
          *(ahalf4 *)(qrow + 32 * i + 8 * g + 4 * hl) = hq;
        }
      }
    }
    return;
  }
  if (myq < N) {
    float *orow = out + (size_t)myq * E + h * D + 128 * half;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * i + 8 * g + 4 * hl;
        *(float4 *)(orow + dd) = make_float4(o[i][4 * g] * inv, o[i][4 * g + 1] * inv, o[i][4 * g + 2] * inv,
                                             o[i][4 * g + 3] * inv);
      }
  }
}

bool attn_prefill_supported(int d) { return d == 64 || d == 96 || d == 128 || d == 256; }
// (head dim 256: the two-wave kernel, which also writes the out-projection's fp16 operand)
bool attn_prefill_quantizes(int d) { return d == 256; }

template <int D>
size_t attn_prefill_lds() {
  return (size_t)(2 * AP_BK * (D + 8) + 2 * D * (AP_BK + 8)) * sizeof(_Float16);
}

int attn_prefill_ldt(int nk) { return (nk + AP_BK - 1) / AP_BK * AP_BK; }
_Float16 *attn_prefill_k16(void *scratch, int E, int nk) { return (_Float16 *)scratch; }
_Float16 *attn_prefill_vt16(void *scratch, int E, int nk) {
  return (_Float16 *)scratch + (size_t)attn_prefill_ldt(nk) * E;
}

int launch_attn_prefill_f16(const float *Q, const float *kc, const float *vc, int d, int H, int N, int n_past,
                            float scale, float *out, hipStream_t s, void *scratch, size_t scratch_bytes, bool fresh,
                            void *out16) {
  if (!attn_prefill_supported(d)) {
    set_error("attention prefill: head dim must be 64, 96, 128 or 256");
    return VSIM_EINVAL;
  }
  if (out16 && !attn_prefill_quantizes(d)) {
    set_error("attention prefill: the quantized fp16 output needs head dim 256");
    return VSIM_EINVAL;
  }
  const int E = d * H, nk = n_past + N;
  if (E % 64) {  // k_kv_f16 copies 64-column tiles: a partial last tile would be left unwritten
    set_error("attention prefill: n_embd must be a multiple of 64");
    return VSIM_EINVAL;
  }
  const int ldt = attn_prefill_ldt(nk);
  const size_t need = attn_prefill_scratch(E, nk);
  _Float16 *buf = (_Float16 *)scratch;
  const bool own = !buf || scratch_bytes < need;
  if (own && fresh) {
    set_error("attention prefill: fresh keys need the caller's scratch");
    return VSIM_EINVAL;
  }
  if (own) VSIM_HIP(hipMallocAsync((void **)&buf, need, s));
  _Float16 *k16 = attn_prefill_k16(buf, E, nk), *vt16 = attn_prefill_vt16(buf, E, nk);
  const int f0 = fresh ? n_past : 0, f1 = fresh ? nk : 0;  // keys already converted
  if (!(fresh && n_past == 0 && nk == ldt))  // (else every key is fresh and there is no padding)
    hipLaunchKernelGGL(k_kv_f16, dim3(ldt / 64, E / 64), dim3(256), 0, s, kc, vc, E, d, nk, ldt, k16, vt16, f0, f1);
  const float qscale = scale * 1.4426950408889634f;  // exp(x) = exp2(x * log2 e)
  const dim3 grid(((N + AP_BQ - 1) / AP_BQ) * H);
  if (d == 256) {
    if (int rc = attn_prefill_prepare()) return rc;
    hipLaunchKernelGGL(k_attn_prefill_pair, grid, dim3(AP2_THREADS), ap2_lds(), s, Q, k16, vt16, E, H, N, n_past, ldt,
                       qscale, out, (_Float16 *)out16);
    VSIM_HIP(hipGetLastError());
    if (own) VSIM_HIP(hipFreeAsync(buf, s));
    return VSIM_OK;
  }
#define APL(DD)                                                                                                   \
  hipLaunchKernelGGL(k_attn_prefill_f16<DD>, grid, dim3(AP_THREADS), attn_prefill_lds<DD>(), s, Q, k16, vt16, E, H, \
                     N, n_past, ldt, qscale, out)
  switch (d) {
    case 64: APL(64); break;
    case 96: APL(96); break;
    default: APL(128); break;
  }
#undef APL
  VSIM_HIP(hipGetLastError());
  if (own) VSIM_HIP(hipFreeAsync(buf, s));
  return VSIM_OK;
}

// the pair kernel's LDS attribute, once per process; the other instances' attributes are read
// so that their code object is loaded before a timed prompt (vsim_model_reserve)
int attn_prefill_prepare() {
  static std::once_flag once;
  static int rc = VSIM_OK;
  std::call_once(once, [] {
    hipFuncAttributes fa;
    if (hipFuncSetAttribute((const void *)k_attn_prefill_pair, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)ap2_lds()) != hipSuccess ||
        hipFuncGetAttributes(&fa, (const void *)k_attn_prefill_f16<64>) != hipSuccess ||
        hipFuncGetAttributes(&fa, (const void *)k_attn_prefill_f16<96>) != hipSuccess ||
        hipFuncGetAttributes(&fa, (const void *)k_attn_prefill_f16<128>) != hipSuccess ||
        hipFuncGetAttributes(&fa, (const void *)k_kv_f16) != hipSuccess) {
      set_error("attention prefill: kernel attributes refused");
      rc = VSIM_EHIP;
    }
  });
  return rc;
}

size_t attn_prefill_scratch(int E, int nk) {
  const size_t ldt = (size_t)(nk + AP_BK - 1) / AP_BK * AP_BK;
  return 2 * ldt * E * sizeof(_Float16);
}

}  // namespace vsim
