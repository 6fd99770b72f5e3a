// vsim_amd/csrc/attn.hpp — single-token attention for one head (used by k_attn_decode in
// layer.hip and by the fused layer tail in gemv_chain.hip).
//
// Per head: RoPE on q and the new k, KV-cache write, KQ (double accumulator), scale/softmax
// (fp16 exp table), KQV (sequential float mad), quantization of the head's output for the
// out-projection.  Every value with the reference's operation order and rounding.
#pragma once

#include "kern.hpp"

namespace vsim {

// (diagnostic builds define ATT_STAMP(i) to stamp the phases of a head; nothing otherwise)
#ifndef ATT_STAMP
#define ATT_STAMP(i)
#endif

// One workgroup per head.  KQ: 16 lanes per key (four keys per wave instruction, KB
// steps loaded at once), products over the head dimension summed as a tree in double; the
// reference's sequential double sum lies within 2*d*2^-53*sum|p| of it, so when both ends of
// that interval round to the same float the score is the reference's, otherwise the key is
// redone sequentially by one lane (ggml.c:4760-4800 for the f32 dot with a double
// accumulator).  KQV keeps the reference's sequential float chain over the keys, one chain
// per output element; the V rows stream through LDS tiles, three tiles in flight.
constexpr int ATT_KB = 4;       // KQ: four-key steps per wave per load batch
constexpr int ATT_DPL = 4;      // max float4 of the head dimension per lane in KQ (d <= 256)

// One head (h) per workgroup of NT >= d threads; sm: attn_lds_floats(d, n_ctx) floats of LDS.
// Work item hs = head * S + part, S = A.nsplit (>= 1): every part computes the head's scores
// and softmax (identical in each), then the KQV chains and quantization of output columns
// [part*c, part*c + c), c = d / S, so a head's V rows spread over S CUs.  Every part writes
// the same new K/V cache row (identical bytes) before reading it back.
template <int NT, bool CO = false>
__device__ __forceinline__ void attn_body(const AttnJob &A, int hs, float *sm) {
  constexpr int ATT_THREADS = NT, ATT_WAVES = NT / 64;
  const int S = A.nsplit > 1 ? A.nsplit : 1, h = hs / S, part = hs % S;
  const int d = A.d, E = A.d * A.H, c = d / S, c0 = part * c;
  const int n_past = *A.npast;
  const int nk = n_past + 1;
  float *qh = sm;           // [d]
  float *kh = sm + d;       // [d]
  float *pr = sm + 2 * d;   // [nk] scores / probabilities
  __shared__ float shf[ATT_WAVES];
  __shared__ double shd[ATT_WAVES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < d; i += ATT_THREADS) {
    qh[i] = A.q[h * d + i];
    kh[i] = A.k[h * d + i];
    A.vc[(size_t)n_past * E + h * d + i] = A.v[h * d + i];
  }
  __syncthreads();
  // RoPE (ggml.c:6117-6152 / 5952-5973), position p = n_past for both q (mode 0) and k
  const int half = A.n_rot / 2;
  for (int j = tid; j < half; j += ATT_THREADS) {
    const double2 c = A.cs[(size_t)n_past * half + j];
    const int i0 = A.style == 0 ? j : 2 * j, i1 = A.style == 0 ? j + half : 2 * j + 1;
    const double q0 = qh[i0], q1 = qh[i1], k0 = kh[i0], k1 = kh[i1];
    if (A.style == 0) {
      qh[i0] = (float)(c.x * q0 - c.y * q1);
      qh[i1] = (float)(c.x * q1 + c.y * q0);
      kh[i0] = (float)(c.x * k0 - c.y * k1);
      kh[i1] = (float)(c.x * k1 + c.y * k0);
    } else {
      qh[i0] = (float)(q0 * c.x - q1 * c.y);
      qh[i1] = (float)(q0 * c.y + q1 * c.x);
      kh[i0] = (float)(k0 * c.x - k1 * c.y);
      kh[i1] = (float)(k0 * c.y + k1 * c.x);
    }
  }
  __syncthreads();
  for (int i = tid; i < d; i += ATT_THREADS) A.kc[(size_t)n_past * E + h * d + i] = kh[i];
  // The new key's row is read back below by whichever wave holds key n_past (wave n_past/16 %
  // waves), not only by the threads that stored it: the barrier (its release drains the stores)
  // orders them.  r05: until then that read raced the store whenever n_past >= 16.
  __syncthreads();
  ATT_STAMP(0);
  // KQ[k] = (float) sum_i (double)(K[k][i] * q[i]) in order i = 0..d-1; then * scale.
  // Row r (lanes 16r..16r+15) of a wave takes one key per step; lane l16 covers the float4s
  // at 4*l16 + 64*e of the head dimension.  A wave loads ATT_KB steps (4*ATT_KB keys) at once.
  float mx = -INFINITY;
  {
    const int row = lane >> 4, l16 = lane & 15;
    float4 q4[ATT_DPL];
#pragma unroll
    for (int e = 0; e < ATT_DPL; ++e) {
      const int i = 4 * l16 + 64 * e;
      q4[e] = i < d ? *(const float4 *)(qh + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int k0 = wid * 4 * ATT_KB; k0 < nk; k0 += ATT_WAVES * 4 * ATT_KB) {
      float4 kv[ATT_KB][ATT_DPL];
#pragma unroll
      for (int j = 0; j < ATT_KB; ++j) {
        const int k = min(k0 + 4 * j + row, nk - 1);
        const float *kr = A.kc + (size_t)k * E + h * d;
#pragma unroll
        for (int e = 0; e < ATT_DPL; ++e) {
          const int i = 4 * l16 + 64 * e;
          kv[j][e] = i < d ? *(const float4 *)(kr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < ATT_KB; ++j) {
        const int k = k0 + 4 * j + row;
        double t = 0.0, ta = 0.0;
#pragma unroll
        for (int e = 0; e < ATT_DPL; ++e) {
          const double p0 = (double)(kv[j][e].x * q4[e].x), p1 = (double)(kv[j][e].y * q4[e].y);
          const double p2 = (double)(kv[j][e].z * q4[e].z), p3 = (double)(kv[j][e].w * q4[e].w);
          t += (p0 + p1) + (p2 + p3);
          ta += (fabs(p0) + fabs(p1)) + (fabs(p2) + fabs(p3));
        }
        // sum over the row's 16 lanes (every lane of the row ends with the total)
        auto add = [](double a, double b) { return a + b; };
        t = add(t, dpp::mov<dpp::QP_XOR1, 0xF>(t, 0.0));
        ta = add(ta, dpp::mov<dpp::QP_XOR1, 0xF>(ta, 0.0));
        t = add(t, dpp::mov<dpp::QP_XOR2, 0xF>(t, 0.0));
        ta = add(ta, dpp::mov<dpp::QP_XOR2, 0xF>(ta, 0.0));
        t = add(t, dpp::mov<dpp::HALF_MIRROR, 0xF>(t, 0.0));
        ta = add(ta, dpp::mov<dpp::HALF_MIRROR, 0xF>(ta, 0.0));
        t = add(t, dpp::mov<dpp::MIRROR, 0xF>(t, 0.0));
        ta = add(ta, dpp::mov<dpp::MIRROR, 0xF>(ta, 0.0));
        const double bnd = 2.0 * d * 0x1.0p-53 * ta;
        float sc = (float)(t - bnd);
        if (k < nk && sc != (float)(t + bnd)) {  // row-uniform: redo this key in the reference order
          if (l16 == 0) {
            const float *kr = A.kc + (size_t)k * E + h * d;
            double acc = 0.0;
            for (int i = 0; i < d; ++i) acc += (double)(kr[i] * qh[i]);
            sc = (float)acc;
          }
        }
        sc = sc * A.scale;
        if (A.alibi) sc = A.alibi[h] + sc;  // (float)(0 + 1) * m_h, added as ggml_alibi does
        if (k < nk) {
          if (l16 == 0) pr[k] = sc;
          mx = mx > sc ? mx : sc;
        }
      }
    }
  }
  ATT_STAMP(1);
  // max, exp via table, exact double sum (fp16 values: any order), 1/sum
  mx = wave_max_f(mx);
  if (lane == 0) shf[wid] = mx;
  __syncthreads();
  mx = shf[0];
  for (int w = 1; w < ATT_WAVES; ++w) mx = mx > shf[w] ? mx : shf[w];
  double sum = 0.0;
  for (int k = tid; k < nk; k += ATT_THREADS) {
    const float val = h2f(A.etab[f2h(pr[k] - mx)]);
    pr[k] = val;
    sum += (double)val;
  }
  sum = wave_sum_d(sum);
  if (lane == 0) shd[wid] = sum;
  __syncthreads();
  sum = 0.0;
  for (int w = 0; w < ATT_WAVES; ++w) sum += shd[w];
  const float inv = (float)(1.0 / sum);
  for (int k = tid; k < nk; k += ATT_THREADS) pr[k] = pr[k] * inv;
  __syncthreads();
  ATT_STAMP(2);
  // KQV: y[dd] = sum_k V[k][dd] * p[k], sequential float chain from 0.0f (product and sum
  // rounded separately), thread j < c for column dd = c0 + j.  Every thread loads V tiles
  // (KT keys x c floats, float4 per slot) three tiles ahead into registers and stores them
  // into two LDS buffers; the chains read the tile from LDS.  (The KV-cache row n_past,
  // written above by this workgroup, is read back after the barriers.)
  float y = 0.0f;  // (c <= ATT_THREADS: one output element per thread)
  // --threads > 1: the pool gives thread t the keys [t*dc, t*dc + dc), each summed from 0 into
  // its own work row, and FINALIZE adds the rows in thread order, empty ones as +0
  const int nth = A.kqv_nth > 1 ? A.kqv_nth : 1, dc = (nk + nth - 1) / nth;
  float tot = 0.0f;
  bool run0 = true;
  {
    constexpr int PER = (ATT_VTF / 4 + ATT_THREADS - 1) / ATT_THREADS;  // float4 per thread per tile
    const int KT = ATT_VTF / c, nt = (nk + KT - 1) / KT, n4 = KT * c / 4;
    float *const vt0 = sm + ((2 * d + A.n_ctx + 3) & ~3);  // buffer b at vt0 + b * ATT_VTF
// (macros, not lambdas: the register ring must not be passed by address, or the compiler
// keeps it in scratch and waits for every load)
#define ATT_TLOAD(R, T)                                                              \
  _Pragma("unroll") for (int q = 0; q < PER; ++q) {                                  \
    const int f = min(tid + ATT_THREADS * q, n4 - 1);                                \
    const int key = min((T) * KT + (4 * f) / c, nk - 1), col = c0 + (4 * f) % c;     \
    R[q] = *(const f32x4 *)(A.vc + (size_t)key * E + h * d + col);                   \
  }
    f32x4 ra[PER], rb[PER], rc[PER];  // tiles t, t+1, t+2 in flight (clang vectors: HIP's
                                      // float4 class arrays are not promoted to registers)
    ATT_TLOAD(ra, 0)
    if (nt > 1) { ATT_TLOAD(rb, 1) }
    if (nt > 2) { ATT_TLOAD(rc, 2) }
    for (int t = 0; t < nt; ++t) {
      float *buf = vt0 + (t & 1) * ATT_VTF;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int f = tid + ATT_THREADS * q;
        if (f < n4) *(f32x4 *)(buf + 4 * f) = ra[q];
        ra[q] = rb[q];
        rb[q] = rc[q];
      }
      __syncthreads();
      if (t + 3 < nt) { ATT_TLOAD(rc, t + 3) }
      if (tid < c && nth > 1) {  // the reference pool's key runs (--threads > 1)
        const int kn = min(KT, nk - t * KT);
        const float *pt = pr + t * KT;
        for (int j = 0; j < kn; ++j) {
          const int kg = t * KT + j;
          if (kg > 0 && kg % dc == 0) {  // run boundary: FINALIZE's dst += partial, in run order
            tot = run0 ? y : tot + y;
            run0 = false;
            y = 0.0f;
          }
          y = y + buf[j * c + tid] * pt[j];
        }
      } else if (tid < c) {  // the chain: LDS reads eight keys ahead of the dependent adds
        const int kn = min(KT, nk - t * KT);
        const float *pt = pr + t * KT;
        int j = 0;
        for (; j + 8 <= kn; j += 8) {
          float v[8], p[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            v[u] = buf[(j + u) * c + tid];
            p[u] = pt[j + u];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) y = y + v[u] * p[u];
        }
        for (; j < kn; ++j) y = y + buf[j * c + tid] * pt[j];
      }
    }
#undef ATT_TLOAD
    if (nth > 1) {
      if (!run0) y = tot + y;
      if (nth > (nk + dc - 1) / dc) y = y + 0.0f;  // the trailing empty work rows
    }
    if (tid < c && A.out) st_out<CO>(A.out + h * d + c0 + tid, y);
  }
  ATT_STAMP(3);
  // quantize the part's outputs: wave w holds columns c0 + 64w .. +63, two 32-blocks
  if (wid * 64 < c) {
    const int blk = (h * d + c0 + wid * 64) / QK + (lane >> 5);
    const bool ok = wid * 64 + (lane & ~31) < c;
    quantize_half<CO>(y, lane, ok, A.oq_qs + (size_t)blk * 16, A.oq_d + blk, A.oxd + (size_t)blk * QK);
  }
}

}  // namespace vsim
