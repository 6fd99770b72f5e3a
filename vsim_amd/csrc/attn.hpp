// vsim_amd/csrc/attn.hpp — single-token attention for one head (used by k_attn_decode in
// layer.hip and by the fused layer tail in gemv_chain.hip).
//
// Per head: RoPE on q and the new k, KV-cache write, KQ (double accumulator), scale/softmax
// (fp16 exp table), KQV (sequential float mad), quantization of the head's output for the
// out-projection.  Every value with the reference's operation order and rounding.
#pragma once

#include "kern.hpp"

namespace vsim {

// One workgroup per head.  KQ: one wave per key, products over the head
// dimension summed as a tree in double; the reference's sequential double sum lies within
// 2*d*2^-53*sum|p| of it, so when both ends of that interval round to the same float the
// score is the reference's, otherwise lane 0 redoes the key sequentially (ggml.c:4760-4800
// for the f32 dot with a double accumulator).  KQV keeps the reference's sequential float
// chain over the keys, one chain per output element.
constexpr int ATT_KB = 4;   // keys per wave per load group
constexpr int ATT_DPL = 4;  // max head-dim elements per lane (d <= 256)

// One head (h) per workgroup of NT threads; sm: (2d + n_past + 1) floats of LDS.
template <int NT>
__device__ __forceinline__ void attn_body(const AttnJob &A, int h, float *sm) {
  constexpr int ATT_THREADS = NT, ATT_WAVES = NT / 64;
  const int d = A.d, E = A.d * A.H;
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
  // KQ[k] = (float) sum_i (double)(K[k][i] * q[i]) in order i = 0..d-1; then * scale.
  // Each wave takes keys in groups of ATT_KB and loads the whole group before reducing, so
  // the cache reads of a group overlap (one wave per key would pay the latency per key).
  float mx = -INFINITY;
  for (int k0 = wid * ATT_KB; k0 < nk; k0 += ATT_WAVES * ATT_KB) {
    float kv[ATT_KB][ATT_DPL];
#pragma unroll
    for (int j = 0; j < ATT_KB; ++j) {
      const int k = min(k0 + j, nk - 1);
      const float *kr = k == n_past ? kh : A.kc + (size_t)k * E + h * d;
#pragma unroll
      for (int e = 0; e < ATT_DPL; ++e) {
        const int i = lane + 64 * e;
        kv[j][e] = i < d ? kr[i] : 0.0f;
      }
    }
#pragma unroll
    for (int j = 0; j < ATT_KB; ++j) {
      const int k = k0 + j;
      if (k >= nk) break;  // wave-uniform
      double t = 0.0, ta = 0.0;
#pragma unroll
      for (int e = 0; e < ATT_DPL; ++e) {
        const int i = lane + 64 * e;
        if (i < d) {
          const double p = (double)(kv[j][e] * qh[i]);
          t += p;
          ta += fabs(p);
        }
      }
      t = wave_sum_d(t);
      ta = wave_sum_d(ta);
      const double bnd = 2.0 * d * 0x1.0p-53 * ta;
      float sc = (float)(t - bnd);
      if (sc != (float)(t + bnd)) {  // wave-uniform: redo this key in the reference order
        const float *kr = k == n_past ? kh : A.kc + (size_t)k * E + h * d;
        double acc = 0.0;
        if (lane == 0)
          for (int i = 0; i < d; ++i) acc += (double)(kr[i] * qh[i]);
        sc = (float)__shfl(acc, 0, 64);
      }
      sc = sc * A.scale;
      if (lane == 0) pr[k] = sc;
      mx = mx > sc ? mx : sc;
    }
  }
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
  // KQV: y[dd] = sum_k V[k][dd] * p[k], sequential float chain from 0.0f; V rows loaded
  // 16 keys ahead of the chain
  for (int dd0 = 0; dd0 < d; dd0 += ATT_THREADS) {
    const int dd = dd0 + tid;
    float y = 0.0f;
    if (dd < d) {
      const float *vcol = A.vc + h * d + dd;
      int k = 0;
      for (; k + 16 <= nk; k += 16) {
        float vv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) vv[j] = vcol[(size_t)(k + j) * E];
#pragma unroll
        for (int j = 0; j < 16; ++j) y = y + vv[j] * pr[k + j];
      }
      for (; k < nk; ++k) y = y + vcol[(size_t)k * E] * pr[k];
      if (A.out) A.out[h * d + dd] = y;
    }
    // quantize the head's outputs, two 32-blocks per wave
    if (dd0 + wid * 64 < d) {
      const int blk = (h * d + dd0 + wid * 64) / QK + (lane >> 5);
      const bool ok = dd0 + wid * 64 + (lane & ~31) < d;
      quantize_half(y, lane, ok, A.oq_qs + (size_t)blk * 16, A.oq_d + blk, A.oxd + (size_t)blk * QK);
    }
  }
}

}  // namespace vsim
