// vsim_amd/csrc/attn_exact.hip — exact-mode attention products for prompt batches: KQ and KQV
// as register-tiled GEMMs whose inner loops keep the reference's order.
//
//  * KQ (ggml_compute_forward_mul_mat_f32, ggml.c:4495-4534, ggml_vec_dot_f32 399-434):
//      kq[h][q][k] = (float) sum_i (double)(K[k][h d + i] * Q[q][h d + i])
//    each product rounded to float, added in double in order i = 0 .. d-1.  A thread owns a
//    4 x 4 block of (query, key) sums, 16 double accumulators, and adds one product to each per i.
//  * KQV (ggml.c:4535-4581, ggml_vec_mad_f32 610-639, one key run: --threads 1):
//      out[q][h d + c] = chain over k of  y = y + V[k][h d + c] * S[h][q][k]
//    float product and float sum, in key order.  A thread owns 4 x 4 (query, column) chains.
// Causal skipping (n_past >= 0, the prompt's own diag_mask_inf, ggml.c:5764-5798): KQ tiles whose
// keys are all masked for all their queries are not computed (the mask overwrites them with -inf
// before anything reads them); KQV stops at the tile's last unmasked key, since every later
// probability is exactly 0 and y + (+-0) == y for every y the chain can hold (it starts at +0
// and an IEEE sum is -0 only when both operands are).
#include "kern.hpp"

namespace vsim {

constexpr int AX_T = 64, AX_C = 32, AX_THREADS = 256, AX_LD = AX_T + 4;

// kq[(h n + q) nk + k] for q < n, k < nk (the tile grid: key tiles x query tiles x heads)
__global__ void __launch_bounds__(AX_THREADS) k_kq_tile(const float *__restrict__ K, int ldk, const float *__restrict__ Q,
                                                         int ldq, int d, int n, int nk, int n_past,
                                                         float *__restrict__ out) {
  __shared__ __attribute__((aligned(16))) float Ks[AX_C][AX_LD];
  __shared__ __attribute__((aligned(16))) float Qs[AX_C][AX_LD];
  const int k0 = blockIdx.x * AX_T, q0 = blockIdx.y * AX_T, h = blockIdx.z;
  if (n_past >= 0 && k0 > n_past + min(q0 + AX_T, n) - 1) return;  // every key masked for every query
  const int tid = threadIdx.x, tk = tid % 16, tq = tid / 16;
  // staging: row r = tid / 4 (key or query), 8 consecutive i from (tid % 4) * 8
  const int sr = tid >> 2, si = (tid & 3) * 8;
  const float *kr = K + (size_t)min(k0 + sr, nk - 1) * ldk + (size_t)h * d;
  const float *qr = Q + (size_t)min(q0 + sr, n - 1) * ldq + (size_t)h * d;
  double acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  for (int i0 = 0; i0 < d; i0 += AX_C) {
    f32x4 kv[2], qv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = i0 + si + 4 * u;  // d % 4 == 0: a vector is wholly inside or outside the row
      kv[u] = i < d ? *(const f32x4 *)(kr + i) : f32x4{0.f, 0.f, 0.f, 0.f};
      qv[u] = i < d ? *(const f32x4 *)(qr + i) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        Ks[si + 4 * u + e][sr] = kv[u][e];
        Qs[si + 4 * u + e][sr] = qv[u][e];
      }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < AX_C; ++i) {  // (zero padding past d adds +0: exact)
      const f32x4 kk = *(const f32x4 *)&Ks[i][4 * tk];
      const f32x4 qq = *(const f32x4 *)&Qs[i][4 * tq];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = acc[a][b] + (double)(qq[a] * kk[b]);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q = q0 + 4 * tq + a, k = k0 + 4 * tk;
    if (q >= n) continue;
    float *o = out + ((size_t)h * n + q) * nk + k;
    const f32x4 v = {(float)acc[a][0], (float)acc[a][1], (float)acc[a][2], (float)acc[a][3]};
    if (k + 3 < nk && (nk & 3) == 0) {
      *(f32x4 *)o = v;
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (k + b < nk) o[b] = v[b];
    }
  }
}

// out[q][h d + c] (merged) or out[(h n + q) d + c] (the [d, N, H] tensor); tiles of 64 columns
// x 64 queries x heads
__global__ void __launch_bounds__(AX_THREADS) k_kqv_tile(const float *__restrict__ V, int ldv,
                                                          const float *__restrict__ S, int d, int H, int n, int nk,
                                                          int n_past, float *__restrict__ out, int merged) {
  __shared__ __attribute__((aligned(16))) float Vs[AX_C][AX_LD];
  __shared__ __attribute__((aligned(16))) float Ss[AX_C][AX_LD];
  const int c0 = blockIdx.x * AX_T, q0 = blockIdx.y * AX_T, h = blockIdx.z;
  const int tid = threadIdx.x, tc = tid % 16, tq = tid / 16;
  const int kend = n_past >= 0 ? min(nk, n_past + min(q0 + AX_T, n)) : nk;  // keys past it: probability 0
  // staging V: key row kk = tid / 8 (32 rows), 8 consecutive columns from (tid % 8) * 8
  const int vk = tid >> 3, vc = (tid & 7) * 8;
  const float *vbase = V + (size_t)h * d + c0 + vc;
  // staging S: query row sq = tid / 4 (64 rows), 8 consecutive keys from (tid % 4) * 8
  const int sq = tid >> 2, sk = (tid & 3) * 8;
  const float *srow = S + ((size_t)h * n + min(q0 + sq, n - 1)) * nk;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.0f;
  for (int kb = 0; kb < kend; kb += AX_C) {
    f32x4 vv[2];
    float sv[8];
    {
      const int k = kb + vk;
      const bool kin = k < kend;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = c0 + vc + 4 * u;  // d % 4 == 0
        vv[u] = kin && c < d ? *(const f32x4 *)(vbase + (size_t)k * ldv + 4 * u) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sv[e] = kb + sk + e < kend ? srow[kb + sk + e] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) *(f32x4 *)&Vs[vk][vc + 4 * u] = vv[u];
#pragma unroll
    for (int e = 0; e < 8; ++e) Ss[sk + e][sq] = sv[e];
    __syncthreads();
    auto step = [&](int kk) __attribute__((always_inline)) {
      const f32x4 vr = *(const f32x4 *)&Vs[kk][4 * tc];
      const f32x4 sr = *(const f32x4 *)&Ss[kk][4 * tq];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = acc[a][b] + vr[b] * sr[a];  // y += x*v
    };
    const int kn = min(AX_C, kend - kb);  // (workgroup-uniform)
    if (kn == AX_C) {
#pragma unroll 8
      for (int kk = 0; kk < AX_C; ++kk) step(kk);
    } else {
      for (int kk = 0; kk < kn; ++kk) step(kk);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q = q0 + 4 * tq + a, c = c0 + 4 * tc;
    if (q >= n || c >= d) continue;
    float *o = merged ? out + (size_t)q * H * d + (size_t)h * d + c : out + ((size_t)h * n + q) * d + c;
    *(f32x4 *)o = f32x4{acc[a][0], acc[a][1], acc[a][2], acc[a][3]};  // (d % 4 == 0, c % 4 == 0)
  }
}

int launch_kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int n, float *kq, hipStream_t s,
              int n_past) {
  if (d % 4 || ldk % 4 || ldq % 4 || d <= 0 || H <= 0 || nk <= 0 || n <= 0) {
    set_error("kq: d and strides must be positive multiples of 4");
    return VSIM_EINVAL;
  }
  hipLaunchKernelGGL(k_kq_tile, dim3((nk + AX_T - 1) / AX_T, (n + AX_T - 1) / AX_T, H), dim3(AX_THREADS), 0, s, K, ldk,
                     Q, ldq, d, n, nk, n_past, kq);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

int launch_kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int n, float *out, int merged,
               hipStream_t s, int n_past) {
  if (d % 4 || ldv % 4 || d <= 0 || H <= 0 || nk <= 0 || n <= 0) {
    set_error("kqv: d and the V stride must be positive multiples of 4");
    return VSIM_EINVAL;
  }
  hipLaunchKernelGGL(k_kqv_tile, dim3((d + AX_T - 1) / AX_T, (n + AX_T - 1) / AX_T, H), dim3(AX_THREADS), 0, s, V, ldv,
                     S, d, H, n, nk, n_past, out, merged);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
