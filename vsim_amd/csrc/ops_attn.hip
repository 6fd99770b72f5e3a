// vsim_amd/csrc/ops_attn.hip — decode attention over the F32 KV cache.
//
//   RoPE GPT-NeoX rotate-half   ggml.c:6086-6153  (mode 0 on Q, mode 1 in place on K)
//   RoPE GPT-J pairs            ggml.c:5919-5974
//   KQ  = mul_mat(K, Q)         ggml.c:4495-4534 + ggml_vec_dot_f32 (double accumulator)
//   scale / diag_mask_inf / soft_max   ggml.c:5492-5525, 5764-5798, 5825-5893
//   KQV = mul_mat(V_trans, S)   ggml.c:4535-4581 + ggml_vec_mad_f32 (sequential float mad)
// Cache layout is the reference's: layer il, position p at element (il*n_ctx + p)*E
// (vsim.cpp:555-556), head h occupying [h*d, (h+1)*d).
#include "common.hpp"
#include "../../include/vsim_hip.h"

namespace vsim {

void rope_table_host(double2 *cs, int n_pos, int n_dims) {
  const int half = n_dims / 2;
  for (int j = 0; j < half; ++j) {
    // GPT-NeoX: pow(10000, 2*(-i0)/n_dims) with i0 = j; GPT-J: pow(10000, (-i0)/n_dims)
    // with i0 = 2j — the same double (2*(-j) == -(2j) exactly).
    const double theta = pow(10000.0, 2 * ((double)-j) / n_dims);
    for (int p = 0; p < n_pos; ++p) {
      cs[(size_t)p * half + j].x = cos(p * theta);
      cs[(size_t)p * half + j].y = sin(p * theta);
    }
  }
}

void alibi_slopes_host(float *m, int n_head) {
  const int n_heads_log2_floor = 1 << (int)floor(log2(n_head));
  const float m0 = pow(2.0, -8.0 / n_heads_log2_floor);
  const float m1 = pow(2.0, -4.0 / n_heads_log2_floor);
  for (int k = 0; k < n_head; ++k)
    m[k] = k < n_heads_log2_floor ? (float)pow(m0, k + 1) : (float)pow(m1, 2 * (k - n_heads_log2_floor) + 1);
}

// one thread per rotated pair; x[T][H][d]
__device__ __forceinline__ void rope_pair(float *v, int style, int j, int n_dims, double2 c) {
  if (style == 0) {
    const double x1 = v[j], x2 = v[j + n_dims / 2];
    v[j] = (float)(c.x * x1 - c.y * x2);
    v[j + n_dims / 2] = (float)(c.x * x2 + c.y * x1);
  } else {
    const double x0 = v[2 * j], x1 = v[2 * j + 1];
    v[2 * j] = (float)(x0 * c.x - x1 * c.y);
    v[2 * j + 1] = (float)(x0 * c.y + x1 * c.x);
  }
}

__global__ void k_rope(int style, float *x, int d, int H, int T, int n_past, int n_dims, int mode,
                       const double2 *__restrict__ cs) {
  const int half = n_dims / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int t0 = mode == 0 ? 0 : n_past;
  const int nt = T - t0;
  if (nt <= 0 || i >= nt * H * half) return;
  const int j = i % half, h = (i / half) % H, t = t0 + i / (half * H);
  const int p = mode == 0 ? n_past + t : t;
  rope_pair(x + ((size_t)t * H + h) * d, style, j, n_dims, cs[(size_t)p * half + j]);
}

int launch_rope(int style, float *x, int d, int H, int T, int n_past, int n_dims, int mode, const double2 *cs,
                hipStream_t s) {
  if (n_dims % 2 || n_dims > d) { set_error("rope: bad n_dims"); return VSIM_EINVAL; }
  const int nt = mode == 0 ? T : T - n_past;
  if (nt <= 0) return VSIM_OK;
  const int n = nt * H * (n_dims / 2);
  hipLaunchKernelGGL(k_rope, dim3((n + 255) / 256), dim3(256), 0, s, style, x, d, H, T, n_past, n_dims, mode, cs);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// Fused: rope Q (mode 0, p = n_past+t) in place; rope the new K rows and store them at
// cache position n_past+t; copy V rows (vsim.cpp:555-580: ggml_cpy into the cache view,
// then gptneox_rope mode 1 in place on positions >= n_past — same values).
__global__ void k_rope_kv_write(int style, float *__restrict__ Q, const float *__restrict__ K,
                                const float *__restrict__ V, float *__restrict__ kc, float *__restrict__ vc, int d,
                                int H, int N, int n_past, int n_dims, const double2 *__restrict__ cs) {
  const int E = d * H;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * E) return;
  const int t = i / E, e = i % E, h = e / d, dd = e % d;
  const int p = n_past + t;
  const int half = n_dims / 2;
  vc[(size_t)p * E + e] = V[i];
  // pair owner: NeoX (dd < half) owns (dd, dd+half); GPT-J (dd even, dd < n_dims) owns (dd, dd+1)
  const bool rot = dd < n_dims;
  const bool owner = style == 0 ? dd < half : ((dd & 1) == 0 && dd < n_dims);
  if (!rot) {
    kc[(size_t)p * E + e] = K[i];
    return;
  }
  if (!owner) return;
  const int j = style == 0 ? dd : dd / 2;
  const double2 c = cs[(size_t)p * half + j];
  const int o = style == 0 ? half : 1;
  const float *kr = K + (size_t)t * E + h * d;
  float *kd = kc + (size_t)p * E + h * d;
  float *qr = Q + (size_t)t * E + h * d;
  if (style == 0) {
    const double k1 = kr[dd], k2 = kr[dd + o];
    kd[dd] = (float)(c.x * k1 - c.y * k2);
    kd[dd + o] = (float)(c.x * k2 + c.y * k1);
    const double q1 = qr[dd], q2 = qr[dd + o];
    qr[dd] = (float)(c.x * q1 - c.y * q2);
    qr[dd + o] = (float)(c.x * q2 + c.y * q1);
  } else {
    const double k0 = kr[dd], k1 = kr[dd + 1];
    kd[dd] = (float)(k0 * c.x - k1 * c.y);
    kd[dd + 1] = (float)(k0 * c.y + k1 * c.x);
    const double q0 = qr[dd], q1 = qr[dd + 1];
    qr[dd] = (float)(q0 * c.x - q1 * c.y);
    qr[dd + 1] = (float)(q0 * c.y + q1 * c.x);
  }
}

int launch_rope_kv_write(int style, float *Q, const float *K, const float *V, float *kcache, float *vcache, int d,
                         int H, int N, int n_past, int n_dims, const double2 *cs, hipStream_t s) {
  const int n = N * d * H;
  hipLaunchKernelGGL(k_rope_kv_write, dim3((n + 255) / 256), dim3(256), 0, s, style, Q, K, V, kcache, vcache, d, H, N,
                     n_past, n_dims, cs);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

// (KQ and KQV: attn_exact.hip)

// scale -> mask -> softmax, one 256-thread block per row of nc (row r = (z, j)).
// The fp16-valued exps sum exactly in double in any order (multiples of 2^-24, < 2^11).
// alibi (BLOOM, may be null): per-head slopes m_k; after the scale each score gets
// (j+1)*m_k added, j the query row (ggml_alibi, ggml.c:6184-6244), before the mask.
__global__ void __launch_bounds__(256) k_attn_softmax(float *p, int nc, int nr, int n_past, float scale,
                                                       const uint16_t *__restrict__ etab,
                                                       const float *__restrict__ alibi) {
  __shared__ float shf[4];
  __shared__ double shd[4];
  const int row = blockIdx.x;
  const int j = row % nr;
  float *x = p + (size_t)row * nc;
  const float ab = alibi ? (float)(j + 1) * alibi[row / nr] : 0.0f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < nc; i += 256) {
    float v = x[i] * scale;
    if (alibi) v = ab + v;
    if (i >= n_past && i > n_past + j) v = -INFINITY;
    x[i] = v;
    mx = mx > v ? mx : v;
  }
  mx = wave_max_f(mx);
  if (lane == 0) shf[wid] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(shf[0], shf[1]), fmaxf(shf[2], shf[3]));
  double sum = 0.0;
  for (int i = threadIdx.x; i < nc; i += 256) {
    const float v = x[i];
    float val = 0.0f;
    if (v != -INFINITY) {
      val = h2f(etab[f2h(v - mx)]);
      sum += (double)val;
    }
    x[i] = val;
  }
  sum = wave_sum_d(sum);
  if (lane == 0) shd[wid] = sum;
  __syncthreads();
  sum = (shd[0] + shd[1]) + (shd[2] + shd[3]);
  const float inv = (float)(1.0 / sum);
  for (int i = threadIdx.x; i < nc; i += 256) x[i] = x[i] * inv;
}

int launch_attn_softmax(float *p, int nc, int nr, int nz, int n_past, float scale, hipStream_t s,
                        const float *alibi) {
  DevTables t;
  if (int rc = tables_get(&t)) return rc;
  hipLaunchKernelGGL(k_attn_softmax, dim3(nr * nz), dim3(256), 0, s, p, nc, nr, n_past, scale, t.exp_f16, alibi);
  VSIM_HIP(hipGetLastError());
  return VSIM_OK;
}

}  // namespace vsim
