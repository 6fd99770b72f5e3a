// oracle/vsim_oracle.cpp — TEST INFRASTRUCTURE ONLY (parity checker, cpu_baseline).
//
// A CPU restatement of NAIST-Archlab/vsim's Q4_0 decode path, written from the
// reference's behaviour (file:line cited per function).  Built with -O2 -msse3
// -ffp-contract=off like the reference x86 build (Makefile-ubuntu:5-6): scalar code,
// no FMA, ggml_float == double (ggml.c:66).  The product (libvsim_hip.so) never links
// or calls this file; tests compare the HIP path against it, and it is itself pinned
// bit-for-bit against the reference binary built from /root/reference (oracle/Makefile).

#include "vsim_oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int QK = 32;
constexpr int QBYTES = 20;  // sizeof(float) + QK/2, ggml.c:907-909

// ---- fp16 <-> fp32 (bit-exact restatement of ggml.c:95-142) --------------------------
inline float bits_f(uint32_t w) { float f; std::memcpy(&f, &w, 4); return f; }
inline uint32_t f_bits(float f) { uint32_t w; std::memcpy(&w, &f, 4); return w; }

float h2f(uint16_t h) {
  const uint32_t w = (uint32_t)h << 16;
  const uint32_t sign = w & 0x80000000u;
  const uint32_t two_w = w + w;
  const float normalized = bits_f((two_w >> 4) + (0xE0u << 23)) * 0x1.0p-112f;
  const float denormalized = bits_f((two_w >> 17) | (126u << 23)) - 0.5f;
  const uint32_t r = sign | (two_w < (1u << 27) ? f_bits(denormalized) : f_bits(normalized));
  return bits_f(r);
}

uint16_t f2h(float f) {
  float base = (std::fabs(f) * 0x1.0p+112f) * 0x1.0p-110f;
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

// ggml.c:1240-1251: the 64K tables built at first ggml_init
float    g_f32_f16[65536];
uint16_t g_gelu_f16[65536];
uint16_t g_exp_f16[65536];
bool     g_tables_ready = false;

// ggml.c:789-791: GELU_COEF_A / SQRT_2_OVER_PI are ggml_float (double) constants
float gelu_scalar(float x) {
  const double A = 0.044715, S = 0.79788456;
  return 0.5 * x * (1.0 + std::tanh(S * x * (1.0 + A * x * x)));
}

void init_tables_once() {
  if (g_tables_ready) return;
  for (int i = 0; i < 65536; ++i) {
    const float f = g_f32_f16[i] = h2f((uint16_t)i);
    g_gelu_f16[i] = f2h(gelu_scalar(f));
    g_exp_f16[i] = f2h((float)std::exp((double)f));
  }
  g_tables_ready = true;
}

inline float lut_h2f(uint16_t h) { return g_f32_f16[h]; }

// ---- Q4_0 -------------------------------------------------------------------------------
// ggml.c:209-251 quantize_row_q4_0
void quantize_row(const float *x, uint8_t *y, int k) {
  const int nb = k / QK;
  for (int i = 0; i < nb; i++) {
    float amax = 0.0f;
    for (int l = 0; l < QK; l++) {
      const float v = x[i * QK + l];
      amax = amax > std::fabs(v) ? amax : std::fabs(v);
    }
    const float d = amax / ((1 << 3) - 1);
    const float id = d ? 1.0f / d : 0.0f;
    std::memcpy(y + i * QBYTES, &d, 4);
    uint8_t *pb = y + i * QBYTES + 4;
    for (int l = 0; l < QK; l += 2) {
      const float v0 = x[i * QK + l + 0] * id;
      const float v1 = x[i * QK + l + 1] * id;
      const uint8_t vi0 = (uint8_t)(((int8_t)std::round((double)v0)) + 8);
      const uint8_t vi1 = (uint8_t)(((int8_t)std::round((double)v1)) + 8);
      pb[l / 2] = (uint8_t)(vi0 | (vi1 << 4));
    }
  }
}

// ggml.c:301-334 dequantize_row_q4_0
void dequantize_row(const uint8_t *x, float *y, int k) {
  const int nb = k / QK;
  for (int i = 0; i < nb; i++) {
    float d;
    std::memcpy(&d, x + i * QBYTES, 4);
    const uint8_t *pp = x + i * QBYTES + 4;
    for (int l = 0; l < QK; l += 2) {
      const uint8_t vi = pp[l / 2];
      const int8_t vi0 = vi & 0xf;
      const int8_t vi1 = vi >> 4;
      y[i * QK + l + 0] = (vi0 - 8) * d;
      y[i * QK + l + 1] = (vi1 - 8) * d;
    }
  }
}

// imax.c:1191-1229 (== ggml_vec_dot_q4_0, ggml.c:472-511): one sequential float chain
float vec_dot_q4(int n, const uint8_t *x, const uint8_t *y) {
  const int nb = n / QK;
  float sumf = 0.0f;
  for (int i = 0; i < nb; i++) {
    float d0, d1;
    std::memcpy(&d0, x + i * QBYTES, 4);
    std::memcpy(&d1, y + i * QBYTES, 4);
    const uint8_t *p0 = x + i * QBYTES + 4;
    const uint8_t *p1 = y + i * QBYTES + 4;
    for (int j = 0; j < QK / 2; j++) {
      const uint8_t v0 = p0[j];
      const uint8_t v1 = p1[j];
      const float f0 = d0 * ((int8_t)(v0 & 0xf) - 8);
      const float f1 = d0 * ((int8_t)(v0 >> 4) - 8);
      const float f2 = d1 * ((int8_t)(v1 & 0xf) - 8);
      const float f3 = d1 * ((int8_t)(v1 >> 4) - 8);
      sumf += f0 * f2 + f1 * f3;
    }
  }
  return sumf;
}

template <class F>
void parallel_rows(int nr, int nthreads, F &&fn) {
  if (nthreads <= 1 || nr < 64) { fn(0, nr); return; }
  std::vector<std::thread> th;
  const int dr = (nr + nthreads - 1) / nthreads;  // ggml.c row split, imax.c:1184-1188
  for (int t = 0; t < nthreads; ++t) {
    const int r0 = dr * t, r1 = std::min(r0 + dr, nr);
    if (r0 >= r1) break;
    th.emplace_back([=, &fn] { fn(r0, r1); });
  }
  for (auto &t : th) t.join();
}

// Work items [0, n) pulled from a shared counter by nthreads threads (the items are
// independent, so the split changes nothing but the balance).
template <class F>
void parallel_items(int n, int nthreads, F &&fn) {
  if (nthreads <= 1 || n <= 1) { for (int i = 0; i < n; ++i) fn(i); return; }
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < std::min(nthreads, n); ++t)
    th.emplace_back([&] { for (int i; (i = next.fetch_add(1)) < n;) fn(i); });
  for (auto &t : th) t.join();
}

bool cpu_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2");
  return ok;
}

typedef float v8f __attribute__((vector_size(32)));
typedef double v4d __attribute__((vector_size(32)));
typedef float v4f __attribute__((vector_size(16)));

// The dot of imax.c:1191-1229 for 8 activation rows at once: lane t of every vector is
// token t's own chain, with the reference's operations in the reference's order (the
// dequantized factors d*(q-8) are the same float products, each pair term is
// (f0*f2) + (f1*f3) rounded step by step, added to the lane's running sum; no FMA exists
// in this target).  Only the speed of the oracle changes, not one bit of its results
// (tests/test_oracle_golden.py holds it to the reference's goldens, prompt shapes included).
// wf: R rows of dequantized weights [R][K]; xt: the token group's factors [K][8].
template <int R>
__attribute__((target("avx2"))) void dot_rows_tok8(const float *wf, int K, const float *xt, v8f *acc) {
  v8f a[R];
  for (int r = 0; r < R; ++r) a[r] = v8f{};
  for (int k = 0; k < K; k += 2) {
    v8f x0, x1;
    std::memcpy(&x0, xt + (size_t)k * 8, 32);
    std::memcpy(&x1, xt + (size_t)k * 8 + 8, 32);
    for (int r = 0; r < R; ++r) {
      const float w0 = wf[(size_t)r * K + k], w1 = wf[(size_t)r * K + k + 1];
      a[r] = a[r] + ((w0 * x0) + (w1 * x1));
    }
  }
  for (int r = 0; r < R; ++r) acc[r] = a[r];
}

// ggml.c:4891-5165 + imax.c:1182-1230 for N >= 8 activation rows: the 8-token groups go
// through dot_rows_tok8 (4 weight rows per pass), the remaining N % 8 tokens through the
// scalar vec_dot_q4.
void mul_mat_q_tok8(const uint8_t *W, int M, int K, const uint8_t *xq, int N, float *y, int nthreads) {
  const size_t rb = (size_t)K / QK * QBYTES;
  const int nb = K / QK, G = N / 8;
  std::vector<float> xt((size_t)G * K * 8);
  parallel_items(G, nthreads, [&](int g) {
    for (int t = 0; t < 8; ++t) {
      const uint8_t *x = xq + (size_t)(8 * g + t) * rb;
      float *o = xt.data() + (size_t)g * K * 8 + t;
      for (int i = 0; i < nb; ++i) {
        float d1;
        std::memcpy(&d1, x + i * QBYTES, 4);
        const uint8_t *p1 = x + i * QBYTES + 4;
        for (int j = 0; j < QK / 2; ++j) {
          const uint8_t v1 = p1[j];
          o[(size_t)(i * QK + 2 * j) * 8] = d1 * ((int8_t)(v1 & 0xf) - 8);
          o[(size_t)(i * QK + 2 * j + 1) * 8] = d1 * ((int8_t)(v1 >> 4) - 8);
        }
      }
    }
  });
  constexpr int R = 4;
  const int nblk = (M + R - 1) / R;
  parallel_items(nblk, nthreads, [&](int blk) {
    const int r0 = blk * R, nr = std::min(R, M - r0);
    std::vector<float> wf((size_t)R * K);
    for (int r = 0; r < nr; ++r) {  // f0 = d0*(q-8) as imax.c:1203-1206
      const uint8_t *w = W + (size_t)(r0 + r) * rb;
      for (int i = 0; i < nb; ++i) {
        float d0;
        std::memcpy(&d0, w + i * QBYTES, 4);
        const uint8_t *p0 = w + i * QBYTES + 4;
        for (int j = 0; j < QK / 2; ++j) {
          const uint8_t v0 = p0[j];
          wf[(size_t)r * K + i * QK + 2 * j] = d0 * ((int8_t)(v0 & 0xf) - 8);
          wf[(size_t)r * K + i * QK + 2 * j + 1] = d0 * ((int8_t)(v0 >> 4) - 8);
        }
      }
    }
    for (int g = 0; g < G; ++g) {
      v8f acc[R];
      const float *xg = xt.data() + (size_t)g * K * 8;
      if (nr == R) {
        dot_rows_tok8<R>(wf.data(), K, xg, acc);
      } else {
        for (int r = 0; r < nr; ++r) dot_rows_tok8<1>(wf.data() + (size_t)r * K, K, xg, acc + r);
      }
      for (int r = 0; r < nr; ++r)
        for (int t = 0; t < 8; ++t) y[(size_t)(8 * g + t) * M + r0 + r] = acc[r][t];
    }
    for (int ic = 8 * G; ic < N; ++ic)
      for (int r = 0; r < nr; ++r) y[(size_t)ic * M + r0 + r] = vec_dot_q4(K, W + (size_t)(r0 + r) * rb, xq + ic * rb);
  });
}

// ggml.c:4891-5165 + imax.c:1182-1230: dst[ic*M + ir] = dot(W row ir, xq row ic).
// Rows are independent chains, so the result does not depend on nthreads.
void mul_mat_q(const uint8_t *W, int M, int K, const uint8_t *xq, int N, float *y, int nthreads) {
  const size_t rb = (size_t)K / QK * QBYTES;
  if (N >= 8 && cpu_avx2()) {
    mul_mat_q_tok8(W, M, K, xq, N, y, nthreads);
    return;
  }
  parallel_rows(M, nthreads, [&](int r0, int r1) {
    for (int ir = r0; ir < r1; ++ir)
      for (int ic = 0; ic < N; ++ic) y[(size_t)ic * M + ir] = vec_dot_q4(K, W + ir * rb, xq + ic * rb);
  });
}

void mul_mat_f(const uint8_t *W, int M, int K, const float *x, int N, float *y, int nthreads) {
  const size_t rb = (size_t)K / QK * QBYTES;
  std::vector<uint8_t> wdata(rb * N);  // INIT phase, ggml.c:5024-5041
  parallel_items(N, N >= 64 ? nthreads : 1,
                 [&](int ic) { quantize_row(x + (size_t)ic * K, wdata.data() + ic * rb, K); });
  mul_mat_q(W, M, K, wdata.data(), N, y, nthreads);
}

// ggml.c:4246-4304 ggml_compute_forward_norm_f32
void norm_row(const float *x, float *y, int n) {
  const double eps = 1e-5f;
  double mean = 0.0;
  for (int i = 0; i < n; i++) mean += x[i];
  mean /= n;
  double sum2 = 0.0;
  for (int i = 0; i < n; i++) {
    double v = x[i] - mean;
    y[i] = v;
    sum2 += v * v;
  }
  const float scale = 1.0 / std::sqrt(sum2 / n + eps);
  for (int i = 0; i < n; i++) y[i] *= scale;
}

// ggml.c:4113-4152 + 795-803: GELU through the fp16 table
void gelu(const float *x, float *y, int n) {
  for (int i = 0; i < n; i++) y[i] = lut_h2f(g_gelu_f16[f2h(x[i])]);
}

// ggml.c:5825-5893 ggml_compute_forward_soft_max_f32 (one row)
void soft_max_row(float *p, int nc) {
  double max = -INFINITY;
  for (int i = 0; i < nc; ++i) max = max > p[i] ? max : p[i];
  const float fmax_ = (float)max;
  double sum = 0.0;
  for (int i = 0; i < nc; i++) {
    if (p[i] == -INFINITY) {
      p[i] = 0.0f;
    } else {
      const uint16_t s = f2h(p[i] - fmax_);
      const float val = lut_h2f(g_exp_f16[s]);
      sum += val;
      p[i] = val;
    }
  }
  sum = 1.0 / sum;
  const float v = (float)sum;
  for (int i = 0; i < nc; i++) p[i] *= v;
}

// ggml.c:6086-6153 ggml_compute_forward_gptneox_rope_f32 (rotate-half)
void rope_neox(float *x, int d, int H, int T, int n_past, int n_dims, int mode) {
  for (int i2 = (mode == 0 ? 0 : n_past); i2 < T; i2++) {
    const int p = (mode == 0 ? n_past + i2 : i2);
    for (int i1 = 0; i1 < H; i1++) {
      for (int i0 = 0; i0 < n_dims / 2; i0++) {
        const double theta = std::pow(10000.0, 2 * ((double)-i0) / n_dims);
        const double c = std::cos(p * theta), s = std::sin(p * theta);
        float *v = x + ((size_t)i2 * H + i1) * d + i0;
        const double x1 = v[0], x2 = v[n_dims / 2];
        v[0] = (c * x1 - s * x2);
        v[n_dims / 2] = (c * x2 + s * x1);
      }
    }
  }
}

// ggml.c:5919-5974 ggml_compute_forward_rope_f32 (GPT-J interleaved pairs)
void rope_gptj(float *x, int d, int H, int T, int n_past, int n_dims, int mode) {
  for (int i2 = (mode == 0 ? 0 : n_past); i2 < T; i2++) {
    const int p = (mode == 0 ? n_past + i2 : i2);
    for (int i1 = 0; i1 < H; i1++) {
      for (int i0 = 0; i0 < n_dims; i0 += 2) {
        const double theta = std::pow(10000.0, ((double)-i0) / n_dims);
        const double c = std::cos(p * theta), s = std::sin(p * theta);
        float *v = x + ((size_t)i2 * H + i1) * d + i0;
        const double x0 = v[0], x1 = v[1];
        v[0] = x0 * c - x1 * s;
        v[1] = x0 * s + x1 * c;
      }
    }
  }
}

// ggml.c:4495-4534 (non-transposed src0) + ggml_vec_dot_f32 ggml.c:399-434: per (head, key,
// query) sumf += x[i]*y[i] in double (float products), cast to float.  For 8 or more queries
// the queries of a head go 8 at a time through vectors (lane q = query q's own sum, same order);
// heads run on nthreads threads.
__attribute__((target("avx2"))) void kq_head_q8(const float *K, int ldk, const float *Qt, int d, int nk, int nq8,
                                                float *out, int N) {
  for (int k = 0; k < nk; ++k) {
    const float *kr = K + (size_t)k * ldk;
    for (int g = 0; g < nq8; ++g) {
      v4d s0{}, s1{};
      const float *qg = Qt + (size_t)g * d * 8;
      for (int i = 0; i < d; ++i) {
        v8f qv;
        std::memcpy(&qv, qg + (size_t)i * 8, 32);
        const v8f pr = kr[i] * qv;
        const v4f lo = {pr[0], pr[1], pr[2], pr[3]}, hi = {pr[4], pr[5], pr[6], pr[7]};
        s0 = s0 + __builtin_convertvector(lo, v4d);
        s1 = s1 + __builtin_convertvector(hi, v4d);
      }
      for (int t = 0; t < 4; ++t) out[(size_t)(8 * g + t) * nk + k] = (float)s0[t];
      for (int t = 0; t < 4; ++t) out[(size_t)(8 * g + 4 + t) * nk + k] = (float)s1[t];
    }
  }
  (void)N;
}

void kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int N, float *out, int nthreads = 1) {
  const int nq8 = cpu_avx2() ? N / 8 : 0;
  parallel_items(H, nthreads, [&](int h) {
    if (nq8) {
      std::vector<float> Qt((size_t)nq8 * d * 8);  // [group][i][8]
      for (int q = 0; q < 8 * nq8; ++q)
        for (int i = 0; i < d; ++i) Qt[((size_t)(q / 8) * d + i) * 8 + q % 8] = Q[(size_t)q * ldq + h * d + i];
      kq_head_q8(K + h * d, ldk, Qt.data(), d, nk, nq8, out + (size_t)h * N * nk, N);
    }
    for (int k = 0; k < nk; ++k)
      for (int q = 8 * nq8; q < N; ++q) {
        const float *kr = K + (size_t)k * ldk + h * d;
        const float *qr = Q + (size_t)q * ldq + h * d;
        double sumf = 0.0;
        for (int i = 0; i < d; ++i) sumf += kr[i] * qr[i];
        out[((size_t)h * N + q) * nk + k] = (float)sumf;
      }
  });
}

// ggml.c:4535-4581 (transposed src0, nth == 1) + ggml_vec_mad_f32 ggml.c:610-639; the
// (head, query) rows are independent and run on nthreads threads
void kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int N, float *out, int nthreads = 1) {
  parallel_items(H * N, H * N >= 64 ? nthreads : 1, [&](int hq) {
    const int h = hq / N, q = hq % N;
    float *y = out + ((size_t)h * N + q) * d;
    for (int i = 0; i < d; ++i) y[i] = 0.0f;
    const float *srow = S + ((size_t)h * N + q) * nk;
    for (int k = 0; k < nk; ++k) {
      const float v = srow[k];
      const float *x = V + (size_t)k * ldv + h * d;
      for (int i = 0; i < d; ++i) y[i] += x[i] * v;
    }
  });
}

// ggml.c:6184-6244 ggml_compute_forward_alibi_f32 on p[nz][nr][nc] (ne0 = nc keys, ne1 = nr
// query rows, ne2 = nz heads): dst = (j+1)*m_k + src with the head slopes in float from
// double pow (m0 = 2^(-8/n), m1 = 2^(-4/n), n = 2^floor(log2(n_head))).  As in the
// reference, the bias depends on the query row j, not on the key position.
void alibi(float *p, int nc, int nr, int nz, int n_head) {
  const int n_heads_log2_floor = 1 << (int)std::floor(std::log2(n_head));
  const float m0 = std::pow(2.0, -8.0 / n_heads_log2_floor);
  const float m1 = std::pow(2.0, -4.0 / n_heads_log2_floor);
  for (int k = 0; k < nz; ++k) {
    const float m_k = k < n_heads_log2_floor ? (float)std::pow(m0, k + 1)
                                             : (float)std::pow(m1, 2 * (k - n_heads_log2_floor) + 1);
    for (int j = 0; j < nr; ++j)
      for (int i = 0; i < nc; ++i) {
        float *x = p + ((size_t)k * nr + j) * nc + i;
        *x = (j + 1) * m_k + *x;
      }
  }
}

// ---- model --------------------------------------------------------------------------------
struct Layer {
  std::vector<float> ln1_w, ln1_b, ln2_w, ln2_b;
  std::vector<uint8_t> wq, wk, wv, wo, wfc, wproj;
  std::vector<float> bq, bk, bv, bo, bfc, bproj;
  std::vector<uint8_t> wqkv;  // BLOOM: fused [3E][E], rows q | k | v (the converter's order)
  std::vector<float> bqkv;
};

struct Model {
  int arch = VO_ARCH_GPTNEOX;
  int32_t n_vocab = 0, n_embd = 0, n_head = 0, n_layer = 0, n_rot = 0, par_res = 1, ftype = 2;
  int n_ctx = 512;
  std::vector<uint8_t> wte, lmh;
  std::vector<float> lnf_w, lnf_b, lmh_b;
  std::vector<float> emb_w, emb_b;  // BLOOM word_embeddings_layernorm
  std::vector<Layer> layers;
  std::vector<float> mem_k, mem_v;  // [L][n_ctx][E], vsim.cpp:349-366
};

bool read_all(std::ifstream &f, void *p, size_t n) {
  f.read((char *)p, n);
  return (size_t)f.gcount() == n;
}

using SlotMap = std::map<std::string, std::pair<void *, size_t>>;
void build_slots(Model *m, SlotMap &slots);
bool read_tensors(std::ifstream &f, SlotMap &slots);

// vsim.cpp:108-458 (GPT-NeoX) and convert_gptj_to_ggml.py:106-126 (GPT-J) formats.
Model *load_model(const char *path, int arch, int n_ctx) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return nullptr;
  uint32_t magic = 0;
  read_all(f, &magic, 4);
  if (magic != 0x67676d6c) return nullptr;
  auto *m = new Model();
  m->arch = arch;
  m->n_ctx = n_ctx;
  read_all(f, &m->n_vocab, 4);
  read_all(f, &m->n_embd, 4);
  if (arch == VO_ARCH_BLOOM) {  // convert_bloom_to_ggml.py:79-85: vocab, hidden, multiple_of, heads, layers, ftype
    int32_t n_mult = 0;
    read_all(f, &n_mult, 4);
    m->n_rot = 0;
    m->par_res = 0;
  }
  read_all(f, &m->n_head, 4);
  read_all(f, &m->n_layer, 4);
  if (arch != VO_ARCH_BLOOM) read_all(f, &m->n_rot, 4);
  if (arch == VO_ARCH_GPTNEOX) read_all(f, &m->par_res, 4);
  read_all(f, &m->ftype, 4);
  int32_t nv = m->n_vocab;
  if (arch == VO_ARCH_GPTJ) read_all(f, &nv, 4);  // explicit vocab count
  for (int i = 0; i < nv; ++i) {
    uint32_t len;
    read_all(f, &len, 4);
    std::string w(len, 0);
    read_all(f, &w[0], len);
  }
  SlotMap slots;
  build_slots(m, slots);
  if (!read_tensors(f, slots)) {
    delete m;
    return nullptr;
  }
  m->mem_k.assign((size_t)m->n_layer * n_ctx * m->n_embd, 0.0f);
  m->mem_v.assign((size_t)m->n_layer * n_ctx * m->n_embd, 0.0f);
  return m;
}

// name -> (vector, kind 0 = F32 / 1 = Q4_0), each vector sized to its tensor.  Names of
// vsim.cpp:287-346 (GPT-NeoX), HF GPTJForCausalLM via convert_gptj_to_ggml.py, and
// convert_bloom_to_ggml.py:22-34 (BLOOM).
void build_slots(Model *m, SlotMap &slots) {
  const int E = m->n_embd, L = m->n_layer, V = m->n_vocab;
  const int arch = m->arch;
  m->layers.resize(L);
  auto f32slot = [&](const std::string &n, std::vector<float> &v, size_t ne) { v.resize(ne); slots[n] = {&v, 0}; };
  auto q4slot = [&](const std::string &n, std::vector<uint8_t> &v, size_t ne) { v.resize(ne / QK * QBYTES); slots[n] = {&v, 1}; };
  if (arch == VO_ARCH_GPTNEOX) {
    q4slot("gpt_neox.embed_in.weight", m->wte, (size_t)E * V);
    f32slot("gpt_neox.final_layer_norm.weight", m->lnf_w, E);
    f32slot("gpt_neox.final_layer_norm.bias", m->lnf_b, E);
    q4slot("embed_out.weight", m->lmh, (size_t)E * V);
    for (int i = 0; i < L; ++i) {
      auto &l = m->layers[i];
      const std::string p = "gpt_neox.layers." + std::to_string(i) + ".";
      f32slot(p + "input_layernorm.weight", l.ln1_w, E);
      f32slot(p + "input_layernorm.bias", l.ln1_b, E);
      f32slot(p + "post_attention_layernorm.weight", l.ln2_w, E);
      f32slot(p + "post_attention_layernorm.bias", l.ln2_b, E);
      q4slot(p + "attention.query.weight", l.wq, (size_t)E * E);
      f32slot(p + "attention.query.bias", l.bq, E);
      q4slot(p + "attention.key.weight", l.wk, (size_t)E * E);
      f32slot(p + "attention.key.bias", l.bk, E);
      q4slot(p + "attention.value.weight", l.wv, (size_t)E * E);
      f32slot(p + "attention.value.bias", l.bv, E);
      q4slot(p + "attention.dense.weight", l.wo, (size_t)E * E);
      f32slot(p + "attention.dense.bias", l.bo, E);
      q4slot(p + "mlp.dense_h_to_4h.weight", l.wfc, (size_t)E * 4 * E);
      f32slot(p + "mlp.dense_h_to_4h.bias", l.bfc, 4 * E);
      q4slot(p + "mlp.dense_4h_to_h.weight", l.wproj, (size_t)E * 4 * E);
      f32slot(p + "mlp.dense_4h_to_h.bias", l.bproj, E);
    }
  } else if (arch == VO_ARCH_BLOOM) {  // convert_bloom_to_ggml.py:22-34 names
    q4slot("tok_embeddings.weight", m->wte, (size_t)E * V);
    f32slot("norm.weight", m->emb_w, E);
    f32slot("norm.bias", m->emb_b, E);
    f32slot("output_norm.weight", m->lnf_w, E);
    f32slot("output_norm.bias", m->lnf_b, E);
    q4slot("output.weight", m->lmh, (size_t)E * V);
    for (int i = 0; i < L; ++i) {
      auto &l = m->layers[i];
      const std::string p = "layers." + std::to_string(i) + ".";
      f32slot(p + "attention_norm.weight", l.ln1_w, E);
      f32slot(p + "attention_norm.bias", l.ln1_b, E);
      q4slot(p + "attention.query_key_value.weight", l.wqkv, (size_t)E * 3 * E);
      f32slot(p + "attention.query_key_value.bias", l.bqkv, 3 * E);
      q4slot(p + "attention.wo.weight", l.wo, (size_t)E * E);
      f32slot(p + "attention.wo.bias", l.bo, E);
      f32slot(p + "ffn_norm.weight", l.ln2_w, E);
      f32slot(p + "ffn_norm.bias", l.ln2_b, E);
      q4slot(p + "feed_forward.w1.weight", l.wfc, (size_t)E * 4 * E);
      f32slot(p + "feed_forward.w1.bias", l.bfc, 4 * E);
      q4slot(p + "feed_forward.w2.weight", l.wproj, (size_t)E * 4 * E);
      f32slot(p + "feed_forward.w2.bias", l.bproj, E);
    }
  } else {
    q4slot("transformer.wte.weight", m->wte, (size_t)E * V);
    f32slot("transformer.ln_f.weight", m->lnf_w, E);
    f32slot("transformer.ln_f.bias", m->lnf_b, E);
    q4slot("lm_head.weight", m->lmh, (size_t)E * V);
    f32slot("lm_head.bias", m->lmh_b, V);
    for (int i = 0; i < L; ++i) {
      auto &l = m->layers[i];
      const std::string p = "transformer.h." + std::to_string(i) + ".";
      f32slot(p + "ln_1.weight", l.ln1_w, E);
      f32slot(p + "ln_1.bias", l.ln1_b, E);
      q4slot(p + "attn.q_proj.weight", l.wq, (size_t)E * E);
      q4slot(p + "attn.k_proj.weight", l.wk, (size_t)E * E);
      q4slot(p + "attn.v_proj.weight", l.wv, (size_t)E * E);
      q4slot(p + "attn.out_proj.weight", l.wo, (size_t)E * E);
      q4slot(p + "mlp.fc_in.weight", l.wfc, (size_t)E * 4 * E);
      f32slot(p + "mlp.fc_in.bias", l.bfc, 4 * E);
      q4slot(p + "mlp.fc_out.weight", l.wproj, (size_t)E * 4 * E);
      f32slot(p + "mlp.fc_out.bias", l.bproj, E);
    }
  }
}

// Tensor records until EOF (vsim.cpp:375-448): every one must name a slot of the right type
// and size.
bool read_tensors(std::ifstream &f, SlotMap &slots) {
  while (true) {
    int32_t n_dims, length, ftype;
    if (!read_all(f, &n_dims, 4)) break;
    if (n_dims < 1 || n_dims > 4) return false;
    read_all(f, &length, 4);
    read_all(f, &ftype, 4);
    if (length <= 0 || length > 1024) return false;
    size_t ne = 1;
    for (int i = 0; i < n_dims; ++i) {
      int32_t d;
      read_all(f, &d, 4);
      ne *= d;
    }
    std::string name(length, 0);
    read_all(f, &name[0], length);
    auto it = slots.find(name);
    if (it == slots.end()) {
      fprintf(stderr, "oracle: unknown tensor '%s'\n", name.c_str());
      return false;
    }
    if (it->second.second == 0) {
      auto *v = (std::vector<float> *)it->second.first;
      if (ftype != 0 || v->size() != ne || !read_all(f, v->data(), ne * 4)) return false;
    } else {
      auto *v = (std::vector<uint8_t> *)it->second.first;
      if (ftype != 2 || v->size() != ne / QK * QBYTES || !read_all(f, v->data(), v->size())) return false;
    }
  }
  return true;
}

void affine(std::vector<float> &x, const std::vector<float> &w, const std::vector<float> &b, int E, int N) {
  // ggml_add(ggml_mul(ggml_repeat(w, x), x), ggml_repeat(b, x))
  for (int t = 0; t < N; ++t)
    for (int i = 0; i < E; ++i) x[(size_t)t * E + i] = (w[i] * x[(size_t)t * E + i]) + b[i];
}

void add_bias(std::vector<float> &x, const std::vector<float> &b, int E, int N) {
  for (int t = 0; t < N; ++t)
    for (int i = 0; i < E; ++i) x[(size_t)t * E + i] = x[(size_t)t * E + i] + b[i];
}

// The BLOOM graph (no reference program composes it, SURVEY.md finding 2): the op sequence
// of the bloomz.cpp-style graph the reference's converter and quantizer target
// (convert_bloom_to_ggml.py, quantize_bloom.cpp), from reference ops only: embedding +
// word_embeddings_layernorm; per layer LN -> fused QKV (+bias; rows q|k|v) -> KQ -> scale
// -> ggml_alibi -> diag_mask_inf -> soft_max -> KQV -> wo (+bias) -> inpFF = attn + inpL
// -> LN -> w1 (+bias) -> GELU -> w2 (+bias) -> inpL = ff + inpFF; output_norm; lm_head.
void eval_bloom(Model &m, int n_past, const int32_t *tok, int N, float *logits, int nthreads) {
  const int E = m.n_embd, H = m.n_head, d = E / H, L = m.n_layer, V = m.n_vocab, F = 4 * E;
  const int n_ctx = m.n_ctx, nk = n_past + N;
  std::vector<float> inpL((size_t)E * N), cur((size_t)E * N), qkv((size_t)3 * E * N), Q((size_t)E * N),
      attn((size_t)E * N), inpFF((size_t)E * N), fch((size_t)F * N), ff((size_t)E * N);
  std::vector<float> KQ((size_t)H * N * nk), KQV((size_t)H * N * d);
  const size_t rbE = (size_t)E / QK * QBYTES;
  for (int t = 0; t < N; ++t) dequantize_row(m.wte.data() + (size_t)tok[t] * rbE, cur.data() + (size_t)t * E, E);
  for (int t = 0; t < N; ++t) norm_row(cur.data() + (size_t)t * E, inpL.data() + (size_t)t * E, E);
  affine(inpL, m.emb_w, m.emb_b, E, N);
  const float scale = (float)(1.0f / std::sqrt((double)(float(E) / H)));  // as vsim.cpp:589
  for (int il = 0; il < L; ++il) {
    Layer &l = m.layers[il];
    for (int t = 0; t < N; ++t) norm_row(inpL.data() + (size_t)t * E, cur.data() + (size_t)t * E, E);
    affine(cur, l.ln1_w, l.ln1_b, E, N);
    mul_mat_f(l.wqkv.data(), 3 * E, E, cur.data(), N, qkv.data(), nthreads);
    add_bias(qkv, l.bqkv, 3 * E, N);
    float *mk = m.mem_k.data() + (size_t)il * n_ctx * E;
    float *mv = m.mem_v.data() + (size_t)il * n_ctx * E;
    for (int t = 0; t < N; ++t) {  // views at offsets 0, E, 2E of each [3E] row
      std::memcpy(Q.data() + (size_t)t * E, qkv.data() + (size_t)t * 3 * E, sizeof(float) * E);
      std::memcpy(mk + (size_t)(n_past + t) * E, qkv.data() + (size_t)t * 3 * E + E, sizeof(float) * E);
      std::memcpy(mv + (size_t)(n_past + t) * E, qkv.data() + (size_t)t * 3 * E + 2 * E, sizeof(float) * E);
    }
    kq(mk, E, Q.data(), E, d, H, nk, N, KQ.data(), nthreads);
    for (auto &v : KQ) v *= scale;
    alibi(KQ.data(), nk, N, H, H);
    for (int h = 0; h < H; ++h)
      for (int j = 0; j < N; ++j)
        for (int i = n_past; i < nk; ++i)
          if (i > n_past + j) KQ[((size_t)h * N + j) * nk + i] = -INFINITY;
    for (int r = 0; r < H * N; ++r) soft_max_row(KQ.data() + (size_t)r * nk, nk);
    kqv(mv, E, KQ.data(), d, H, nk, N, KQV.data(), nthreads);
    for (int t = 0; t < N; ++t)
      for (int h = 0; h < H; ++h)
        for (int i = 0; i < d; ++i) cur[(size_t)t * E + h * d + i] = KQV[((size_t)h * N + t) * d + i];
    mul_mat_f(l.wo.data(), E, E, cur.data(), N, attn.data(), nthreads);
    add_bias(attn, l.bo, E, N);
    for (size_t i = 0; i < inpFF.size(); ++i) inpFF[i] = attn[i] + inpL[i];
    for (int t = 0; t < N; ++t) norm_row(inpFF.data() + (size_t)t * E, cur.data() + (size_t)t * E, E);
    affine(cur, l.ln2_w, l.ln2_b, E, N);
    mul_mat_f(l.wfc.data(), F, E, cur.data(), N, fch.data(), nthreads);
    add_bias(fch, l.bfc, F, N);
    gelu(fch.data(), fch.data(), F * N);
    mul_mat_f(l.wproj.data(), E, F, fch.data(), N, ff.data(), nthreads);
    add_bias(ff, l.bproj, E, N);
    for (size_t i = 0; i < inpL.size(); ++i) inpL[i] = ff[i] + inpFF[i];
  }
  for (int t = 0; t < N; ++t) norm_row(inpL.data() + (size_t)t * E, cur.data() + (size_t)t * E, E);
  affine(cur, m.lnf_w, m.lnf_b, E, N);
  std::vector<float> lg((size_t)V);  // the last row only, as in eval()
  mul_mat_f(m.lmh.data(), V, E, cur.data() + (size_t)E * (N - 1), 1, lg.data(), nthreads);
  std::memcpy(logits, lg.data(), sizeof(float) * V);
}

// vsim.cpp:470-747 (GPT-NeoX) ; the GPT-J graph is the same op sequence with ggml_rope
// (ggml.c:5919-5974), one LayerNorm feeding attention and MLP, no q/k/v/out biases and a
// biased lm_head.  Returns logits of the last token in `logits` (vsim.cpp:736-737).
void eval(Model &m, int n_past, const int32_t *tok, int N, float *logits, int nthreads) {
  if (m.arch == VO_ARCH_BLOOM) {
    eval_bloom(m, n_past, tok, N, logits, nthreads);
    return;
  }
  const int E = m.n_embd, H = m.n_head, d = E / H, L = m.n_layer, V = m.n_vocab, F = 4 * E;
  const int n_ctx = m.n_ctx;
  const bool gptj = m.arch == VO_ARCH_GPTJ;
  std::vector<float> inpL((size_t)E * N), cur((size_t)E * N), Q((size_t)E * N), Kc((size_t)E * N),
      Vc((size_t)E * N), ff((size_t)E * N), fch((size_t)F * N), attn((size_t)E * N);
  const size_t rbE = (size_t)E / QK * QBYTES;
  for (int t = 0; t < N; ++t) dequantize_row(m.wte.data() + (size_t)tok[t] * rbE, inpL.data() + (size_t)t * E, E);
  const int nk = n_past + N;
  std::vector<float> KQ((size_t)H * N * nk), KQV((size_t)H * N * d);
  // vsim.cpp:589: unqualified sqrt(float) binds ::sqrt(double) under -std=c++11
  const float scale = (float)(1.0f / std::sqrt((double)(float(E) / H)));
  for (int il = 0; il < L; ++il) {
    Layer &l = m.layers[il];
    for (int t = 0; t < N; ++t) norm_row(inpL.data() + (size_t)t * E, cur.data() + (size_t)t * E, E);
    affine(cur, l.ln1_w, l.ln1_b, E, N);
    mul_mat_f(l.wq.data(), E, E, cur.data(), N, Q.data(), nthreads);
    mul_mat_f(l.wk.data(), E, E, cur.data(), N, Kc.data(), nthreads);
    mul_mat_f(l.wv.data(), E, E, cur.data(), N, Vc.data(), nthreads);
    if (!gptj) {
      add_bias(Q, l.bq, E, N);
      add_bias(Kc, l.bk, E, N);
      add_bias(Vc, l.bv, E, N);
    }
    float *mk = m.mem_k.data() + (size_t)il * n_ctx * E;
    float *mv = m.mem_v.data() + (size_t)il * n_ctx * E;
    std::memcpy(mk + (size_t)n_past * E, Kc.data(), sizeof(float) * E * N);
    std::memcpy(mv + (size_t)n_past * E, Vc.data(), sizeof(float) * E * N);
    if (gptj) {
      rope_gptj(Q.data(), d, H, N, n_past, m.n_rot, 0);
      rope_gptj(mk, d, H, nk, n_past, m.n_rot, 1);
    } else {
      rope_neox(Q.data(), d, H, N, n_past, m.n_rot, 0);
      rope_neox(mk, d, H, nk, n_past, m.n_rot, 1);
    }
    kq(mk, E, Q.data(), E, d, H, nk, N, KQ.data(), nthreads);
    // scale, diag_mask_inf, soft_max: row by row (each row's ops are the reference's)
    parallel_items(H * N, H * N >= 64 ? nthreads : 1, [&](int r) {
      float *row = KQ.data() + (size_t)r * nk;
      const int j = r % N;
      for (int i = 0; i < nk; ++i) row[i] *= scale;
      for (int i = n_past; i < nk; ++i)
        if (i > n_past + j) row[i] = -INFINITY;
      soft_max_row(row, nk);
    });
    kqv(mv, E, KQ.data(), d, H, nk, N, KQV.data(), nthreads);
    for (int t = 0; t < N; ++t)
      for (int h = 0; h < H; ++h)
        for (int i = 0; i < d; ++i) cur[(size_t)t * E + h * d + i] = KQV[((size_t)h * N + t) * d + i];
    mul_mat_f(l.wo.data(), E, E, cur.data(), N, attn.data(), nthreads);
    if (!gptj) add_bias(attn, l.bo, E, N);  // bias + cur (commutative)
    // feed-forward input: GPT-J reuses the ln_1 output; GPT-NeoX parallel residual
    // normalises inpL again with post_attention_layernorm (vsim.cpp:660-696).
    if (gptj) {
      for (int t = 0; t < N; ++t) norm_row(inpL.data() + (size_t)t * E, ff.data() + (size_t)t * E, E);
      affine(ff, l.ln1_w, l.ln1_b, E, N);
    } else if (m.par_res == 1) {
      for (int t = 0; t < N; ++t) norm_row(inpL.data() + (size_t)t * E, ff.data() + (size_t)t * E, E);
      affine(ff, l.ln2_w, l.ln2_b, E, N);
    } else {
      for (size_t i = 0; i < ff.size(); ++i) ff[i] = attn[i] + inpL[i];
      std::vector<float> tmp(ff.size());
      for (int t = 0; t < N; ++t) norm_row(ff.data() + (size_t)t * E, tmp.data() + (size_t)t * E, E);
      ff.swap(tmp);
      affine(ff, l.ln2_w, l.ln2_b, E, N);
    }
    mul_mat_f(l.wfc.data(), F, E, ff.data(), N, fch.data(), nthreads);
    add_bias(fch, l.bfc, F, N);
    gelu(fch.data(), fch.data(), F * N);
    mul_mat_f(l.wproj.data(), E, F, fch.data(), N, ff.data(), nthreads);
    add_bias(ff, l.bproj, E, N);
    if (gptj || m.par_res == 1) {
      for (size_t i = 0; i < inpL.size(); ++i) inpL[i] = inpL[i] + (attn[i] + ff[i]);
    } else {
      // vsim.cpp:657: inpL = ggml_add(inpFF, inpL) — only the FF output is added back
      for (size_t i = 0; i < inpL.size(); ++i) inpL[i] = ff[i] + inpL[i];
    }
  }
  for (int t = 0; t < N; ++t) norm_row(inpL.data() + (size_t)t * E, cur.data() + (size_t)t * E, E);
  affine(cur, m.lnf_w, m.lnf_b, E, N);
  // lm_head (vsim.cpp:716-718) runs over all N rows and only the last row is returned
  // (vsim.cpp:736-737); every output row is its own chains over its own activation row, so
  // the last row alone gives the same bits
  std::vector<float> lg((size_t)V);
  mul_mat_f(m.lmh.data(), V, E, cur.data() + (size_t)E * (N - 1), 1, lg.data(), nthreads);
  if (gptj) add_bias(lg, m.lmh_b, V, 1);
  std::memcpy(logits, lg.data(), sizeof(float) * V);
}

// utils.cpp:339-422 sample_top_p_top_k_repeat_penalty
int sample(const float *logits, int n_logits, std::vector<int32_t> &last_n, double repeat_penalty, int top_k,
           double top_p, double temp, std::mt19937 &rng) {
  std::vector<std::pair<double, int32_t>> logits_id;
  logits_id.reserve(n_logits);
  const double scale = 1.0 / temp;
  for (int i = 0; i < n_logits; ++i) {
    if (std::find(last_n.begin(), last_n.end(), i) != last_n.end()) {
      if (logits[i] < 0.0)
        logits_id.push_back(std::make_pair(logits[i] * scale * repeat_penalty, i));
      else
        logits_id.push_back(std::make_pair(logits[i] * scale / repeat_penalty, i));
    } else {
      logits_id.push_back(std::make_pair(logits[i] * scale, i));
    }
  }
  std::partial_sort(logits_id.begin(), logits_id.begin() + top_k, logits_id.end(),
                    [](const std::pair<double, int32_t> &a, const std::pair<double, int32_t> &b) {
                      return a.first > b.first;
                    });
  logits_id.resize(top_k);
  double maxl = -INFINITY;
  for (const auto &kv : logits_id) maxl = std::max(maxl, kv.first);
  std::vector<double> probs;
  probs.reserve(logits_id.size());
  double sum = 0.0;
  for (const auto &kv : logits_id) {
    double p = std::exp(kv.first - maxl);
    probs.push_back(p);
    sum += p;
  }
  for (auto &p : probs) p /= sum;
  if (top_p < 1.0f) {
    double cumsum = 0.0f;
    for (int i = 0; i < (int)probs.size(); i++) {
      cumsum += probs[i];
      if (cumsum >= top_p) {
        probs.resize(i + 1);
        logits_id.resize(i + 1);
        break;
      }
    }
    cumsum = 1.0 / cumsum;
    for (int i = 0; i < (int)probs.size(); i++) probs[i] *= cumsum;
  }
  std::discrete_distribution<> dist(probs.begin(), probs.end());
  int idx = dist(rng);
  return logits_id[idx].second;
}

}  // namespace

extern "C" {

void vo_init_tables(void) { init_tables_once(); }
float vo_fp16_to_fp32(uint16_t h) { return h2f(h); }
uint16_t vo_fp32_to_fp16(float f) { return f2h(f); }
void vo_tables(uint16_t *exp_f16, uint16_t *gelu_f16) {
  init_tables_once();
  std::memcpy(exp_f16, g_exp_f16, sizeof(g_exp_f16));
  std::memcpy(gelu_f16, g_gelu_f16, sizeof(g_gelu_f16));
}

void vo_quantize_row_q4_0(const float *x, void *y, int k) { quantize_row(x, (uint8_t *)y, k); }
void vo_dequantize_row_q4_0(const void *x, float *y, int k) { dequantize_row((const uint8_t *)x, y, k); }
void vo_vec_dot_q4_0(int n, float *s, const void *x, const void *y) {
  *s = vec_dot_q4(n, (const uint8_t *)x, (const uint8_t *)y);
}
void vo_mul_mat_q4_0_f32(const void *W, int M, int K, const float *x, int N, float *y, int nthreads) {
  mul_mat_f((const uint8_t *)W, M, K, x, N, y, nthreads);
}
void vo_mul_mat_q4_0_q(const void *W, int M, int K, const void *xq, int N, float *y, int nthreads) {
  mul_mat_q((const uint8_t *)W, M, K, (const uint8_t *)xq, N, y, nthreads);
}
void vo_norm_f32(const float *x, float *y, int n, int rows) {
  for (int r = 0; r < rows; ++r) norm_row(x + (size_t)r * n, y + (size_t)r * n, n);
}
void vo_gelu_f32(const float *x, float *y, int n) { init_tables_once(); gelu(x, y, n); }
void vo_soft_max_f32(float *p, int nc, int nr) {
  init_tables_once();
  for (int r = 0; r < nr; ++r) soft_max_row(p + (size_t)r * nc, nc);
}
void vo_scale_f32(float *p, int n, float v) { for (int i = 0; i < n; ++i) p[i] *= v; }
void vo_alibi_f32(float *p, int nc, int nr, int nz, int n_head) { alibi(p, nc, nr, nz, n_head); }
void vo_diag_mask_inf_f32(float *p, int nc, int nr, int nz, int n_past) {
  for (int k = 0; k < nz; k++)
    for (int j = 0; j < nr; j++)
      for (int i = n_past; i < nc; i++)
        if (i > n_past + j) p[((size_t)k * nr + j) * nc + i] = -INFINITY;
}
void vo_rope_neox(float *x, int d, int H, int T, int n_past, int n_dims, int mode) {
  rope_neox(x, d, H, T, n_past, n_dims, mode);
}
void vo_rope_gptj(float *x, int d, int H, int T, int n_past, int n_dims, int mode) {
  rope_gptj(x, d, H, T, n_past, n_dims, mode);
}
void vo_kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int N, float *KQ) {
  kq(K, ldk, Q, ldq, d, H, nk, N, KQ);
}
void vo_kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int N, float *out) {
  kqv(V, ldv, S, d, H, nk, N, out);
}
void vo_get_rows_q4_0(const void *W, int K, const int32_t *rows, int n, float *y) {
  const size_t rb = (size_t)K / QK * QBYTES;
  for (int i = 0; i < n; ++i) dequantize_row((const uint8_t *)W + rows[i] * rb, y + (size_t)i * K, K);
}

void *vo_model_load(const char *path, int arch, int n_ctx) {
  init_tables_once();
  return load_model(path, arch, n_ctx);
}
// Synthetic weights generated in place (cpu_baseline sample of a full-width config):
// N(0, std) matrices / biases, 1 + N(0, std) LN gains, quantized with quantize_row_q4_0.
void *vo_model_synthetic(int arch, int n_vocab, int n_embd, int n_head, int n_layer, int n_rot, int n_ctx,
                         uint64_t seed, float stddev) {
  init_tables_once();
  auto *m = new Model();
  m->arch = arch;
  m->n_vocab = n_vocab; m->n_embd = n_embd; m->n_head = n_head; m->n_layer = n_layer; m->n_rot = n_rot;
  m->par_res = 1; m->ftype = 2; m->n_ctx = n_ctx;
  const int E = n_embd, F = 4 * E, V = n_vocab;
  // counter-seeded xorshift64* per row so rows can be generated in parallel
  auto rowgen = [](uint64_t st, float *out, int k, float sd) {
    st = st * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    for (int i = 0; i < k; i += 2) {
      st ^= st >> 12; st ^= st << 25; st ^= st >> 27;
      const uint64_t a = st * 0x2545F4914F6CDD1Dull;
      st ^= st >> 12; st ^= st << 25; st ^= st >> 27;
      const uint64_t b = st * 0x2545F4914F6CDD1Dull;
      const float u1 = ((a >> 40) + 1) * (1.0f / 16777217.0f), u2 = (b >> 40) * (1.0f / 16777216.0f);
      const float r = std::sqrt(-2.0f * std::log(u1)) * sd;
      out[i] = r * std::cos(6.2831853f * u2);
      if (i + 1 < k) out[i + 1] = r * std::sin(6.2831853f * u2);
    }
  };
  uint64_t tensor_id = seed << 20;
  const int nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  auto q4 = [&](std::vector<uint8_t> &v, size_t rows, int k) {
    v.resize(rows * (k / QK) * QBYTES);
    const uint64_t tid = ++tensor_id;
    parallel_rows((int)rows, nth, [&](int r0, int r1) {
      std::vector<float> tmp(k);
      for (int r = r0; r < r1; ++r) {
        rowgen((tid << 32) ^ (uint64_t)r, tmp.data(), k, stddev);
        quantize_row(tmp.data(), v.data() + (size_t)r * (k / QK) * QBYTES, k);
      }
    });
  };
  auto f32 = [&](std::vector<float> &v, int n, float mean) {
    v.resize(n);
    rowgen(++tensor_id, v.data(), n, stddev);
    for (auto &x : v) x += mean;
  };
  q4(m->wte, V, E);
  q4(m->lmh, V, E);
  f32(m->lnf_w, E, 1.0f); f32(m->lnf_b, E, 0.0f); f32(m->lmh_b, V, 0.0f);
  m->layers.resize(n_layer);
  for (auto &l : m->layers) {
    f32(l.ln1_w, E, 1.0f); f32(l.ln1_b, E, 0.0f); f32(l.ln2_w, E, 1.0f); f32(l.ln2_b, E, 0.0f);
    q4(l.wq, E, E); q4(l.wk, E, E); q4(l.wv, E, E); q4(l.wo, E, E);
    q4(l.wfc, F, E); q4(l.wproj, E, F);
    f32(l.bq, E, 0.0f); f32(l.bk, E, 0.0f); f32(l.bv, E, 0.0f); f32(l.bo, E, 0.0f);
    f32(l.bfc, F, 0.0f); f32(l.bproj, E, 0.0f);
    if (arch == VO_ARCH_BLOOM) { q4(l.wqkv, 3 * E, E); f32(l.bqkv, 3 * E, 0.0f); }
  }
  if (arch == VO_ARCH_BLOOM) { f32(m->emb_w, E, 1.0f); f32(m->emb_b, E, 0.0f); m->par_res = 0; m->n_rot = 0; }
  m->mem_k.assign((size_t)n_layer * n_ctx * E, 0.0f);
  m->mem_v.assign((size_t)n_layer * n_ctx * E, 0.0f);
  return m;
}

// An empty model of the given shape whose tensors are then set one by one by name
// (vo_model_set_tensor): the parity tests copy a device model's weights in.
void *vo_model_create(int arch, int n_vocab, int n_embd, int n_head, int n_layer, int n_rot, int par_res, int n_ctx) {
  init_tables_once();
  auto *m = new Model();
  m->arch = arch;
  m->n_vocab = n_vocab; m->n_embd = n_embd; m->n_head = n_head; m->n_layer = n_layer;
  m->n_rot = arch == VO_ARCH_BLOOM ? 0 : n_rot;
  m->par_res = arch == VO_ARCH_BLOOM ? 0 : arch == VO_ARCH_GPTJ ? 1 : par_res;
  m->ftype = 2; m->n_ctx = n_ctx;
  SlotMap slots;
  build_slots(m, slots);
  m->mem_k.assign((size_t)n_layer * n_ctx * n_embd, 0.0f);
  m->mem_v.assign((size_t)n_layer * n_ctx * n_embd, 0.0f);
  return m;
}
/* Q4_0 tensors in the file's AoS blocks, F32 as floats; -1: unknown name or wrong size */
int vo_model_set_tensor(void *mp, const char *name, const void *data, size_t nbytes) {
  auto *m = (Model *)mp;
  SlotMap slots;
  build_slots(m, slots);  // (same sizes again: the vectors keep what is already set)
  auto it = slots.find(name);
  if (it == slots.end()) return -1;
  if (it->second.second == 0) {
    auto *v = (std::vector<float> *)it->second.first;
    if (v->size() * 4 != nbytes) return -1;
    std::memcpy(v->data(), data, nbytes);
  } else {
    auto *v = (std::vector<uint8_t> *)it->second.first;
    if (v->size() != nbytes) return -1;
    std::memcpy(v->data(), data, nbytes);
  }
  return 0;
}

void vo_model_hparams(void *mp, int32_t *o) {
  auto *m = (Model *)mp;
  o[0] = m->n_vocab; o[1] = m->n_embd; o[2] = m->n_head; o[3] = m->n_layer;
  o[4] = m->n_rot; o[5] = m->par_res; o[6] = m->ftype; o[7] = m->n_ctx;
}
int vo_model_eval(void *mp, int n_past, const int32_t *tokens, int N, float *logits, int nthreads) {
  auto *m = (Model *)mp;
  if (N <= 0 || n_past + N > m->n_ctx) return -1;
  eval(*m, n_past, tokens, N, logits, nthreads);
  return 0;
}
void vo_model_free(void *mp) { delete (Model *)mp; }

// vsim.cpp:749-910 main_gptneox decode loop; returns the ids it prints between
// "<|BEGIN>" and "<END|>" (prompt echoed in n_batch+1 chunks, then sampled ids).
int vo_generate(void *mp, const int32_t *prompt, int n_prompt, int n_predict, int seed, int top_k, float top_p,
                float temp, int repeat_last_n, float repeat_penalty, int n_batch, int32_t *out, int out_cap,
                int nthreads) {
  auto *m = (Model *)mp;
  std::mt19937 rng(seed);
  std::vector<int32_t> embd_inp(prompt, prompt + n_prompt);
  n_predict = std::min(n_predict, m->n_ctx - (int)embd_inp.size());
  std::vector<float> logits(m->n_vocab);
  const int32_t warm[5] = {1, 2, 3, 4, 5};
  eval(*m, 0, warm, 5, logits.data(), nthreads);
  std::vector<int32_t> last_n(repeat_last_n, 0);
  std::vector<int32_t> embd;
  int n_past = 0, n_out = 0;
  for (int i = (int)embd.size(); i < (int)embd_inp.size() + n_predict; i++) {
    if (!embd.empty()) eval(*m, n_past, embd.data(), (int)embd.size(), logits.data(), nthreads);
    n_past += (int)embd.size();
    embd.clear();
    if (i >= (int)embd_inp.size()) {
      const int id = sample(logits.data(), m->n_vocab, last_n, repeat_penalty, (int)(float)top_k, top_p, temp, rng);
      last_n.erase(last_n.begin());
      last_n.push_back(id);
      embd.push_back(id);
    } else {
      for (int k = i; k < (int)embd_inp.size(); k++) {
        embd.push_back(embd_inp[k]);
        last_n.erase(last_n.begin());
        last_n.push_back(embd_inp[k]);
        if ((int)embd.size() > n_batch) break;
      }
      i += (int)embd.size() - 1;
    }
    for (auto id : embd)
      if (n_out < out_cap) out[n_out++] = id;
    if (embd.back() == 2) break;
  }
  return n_out;
}

}  // extern "C"
