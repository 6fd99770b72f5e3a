// vsim_amd/csrc/kern.hpp — device building blocks shared by the kernel files.
#pragma once

#include <type_traits>

#include "common.hpp"

namespace vsim {

// ------------------------------------------------------------------ activation factors
// xd, the exact path's dequantized activation d*(q-8), is stored pair-interleaved: within
// each group of four elements the middle two swap places, (x0, x2, x1, x3).  Two adjacent
// floats then hold the same factor slot (first or second) of two consecutive byte pairs,
// which is what one packed multiply needs (pair_terms4_x).
__host__ __device__ constexpr int xd_slot(int l) { return (l & ~3) | ((l & 1) << 1) | ((l >> 1) & 1); }

// ------------------------------------------------------------------ activation quantize
// One thread per 32-block.  Bit-identical to quantize_row_q4_0: fp32 amax, d = amax/7
// (correctly rounded division), id = 1/d, q = (int8)round(x*id) + 8 with round-half-
// away-from-zero, nibble pairs (q[2l], q[2l+1]).  Also emits xd = d*(q-8) per element,
// the activation factor f2/f3 of the reference dot (ggml.c:497-498).
// quantize_row_q4_0 of one 32-block: returns d; w = the 16 packed nibble bytes, out = the
// dequantized values d*(q-8) (one rounding each, as d*(float)(q-8) in dequantize_row_q4_0).
__device__ __forceinline__ float q4_block(const float *v, uint32_t w[4], float *out) {
  float amax = 0.0f;
#pragma unroll
  for (int l = 0; l < QK; ++l) amax = amax > fabsf(v[l]) ? amax : fabsf(v[l]);
  const float d = amax / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = 0;
#pragma unroll
  for (int l = 0; l < QK; l += 2) {
    const int q0 = x86_round_i8(v[l] * id) + 8;
    const int q1 = x86_round_i8(v[l + 1] * id) + 8;
    w[l / 8] |= (uint32_t)((q0 & 0xF) | ((q1 & 0xF) << 4)) << (8 * ((l / 2) & 3));
    out[l] = d * (float)(q0 - 8);
    out[l + 1] = d * (float)(q1 - 8);
  }
  return d;
}

__device__ __forceinline__ void quantize_block(const float *v, uint8_t *qs_out, float *d_out, float *xd_out) {
  uint32_t w[4];
  float out[QK];
  const float d = q4_block(v, w, out);
  *(uint4 *)qs_out = make_uint4(w[0], w[1], w[2], w[3]);
  *d_out = d;
  if (xd_out) {
    float4 *o = (float4 *)xd_out;
#pragma unroll
    for (int i = 0; i < QK / 4; ++i) o[i] = make_float4(out[4 * i], out[4 * i + 2], out[4 * i + 1], out[4 * i + 3]);
  }
}

// ------------------------------------------------------------------ pair products
// The reference's per-byte term (imax.c:1219-1226): f0 = d0*(lo-8), f1 = d0*(hi-8),
// p = f0*f2 + f1*f3, every product and the sum rounded separately (no FMA).  The nibble
// value n - 8 is formed exactly as (2^23 + n) - (2^23 + 8): v_perm_b32 places nibble byte k
// under the exponent byte 0x4B, and the subtraction pairs up into v_pk_add_f32.
__device__ __forceinline__ void pair_terms4(uint32_t w, float d0, const float *x8, float *p4) {
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float n0 = __uint_as_float(__builtin_amdgcn_perm(0x4B4B4B4Bu, lo, 0x040C0C00u | k)) - 8388616.0f;
    const float n1 = __uint_as_float(__builtin_amdgcn_perm(0x4B4B4B4Bu, hi, 0x040C0C00u | k)) - 8388616.0f;
    const float f0 = d0 * n0, f1 = d0 * n1;
    p4[k] = f0 * x8[2 * k] + f1 * x8[2 * k + 1];
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// v_cvt_f32_ubyteK: byte K of a word as float, one instruction (left to itself the compiler
// extracts each byte first)
template <int K>
__device__ __forceinline__ float cvt_ubyte(uint32_t w) {
  float f;
  if (K == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(w));
  if (K == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(w));
  if (K == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(w));
  if (K == 3) asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(w));
  return f;
}

// The same terms with f = d0*(n-8) as one fused multiply-add: fma(n, d0, -8*d0) rounds the
// exact product d0*(n-8) once, as the reference's d0*(float)(n-8) does (-8*d0 is exact, n
// exact), for every finite d0.  n comes from v_cvt_f32_ubyteN on the masked nibble bytes.
// Zero signs of a term may differ from the reference (0*(n-8) vs fma's +0); a chain that
// starts at +0 is unaffected by the sign of a zero term.
__device__ __forceinline__ void pair_terms4_fma(uint32_t w, f32x2 d2, f32x2 m2, const f32x2 *x4, float *p4) {
  const uint32_t lo = w & 0x0F0F0F0Fu, hi = (w >> 4) & 0x0F0F0F0Fu;
  auto term = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    f32x2 n;
    n.x = cvt_ubyte<k>(lo);
    n.y = cvt_ubyte<k>(hi);
    const f32x2 f = __builtin_elementwise_fma(n, d2, m2);
    const f32x2 t = f * x4[k];
    p4[k] = t.x + t.y;
  };
  term(std::integral_constant<int, 0>{});
  term(std::integral_constant<int, 1>{});
  term(std::integral_constant<int, 2>{});
  term(std::integral_constant<int, 3>{});
}

// The four terms of a word with pairs packed across the two lanes of each vector op: byte k
// of lo (hi) holds the first (second) nibble of pair k, and v_cvt_pk_f32_fp8 turns two of
// those bytes into floats at once -- an e4m3 byte with value n in 0..15 decodes to exactly
// n * 2^-9, so with d512 = 512*d0 the fma gives d0*(n-8) exactly as above.  xw holds the
// pair-interleaved factors (xd_slot): xw[0] = {x0, x2} (first factors of pairs 0 and 1),
// xw[1] = {x1, x3}, xw[2] = {x4, x6}, xw[3] = {x5, x7}.  Per word: 3 integer ops, 4
// conversions, 4 fma, 4 mul, 2 add (all packed) for the reference's 4 x 7 scalar ops.
__device__ __forceinline__ void pair_terms4_x(uint32_t w, f32x2 d512, f32x2 m2, const f32x2 *xw, float *p4) {
  const int lo = (int)(w & 0x0F0F0F0Fu), hi = (int)((w >> 4) & 0x0F0F0F0Fu);
  const f32x2 f01 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(lo, false), d512, m2);
  const f32x2 g01 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(hi, false), d512, m2);
  const f32x2 f23 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(lo, true), d512, m2);
  const f32x2 g23 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(hi, true), d512, m2);
  const f32x2 t01 = f01 * xw[0] + g01 * xw[1];
  const f32x2 t23 = f23 * xw[2] + g23 * xw[3];
  p4[0] = t01.x;
  p4[1] = t01.y;
  p4[2] = t23.x;
  p4[3] = t23.y;
}

// The same four terms with the activation factors broadcast by DPP instead of held per lane: a
// half-wave works on one block, and its 32 factors sit in two VGPRs, F0 = memory slots 0-15 and
// F1 = slots 16-31 of its block in each 16-lane row (rows 0-1: the lower half's block, rows 2-3:
// the upper half's).  row_newbcast:n hands every lane of a row that row's lane n, folded into the
// v_mul_f32 that uses it, so a product costs one plain multiply and no factor registers or LDS
// broadcast reads; the products and sums round exactly as pair_terms4_x's packed ones.
template <int POS>
__device__ __forceinline__ float xbcast(float f0, float f1) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(POS < 16 ? f0 : f1), 0x150 + (POS & 15), 0xF, 0xF,
                                                    false));
}
template <int W>  // word W of the block: pairs 4W .. 4W+3, natural factor elements 8W .. 8W+7
__device__ __forceinline__ void pair_terms4_dpp(uint32_t w, f32x2 d512, f32x2 m2, float F0, float F1, float *p4) {
  const int lo = (int)(w & 0x0F0F0F0Fu), hi = (int)((w >> 4) & 0x0F0F0F0Fu);
  const f32x2 f01 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(lo, false), d512, m2);
  const f32x2 g01 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(hi, false), d512, m2);
  const f32x2 f23 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(lo, true), d512, m2);
  const f32x2 g23 = __builtin_elementwise_fma(__builtin_amdgcn_cvt_pk_f32_fp8(hi, true), d512, m2);
  // pair 4W + k takes natural elements 8W + 2k (first factor) and 8W + 2k + 1, at memory slots xd_slot()
  p4[0] = xbcast<xd_slot(8 * W + 0)>(F0, F1) * f01.x + xbcast<xd_slot(8 * W + 1)>(F0, F1) * g01.x;
  p4[1] = xbcast<xd_slot(8 * W + 2)>(F0, F1) * f01.y + xbcast<xd_slot(8 * W + 3)>(F0, F1) * g01.y;
  p4[2] = xbcast<xd_slot(8 * W + 4)>(F0, F1) * f23.x + xbcast<xd_slot(8 * W + 5)>(F0, F1) * g23.x;
  p4[3] = xbcast<xd_slot(8 * W + 6)>(F0, F1) * f23.y + xbcast<xd_slot(8 * W + 7)>(F0, F1) * g23.y;
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }

// LDS-DMA: each lane's 16 (4) bytes from its own global address land lane-linearly at the
// wave-uniform LDS address.  Inline asm keeps the load out of the compiler's wait-count
// bookkeeping: completion is retired by the explicit vmcnt waits.  nt: streamed once (the
// GEMV weights); without it the lines stay in L2 for the other workgroups (GEMM operands).
template <bool NT = true>
__device__ __forceinline__ void glds16(const void *g, uint32_t lds) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
// (sc1: device-coherent, for data another XCD wrote write-through in the same launch)
__device__ __forceinline__ void glds16_sc1(const void *g, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
template <bool NT = true>
__device__ __forceinline__ void glds4(const void *g, uint32_t lds) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4_sc1(const void *g, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

constexpr int NORM_THREADS = 256;

__device__ __forceinline__ int ulp_exp(float x) {
  const uint32_t b = __float_as_uint(x) & 0x7FFFFFFFu;
  if (b == 0) return 1 << 30;
  const int e = (int)(b >> 23);
  return e == 0 ? -149 : e - 150;
}

}  // namespace vsim

namespace vsim {

// ------------------------------------------------------------------ sequential double sum
// The reference's mean sum, s = ((0 + x0) + x1) + ... in double over a float row (ggml.c:
// 4264-4270), by one wave without running the n dependent adds when it can prove the result:
// chunks of 256 elements (4 per lane), and per chunk
//  * a certificate that every partial sum of the chunk is exact in double (its elements are
//    multiples of 2^umin and sum|x| < 2^(53+umin)), so the chunk's prefix sums P_j are exact
//    in any order (a lane-local sum, then a wave scan);
//  * speculation from the running value s at the chunk's position b: T_j = s + (P_j - P_b),
//    each checked with TwoSum.  While every T_j is exact, each sequential add was exact and
//    the sequential value after j elements is T_j; at the first j whose add rounds, the
//    sequential value is RN(s + (P_j - P_b)) = T_j (the exact operand of that one rounding),
//    and speculation restarts there.  A chunk that fails its certificate, or rounds more than
//    CAP times, is added sequentially by lane 0 from where it stands.
// Rows with one tiny element (why the whole-row certificate fails on ~3 % of rows) pass every
// chunk certificate and speculate without a restart: 16 chunk steps instead of 4096 adds.
__device__ __forceinline__ double rl_d(double v, int l) {  // lane l's v (l wave-uniform)
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xFFFFFFFF), l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double seq_sum_exact_inl(const float *row, int n, int lane) {
  constexpr int CAP = 32;
  const int n4 = n / 4;
  double s = 0.0;
  for (int c4 = 0; c4 < n4; c4 += 64) {
    const int i4 = c4 + lane;
    const float4 v = i4 < n4 ? ((const float4 *)row)[i4] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float e[4] = {v.x, v.y, v.z, v.w};
    int um = 1 << 30;
    double sa = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      um = min(um, ulp_exp(e[k]));
      sa += (double)fabsf(e[k]);
    }
    um = wave_min_i(um);
    sa = wave_sum_d(sa);
    const int cn = min(256, n - 4 * c4);  // elements in this chunk
    int b = 0;                            // elements of the chunk already in s
    if (um == (1 << 30) || sa * (1.0 + 0x1.0p-30) < ldexp(1.0, 53 + um)) {
      // exact prefix sums: p[k] = elements 0 .. 4 lane + k of the chunk
      double p[4];
      p[0] = e[0];
#pragma unroll
      for (int k = 1; k < 4; ++k) p[k] = p[k - 1] + (double)e[k];
      double x = p[3];  // inclusive scan of the lanes' sums
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const double t = __shfl_up(x, d, 64);
        if (lane >= d) x += t;
      }
      const double ex = x - p[3];
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] += ex;
      double pb = 0.0;  // P_b
      for (int r = 0; r <= CAP; ++r) {
        // first element position j (1-based within the chunk, j > b) whose add rounds
        int jl = 1 << 30;
#pragma unroll
        for (int k = 3; k >= 0; --k) {
          const int j = 4 * lane + k + 1;
          if (j > b && j <= cn) {
            const double d = p[k] - pb, t = s + d, bb = t - s, er = (s - (t - bb)) + (d - bb);
            if (er != 0.0 || t != t) jl = j;
          }
        }
        const int j = wave_min_i(jl);
        if (j == (1 << 30)) {  // every remaining add exact (n % 4 == 0: the chunk ends on a lane's p[3])
          s = s + (rl_d(p[3], (cn - 1) >> 2) - pb);
          b = cn;
          break;
        }
        const int kj = (j - 1) & 3;
        const double pj = rl_d(kj == 0 ? p[0] : kj == 1 ? p[1] : kj == 2 ? p[2] : p[3], (j - 1) >> 2);
        s = s + (pj - pb);  // the one rounding of step j
        pb = pj;
        b = j;
      }
    }
    if (b < cn) {  // certificate failed or too many roundings: the rest of the chunk in order
      double m = s;
      if (lane == 0)
        for (int j = b; j < cn; ++j) m += (double)row[4 * c4 + j];
      s = rl_d(m, 0);
    }
  }
  return s;
}
__device__ __noinline__ double seq_sum_exact(const float *row, int n, int lane) { return seq_sum_exact_inl(row, n, lane); }

// ------------------------------------------------------------------ exact LayerNorm core
// ggml_compute_forward_norm_f32 (ggml.c:4246-4304) for one row by one NT-thread block,
// result left in `row` (LDS, n floats, in place).  The reference sums sequentially in
// double; we sum in parallel and prove the sum equal to the sequential one, falling back
// to the sequential loop otherwise:
//  * mean: every partial sum of floats that are multiples of 2^umin is exact in double
//    while sum|x| < 2^(53+umin), so then any order gives the sequential value;
//  * variance: sequential and tree sums of w_i = v_i^2 >= 0 differ by at most
//    (2n+64)*2^-53*sum(w); if both ends of that interval give the same float scale
//    (the map S -> (float)(1/sqrt(S/n+eps)) is monotone) the scale is the reference's.
// Optional affine y = w*y + b (ggml_add(ggml_mul(repeat(w), cur), repeat(b))).
// Optional residual join first (the previous layer's, vsim.cpp:694-695): the normalized row is
// v = x + ((ja + jab) + (jf + jfb)) (jab, jfb may be null), or with one side only (serial
// residual graphs, vsim.cpp:628, 659 and BLOOM): v = x + (ja + jab) or v = x + (jf + jfb);
// written to jout when jout != null.
// stats (optional): [0] mean fallbacks, [1] variance fallbacks.
// CERT = false (fast-mode prompt batches only): the tree sums are used as they are, without
// the certificate and its sequential fallbacks (a fallback row costs one lane ~25-50 us).
// n % 4 == 0; float4 accesses, NT threads x 4 elements per pass, so for n <= 4*NT every load
// of a pass issues at once (a loop of scalar loads behind branches serialized on their
// latency and dominated the kernel).
template <int NT, bool CERT = true, int UP = 4>
__device__ void ln_exact_lds_t(const float *__restrict__ x, float *row, int n, const float *__restrict__ gw,
                               const float *__restrict__ gb, unsigned *stats, const float *__restrict__ ja = nullptr,
                               const float *__restrict__ jab = nullptr, const float *__restrict__ jf = nullptr,
                               const float *__restrict__ jfb = nullptr, float *__restrict__ jout = nullptr,
                               int s0 = 0, int s1 = 1 << 30) {
  // [s0, s1): the float4 slice of the row this workgroup normalizes (and writes to jout);
  // the statistics always cover the whole row
  constexpr int NW = NT / 64;
  __shared__ double shs[NW], shsa[NW];
  __shared__ int shu[NW];
  __shared__ double bcast_d;
  __shared__ float bcast_f;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n4 = n / 4;
  const double eps = 1e-5f;
  double s = 0.0, sa = 0.0;
  int um = 1 << 30;
  // affine factors of this thread's first float4, loaded up front (used in the last pass)
  const int i0 = max(s0, 0) + (int)threadIdx.x;  // this thread's first float4 of the slice
  float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), b0 = w0;
  if (gw && i0 < min(s1, n4)) {
    w0 = ((const float4 *)gw)[i0];
    b0 = ((const float4 *)gb)[i0];
  }
  auto join = [&](int i, float4 v, float4 a, float4 ab, float4 f, float4 fb) {
    if (ja || jf) {
      if (jab) a = make_float4(a.x + ab.x, a.y + ab.y, a.z + ab.z, a.w + ab.w);
      if (jfb) f = make_float4(f.x + fb.x, f.y + fb.y, f.z + fb.z, f.w + fb.w);
      const float4 t = !jf ? a : !ja ? f : make_float4(a.x + f.x, a.y + f.y, a.z + f.z, a.w + f.w);
      v = make_float4(v.x + t.x, v.y + t.y, v.z + t.z, v.w + t.w);
      if (jout && i >= s0 && i < s1) ((float4 *)jout)[i] = v;
    }
    ((float4 *)row)[i] = v;
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s += (double)e[j];
      sa += (double)fabsf(e[j]);
      um = min(um, ulp_exp(e[j]));
    }
  };
  auto ld4 = [](const float *p, int i) {
    return p ? ((const float4 *)p)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  // rows up to UP * NT float4: every load issued before any arithmetic
  if (n4 <= UP * NT) {
    float4 v[UP], a[UP], ab[UP], f[UP], fb[UP];
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const int i = (int)threadIdx.x + u * NT;
      if (i < n4) {
        v[u] = ((const float4 *)x)[i];
        a[u] = ld4(ja, i);
        ab[u] = ld4(jab, i);
        f[u] = ld4(jf, i);
        fb[u] = ld4(jfb, i);
      }
    }
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const int i = (int)threadIdx.x + u * NT;
      if (i < n4) join(i, v[u], a[u], ab[u], f[u], fb[u]);
    }
  } else {
    for (int i = threadIdx.x; i < n4; i += NT)
      join(i, ((const float4 *)x)[i], ld4(ja, i), ld4(jab, i), ld4(jf, i), ld4(jfb, i));
  }
  s = wave_sum_d(s);
  sa = wave_sum_d(sa);
  um = wave_min_i(um);
  if (lane == 0) {
    shs[wid] = s;
    shsa[wid] = sa;
    shu[wid] = um;
  }
  __syncthreads();
  s = 0.0;
  sa = 0.0;
  um = 1 << 30;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    s += shs[w];
    sa += shsa[w];
    um = min(um, shu[w]);
  }
  const bool exact = !CERT || (um == (1 << 30)) || sa * (1.0 + 0x1.0p-30) < ldexp(1.0, 53 + um);
  if (!exact) {
    if (wid == 0) {
      const double m = seq_sum_exact(row, n, lane);
      if (lane == 0) {
        bcast_d = m;
        if (stats) atomicAdd(&stats[0], 1u);
      }
    }
    __syncthreads();
    s = bcast_d;
  }
  const double mean = s / n;
  double s2 = 0.0;
  for (int i = threadIdx.x; i < n4; i += NT) {
    const float4 v4 = ((const float4 *)row)[i];
    const float e[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double v = (double)e[j] - mean;
      s2 += v * v;
    }
  }
  s2 = wave_sum_d(s2);
  __syncthreads();  // everyone has read shs above
  if (lane == 0) shs[wid] = s2;
  __syncthreads();
  s2 = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) s2 += shs[w];
  const double B = (2.0 * n + 64.0) * 0x1.0p-53 * s2;
  const float sc_lo = (float)(1.0 / sqrt((s2 + B) / n + eps));
  const float sc_hi = (float)(1.0 / sqrt((s2 - B > 0.0 ? s2 - B : 0.0) / n + eps));
  float scale = sc_lo;
  if (CERT && sc_lo != sc_hi) {
    if (threadIdx.x == 0) {
      double q = 0.0;
      for (int i = 0; i < n; ++i) {
        const double v = (double)row[i] - mean;
        q += v * v;
      }
      bcast_f = (float)(1.0 / sqrt(q / n + eps));
      if (stats) atomicAdd(&stats[1], 1u);
    }
    __syncthreads();
    scale = bcast_f;
  }
  for (int i = max(s0, 0) + (int)threadIdx.x; i < min(s1, n4); i += NT) {
    const float4 v4 = ((const float4 *)row)[i];
    float e[4] = {v4.x, v4.y, v4.z, v4.w};
    float4 w4 = w0, b4 = b0;
    if (gw && i != i0) {
      w4 = ((const float4 *)gw)[i];
      b4 = ((const float4 *)gb)[i];
    }
    const float wv[4] = {w4.x, w4.y, w4.z, w4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = (float)((double)e[j] - mean);
      v = v * scale;
      if (gw) v = (wv[j] * v) + bv[j];
      e[j] = v;
    }
    ((float4 *)row)[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
  __syncthreads();
}

__device__ __forceinline__ void ln_exact_lds(const float *__restrict__ x, float *row, int n, const float *__restrict__ gw,
                                             const float *__restrict__ gb, unsigned *stats) {
  ln_exact_lds_t<NORM_THREADS>(x, row, n, gw, gb, stats);
}

// Quantize one 32-value block per half-wave (lanes 0-31 -> block A, 32-63 -> block B) with
// quantize_row_q4_0 semantics (see quantize_block_lanes below).
// Stores of data that workgroups on other XCDs read later in the same launch (k_layer_exact):
// agent-scope relaxed atomic stores are sc1 (write-through) stores, visible device-wide after
// the storing wave's vmcnt drain, without the L2 write-back a release fence costs every
// producer workgroup (MI355X_MICROARCH.md, inter-workgroup visibility).
template <bool CO, typename T>
__device__ __forceinline__ void st_out(T *p, T v) {
  if constexpr (CO) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// quantize_row_q4_0 of one 32-block held one value per lane by a half-wave (lanes 0-31:
// block A, 32-63: block B): returns the lane's code q (0..15) and the block's scale d.
__device__ __forceinline__ int q4_half(float v, float &d) {
  // amax over the half-wave: DPP within rows of 16 lanes, then rows 0<->1 and 2<->3 by
  // ds_swizzle (xor 16); no LDS round trips in the dependent chain
  auto mx = [](float a, float b) { return a > b ? a : b; };
  float a = fabsf(v);
  a = mx(a, dpp::mov<dpp::QP_XOR1, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::QP_XOR2, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::HALF_MIRROR, 0xF>(a, 0.0f));
  a = mx(a, dpp::mov<dpp::MIRROR, 0xF>(a, 0.0f));
  a = mx(a, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(a), 0x401F)));
  d = a / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  return x86_round_i8(v * id) + 8;
}

template <bool CO = false>
__device__ __forceinline__ void quantize_half(float v, int lane, bool ok, uint8_t *qs_out, float *d_out,
                                              float *xd_out) {
  float d;
  const int q = q4_half(v, d);
  const int l = lane & 31;
  // byte of pair l/2 (nibbles of lanes 2j, 2j+1), then OR of each 8-lane group's bytes into
  // its word: xor 1, xor 2, and the half-row mirror (lane i <-> 7-i) reach all 8 lanes
  const int qn = dpp::mov<dpp::QP_XOR1, 0xF>(q, 0);
  const uint32_t byte = (l & 1) ? (uint32_t)((qn & 0xF) | ((q & 0xF) << 4)) : (uint32_t)((q & 0xF) | ((qn & 0xF) << 4));
  uint32_t word = byte << (8 * ((l >> 1) & 3));
  word |= (uint32_t)dpp::mov<dpp::QP_XOR2, 0xF>((int)word, 0);
  word |= (uint32_t)dpp::mov<dpp::HALF_MIRROR, 0xF>((int)word, 0);
  if (ok) {
    if ((l & 7) == 0) st_out<CO>((uint32_t *)qs_out + (l >> 3), word);
    if (l == 0) st_out<CO>(d_out, d);
    st_out<CO>(xd_out + xd_slot(l), d * (float)(q - 8));
  }
}

// Quantize one 32-element block held by lanes 0..31 of a wave (value v in lane l = element
// l): quantize_row_q4_0 semantics; writes the 16 nibble bytes, d and the 32 xd factors.
// Must be called by all 64 lanes of the wave (lanes 32..63 pass v = 0 and write nothing).
__device__ __forceinline__ void quantize_block_lanes(float v, int lane, uint8_t *qs_out, float *d_out,
                                                     float *xd_out) {
  float a = lane < 32 ? fabsf(v) : 0.0f;
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    const float t = __shfl_xor(a, o, 64);
    a = a > t ? a : t;
  }
  const float amax = a;
  const float d = amax / 7.0f;
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  const int q = x86_round_i8(v * id) + 8;
  // byte j = q[2j] | q[2j+1] << 4 ; word w = bytes 4w..4w+3
  const int qn = __shfl_xor(q, 1, 64);
  const uint32_t byte = (lane & 1) ? 0u : (uint32_t)((q & 0xF) | ((qn & 0xF) << 4));
  uint32_t word = byte << (8 * ((lane >> 1) & 3));
  word |= __shfl_xor(word, 2, 64);
  word |= __shfl_xor(word, 4, 64);
  if (lane < 32) {
    if ((lane & 7) == 0) ((uint32_t *)qs_out)[lane >> 3] = word;
    if (lane == 0) *d_out = d;
    xd_out[xd_slot(lane)] = d * (float)(q - 8);
  }
}

// One LayerNorm job (join, norm, affine) by one NT-thread workgroup, then quantize_row_q4_0 of
// the normalized blocks [b0, b1) by whole waves, two 32-blocks per wave step (k_ln_quant: a
// slice per workgroup).  row: n floats of LDS.
template <int NT>
__device__ __forceinline__ void ln_quant_job(const LnQuantJob &J, float *row, int n, unsigned *stats, int b0, int b1) {
  const int lane = threadIdx.x & 63;
  ln_exact_lds_t<NT>(J.x, row, n, J.w, J.b, stats, J.ja, J.jab, J.jf, J.jfb, J.jout, b0 * QK / 4, b1 * QK / 4);
  for (int b2 = threadIdx.x >> 6; b0 + 2 * b2 < b1; b2 += NT / 64) {
    const int b = b0 + 2 * b2 + (lane >> 5);
    const bool ok = b < b1;
    const float v = ok ? row[b * QK + (lane & 31)] : 0.0f;
    quantize_half(v, lane, ok, J.qs + (size_t)b * 16, J.d + b, J.xd + (size_t)b * QK);
  }
}

}  // namespace vsim
