// tools/chain_lat.hip — dependent-chain latency of the VALU forms that can carry the exact
// decode chain (sumf = sumf + t, one rounding per step), one wave on one SIMD, operands in VGPRs.
// Cycles from s_memtime (shader clock) and the clock itself from s_memrealtime (100 MHz).
//   v_add_f32 e32 / e64, v_fmac_f32 (t * 1.0 + acc: one rounding of acc + t, the same value),
//   v_fma_f32 (acc * 1.0 + t), v_pk_add_f32 (two chains per instruction), v_add_f64,
//   v_add_u32 (integer baseline), v_mov_b32 (pass-through baseline).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/chain_lat tools/chain_lat.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define STEP_ADD "v_add_f32 %0, %0, %1\n\t"
#define STEP_ADD64 "v_add_f32_e64 %0, %0, %1\n\t"
#define STEP_FMAC "v_fmac_f32 %0, 1.0, %1\n\t"
#define STEP_FMA "v_fma_f32 %0, %0, 1.0, %1\n\t"
#define STEP_MUL "v_mul_f32 %0, %0, %1\n\t"
#define STEP_U32 "v_add_u32 %0, %0, %1\n\t"
#define STEP_MOV "v_mov_b32 %0, %0\n\t"
#define X8(s) s s s s s s s s
#define X64(s) X8(X8(s))

template <int V>
__global__ void k_chain(float *out, unsigned long long *cyc, int n, float inc) {
  float a = threadIdx.x * 1e-3f;
  double ad = a;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 ap = {a, a + 1.0f}, ip = {inc, inc};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
    if constexpr (V == 0) asm volatile(X64(STEP_ADD) : "+v"(a) : "v"(inc));
    if constexpr (V == 1) asm volatile(X64(STEP_ADD64) : "+v"(a) : "v"(inc));
    if constexpr (V == 2) asm volatile(X64(STEP_FMAC) : "+v"(a) : "v"(inc));
    if constexpr (V == 3) asm volatile(X64(STEP_FMA) : "+v"(a) : "v"(inc));
    if constexpr (V == 4) asm volatile(X64("v_pk_add_f32 %0, %0, %1\n\t") : "+v"(ap) : "v"(ip));
    if constexpr (V == 5) asm volatile(X64("v_add_f64 %0, %0, %1\n\t") : "+v"(ad) : "v"((double)inc));
    if constexpr (V == 6) asm volatile(X64(STEP_MUL) : "+v"(a) : "v"(inc));
    if constexpr (V == 7) asm volatile(X64(STEP_U32) : "+v"(a) : "v"(inc));
    if constexpr (V == 8) asm volatile(X64(STEP_MOV) : "+v"(a));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[threadIdx.x] = a + (float)ad + ap.x + ap.y;
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = r1 - r0;
  }
}

static const char *kName[] = {"v_add_f32 (e32)", "v_add_f32 (e64)", "v_fmac_f32 (t*1+acc)", "v_fma_f32 (acc*1+t)",
                              "v_pk_add_f32 (2 chains)", "v_add_f64", "v_mul_f32", "v_add_u32", "v_mov_b32"};

template <int V>
void run(float *out, unsigned long long *cyc) {
  const int n = 2048;
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((k_chain<V>), 1, 64, 0, 0, out, cyc, n, 1e-7f);
  unsigned long long c[2];
  (void)hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
  const double steps = n * 64.0;
  printf("%-26s %6.2f cycles per dependent step, %6.3f ns (clock %.2f GHz)\n", kName[V], c[0] / steps,
         c[1] * 10.0 / steps, c[0] / (c[1] * 10.0));
}

int main() {
  float *out;
  unsigned long long *cyc;
  (void)hipMalloc(&out, 256);
  (void)hipMalloc(&cyc, 16);
  run<0>(out, cyc);
  run<1>(out, cyc);
  run<2>(out, cyc);
  run<3>(out, cyc);
  run<4>(out, cyc);
  run<5>(out, cyc);
  run<6>(out, cyc);
  run<7>(out, cyc);
  run<8>(out, cyc);
  return 0;
}
