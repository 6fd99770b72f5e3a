// tools/lat_probe.hip — dependent-add latency of one wave on gfx950 by exec width.
// A single wave runs N dependent v_add_f32 on registers only; cycles from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ACTIVE, int CH>
__global__ void k_lat(float *out, unsigned long long *cyc, int n, float inc) {
  const int lane = threadIdx.x;
  float s[CH];
#pragma unroll
  for (int h = 0; h < CH; ++h) s[h] = lane * 1e-3f + h;
  unsigned long long t0 = 0, t1 = 0;
  if (lane < ACTIVE) {
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int h = 0; h < CH; ++h) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[h]) : "v"(inc));
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  float r = 0.f;
#pragma unroll
  for (int h = 0; h < CH; ++h) r += s[h];
  out[lane] = r;
  if (lane == 0) cyc[0] = t1 - t0;
}

template <int ACTIVE, int CH>
void run(float *out, unsigned long long *cyc) {
  const int n = 4096;
  hipLaunchKernelGGL((k_lat<ACTIVE, CH>), 1, 64, 0, 0, out, cyc, n, 1e-7f);
  hipLaunchKernelGGL((k_lat<ACTIVE, CH>), 1, 64, 0, 0, out, cyc, n, 1e-7f);
  unsigned long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("active lanes %2d, %d chains: %.2f cycles per add step (s_memtime)\n", ACTIVE, CH, (double)c / (n * 16.0));
}

int main() {
  float *out;
  unsigned long long *cyc;
  (void)hipMalloc(&out, 256);
  (void)hipMalloc(&cyc, 8);
  run<64, 1>(out, cyc);
  run<32, 1>(out, cyc);
  run<16, 1>(out, cyc);
  run<1, 1>(out, cyc);
  run<64, 2>(out, cyc);
  run<32, 2>(out, cyc);
  run<64, 4>(out, cyc);
  // wall clock reference for the s_memtime rate
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k_lat<64, 1>), 1, 64, 0, 0, out, cyc, 65536, 1e-7f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long c;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("65536x16 adds: %.3f ms wall, %llu memtime ticks -> %.3f GHz tick rate, %.2f ns per add\n", ms, c,
         c / (ms * 1e6), ms * 1e6 / (65536.0 * 16));
  return 0;
}
