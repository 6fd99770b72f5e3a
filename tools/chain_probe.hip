// tools/chain_probe.hip — dependent fp32 add-chain latency on gfx950 (one wave per CU),
// by active-lane count and instruction form.  Prints shader cycles (clock64) per add.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k_chain(float *out, long long *cyc, int n, int active) {
  __shared__ float4 P[64 * 65];
  for (int i = threadIdx.x; i < 64 * 65; i += blockDim.x) P[i] = make_float4(i * 1e-3f, 1.f, 2.f, 3.f);
  __syncthreads();
  float s = 0.f;
  long long t0 = clock64();
  if ((int)threadIdx.x < active) {
    for (int it = 0; it < n; it += 16) {
      float4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = P[threadIdx.x * 65 + ((it + j) & 63)];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (MODE == 0) { s = s + v[j].x; s = s + v[j].y; s = s + v[j].z; s = s + v[j].w; }
        if (MODE == 1) {
          s = __builtin_fmaf(v[j].x, 1.0f, s); s = __builtin_fmaf(v[j].y, 1.0f, s);
          s = __builtin_fmaf(v[j].z, 1.0f, s); s = __builtin_fmaf(v[j].w, 1.0f, s);
        }
      }
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int MODE>
void run(const char *name, int active, float *out, long long *cyc) {
  const int n = 1 << 14;
  hipLaunchKernelGGL(k_chain<MODE>, 1, 64, 0, 0, out, cyc, n, active);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_chain<MODE>, 1, 64, 0, 0, out, cyc, n, active);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-10s lanes=%2d: %.2f clk/add, %.2f ns/add wall\n", name, active, (double)c / (4.0 * n), ms * 1e6 / (4.0 * n));
}

int main() {
  float *out; long long *cyc;
  (void)hipMalloc(&out, 1024 * 4); (void)hipMalloc(&cyc, 16);
  for (int a : {64, 32, 16, 1}) { run<0>("v_add", a, out, cyc); run<1>("v_fma(,1,)", a, out, cyc); }
  return 0;
}
