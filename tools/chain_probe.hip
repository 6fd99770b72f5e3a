// tools/chain_probe.hip — measures the dependent fp32 add chain on gfx950 (one wave),
// from registers and fed from LDS, in shader cycles (s_memtime) and ns.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_reg(float *out, long long *cyc, int n, float a) {
  float s = threadIdx.x;
  float v0 = a, v1 = a * 1.5f, v2 = a * 0.25f, v3 = a * 3.0f;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    s = s + v0; s = s + v1; s = s + v2; s = s + v3;
    v0 = v0 * 1.0000001f;  // independent of s
  }
  long long t1 = clock64();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_lds(float *out, long long *cyc, int n) {
  __shared__ float4 P[64 * 65];
  for (int i = threadIdx.x; i < 64 * 65; i += blockDim.x) P[i] = make_float4(i * 1e-3f, 1.f, 2.f, 3.f);
  __syncthreads();
  float s = 0.f;
  long long t0 = clock64();
  for (int it = 0; it < n; it += 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float4 v = P[threadIdx.x * 65 + ((it + j) & 63)];
      s = s + v.x; s = s + v.y; s = s + v.z; s = s + v.w;
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  float *out; long long *cyc;
  hipMalloc(&out, 1024 * 4); hipMalloc(&cyc, 16);
  const int n = 1 << 14;
  for (int rep = 0; rep < 2; ++rep) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_reg, 1, 64, 0, 0, out, cyc, n, 0.5f);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("reg chain: %d adds, %lld clk64 ticks (%.2f / add), %.2f ns/add wall\n", 4 * n, c, (double)c / (4.0 * n), ms * 1e6 / (4.0 * n));
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_lds, 1, 64, 0, 0, out, cyc, n);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("lds chain: %d adds, %lld clk64 ticks (%.2f / add), %.2f ns/add wall\n", 4 * n, c, (double)c / (4.0 * n), ms * 1e6 / (4.0 * n));
  }
  return 0;
}
