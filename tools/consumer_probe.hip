// tools/consumer_probe.hip — what a chain-consumer wave costs per add on gfx950.
// One workgroup per CU (many CUs busy), wave 0 runs NCH lanes-wide dependent add chains
// over LDS-resident pairs in chunks of CP; the other waves only join the barrier.
// Variants: SYNC 0 = no barrier, 1 = __syncthreads per chunk; CH = chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CP, int SYNC, int CH>
__global__ void __launch_bounds__(512) k_cons(float *out, long long *cyc, int nchunks) {
  constexpr int LD = CP + 4;
  __shared__ __attribute__((aligned(16))) float P[2][CH][32 * LD];
  for (int i = threadIdx.x; i < 2 * CH * 32 * LD; i += blockDim.x) (&P[0][0][0])[i] = (i & 7) * 1e-3f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float s[CH];
#pragma unroll
  for (int h = 0; h < CH; ++h) s[h] = 0.f;
  long long t0 = clock64();
  for (int c = 0; c < nchunks; ++c) {
    if (wave == 0 && lane < 32) {
      float4 v[CH][CP / 4];
#pragma unroll
      for (int j = 0; j < CP / 4; ++j)
#pragma unroll
        for (int h = 0; h < CH; ++h) v[h][j] = *(const float4 *)(&P[c & 1][h][lane * LD + 4 * j]);
#pragma unroll
      for (int j = 0; j < CP / 4; ++j) {
#pragma unroll
        for (int h = 0; h < CH; ++h) s[h] = s[h] + v[h][j].x;
#pragma unroll
        for (int h = 0; h < CH; ++h) s[h] = s[h] + v[h][j].y;
#pragma unroll
        for (int h = 0; h < CH; ++h) s[h] = s[h] + v[h][j].z;
#pragma unroll
        for (int h = 0; h < CH; ++h) s[h] = s[h] + v[h][j].w;
      }
    }
    if (SYNC) __syncthreads();
  }
  long long t1 = clock64();
  float r = 0.f;
#pragma unroll
  for (int h = 0; h < CH; ++h) r += s[h];
  if (threadIdx.x < 32) out[blockIdx.x * 32 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CP, int SYNC, int CH>
void run(float *out, long long *cyc) {
  const int adds = 8192, nch = adds / CP, grid = 128;
  hipLaunchKernelGGL((k_cons<CP, SYNC, CH>), grid, 512, 0, 0, out, cyc, nch);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_cons<CP, SYNC, CH>), grid, 512, 0, 0, out, cyc, nch);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("CP=%3d sync=%d chains=%d: %.2f clk/add, kernel %.2f us (floor at 3.37 ns/add: %.2f us)\n", CP, SYNC, CH,
         (double)c / adds, ms * 1e3, adds * 3.37e-3);
}

int main() {
  float *out;
  long long *cyc;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMalloc(&cyc, 4096);
  run<64, 0, 1>(out, cyc);
  run<64, 1, 1>(out, cyc);
  run<128, 0, 1>(out, cyc);
  run<128, 1, 1>(out, cyc);
  run<256, 1, 1>(out, cyc);
  run<64, 1, 2>(out, cyc);
  run<128, 1, 2>(out, cyc);
  run<64, 1, 4>(out, cyc);
  return 0;
}
