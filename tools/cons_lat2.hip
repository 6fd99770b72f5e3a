// tools/cons_lat2.hip — what sets the exact-decode consumer's cycles per add: one wave per CU
// (every CU busy), a dependent v_add_f32 chain per lane over pair terms in LDS, variants:
//   b128      : rolling window of WIN ds_read_b128, 4 adds per read (gemv_chain.hip's loop)
//   b128-32   : the same with lanes 32-63 masked off (chain32's consumer has 32 rows)
//   b64       : ds_read_b64, 2 adds per read
//   batch8    : 8 ds_read_b128 issued back to back, then their 32 adds (one wait per 32 adds)
//   noread    : the adds alone on register-resident terms (the chain's own floor)
//   2chain    : two independent chains per lane interleaved, reads as b128 (two rows per lane)
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int CP = 128, LD = CP + 4;

template <int V>
__global__ void __launch_bounds__(64) k_cons(float *out, unsigned long long *cyc, int nrep) {
  __shared__ __attribute__((aligned(16))) float P[2][64 * LD];
  const int lane = threadIdx.x;
  for (int i = lane; i < 2 * 64 * LD; i += 64) (&P[0][0])[i] = (i & 15) * 1e-3f;
  __syncthreads();
  float acc = 0.f, acc2 = 0.f;
  const float *pc = &P[0][lane * LD];
  const float *pd = &P[1][lane * LD];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (V == 1 && lane >= 32) {
  } else {
    for (int r = 0; r < nrep; ++r) {
      if constexpr (V == 0 || V == 1) {
        float4 win[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) win[j] = *(const float4 *)(pc + 4 * j);
#pragma unroll
        for (int j = 0; j < CP / 4; ++j) {
          const float4 v = win[j % 8];
          acc = acc + v.x;
          acc = acc + v.y;
          acc = acc + v.z;
          acc = acc + v.w;
          const int jn = (j + 8) % (CP / 4);
          win[j % 8] = *(const float4 *)(pc + 4 * jn);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      } else if constexpr (V == 2) {
        float2 win[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) win[j] = *(const float2 *)(pc + 2 * j);
#pragma unroll
        for (int j = 0; j < CP / 2; ++j) {
          const float2 v = win[j % 16];
          acc = acc + v.x;
          acc = acc + v.y;
          win[j % 16] = *(const float2 *)(pc + 2 * ((j + 16) % (CP / 2)));
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      } else if constexpr (V == 3) {
#pragma unroll
        for (int g = 0; g < CP / 32; ++g) {
          float4 w[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) w[j] = *(const float4 *)(pc + 32 * g + 4 * j);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            acc = acc + w[j].x;
            acc = acc + w[j].y;
            acc = acc + w[j].z;
            acc = acc + w[j].w;
          }
        }
      } else if constexpr (V == 4) {
        const float4 w = *(const float4 *)pc;
#pragma unroll
        for (int j = 0; j < CP / 4; ++j) {
          acc = acc + w.x;
          acc = acc + w.y;
          acc = acc + w.z;
          acc = acc + w.w;
        }
      } else if constexpr (V == 5) {
        float4 win[8], wim[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          win[j] = *(const float4 *)(pc + 4 * j);
          wim[j] = *(const float4 *)(pd + 4 * j);
        }
#pragma unroll
        for (int j = 0; j < CP / 4; ++j) {
          const float4 v = win[j % 8], u = wim[j % 8];
          acc = acc + v.x;
          acc2 = acc2 + u.x;
          acc = acc + v.y;
          acc2 = acc2 + u.y;
          acc = acc + v.z;
          acc2 = acc2 + u.z;
          acc = acc + v.w;
          acc2 = acc2 + u.w;
          const int jn = (j + 8) % (CP / 4);
          win[j % 8] = *(const float4 *)(pc + 4 * jn);
          wim[j % 8] = *(const float4 *)(pd + 4 * jn);
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = acc + acc2;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

static const char *kName[] = {"b128 (window 8)", "b128, lanes 0-31", "b64 (window 16)", "batch8 b128",
                              "noread", "2 chains/lane, b128"};

template <int V>
void run(float *out, unsigned long long *cyc, unsigned long long *h, int grid) {
  const int nrep = 64;
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_cons<V>), grid, 64, 0, 0, out, cyc, nrep);
  (void)hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; ++i) s += h[i];
  printf("%-22s %5.2f cycles per add step of one chain\n", kName[V], s / grid / (nrep * (double)CP));
}

int main() {
  const int grid = 256;
  float *out;
  unsigned long long *cyc, h[256];
  (void)hipMalloc(&out, grid * 256);
  (void)hipMalloc(&cyc, grid * 8);
  run<0>(out, cyc, h, grid);
  run<1>(out, cyc, h, grid);
  run<2>(out, cyc, h, grid);
  run<3>(out, cyc, h, grid);
  run<4>(out, cyc, h, grid);
  run<5>(out, cyc, h, grid);
  return 0;
}
