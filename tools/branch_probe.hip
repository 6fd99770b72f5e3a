// tools/branch_probe.hip -- do two independent branches of a captured hipGraph run at the same
// time on MI355X?  Two kernels that each spin ~T us on 128 single-wave workgroups: one
// stream back to back, two streams (fork/join by events) eagerly, and the same fork/join
// captured into a graph and replayed.  Concurrent branches take ~T, serialized ones ~2T.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/branch_probe tools/branch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void spin(long ticks, unsigned *out) {
  const long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}

int main() {
  const long ticks = 100 * 40;  // 40 us
  unsigned *buf;
  CK(hipMalloc(&buf, 4096 * sizeof(unsigned)));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join, e0, e1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto pair_serial = [&]() {
    hipLaunchKernelGGL(spin, dim3(128), dim3(64), 0, s0, ticks, buf);
    hipLaunchKernelGGL(spin, dim3(128), dim3(64), 0, s0, ticks, buf + 1024);
  };
  auto pair_fork = [&]() {
    hipEventRecord(fork, s0);
    hipStreamWaitEvent(s1, fork, 0);
    hipLaunchKernelGGL(spin, dim3(128), dim3(64), 0, s0, ticks, buf);
    hipLaunchKernelGGL(spin, dim3(128), dim3(64), 0, s1, ticks, buf + 1024);
    hipEventRecord(join, s1);
    hipStreamWaitEvent(s0, join, 0);
  };
  const int reps = 20;
  auto timeit = [&](const char *name, auto f) -> int {
    f();
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(e0, s0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1, s0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.1f us per pair (one kernel spins 40 us)\n", name, 1e3f * ms / reps);
    return 0;
  };
  if (timeit("one stream, back to back", pair_serial)) return 1;
  if (timeit("two streams, fork/join", pair_fork)) return 1;
  // the fork/join captured into a graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 4; ++i) pair_fork();
  CK(hipStreamEndCapture(s0, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  printf("graph nodes: %zu (4 fork/join pairs)\n", nn);
  auto graph_run = [&]() { hipGraphLaunch(ge, s0); };
  graph_run();
  CK(hipStreamSynchronize(s0));
  CK(hipEventRecord(e0, s0));
  for (int i = 0; i < reps; ++i) graph_run();
  CK(hipEventRecord(e1, s0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s %8.1f us per pair\n", "graph of fork/join pairs", 1e3f * ms / reps / 4);
  // the same pairs captured from one stream (serial chain) for the graph baseline
  hipGraph_t g2;
  hipGraphExec_t ge2;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 4; ++i) pair_serial();
  CK(hipStreamEndCapture(s0, &g2));
  CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
  hipGraphLaunch(ge2, s0);
  CK(hipStreamSynchronize(s0));
  CK(hipEventRecord(e0, s0));
  for (int i = 0; i < reps; ++i) hipGraphLaunch(ge2, s0);
  CK(hipEventRecord(e1, s0));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s %8.1f us per pair\n", "graph of serial pairs", 1e3f * ms / reps / 4);
  return 0;
}
