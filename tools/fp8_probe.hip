#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned *in, float *out) {
  unsigned w = in[threadIdx.x];
  f32x2 a, b;
  a = __builtin_amdgcn_cvt_pk_f32_fp8(w, false);
  b = __builtin_amdgcn_cvt_pk_f32_fp8(w, true);
  out[4 * threadIdx.x] = a.x; out[4 * threadIdx.x + 1] = a.y; out[4 * threadIdx.x + 2] = b.x; out[4 * threadIdx.x + 3] = b.y;
}
int main() {
  unsigned h[16]; for (int i = 0; i < 16; ++i) h[i] = i | ((15 - i) << 8) | (i << 16) | (7 << 24);
  unsigned *din; float *dout; hipMalloc(&din, 64); hipMalloc(&dout, 256);
  hipMemcpy(din, h, 64, hipMemcpyHostToDevice);
  k<<<1, 16>>>(din, dout);
  float o[64]; hipMemcpy(o, dout, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i) {
    float e[4] = {i / 512.0f, (15 - i) / 512.0f, i / 512.0f, 7 / 512.0f};
    for (int j = 0; j < 4; ++j) if (o[4 * i + j] != e[j]) { bad++; printf("i=%d j=%d got %g want %g\n", i, j, o[4*i+j], e[j]); }
  }
  printf("fp8 nibble decode: %s\n", bad ? "MISMATCH" : "n * 2^-9 exact");
  return bad != 0;
}
