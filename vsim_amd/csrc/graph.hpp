// vsim_amd/csrc/graph.hpp — strided F32 kernels of the ggml graph executor (graph.hip).
#pragma once

#include "common.hpp"

namespace vsim {

// one operand: device base, shape, byte strides (ggml_tensor ne / nb)
struct GT {
  const char *p;
  int ne[4];
  long long nb[4];
};

int launch_g_dup(float *dst, const GT &s, long long n, hipStream_t st);
int launch_g_binop(int op, char *d, long long dnb1, const char *a, long long anb1, const char *b, long long bnb0,
                   long long bnb1, int nc, long long nr, hipStream_t st);
int launch_g_repeat(char *d, long long dnb1, const char *s, long long snb1, int nc, int nr, int nc0, int nr0,
                    hipStream_t st);
int launch_g_scale(char *x, long long nb1, int nc, long long nr, float v, hipStream_t st);
int launch_g_diag_mask(char *x, long long nb0, long long nb1, long long nb2, int nc, int nr, int nz, int n_past,
                       hipStream_t st);
int launch_g_mm_dot(const GT &d, const GT &a, const GT &b, int K, hipStream_t st);
int launch_g_mm_mad(float *dst, const GT &a, const GT &b, int nc, int nth, int ne0, int ne1, int ne2, int ne3,
                    hipStream_t st);

}  // namespace vsim
