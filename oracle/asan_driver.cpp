// oracle/asan_driver.cpp — TEST INFRASTRUCTURE ONLY (tests/test_sanitizers.py).
// Runs the CPU restatement (vsim_oracle.cpp, compiled into this binary) under
// -fsanitize=address,undefined: a model file is loaded, a prompt batch, decode steps at 1 and
// 3 threads, the sampler loop, and every op entry point on small shapes.  Any out-of-bounds
// access, leak, or undefined behaviour aborts with the sanitizer's report.
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include "vsim_oracle.h"

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: asan_driver MODEL ARCH\n");
    return 2;
  }
  const int arch = atoi(argv[2]);
  vo_init_tables();
  void *m = vo_model_load(argv[1], arch, 64);
  if (!m) {
    fprintf(stderr, "load failed\n");
    return 1;
  }
  int32_t hp[8];
  vo_model_hparams(m, hp);
  const int V = hp[0];
  std::vector<float> logits(V);
  const int32_t prompt[5] = {1, 2, 3, 4, 5 % V};
  if (vo_model_eval(m, 0, prompt, 5, logits.data(), 1)) return 1;
  int n_past = 5;
  for (int t = 0; t < 6; ++t) {
    int best = 0;
    for (int i = 1; i < V; ++i)
      if (logits[i] > logits[best]) best = i;
    const int32_t tok = best;
    if (vo_model_eval(m, n_past++, &tok, 1, logits.data(), t % 2 ? 3 : 1)) return 1;
  }
  vo_model_free(m);
  m = vo_model_load(argv[1], arch, 64);
  std::vector<int32_t> out(64);
  const int n = vo_generate(m, prompt, 5, 12, 42, 20, 0.95f, 0.85f, 64, 1.3f, 8, out.data(), (int)out.size(), 2);
  vo_model_free(m);
  if (n <= 5) return 1;
  // op entry points on odd shapes
  const int K = 96, M = 37, N = 3;
  std::vector<float> x(K * N), y(M * N);
  for (int i = 0; i < K * N; ++i) x[i] = std::sin(0.37f * i);
  std::vector<uint8_t> w(M * K / 32 * 20), xq(N * K / 32 * 20);
  std::vector<float> wf(M * K);
  for (int i = 0; i < M * K; ++i) wf[i] = std::cos(0.11f * i);
  for (int r = 0; r < M; ++r) vo_quantize_row_q4_0(wf.data() + r * K, w.data() + r * (K / 32 * 20), K);
  vo_mul_mat_q4_0_f32(w.data(), M, K, x.data(), N, y.data(), 3);
  for (int r = 0; r < N; ++r) vo_quantize_row_q4_0(x.data() + r * K, xq.data() + r * (K / 32 * 20), K);
  vo_mul_mat_q4_0_q(w.data(), M, K, xq.data(), N, y.data(), 2);
  std::vector<float> z(K * N);
  vo_norm_f32(x.data(), z.data(), K, N);
  vo_gelu_f32(x.data(), z.data(), K * N);
  std::vector<float> p(12 * 5 * 2);
  for (size_t i = 0; i < p.size(); ++i) p[i] = 0.01f * i;
  vo_scale_f32(p.data(), (int)p.size(), 0.5f);
  vo_diag_mask_inf_f32(p.data(), 12, 5, 2, 7);
  vo_alibi_f32(p.data(), 12, 5, 2, 2);
  vo_soft_max_f32(p.data(), 12, 10);
  const int d = 8, H = 3, T = 4;
  std::vector<float> q(d * H * T);
  for (size_t i = 0; i < q.size(); ++i) q[i] = 0.1f * i;
  vo_rope_neox(q.data(), d, H, T, 2, 4, 0);
  vo_rope_gptj(q.data(), d, H, T, 2, 4, 1);
  std::vector<float> kq(H * T * T), kqv(H * T * d);
  vo_kq(q.data(), d * H, q.data(), d * H, d, H, T, T, kq.data());
  vo_kqv(q.data(), d * H, kq.data(), d, H, T, T, kqv.data());
  const int32_t rows[3] = {0, 5, 36};
  std::vector<float> g(3 * K);
  vo_get_rows_q4_0(w.data(), K, rows, 3, g.data());
  printf("asan_driver: ok (%d ids)\n", n);
  return 0;
}
