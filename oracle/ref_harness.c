/* oracle/ref_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * Per-op golden-vector driver: our own code, linked against the REFERENCE's ggml.o,
 * imax.o and monitor.o (compiled in place from /root/reference by oracle/Makefile).
 * Each command builds the exact ggml graph shape the reference's gptneox_eval builds
 * for that op (vsim.cpp:470-747), runs ggml_graph_compute with n_threads = 1, and writes
 * the raw output.  tests/golden/make_golden.py drives it; the fixtures it writes are
 * data only (inputs + reference outputs).
 *
 * usage: ref_harness <op> <int params...> <input files...> <output file>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ggml.h"

static void *slurp(const char *path, size_t want) {
  FILE *f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "harness: cannot open %s\n", path); exit(2); }
  void *p = malloc(want ? want : 1);
  size_t got = fread(p, 1, want, f);
  fclose(f);
  if (got != want) { fprintf(stderr, "harness: %s has %zu bytes, want %zu\n", path, got, want); exit(2); }
  return p;
}

static void spit(const char *path, const void *p, size_t n) {
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(p, 1, n, f) != n) { fprintf(stderr, "harness: cannot write %s\n", path); exit(2); }
  fclose(f);
}

static struct ggml_context *mk_ctx(size_t mb) {
  struct ggml_init_params ip = { .mem_size = mb * 1024 * 1024, .mem_buffer = NULL };
  return ggml_init(ip);
}

static void run(struct ggml_context *ctx, struct ggml_tensor *out) {
  struct ggml_cgraph gf = ggml_build_forward(out);
  gf.n_threads = 1;
  ggml_graph_compute(ctx, &gf);
}

#define ARG(i) atoi(argv[i])

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const char *op = argv[1];
  struct ggml_context *ctx = mk_ctx(512);

  if (!strcmp(op, "qrow")) {               /* qrow K in.f32 out.q4          ggml.c:209-251 */
    int K = ARG(2);
    float *x = slurp(argv[3], (size_t)K * 4);
    void *y = malloc((size_t)K / 32 * 20);
    quantize_row_q4_0(x, y, K);
    spit(argv[4], y, (size_t)K / 32 * 20);
  } else if (!strcmp(op, "mulmat")) {      /* mulmat M K N w.q4 x.f32 out   ggml.c:4891-5165 */
    int M = ARG(2), K = ARG(3), N = ARG(4);
    struct ggml_tensor *w = ggml_new_tensor_2d(ctx, GGML_TYPE_Q4_0, K, M);
    struct ggml_tensor *x = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, N);
    void *wd = slurp(argv[5], ggml_nbytes(w)); memcpy(w->data, wd, ggml_nbytes(w));
    void *xd = slurp(argv[6], ggml_nbytes(x)); memcpy(x->data, xd, ggml_nbytes(x));
    struct ggml_tensor *y = ggml_mul_mat(ctx, w, x);
    run(ctx, y);
    spit(argv[7], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "norm")) {        /* norm n rows in out            ggml.c:4246-4304 */
    int n = ARG(2), r = ARG(3);
    struct ggml_tensor *x = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, n, r);
    void *xd = slurp(argv[4], ggml_nbytes(x)); memcpy(x->data, xd, ggml_nbytes(x));
    struct ggml_tensor *y = ggml_norm(ctx, x);
    run(ctx, y);
    spit(argv[5], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "gelu")) {        /* gelu n in out                 ggml.c:4113-4152 */
    int n = ARG(2);
    struct ggml_tensor *x = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, n);
    void *xd = slurp(argv[3], ggml_nbytes(x)); memcpy(x->data, xd, ggml_nbytes(x));
    struct ggml_tensor *y = ggml_gelu(ctx, x);
    run(ctx, y);
    spit(argv[4], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "attnsm")) {      /* attnsm nc nr nz n_past scale in out: scale -> mask -> softmax (vsim.cpp:586-596) */
    int nc = ARG(2), nr = ARG(3), nz = ARG(4), n_past = ARG(5);
    float sc = (float)atof(argv[6]);
    struct ggml_tensor *x = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, nc, nr, nz);
    void *xd = slurp(argv[7], ggml_nbytes(x)); memcpy(x->data, xd, ggml_nbytes(x));
    struct ggml_tensor *y = ggml_soft_max(ctx, ggml_diag_mask_inf(ctx, ggml_scale(ctx, x, ggml_new_f32(ctx, sc)), n_past));
    run(ctx, y);
    spit(argv[8], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "attnsm_alibi")) {
    /* attnsm_alibi nc nr nz n_past n_head scale in out: scale -> alibi -> mask -> softmax
       (the BLOOM attention scores; ggml_alibi ggml.c:2949, 6184-6244) */
    int nc = ARG(2), nr = ARG(3), nz = ARG(4), n_past = ARG(5), n_head = ARG(6);
    float sc = (float)atof(argv[7]);
    struct ggml_tensor *x = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, nc, nr, nz);
    void *xd = slurp(argv[8], ggml_nbytes(x)); memcpy(x->data, xd, ggml_nbytes(x));
    struct ggml_tensor *y = ggml_soft_max(ctx, ggml_diag_mask_inf(ctx,
        ggml_alibi(ctx, ggml_scale(ctx, x, ggml_new_f32(ctx, sc)), n_past, n_head), n_past));
    run(ctx, y);
    spit(argv[9], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "rope_neox") || !strcmp(op, "rope_gptj")) {
    /* rope_* d H T n_past n_dims mode in out        ggml.c:6086-6153 / 5919-5974 */
    int d = ARG(2), H = ARG(3), T = ARG(4), n_past = ARG(5), n_dims = ARG(6), mode = ARG(7);
    struct ggml_tensor *x = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, d, H, T);
    void *xd = slurp(argv[8], ggml_nbytes(x)); memcpy(x->data, xd, ggml_nbytes(x));
    struct ggml_tensor *y = !strcmp(op, "rope_neox") ? ggml_gptneox_rope(ctx, x, n_past, n_dims, mode)
                                                     : ggml_rope(ctx, x, n_past, n_dims, mode);
    run(ctx, y);
    spit(argv[9], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "kq")) {          /* kq d H nk N K.f32 Q.f32 out   vsim.cpp:573-583 */
    int d = ARG(2), H = ARG(3), nk = ARG(4), N = ARG(5);
    struct ggml_tensor *km = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, d * H * nk);
    struct ggml_tensor *qm = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, d, H, N);
    void *kd = slurp(argv[6], ggml_nbytes(km)); memcpy(km->data, kd, ggml_nbytes(km));
    void *qd = slurp(argv[7], ggml_nbytes(qm)); memcpy(qm->data, qd, ggml_nbytes(qm));
    struct ggml_tensor *K = ggml_permute(ctx, ggml_reshape_3d(ctx, km, d, H, nk), 0, 2, 1, 3);
    struct ggml_tensor *Q = ggml_permute(ctx, qm, 0, 2, 1, 3);
    struct ggml_tensor *y = ggml_mul_mat(ctx, K, Q);
    run(ctx, y);
    spit(argv[8], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "kqv")) {         /* kqv d H nk N V.f32 S.f32 out  vsim.cpp:599-607 */
    int d = ARG(2), H = ARG(3), nk = ARG(4), N = ARG(5);
    struct ggml_tensor *vm = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, d * H * nk);
    struct ggml_tensor *s = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, nk, N, H);
    void *vd = slurp(argv[6], ggml_nbytes(vm)); memcpy(vm->data, vd, ggml_nbytes(vm));
    void *sd = slurp(argv[7], ggml_nbytes(s)); memcpy(s->data, sd, ggml_nbytes(s));
    struct ggml_tensor *Vt = ggml_permute(ctx, ggml_reshape_3d(ctx, vm, d, H, nk), 1, 2, 0, 3);
    struct ggml_tensor *y = ggml_mul_mat(ctx, Vt, s);
    run(ctx, y);
    spit(argv[8], y->data, ggml_nbytes(y));
  } else if (!strcmp(op, "getrows")) {     /* getrows K V n w.q4 idx.i32 out  ggml.c:5603-5628 */
    int K = ARG(2), V = ARG(3), n = ARG(4);
    struct ggml_tensor *w = ggml_new_tensor_2d(ctx, GGML_TYPE_Q4_0, K, V);
    struct ggml_tensor *ix = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, n);
    void *wd = slurp(argv[5], ggml_nbytes(w)); memcpy(w->data, wd, ggml_nbytes(w));
    void *id = slurp(argv[6], ggml_nbytes(ix)); memcpy(ix->data, id, ggml_nbytes(ix));
    struct ggml_tensor *y = ggml_get_rows(ctx, w, ix);
    run(ctx, y);
    spit(argv[7], y->data, ggml_nbytes(y));
  } else {
    fprintf(stderr, "harness: unknown op %s\n", op);
    return 2;
  }
  ggml_free(ctx);
  return 0;
}
