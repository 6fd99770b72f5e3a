/* oracle/vsim_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Q4_0 decode path (NAIST-Archlab/vsim ggml.c /
 * imax.c / vsim.cpp), used as the parity checker by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg.  Never linked into libvsim_hip.so.
 *
 * Numerics follow the reference x86 build (Makefile-ubuntu:5-6: -O2 -msse3, no FMA,
 * scalar paths, ggml_float == double).  Pinned against the reference binary built from
 * /root/reference (oracle/Makefile `ref`) by tests/test_oracle_golden.py.
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* VO_ARCH_BLOOM: the BLOOM graph no reference program composes (SURVEY.md finding 2), built
 * from reference ops incl. ggml_alibi (ggml.c:6184-6244); file format of
 * converters/convert_bloom_to_ggml.py + quantize_bloom.cpp */
enum { VO_ARCH_GPTNEOX = 0, VO_ARCH_GPTJ = 1, VO_ARCH_BLOOM = 2 };

void     vo_init_tables(void);
float    vo_fp16_to_fp32(uint16_t h);
uint16_t vo_fp32_to_fp16(float f);
void     vo_tables(uint16_t *exp_f16, uint16_t *gelu_f16);   /* 65536 entries each */

void vo_quantize_row_q4_0(const float *x, void *y, int k);
void vo_dequantize_row_q4_0(const void *x, float *y, int k);
void vo_vec_dot_q4_0(int n, float *s, const void *x, const void *y);
/* y[N][M] = W[M][K] (Q4_0 rows) . x[N][K] (F32, quantized to Q4_0 first) */
void vo_mul_mat_q4_0_f32(const void *W, int M, int K, const float *x, int N, float *y, int nthreads);
/* same with already-quantized activations xq[N][K/32*20] */
void vo_mul_mat_q4_0_q(const void *W, int M, int K, const void *xq, int N, float *y, int nthreads);

void vo_norm_f32(const float *x, float *y, int n, int rows);
void vo_gelu_f32(const float *x, float *y, int n);
void vo_soft_max_f32(float *p, int nc, int nr);
void vo_scale_f32(float *p, int n, float v);
void vo_diag_mask_inf_f32(float *p, int nc, int nr, int nz, int n_past);
/* ggml_alibi (ggml.c:6184-6244) on p[nz][nr][nc]: p += (row j + 1) * m_head, the head slopes
 * of the reference (which depend on the query row j, not on the key column) */
void vo_alibi_f32(float *p, int nc, int nr, int nz, int n_head);
/* x: [T][H][d] float rows (ne0=d, ne1=H, ne2=T).  mode 0: p = n_past+i2 for all i2;
 * mode 1: only i2 >= n_past, p = i2. */
void vo_rope_neox(float *x, int d, int H, int T, int n_past, int n_dims, int mode);
void vo_rope_gptj(float *x, int d, int H, int T, int n_past, int n_dims, int mode);
/* KQ[h][q][k] = sum_dd K[k*ldk + h*d + dd] * Q[q*ldq + h*d + dd]   (double accumulator) */
void vo_kq(const float *K, int ldk, const float *Q, int ldq, int d, int H, int nk, int N, float *KQ);
/* out[h][q][dd] = sum_k V[k*ldv + h*d + dd] * S[h][q][k]           (float, sequential k) */
void vo_kqv(const float *V, int ldv, const float *S, int d, int H, int nk, int N, float *out);
void vo_get_rows_q4_0(const void *W, int K, const int32_t *rows, int n, float *y);

/* whole model (ggml file formats of vsim.cpp:108-458 and convert_gptj_to_ggml.py) */
void *vo_model_load(const char *path, int arch, int n_ctx);
void *vo_model_synthetic(int arch, int n_vocab, int n_embd, int n_head, int n_layer, int n_rot, int n_ctx,
                         uint64_t seed, float stddev);
/* an empty model of this shape; tensors then set by their ggml-file names (Q4_0 as AoS
 * blocks, F32 as floats); set_tensor returns -1 for an unknown name or a wrong size */
void *vo_model_create(int arch, int n_vocab, int n_embd, int n_head, int n_layer, int n_rot, int par_res, int n_ctx);
int   vo_model_set_tensor(void *m, const char *name, const void *data, size_t nbytes);
void  vo_model_hparams(void *m, int32_t *out8); /* n_vocab n_embd n_head n_layer n_rot par_res ftype n_ctx */
int   vo_model_eval(void *m, int n_past, const int32_t *tokens, int N, float *logits, int nthreads);
/* run only layers [l0,l1) + optional head on a prepared residual (cpu_baseline sampling) */
void  vo_model_free(void *m);

/* utils.cpp:339-422 sampler (std::mt19937 + std::discrete_distribution) and the
 * main_gptneox decode loop (vsim.cpp:749-910).  Returns number of ids written to out. */
int vo_generate(void *m, const int32_t *prompt, int n_prompt, int n_predict, int seed,
                int top_k, float top_p, float temp, int repeat_last_n, float repeat_penalty,
                int n_batch, int32_t *out, int out_cap, int nthreads);

#ifdef __cplusplus
}
#endif
