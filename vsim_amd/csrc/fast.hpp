// vsim_amd/csrc/fast.hpp — parameter blocks and launchers of the fast-mode decode step
// (fast_decode.hip), shared with the model executor (model.cpp).
#pragma once

#include "common.hpp"

namespace vsim {

// ------------------------------------------------------------------ parameters
constexpr int FD_WAVES = 8;          // waves per K1 / K2 GEMV workgroup
constexpr int FD_OWAVES = 16;        // waves per K3 workgroup (only E/32 tiles)
constexpr int FD_U = 4;              // 16-byte weight loads in flight per lane and batch
constexpr int FD_MAXE = 8192;        // largest n_embd / activation length handled
constexpr int FD_CHUNK = 64;         // attention positions per chunk workgroup
constexpr int FD_SF = 2;
constexpr size_t FD_PAD = 64 << 10;  // readable slack after the weight arena (TileStream)             // fc_out K splits (partial rows summed by K3)
// GEMV epilogues: store (+bias); fc_in bias + GELU + quantize; Q with RoPE; K with RoPE
// into the KV cache at n_past; V into the cache at n_past
enum { FE_STORE = 0, FE_GELU_Q = 1, FE_ROPE_Q = 2, FE_ROPE_K = 3, FE_V = 4 };

struct FastJob {
  W4 w;
  const float *bias;  // FE_STORE / FE_GELU_Q (may be null for FE_STORE)
  float *y;           // FE_STORE / FE_ROPE_Q: output rows; FE_ROPE_K / FE_V: the layer's
                      // cache [n_ctx][E] (row n_past is written)
  int epi;
  int act;            // which activation row (FastGemv::xq/xd) feeds this job (0 or 1)
};

// LayerNorm(s) of the joined residual row, quantized into Q4 SoA activation rows
struct FastLn {
  const float *x;                   // residual row [E]
  const float *w[2], *b[2];         // affine of each LayerNorm
  uint8_t *qs[2];                   // output activation i: nibble plane [E/32][16] ...
  float *d[2];                      // ... and scales [E/32]
  int n, E;                         // n = 1 or 2 LayerNorms
};

// K1: a batch of GEMVs over the same-K activations (Q4 SoA, chosen per job by `act`)
struct FastGemv {
  const uint8_t *xq[2];
  const float *xd[2];
  FastJob j[4];
  int nj;
  const uint16_t *gelu_tab;         // FE_GELU_Q: table_gelu_f16 (ggml.c:1247)
  uint8_t *oq_qs;                   // FE_GELU_Q: output activation, Q4 SoA
  float *oq_d;
  // RoPE epilogues (ggml.c:6086-6153 style 0 / 5919-5974 style 1): pairs within a tile
  const int *npast;
  const double2 *cs;                // [n_ctx][n_rot/2]
  int d, n_rot, style;
  // LayerNorm in the prologue (lnx non-null): every workgroup normalizes the residual row
  // lnx with the affine of its job's `act` and quantizes it into LDS, while its first weight
  // batch is in flight; xq/xd are then unused
  const float *lnx;
  const float *lnw[2], *lnb[2];
  unsigned *clear;                  // non-null: workgroup 0 zeroes clear[0 .. nclear)
  int nclear;                       // (the per-head chunk counters of this layer's K2)
};

struct FastTail {
  // fc_out split over K: tile t, split s -> partial rows ffp[s][32t .. 32t+31]
  W4 wf;
  const uint8_t *xf_qs;  // fc_out activation (K1's GELU output), Q4 SoA
  const float *xf_d;
  float *ffp;
  int sf;
  // attention chunks (q after RoPE; the new K/V row is already in the cache)
  const float *q;          // [E]
  const float *kc, *vc;    // this layer's cache [n_ctx][E]
  const int *npast;
  int d, H, nchunk;
  float scale;
  float *part;             // [H][nchunk][d + 2]: m, l, o[d]
  // the chunk workgroup of a head that counts last in hcnt[4h] merges the head's chunks
  // and quantizes the attention output into (oq_qs, oq_d), the out-projection's input
  unsigned *hcnt;
  uint8_t *oq_qs;
  float *oq_d;
};

struct FastOproj {
  W4 w;                    // out-projection E x E
  const uint8_t *xq;       // merged attention output, Q4 SoA (FastTail::oq_qs / oq_d)
  const float *xd;
  int d;
  const float *bo;         // may be null (GPT-J)
  const float *ffp;        // [sf][E]
  int sf;
  const float *bproj;
  const float *x;          // residual in
  float *out;              // residual out
};

int launch_fast_ln(const FastLn &P, hipStream_t s);
int launch_fast_gemv(const FastGemv &P, int E, hipStream_t s);
int launch_fast_tail(const FastTail &A, hipStream_t s);
int launch_fast_oproj_join(const FastOproj &P, hipStream_t s);

}  // namespace vsim
