// vsim_amd/csrc/model.cpp — device-resident model executor (layer 3 of vsim_hip.h).
//
// One eval = the reference's gptneox_eval graph (vsim.cpp:470-747) or the GPT-J graph
// built from the same ggml ops, executed as a fixed sequence of HIP kernels on one
// stream.  Weights (Q4 SoA), LayerNorm/bias vectors, the F32 KV cache
// ([layer][n_ctx][E], vsim.cpp:349-366) and all activations stay in HBM; per eval the
// host sends the token ids and receives one logits row (vsim.cpp:736-737).
// A pipeline stage owns layers [l0, l1); stages exchange the residual inpL ([N][E] f32).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <vector>

#include "common.hpp"
#include "fast.hpp"
#include "../../include/vsim_hip.h"

using namespace vsim;

namespace {

enum Kind { KQ4 = 0, KF32 = 1 };

struct Slot {
  void *ptr;
  int kind;
  int rows, k;  // Q4: rows x k ; F32: k elements (rows = 1)
  int layer;    // -1 for global tensors
  bool loaded;
};

struct LayerW {
  // (BLOOM: wq/wk/wv are the three row blocks of the fused query_key_value tensor, each
  // repacked on its own; bq/bk/bv point into its one bias vector)
  void *wq = nullptr, *wk = nullptr, *wv = nullptr, *wo = nullptr, *wfc = nullptr, *wproj = nullptr;
  float *ln1_w = nullptr, *ln1_b = nullptr, *ln2_w = nullptr, *ln2_b = nullptr;
  float *bq = nullptr, *bk = nullptr, *bv = nullptr, *bo = nullptr, *bfc = nullptr, *bproj = nullptr;
};

}  // namespace

struct vsim_model {
  int arch = VSIM_ARCH_GPTNEOX;
  unsigned *err_dev = nullptr, *err_host = nullptr;  // this model's bounded-wait timeouts (spin_check)
  unsigned err_seen = 0;
  vsim_hparams hp{};
  int n_ctx = 512, device = 0, l0 = 0, l1 = 0;
  bool first = true, last = true;
  int mode = VSIM_MODE_EXACT;
  bool graph_enabled = false;
  hipStream_t stream = nullptr;

  uint8_t *warena = nullptr;  // all weights of this stage
  size_t wbytes = 0;
  std::map<std::string, Slot> slots;
  std::vector<LayerW> layers;
  void *wte = nullptr, *lmh = nullptr;
  float *lnf_w = nullptr, *lnf_b = nullptr, *lmh_b = nullptr;
  float *emb_w = nullptr, *emb_b = nullptr;  // BLOOM word_embeddings_layernorm
  float *alibi = nullptr;                    // BLOOM: device head slopes [n_head]

  float *kcache = nullptr, *vcache = nullptr;
  double2 *rope_cs = nullptr;

  // scratch, sized for n_max tokens
  int n_max = 0;
  float *inpL = nullptr, *cur1 = nullptr, *cur2 = nullptr, *Qb = nullptr, *Kb = nullptr, *Vb = nullptr;
  float *attn_in = nullptr, *attn = nullptr, *ff = nullptr, *fch = nullptr, *kq = nullptr, *logits = nullptr;
  uint8_t *xq1 = nullptr, *xq2 = nullptr, *xq3 = nullptr;
  float *xd1 = nullptr, *xd2 = nullptr, *xd3 = nullptr;
  int32_t *tok_dev = nullptr;
  int32_t *tok_host = nullptr;  // pinned
  float *logit_host = nullptr;  // pinned
  int kernels_last = 0;

  // fused single-token decode step (layer.hip) and its hipGraph
  uint8_t *xqa = nullptr;     // attention output, quantized
  float *xda = nullptr;
  float *inpL2 = nullptr;     // second residual buffer (the join alternates between the two)
  float *resid_final = nullptr;  // where the last fused step left the stage's residual
  int *npast_dev = nullptr, *npast_host = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  // greedy variant of the decode graph: device argmax, 4-byte copy-out instead of the logits
  hipGraph_t graph_am = nullptr;
  hipGraphExec_t gexec_am = nullptr;
  int graph_am_mode = -1;
  int *am_dev = nullptr, *am_host = nullptr;
  unsigned long long *am_ws = nullptr;  // the argmax's key and workgroup count (zero between launches)
  // device-resident greedy loop (vsim_model_generate): graph without uploads; the argmax
  // kernel feeds tok_dev / npast_dev and records into hist_dev[n_ctx]
  hipGraph_t graph_gen = nullptr;
  hipGraphExec_t gexec_gen = nullptr;
  int graph_gen_mode = -1;
  int *hist_dev = nullptr;
  // pipeline stage step (vsim_model_stage_*): device buffers the caller binds (the token in
  // on the first stage, the residual in / out between stages, the greedy token out on the
  // last), a graph of the whole step that ends by advancing n_past on the device, and the
  // host's count of enqueued steps (n_ctx bound)
  const int32_t *st_tok_in = nullptr;
  const float *st_resid_in = nullptr;
  float *st_resid_out = nullptr;
  int32_t *st_tok_out = nullptr;
  hipGraph_t graph_st = nullptr;
  hipGraphExec_t gexec_st = nullptr;
  int graph_st_mode = -1;
  int st_npast = -1;
  unsigned *tail_done = nullptr;  // the fast decode step's per-head counters (fast_decode.hip)
  // the tail LayerNorm's hand-off buffers (TailLn): the step epoch, the out-projection's and the joined row's
  // granules [E], the per-tile partial sums [2 E/32]; zeroed at allocation (tag 0 never matches)
  unsigned *lnt_ep = nullptr;
  unsigned long long *lnt_og = nullptr, *lnt_jg = nullptr;
  uint4 *lnt_rec = nullptr;
  unsigned long long *tail_hflag = nullptr;  // the tail heads' flags (TailSync), in the same allocation
  // fast-mode decode step (fast_decode.hip): fc_out split-K partial rows and attention
  // chunk partials (both consumed by the layer's k_fast_oproj_join)
  float *fast_ffp = nullptr, *fast_part = nullptr;
  void *pf_scratch = nullptr;  // fast prefill: fp16 K / V^T copies (attn_prefill.hip)
  void *pf_x16 = nullptr;      // fast prefill: fp16 GEMM operands, [n_max][E] then [n_max][4E]
  size_t pf_bytes = 0;

  int graph_mode = -1;
  // graph executor's fast path (graph.cpp): weights and KV cache borrowed from its device
  // mirrors (not freed here), the KQV key grouping of the caller's thread count and the
  // scale the graph carries (0: computed from the hparams)
  bool borrowed = false;
  int kqv_nth = 1;
  float attn_scale = 0.0f;
  int graph_kernels_kind[4] = {0, 0, 0, 0};  // per decode_graph kind: kernels in one replay

  // Per-kernel profiling (bench.py's live roofline): with profiling on, the decode step runs
  // eagerly and an event pair brackets every launch, tagged with the kernel's name and the
  // algorithmic bytes it moves (Q4_0 weights at 0.625 B/weight, KV rows, activations).
  struct ProfRec {
    size_t ev;
    std::string kind;
    double bytes;
  };
  struct ProfKind {
    std::string name;
    double ms = 0.0, bytes = 0.0;
    long n = 0;
  };
  bool profile = false;
  int prof_npast = 0;  // n_past of the step being enqueued (host copy, for the KV byte counts)
  std::vector<hipEvent_t> prof_events;
  std::vector<ProfRec> prof_pending;
  size_t prof_used = 0;
  std::vector<ProfKind> prof_kinds;
};

namespace {

int E_(const vsim_model *m) { return m->hp.n_embd; }

void free_scratch(vsim_model *m) {
  void *ps[] = {m->inpL, m->cur1, m->cur2, m->Qb, m->Kb, m->Vb, m->attn_in, m->attn, m->ff, m->fch, m->kq,
                m->logits, m->xq1, m->xq2, m->xq3, m->xd1, m->xd2, m->xd3, m->tok_dev};
  for (void *p : ps)
    if (p) (void)hipFree(p);
  if (m->tok_host) (void)hipHostFree(m->tok_host);
  if (m->logit_host) (void)hipHostFree(m->logit_host);
  if (m->gexec) (void)hipGraphExecDestroy(m->gexec);
  if (m->graph) (void)hipGraphDestroy(m->graph);
  if (m->gexec_am) (void)hipGraphExecDestroy(m->gexec_am);
  if (m->graph_am) (void)hipGraphDestroy(m->graph_am);
  if (m->am_dev) (void)hipFree(m->am_dev);
  if (m->am_ws) (void)hipFree(m->am_ws);
  m->am_ws = nullptr;
  if (m->am_host) (void)hipHostFree(m->am_host);
  m->gexec_am = nullptr;
  m->graph_am = nullptr;
  m->graph_am_mode = -1;
  m->am_dev = m->am_host = nullptr;
  if (m->gexec_gen) (void)hipGraphExecDestroy(m->gexec_gen);
  if (m->graph_gen) (void)hipGraphDestroy(m->graph_gen);
  if (m->hist_dev) (void)hipFree(m->hist_dev);
  if (m->tail_done) (void)hipFree(m->tail_done);
  m->tail_done = nullptr;
  if (m->lnt_ep) (void)hipFree(m->lnt_ep);
  m->lnt_ep = nullptr;
  m->lnt_og = m->lnt_jg = nullptr;
  m->lnt_rec = nullptr;
  m->tail_hflag = nullptr;
  if (m->pf_scratch) (void)hipFree(m->pf_scratch);
  m->pf_scratch = nullptr;
  if (m->pf_x16) (void)hipFree(m->pf_x16);
  m->pf_x16 = nullptr;
  m->pf_bytes = 0;
  if (m->fast_ffp) (void)hipFree(m->fast_ffp);
  if (m->fast_part) (void)hipFree(m->fast_part);
  m->fast_ffp = m->fast_part = nullptr;
  m->gexec_gen = nullptr;
  m->graph_gen = nullptr;
  m->graph_gen_mode = -1;
  m->hist_dev = nullptr;
  if (m->gexec_st) (void)hipGraphExecDestroy(m->gexec_st);
  if (m->graph_st) (void)hipGraphDestroy(m->graph_st);
  m->gexec_st = nullptr;
  m->graph_st = nullptr;
  m->graph_st_mode = -1;
  if (m->xqa) (void)hipFree(m->xqa);
  if (m->xda) (void)hipFree(m->xda);
  if (m->inpL2) (void)hipFree(m->inpL2);
  m->inpL2 = nullptr;
  if (m->npast_dev) (void)hipFree(m->npast_dev);
  if (m->npast_host) (void)hipHostFree(m->npast_host);
  m->gexec = nullptr;
  m->graph = nullptr;
  m->graph_mode = -1;
  m->xqa = nullptr;
  m->xda = nullptr;
  m->npast_dev = m->npast_host = nullptr;
  m->st_npast = -1;  // the device n_past went with npast_dev: stage_step needs a new stage_begin
  m->inpL = m->cur1 = m->cur2 = m->Qb = m->Kb = m->Vb = m->attn_in = m->attn = m->ff = m->fch = m->kq = m->logits =
      nullptr;
  m->xq1 = m->xq2 = m->xq3 = nullptr;
  m->xd1 = m->xd2 = m->xd3 = nullptr;
  m->tok_dev = nullptr;
  m->tok_host = nullptr;
  m->logit_host = nullptr;
  m->n_max = 0;
}

int ensure_scratch(vsim_model *m, int N) {
  if (N <= m->n_max) return VSIM_OK;
  VSIM_HIP(hipStreamSynchronize(m->stream));
  free_scratch(m);
  const int n = N < 16 ? 16 : N;
  const size_t E = E_(m), F = 4 * E, V = m->hp.n_vocab, H = m->hp.n_head;
  auto fa = [&](float **p, size_t cnt) { return hipMalloc((void **)p, cnt * sizeof(float)); };
  auto ba = [&](uint8_t **p, size_t k) { return hipMalloc((void **)p, (size_t)n * k / QK * QBYTES); };
  VSIM_HIP(fa(&m->inpL, n * E));
  VSIM_HIP(fa(&m->cur1, n * E));
  VSIM_HIP(fa(&m->cur2, n * E));
  VSIM_HIP(fa(&m->Qb, n * E));
  VSIM_HIP(fa(&m->Kb, n * E));
  VSIM_HIP(fa(&m->Vb, n * E));
  VSIM_HIP(fa(&m->attn_in, n * E));
  VSIM_HIP(fa(&m->attn, n * E));
  VSIM_HIP(fa(&m->ff, n * E));
  VSIM_HIP(fa(&m->fch, n * F));
  VSIM_HIP(fa(&m->kq, (size_t)n * H * m->n_ctx));
  VSIM_HIP(fa(&m->logits, V));
  VSIM_HIP(ba(&m->xq1, E));
  VSIM_HIP(ba(&m->xq2, E));
  VSIM_HIP(ba(&m->xq3, F));
  VSIM_HIP(fa(&m->xd1, n * E));
  VSIM_HIP(fa(&m->xd2, n * E));
  VSIM_HIP(fa(&m->xd3, n * F));
  VSIM_HIP(hipMalloc((void **)&m->tok_dev, n * sizeof(int32_t)));
  VSIM_HIP(hipHostMalloc((void **)&m->tok_host, n * sizeof(int32_t), hipHostMallocDefault));
  VSIM_HIP(hipHostMalloc((void **)&m->logit_host, V * sizeof(float), hipHostMallocDefault));
  VSIM_HIP(ba(&m->xqa, E));
  VSIM_HIP(fa(&m->xda, n * E));
  VSIM_HIP(fa(&m->inpL2, E));
  VSIM_HIP(hipMalloc((void **)&m->npast_dev, sizeof(int)));
  VSIM_HIP(hipHostMalloc((void **)&m->npast_host, sizeof(int), hipHostMallocDefault));
  VSIM_HIP(hipMalloc((void **)&m->am_dev, sizeof(int)));
  VSIM_HIP(hipMalloc((void **)&m->am_ws, 2 * sizeof(unsigned long long)));
  VSIM_HIP(hipMemset(m->am_ws, 0, 2 * sizeof(unsigned long long)));
  VSIM_HIP(hipHostMalloc((void **)&m->am_host, sizeof(int), hipHostMallocDefault));
  VSIM_HIP(hipMalloc((void **)&m->hist_dev, (size_t)m->n_ctx * sizeof(int)));
  // counters of the fused layer kernels at [0], [64], [128] (separate 256-byte lines)
  // (k_layer_exact: one set per layer, [il - l0][256], zeroed by a memset node per token)
  const size_t ncnt = (size_t)std::max(1, m->l1 - m->l0) * 256;
  VSIM_HIP(hipMalloc((void **)&m->tail_done, ncnt * sizeof(unsigned)));
  VSIM_HIP(hipMemset(m->tail_done, 0, ncnt * sizeof(unsigned)));
  {
    // one allocation: epoch (own 256-byte line), og [E], jg [E], rec [2 E/32], the heads' flags
    const size_t lb = 256 + 2 * E * sizeof(unsigned long long) + 2 * (E / QK) * sizeof(uint4) +
                      TAIL_MAX_HEADS * sizeof(unsigned long long);
    uint8_t *p = nullptr;
    VSIM_HIP(hipMalloc((void **)&p, lb));
    VSIM_HIP(hipMemset(p, 0, lb));
    m->lnt_ep = (unsigned *)p;
    m->lnt_og = (unsigned long long *)(p + 256);
    m->lnt_jg = m->lnt_og + E;
    m->lnt_rec = (uint4 *)(m->lnt_jg + E);
    m->tail_hflag = (unsigned long long *)(m->lnt_rec + 2 * (E / QK));
  }
  {
    const size_t d = E / H, nch = (m->n_ctx + FD_CHUNK - 1) / FD_CHUNK;
    VSIM_HIP(fa(&m->fast_ffp, 8 * E));
    if (n >= GEMM_MIN_N) VSIM_HIP(hipMalloc(&m->pf_x16, (size_t)n * (E + F) * sizeof(uint16_t)));
    VSIM_HIP(fa(&m->fast_part, H * nch * (d + 2)));
    VSIM_HIP(hipMemset(m->fast_part, 0, H * nch * (d + 2) * sizeof(float)));  // finite stale values
  }
  m->n_max = n;
  return VSIM_OK;
}

// Register every tensor this stage owns, with its ggml-file name and byte size.
void plan_slots(vsim_model *m, std::vector<std::pair<std::string, Slot>> &out) {
  const int E = m->hp.n_embd, V = m->hp.n_vocab, F = 4 * E;
  auto q = [&](const std::string &n, int rows, int k, int layer) { out.push_back({n, Slot{nullptr, KQ4, rows, k, layer, false}}); };
  auto f = [&](const std::string &n, int k, int layer) { out.push_back({n, Slot{nullptr, KF32, 1, k, layer, false}}); };
  if (m->arch == VSIM_ARCH_GPTNEOX) {
    if (m->first) q("gpt_neox.embed_in.weight", V, E, -1);
    if (m->last) {
      f("gpt_neox.final_layer_norm.weight", E, -1);
      f("gpt_neox.final_layer_norm.bias", E, -1);
      q("embed_out.weight", V, E, -1);
    }
    for (int i = m->l0; i < m->l1; ++i) {
      const std::string p = "gpt_neox.layers." + std::to_string(i) + ".";
      f(p + "input_layernorm.weight", E, i);
      f(p + "input_layernorm.bias", E, i);
      f(p + "post_attention_layernorm.weight", E, i);
      f(p + "post_attention_layernorm.bias", E, i);
      q(p + "attention.query.weight", E, E, i);
      f(p + "attention.query.bias", E, i);
      q(p + "attention.key.weight", E, E, i);
      f(p + "attention.key.bias", E, i);
      q(p + "attention.value.weight", E, E, i);
      f(p + "attention.value.bias", E, i);
      q(p + "attention.dense.weight", E, E, i);
      f(p + "attention.dense.bias", E, i);
      q(p + "mlp.dense_h_to_4h.weight", F, E, i);
      f(p + "mlp.dense_h_to_4h.bias", F, i);
      q(p + "mlp.dense_4h_to_h.weight", E, F, i);
      f(p + "mlp.dense_4h_to_h.bias", E, i);
    }
  } else if (m->arch == VSIM_ARCH_BLOOM) {  // convert_bloom_to_ggml.py:22-34 names
    if (m->first) {
      q("tok_embeddings.weight", V, E, -1);
      f("norm.weight", E, -1);
      f("norm.bias", E, -1);
    }
    if (m->last) {
      f("output_norm.weight", E, -1);
      f("output_norm.bias", E, -1);
      q("output.weight", V, E, -1);
    }
    for (int i = m->l0; i < m->l1; ++i) {
      const std::string p = "layers." + std::to_string(i) + ".";
      f(p + "attention_norm.weight", E, i);
      f(p + "attention_norm.bias", E, i);
      q(p + "attention.query_key_value.weight/q", E, E, i);  // the file tensor's row blocks
      q(p + "attention.query_key_value.weight/k", E, E, i);
      q(p + "attention.query_key_value.weight/v", E, E, i);
      f(p + "attention.query_key_value.bias", 3 * E, i);
      q(p + "attention.wo.weight", E, E, i);
      f(p + "attention.wo.bias", E, i);
      f(p + "ffn_norm.weight", E, i);
      f(p + "ffn_norm.bias", E, i);
      q(p + "feed_forward.w1.weight", F, E, i);
      f(p + "feed_forward.w1.bias", F, i);
      q(p + "feed_forward.w2.weight", E, F, i);
      f(p + "feed_forward.w2.bias", E, i);
    }
  } else {
    if (m->first) q("transformer.wte.weight", V, E, -1);
    if (m->last) {
      f("transformer.ln_f.weight", E, -1);
      f("transformer.ln_f.bias", E, -1);
      q("lm_head.weight", V, E, -1);
      f("lm_head.bias", V, -1);
    }
    for (int i = m->l0; i < m->l1; ++i) {
      const std::string p = "transformer.h." + std::to_string(i) + ".";
      f(p + "ln_1.weight", E, i);
      f(p + "ln_1.bias", E, i);
      q(p + "attn.q_proj.weight", E, E, i);
      q(p + "attn.k_proj.weight", E, E, i);
      q(p + "attn.v_proj.weight", E, E, i);
      q(p + "attn.out_proj.weight", E, E, i);
      q(p + "mlp.fc_in.weight", F, E, i);
      f(p + "mlp.fc_in.bias", F, i);
      q(p + "mlp.fc_out.weight", E, F, i);
      f(p + "mlp.fc_out.bias", E, i);
    }
  }
}

// bytes of the tensor in the ggml file (AoS blocks) and on the device (W4T32, padded)
size_t slot_bytes(const Slot &s) {
  return s.kind == KQ4 ? (size_t)s.rows * s.k / QK * QBYTES : (size_t)s.k * sizeof(float);
}
size_t slot_dev_bytes(const Slot &s) { return s.kind == KQ4 ? w4_bytes(s.rows, s.k) : (size_t)s.k * sizeof(float); }

void bind_pointers(vsim_model *m) {
  auto P = [&](const std::string &n) -> void * {
    auto it = m->slots.find(n);
    return it == m->slots.end() ? nullptr : it->second.ptr;
  };
  auto F = [&](const std::string &n) { return (float *)P(n); };
  m->layers.assign(m->l1 - m->l0, LayerW{});
  if (m->arch == VSIM_ARCH_GPTNEOX) {
    m->wte = P("gpt_neox.embed_in.weight");
    m->lnf_w = F("gpt_neox.final_layer_norm.weight");
    m->lnf_b = F("gpt_neox.final_layer_norm.bias");
    m->lmh = P("embed_out.weight");
    for (int i = m->l0; i < m->l1; ++i) {
      LayerW &L = m->layers[i - m->l0];
      const std::string p = "gpt_neox.layers." + std::to_string(i) + ".";
      L.ln1_w = F(p + "input_layernorm.weight");
      L.ln1_b = F(p + "input_layernorm.bias");
      L.ln2_w = F(p + "post_attention_layernorm.weight");
      L.ln2_b = F(p + "post_attention_layernorm.bias");
      L.wq = P(p + "attention.query.weight");
      L.bq = F(p + "attention.query.bias");
      L.wk = P(p + "attention.key.weight");
      L.bk = F(p + "attention.key.bias");
      L.wv = P(p + "attention.value.weight");
      L.bv = F(p + "attention.value.bias");
      L.wo = P(p + "attention.dense.weight");
      L.bo = F(p + "attention.dense.bias");
      L.wfc = P(p + "mlp.dense_h_to_4h.weight");
      L.bfc = F(p + "mlp.dense_h_to_4h.bias");
      L.wproj = P(p + "mlp.dense_4h_to_h.weight");
      L.bproj = F(p + "mlp.dense_4h_to_h.bias");
    }
  } else if (m->arch == VSIM_ARCH_BLOOM) {
    m->wte = P("tok_embeddings.weight");
    m->emb_w = F("norm.weight");
    m->emb_b = F("norm.bias");
    m->lnf_w = F("output_norm.weight");
    m->lnf_b = F("output_norm.bias");
    m->lmh = P("output.weight");
    const int E = m->hp.n_embd;
    for (int i = m->l0; i < m->l1; ++i) {
      LayerW &L = m->layers[i - m->l0];
      const std::string p = "layers." + std::to_string(i) + ".";
      L.ln1_w = F(p + "attention_norm.weight");
      L.ln1_b = F(p + "attention_norm.bias");
      L.ln2_w = F(p + "ffn_norm.weight");
      L.ln2_b = F(p + "ffn_norm.bias");
      L.wq = P(p + "attention.query_key_value.weight/q");
      L.wk = P(p + "attention.query_key_value.weight/k");
      L.wv = P(p + "attention.query_key_value.weight/v");
      L.bq = F(p + "attention.query_key_value.bias");
      L.bk = L.bq + E;
      L.bv = L.bq + 2 * E;
      L.wo = P(p + "attention.wo.weight");
      L.bo = F(p + "attention.wo.bias");
      L.wfc = P(p + "feed_forward.w1.weight");
      L.bfc = F(p + "feed_forward.w1.bias");
      L.wproj = P(p + "feed_forward.w2.weight");
      L.bproj = F(p + "feed_forward.w2.bias");
    }
  } else {
    m->wte = P("transformer.wte.weight");
    m->lnf_w = F("transformer.ln_f.weight");
    m->lnf_b = F("transformer.ln_f.bias");
    m->lmh = P("lm_head.weight");
    m->lmh_b = F("lm_head.bias");
    for (int i = m->l0; i < m->l1; ++i) {
      LayerW &L = m->layers[i - m->l0];
      const std::string p = "transformer.h." + std::to_string(i) + ".";
      L.ln1_w = F(p + "ln_1.weight");
      L.ln1_b = F(p + "ln_1.bias");
      L.wq = P(p + "attn.q_proj.weight");
      L.wk = P(p + "attn.k_proj.weight");
      L.wv = P(p + "attn.v_proj.weight");
      L.wo = P(p + "attn.out_proj.weight");
      L.wfc = P(p + "mlp.fc_in.weight");
      L.bfc = F(p + "mlp.fc_in.bias");
      L.wproj = P(p + "mlp.fc_out.weight");
      L.bproj = F(p + "mlp.fc_out.bias");
    }
  }
}

#define RC(x)                    \
  do {                           \
    int rc_ = (x);               \
    if (rc_) return rc_;         \
  } while (0)

// Bounded cross-workgroup waits that gave up (k_layer_tail, the barrier-free chain GEMV, the
// stream-K finisher) count into the model's own device word (m->err_dev: every launch this model
// enqueues gets it through ErrScope, so another model's or a standalone op's timeout never fails
// this one).  spin_read enqueues its copy to pinned host memory ahead of the call's stream sync;
// spin_check, after that sync, fails the call with VSIM_ESPIN when it grew: some tile went on
// with incomplete data, so the results are not the reference's.
struct ErrScope {
  unsigned *old;
  explicit ErrScope(vsim_model *m) : old(set_spin_error_target(m->err_dev)) {}
  ~ErrScope() { set_spin_error_target(old); }
};
int spin_read(vsim_model *m) {
  VSIM_HIP(hipMemcpyAsync(m->err_host, m->err_dev, sizeof(unsigned), hipMemcpyDeviceToHost, m->stream));
  return VSIM_OK;
}
int spin_check(vsim_model *m) {
  const unsigned n = *(volatile unsigned *)m->err_host;
  if (n > m->err_seen) {
    const unsigned grew = n - m->err_seen;
    m->err_seen = n;
    add_model_spin_timeouts(grew);
    // a workgroup that gave up may have left the argmax workspace mid-update: zero it again
    (void)hipMemsetAsync(m->am_ws, 0, 2 * sizeof(unsigned long long), m->stream);
    (void)hipStreamSynchronize(m->stream);
    set_error("a bounded cross-workgroup wait gave up " + std::to_string(grew) +
              " time(s) in this call (device " + std::to_string(m->device) + "): results not valid");
    return VSIM_ESPIN;
  }
  return VSIM_OK;
}

// Profiling brackets (eager launches only): prof_begin records the start event and returns
// its slot (-1 when profiling is off); prof_end records the end and tags the pair.
long prof_begin(vsim_model *m) {
  if (!m->profile) return -1;
  if (m->prof_used + 2 > m->prof_events.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
    m->prof_events.push_back(a);
    m->prof_events.push_back(b);
  }
  const size_t i = m->prof_used;
  m->prof_used += 2;
  (void)hipEventRecord(m->prof_events[i], m->stream);
  return (long)i;
}
void prof_end(vsim_model *m, long ev, const std::string &kind, double bytes) {
  if (ev < 0) return;
  (void)hipEventRecord(m->prof_events[ev + 1], m->stream);
  m->prof_pending.push_back({(size_t)ev, kind, bytes});
}
// after the stream synchronised: fold the pending pairs into the per-kernel totals
int prof_collect(vsim_model *m) {
  for (const auto &r : m->prof_pending) {
    float ms = 0.0f;
    VSIM_HIP(hipEventElapsedTime(&ms, m->prof_events[r.ev], m->prof_events[r.ev + 1]));
    size_t k = 0;
    while (k < m->prof_kinds.size() && m->prof_kinds[k].name != r.kind) ++k;
    if (k == m->prof_kinds.size()) {
      m->prof_kinds.emplace_back();
      m->prof_kinds.back().name = r.kind;
    }
    m->prof_kinds[k].ms += ms;
    m->prof_kinds[k].bytes += r.bytes;
    m->prof_kinds[k].n += 1;
  }
  m->prof_pending.clear();
  m->prof_used = 0;
  return VSIM_OK;
}

double w4_algo_bytes(const W4 &w) { return (double)w.rows * w.k / QK * QBYTES; }

// Quantize an activation and run one GEMV in the model's mode.  x16 non-null (fast-mode
// prompt batches): the activation is already the GEMM's fp16 operand (launch_act_quant_f16).
// gq (fc_in of a long prompt): bias gq_bias + GELU + quantize of the product straight into the
// next GEMM's fp16 operand gq, in the GEMM's epilogue; epi: RoPE or the residual join in the
// epilogue (G2Epi); *fused tells the caller whether either ran.
int mm(vsim_model *m, const void *W, int M, int K, const float *x, int N, uint8_t *xq, float *xd, bool quantize,
       const float *bias, float *y, int &nk, const void *x16 = nullptr, void *gq = nullptr,
       const float *gq_bias = nullptr, bool *fused = nullptr, const G2Epi *epi = nullptr) {
  if (fused) *fused = false;
  if (quantize && !x16) {
    RC(launch_q4_quantize(x, K, N, xq, xd, m->stream));
    ++nk;
  }
  // long prompt: the 256-wide-tile GEMM, the Q4_0 weight dequantized to fp16 in LDS
  if (x16 && N >= G2_MIN_N && K % 64 == 0) {
    const bool gelu = gq && gq_bias && M % QK == 0;
    const long ev = prof_begin(m);
    RC(launch_gemm_q4_256(w4_view(W, M, K), x16, N, gelu ? gq_bias : bias, y, m->stream, gelu ? gq : nullptr,
                          gelu ? nullptr : epi));
    prof_end(m, ev, "k_gemm_f16_256 (prompt)", (double)M * K / QK * QBYTES);
    ++nk;
    if (fused) *fused = gelu || epi;
    return VSIM_OK;
  }
  const long ev = prof_begin(m);
  if (x16) {
    RC(launch_gemm_f16x(w4_view(W, M, K), x16, N, bias, y, m->stream));
  } else {
    RC(launch_q4_gemv(W, M, K, xq, xd, N, bias, y, m->mode, m->stream));
  }
  prof_end(m, ev, x16 ? "k_gemm_f16 (prompt)" : N > 1 ? "gemv (prompt rows)" : "gemv (general path)",
           (double)M * K / QK * QBYTES);
  ++nk;
  return VSIM_OK;
}

// The BLOOM layer (oracle eval_bloom): LN -> q/k/v (+bias) -> KV write -> KQ -> scale ->
// alibi -> mask -> softmax -> KQV -> wo (+bias) -> inpFF = attn + inpL -> LN -> w1 (+bias) ->
// GELU -> w2 (+bias) -> inpL = ff + inpFF.
int run_layer_bloom(vsim_model *m, int il, int n_past, int N, int &nk) {
  const LayerW &L = m->layers[il - m->l0];
  const int E = m->hp.n_embd, H = m->hp.n_head, d = E / H, F = 4 * E;
  hipStream_t s = m->stream;
  // fast-mode prompt batch: GEMM operands straight to fp16 in the model's scratch (as run_layer)
  const bool pf = m->mode == VSIM_MODE_FAST && N >= GEMM_MIN_N && m->pf_x16;
  void *xa = pf ? m->pf_x16 : nullptr;
  void *xb = pf ? (void *)((uint16_t *)m->pf_x16 + (size_t)N * E) : nullptr;
  auto act16 = [&](const float *x, int K, void *x16, const float *gbias, bool gelu) -> int {
    if (!pf) return VSIM_OK;
    ++nk;
    return launch_act_quant_f16(x, K, N, gbias, gelu, x16, s);
  };
  // LayerNorm (straight to the GEMM's fp16 operand in a prompt batch)
  auto norm = [&](const float *x, float *y, const float *w, const float *b, void *x16) -> int {
    ++nk;
    return pf ? launch_norm_f16q(x, x16, E, N, w, b, s) : launch_norm(x, y, E, N, w, b, s);
  };
  RC(norm(m->inpL, m->cur1, L.ln1_w, L.ln1_b, xa));
  RC(mm(m, L.wq, E, E, m->cur1, N, m->xq1, m->xd1, true, L.bq, m->Qb, nk, xa));
  RC(mm(m, L.wk, E, E, m->cur1, N, m->xq1, m->xd1, false, L.bk, m->Kb, nk, xa));
  RC(mm(m, L.wv, E, E, m->cur1, N, m->xq1, m->xd1, false, L.bv, m->Vb, nk, xa));
  const size_t loff = (size_t)(il - m->l0) * m->n_ctx * E;
  float *kc = m->kcache + loff, *vc = m->vcache + loff;
  RC(launch_rope_kv_write(0, m->Qb, m->Kb, m->Vb, kc, vc, d, H, N, n_past, 0, m->rope_cs, s)); ++nk;  // no rotary
  const int nkv = n_past + N;
  const float scale = (float)(1.0f / std::sqrt((double)(float(E) / H)));
  RC(launch_kq(kc, E, m->Qb, E, d, H, nkv, N, m->kq, s, n_past)); ++nk;
  RC(launch_attn_softmax(m->kq, nkv, N, H, n_past, scale, s, m->alibi)); ++nk;
  RC(launch_kqv(vc, E, m->kq, d, H, nkv, N, m->attn_in, 1, s, n_past)); ++nk;
  RC(act16(m->attn_in, E, xb, nullptr, false));
  RC(mm(m, L.wo, E, E, m->attn_in, N, m->xq2, m->xd2, true, L.bo, m->attn, nk, xb));
  // inpFF = attn + inpL (kept in cur2), its LayerNorm into cur1
  VSIM_HIP(hipMemcpyAsync(m->cur2, m->attn, sizeof(float) * N * E, hipMemcpyDeviceToDevice, s));
  RC(launch_add_bias(m->cur2, m->inpL, N * E, 1, s)); ++nk;
  RC(norm(m->cur2, m->cur1, L.ln2_w, L.ln2_b, xa));
  bool gq = false;
  RC(mm(m, L.wfc, F, E, m->cur1, N, m->xq2, m->xd2, true, nullptr, m->fch, nk, xa, xb, L.bfc, &gq));
  if (pf) {
    if (!gq) RC(act16(m->fch, F, xb, L.bfc, true));  // bias + GELU + quantize, one pass
  } else {
    RC(launch_gelu(m->fch, m->fch, N * F, L.bfc, F, s)); ++nk;
  }
  RC(mm(m, L.wproj, E, F, m->fch, N, m->xq3, m->xd3, true, L.bproj, m->ff, nk, xb));
  // inpL = ff + inpFF
  VSIM_HIP(hipMemcpyAsync(m->inpL, m->cur2, sizeof(float) * N * E, hipMemcpyDeviceToDevice, s));
  RC(launch_add_bias(m->inpL, m->ff, N * E, 1, s)); ++nk;
  return VSIM_OK;
}

int run_layer(vsim_model *m, int il, int n_past, int N, int &nk) {
  if (m->arch == VSIM_ARCH_BLOOM) return run_layer_bloom(m, il, n_past, N, nk);
  const LayerW &L = m->layers[il - m->l0];
  const int E = m->hp.n_embd, H = m->hp.n_head, d = E / H, F = 4 * E;
  const bool gptj = m->arch == VSIM_ARCH_GPTJ;
  hipStream_t s = m->stream;
  // fast-mode prompt batch: every activation goes once from f32 to the GEMM's fp16 operand
  // (quantize_row_q4_0 values, k_act_quant_f16; the GELU folded into fc_out's)
  // (operands in the model's scratch, pf_x16: [N][E] norm outputs, then [N][F] attention /
  // GELU outputs)
  const bool pf = m->mode == VSIM_MODE_FAST && N >= GEMM_MIN_N && m->pf_x16;
  struct {
    void *a, *b;
  } X = {m->pf_x16, pf ? (void *)((uint16_t *)m->pf_x16 + (size_t)N * E) : nullptr};
  if (!pf) X.a = nullptr;
  auto act16 = [&](const float *x, int K, void *x16, const float *gbias, bool gelu) -> int {
    if (!pf) return VSIM_OK;
    ++nk;
    return launch_act_quant_f16(x, K, N, gbias, gelu, x16, s);
  };
  // input LayerNorm + affine (vsim.cpp:526-533)
  auto norm = [&](const float *x, float *y, const float *w, const float *b, void *x16) -> int {
    ++nk;  // (prompt batch: straight to the GEMM's fp16 operand)
    return pf ? launch_norm_f16q(x, x16, E, N, w, b, s) : launch_norm(x, y, E, N, w, b, s);
  };
  RC(norm(m->inpL, m->cur1, L.ln1_w, L.ln1_b, X.a));
  const size_t loff = (size_t)(il - m->l0) * m->n_ctx * E;
  float *kc = m->kcache + loff, *vc = m->vcache + loff;
  // long GPT-J prompt: RoPE and the KV-cache write (vsim.cpp:553-580) in the Q/K/V GEMMs'
  // epilogues -- K and V straight into their cache rows -- instead of a pass of their own
  const bool g2 = pf && N >= G2_MIN_N && E % 64 == 0;
  const bool rope_epi = g2 && gptj;
  G2Epi er;
  er.cs = m->rope_cs;
  er.d = d;
  er.n_rot = m->hp.n_rot;
  er.p0 = n_past;
  float *kout = rope_epi ? kc + (size_t)n_past * E : m->Kb, *vout = rope_epi ? vc + (size_t)n_past * E : m->Vb;
  // ... and the new keys' fp16 copies for the prompt attention (K rows, V^T columns), which
  // then converts only the cached keys before them
  const bool attn16 = m->mode == VSIM_MODE_FAST && N >= 8 && attn_prefill_supported(d) && E % 64 == 0;
  if (attn16 && !m->pf_scratch) {  // (prompt evals are never graph-captured: allocating here is safe)
    m->pf_bytes = attn_prefill_scratch(E, m->n_ctx);
    VSIM_HIP(hipMalloc(&m->pf_scratch, m->pf_bytes));
  }
  const bool kv16_epi = rope_epi && attn16;
  G2Epi ek = er, ev;
  if (kv16_epi) {
    ek.h16 = attn_prefill_k16(m->pf_scratch, E, n_past + N);
    ev.h16 = attn_prefill_vt16(m->pf_scratch, E, n_past + N);
    ev.h16_t = 1;
    ev.h16_ld = attn_prefill_ldt(n_past + N);
    ev.p0 = n_past;
  }
  // Q, K, V (+ bias for GPT-NeoX, vsim.cpp:540-547); a long GPT-J prompt's Q and K (both RoPE
  // epilogues, no bias) as one launch of both tile grids
  if (rope_epi && gemm_pair_enabled(E, E)) {
    const long ev = prof_begin(m);
    RC(launch_gemm_q4_256_pair(w4_view(L.wq, E, E), w4_view(L.wk, E, E), X.a, N, m->Qb, kout, er, ek, s));
    prof_end(m, ev, "k_gemm_f16_256 (prompt)", 2.0 * E * E / QK * QBYTES);
    ++nk;
  } else {
    RC(mm(m, L.wq, E, E, m->cur1, N, m->xq1, m->xd1, true, gptj ? nullptr : L.bq, m->Qb, nk, X.a, nullptr, nullptr,
          nullptr, rope_epi ? &er : nullptr));
    RC(mm(m, L.wk, E, E, m->cur1, N, m->xq1, m->xd1, false, gptj ? nullptr : L.bk, kout, nk, X.a, nullptr, nullptr,
          nullptr, rope_epi ? &ek : nullptr));
  }
  RC(mm(m, L.wv, E, E, m->cur1, N, m->xq1, m->xd1, false, gptj ? nullptr : L.bv, vout, nk, X.a, nullptr, nullptr,
        nullptr, kv16_epi ? &ev : nullptr));
  // KV write + RoPE (vsim.cpp:553-580)
  if (!rope_epi) {
    RC(launch_rope_kv_write(gptj ? 1 : 0, m->Qb, m->Kb, m->Vb, kc, vc, d, H, N, n_past, m->hp.n_rot, m->rope_cs, s));
    ++nk;
  }
  // attention (vsim.cpp:583-616)
  const int nkv = n_past + N;
  const float scale = (float)(1.0f / std::sqrt((double)(float(E) / H)));
  // (head dim 256: the attention writes the out-projection's fp16 operand itself)
  const bool attn_q16 = attn16 && pf && attn_prefill_quantizes(d);
  if (attn16) {
    // fast-mode prompt: one-pass fp16 MFMA attention (attn_prefill.hip)
    RC(launch_attn_prefill_f16(m->Qb, kc, vc, d, H, N, n_past, scale, m->attn_in, s, m->pf_scratch, m->pf_bytes,
                               kv16_epi, attn_q16 ? X.b : nullptr));
    nk += 2;
  } else {
    RC(launch_kq(kc, E, m->Qb, E, d, H, nkv, N, m->kq, s, n_past)); ++nk;
    RC(launch_attn_softmax(m->kq, nkv, N, H, n_past, scale, s)); ++nk;
    RC(launch_kqv(vc, E, m->kq, d, H, nkv, N, m->attn_in, 1, s, n_past)); ++nk;
  }
  if (!attn_q16) RC(act16(m->attn_in, E, X.b, nullptr, false));
  RC(mm(m, L.wo, E, E, m->attn_in, N, m->xq2, m->xd2, true, gptj ? nullptr : L.bo, m->attn, nk, X.b));
  // feed-forward input
  const uint8_t *fxq = m->xq1;
  const float *fxd = m->xd1;
  bool fquant = false;
  const float *fx = m->cur1;
  if (!gptj) {
    if (m->hp.use_parallel_residual) {
      RC(norm(m->inpL, m->cur2, L.ln2_w, L.ln2_b, X.a));
    } else {
      // inpFF = cur + inpL ; norm ; affine  (vsim.cpp:631-649)
      VSIM_HIP(hipMemcpyAsync(m->cur2, m->attn, sizeof(float) * N * E, hipMemcpyDeviceToDevice, s));
      RC(launch_add_bias(m->cur2, m->inpL, N * E, 1, s)); ++nk;  // cur + inpL elementwise
      RC(norm(m->cur2, m->cur2, L.ln2_w, L.ln2_b, X.a));
    }
    fx = m->cur2;
    fxq = m->xq2;
    fxd = m->xd2;
    fquant = true;
  }
  // (the norms above wrote the prompt batch's fp16 operand already)
  bool gq = false;
  RC(mm(m, L.wfc, F, E, fx, N, (uint8_t *)fxq, (float *)fxd, fquant, nullptr, m->fch, nk, X.a, X.b, L.bfc, &gq));
  if (pf) {
    if (!gq) RC(act16(m->fch, F, X.b, L.bfc, true));  // bias + GELU + quantize, one pass
  } else {
    RC(launch_gelu(m->fch, m->fch, N * F, L.bfc, F, s)); ++nk;
  }
  // fc_out; a long prompt joins the residual in its epilogue (vsim.cpp:694-695 or 657)
  const bool serial = !gptj && !m->hp.use_parallel_residual;
  G2Epi ej;
  ej.res = m->inpL;
  ej.res_a = serial ? nullptr : m->attn;
  const bool join_epi = g2;
  bool joined = false;
  RC(mm(m, L.wproj, E, F, m->fch, N, m->xq3, m->xd3, true, L.bproj, join_epi ? m->inpL : m->ff, nk, X.b, nullptr,
        nullptr, &joined, join_epi ? &ej : nullptr));
  if (joined != join_epi) {
    set_error("prompt layer: residual epilogue not taken");
    return VSIM_EINVAL;
  }
  if (!joined) {
    RC(launch_add_residual(m->inpL, m->attn, m->ff, N * E, serial ? 1 : 0, s));
    ++nk;
  }
  return VSIM_OK;
}

// Fast-mode single-token step (fast_decode.hip): 3 launches per layer.  Same buffers and
// the same replayable form as enqueue_decode (token and n_past from device memory).
// Shapes the fast step handles: head dim a multiple of 32 up to 256, rotary pairs inside one
// 32-row tile (GPT-J pairs; GPT-NeoX rotate-half with n_rot <= 32), n_embd <= 8192.
// fc_out K splits: FD_SF, doubled until one split's activation slice fits the LDS staging
// (at most FD_MAXE values)
int fast_sf(const vsim_model *m) {
  int sf = FD_SF;
  while (sf < 8 && 4 * m->hp.n_embd / sf > FD_MAXE) sf *= 2;
  return sf;
}

bool fast_decode_ok(const vsim_model *m) {
  const int E = m->hp.n_embd, H = m->hp.n_head, d = E / H;
  const int nch = (m->n_ctx + FD_CHUNK - 1) / FD_CHUNK;
  return d % 32 == 0 && d <= 256 && E <= 8192 && E % 128 == 0 &&
         (m->arch == VSIM_ARCH_GPTJ || (m->arch == VSIM_ARCH_GPTNEOX && m->hp.use_parallel_residual == 1)) &&
         (m->arch == VSIM_ARCH_GPTJ || m->hp.n_rot <= 32) && 2 * H * nch <= 4096;
}

int enqueue_decode_fast(vsim_model *m, int &nk) {
  const int E = m->hp.n_embd, H = m->hp.n_head, d = E / H, F = 4 * E, V = m->hp.n_vocab;
  const bool gptj = m->arch == VSIM_ARCH_GPTJ;
  hipStream_t s = m->stream;
  DevTables tab;
  RC(tables_get(&tab));
  const int nbE = E / QK, nbF = F / QK;
  uint8_t *q1 = m->xq1, *q3 = m->xq3;
  float *d1 = (float *)(q1 + (size_t)nbE * 16), *d2 = (float *)(m->xq2 + (size_t)nbE * 16);
  float *d3 = (float *)(q3 + (size_t)nbF * 16);
  if (m->first) {
    RC(launch_get_rows(m->wte, E, V, m->tok_dev, 1, m->inpL, s));
    ++nk;
  }
  const float scale = (float)(1.0f / std::sqrt((double)(float(E) / H)));
  const int nchunk = (m->n_ctx + FD_CHUNK - 1) / FD_CHUNK;
  const double kv_bytes = 2.0 * ((double)m->prof_npast + 1) * E * sizeof(float);
  float *R[2] = {m->inpL, m->inpL2};
  int cur = 0;
  for (int il = m->l0; il < m->l1; ++il) {
    const LayerW &L = m->layers[il - m->l0];
    const size_t loff = (size_t)(il - m->l0) * m->n_ctx * E;
    // LayerNorm(s) -> Q4 activations in the GEMV's prologue (GPT-J: one LayerNorm feeds
    // attention and MLP), then {fc_in -> GELU -> quantize, Q, K, V}
    FastGemv P{};
    P.lnx = R[cur];
    P.lnw[0] = L.ln1_w;
    P.lnb[0] = L.ln1_b;
    P.lnw[1] = gptj ? L.ln1_w : L.ln2_w;
    P.lnb[1] = gptj ? L.ln1_b : L.ln2_b;
    P.xq[0] = q1;
    P.xd[0] = d1;
    P.xq[1] = gptj ? q1 : m->xq2;
    P.xd[1] = gptj ? d1 : d2;
    P.nj = 4;
    P.j[0] = FastJob{w4_view(L.wfc, F, E), L.bfc, nullptr, FE_GELU_Q, 1};
    P.j[1] = FastJob{w4_view(L.wq, E, E), gptj ? nullptr : L.bq, m->Qb, FE_ROPE_Q, 0};
    P.j[2] = FastJob{w4_view(L.wk, E, E), gptj ? nullptr : L.bk, m->kcache + loff, FE_ROPE_K, 0};
    P.j[3] = FastJob{w4_view(L.wv, E, E), gptj ? nullptr : L.bv, m->vcache + loff, FE_V, 0};
    P.gelu_tab = tab.gelu_f16;
    P.clear = m->tail_done;  // K2's per-head counters (tail_done[4h])
    P.nclear = 4 * H;
    P.oq_qs = q3;
    P.oq_d = d3;
    P.npast = m->npast_dev;
    P.cs = m->rope_cs;
    P.d = d;
    P.n_rot = m->hp.n_rot;
    P.style = gptj ? 1 : 0;
    long ev = prof_begin(m);
    RC(launch_fast_gemv(P, E, s));
    prof_end(m, ev, "k_fast_gemv (fc_in, Q, K, V)", w4_algo_bytes(P.j[0].w) + 3 * w4_algo_bytes(P.j[1].w));
    ++nk;
    // fc_out split over K | attention chunks
    FastTail T{};
    T.wf = w4_view(L.wproj, E, F);
    T.xf_qs = q3;
    T.xf_d = d3;
    T.ffp = m->fast_ffp;
    T.sf = fast_sf(m);
    T.q = m->Qb;
    T.kc = m->kcache + loff;
    T.vc = m->vcache + loff;
    T.npast = m->npast_dev;
    T.d = d;
    T.H = H;
    T.nchunk = nchunk;
    T.scale = scale;
    T.part = m->fast_part;
    T.hcnt = m->tail_done;
    T.oq_qs = m->xqa;
    T.oq_d = (float *)(m->xqa + (size_t)(E / QK) * 16);
    // attention merge + out-projection + residual join into the other buffer
    FastOproj O{};
    O.w = w4_view(L.wo, E, E);
    O.xq = T.oq_qs;
    O.xd = T.oq_d;
    O.d = d;
    O.bo = gptj ? nullptr : L.bo;
    O.ffp = m->fast_ffp;
    O.sf = fast_sf(m);
    O.bproj = L.bproj;
    O.x = R[cur];
    O.out = R[cur ^ 1];
    ev = prof_begin(m);
    RC(launch_fast_tail(T, s));
    prof_end(m, ev, "k_fast_tail (fc_out + attention)", w4_algo_bytes(T.wf) + kv_bytes);
    ++nk;
    ev = prof_begin(m);
    RC(launch_fast_oproj_join(O, s));
    prof_end(m, ev, "k_fast_oproj_join", w4_algo_bytes(O.w));
    ++nk;
    cur ^= 1;
  }
  if (m->last) {
    FastGemv P{};
    P.lnx = R[cur];
    P.lnw[0] = P.lnw[1] = m->lnf_w;
    P.lnb[0] = P.lnb[1] = m->lnf_b;
    P.xq[0] = P.xq[1] = q1;
    P.xd[0] = P.xd[1] = d1;
    P.nj = 1;
    P.j[0] = FastJob{w4_view(m->lmh, V, E), gptj ? m->lmh_b : nullptr, m->logits, FE_STORE, 0};
    const long ev = prof_begin(m);
    RC(launch_fast_gemv(P, E, s));
    prof_end(m, ev, "k_fast_gemv (lm_head)", w4_algo_bytes(P.j[0].w));
    ++nk;
  }
  m->resid_final = R[cur];
  return VSIM_OK;
}

// Exact mode: the single-token decode step as fused launches per layer (layer.hip,
// gemv_chain.hip).  Reads the token from tok_dev and n_past from npast_dev, so the enqueued
// sequence is replayable (hipGraph).
//   1. k_ln_quant: (join of the previous layer +) input LayerNorm (+ post_attention
//      LayerNorm for GPT-NeoX), quantized -- since r06 only for the first layer of the step
//      (or when the previous tail could not run it, TailLn)
//   2. k_gemv_solo: {fc_in (+ bias, GELU, requantize), Q, K, V}
//   3. k_layer_tail: fc_out beside the attention heads and the out-projection, then the join
//      and the next layer's LayerNorm(s) (or the final norm) quantized (TailLn; without it the
//      biases join in the next step 1)
// fc_out's K = 4E chain (vsim.cpp:680-690) is the layer's longest dependency, so the
// attention branch fills the CUs beside it instead of running before it.
// Serial-residual graphs (BLOOM; GPT-NeoX with use_parallel_residual = 0, vsim.cpp:626-658)
// feed the MLP from the attention's residual, so nothing runs beside fc_out; 6 launches:
//   1. k_ln_quant (join of the previous layer's MLP output +) input LayerNorm
//   2. GEMV {Q, K, V} (+ bias)
//   3. k_layer_tail without fc_out: the heads (BLOOM: ALiBi) and the out-projection
//   4. k_ln_quant: attn + bias + x joined, post-attention LayerNorm (BLOOM keeps the joined
//      row as the residual, inpFF; GPT-NeoX's serial graph adds the MLP to the old one)
//   5. GEMV fc_in (+ bias, GELU, requantize)       6. GEMV fc_out
int enqueue_decode(vsim_model *m, int &nk) {
  if (m->mode == VSIM_MODE_FAST && fast_decode_ok(m)) return enqueue_decode_fast(m, nk);
  const int E = m->hp.n_embd, H = m->hp.n_head, d = E / H, F = 4 * E, V = m->hp.n_vocab;
  const bool gptj = m->arch == VSIM_ARCH_GPTJ, bloom = m->arch == VSIM_ARCH_BLOOM;
  const bool serial = bloom || (!gptj && !m->hp.use_parallel_residual);
  hipStream_t s = m->stream;
  DevTables tab;
  RC(tables_get(&tab));
  const int nbE = E / QK, nbF = F / QK;
  uint8_t *q1 = m->xq1, *q2 = m->xq2, *q3 = m->xq3, *qa = m->xqa;
  float *d1 = (float *)(q1 + (size_t)nbE * 16), *d2 = (float *)(q2 + (size_t)nbE * 16);
  float *d3 = (float *)(q3 + (size_t)nbF * 16), *da = (float *)(qa + (size_t)nbE * 16);
  if (m->first && bloom) {  // word embeddings + word_embeddings_layernorm
    RC(launch_get_rows(m->wte, E, V, m->tok_dev, 1, m->cur1, s));
    RC(launch_norm(m->cur1, m->inpL, E, 1, m->emb_w, m->emb_b, s));
    nk += 2;
  } else if (m->first) {
    RC(launch_get_rows(m->wte, E, V, m->tok_dev, 1, m->inpL, s));
    ++nk;
  }
  const float scale = (float)(1.0f / std::sqrt((double)(float(E) / H)));
  // algorithmic bytes of the profiled launches: KV rows read (P + 1) and
  // written by the attention, rows of E floats read / written by the LayerNorm step
  const double kv_bytes = 2.0 * ((double)m->prof_npast + 1) * E * sizeof(float);
  // reads: the row (+ the four join vectors), each norm's affine; writes: the joined row, each
  // norm's factors xd (E floats) and Q4 row (0.625 B per value)
  auto ln_bytes = [&](int nnorm, bool join) {
    return 4.0 * E * (1 + (join ? 5 : 0) + 3 * nnorm) + 0.625 * E * nnorm;
  };
  // The residual join of layer l (inpL += attn + ff, vsim.cpp:694-695) runs inside layer
  // l+1's LayerNorm kernel (or the final norm); the joined row goes to the other of the two
  // residual buffers, so both norm workgroups of GPT-NeoX can read the old one.
  float *R[2] = {m->inpL, m->inpL2};
  int cur = 0;
  bool pending = false, ln_done = false;
  const float *pend_a = nullptr, *pend_ab = nullptr, *pend_fb = nullptr;
  auto join_into = [&](LnQuantJob &j, bool write) {
    j.ja = pend_a;
    j.jab = pend_ab;
    j.jf = m->ff;
    j.jfb = pend_fb;
    j.jout = write ? R[cur ^ 1] : nullptr;
  };
  auto job = [&](GemvBatch &Bt, int i, void *W, int M, int K, const float *xd, const uint8_t *xq, const float *xdd,
                 const float *bias, float *y) {
    GemvJob &J = Bt.j[i];
    J.w = w4_view(W, M, K);
    J.xd = xd;
    J.xqs = xq;
    J.xdd = xdd;
    J.bias = bias;
    J.y = y;
    J.epi = EPI_STORE;
  };
  // the attention heads fuse into k_layer_tail while their LDS (scores over n_ctx) fits it
  const bool tail = m->mode == VSIM_MODE_EXACT && (size_t)attn_lds_floats(d, m->n_ctx) * sizeof(float) <= 75264;
  // the next layer's LayerNorm inside the tail (TailLn; parallel-residual graphs: the tail is
  // where both branches of the layer end)
  const bool lnt_ok = tail && !serial && m->l1 <= 255 && tail_ln_ok(E);
  auto attn_job = [&](size_t loff) {
    AttnJob A{};
    A.q = m->Qb;
    A.k = m->Kb;
    A.v = m->Vb;
    A.kc = m->kcache + loff;
    A.vc = m->vcache + loff;
    A.npast = m->npast_dev;
    A.cs = m->rope_cs;
    A.etab = tab.exp_f16;
    A.d = d;
    A.H = H;
    A.n_rot = bloom ? 0 : m->hp.n_rot;
    A.style = gptj ? 1 : 0;
    A.n_ctx = m->n_ctx;
    // each head over two workgroups (its KQV columns halved; the scores computed by both) in the
    // parallel-residual fused tail, where it was measured: r05, 248-token GPT-J lines 608.9 / 612.5
    // vs 606.9 / 610.8 tok/s unsplit, 602.6 / 601.3 at four (profiles/r05_tail_variants_ab.txt).
    // The largest split <= ATT_SPLIT whose column parts are whole 32-blocks; the serial graphs'
    // heads and the standalone k_attn_decode stay one workgroup per head.  (A/B builds:
    // tools/build_variant.sh NAME model.cpp 's/ATT_SPLIT = 2/ATT_SPLIT = 1/'.)
    constexpr int ATT_SPLIT = 2;
    A.nsplit = 1;
    for (int sp = tail && !serial ? ATT_SPLIT : 1; sp > 1; --sp)
      if (d % sp == 0 && (d / sp) % QK == 0) {
        A.nsplit = sp;
        break;
      }
    A.scale = m->attn_scale != 0.0f ? m->attn_scale : scale;
    A.kqv_nth = m->kqv_nth;
    A.alibi = bloom ? m->alibi : nullptr;
    A.oq_qs = qa;
    A.oq_d = da;
    A.oxd = m->xda;
    A.out = nullptr;
    return A;
  };
  auto gemv = [&](const GemvBatch &Bt, const char *what, double bytes) -> int {
    const long ev = prof_begin(m);
    RC(launch_gemv_epi(Bt, m->mode, s));
    if (ev >= 0)
      prof_end(m, ev, std::string(m->mode != VSIM_MODE_EXACT ? "k_gemv_fast_epi" : gemv_chain_solo(Bt) ? "k_gemv_solo"
                                                                                                  : "k_gemv_chain32") +
                          " (" + what + ")", bytes);
    ++nk;
    return VSIM_OK;
  };
  for (int il = m->l0; il < m->l1; ++il) {
    const LayerW &L = m->layers[il - m->l0];
    const size_t loff = (size_t)(il - m->l0) * m->n_ctx * E;
    if (serial) {
      // 1. (join +) input LayerNorm + quantize
      LnQuantJob j1{R[cur], L.ln1_w, L.ln1_b, q1, d1, m->xd1};
      if (pending) join_into(j1, true);
      if (tail && il == m->l0) j1.ep = m->lnt_ep;  // the step's epoch (the tail's flags)
      long ev = prof_begin(m);
      RC(launch_ln_quant(j1, nullptr, E, s));
      prof_end(m, ev, "k_ln_quant", ln_bytes(1, pending));
      ++nk;
      if (pending) cur ^= 1;
      // 2. Q, K, V (+ bias; BLOOM: the fused query_key_value's row blocks)
      GemvBatch B{};
      B.nj = 3;
      job(B, 0, L.wq, E, E, m->xd1, q1, d1, L.bq, m->Qb);
      job(B, 1, L.wk, E, E, m->xd1, q1, d1, L.bk, m->Kb);
      job(B, 2, L.wv, E, E, m->xd1, q1, d1, L.bv, m->Vb);
      RC(gemv(B, "Q, K, V", 3 * w4_algo_bytes(B.j[0].w)));
      // 3. heads + out-projection (its bias joins in step 4)
      const AttnJob A = attn_job(loff);
      GemvBatch Bo{};
      Bo.nj = 1;
      job(Bo, 0, L.wo, E, E, m->xda, qa, da, nullptr, m->attn);
      if (tail) {
        GemvBatch none{};
        ev = prof_begin(m);
        RC(launch_layer_tail(none, Bo, A, TailSync{m->tail_hflag, m->lnt_ep, il}, m->n_ctx, s));
        prof_end(m, ev, "k_layer_tail (attention + out-proj)", w4_algo_bytes(Bo.j[0].w) + kv_bytes);
        ++nk;
      } else {
        ev = prof_begin(m);
        RC(launch_attn_decode(A, m->n_ctx, s));
        prof_end(m, ev, "k_attn_decode", kv_bytes);
        ++nk;
        RC(gemv(Bo, "out-proj", w4_algo_bytes(Bo.j[0].w)));
      }
      // 4. inpFF = (attn + b_o) + x, post-attention LayerNorm + quantize
      LnQuantJob j2{R[cur], L.ln2_w, L.ln2_b, q2, d2, m->xd2};
      j2.ja = m->attn;
      j2.jab = L.bo;
      j2.jout = bloom ? R[cur ^ 1] : nullptr;
      ev = prof_begin(m);
      RC(launch_ln_quant(j2, nullptr, E, s));
      prof_end(m, ev, "k_ln_quant", ln_bytes(1, true));
      ++nk;
      if (bloom) cur ^= 1;
      // 5. fc_in (+ bias, GELU, requantize)   6. fc_out (its bias joins in the next step 1)
      GemvBatch Bi{};
      Bi.nj = 1;
      job(Bi, 0, L.wfc, F, E, m->xd2, q2, d2, L.bfc, nullptr);
      Bi.j[0].epi = EPI_GELU_Q;
      Bi.j[0].gelu_tab = tab.gelu_f16;
      Bi.j[0].oq_qs = q3;
      Bi.j[0].oq_d = d3;
      Bi.j[0].oxd = m->xd3;
      RC(gemv(Bi, "fc_in", w4_algo_bytes(Bi.j[0].w)));
      GemvBatch Bf{};
      Bf.nj = 1;
      job(Bf, 0, L.wproj, E, F, m->xd3, q3, d3, nullptr, m->ff);
      RC(gemv(Bf, "fc_out", w4_algo_bytes(Bf.j[0].w)));
      pending = true;
      pend_a = nullptr;
      pend_ab = nullptr;
      pend_fb = L.bproj;
      continue;
    }
    // 1. (join +) LayerNorm(s) + quantize, unless the previous layer's tail ran them (TailLn)
    const TailSync sy{m->tail_hflag, m->lnt_ep, il};  // the heads' flags of this layer's tail
    long ev = -1;
    if (!ln_done) {
      LnQuantJob j1{R[cur], L.ln1_w, L.ln1_b, q1, d1, m->xd1};
      LnQuantJob j2{R[cur], L.ln2_w, L.ln2_b, q2, d2, m->xd2};
      if (pending) {
        join_into(j1, true);
        join_into(j2, false);
      }
      if (tail && il == m->l0) j1.ep = m->lnt_ep;  // the step's first norm advances the epoch
      ev = prof_begin(m);
      RC(launch_ln_quant(j1, gptj ? nullptr : &j2, E, s));
      prof_end(m, ev, "k_ln_quant", ln_bytes(gptj ? 1 : 2, pending));
      ++nk;
      if (pending) cur ^= 1;
    }
    ln_done = false;
    // 2. {fc_in (+bias, GELU, requantize), Q, K, V}
    GemvBatch B{};
    B.nj = 4;
    job(B, 0, L.wfc, F, E, gptj ? m->xd1 : m->xd2, gptj ? q1 : q2, gptj ? d1 : d2, L.bfc, nullptr);
    B.j[0].epi = EPI_GELU_Q;
    B.j[0].gelu_tab = tab.gelu_f16;
    B.j[0].oq_qs = q3;
    B.j[0].oq_d = d3;
    B.j[0].oxd = m->xd3;
    job(B, 1, L.wq, E, E, m->xd1, q1, d1, gptj ? nullptr : L.bq, m->Qb);
    job(B, 2, L.wk, E, E, m->xd1, q1, d1, gptj ? nullptr : L.bk, m->Kb);
    job(B, 3, L.wv, E, E, m->xd1, q1, d1, gptj ? nullptr : L.bv, m->Vb);
    ev = prof_begin(m);
    RC(launch_gemv_epi(B, m->mode, s));
    prof_end(m, ev, m->mode == VSIM_MODE_EXACT ? "k_gemv_solo (fc_in, Q, K, V)" : "k_gemv_fast_epi (fc_in, Q, K, V)",
             w4_algo_bytes(B.j[0].w) + 3 * w4_algo_bytes(B.j[1].w));
    ++nk;
    // 3. attention for the new token (attn.hpp), fc_out and the out-projection
    const AttnJob A = attn_job(loff);
    GemvBatch Bf{}, Bo{};
    Bf.nj = 1;
    job(Bf, 0, L.wproj, E, F, m->xd3, q3, d3, nullptr, m->ff);
    Bo.nj = 1;
    job(Bo, 0, L.wo, E, E, m->xda, qa, da, nullptr, m->attn);
    // the next LayerNorm inside this tail: every layer but a non-last stage's last one
    const bool lnt = tail && lnt_ok && (il + 1 < m->l1 || m->last);
    if (lnt) {
      TailLn N{};
      N.x = R[cur];
      N.ab = gptj ? nullptr : L.bo;
      N.fb = L.bproj;
      N.jout = R[cur ^ 1];
      if (il + 1 < m->l1) {  // the next layer's input norm(s)
        const LayerW &Ln = m->layers[il + 1 - m->l0];
        N.w1 = Ln.ln1_w;
        N.b1 = Ln.ln1_b;
        if (!gptj) {
          N.w2 = Ln.ln2_w;
          N.b2 = Ln.ln2_b;
          N.q2 = q2;
          N.d2 = d2;
          N.xd2 = m->xd2;
        }
      } else {  // the final norm, for the lm_head
        N.w1 = m->lnf_w;
        N.b1 = m->lnf_b;
      }
      N.q1 = q1;
      N.d1 = d1;
      N.xd1 = m->xd1;
      N.og = m->lnt_og;
      N.jg = m->lnt_jg;
      N.rec = m->lnt_rec;
      N.ep = m->lnt_ep;
      N.stats = dev_stats();
      N.il = il;
      ev = prof_begin(m);
      RC(launch_layer_tail(Bf, Bo, A, sy, m->n_ctx, s, &N));
      prof_end(m, ev, "k_layer_tail (fc_out + attention + out-proj + join + LayerNorm)",
               w4_algo_bytes(Bf.j[0].w) + w4_algo_bytes(Bo.j[0].w) + kv_bytes + ln_bytes(N.w2 ? 2 : 1, true));
      ++nk;
      cur ^= 1;
      ln_done = true;
      pending = false;
      continue;
    }
    if (tail) {
      ev = prof_begin(m);
      RC(launch_layer_tail(Bf, Bo, A, sy, m->n_ctx, s));
      prof_end(m, ev, "k_layer_tail (fc_out + attention + out-proj)",
               w4_algo_bytes(Bf.j[0].w) + w4_algo_bytes(Bo.j[0].w) + kv_bytes);
      ++nk;
    } else {
      ev = prof_begin(m);
      RC(launch_attn_decode(A, m->n_ctx, s));
      prof_end(m, ev, "k_attn_decode", kv_bytes);
      ++nk;
      Bf.j[1] = Bo.j[0];
      Bf.nj = 2;
      ev = prof_begin(m);
      RC(launch_gemv_epi(Bf, m->mode, s));
      prof_end(m, ev, m->mode == VSIM_MODE_EXACT ? "k_gemv_chain32 (fc_out, out-proj)" : "k_gemv_fast_epi (fc_out, out-proj)",
               w4_algo_bytes(Bf.j[0].w) + w4_algo_bytes(Bf.j[1].w));
      ++nk;
    }
    pending = true;
    pend_a = m->attn;
    pend_ab = gptj ? nullptr : L.bo;
    pend_fb = L.bproj;
  }
  if (m->last) {
    if (!ln_done) {
      LnQuantJob jf{R[cur], m->lnf_w, m->lnf_b, q1, d1, m->xd1};
      if (pending) join_into(jf, true);
      long ev = prof_begin(m);
      RC(launch_ln_quant(jf, nullptr, E, s));
      prof_end(m, ev, "k_ln_quant", ln_bytes(1, pending));
      ++nk;
      if (pending) cur ^= 1;
    }
    GemvBatch B{};
    B.nj = 1;
    job(B, 0, m->lmh, V, E, m->xd1, q1, d1, gptj ? m->lmh_b : nullptr, m->logits);
    const long ev = prof_begin(m);
    RC(launch_gemv_epi(B, m->mode, s));
    prof_end(m, ev, m->mode == VSIM_MODE_EXACT ? "k_gemv_solo (lm_head)" : "k_gemv_fast_epi (lm_head)",
             w4_algo_bytes(B.j[0].w));
    ++nk;
  } else if (pending) {
    RC(launch_residual_join(R[cur], pend_a, pend_ab, m->ff, pend_fb, R[cur ^ 1], E, s));
    ++nk;
    cur ^= 1;
  }
  m->resid_final = R[cur];
  return VSIM_OK;
}

// every graph has a single-token step (the serial-residual ones with 6 launches per layer)
bool fused_ok(const vsim_model *, int N) { return N == 1; }

thread_local std::string t_err;

}  // namespace

namespace vsim {
void set_error(const std::string &msg) { t_err = msg; }
int hip_fail(hipError_t e, const char *what) {
  t_err = std::string(what) + ": " + hipGetErrorString(e);
  return VSIM_EHIP;
}
}  // namespace vsim

extern "C" {

const char *vsim_last_error(void) { return t_err.c_str(); }

int vsim_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

size_t vsim_q4_bytes(int rows, int k) { return w4_bytes(rows, k); }

}  // extern "C"

namespace vsim {
// vsim_model_create, or (borrow != null) a whole-model GPT-NeoX / GPT-J executor whose weight
// slots point at device buffers the caller owns (ggml tensor name -> W4T32 / F32 device
// pointer, every slot must be there) and whose KV cache is kc / vc ([layer][n_ctx][E] f32):
// the graph executor's fast path, graph.cpp.
int model_create_impl(int arch, const vsim_hparams *hp, int n_ctx, int device, int layer_begin, int layer_end,
                      const std::map<std::string, void *> *borrow, float *kc, float *vc, vsim_model **out) {
  if (!hp || !out) { set_error("model_create: null argument"); return VSIM_EINVAL; }
  if (arch != VSIM_ARCH_GPTNEOX && arch != VSIM_ARCH_GPTJ && arch != VSIM_ARCH_BLOOM) {
    set_error("model_create: unknown arch");
    return VSIM_EINVAL;
  }
  if (hp->n_embd % hp->n_head || hp->n_embd % 128 || hp->n_rot > hp->n_embd / hp->n_head || hp->n_rot % 2 ||
      n_ctx <= 0) {
    set_error("model_create: unsupported hparams (n_embd % 128, n_rot <= head dim, even n_rot)");
    return VSIM_EINVAL;
  }
  if (layer_end < 0) layer_end = hp->n_layer;
  if (layer_begin < 0 || layer_begin >= layer_end || layer_end > hp->n_layer) {
    set_error("model_create: bad layer range");
    return VSIM_EINVAL;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) { set_error("model_create: no such device"); return VSIM_ENODEV; }
  VSIM_HIP(hipSetDevice(device));
  auto *m = new vsim_model();
  m->arch = arch;
  m->hp = *hp;
  m->n_ctx = n_ctx;
  m->device = device;
  m->l0 = layer_begin;
  m->l1 = layer_end;
  m->first = layer_begin == 0;
  m->last = layer_end == hp->n_layer;
  auto fail = [&](int rc) { vsim_model_free(m); return rc; };
  if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(hip_fail(hipErrorUnknown, "stream"));
  std::vector<std::pair<std::string, Slot>> plan;
  plan_slots(m, plan);
  if (borrow) {
    if (arch == VSIM_ARCH_BLOOM || !kc || !vc) { set_error("model_create: borrowed weights: GPT-NeoX / GPT-J only"); return fail(VSIM_EINVAL); }
    for (auto &ps : plan) {
      auto it = borrow->find(ps.first);
      if (it == borrow->end() || !it->second) {
        set_error("model_create: borrowed weights: no device buffer for " + ps.first);
        return fail(VSIM_EINVAL);
      }
      ps.second.ptr = it->second;
      ps.second.loaded = true;
      m->slots[ps.first] = ps.second;
    }
    m->borrowed = true;
    m->kcache = kc;
    m->vcache = vc;
    bind_pointers(m);
  }
  size_t tot = 0;
  for (auto &ps : plan) tot += (slot_dev_bytes(ps.second) + 255) & ~(size_t)255;
  const size_t E = hp->n_embd, nl = layer_end - layer_begin;
  if (!borrow) {
    // + FD_PAD: the fast GEMV streams whole 16-block batches and zeroes the scales of slots past
    // a wave's range, so it may read up to 8 KB past a tensor (fast_decode.hip TileStream)
    if (hipMalloc((void **)&m->warena, tot + FD_PAD) != hipSuccess) { set_error("model_create: weight alloc failed"); return fail(VSIM_ENOMEM); }
    m->wbytes = tot;
    size_t off = 0;
    for (auto &ps : plan) {
      ps.second.ptr = m->warena + off;
      off += (slot_dev_bytes(ps.second) + 255) & ~(size_t)255;
      m->slots[ps.first] = ps.second;
    }
    bind_pointers(m);
    if (hipMalloc((void **)&m->kcache, nl * n_ctx * E * sizeof(float)) != hipSuccess ||
        hipMalloc((void **)&m->vcache, nl * n_ctx * E * sizeof(float)) != hipSuccess) {
      set_error("model_create: KV cache alloc failed");
      return fail(VSIM_ENOMEM);
    }
    (void)hipMemset(m->kcache, 0, nl * n_ctx * E * sizeof(float));
    (void)hipMemset(m->vcache, 0, nl * n_ctx * E * sizeof(float));
  } else {
    m->wbytes = tot;
  }
  const int half = hp->n_rot / 2 > 0 ? hp->n_rot / 2 : 1;
  std::vector<double2> cs((size_t)n_ctx * half);
  if (hp->n_rot > 0) rope_table_host(cs.data(), n_ctx, hp->n_rot);
  if (hipMalloc((void **)&m->rope_cs, cs.size() * sizeof(double2)) != hipSuccess) return fail(VSIM_ENOMEM);
  if (hipMemcpy(m->rope_cs, cs.data(), cs.size() * sizeof(double2), hipMemcpyHostToDevice) != hipSuccess)
    return fail(hip_fail(hipErrorUnknown, "rope table upload"));
  if (arch == VSIM_ARCH_BLOOM) {
    m->hp.n_rot = 0;
    m->hp.use_parallel_residual = 0;
    std::vector<float> sl(hp->n_head);
    alibi_slopes_host(sl.data(), hp->n_head);
    if (hipMalloc((void **)&m->alibi, sl.size() * sizeof(float)) != hipSuccess) return fail(VSIM_ENOMEM);
    if (hipMemcpy(m->alibi, sl.data(), sl.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
      return fail(hip_fail(hipErrorUnknown, "alibi slopes upload"));
  }
  DevTables t;
  if (int rc = tables_get(&t)) return fail(rc);
  if (hipMalloc((void **)&m->err_dev, sizeof(unsigned)) != hipSuccess || hipMemset(m->err_dev, 0, sizeof(unsigned)) != hipSuccess ||
      hipHostMalloc((void **)&m->err_host, sizeof(unsigned), hipHostMallocDefault) != hipSuccess)
    return fail(VSIM_ENOMEM);
  *m->err_host = 0;
  if (int rc = ensure_scratch(m, 16)) return fail(rc);
  *out = m;
  return VSIM_OK;
}

// The borrowed model's per-call settings: the reference pool's KQV grouping (cgraph->n_threads)
// and the graph's own attention scale; a change drops the captured decode graphs.
int model_set_attn(vsim_model *m, int kqv_nth, float scale) {
  if (kqv_nth < 1) kqv_nth = 1;
  if (m->kqv_nth == kqv_nth && m->attn_scale == scale) return VSIM_OK;
  VSIM_HIP(hipStreamSynchronize(m->stream));
  m->kqv_nth = kqv_nth;
  m->attn_scale = scale;
  m->graph_mode = m->graph_am_mode = m->graph_gen_mode = m->graph_st_mode = -1;  // recapture on next use
  return VSIM_OK;
}
}  // namespace vsim

extern "C" {

int vsim_model_create(int arch, const vsim_hparams *hp, int n_ctx, int device, int layer_begin, int layer_end,
                      vsim_model **out) {
  return model_create_impl(arch, hp, n_ctx, device, layer_begin, layer_end, nullptr, nullptr, nullptr, out);
}

void vsim_model_free(vsim_model *m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  if (m->stream) (void)hipStreamSynchronize(m->stream);
  if (m->alibi) (void)hipFree(m->alibi);
  free_scratch(m);
  if (m->warena) (void)hipFree(m->warena);
  if (m->kcache && !m->borrowed) (void)hipFree(m->kcache);
  if (m->vcache && !m->borrowed) (void)hipFree(m->vcache);
  if (m->rope_cs) (void)hipFree(m->rope_cs);
  if (m->err_dev) (void)hipFree(m->err_dev);
  if (m->err_host) (void)hipHostFree(m->err_host);
  if (m->stream) (void)gemm_release_stream(m->stream);  // the prompt GEMM's stream-K workspace
  if (m->stream) (void)hipStreamDestroy(m->stream);
  for (hipEvent_t e : m->prof_events) (void)hipEventDestroy(e);
  delete m;
}

int vsim_model_set_tensor(vsim_model *m, const char *name, const void *host, size_t nbytes) {
  if (m->borrowed) { set_error("set_tensor: the weights belong to the graph executor"); return VSIM_EINVAL; }
  {  // BLOOM's fused query_key_value weight: three [E][E] row blocks, q | k | v
    const std::string n(name), suf = "attention.query_key_value.weight";
    if (m->arch == VSIM_ARCH_BLOOM && n.size() >= suf.size() && n.compare(n.size() - suf.size(), suf.size(), suf) == 0) {
      const char *parts[3] = {"/q", "/k", "/v"};
      if (nbytes % 3 != 0) { set_error("set_tensor: fused qkv size"); return VSIM_EINVAL; }
      for (int i = 0; i < 3; ++i)
        RC(vsim_model_set_tensor(m, (n + parts[i]).c_str(), (const uint8_t *)host + i * (nbytes / 3), nbytes / 3));
      return VSIM_OK;
    }
  }
  auto it = m->slots.find(name);
  if (it == m->slots.end()) { set_error(std::string("set_tensor: unknown tensor ") + name); return VSIM_EINVAL; }
  Slot &s = it->second;
  if (nbytes != slot_bytes(s)) { set_error(std::string("set_tensor: wrong size for ") + name); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  if (s.kind == KF32) {
    VSIM_HIP(hipMemcpy(s.ptr, host, nbytes, hipMemcpyHostToDevice));
  } else {
    void *stage = nullptr;
    VSIM_HIP(hipMalloc(&stage, nbytes));
    hipError_t e = hipMemcpy(stage, host, nbytes, hipMemcpyHostToDevice);
    int rc = e == hipSuccess ? launch_q4_repack(stage, s.ptr, s.rows, s.k, m->stream) : hip_fail(e, "upload");
    if (rc == 0) rc = hipStreamSynchronize(m->stream) == hipSuccess ? 0 : VSIM_EHIP;
    (void)hipFree(stage);
    if (rc) return rc;
  }
  s.loaded = true;
  return VSIM_OK;
}

int vsim_model_get_tensor(vsim_model *m, const char *name, void *host, size_t nbytes) {
  if (!m || !name || !host) { set_error("get_tensor: null argument"); return VSIM_EINVAL; }
  {  // BLOOM's fused query_key_value weight: the three row blocks back to back
    const std::string n(name), suf = "attention.query_key_value.weight";
    if (m->arch == VSIM_ARCH_BLOOM && n.size() >= suf.size() && n.compare(n.size() - suf.size(), suf.size(), suf) == 0) {
      const char *parts[3] = {"/q", "/k", "/v"};
      if (nbytes % 3 != 0) { set_error("get_tensor: fused qkv size"); return VSIM_EINVAL; }
      for (int i = 0; i < 3; ++i)
        RC(vsim_model_get_tensor(m, (n + parts[i]).c_str(), (uint8_t *)host + i * (nbytes / 3), nbytes / 3));
      return VSIM_OK;
    }
  }
  auto it = m->slots.find(name);
  if (it == m->slots.end()) { set_error(std::string("get_tensor: unknown tensor ") + name); return VSIM_EINVAL; }
  const Slot &s = it->second;
  if (nbytes != slot_bytes(s)) { set_error(std::string("get_tensor: wrong size for ") + name); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  VSIM_HIP(hipStreamSynchronize(m->stream));
  if (s.kind == KF32) {
    VSIM_HIP(hipMemcpy(host, s.ptr, nbytes, hipMemcpyDeviceToHost));
    return VSIM_OK;
  }
  void *stage = nullptr;
  VSIM_HIP(hipMalloc(&stage, nbytes));
  int rc = launch_q4_unpack(s.ptr, stage, s.rows, s.k, m->stream);
  if (rc == 0 && hipStreamSynchronize(m->stream) != hipSuccess) rc = hip_fail(hipErrorUnknown, "unpack");
  if (rc == 0 && hipMemcpy(host, stage, nbytes, hipMemcpyDeviceToHost) != hipSuccess) rc = hip_fail(hipErrorUnknown, "download");
  (void)hipFree(stage);
  return rc;
}

int vsim_model_randomize(vsim_model *m, uint64_t seed, float stddev) {
  if (m->borrowed) { set_error("randomize: the weights belong to the graph executor"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  uint64_t id = 0;
  for (auto &kv : m->slots) {
    Slot &s = kv.second;
    const uint64_t sd = seed * 0x9E3779B97F4A7C15ull + (++id) * 0xD1B54A32D192ED03ull;
    const bool gain = kv.first.find("norm.weight") != std::string::npos || kv.first.find("ln_") != std::string::npos
                          ? kv.first.find(".weight") != std::string::npos
                          : false;
    if (s.kind == KQ4)
      RC(launch_randn_q4(s.ptr, s.rows, s.k, sd, stddev, m->stream));
    else
      RC(launch_randn_f32((float *)s.ptr, s.k, sd, stddev, gain ? 1.0f : 0.0f, m->stream));
    s.loaded = true;
  }
  VSIM_HIP(hipStreamSynchronize(m->stream));
  return VSIM_OK;
}

// The ggml model file (vsim.cpp:108-458; convert_gptj_to_ggml.py; convert_bloom_to_ggml.py):
// header, vocab, then tensor records {n_dims, name_len, ftype, ne[n_dims], name, data} to EOF.
// Checked as gptneox_model_load checks them (vsim.cpp:398-438): every header field read, every
// record's name known, its element count and its shape those of the tensor the graph expects
// (ne[0] = the inner dimension K, ne[1] = rows), its type the expected one, no tensor missing.
// F32 / F16 weight files (f16 = 0 / 1, vsim.cpp:179-190) take the reference's F32 / F16 mul_mat,
// which is not this library's path: they are refused with that reason.
int vsim_model_load_file(const char *path, int arch, int n_ctx, int device, int layer_begin, int layer_end,
                         vsim_model **out) {
  if (!path || !out) { set_error("load: null argument"); return VSIM_EINVAL; }
  std::ifstream f(path, std::ios::binary);
  if (!f) { set_error(std::string("load: cannot open ") + path); return VSIM_EFILE; }
  auto rd = [&](void *p, size_t n) { f.read((char *)p, n); return (size_t)f.gcount() == n; };
  auto bad = [](const std::string &why) { set_error("load: " + why); return VSIM_EFILE; };
  uint32_t magic = 0;
  if (!rd(&magic, 4) || magic != 0x67676d6c) return bad("bad magic");
  vsim_hparams hp{};
  int32_t ftype = 0;
  bool ok = rd(&hp.n_vocab, 4) && rd(&hp.n_embd, 4);
  if (arch == VSIM_ARCH_BLOOM) {  // convert_bloom_to_ggml.py:79-85: ..., multiple_of, n_head, n_layer, ftype
    int32_t n_mult = 0;
    ok = ok && rd(&n_mult, 4) && rd(&hp.n_head, 4) && rd(&hp.n_layer, 4);
    hp.n_rot = 0;
  } else {
    ok = ok && rd(&hp.n_head, 4) && rd(&hp.n_layer, 4) && rd(&hp.n_rot, 4);
  }
  hp.use_parallel_residual = arch == VSIM_ARCH_BLOOM ? 0 : 1;
  if (arch == VSIM_ARCH_GPTNEOX) ok = ok && rd(&hp.use_parallel_residual, 4);
  ok = ok && rd(&ftype, 4);
  if (!ok) return bad("truncated header");
  if (hp.n_vocab <= 0 || hp.n_embd <= 0 || hp.n_head <= 0 || hp.n_layer <= 0 || hp.n_rot < 0)
    return bad("header values out of range");
  if (ftype == 0 || ftype == 1)
    return bad("F32 / F16 weight files take the reference's F32 / F16 mul_mat (vsim.cpp:179-190); this library "
               "runs the Q4_0 path: quantize the file to Q4_0 (f16 == 2) first");
  if (ftype != 2) return bad("only Q4_0 (f16 == 2) files are supported");
  int32_t nv = hp.n_vocab;
  if (arch == VSIM_ARCH_GPTJ && !rd(&nv, 4)) return bad("truncated vocab count");
  if (nv < 0 || nv > (1 << 24)) return bad("vocab count out of range");
  for (int i = 0; i < nv; ++i) {
    uint32_t len = 0;
    if (!rd(&len, 4) || len > (1u << 20)) return bad("truncated or corrupt vocab");
    f.seekg(len, std::ios::cur);
    if (!f) return bad("truncated vocab");
  }
  vsim_model *m = nullptr;
  if (layer_end < 0) layer_end = hp.n_layer;
  RC(vsim_model_create(arch, &hp, n_ctx, device, layer_begin, layer_end, &m));
  std::map<std::string, Slot> full;  // every tensor of the whole model (all stages)
  {
    vsim_model whole;
    whole.arch = arch;
    whole.hp = hp;
    whole.l0 = 0;
    whole.l1 = hp.n_layer;
    std::vector<std::pair<std::string, Slot>> plan;
    plan_slots(&whole, plan);
    for (auto &ps : plan) full[ps.first] = ps.second;
  }
  auto fail_load = [&](const std::string &why) {
    vsim_model_free(m);
    return bad(why);
  };
  std::vector<char> buf;
  while (true) {
    int32_t nd = 0, ln = 0, ft = 0;
    if (!rd(&nd, 4)) break;  // end of file between records
    if (!rd(&ln, 4) || !rd(&ft, 4)) return fail_load("truncated tensor record");
    if (nd < 1 || nd > 2 || ln < 1 || ln > 512) return fail_load("corrupt tensor record (n_dims / name length)");
    int32_t dims[2] = {1, 1};
    size_t ne = 1;
    for (int i = 0; i < nd; ++i) {
      if (!rd(&dims[i], 4) || dims[i] <= 0) return fail_load("corrupt tensor dimensions");
      ne *= (size_t)dims[i];
    }
    std::string name(ln, 0);
    if (!rd(&name[0], ln)) return fail_load("truncated tensor name");
    if (ft != 0 && ft != 2) return fail_load("unsupported tensor type in " + name);
    if (ft == 2 && dims[0] % QK) return fail_load("Q4_0 tensor " + name + " with ne[0] not a multiple of 32");
    const size_t nbytes = ft == 0 ? ne * 4 : ne / QK * QBYTES;
    // the tensor as the whole model's graph expects it (BLOOM's fused query_key_value: the
    // slot of its first row block, three times the rows)
    const bool fused = full.find(name) == full.end() && full.find(name + "/q") != full.end();
    auto fit = full.find(fused ? name + "/q" : name);
    if (fit == full.end()) return fail_load("unknown tensor " + name);
    const Slot &sl = fit->second;
    if ((sl.kind == KQ4) != (ft == 2)) return fail_load("type mismatch " + name);
    const int want_rows = sl.kind == KQ4 ? sl.rows * (fused ? 3 : 1) : 1;
    if (dims[0] != sl.k || (nd == 2 ? dims[1] : 1) != want_rows) {
      char msg[256];
      snprintf(msg, sizeof msg, "tensor %s has the wrong shape in the model file: got [%d, %d], expected [%d, %d]",
               name.c_str(), dims[0], nd == 2 ? dims[1] : 1, sl.k, want_rows);
      return fail_load(msg);
    }
    if (m->slots.find(fused ? name + "/q" : name) == m->slots.end()) {  // another pipeline stage's tensor
      f.seekg(nbytes, std::ios::cur);
      if (!f) return fail_load("truncated tensor " + name);
      continue;
    }
    buf.resize(nbytes);
    if (!rd(buf.data(), nbytes)) return fail_load("truncated tensor " + name);
    if (int rc = vsim_model_set_tensor(m, name.c_str(), buf.data(), nbytes)) {
      vsim_model_free(m);
      return rc;
    }
  }
  for (auto &kv : m->slots)
    if (!kv.second.loaded) return fail_load("tensor missing from file: " + kv.first);
  *out = m;
  return VSIM_OK;
}

int vsim_model_set_mode(vsim_model *m, int mode) {
  if (mode != VSIM_MODE_EXACT && mode != VSIM_MODE_FAST) { set_error("set_mode: bad mode"); return VSIM_EINVAL; }
  m->mode = mode;
  return VSIM_OK;
}

int vsim_model_set_graph(vsim_model *m, int enable) {
  m->graph_enabled = enable != 0;
  return VSIM_OK;
}

int vsim_model_hparams(const vsim_model *m, vsim_hparams *hp, int *n_ctx, int *lb, int *le) {
  if (hp) *hp = m->hp;
  if (n_ctx) *n_ctx = m->n_ctx;
  if (lb) *lb = m->l0;
  if (le) *le = m->l1;
  return VSIM_OK;
}

void *vsim_model_stream(vsim_model *m) { return (void *)m->stream; }
const float *vsim_model_logits_dev(vsim_model *m) { return m->logits; }

int vsim_model_info(vsim_model *m, int *kernels_per_eval, int *graph_enabled, size_t *weight_bytes) {
  if (kernels_per_eval) *kernels_per_eval = m->kernels_last;
  if (graph_enabled) *graph_enabled = m->graph_enabled ? 1 : 0;
  if (weight_bytes) *weight_bytes = m->wbytes;
  return VSIM_OK;
}

}  // extern "C"

namespace {

// token (first stage) and n_past from their pinned host words
int upload_step(vsim_model *m) {
  if (m->first)
    VSIM_HIP(hipMemcpyAsync(m->tok_dev, m->tok_host, sizeof(int32_t), hipMemcpyHostToDevice, m->stream));
  VSIM_HIP(hipMemcpyAsync(m->npast_dev, m->npast_host, sizeof(int), hipMemcpyHostToDevice, m->stream));
  return VSIM_OK;
}

__global__ void k_npast_advance(int *npast) { npast[0] += 1; }

// One pipeline-stage step from the bound device buffers: token (first stage) or residual
// (other stages) in, this stage's layers, then the residual out (non-last stages) or the
// device argmax into the bound token word (last stage), then n_past + 1 on the device.
int enqueue_stage(vsim_model *m, int &nk) {
  hipStream_t s = m->stream;
  const int E = m->hp.n_embd;
  if (m->first) {
    VSIM_HIP(hipMemcpyAsync(m->tok_dev, m->st_tok_in, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
  } else {
    VSIM_HIP(hipMemcpyAsync(m->inpL, m->st_resid_in, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
  }
  RC(enqueue_decode(m, nk));
  if (m->last) {
    RC(launch_argmax(m->logits, m->hp.n_vocab, m->st_tok_out, m->am_ws, s));
    ++nk;
  } else {
    VSIM_HIP(hipMemcpyAsync(m->st_resid_out, m->resid_final, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
  }
  hipLaunchKernelGGL(k_npast_advance, dim3(1), dim3(1), 0, s, m->npast_dev);
  VSIM_HIP(hipGetLastError());
  ++nk;
  return VSIM_OK;
}

// Capture (once per mode) the whole single-token step as a hipGraph: uploads, the decode
// kernels, and either the logits copy-out or the device argmax and its 4-byte copy-out.
// kind 2: the device-resident greedy loop's step -- no uploads, no copy-out; the argmax
// feeds the next step (launch_argmax_gen).
int decode_graph(vsim_model *m, int kind) {
  const bool argmax = kind == 1, gen = kind == 2, stage = kind == 3;
  hipGraph_t &graph = stage ? m->graph_st : gen ? m->graph_gen : argmax ? m->graph_am : m->graph;
  hipGraphExec_t &gexec = stage ? m->gexec_st : gen ? m->gexec_gen : argmax ? m->gexec_am : m->gexec;
  int &gmode = stage ? m->graph_st_mode : gen ? m->graph_gen_mode : argmax ? m->graph_am_mode : m->graph_mode;
  if (gexec && gmode == m->mode) return VSIM_OK;
  if (gexec) (void)hipGraphExecDestroy(gexec);
  if (graph) (void)hipGraphDestroy(graph);
  gexec = nullptr;
  graph = nullptr;
  hipStream_t s = m->stream;
  const int V = m->hp.n_vocab;
  VSIM_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  int gk = 0;
  int rc = gen || stage ? VSIM_OK : upload_step(m);
  if (rc == 0 && stage) {
    rc = enqueue_stage(m, gk);
  } else if (rc == 0) {
    rc = enqueue_decode(m, gk);
  }
  if (rc == 0 && stage) {
  } else if (rc == 0 && gen) {
    rc = launch_argmax_gen(m->logits, V, m->am_dev, m->am_ws, m->tok_dev, m->npast_dev, m->hist_dev, s);
    ++gk;
  } else if (rc == 0 && argmax) {
    rc = launch_argmax(m->logits, V, m->am_dev, m->am_ws, s);
    ++gk;
    if (rc == 0 && hipMemcpyAsync(m->am_host, m->am_dev, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess)
      rc = hip_fail(hipErrorUnknown, "capture argmax copy");
  } else if (rc == 0 &&
             hipMemcpyAsync(m->logit_host, m->logits, sizeof(float) * V, hipMemcpyDeviceToHost, s) != hipSuccess) {
    rc = hip_fail(hipErrorUnknown, "capture logits copy");
  }
  hipGraph_t g = nullptr;
  const hipError_t ce = hipStreamEndCapture(s, &g);
  if (rc) return rc;
  if (ce != hipSuccess) return hip_fail(ce, "hipStreamEndCapture");
  graph = g;
  VSIM_HIP(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
  gmode = m->mode;
  m->graph_kernels_kind[kind] = gk;
  return VSIM_OK;
}

}  // namespace

extern "C" {

int vsim_model_eval_argmax(vsim_model *m, int n_past, int32_t token, int32_t *next_token) {
  if (!m || !next_token) { set_error("eval_argmax: null argument"); return VSIM_EINVAL; }
  if (!m->first || !m->last || !fused_ok(m, 1)) {
    set_error("eval_argmax: needs a whole-model stage with the single-token decode path");
    return VSIM_EINVAL;
  }
  if (n_past < 0 || n_past + 1 > m->n_ctx) { set_error("eval_argmax: n_past + 1 exceeds n_ctx"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  const ErrScope es(m);
  RC(ensure_scratch(m, 1));
  const int V = m->hp.n_vocab;
  if (token < 0 || token >= V) { set_error("eval_argmax: token id out of range"); return VSIM_EINVAL; }
  m->tok_host[0] = token;
  m->npast_host[0] = n_past;
  m->prof_npast = n_past;
  m->st_npast = -1;  // this step sets the device n_past: a stage step needs a new stage_begin
  hipStream_t s = m->stream;
  if (m->graph_enabled && !m->profile) {
    RC(decode_graph(m, 1));
    VSIM_HIP(hipGraphLaunch(m->gexec_am, s));
    m->kernels_last = m->graph_kernels_kind[1];
  } else {
    int nk = 0;
    RC(upload_step(m));
    RC(enqueue_decode(m, nk));
    RC(launch_argmax(m->logits, V, m->am_dev, m->am_ws, s));
    VSIM_HIP(hipMemcpyAsync(m->am_host, m->am_dev, sizeof(int), hipMemcpyDeviceToHost, s));
    m->kernels_last = nk + 1;
  }
  RC(spin_read(m));
  VSIM_HIP(hipStreamSynchronize(s));
  RC(spin_check(m));
  *next_token = m->am_host[0];
  if (m->profile) RC(prof_collect(m));
  return VSIM_OK;
}

int vsim_model_generate(vsim_model *m, int n_past, int32_t token, int n_steps, int32_t *tokens_out) {
  if (!m || !tokens_out || n_steps < 0) { set_error("generate: bad argument"); return VSIM_EINVAL; }
  if (!m->first || !m->last || !fused_ok(m, 1)) {
    set_error("generate: needs a whole-model stage with the single-token decode path");
    return VSIM_EINVAL;
  }
  if (n_past < 0 || n_past + n_steps > m->n_ctx) { set_error("generate: n_past + n_steps exceeds n_ctx"); return VSIM_EINVAL; }
  if (n_steps == 0) return VSIM_OK;
  VSIM_HIP(hipSetDevice(m->device));
  const ErrScope es(m);
  RC(ensure_scratch(m, 1));
  if (token < 0 || token >= m->hp.n_vocab) { set_error("generate: token id out of range"); return VSIM_EINVAL; }
  hipStream_t s = m->stream;
  m->tok_host[0] = token;
  m->npast_host[0] = n_past;
  m->prof_npast = n_past;
  m->st_npast = -1;  // the loop advances the device n_past: a stage step needs a new stage_begin
  RC(upload_step(m));
  if (m->graph_enabled && !m->profile) {
    RC(decode_graph(m, 2));
    for (int i = 0; i < n_steps; ++i) VSIM_HIP(hipGraphLaunch(m->gexec_gen, s));
    m->kernels_last = m->graph_kernels_kind[2];  // kernels of one decode step (argmax included)
  } else {
    for (int i = 0; i < n_steps; ++i) {
      int nk = 0;
      m->prof_npast = n_past + i;
      RC(enqueue_decode(m, nk));
      RC(launch_argmax_gen(m->logits, m->hp.n_vocab, m->am_dev, m->am_ws, m->tok_dev, m->npast_dev, m->hist_dev, s));
      m->kernels_last = nk + 1;
    }
  }
  VSIM_HIP(hipMemcpyAsync(tokens_out, m->hist_dev + n_past, sizeof(int32_t) * n_steps, hipMemcpyDeviceToHost, s));
  RC(spin_read(m));
  VSIM_HIP(hipStreamSynchronize(s));
  RC(spin_check(m));
  if (m->profile) RC(prof_collect(m));
  return VSIM_OK;
}

int vsim_model_reserve(vsim_model *m, int n_tokens) {
  if (!m) { set_error("reserve: null model"); return VSIM_EINVAL; }
  if (n_tokens <= 0 || n_tokens > m->n_ctx) { set_error("reserve: n_tokens must be in 1..n_ctx"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  RC(ensure_scratch(m, n_tokens));
  const int E = E_(m), d = E / m->hp.n_head;
  if (n_tokens >= 8 && attn_prefill_supported(d) && E % 64 == 0) {
    if (!m->pf_scratch) {
      m->pf_bytes = attn_prefill_scratch(E, m->n_ctx);
      VSIM_HIP(hipMalloc(&m->pf_scratch, m->pf_bytes));
    }
    RC(attn_prefill_prepare());
  }
  if (n_tokens >= G2_MIN_N) RC(gemm_reserve_stream(m->stream));
  VSIM_HIP(hipStreamSynchronize(m->stream));
  return VSIM_OK;
}

int vsim_model_eval(vsim_model *m, int n_past, const int32_t *tokens, int N, const float *resid_in, float *resid_out,
                    float *logits) {
  if (!m) { set_error("eval: null model"); return VSIM_EINVAL; }
  if (N <= 0 || n_past < 0 || n_past + N > m->n_ctx) { set_error("eval: n_past + N exceeds n_ctx"); return VSIM_EINVAL; }
  m->st_npast = -1;  // an eval sets the device n_past: a stage step needs a new stage_begin
  VSIM_HIP(hipSetDevice(m->device));
  const ErrScope es(m);
  RC(ensure_scratch(m, N));
  const int E = m->hp.n_embd, V = m->hp.n_vocab;
  hipStream_t s = m->stream;
  int nk = 0;
  if (fused_ok(m, N)) {
    if (m->first) {
      if (!tokens) { set_error("eval: first stage needs tokens"); return VSIM_EINVAL; }
      if (tokens[0] < 0 || tokens[0] >= V) { set_error("eval: token id out of range"); return VSIM_EINVAL; }
      m->tok_host[0] = tokens[0];
    } else {
      if (!resid_in) { set_error("eval: non-first stage needs resid_in"); return VSIM_EINVAL; }
      VSIM_HIP(hipMemcpyAsync(m->inpL, resid_in, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
    }
    m->npast_host[0] = n_past;
  m->prof_npast = n_past;
    const bool use_graph = m->graph_enabled && m->first && m->last && !m->profile;
    if (use_graph) {
      // the token / n_past uploads are nodes of the graph (they read the pinned host words
      // when the graph runs)
      RC(decode_graph(m, 0));
      VSIM_HIP(hipGraphLaunch(m->gexec, s));
      nk = m->graph_kernels_kind[0];
    } else {
      RC(upload_step(m));
      RC(enqueue_decode(m, nk));
      if (m->last && logits)
        VSIM_HIP(hipMemcpyAsync(m->logit_host, m->logits, sizeof(float) * V, hipMemcpyDeviceToHost, s));
      else if (!m->last && resid_out)
        VSIM_HIP(hipMemcpyAsync(resid_out, m->resid_final, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
    }
  } else {
    // general path: prompt batches (N > 1) and the serial-residual GPT-NeoX variant
    if (m->first) {
      if (!tokens) { set_error("eval: first stage needs tokens"); return VSIM_EINVAL; }
      for (int i = 0; i < N; ++i) {
        if (tokens[i] < 0 || tokens[i] >= V) { set_error("eval: token id out of range"); return VSIM_EINVAL; }
        m->tok_host[i] = tokens[i];
      }
      VSIM_HIP(hipMemcpyAsync(m->tok_dev, m->tok_host, N * sizeof(int32_t), hipMemcpyHostToDevice, s));
      if (m->arch == VSIM_ARCH_BLOOM) {  // word embeddings + word_embeddings_layernorm
        RC(launch_get_rows(m->wte, E, V, m->tok_dev, N, m->cur1, s));
        RC(launch_norm(m->cur1, m->inpL, E, N, m->emb_w, m->emb_b, s));
        nk += 2;
      } else {
        RC(launch_get_rows(m->wte, E, V, m->tok_dev, N, m->inpL, s));
        ++nk;
      }
    } else {
      if (!resid_in) { set_error("eval: non-first stage needs resid_in"); return VSIM_EINVAL; }
      VSIM_HIP(hipMemcpyAsync(m->inpL, resid_in, sizeof(float) * N * E, hipMemcpyDeviceToDevice, s));
    }
    for (int il = m->l0; il < m->l1; ++il) RC(run_layer(m, il, n_past, N, nk));
    if (m->last) {
      // only the last row's logits leave the eval (vsim.cpp:736-737); rows are independent
      const float *xl = m->inpL + (size_t)(N - 1) * E;
      RC(launch_norm(xl, m->cur1, E, 1, m->lnf_w, m->lnf_b, s));
      ++nk;
      RC(mm(m, m->lmh, V, E, m->cur1, 1, m->xq1, m->xd1, true, m->arch == VSIM_ARCH_GPTJ ? m->lmh_b : nullptr,
            m->logits, nk));
      if (logits) VSIM_HIP(hipMemcpyAsync(m->logit_host, m->logits, sizeof(float) * V, hipMemcpyDeviceToHost, s));
    } else if (resid_out) {
      VSIM_HIP(hipMemcpyAsync(resid_out, m->inpL, sizeof(float) * N * E, hipMemcpyDeviceToDevice, s));
    }
  }
  RC(spin_read(m));
  VSIM_HIP(hipStreamSynchronize(s));
  RC(spin_check(m));
  if (m->last && logits) memcpy(logits, m->logit_host, sizeof(float) * V);
  m->kernels_last = nk;
  if (m->profile) RC(prof_collect(m));
  return VSIM_OK;
}

int vsim_model_stage_bind(vsim_model *m, const int32_t *tok_in, const float *resid_in, float *resid_out,
                          int32_t *tok_out) {
  if (!m) { set_error("stage_bind: null model"); return VSIM_EINVAL; }
  if ((m->first && !tok_in) || (!m->first && !resid_in) || (m->last && !tok_out) || (!m->last && !resid_out)) {
    set_error("stage_bind: first stage needs tok_in, later stages resid_in, the last tok_out, the others resid_out");
    return VSIM_EINVAL;
  }
  if (!fused_ok(m, 1)) { set_error("stage_bind: needs the single-token decode path"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  RC(ensure_scratch(m, 1));
  if (m->st_tok_in != tok_in || m->st_resid_in != resid_in || m->st_resid_out != resid_out || m->st_tok_out != tok_out) {
    // the captured step reads the bound addresses: recapture on the next step
    if (m->gexec_st) (void)hipGraphExecDestroy(m->gexec_st);
    if (m->graph_st) (void)hipGraphDestroy(m->graph_st);
    m->gexec_st = nullptr;
    m->graph_st = nullptr;
    m->graph_st_mode = -1;
  }
  m->st_tok_in = tok_in;
  m->st_resid_in = resid_in;
  m->st_resid_out = resid_out;
  m->st_tok_out = tok_out;
  return VSIM_OK;
}

int vsim_model_stage_begin(vsim_model *m, int n_past) {
  if (!m || n_past < 0 || n_past >= m->n_ctx) { set_error("stage_begin: n_past outside the context"); return VSIM_EINVAL; }
  if (!m->st_tok_in && !m->st_resid_in) { set_error("stage_begin: stage_bind first"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  RC(ensure_scratch(m, 1));
  m->npast_host[0] = n_past;
  VSIM_HIP(hipMemcpyAsync(m->npast_dev, m->npast_host, sizeof(int), hipMemcpyHostToDevice, m->stream));
  VSIM_HIP(hipStreamSynchronize(m->stream));
  m->st_npast = n_past;
  return VSIM_OK;
}

int vsim_model_stage_step(vsim_model *m) {
  if (!m || m->st_npast < 0) { set_error("stage_step: stage_begin first"); return VSIM_EINVAL; }
  if (m->st_npast + 1 > m->n_ctx) { set_error("stage_step: context full"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  const ErrScope es(m);
  m->prof_npast = m->st_npast;
  if (m->graph_enabled && !m->profile) {
    RC(decode_graph(m, 3));
    VSIM_HIP(hipGraphLaunch(m->gexec_st, m->stream));
    m->kernels_last = m->graph_kernels_kind[3];
  } else {
    int nk = 0;
    RC(enqueue_stage(m, nk));
    m->kernels_last = nk;
  }
  m->st_npast++;
  if (m->profile) {
    RC(spin_read(m));
    VSIM_HIP(hipStreamSynchronize(m->stream));
    RC(spin_check(m));
    RC(prof_collect(m));
  }
  return VSIM_OK;  // (steps run asynchronously: vsim_model_sync checks them)
}

int vsim_model_debug_poison(vsim_model *m, int n_tokens) {
  if (!m || n_tokens <= 0) { set_error("debug_poison: bad argument"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  RC(ensure_scratch(m, n_tokens));
  const int E = m->hp.n_embd;
  if (!m->pf_scratch) {
    m->pf_bytes = attn_prefill_scratch(E, m->n_ctx);
    VSIM_HIP(hipMalloc(&m->pf_scratch, m->pf_bytes));
  }
  const size_t n = m->n_max, F = 4 * (size_t)E, V = m->hp.n_vocab, H = m->hp.n_head;
  const size_t nl = (size_t)std::max(1, m->l1 - m->l0);
  struct Buf {
    void *p;
    size_t bytes;
  } bufs[] = {
      {m->inpL, n * E * 4}, {m->cur1, n * E * 4}, {m->cur2, n * E * 4}, {m->Qb, n * E * 4}, {m->Kb, n * E * 4},
      {m->Vb, n * E * 4}, {m->attn_in, n * E * 4}, {m->attn, n * E * 4}, {m->ff, n * E * 4}, {m->fch, n * F * 4},
      {m->kq, n * H * m->n_ctx * 4}, {m->logits, V * 4}, {m->xq1, n * E / QK * QBYTES},
      {m->xq2, n * E / QK * QBYTES}, {m->xq3, n * F / QK * QBYTES}, {m->xd1, n * E * 4}, {m->xd2, n * E * 4},
      {m->xd3, n * F * 4}, {m->xqa, n * E / QK * QBYTES}, {m->xda, n * E * 4}, {m->inpL2, (size_t)E * 4},
      {m->pf_scratch, m->pf_bytes & ~(size_t)3}, {m->pf_x16, n >= (size_t)GEMM_MIN_N ? n * (E + F) * 2 : 0},
      {m->kcache, nl * m->n_ctx * E * 4}, {m->vcache, nl * m->n_ctx * E * 4}};
  for (const Buf &b : bufs)
    if (b.p && b.bytes) VSIM_HIP(hipMemsetD32Async((hipDeviceptr_t)b.p, 0x7FC00000u, b.bytes / 4, m->stream));
  VSIM_HIP(hipStreamSynchronize(m->stream));
  return VSIM_OK;
}

int vsim_model_sync(vsim_model *m) {
  if (!m) { set_error("sync: null model"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(m->device));
  RC(spin_read(m));
  VSIM_HIP(hipStreamSynchronize(m->stream));
  return spin_check(m);
}

int vsim_model_set_profile(vsim_model *m, int enable) {
  m->profile = enable != 0;
  m->prof_kinds.clear();
  m->prof_pending.clear();
  m->prof_used = 0;
  return VSIM_OK;
}

int vsim_model_profile_stats(vsim_model *m, double *gemv_ms, long *gemv_launches, double *gemv_bytes) {
  double ms = 0.0, by = 0.0;
  long n = 0;
  for (const auto &k : m->prof_kinds) {
    ms += k.ms;
    by += k.bytes;
    n += k.n;
  }
  if (gemv_ms) *gemv_ms = ms;
  if (gemv_launches) *gemv_launches = n;
  if (gemv_bytes) *gemv_bytes = by;
  return VSIM_OK;
}

int vsim_model_profile_kernel(vsim_model *m, int i, char *name, int name_cap, double *ms, long *launches,
                              double *bytes) {
  if (!m || i < 0 || i >= (int)m->prof_kinds.size()) return VSIM_EINVAL;
  const auto &k = m->prof_kinds[i];
  if (name && name_cap > 0) {
    std::strncpy(name, k.name.c_str(), (size_t)name_cap - 1);
    name[name_cap - 1] = 0;
  }
  if (ms) *ms = k.ms;
  if (launches) *launches = k.n;
  if (bytes) *bytes = k.bytes;
  return VSIM_OK;
}

}  // extern "C"
