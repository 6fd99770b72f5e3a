// vsim_amd/csrc/graph.cpp — device executor for the reference's ggml_cgraph.
//
// vsim_graph_compute(ctx, cgraph) takes the place of ggml_graph_compute (ggml.c:8245-8700) at
// vsim.cpp:725: it walks cgraph->nodes[] in insertion order, as ggml_compute_forward
// (ggml.c:7562-7756) does, and runs every node on the GPU.  The tensors keep their host
// addresses; the device holds mirrors at the same offsets:
//   * the eval's context arena (ctx0's mem_buffer, vsim.cpp:490-511) is mirrored whole, so a
//     node, a view or a permute of it resolves to dev_arena + (data - mem_buffer);
//   * every leaf outside the arena (the model's weights and KV cache, vsim.cpp:253-265) is
//     uploaded once on first sight and kept: Q4_0 matrices in the W4T32 layout the GEMV
//     kernels read, F32 tensors as they are.  The KV cache then lives on the device: the
//     cpy nodes write views of it there and the attention views read it there;
//   * leafs inside the arena (token ids, rope / mask parameters, the scale) are uploaded
//     before each compute; only the last node's bytes come back (vsim.cpp:736-737 reads the
//     last row of the logits).
// Numerics are the exact mode of every op (bit-identical to the reference's CPU kernels); the
// one reduction whose grouping depends on the thread count, the transposed F32 mul_mat (KQV),
// is grouped by cgraph->n_threads exactly as the reference's pool groups it.
// Every node is validated before any runs; an unsupported node leaves host state untouched.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "graph.hpp"
#include "../../include/vsim_hip.h"

using namespace vsim;

namespace {

struct Ext {
  size_t bytes;
  char *dev;  // F32 / I32 copy (null for Q4_0)
  void *w4;   // Q4_0: W4T32 copy
  int type, ne0, ne1;
};

struct OpProf {
  double ms = 0.0;
  long calls = 0;
};

struct Exec {
  std::mutex mu;
  bool ready = false;
  int device = 0;
  hipStream_t stream = nullptr;
  const char *arena_host = nullptr;
  size_t arena_bytes = 0;
  char *arena_dev = nullptr;
  std::map<const char *, Ext> ext;  // external tensors by host start address
  void *xq = nullptr;
  float *xd = nullptr, *tmp = nullptr;
  size_t xq_cap = 0, xd_cap = 0, tmp_cap = 0;
  double2 *cs = nullptr;
  int cs_pos = 0, cs_dims = 0;
  uint64_t computes = 0, nodes = 0, h2d = 0, d2h = 0;
  bool prof = false;
  OpProf op[GGML_OP_COUNT + 2];  // + Q4_0 mul_mat, F32 mul_mat split out of MUL_MAT
  uint64_t ext_gen = 0;          // bumped whenever a mirror of an external tensor changes
  // decode fast path: the model executor bound to the mirrors of one set of matched tensors
  struct Fast {
    vsim_model *m = nullptr;
    std::vector<const void *> key;  // the matched weight / cache tensors the model is bound to
    uint64_t gen = 0;
    int nth = 0;
    float scale = 0.0f;
  } fast;
  bool fast_off = false;
  uint64_t fast_evals = 0, fast_plans = 0;
} X;

constexpr int PROF_MM_Q4 = GGML_OP_COUNT, PROF_MM_F32 = GGML_OP_COUNT + 1;

int grow(void **p, size_t *cap, size_t want) {
  if (want <= *cap) return VSIM_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t n = want + want / 2;
  VSIM_HIP(hipMalloc(p, n));
  *cap = n;
  return VSIM_OK;
}

void print_profile_at_exit();
void print_stats_at_exit() {
  // stderr: the front-end reads stdout (cformers/interface.py parses the token stream)
  fprintf(stderr, "vsim_graph_compute: %llu computes, %llu on the decode fast path, %llu fast-path plans\n",
          (unsigned long long)X.computes, (unsigned long long)X.fast_evals, (unsigned long long)X.fast_plans);
}

int ensure_ready() {
  if (X.ready) return VSIM_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("graph_compute: no HIP device");
    return VSIM_ENODEV;
  }
  const char *e = getenv("VSIM_DEVICE");
  X.device = e ? atoi(e) : 0;
  if (X.device < 0 || X.device >= ndev) X.device = 0;
  VSIM_HIP(hipSetDevice(X.device));
  VSIM_HIP(hipStreamCreateWithFlags(&X.stream, hipStreamNonBlocking));
  DevTables t;
  if (int rc = tables_get(&t)) return rc;
  X.prof = getenv("VSIM_GRAPH_PROFILE") && atoi(getenv("VSIM_GRAPH_PROFILE")) != 0;
  X.fast_off = getenv("VSIM_GRAPH_FAST") && atoi(getenv("VSIM_GRAPH_FAST")) == 0;
  if (getenv("VSIM_GRAPH_STATS") && atoi(getenv("VSIM_GRAPH_STATS")) != 0) atexit(print_stats_at_exit);
  // like the reference's show_time_sep at the end of a run (vsim.cpp:905-908)
  if (X.prof) atexit(print_profile_at_exit);
  X.ready = true;
  return VSIM_OK;
}

// bytes spanned by a tensor (ggml_nbytes for contiguous ones; the furthest element + 1 for views)
size_t span(const ggml_tensor *t) {
  const size_t ts = t->type == GGML_TYPE_Q4_0 ? 20 : t->type == GGML_TYPE_Q4_1 ? 24 : t->type == GGML_TYPE_F16 ? 2
                    : t->type == GGML_TYPE_I8 ? 1 : t->type == GGML_TYPE_I16 ? 2 : 4;
  const int blck = (t->type == GGML_TYPE_Q4_0 || t->type == GGML_TYPE_Q4_1) ? 32 : 1;
  size_t s = ts * ((size_t)t->ne[0] / blck);
  for (int i = 1; i < 4; ++i)
    if (t->ne[i] > 1) s += (size_t)(t->ne[i] - 1) * t->nb[i];
  return s;
}

bool in_arena(const void *p) {
  const char *c = (const char *)p;
  return X.arena_host && c >= X.arena_host && c < X.arena_host + X.arena_bytes;
}

// device address of a host address (null if it is in no mirror)
char *dev_of(const void *p, size_t bytes) {
  const char *c = (const char *)p;
  if (in_arena(c)) return c + bytes <= X.arena_host + X.arena_bytes ? X.arena_dev + (c - X.arena_host) : nullptr;
  auto it = X.ext.upper_bound(c);
  if (it == X.ext.begin()) return nullptr;
  --it;
  if (!it->second.dev || c + bytes > it->first + it->second.bytes) return nullptr;
  return it->second.dev + (c - it->first);
}

char *dev_of_t(const ggml_tensor *t) { return dev_of(t->data, span(t)); }

const Ext *q4_of(const ggml_tensor *t) {
  auto it = X.ext.find((const char *)t->data);
  if (it == X.ext.end() || !it->second.w4 || it->second.ne0 != t->ne[0] || it->second.ne1 != t->ne[1]) return nullptr;
  return &it->second;
}

void drop_fast() {
  if (X.fast.m) vsim_model_free(X.fast.m);
  X.fast = Exec::Fast{};
}

int register_ext(const ggml_tensor *t) {
  const char *h = (const char *)t->data;
  const size_t bytes = span(t);
  auto it = X.ext.find(h);
  if (it != X.ext.end()) {
    if (it->second.bytes == bytes && it->second.type == (int)t->type && it->second.ne0 == t->ne[0] &&
        it->second.ne1 == t->ne[1])
      return VSIM_OK;
    drop_fast();  // the plan's model may point at the buffer freed here
    if (it->second.dev) (void)hipFree(it->second.dev);
    if (it->second.w4) (void)hipFree(it->second.w4);
    X.ext.erase(it);
    ++X.ext_gen;
  }
  Ext e{bytes, nullptr, nullptr, (int)t->type, t->ne[0], t->ne[1]};
  if (t->type == GGML_TYPE_Q4_0) {
    if (t->ne[2] != 1 || t->ne[3] != 1 || t->ne[0] % QK || t->nb[1] != (size_t)t->ne[0] / QK * QBYTES) {
      set_error("graph_compute: Q4_0 leaf is not a 2-D row-major matrix");
      return VSIM_EINVAL;
    }
    void *stage = nullptr;
    VSIM_HIP(hipMalloc(&e.w4, w4_bytes(t->ne[1], t->ne[0])));
    VSIM_HIP(hipMalloc(&stage, bytes));
    VSIM_HIP(hipMemcpyAsync(stage, h, bytes, hipMemcpyHostToDevice, X.stream));
    int rc = launch_q4_repack(stage, e.w4, t->ne[1], t->ne[0], X.stream);
    if (hipStreamSynchronize(X.stream) != hipSuccess && !rc) rc = VSIM_EHIP;
    (void)hipFree(stage);
    if (rc) return rc;
  } else if (t->type == GGML_TYPE_F32 || t->type == GGML_TYPE_I32) {
    VSIM_HIP(hipMalloc((void **)&e.dev, bytes));
    VSIM_HIP(hipMemcpyAsync(e.dev, h, bytes, hipMemcpyHostToDevice, X.stream));
  } else {
    set_error("graph_compute: leaf type other than Q4_0 / F32 / I32");
    return VSIM_EINVAL;
  }
  X.h2d += bytes;
  X.ext[h] = e;
  ++X.ext_gen;
  return VSIM_OK;
}

bool contiguous(const ggml_tensor *t) {
  const size_t es = t->type == GGML_TYPE_Q4_0 ? 20 : 4;
  const int blck = t->type == GGML_TYPE_Q4_0 ? 32 : 1;
  return t->nb[0] == es && t->nb[1] == t->nb[0] * (t->ne[0] / blck) && t->nb[2] == t->nb[1] * t->ne[1] &&
         t->nb[3] == t->nb[2] * t->ne[2];
}
long long nrows(const ggml_tensor *t) { return (long long)t->ne[1] * t->ne[2] * t->ne[3]; }
long long nelem(const ggml_tensor *t) { return (long long)t->ne[0] * nrows(t); }
bool same_shape(const ggml_tensor *a, const ggml_tensor *b) {
  return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}
GT gt(const ggml_tensor *t, const char *dev) {
  GT g;
  g.p = dev;
  for (int i = 0; i < 4; ++i) {
    g.ne[i] = t->ne[i];
    g.nb[i] = (long long)t->nb[i];
  }
  return g;
}

int fail(const char *what, const ggml_tensor *n) {
  char buf[256];
  snprintf(buf, sizeof buf, "graph_compute: %s (op %d, ne %d %d %d %d)", what, (int)n->op, n->ne[0], n->ne[1],
           n->ne[2], n->ne[3]);
  set_error(buf);
  return VSIM_EINVAL;
}

int rope_table(int n_pos, int n_dims) {
  if (X.cs && n_dims == X.cs_dims && n_pos <= X.cs_pos) return VSIM_OK;
  const int pos = std::max(n_pos, std::max(X.cs_pos, 512));
  std::vector<double2> h((size_t)pos * (n_dims / 2));
  rope_table_host(h.data(), pos, n_dims);
  if (X.cs) (void)hipFree(X.cs);
  X.cs = nullptr;
  VSIM_HIP(hipMalloc((void **)&X.cs, h.size() * sizeof(double2)));
  VSIM_HIP(hipMemcpyAsync(X.cs, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice, X.stream));
  VSIM_HIP(hipStreamSynchronize(X.stream));
  X.cs_pos = pos;
  X.cs_dims = n_dims;
  return VSIM_OK;
}

#define NEED(cond, what)              \
  do {                                \
    if (!(cond)) return fail(what, n); \
  } while (0)

// Checks node n (dry) or runs it.  nth: the graph's n_threads.
int node(const ggml_tensor *n, int nth, bool dry) {
  const ggml_tensor *a = n->src0, *b = n->src1;
  hipStream_t s = X.stream;
  switch (n->op) {
    case GGML_OP_NONE:
    case GGML_OP_RESHAPE:
    case GGML_OP_VIEW:
    case GGML_OP_PERMUTE:
    case GGML_OP_TRANSPOSE:
      return VSIM_OK;  // aliases: the forward pass does nothing (ggml.c:5700-5760)
    case GGML_OP_DUP:
    case GGML_OP_CPY: {
      const ggml_tensor *dst = n->op == GGML_OP_CPY ? b : n;
      NEED(a && dst && a->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_F32, "cpy: F32 only");
      NEED(contiguous(dst) && nelem(dst) == nelem(a), "cpy: destination must be contiguous, same element count");
      char *da = dev_of_t(a), *dd = dev_of_t(dst);
      NEED(da && dd, "cpy: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_g_dup((float *)dd, gt(a, da), nelem(a), s);
    }
    case GGML_OP_ADD:
    case GGML_OP_MUL: {
      NEED(a && b && same_shape(a, b) && same_shape(a, n), "add/mul: shapes differ");
      NEED(a->type == GGML_TYPE_F32 && b->type == GGML_TYPE_F32 && n->type == GGML_TYPE_F32, "add/mul: F32 only");
      NEED(n->nb[0] == 4 && a->nb[0] == 4, "add/mul: dim 0 must be contiguous");
      NEED(n->op == GGML_OP_ADD || b->nb[0] == 4, "mul: src1 dim 0 must be contiguous");
      // rows j of every operand at j * nb1 (ggml_nrows rows, as the reference indexes them)
      NEED(n->ne[2] * n->ne[3] == 1 || (contiguous(n) && contiguous(a) && (b->nb[0] != 4 || contiguous(b))),
           "add/mul: higher dims must be contiguous");
      char *da = dev_of_t(a), *db = dev_of_t(b), *dn = dev_of_t(n);
      NEED(da && db && dn, "add/mul: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_g_binop(n->op == GGML_OP_ADD ? 0 : 1, dn, (long long)n->nb[1], da, (long long)a->nb[1], db,
                            (long long)b->nb[0], (long long)b->nb[1], n->ne[0], nrows(n), s);
    }
    case GGML_OP_REPEAT: {
      NEED(a && a->ne[2] == 1 && a->ne[3] == 1 && n->ne[2] == 1 && n->ne[3] == 1, "repeat: 2-D only");
      NEED(a->ne[0] > 0 && a->ne[1] > 0 && n->ne[0] % a->ne[0] == 0 && n->ne[1] % a->ne[1] == 0, "repeat: shape");
      NEED(a->nb[0] == 4 && n->nb[0] == 4, "repeat: dim 0 must be contiguous");
      char *da = dev_of_t(a), *dn = dev_of_t(n);
      NEED(da && dn, "repeat: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_g_repeat(dn, (long long)n->nb[1], da, (long long)a->nb[1], n->ne[0], n->ne[1], a->ne[0], a->ne[1],
                             s);
    }
    case GGML_OP_GELU: {
      NEED(a && contiguous(a) && contiguous(n) && same_shape(a, n), "gelu: contiguous operands");
      char *da = dev_of_t(a), *dn = dev_of_t(n);
      NEED(da && dn, "gelu: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_gelu((const float *)da, (float *)dn, (int)nelem(n), nullptr, 1, s);
    }
    case GGML_OP_NORM: {
      NEED(a && contiguous(a) && contiguous(n) && same_shape(a, n) && a->type == GGML_TYPE_F32, "norm: contiguous F32");
      char *da = dev_of_t(a), *dn = dev_of_t(n);
      NEED(da && dn, "norm: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_norm((const float *)da, (float *)dn, n->ne[0], (int)nrows(n), nullptr, nullptr, s);
    }
    case GGML_OP_SCALE: {
      NEED(a && b && n->data == a->data && contiguous(n) && nelem(b) == 1 && b->type == GGML_TYPE_F32,
           "scale: in place on a contiguous tensor by an F32 scalar");
      char *dn = dev_of_t(n);
      NEED(dn, "scale: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_g_scale(dn, (long long)n->nb[1], n->ne[0], nrows(n), *(const float *)b->data, s);
    }
    case GGML_OP_DIAG_MASK_INF: {
      NEED(a && b && n->data == a->data && nelem(b) == 1 && b->type == GGML_TYPE_I32 && n->nb[0] == 4,
           "diag_mask_inf: in place, I32 n_past");
      char *dn = dev_of_t(n);
      NEED(dn, "diag_mask_inf: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      const int nr = n->ne[1], nz = (int)(nrows(n) / nr);
      return launch_g_diag_mask(dn, 4, (long long)n->nb[1], (long long)n->nb[2], n->ne[0], nr, nz,
                                *(const int32_t *)b->data, s);
    }
    case GGML_OP_SOFT_MAX: {
      NEED(a && n->data == a->data && contiguous(n), "soft_max: in place on a contiguous tensor");
      char *dn = dev_of_t(n);
      NEED(dn, "soft_max: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      // scale 1 and a mask that masks nothing: the plain soft_max of ggml.c:5825-5893
      return launch_attn_softmax((float *)dn, n->ne[0], (int)nrows(n), 1, n->ne[0], 1.0f, s);
    }
    case GGML_OP_ROPE:
    case GGML_OP_GPTNEOX_ROPE: {
      NEED(a && b && n->data == a->data && contiguous(n) && n->type == GGML_TYPE_F32 && n->ne[3] == 1,
           "rope: in place on a contiguous [d, H, T] tensor");
      NEED(b->type == GGML_TYPE_I32 && nelem(b) == 3, "rope: parameters {n_past, n_dims, mode}");
      const int32_t *pr = (const int32_t *)b->data;
      const int n_past = pr[0], n_dims = pr[1], mode = pr[2];
      NEED(n_dims > 0 && n_dims % 2 == 0 && n_dims <= n->ne[0] && (mode == 0 || mode == 1), "rope: parameters");
      char *dn = dev_of_t(n);
      NEED(dn, "rope: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      const int T = n->ne[2];
      if (int rc = rope_table(mode == 0 ? n_past + T : T, n_dims)) return rc;
      return launch_rope(n->op == GGML_OP_GPTNEOX_ROPE ? 0 : 1, (float *)dn, n->ne[0], n->ne[1], T, n_past, n_dims,
                         mode, X.cs, s);
    }
    case GGML_OP_GET_ROWS: {
      NEED(a && b && a->type == GGML_TYPE_Q4_0 && b->type == GGML_TYPE_I32 && contiguous(n), "get_rows: Q4_0 rows");
      const Ext *w = q4_of(a);
      char *db = dev_of_t(b), *dn = dev_of_t(n);
      NEED(w && db && dn, "get_rows: operand outside the mirrored memory");
      if (dry) return VSIM_OK;
      return launch_get_rows(w->w4, a->ne[0], a->ne[1], (const int32_t *)db, b->ne[0], (float *)dn, s);
    }
    case GGML_OP_MUL_MAT: {
      NEED(a && b && b->type == GGML_TYPE_F32 && n->type == GGML_TYPE_F32, "mul_mat: src1 F32");
      if (a->type == GGML_TYPE_Q4_0) {
        // ggml.c:4891-5165: src1 rows re-quantized (INIT), each weight row dotted (COMPUTE)
        const int K = a->ne[0], M = a->ne[1], N = b->ne[1];
        NEED(b->ne[0] == K && b->ne[2] == 1 && b->ne[3] == 1 && b->nb[0] == 4, "mul_mat q4: src1 [K, N]");
        NEED(n->ne[0] == M && n->ne[1] == N && contiguous(n), "mul_mat q4: dst [M, N] contiguous");
        const Ext *w = q4_of(a);
        char *db = dev_of_t(b), *dn = dev_of_t(n);
        NEED(w && db && dn, "mul_mat q4: operand outside the mirrored memory");
        if (dry) return VSIM_OK;
        const float *x = (const float *)db;
        if (b->nb[1] != (size_t)K * 4) {  // rows gathered first
          if (int rc = grow((void **)&X.tmp, &X.tmp_cap, (size_t)K * N * 4)) return rc;
          if (int rc = launch_g_dup(X.tmp, gt(b, db), (long long)K * N, s)) return rc;
          x = X.tmp;
        }
        if (int rc = grow(&X.xq, &X.xq_cap, (size_t)N * K / QK * QBYTES)) return rc;
        if (int rc = grow((void **)&X.xd, &X.xd_cap, (size_t)N * K * 4)) return rc;
        if (int rc = launch_q4_quantize(x, K, N, X.xq, X.xd, s)) return rc;
        return launch_q4_gemv(w->w4, M, K, X.xq, X.xd, N, nullptr, (float *)dn, VSIM_MODE_EXACT, s);
      }
      NEED(a->type == GGML_TYPE_F32, "mul_mat: src0 Q4_0 or F32");
      NEED(a->ne[0] == b->ne[0] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3], "mul_mat f32: shapes");
      NEED(n->ne[0] == a->ne[1] && n->ne[1] == b->ne[1] && n->ne[2] == a->ne[2] && n->ne[3] == b->ne[3],
           "mul_mat f32: dst shape");
      char *da = dev_of_t(a), *db = dev_of_t(b), *dn = dev_of_t(n);
      NEED(da && db && dn, "mul_mat f32: operand outside the mirrored memory");
      if (a->nb[1] >= a->nb[0]) {  // ggml.c:4495-4534
        NEED(a->nb[0] == 4 && b->nb[0] == 4 && n->nb[0] == 4, "mul_mat f32: rows must be contiguous");
        if (dry) return VSIM_OK;
        return launch_g_mm_dot(gt(n, dn), gt(a, da), gt(b, db), a->ne[0], s);
      }
      // ggml.c:4535-4581 + FINALIZE 4469-4493
      NEED(a->nb[1] == 4 && contiguous(n), "mul_mat f32 (transposed src0): src0 dim-1 stride 4, dst contiguous");
      if (dry) return VSIM_OK;
      return launch_g_mm_mad((float *)dn, gt(a, da), gt(b, db), b->ne[0], nth, n->ne[0], n->ne[1], n->ne[2], n->ne[3],
                             s);
    }
    default:
      return fail("unsupported op", n);
  }
}

// ------------------------------------------------------------------ decode fast path
// gptneox_eval (vsim.cpp:470-747) for one token with use_parallel_residual = 1, in the node
// order ggml_build_forward_expand gives it.  With N = 1 every ggml_repeat of a [E] vector onto
// a [E, 1] row returns the vector itself (same shape), so the biases and LayerNorm factors are
// direct operands.  get_rows; per layer 42 nodes
//   +0..2   norm(inpL), mul(ln1_w, .), add(., ln1_b)                      -> cur
//   +3..6   mul_mat(wk, cur), add(., bk); view(memory_k), cpy             (K row to the cache)
//   +7..10  mul_mat(wv, cur), add(., bv); view(memory_v), cpy             (V row to the cache)
//   +11..13 view(memory_v), reshape, permute                              -> V_trans
//   +14..17 view(memory_k), reshape, gptneox_rope(mode 1), permute        -> K
//   +18..22 mul_mat(wq, cur), add(., bq), cpy, gptneox_rope(mode 0), permute -> Q
//   +23..26 mul_mat(K, Q), scale, diag_mask_inf, soft_max
//   +27..29 mul_mat(V_trans, KQ_soft_max), permute, cpy                   -> merged heads
//   +30..31 mul_mat(wo, .), add(bo, .)                                    -> attn
//   +32..34 norm(inpL), mul(ln2_w, .), add(., ln2_b)                      -> inpFF
//   +35..37 mul_mat(wfc, .), add(bfc, .), gelu
//   +38..39 mul_mat(wproj, .), add(bproj, .)                              -> ff
//   +40..41 add(attn, ff), add(inpL, .)                                   -> inpL
// then norm, mul, add (ln_f) and mul_mat(lm_head) as the last node.
constexpr int NEOX_LAYER_NODES = 42, NEOX_HEAD_NODES = 4;

struct NeoxLayer {
  const ggml_tensor *ln1_w, *ln1_b, *ln2_w, *ln2_b, *wq, *bq, *wk, *bk, *wv, *bv, *wo, *bo, *wfc, *bfc, *wproj,
      *bproj;
};
struct NeoxMatch {
  vsim_graph_match_info info{};
  float scale = 0.0f;
  const ggml_tensor *wte = nullptr, *lnf_w = nullptr, *lnf_b = nullptr, *lmh = nullptr, *memk = nullptr,
                    *memv = nullptr;
  std::vector<NeoxLayer> layers;
};

bool match_neox_decode(const ggml_cgraph *g, NeoxMatch &M, std::string &why) {
  const int nn = g->n_nodes;
  auto node = [&](int i) -> const ggml_tensor * { return i >= 0 && i < nn ? g->nodes[i] : nullptr; };
  auto leaf = [](const ggml_tensor *t) { return t && t->op == GGML_OP_NONE && t->data; };
  auto flat = [](const ggml_tensor *t) { return t->ne[2] == 1 && t->ne[3] == 1; };
  auto is = [](const ggml_tensor *t, int op) { return t && t->op == op; };
  int E = 0, V = 0, H = 0, d = 0, P = -1, n_rot = -1;
  auto vec = [&](const ggml_tensor *t, int n) {
    return leaf(t) && t->type == GGML_TYPE_F32 && t->ne[0] == n && t->ne[1] == 1 && flat(t);
  };
  auto mat = [&](const ggml_tensor *t, int K, int R) {
    return leaf(t) && t->type == GGML_TYPE_Q4_0 && t->ne[0] == K && t->ne[1] == R && flat(t);
  };
  auto row = [](const ggml_tensor *t, int n) { return t->type == GGML_TYPE_F32 && t->ne[0] == n && t->ne[1] == 1; };
#define REQ(c, msg)  \
  do {               \
    if (!(c)) {      \
      why = msg;     \
      return false;  \
    }                \
  } while (0)
  // LayerNorm + affine at nodes i..i+2: norm(x), mul(w, .), add(., b)
  auto ln = [&](int i, const ggml_tensor *x, const ggml_tensor *&w, const ggml_tensor *&b) {
    const ggml_tensor *a = node(i), *m = node(i + 1), *s = node(i + 2);
    if (!(is(a, GGML_OP_NORM) && a->src0 == x && row(a, E) && is(m, GGML_OP_MUL) && m->src1 == a && vec(m->src0, E) &&
          is(s, GGML_OP_ADD) && s->src0 == m && vec(s->src1, E)))
      return false;
    w = m->src0;
    b = s->src1;
    return true;
  };
  // Q4_0 linear + bias at nodes i..i+1 (the bias add in either operand order)
  auto lin = [&](int i, const ggml_tensor *x, int K, int R, const ggml_tensor *&W, const ggml_tensor *&b) {
    const ggml_tensor *mm = node(i), *s = node(i + 1);
    if (!(is(mm, GGML_OP_MUL_MAT) && mm->src1 == x && mat(mm->src0, K, R) && row(mm, R) && is(s, GGML_OP_ADD)))
      return false;
    const ggml_tensor *bias = s->src0 == mm ? s->src1 : s->src1 == mm ? s->src0 : nullptr;
    if (!vec(bias, R)) return false;
    W = mm->src0;
    b = bias;
    return true;
  };
  auto i32s = [](const ggml_tensor *t, int n) {
    return t && t->op == GGML_OP_NONE && t->data && t->type == GGML_TYPE_I32 && t->ne[0] == n && t->ne[1] == 1;
  };
  auto both = [](const ggml_tensor *s, const ggml_tensor *a, const ggml_tensor *b) {
    return (s->src0 == a && s->src1 == b) || (s->src0 == b && s->src1 == a);
  };
  auto cache_view = [&](const ggml_tensor *v, long n) {
    return is(v, GGML_OP_VIEW) && leaf(v->src0) && v->src0->type == GGML_TYPE_F32 && v->src0->ne[1] == 1 &&
           flat(v->src0) && v->ne[0] == n && v->ne[1] == 1;
  };
  const ggml_tensor *n0 = node(0);
  REQ(is(n0, GGML_OP_GET_ROWS), "first node is not get_rows");
  REQ(leaf(n0->src0) && n0->src0->type == GGML_TYPE_Q4_0 && flat(n0->src0) && i32s(n0->src1, 1),
      "get_rows: not one token of a Q4_0 table");
  M.wte = n0->src0;
  E = M.wte->ne[0];
  V = M.wte->ne[1];
  const int F = 4 * E;
  M.info.token = *(const int32_t *)n0->src1->data;
  const ggml_tensor *inpL = n0;
  std::vector<long> koff, kvoff;  // per layer: K-row view and K-range view offsets (floats)
  int i = 1;
  while (i + NEOX_HEAD_NODES < nn) {
    NeoxLayer Y{};
    REQ(ln(i, inpL, Y.ln1_w, Y.ln1_b), "layer: input LayerNorm");
    const ggml_tensor *cur = node(i + 2);
    REQ(lin(i + 3, cur, E, E, Y.wk, Y.bk), "layer: key projection");
    const ggml_tensor *vk = node(i + 5), *ck = node(i + 6);
    REQ(cache_view(vk, E) && is(ck, GGML_OP_CPY) && ck->src0 == node(i + 4) && ck->src1 == vk,
        "layer: K row into memory_k");
    REQ(lin(i + 7, cur, E, E, Y.wv, Y.bv), "layer: value projection");
    const ggml_tensor *vv = node(i + 9), *cv = node(i + 10);
    REQ(cache_view(vv, E) && is(cv, GGML_OP_CPY) && cv->src0 == node(i + 8) && cv->src1 == vv,
        "layer: V row into memory_v");
    if (!M.memk) {
      M.memk = vk->src0;
      M.memv = vv->src0;
    }
    REQ(vk->src0 == M.memk && vv->src0 == M.memv && M.memk != M.memv && M.memk->ne[0] == M.memv->ne[0],
        "layer: one memory_k / memory_v");
    const ggml_tensor *a = node(i + 11), *b = node(i + 12), *c = node(i + 13);
    REQ(is(a, GGML_OP_VIEW) && a->src0 == M.memv && is(b, GGML_OP_RESHAPE) && b->src0 == a && is(c, GGML_OP_PERMUTE) &&
            c->src0 == b && b->ne[0] * b->ne[1] == E && a->ne[0] == (long)E * b->ne[2],
        "layer: V_trans view");
    if (!d) {
      d = b->ne[0];
      H = b->ne[1];
    }
    REQ(b->ne[0] == d && b->ne[1] == H, "layer: head shape");
    const int nk = b->ne[2];  // n_past + 1
    const ggml_tensor *vt = c, *vtv = a;
    a = node(i + 14), b = node(i + 15), c = node(i + 16);
    const ggml_tensor *kp = node(i + 17);
    REQ(is(a, GGML_OP_VIEW) && a->src0 == M.memk && a->ne[0] == (long)E * nk && is(b, GGML_OP_RESHAPE) && b->src0 == a &&
            b->ne[0] == d && b->ne[1] == H && b->ne[2] == nk && is(c, GGML_OP_GPTNEOX_ROPE) && c->src0 == b &&
            i32s(c->src1, 3) && is(kp, GGML_OP_PERMUTE) && kp->src0 == c,
        "layer: K range view + rope");
    const int32_t *kr = (const int32_t *)c->src1->data;
    if (P < 0) {
      P = kr[0];
      n_rot = kr[1];
    }
    REQ(kr[0] == P && kr[1] == n_rot && kr[2] == 1 && nk == P + 1, "layer: K rope parameters");
    koff.push_back(((const char *)vk->data - (const char *)M.memk->data) / 4);
    kvoff.push_back(((const char *)a->data - (const char *)M.memk->data) / 4);
    REQ(((const char *)vv->data - (const char *)M.memv->data) / 4 == koff.back() &&
            ((const char *)vtv->data - (const char *)M.memv->data) / 4 == kvoff.back(),
        "layer: K / V cache offsets differ");
    REQ(lin(i + 18, cur, E, E, Y.wq, Y.bq), "layer: query projection");
    a = node(i + 20), b = node(i + 21), c = node(i + 22);
    REQ(is(a, GGML_OP_CPY) && a->src0 == node(i + 19) && leaf(a->src1) && a->src1->ne[0] == d && a->src1->ne[1] == H &&
            a->src1->ne[2] == 1 && is(b, GGML_OP_GPTNEOX_ROPE) && b->src0 == a && i32s(b->src1, 3) &&
            is(c, GGML_OP_PERMUTE) && c->src0 == b,
        "layer: Q copy + rope");
    const int32_t *qr = (const int32_t *)b->src1->data;
    REQ(qr[0] == P && qr[1] == n_rot && qr[2] == 0, "layer: Q rope parameters");
    const ggml_tensor *qp = c;
    a = node(i + 23), b = node(i + 24), c = node(i + 25);
    const ggml_tensor *sm = node(i + 26);
    REQ(is(a, GGML_OP_MUL_MAT) && a->src0 == kp && a->src1 == qp && is(b, GGML_OP_SCALE) && b->src0 == a &&
            leaf(b->src1) && b->src1->type == GGML_TYPE_F32 && b->src1->ne[0] == 1 && is(c, GGML_OP_DIAG_MASK_INF) &&
            c->src0 == b && i32s(c->src1, 1) && *(const int32_t *)c->src1->data == P && is(sm, GGML_OP_SOFT_MAX) &&
            sm->src0 == c,
        "layer: KQ, scale, mask, soft_max");
    const float sc = *(const float *)b->src1->data;
    if (M.scale == 0.0f) M.scale = sc;
    REQ(sc == M.scale && sc != 0.0f, "layer: attention scale");
    a = node(i + 27), b = node(i + 28), c = node(i + 29);
    REQ(is(a, GGML_OP_MUL_MAT) && a->src0 == vt && a->src1 == sm && is(b, GGML_OP_PERMUTE) && b->src0 == a &&
            is(c, GGML_OP_CPY) && c->src0 == b && leaf(c->src1) && c->src1->ne[0] == E && c->src1->ne[1] == 1,
        "layer: KQV and head merge");
    REQ(lin(i + 30, c, E, E, Y.wo, Y.bo), "layer: output projection");
    const ggml_tensor *attn = node(i + 31);
    REQ(ln(i + 32, inpL, Y.ln2_w, Y.ln2_b), "layer: post-attention LayerNorm (parallel residual)");
    REQ(lin(i + 35, node(i + 34), E, F, Y.wfc, Y.bfc), "layer: fc_in");
    a = node(i + 37);
    REQ(is(a, GGML_OP_GELU) && a->src0 == node(i + 36), "layer: gelu");
    REQ(lin(i + 38, a, F, E, Y.wproj, Y.bproj), "layer: fc_out");
    a = node(i + 40), b = node(i + 41);
    REQ(is(a, GGML_OP_ADD) && both(a, attn, node(i + 39)) && is(b, GGML_OP_ADD) && both(b, inpL, a),
        "layer: residual joins");
    inpL = b;
    M.layers.push_back(Y);
    i += NEOX_LAYER_NODES;
  }
  const int L = (int)M.layers.size();
  REQ(L > 0 && i + NEOX_HEAD_NODES == nn, "node count is not 1 + 42 * n_layer + 4");
  REQ(ln(i, inpL, M.lnf_w, M.lnf_b), "final LayerNorm");
  const ggml_tensor *lm = node(i + 3);
  REQ(is(lm, GGML_OP_MUL_MAT) && lm->src1 == node(i + 2) && mat(lm->src0, E, V) && row(lm, V), "lm_head");
  M.lmh = lm->src0;
  // the cache: memory_k = [n_layer][n_ctx][E] floats (vsim.cpp:357-361), rows at (il*n_ctx + n_past)*E
  const long total = M.memk->ne[0];
  REQ(total % ((long)L * E) == 0, "memory_k size is not n_layer * n_ctx * n_embd");
  const int n_ctx = (int)(total / ((long)L * E));
  for (int il = 0; il < L; ++il)
    REQ(koff[il] == ((long)il * n_ctx + P) * E && kvoff[il] == (long)il * n_ctx * E, "KV cache offsets of a layer");
  REQ(P >= 0 && P + 1 <= n_ctx, "n_past outside the cache");
  REQ(n_rot > 0 && n_rot <= d && n_rot % 2 == 0 && E % 128 == 0, "shape outside the fused step's range");
  M.info.n_layer = L;
  M.info.n_embd = E;
  M.info.n_head = H;
  M.info.n_rot = n_rot;
  M.info.n_vocab = V;
  M.info.n_ctx = n_ctx;
  M.info.n_past = P;
#undef REQ
  return true;
}

// what a plan is bound to: every matched weight and the cache - each tensor struct and its
// data pointer, so a tensor whose struct stays put while its data moves takes a new plan (and
// the per-node path's re-registration) instead of the stale mirrors
std::vector<const void *> plan_key(const NeoxMatch &M) {
  std::vector<const void *> k;
  auto add = [&](const ggml_tensor *t) {
    k.push_back(t);
    k.push_back(t ? t->data : nullptr);
  };
  for (const ggml_tensor *t : {M.wte, M.lmh, M.lnf_w, M.lnf_b, M.memk, M.memv}) add(t);
  for (const NeoxLayer &Y : M.layers)
    for (const ggml_tensor *t : {Y.ln1_w, Y.ln1_b, Y.ln2_w, Y.ln2_b, Y.wq, Y.bq, Y.wk, Y.bk, Y.wv, Y.bv, Y.wo, Y.bo,
                                 Y.wfc, Y.bfc, Y.wproj, Y.bproj})
      add(t);
  return k;
}

std::string layer_name(int il, const char *what) { return "gpt_neox.layers." + std::to_string(il) + "." + what; }

// Build the fast-path model on the mirrors of a matched graph (its leafs are registered).
int build_fast(const NeoxMatch &M, int nth) {
  drop_fast();
  std::map<std::string, void *> bw;
  bool ok = true;
  auto q4 = [&](const std::string &n, const ggml_tensor *t) {
    const Ext *e = q4_of(t);
    ok = ok && e;
    bw[n] = e ? e->w4 : nullptr;
  };
  auto f32 = [&](const std::string &n, const ggml_tensor *t) {
    char *p = dev_of_t(t);
    ok = ok && p;
    bw[n] = p;
  };
  q4("gpt_neox.embed_in.weight", M.wte);
  q4("embed_out.weight", M.lmh);
  f32("gpt_neox.final_layer_norm.weight", M.lnf_w);
  f32("gpt_neox.final_layer_norm.bias", M.lnf_b);
  for (int il = 0; il < (int)M.layers.size(); ++il) {
    const NeoxLayer &Y = M.layers[il];
    f32(layer_name(il, "input_layernorm.weight"), Y.ln1_w);
    f32(layer_name(il, "input_layernorm.bias"), Y.ln1_b);
    f32(layer_name(il, "post_attention_layernorm.weight"), Y.ln2_w);
    f32(layer_name(il, "post_attention_layernorm.bias"), Y.ln2_b);
    q4(layer_name(il, "attention.query.weight"), Y.wq);
    f32(layer_name(il, "attention.query.bias"), Y.bq);
    q4(layer_name(il, "attention.key.weight"), Y.wk);
    f32(layer_name(il, "attention.key.bias"), Y.bk);
    q4(layer_name(il, "attention.value.weight"), Y.wv);
    f32(layer_name(il, "attention.value.bias"), Y.bv);
    q4(layer_name(il, "attention.dense.weight"), Y.wo);
    f32(layer_name(il, "attention.dense.bias"), Y.bo);
    q4(layer_name(il, "mlp.dense_h_to_4h.weight"), Y.wfc);
    f32(layer_name(il, "mlp.dense_h_to_4h.bias"), Y.bfc);
    q4(layer_name(il, "mlp.dense_4h_to_h.weight"), Y.wproj);
    f32(layer_name(il, "mlp.dense_4h_to_h.bias"), Y.bproj);
  }
  float *kc = (float *)dev_of_t(M.memk), *vc = (float *)dev_of_t(M.memv);
  if (!ok || !kc || !vc) {
    set_error("graph fast path: a matched tensor has no device mirror");
    return VSIM_EINVAL;
  }
  const vsim_graph_match_info &I = M.info;
  vsim_hparams hp{I.n_vocab, I.n_embd, I.n_head, I.n_layer, I.n_rot, 1};
  vsim_model *m = nullptr;
  if (int rc = model_create_impl(VSIM_ARCH_GPTNEOX, &hp, I.n_ctx, X.device, 0, I.n_layer, &bw, kc, vc, &m)) return rc;
  vsim_model_set_mode(m, VSIM_MODE_EXACT);
  vsim_model_set_graph(m, 1);
  X.fast.m = m;
  X.fast.key = plan_key(M);
  X.fast.gen = X.ext_gen;
  X.fast.nth = nth;
  X.fast.scale = M.scale;
  ++X.fast_plans;
  return VSIM_OK;
}

// One fused decode step of a matched graph on the current plan: the logits into the last node.
int run_fast(const ggml_cgraph *g, const NeoxMatch &M, int nth) {
  const int32_t tok = M.info.token;
  if (tok < 0 || tok >= M.info.n_vocab) {
    set_error("graph fast path: token id out of range");
    return VSIM_EINVAL;
  }
  ggml_tensor *last = g->nodes[g->n_nodes - 1];
  VSIM_HIP(hipStreamSynchronize(X.stream));  // mirrors uploaded on X.stream are complete
  if (int rc = model_set_attn(X.fast.m, nth, M.scale)) return rc;
  if (int rc = vsim_model_eval(X.fast.m, M.info.n_past, &tok, 1, nullptr, nullptr, (float *)last->data)) return rc;
  X.d2h += (uint64_t)M.info.n_vocab * sizeof(float);
  X.computes++;
  X.nodes += g->n_nodes;
  X.fast_evals++;
  return VSIM_OK;
}

struct GgmlContextHead {  // ggml.c:1022-1024, the first fields of struct ggml_context
  size_t mem_size;
  void *mem_buffer;
};

int compute(struct ggml_context *ctx, struct ggml_cgraph *g) {
  if (!ctx || !g) {
    set_error("graph_compute: null argument");
    return VSIM_EINVAL;
  }
  if (g->n_nodes <= 0) return VSIM_OK;
  if (int rc = ensure_ready()) return rc;
  VSIM_HIP(hipSetDevice(X.device));
  // an n_threads <= 0 graph runs with 8 threads in the reference (ggml.c:8246-8248)
  const int nth = g->n_threads > 0 ? g->n_threads : 8;
  // decode fast path: a recognised single-token gptneox_eval graph on the plan bound to its
  // tensors (built, after mirroring the leafs, when the weights, the cache or the mirrors change)
  const ggml_tensor *n0 = g->nodes[0];
  const bool one_token = !X.fast_off && !X.prof && n0->op == GGML_OP_GET_ROWS && n0->src1 && n0->src1->ne[0] == 1;
  NeoxMatch M;
  std::string why;
  const bool fast = one_token && match_neox_decode(g, M, why);
  if (fast && X.fast.m && X.fast.gen == X.ext_gen && X.fast.key == plan_key(M)) return run_fast(g, M, nth);
  if (one_token && !fast && getenv("VSIM_GRAPH_DEBUG"))
    fprintf(stderr, "vsim_graph_compute: per-node path (%s)\n", why.c_str());
  const GgmlContextHead *h = (const GgmlContextHead *)ctx;
  if (h->mem_buffer != X.arena_host || h->mem_size > X.arena_bytes) {
    if (X.arena_dev) (void)hipFree(X.arena_dev);
    X.arena_dev = nullptr;
    X.arena_host = nullptr;
    X.arena_bytes = 0;
    VSIM_HIP(hipMalloc((void **)&X.arena_dev, h->mem_size));
    X.arena_host = (const char *)h->mem_buffer;
    X.arena_bytes = h->mem_size;
  }
  // leafs: external ones mirrored once, arena ones uploaded now
  for (int i = 0; i < g->n_leafs; ++i) {
    const ggml_tensor *t = g->leafs[i];
    if (!t->data) continue;
    if (!in_arena(t->data)) {
      if (int rc = register_ext(t)) return rc;
    }
  }
  if (fast) {
    if (int rc = build_fast(M, nth)) return rc;
    return run_fast(g, M, nth);
  }
  for (int i = 0; i < g->n_nodes; ++i)
    if (int rc = node(g->nodes[i], nth, true)) return rc;
  for (int i = 0; i < g->n_leafs; ++i) {
    const ggml_tensor *t = g->leafs[i];
    if (t->data && in_arena(t->data)) {
      const size_t nb = span(t);
      VSIM_HIP(hipMemcpyAsync(X.arena_dev + ((const char *)t->data - X.arena_host), t->data, nb,
                              hipMemcpyHostToDevice, X.stream));
      X.h2d += nb;
    }
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (X.prof) {
    VSIM_HIP(hipEventCreate(&e0));
    VSIM_HIP(hipEventCreate(&e1));
  }
  for (int i = 0; i < g->n_nodes; ++i) {
    const ggml_tensor *t = g->nodes[i];
    if (X.prof) VSIM_HIP(hipEventRecord(e0, X.stream));
    if (int rc = node(t, nth, false)) return rc;
    if (X.prof) {
      VSIM_HIP(hipEventRecord(e1, X.stream));
      VSIM_HIP(hipEventSynchronize(e1));
      float ms = 0.0f;
      VSIM_HIP(hipEventElapsedTime(&ms, e0, e1));
      int k = (int)t->op;
      if (t->op == GGML_OP_MUL_MAT) k = t->src0->type == GGML_TYPE_Q4_0 ? PROF_MM_Q4 : PROF_MM_F32;
      if (k >= 0 && k < GGML_OP_COUNT + 2) {
        X.op[k].ms += ms;
        X.op[k].calls++;
      }
    }
  }
  if (X.prof) {
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  // the result: the last node's bytes back to its host address
  const ggml_tensor *last = g->nodes[g->n_nodes - 1];
  const size_t nb = span(last);
  char *dl = dev_of_t(last);
  if (!dl) return fail("result outside the mirrored memory", last);
  VSIM_HIP(hipMemcpyAsync(last->data, dl, nb, hipMemcpyDeviceToHost, X.stream));
  VSIM_HIP(hipStreamSynchronize(X.stream));
  X.d2h += nb;
  X.computes++;
  X.nodes += g->n_nodes;
  return VSIM_OK;
}

// monitor.c:182-262 row names for the ops the executor times
const char *op_name(int k) {
  static const char *names[GGML_OP_COUNT + 2] = {
      "NONE", "COMPUTE_FORWARD_DUP", "COMPUTE_FORWARD_ADD", "COMPUTE_FORWARD_SUB", "COMPUTE_FORWARD_MUL",
      "COMPUTE_FORWARD_DIV", "COMPUTE_FORWARD_SQR", "COMPUTE_FORWARD_SQRT", "COMPUTE_FORWARD_SUM",
      "COMPUTE_FORWARD_MEAN", "COMPUTE_FORWARD_REPEAT", "COMPUTE_FORWARD_ABS", "COMPUTE_FORWARD_SGN",
      "COMPUTE_FORWARD_NEG", "COMPUTE_FORWARD_STEP", "COMPUTE_FORWARD_RELU", "COMPUTE_FORWARD_GELU",
      "COMPUTE_FORWARD_SILU", "COMPUTE_FORWARD_NORM", "COMPUTE_FORWARD_MUL_MAT", "COMPUTE_FORWARD_SCALE",
      "COMPUTE_FORWARD_CPY", "COMPUTE_FORWARD_RESHAPE", "COMPUTE_FORWARD_VIEW", "COMPUTE_FORWARD_PERMUTE",
      "COMPUTE_FORWARD_TRANSPOSE", "COMPUTE_FORWARD_GET_ROWS", "COMPUTE_FORWARD_DIAG_MASK_INF",
      "COMPUTE_FORWARD_SOFT_MAX", "COMPUTE_FORWARD_ROPE", "COMPUTE_FORWARD_GPTNEOX_ROPE", "COMPUTE_FORWARD_ALIBI",
      "COMPUTE_FORWARD_CONV_1D_1S", "COMPUTE_FORWARD_CONV_1D_2S", "COMPUTE_FORWARD_FLASH_ATTN",
      "COMPUTE_FORWARD_FLASH_FF", "COMPUTE_FORWARD_MUL_MAT_Q4_0_F32", "COMPUTE_FORWARD_MUL_MAT_F32"};
  return k >= 0 && k < GGML_OP_COUNT + 2 ? names[k] : "?";
}

}  // namespace

extern "C" int vsim_graph_profile_report(char *buf, size_t cap);

namespace {
void print_profile_at_exit() {
  std::vector<char> buf(16384);
  if (vsim_graph_profile_report(buf.data(), buf.size()) > 0) {
    fputs(buf.data(), stdout);
    fflush(stdout);
  }
}
}  // namespace

extern "C" {

int vsim_graph_compute_rc(struct ggml_context *ctx, struct ggml_cgraph *cgraph) {
  std::lock_guard<std::mutex> lk(X.mu);
  return compute(ctx, cgraph);
}

void vsim_graph_compute(struct ggml_context *ctx, struct ggml_cgraph *cgraph) {
  if (vsim_graph_compute_rc(ctx, cgraph) != VSIM_OK) {
    // the reference's offload layer exits on what it cannot run (imax.c:2042-2049)
    printf("vsim_graph_compute: %s\n", vsim_last_error());
    fflush(stdout);
    exit(1);
  }
}

int vsim_graph_sync_tensor(const struct ggml_tensor *t) {
  std::lock_guard<std::mutex> lk(X.mu);
  if (!t || !X.ready) { set_error("graph_sync_tensor: nothing computed"); return VSIM_EINVAL; }
  char *d = dev_of_t(t);
  if (!d) { set_error("graph_sync_tensor: tensor outside the mirrored memory"); return VSIM_EINVAL; }
  VSIM_HIP(hipSetDevice(X.device));
  VSIM_HIP(hipMemcpy(t->data, d, span(t), hipMemcpyDeviceToHost));
  return VSIM_OK;
}

void vsim_graph_reset(void) {
  std::lock_guard<std::mutex> lk(X.mu);
  drop_fast();
  ++X.ext_gen;
  X.fast_evals = X.fast_plans = 0;
  for (auto &kv : X.ext) {
    if (kv.second.dev) (void)hipFree(kv.second.dev);
    if (kv.second.w4) (void)hipFree(kv.second.w4);
  }
  X.ext.clear();
  if (X.stream && hipSetDevice(X.device) == hipSuccess) (void)gemm_release_stream(X.stream);  // stream-K workspace
  if (X.arena_dev) (void)hipFree(X.arena_dev);
  X.arena_dev = nullptr;
  X.arena_host = nullptr;
  X.arena_bytes = 0;
  X.computes = X.nodes = X.h2d = X.d2h = 0;
  for (auto &o : X.op) o = OpProf{};
}

void vsim_graph_stats(uint64_t *computes, uint64_t *nodes, uint64_t *h2d_bytes, uint64_t *d2h_bytes) {
  std::lock_guard<std::mutex> lk(X.mu);
  if (computes) *computes = X.computes;
  if (nodes) *nodes = X.nodes;
  if (h2d_bytes) *h2d_bytes = X.h2d;
  if (d2h_bytes) *d2h_bytes = X.d2h;
}

int vsim_graph_match(const struct ggml_cgraph *cgraph, vsim_graph_match_info *info) {
  if (!cgraph || cgraph->n_nodes <= 0) { set_error("graph_match: empty graph"); return VSIM_EINVAL; }
  NeoxMatch M;
  std::string why;
  if (!match_neox_decode(cgraph, M, why)) {
    set_error("graph_match: " + why);
    return VSIM_EINVAL;
  }
  if (info) *info = M.info;
  return VSIM_OK;
}

void vsim_graph_fast_stats(uint64_t *fast_evals, uint64_t *plans) {
  std::lock_guard<std::mutex> lk(X.mu);
  if (fast_evals) *fast_evals = X.fast_evals;
  if (plans) *plans = X.fast_plans;
}

int vsim_graph_set_profile(int enable) {
  std::lock_guard<std::mutex> lk(X.mu);
  X.prof = enable != 0;
  for (auto &o : X.op) o = OpProf{};
  return VSIM_OK;
}

int vsim_graph_profile_report(char *buf, size_t cap) {
  std::lock_guard<std::mutex> lk(X.mu);
  if (!buf || cap == 0) { set_error("graph_profile_report: no buffer"); return VSIM_EINVAL; }
  double tot = 0.0;
  for (int k = 0; k < GGML_OP_COUNT + 2; ++k)
    if (k != GGML_OP_MUL_MAT) tot += X.op[k].ms;
  std::string out;
  char line[160];
  snprintf(line, sizeof line, "%-54s: %10s %7s %8s\n", "device time per op (vsim_graph_compute)", "ms", "share", "calls");
  out += line;
  for (int k = 0; k < GGML_OP_COUNT + 2; ++k) {
    if (!X.op[k].calls) continue;
    snprintf(line, sizeof line, "%-54s: %10.3f %6.1f%% %8ld\n", op_name(k), X.op[k].ms,
             tot > 0 ? 100.0 * X.op[k].ms / tot : 0.0, X.op[k].calls);
    out += line;
  }
  snprintf(line, sizeof line, "%-54s: %10.3f %6.1f%%\n", "COMPUTE_NODES (sum)", tot, 100.0);
  out += line;
  const size_t n = std::min(cap - 1, out.size());
  memcpy(buf, out.data(), n);
  buf[n] = 0;
  return (int)out.size();
}

}  // extern "C"
