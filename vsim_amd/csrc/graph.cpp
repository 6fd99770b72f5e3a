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

int register_ext(const ggml_tensor *t) {
  const char *h = (const char *)t->data;
  const size_t bytes = span(t);
  auto it = X.ext.find(h);
  if (it != X.ext.end()) {
    if (it->second.bytes == bytes && it->second.type == (int)t->type && it->second.ne0 == t->ne[0] &&
        it->second.ne1 == t->ne[1])
      return VSIM_OK;
    if (it->second.dev) (void)hipFree(it->second.dev);
    if (it->second.w4) (void)hipFree(it->second.w4);
    X.ext.erase(it);
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
  // an n_threads <= 0 graph runs with 8 threads in the reference (ggml.c:8246-8248)
  const int nth = g->n_threads > 0 ? g->n_threads : 8;
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
  for (auto &kv : X.ext) {
    if (kv.second.dev) (void)hipFree(kv.second.dev);
    if (kv.second.w4) (void)hipFree(kv.second.w4);
  }
  X.ext.clear();
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
