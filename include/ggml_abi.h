/* include/ggml_abi.h — the slice of the reference's ggml ABI that the drop-in entry
 * points of libvsim_hip.so receive.  Layouts must match the reference byte for byte:
 *   struct ggml_tensor          ggml.h:275-305
 *   enum ggml_type / ggml_op    ggml.h:217-272
 *   struct ggml_compute_params  ggml.c:1052-1060 (duplicated in imax.c:1115-1121)
 *   struct ggml_cgraph          ggml.h:308-324
 *   struct ggml_context         opaque in ggml.h:215; its first two fields (mem_size,
 *                               mem_buffer, ggml.c:1022-1024) are read by vsim_graph_compute
 * tests/test_capi.py checks offsetof/sizeof of every field against the values the
 * reference objects were compiled with.
 */
#ifndef VSIM_GGML_ABI_H
#define VSIM_GGML_ABI_H

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#define VSIM_GGML_MAX_DIMS 4
#define VSIM_GGML_MAX_OPT 4
#define VSIM_GGML_MAX_NODES 4096

/* A translation unit that already has the reference's own ggml.h (which defines GGML_MAX_DIMS,
 * ggml.h:202) takes the types from it; the layouts are the same. */
#ifndef GGML_MAX_DIMS
enum ggml_type {
  GGML_TYPE_Q4_0,
  GGML_TYPE_Q4_1,
  GGML_TYPE_I8,
  GGML_TYPE_I16,
  GGML_TYPE_I32,
  GGML_TYPE_F16,
  GGML_TYPE_F32,
  GGML_TYPE_COUNT,
};

/* Only the values the path dispatches on are named; the enum is the reference's
 * (ggml.h:230-272), so the numbering below must stay in step with it. */
enum ggml_op {
  GGML_OP_NONE = 0,
  GGML_OP_DUP, GGML_OP_ADD, GGML_OP_SUB, GGML_OP_MUL, GGML_OP_DIV, GGML_OP_SQR, GGML_OP_SQRT,
  GGML_OP_SUM, GGML_OP_MEAN, GGML_OP_REPEAT, GGML_OP_ABS, GGML_OP_SGN, GGML_OP_NEG, GGML_OP_STEP,
  GGML_OP_RELU, GGML_OP_GELU, GGML_OP_SILU, GGML_OP_NORM,
  GGML_OP_MUL_MAT,
  GGML_OP_SCALE, GGML_OP_CPY, GGML_OP_RESHAPE, GGML_OP_VIEW, GGML_OP_PERMUTE, GGML_OP_TRANSPOSE,
  GGML_OP_GET_ROWS, GGML_OP_DIAG_MASK_INF, GGML_OP_SOFT_MAX, GGML_OP_ROPE, GGML_OP_GPTNEOX_ROPE,
  GGML_OP_ALIBI, GGML_OP_CONV_1D_1S, GGML_OP_CONV_1D_2S, GGML_OP_FLASH_ATTN, GGML_OP_FLASH_FF,
  GGML_OP_COUNT,
};

struct ggml_tensor {
  enum ggml_type type;
  int n_dims;
  int ne[VSIM_GGML_MAX_DIMS];
  size_t nb[VSIM_GGML_MAX_DIMS];
  enum ggml_op op;
  bool is_param;
  struct ggml_tensor *grad;
  struct ggml_tensor *src0;
  struct ggml_tensor *src1;
  struct ggml_tensor *opt[VSIM_GGML_MAX_OPT];
  int n_tasks;
  int perf_runs;
  int64_t perf_cycles;
  int64_t perf_time_us;
  void *data;
  char padding[8];
};

struct ggml_cgraph {
  int n_nodes;
  int n_leafs;
  int n_threads;

  size_t work_size;
  struct ggml_tensor *work;

  struct ggml_tensor *nodes[VSIM_GGML_MAX_NODES];
  struct ggml_tensor *grads[VSIM_GGML_MAX_NODES];
  struct ggml_tensor *leafs[VSIM_GGML_MAX_NODES];

  int perf_runs;
  int64_t perf_cycles;
  int64_t perf_time_us;
};

struct ggml_context;
#endif /* GGML_MAX_DIMS */

enum ggml_task_type {
  GGML_TASK_INIT = 0,
  GGML_TASK_COMPUTE,
  GGML_TASK_FINALIZE,
};

struct ggml_compute_params {
  enum ggml_task_type type;
  int ith, nth;
  size_t wsize;
  void *wdata;
};

#endif /* VSIM_GGML_ABI_H */
