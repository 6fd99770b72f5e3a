/* oracle/graph_probe.c -- TEST INFRASTRUCTURE ONLY (tests/test_graph_match_cpu.py).
 *
 * The reference's vsim.cpp is compiled with -Dggml_graph_compute=probe_compute and linked with
 * this file: every graph the reference's eval loop builds (vsim.cpp:470-747) is first shown to
 * libvsim_hip.so's host-only matcher (vsim_graph_match, the recogniser of the graph executor's
 * decode fast path), which prints one line per graph, and then computed by the reference's own
 * CPU executor (ggml_graph_compute, ggml.c:8245), so the run needs no GPU. */
#include <pthread.h>
#include <signal.h>
#include <stdio.h>

#include "ggml.h"
#include "../include/vsim_hip.h"

void ggml_graph_compute(struct ggml_context *ctx, struct ggml_cgraph *cgraph);

void probe_compute(struct ggml_context *ctx, struct ggml_cgraph *g) {
  vsim_graph_match_info info;
  if (vsim_graph_match(g, &info) == 0)
    printf("\nGRAPHMATCH layers=%d embd=%d head=%d rot=%d vocab=%d ctx=%d past=%d token=%d nodes=%d\n", info.n_layer,
           info.n_embd, info.n_head, info.n_rot, info.n_vocab, info.n_ctx, info.n_past, info.token, g->n_nodes);
  else
    printf("\nGRAPHNOMATCH nodes=%d (%s)\n", g->n_nodes, vsim_last_error());
  fflush(stdout);
  ggml_graph_compute(ctx, g);
}
