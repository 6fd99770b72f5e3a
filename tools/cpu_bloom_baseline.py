#!/usr/bin/env python3
"""BASELINE.json configs[0]: bloom-560m Q4_0 greedy decode, 128 tokens, on the CPU ggml.c path.

The reference's own CLI cannot run BLOOM (vsim.cpp exits on `bloom`, SURVEY.md finding 2); its
CPU path for this config is therefore the composition of the reference's ggml ops that the
oracle restates (oracle/vsim_oracle.cpp, pinned op by op to the reference's outputs, ALiBi
included: tests/golden/ops_attnsm_alibi.npz).  This times that path: a synthetic bloom-560m
(the config's shapes, V = 250,880), the reference's run prompt, then 128 greedy decode tokens,
per-token wall time on this host's cores (all of the job's threads, and one), written as one
JSON line.  Usage: python tools/cpu_bloom_baseline.py [--tokens 128] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

PROMPT = [50278, 12092, 2, 0, 50281]


def run(hp, threads, n_tokens):
    m = O.Model(None, 2, n_ctx=len(PROMPT) + n_tokens + 1,
                synthetic=(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, 0, 7, 0.02))
    t0 = time.perf_counter()
    lg = m.eval(0, PROMPT, nthreads=threads)
    t_prompt = time.perf_counter() - t0
    tok, n_past, toks = int(np.argmax(lg)), len(PROMPT), []
    t0 = time.perf_counter()
    for _ in range(n_tokens):
        lg = m.eval(n_past, [tok], nthreads=threads)
        n_past += 1
        tok = int(np.argmax(lg))
        toks.append(tok)
    dt = time.perf_counter() - t0
    return {"threads": threads, "tokens": n_tokens, "decode_s": round(dt, 3), "tokens_per_s": round(n_tokens / dt, 3),
            "prompt_s": round(t_prompt, 3), "first_tokens": toks[:8]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=128)
    ap.add_argument("--tokens-1t", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    _, hp = mg.CONFIGS["bloom-560m"]
    nth = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        nth = min(nth, int(omp))
    model = ""
    with open("/proc/cpuinfo") as f:
        for ln in f:
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    line = {
        "metric": "bloom-560m Q4_0 greedy decode tokens/s, CPU ggml.c path (BASELINE.json configs[0])",
        "path": "oracle/vsim_oracle.cpp: the reference's ggml ops (ggml.c) composed into the BLOOM graph; "
                "the reference CLI has no BLOOM graph (vsim.cpp exits on bloom)",
        "data": "synthetic weights of bloom-560m's shapes (E=1024, H=16, L=24, V=250880), Q4_0",
        "host": {"model_name": model, "nproc": os.cpu_count(), "threads_used": nth},
        "all_threads": run(hp, nth, a.tokens),
        "one_thread": run(hp, 1, a.tokens_1t),
    }
    print(json.dumps(line), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
