#!/usr/bin/env python3
"""Fast-mode vs exact-mode logits on a full-size synthetic model (GPU).

Exact mode is bit-identical to the reference CPU path (tests/test_gpu_model.py), so this
measures how far the fast integer-dot GEMVs move the logits from the reference.  Both
models get the same device-drawn weights and are teacher-forced with the exact model's
greedy tokens, so every step compares the same inputs.  Reports, per step, the
north-star error max|l_fast - l_exact| / max|l_exact| and top-1 agreement.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="gpt-j-6B")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--std", type=float, default=0.02)
    args = ap.parse_args()
    arch_s, hp = mg.CONFIGS[args.config]
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    hpd = dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer, n_rot=hp.n_rot,
               use_parallel_residual=hp.use_parallel_residual)
    ms = {}
    for mode in (hip.MODE_EXACT, hip.MODE_FAST):
        m = hip.Model.create(arch, hpd, n_ctx=512)
        m.randomize(seed=args.seed, std=args.std)
        m.set_mode(mode)
        m.set_graph(True)
        ms[mode] = m
    prompt = [50278, 12092, 2, 0, 50281]
    n_past, ids = 0, prompt
    rel, agree = [], 0
    for step in range(args.steps + 1):
        le = ms[hip.MODE_EXACT].eval(n_past, ids)
        lf = ms[hip.MODE_FAST].eval(n_past, ids)
        r = float(np.max(np.abs(lf - le)) / np.max(np.abs(le)))
        rel.append(r)
        agree += int(np.argmax(le) == np.argmax(lf))
        n_past += len(ids)
        ids = [int(np.argmax(le))]
    out = {"config": args.config, "steps": len(rel), "max_rel_err": max(rel), "mean_rel_err": float(np.mean(rel)),
           "top1_agree": agree / len(rel), "per_step": [round(x, 8) for x in rel]}
    print(json.dumps(out))
    for m in ms.values():
        m.close()


if __name__ == "__main__":
    main()
