#!/usr/bin/env python3
"""A/B bit-identity of two exact-mode decode schedules on a full-size synthetic model (GPU).

Run once per schedule (the VSIM_* switches are read once per process), e.g.
  VSIM_LAYER=0 python3 tools/layer_ab.py --out a.npz && VSIM_LAYER=1 python3 tools/layer_ab.py --out b.npz
  python3 tools/layer_ab.py --compare a.npz b.npz
Every schedule of exact mode must give the same greedy tokens and the same logits bits.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="gpt-j-6B")
    ap.add_argument("--steps", type=int, default=280)
    ap.add_argument("--layers", type=int, default=0, help="override n_layer (0: the config's)")
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        a, b = (np.load(f) for f in args.compare)
        same_tok = np.array_equal(a["tokens"], b["tokens"])
        same_log = np.array_equal(a["logits"].view(np.uint32), b["logits"].view(np.uint32))
        print(f"tokens identical: {same_tok}  logits bit-identical: {same_log}  "
              f"max|diff| {np.abs(a['logits'] - b['logits']).max():.3g}")
        sys.exit(0 if same_tok and same_log else 1)
    from vsim_amd import hip
    from vsim_amd import modelgen as mg
    arch_s, hp = mg.CONFIGS[args.config]
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    hpd = dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
               n_layer=args.layers or hp.n_layer, n_rot=hp.n_rot,
               use_parallel_residual=hp.use_parallel_residual)
    m = hip.Model.create(arch, hpd, n_ctx=512)
    m.randomize(seed=77, std=0.02)
    m.set_mode(hip.MODE_EXACT)
    m.set_graph(True)
    prompt = [t % hp.n_vocab for t in (50278, 12092, 2, 0, 50281)]  # (valid ids for small vocabs)
    m.eval(0, prompt, want_logits=False)
    toks = m.generate(len(prompt), prompt[-1], args.steps)
    logits = m.eval(len(prompt) + args.steps, [toks[-1]])
    np.savez(args.out, tokens=np.array(toks), logits=np.asarray(logits, np.float32))
    print("saved", args.out, "last tokens", toks[-5:])


if __name__ == "__main__":
    main()
