#!/usr/bin/env python3
"""Fast-mode decode of one library build, for A/B bit-identity of fast-path changes (GPU):
  VSIM_LIB=a.so python3 tools/fast_ab.py --out a.npz; ... --compare a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="gpt-j-6B")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        a, b = (np.load(f) for f in args.compare)
        st = np.array_equal(a["tokens"], b["tokens"])
        sl = np.array_equal(a["logits"].view(np.uint32), b["logits"].view(np.uint32))
        print(f"fast tokens identical: {st}  logits bit-identical: {sl}  max|diff| "
              f"{np.abs(a['logits'] - b['logits']).max():.3g}")
        sys.exit(0 if st and sl else 1)
    from vsim_amd import hip
    from vsim_amd import modelgen as mg
    arch_s, hp = mg.CONFIGS[args.config]
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    m = hip.Model.create(arch, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                    n_layer=args.layers or hp.n_layer, n_rot=hp.n_rot,
                                    use_parallel_residual=hp.use_parallel_residual), n_ctx=512)
    m.randomize(seed=21, std=0.02)
    m.set_mode(hip.MODE_FAST)
    m.set_graph(True)
    prompt = [t % hp.n_vocab for t in (50278, 12092, 2, 0, 50281)]
    m.eval(0, prompt, want_logits=False)
    toks = m.generate(len(prompt), prompt[-1], args.steps)
    lg = m.eval(len(prompt) + args.steps, [toks[-1]])
    np.savez(args.out, tokens=np.array(toks), logits=np.asarray(lg, np.float32))
    print("saved", args.out)


if __name__ == "__main__":
    main()
