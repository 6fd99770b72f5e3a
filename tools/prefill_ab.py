#!/usr/bin/env python3
"""Prompt-eval logits of one library build, for A/B bit-identity of prefill changes (GPU).
  VSIM_LIB=a.so python3 tools/prefill_ab.py --out a.npz; ... --compare a.npz b.npz"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="small-gptj")
    ap.add_argument("--n", type=int, default=96)
    ap.add_argument("--file", action="store_true", help="weights from a generated ggml file instead of randomize()")
    ap.add_argument("--exact", action="store_true")
    ap.add_argument("--first-exact", action="store_true", help="first eval in exact mode, second in fast")
    ap.add_argument("--n2", type=int, default=16, help="tokens of the second eval")
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        a, b = (np.load(f)["logits"] for f in args.compare)
        same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
        h = a.size // 2
        print(f"prefill logits bit-identical: {same}  max|diff| {np.abs(a - b).max():.3g} "
              f"(first eval {np.abs(a[:h] - b[:h]).max():.3g}, second {np.abs(a[h:] - b[h:]).max():.3g})")
        sys.exit(0 if same else 1)
    from vsim_amd import hip
    from vsim_amd import modelgen as mg
    arch_s, hp = mg.CONFIGS[args.config]
    arch = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX, "bloom": hip.ARCH_BLOOM}[arch_s]
    if args.file:
        import tempfile
        path = os.path.join(tempfile.mkdtemp(), "pf.bin")
        mg.write_model(path, arch_s, hp, seed=5, std=0.05)
        m = hip.Model.load(path, arch)
    else:
        m = hip.Model.create(arch, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                        n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual), n_ctx=512)
        m.randomize(seed=5, std=0.05)
    m.set_mode(hip.MODE_EXACT if args.exact else hip.MODE_FAST)
    ids = [(7 * i + 3) % hp.n_vocab for i in range(args.n)]
    if args.first_exact:
        m.set_mode(hip.MODE_EXACT)
    lg = m.eval(0, ids)
    m.set_mode(hip.MODE_EXACT if args.exact else hip.MODE_FAST)
    lg2 = m.eval(args.n, [ids[0]] * args.n2)  # a second batch on top of the cache
    np.savez(args.out, logits=np.concatenate([lg, lg2]).astype(np.float32))
    print("saved", args.out)


if __name__ == "__main__":
    main()
