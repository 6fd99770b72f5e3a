#!/usr/bin/env python3
"""Generate the committed golden fixtures (run in the build container, where
/root/reference exists).  NOT run by the test-suite.

* ops_*.npz   — per-op vectors: seeded inputs + outputs of the REFERENCE's own ggml ops
                (oracle/_ref/ref_harness = our driver linked against the reference
                ggml.o/imax.o compiled from /root/reference, --threads 1).
* e2e.json    — end-to-end vectors from the unmodified reference CLI
                (oracle/_ref/vsim-ref, gptneox, --threads 1) on deterministic synthetic
                model files: `--return_logits` rows (%.8f text) and token streams
                (greedy and sampled), plus the sha256 of each generated model file so
                the tests can prove they regenerated the identical input.

Usage:  make -C oracle ref && python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
from vsim_amd import modelgen as mg  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
VSIM = os.path.join(ROOT, "oracle", "_ref", "vsim-ref")
OUT = os.path.dirname(os.path.abspath(__file__))
TMP = tempfile.mkdtemp(prefix="vsim_golden_")


def tmp(name):
    return os.path.join(TMP, name)


def harness(*args):
    subprocess.run([HARNESS, *[str(a) for a in args]], check=True)


def fread(path, dtype):
    return np.fromfile(path, dtype=dtype)


def activ(rng, n, scale=1.0):
    """Activation-like values incl. tiny magnitudes and exact zeros."""
    x = rng.standard_normal(n).astype(np.float32) * np.float32(scale)
    x[rng.integers(0, n, size=max(1, n // 97))] = 0.0
    tiny = rng.integers(0, n, size=max(1, n // 61))
    x[tiny] *= np.float32(1e-7)
    return x.astype(np.float32)


def gen_ops():
    rng = np.random.Generator(np.random.PCG64(1234))

    # quantize_row_q4_0 — random rows + hand-built edge blocks
    K = 4096
    x = activ(rng, K, 3.0)
    edge = np.zeros(32 * 6, np.float32)
    edge[32:64] = np.array([7, 2.5, -2.5, 3.5, -3.5, 0.5, -0.5, 1.5] * 4, np.float32)  # ties
    edge[64:96] = np.float32(1e-40)  # subnormals
    edge[96:128] = rng.standard_normal(32).astype(np.float32) * np.float32(1e30)
    edge[128:160] = -np.float32(5.0)
    edge[160:192] = np.linspace(-1, 1, 32).astype(np.float32)
    xs = np.concatenate([x, edge]).astype(np.float32)
    xs.tofile(tmp("q.in"))
    harness("qrow", xs.size, tmp("q.in"), tmp("q.out"))
    np.savez_compressed(os.path.join(OUT, "ops_qrow.npz"), x=xs, y=fread(tmp("q.out"), np.uint8))

    # Q4_0 x F32 mul_mat (activation re-quantization inside)
    cases = {}
    for ci, (M, K, N) in enumerate([(64, 64, 1), (256, 128, 1), (300, 256, 3), (128, 1024, 9),
                                    (200, 4096, 1), (32, 16384, 2)]):
        w = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.02))
        xa = activ(rng, N * K, 1.0)
        w.tofile(tmp("w")); xa.tofile(tmp("x"))
        harness("mulmat", M, K, N, tmp("w"), tmp("x"), tmp("y"))
        cases[f"c{ci}_shape"] = np.array([M, K, N], np.int32)
        cases[f"c{ci}_w"] = w
        cases[f"c{ci}_x"] = xa
        cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
    np.savez_compressed(os.path.join(OUT, "ops_mulmat.npz"), **cases)

    # LayerNorm
    cases = {}
    for ci, (n, r, sc) in enumerate([(128, 3, 1.0), (4096, 2, 0.05), (4096, 1, 30.0), (6144, 1, 1.0)]):
        xa = activ(rng, n * r, sc) + np.float32(0.3 * sc)
        xa.astype(np.float32).tofile(tmp("x"))
        harness("norm", n, r, tmp("x"), tmp("y"))
        cases[f"c{ci}_shape"] = np.array([n, r], np.int32)
        cases[f"c{ci}_x"] = xa.astype(np.float32)
        cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
    np.savez_compressed(os.path.join(OUT, "ops_norm.npz"), **cases)

    # GELU over every finite fp16 pattern's neighbourhood + random
    h = np.arange(65536, dtype=np.uint16).view(np.float16).astype(np.float32)
    h = h[np.isfinite(h)]
    h2 = (h * np.float32(1.0004)).astype(np.float32)
    h2 = h2[np.abs(h2) < 65000]  # the reference asserts !isinf on its output
    xa = np.concatenate([h, activ(rng, 8192, 4.0), h2]).astype(np.float32)
    xa.tofile(tmp("x"))
    harness("gelu", xa.size, tmp("x"), tmp("y"))
    np.savez_compressed(os.path.join(OUT, "ops_gelu.npz"), x=xa, y=fread(tmp("y"), np.float32))

    # scale -> diag_mask_inf -> soft_max (vsim.cpp:586-596)
    cases = {}
    for ci, (nc, nr, nz, n_past, sc) in enumerate([(7, 3, 4, 4, 0.17677669), (33, 1, 8, 32, 0.0625),
                                                    (9, 9, 2, 0, 0.125), (512, 1, 2, 511, 0.08838835)]):
        xa = (rng.standard_normal(nc * nr * nz) * 6).astype(np.float32)
        xa.tofile(tmp("x"))
        harness("attnsm", nc, nr, nz, n_past, repr(sc), tmp("x"), tmp("y"))
        cases[f"c{ci}_shape"] = np.array([nc, nr, nz, n_past], np.int32)
        cases[f"c{ci}_scale"] = np.array([sc], np.float32)
        cases[f"c{ci}_x"] = xa
        cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
    np.savez_compressed(os.path.join(OUT, "ops_attnsm.npz"), **cases)

    # RoPE, both styles, both modes
    for op in ("rope_neox", "rope_gptj"):
        cases = {}
        for ci, (d, H, T, n_past, n_dims, mode) in enumerate([(32, 4, 6, 3, 8, 0), (32, 4, 6, 3, 8, 1),
                                                               (256, 2, 5, 0, 64, 0), (64, 1, 300, 290, 64, 1),
                                                               (96, 3, 4, 500, 24, 0), (128, 2, 2, 1, 32, 1)]):
            xa = rng.standard_normal(d * H * T).astype(np.float32)
            xa.tofile(tmp("x"))
            harness(op, d, H, T, n_past, n_dims, mode, tmp("x"), tmp("y"))
            cases[f"c{ci}_shape"] = np.array([d, H, T, n_past, n_dims, mode], np.int32)
            cases[f"c{ci}_x"] = xa
            cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
        np.savez_compressed(os.path.join(OUT, f"ops_{op}.npz"), **cases)

    # KQ (double accumulator) and KQV (sequential float mad) on the cache views
    for op in ("kq", "kqv"):
        cases = {}
        for ci, (d, H, nk, N) in enumerate([(32, 4, 9, 3), (256, 2, 40, 1), (128, 2, 130, 1), (96, 2, 17, 9)]):
            kv = rng.standard_normal(d * H * nk).astype(np.float32)
            if op == "kq":
                other = rng.standard_normal(d * H * N).astype(np.float32)
            else:
                s = rng.random((H, N, nk)).astype(np.float32)
                other = (s / s.sum(-1, keepdims=True)).astype(np.float32).reshape(-1)
            kv.tofile(tmp("a")); other.tofile(tmp("b"))
            harness(op, d, H, nk, N, tmp("a"), tmp("b"), tmp("y"))
            cases[f"c{ci}_shape"] = np.array([d, H, nk, N], np.int32)
            cases[f"c{ci}_a"] = kv
            cases[f"c{ci}_b"] = other
            cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
        np.savez_compressed(os.path.join(OUT, f"ops_{op}.npz"), **cases)

    # get_rows on a Q4_0 embedding
    K, V = 256, 50
    w = mg.quantize_q4_0(rng.standard_normal(K * V).astype(np.float32) * np.float32(0.02))
    idx = np.array([0, 49, 7, 7, 13, 1, 2], np.int32)
    w.tofile(tmp("w")); idx.tofile(tmp("i"))
    harness("getrows", K, V, idx.size, tmp("w"), tmp("i"), tmp("y"))
    np.savez_compressed(os.path.join(OUT, "ops_getrows.npz"), shape=np.array([K, V], np.int32), w=w,
                        idx=idx, y=fread(tmp("y"), np.float32))


def gen_alibi():
    """scale -> ggml_alibi -> diag_mask_inf -> soft_max (the BLOOM score path; ggml_alibi
    requires nc == nr + n_past, ggml.c:6215)."""
    rng = np.random.Generator(np.random.PCG64(4321))
    cases = {}
    for ci, (nr, nz, n_past, sc) in enumerate([(3, 4, 4, 0.17677669), (1, 16, 40, 0.125), (9, 12, 0, 0.125),
                                                (1, 16, 300, 0.125), (5, 6, 7, 0.25)]):
        nc = nr + n_past
        xa = (rng.standard_normal(nc * nr * nz) * 6).astype(np.float32)
        xa.tofile(tmp("x"))
        harness("attnsm_alibi", nc, nr, nz, n_past, nz, repr(sc), tmp("x"), tmp("y"))
        cases[f"c{ci}_shape"] = np.array([nc, nr, nz, n_past], np.int32)
        cases[f"c{ci}_scale"] = np.array([sc], np.float32)
        cases[f"c{ci}_x"] = xa
        cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
    np.savez_compressed(os.path.join(OUT, "ops_attnsm_alibi.npz"), **cases)


def gen_prompt_mulmat():
    """Q4_0 x F32 mul_mat of the reference (ggml.c:4891-5165: INIT re-quantizes the N activation
    rows, COMPUTE the imax.c:1182-1230 dot chains) at prompt shapes, N >= 256 tokens: the cases of
    golden_util.PROMPT_MULMAT_CASES.  Stored: shape, seed, sha256 of the regenerated inputs, y."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_util as gu
    cases = {}
    for ci, (M, K, N, seed) in enumerate(gu.PROMPT_MULMAT_CASES):
        w, xa = gu.prompt_mulmat_inputs(M, K, N, seed)
        w.tofile(tmp("w")); xa.tofile(tmp("x"))
        harness("mulmat", M, K, N, tmp("w"), tmp("x"), tmp("y"))
        cases[f"c{ci}_shape"] = np.array([M, K, N, seed], np.int64)
        cases[f"c{ci}_sha"] = np.array(gu.inputs_sha(w, xa))
        cases[f"c{ci}_y"] = fread(tmp("y"), np.float32)
        print("prompt mulmat", M, K, N)
    np.savez_compressed(os.path.join(OUT, "ops_mulmat_prompt.npz"), **cases)


def run_vsim(model, prompt, extra):
    cmd = [VSIM, "gptneox", "-m", model, "--prompt", prompt, "--threads", "1", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, check=True)
    return r.stdout


def parse_logits(stdout):
    rows = [ln for ln in stdout.splitlines() if ln.startswith("logits:")]
    return [ln.split()[1:-1] if ln.rstrip().endswith("<END|>") else ln.split()[1:] for ln in rows]


def parse_tokens(stdout):
    s = stdout.split("<|BEGIN>", 1)[1].split("<END|>", 1)[0]
    return [int(t) for t in s.split()]


MODELS = {
    # name: (config, seed, std)
    "tiny-neox": ("tiny-neox", 0, 0.02),
    "tiny-neox-hot": ("tiny-neox", 1, 0.08),  # larger weights: sharper logits
    "small-neox": ("small-neox", 0, 0.02),
}
PROMPTS = ["1 2 3 4", "50 12 2 0 7 99 100 3 3 4 5 6", "5", "7 7 7 7 7 7 7 7 7 7 7 7 7 7 7 7 7 7 7 21"]


def gen_e2e():
    out = {"models": {}}
    for name, (cfg, seed, std) in MODELS.items():
        arch, hp = mg.CONFIGS[cfg]
        path = tmp(name + ".bin")
        mg.write_model(path, arch, hp, seed=seed, std=std)
        sha = hashlib.sha256(open(path, "rb").read()).hexdigest()
        ent = {"config": cfg, "seed": seed, "std": std, "sha256": sha, "logits": {}, "greedy": {}, "sampled": {}}
        for p in PROMPTS:
            if any(int(t) >= hp.n_vocab for t in p.split()):
                continue
            rows = parse_logits(run_vsim(path, p, ["--return_logits"]))
            ent["logits"][p] = rows[-1]
            g = run_vsim(path, p, ["--n_predict", "24", "--top_k", "1", "--top_p", "1.0", "--temp", "1.0",
                                   "--repeat_penalty", "1.0", "--seed", "42"])
            ent["greedy"][p] = parse_tokens(g)
            s = run_vsim(path, p, ["--n_predict", "24", "--top_k", "20", "--top_p", "0.95", "--temp", "0.85",
                                   "--repeat_last_n", "64", "--repeat_penalty", "1.3", "--seed", "42"])
            ent["sampled"][p] = parse_tokens(s)
        out["models"][name] = ent
        print(name, sha[:12], {p: len(v) for p, v in ent["greedy"].items()})
    with open(os.path.join(OUT, "e2e.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    for b in (HARNESS, VSIM):
        if not os.path.exists(b):
            sys.exit(f"missing {b}: run `make -C oracle ref` first")
    if sys.argv[1:] == ["alibi"]:  # (added later: regenerates only the ALiBi vectors)
        gen_alibi()
        sys.exit(0)
    if sys.argv[1:] == ["prompt_mulmat"]:  # (added in r03: only the prompt-shape mul_mat vectors)
        gen_prompt_mulmat()
        sys.exit(0)
    gen_ops()
    gen_alibi()
    gen_prompt_mulmat()
    gen_e2e()
    print("fixtures written to", OUT)
