#!/usr/bin/env python3
"""Decode speed of the reference's own eval loop on the GPU (oracle/_ref/vsim-ubuntu.emax7nc:
vsim.cpp with ggml_graph_compute -> vsim_graph_compute, whose decode fast path runs the fused
step) against the whole-model CLI (vsim_amd/_build/vsim-hip), same synthetic model file, same
argv (greedy), both sampling on the host with the reference's sampler.

tokens/s = (B - A) / (t_B - t_A) from two runs of each binary with n_predict A and B, so load
time and the prompt cancel.  Usage: python tools/graph_speed.py [--layers 4] [--out FILE]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
from vsim_amd import modelgen as mg  # noqa: E402

GRAPH = os.path.join(ROOT, "oracle", "_ref", "vsim-ubuntu.emax7nc")
HIP = os.path.join(ROOT, "vsim_amd", "_build", "vsim-hip")
PROMPT = "50278 12092 2 0 50281"


def timed(exe, path, n, env=None):
    args = [exe, "gptneox", "-m", path, "--prompt", PROMPT, "--n_predict", str(n), "--top_k", "1", "--top_p", "1.0",
            "--temp", "1.0", "--repeat_penalty", "1.0", "--seed", "42", "--threads", "1"]
    t0 = time.perf_counter()
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{exe} failed: {r.stdout[-800:]} {r.stderr[-800:]}")
    toks = r.stdout.split("<|BEGIN>", 1)[1].split("<END|>", 1)[0].split()
    return dt, toks, r.stderr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--a", type=int, default=8)
    ap.add_argument("--b", type=int, default=488)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    arch, hp = mg.CONFIGS["pythia-12b"]
    hp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, a.layers, hp.n_rot, hp.use_parallel_residual)
    path = os.path.join(tempfile.gettempdir(), f"pythia-width-{a.layers}l.bin")
    if not os.path.exists(path):
        t0 = time.perf_counter()
        mg.write_model(path + ".tmp", arch, hp, seed=5, std=0.02)
        os.replace(path + ".tmp", path)
        print(f"model written in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    runs = {"graph": [], "vsim_hip": []}
    streams, stats = {}, []
    env = dict(os.environ, VSIM_GRAPH_STATS="1")
    for _ in range(a.reps):  # the two binaries alternate within each rep: the same box state for both
        for name, exe in (("graph", GRAPH), ("vsim_hip", HIP)):
            ta, _, _ = timed(exe, path, a.a, env)
            tb, toks, err = timed(exe, path, a.b, env)
            tps = (a.b - a.a) / (tb - ta)
            runs[name].append(tps)
            streams[name] = toks
            if name == "graph":
                stats = [ln for ln in err.splitlines() if "fast path" in ln][-1:]
            print(f"{name}: {tps:.1f} tok/s ({a.b - a.a} tokens in {tb - ta:.3f} s)", file=sys.stderr, flush=True)
    med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
    ratios = sorted(g / h for g, h in zip(runs["graph"], runs["vsim_hip"]))
    line = {
        "what": "decode tok/s, reference eval loop (vsim.cpp + ggml graph) on vsim_graph_compute vs vsim-hip",
        "model": f"pythia-12b width (E={hp.n_embd}, H={hp.n_head}, V={hp.n_vocab}), {a.layers} layers, synthetic",
        "tokens": a.b - a.a, "graph_tok_s": round(med["graph"], 2), "vsim_hip_tok_s": round(med["vsim_hip"], 2),
        "runs": {k: [round(x, 1) for x in v] for k, v in runs.items()},
        "statistic": f"median of {a.reps} alternating reps; ratio = median of the per-rep ratios",
        "ratio": round(ratios[len(ratios) // 2], 4), "ratio_min": round(ratios[0], 4),
        "streams_equal": streams["graph"] == streams["vsim_hip"], "graph_stats": stats,
    }
    print(json.dumps(line), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
