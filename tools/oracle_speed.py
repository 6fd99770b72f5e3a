#!/usr/bin/env python3
"""Speed of the CPU oracle (oracle/vsim_oracle.cpp, bench.py's cpu_baseline) against the
reference binary itself (oracle/_ref/vsim-ref, compiled from /root/reference by
`make -C oracle ref`), on the same synthetic ggml file, in this container (SURVEY.md §8(d):
"its speed is cross-checked here against the reference binary on identical synthetic files;
report the ratio").

Workload: BASELINE.md §2's probe — one GPT-J-width GPT-NeoX layer (E=4096, F=16384) plus the
50400 x 4096 head, prompt 50278 12092 2 0 50281, greedy.  Decode time per token =
(t(n_predict=13) - t(n_predict=3)) / 10 for both (load and prompt cancel), at 1 thread and at
8 threads.  Tokens must agree at 1 thread (both follow vsim.cpp:749-910 at --threads 1).

Writes profiles/<tag>_oracle_vs_ref_speed.json.  Needs /root/reference (this container only).
"""
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from vsim_amd import modelgen as mg  # noqa: E402
import oracle_py as O  # noqa: E402

VSIM = os.path.join(ROOT, "oracle", "_ref", "vsim-ref")
PROMPT = [50278, 12092, 2, 0, 50281]
GREEDY = ["--top_k", "1", "--top_p", "1.0", "--temp", "1.0", "--repeat_penalty", "1.0", "--seed", "42"]


def ref_run(path, n, threads):
    cmd = [VSIM, "gptneox", "-m", path, "--prompt", " ".join(map(str, PROMPT)), "--threads", str(threads),
           "--n_predict", str(n), *GREEDY]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, check=True)
    dt = time.perf_counter() - t0
    toks = [int(t) for t in r.stdout.split("<|BEGIN>", 1)[1].split("<END|>", 1)[0].split()]
    return dt, toks


def oracle_run(path, n, threads):
    t0 = time.perf_counter()
    m = O.Model(path, 0, n_ctx=512)
    toks = m.generate(PROMPT, n, seed=42, top_k=1, top_p=1.0, temp=1.0, repeat_penalty=1.0, n_batch=8,
                      nthreads=threads)
    dt = time.perf_counter() - t0
    del m
    return dt, toks


def per_token(fn, path, threads, reps=2):
    best = None
    for _ in range(reps):
        a, ta = fn(path, 3, threads)
        b, tb = fn(path, 13, threads)
        v = (b - a) / 10.0
        best = v if best is None else min(best, v)
    return best, tb


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    if not os.path.exists(VSIM):
        sys.exit("missing oracle/_ref/vsim-ref: run `make -C oracle ref` first")
    hp = mg.HParams(50400, 4096, 32, 1, 32, 1)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "gptj_width_1layer.bin")
        mg.write_model(path, "gptneox", hp, seed=0, std=0.02)
        res = {}
        for th in (1, 8):
            r, rt = per_token(ref_run, path, th)
            o, ot = per_token(oracle_run, path, th)
            res[str(th)] = {"ref_ms_per_token": round(r * 1e3, 2), "oracle_ms_per_token": round(o * 1e3, 2),
                            "oracle_over_ref_speed": round(r / o, 3), "tokens_equal": rt == ot}
            print(th, res[str(th)], flush=True)
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    out = {
        "what": "decode ms/token, (t(n_predict=13) - t(n_predict=3)) / 10, best of 2",
        "workload": "GPT-NeoX file, E=4096 H=32 L=1 F=16384 V=50400 (one GPT-J-width layer + head), "
                    "prompt 50278 12092 2 0 50281, greedy",
        "reference": "oracle/_ref/vsim-ref (reference sources compiled by oracle/Makefile, -O2 -msse3)",
        "oracle": "oracle/_build/libvsim_oracle.so via tests/oracle_py.py (vo_generate)",
        "host": {"nproc": os.cpu_count(), "model_name": model, "machine": platform.machine()},
        "threads": res,
    }
    dst = os.path.join(ROOT, "profiles", f"{tag}_oracle_vs_ref_speed.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(dst)


if __name__ == "__main__":
    main()
