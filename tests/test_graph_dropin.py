"""The graph-level drop-in: the reference's own eval loop (vsim.cpp, ggml.c's graph builders)
with its one graph-executor call, vsim.cpp:725 `ggml_graph_compute(ctx0, &gf)`, bound to
vsim_graph_compute (oracle/Makefile `graphdrop`: vsim.cpp compiled with
-Dggml_graph_compute=vsim_graph_compute).  Every node of every eval - get_rows, norm,
repeat/mul/add, the Q4_0 mul_mats, the KV-cache cpy views, gptneox_rope on Q and on the cache
view, KQ, scale, diag_mask_inf, soft_max, KQV, the merge cpy, gelu, lm_head - runs on the GPU
from the device mirrors of the ggml arena and the model's tensors.

Checked against the reference binary built from the same sources (tests/golden/e2e.json at
--threads 1, and a live vsim-ref run at --threads 4, where the KQV thread partials change the
logits, SURVEY.md finding 3): the printed logits rows and token streams must be identical.
"""
import os
import re
import shutil
import subprocess

import pytest

from golden_util import e2e, model_path

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GRAPH = os.path.join(ROOT, "oracle", "_ref", "vsim-graph")
REFBIN = os.path.join(ROOT, "oracle", "_ref", "vsim-ref")


def run(exe, args, threads="1", env=None, stderr=False):
    if not os.path.exists(exe):
        pytest.skip(f"{os.path.relpath(exe, ROOT)} not built (make -C oracle ref graphdrop, needs /root/reference)")
    r = subprocess.run([exe, "gptneox", *args, "--threads", threads], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return (r.stdout, r.stderr) if stderr else r.stdout


def fast_stats(err):
    """(computes, fast-path evals, plans) from VSIM_GRAPH_STATS=1's line on stderr"""
    m = re.search(r"(\d+) computes, (\d+) on the decode fast path, (\d+) fast-path plans", err)
    assert m, err[-1000:]
    return tuple(int(v) for v in m.groups())


def logits_rows(out):
    return [ln.split()[1:] for ln in out.splitlines() if ln.startswith("logits:")]


def tokens(out):
    return [int(t) for t in out.split("<|BEGIN>", 1)[1].split("<END|>", 1)[0].split()]


GREEDY = ["--n_predict", "24", "--top_k", "1", "--top_p", "1.0", "--temp", "1.0", "--repeat_penalty", "1.0",
          "--seed", "42"]


@pytest.mark.parametrize("name", sorted(e2e()["models"]))
def test_graph_compute_matches_reference_logits(name):
    ent = e2e()["models"][name]
    path = model_path(name)
    for prompt, row in ent["logits"].items():
        out = run(GRAPH, ["-m", path, "--prompt", prompt, "--return_logits"])
        assert logits_rows(out)[-1][:-1] == row, prompt


@pytest.mark.parametrize("name", sorted(e2e()["models"]))
def test_graph_compute_matches_reference_streams(name):
    ent = e2e()["models"][name]
    path = model_path(name)
    for prompt, toks in ent["greedy"].items():
        assert tokens(run(GRAPH, ["-m", path, "--prompt", prompt, *GREEDY])) == toks, prompt
    for prompt, toks in list(ent["sampled"].items())[:2]:
        # tests/golden/make_golden.py's sampling arguments
        args = ["-m", path, "--prompt", prompt, "--n_predict", "24", "--top_k", "20", "--top_p", "0.95", "--temp",
                "0.85", "--repeat_last_n", "64", "--repeat_penalty", "1.3", "--seed", "42"]
        assert tokens(run(GRAPH, args)) == toks, prompt


@pytest.mark.parametrize("threads,fast,prompt", [
    ("2", "1", "50 12 2 0 7 99 100 3 3 4 5 6"), ("4", "1", "50 12 2 0 7 99 100 3 3 4 5 6"),
    ("2", "1", "50 12 2 0 7 99 100 3 3 4"), ("4", "1", "50 12 2 0 7 99 100 3 3 4"),
    ("7", "1", "50 12 2 0 7 99 100 3 3 4"), ("4", "0", "50 12 2 0 7 99 100 3 3 4")])
def test_graph_compute_follows_thread_grouping(threads, fast, prompt):
    """The reference's KQV sums per-thread partials (ggml.c:4535-4581, 4469-4493), so its logits
    depend on --threads; the device executor groups the same way from cgraph->n_threads and must
    equal the reference at every thread count.  vsim.cpp feeds the prompt in batches of
    n_batch + 1 = 9 (vsim.cpp:862-876): the 12-token prompt ends with a 3-token batch (per-node
    path), the 10-token one with a single token, whose graph runs on the decode fast path (the
    fused attention's KQV in the pool's key runs, 10 keys over 2, 4 and 7 threads: runs of 5, 3
    and 2 keys, 7 threads leaving 2 empty work rows) -- its logits row is the one printed."""
    name = "small-neox"
    path = model_path(name)
    args = ["-m", path, "--prompt", prompt, "--return_logits", "--n_predict", "6", "--top_k", "1"]
    ref = logits_rows(run(REFBIN, args, threads=threads))
    env = dict(os.environ, VSIM_GRAPH_FAST=fast, VSIM_GRAPH_STATS="1")
    out, err = run(GRAPH, args, threads=threads, env=env, stderr=True)
    got = logits_rows(out)
    computes, fast_evals, plans = fast_stats(err)
    want_fast = 1 if fast == "1" and len(prompt.split()) == 10 else 0
    assert (fast_evals, plans) == (want_fast, want_fast), err[-500:]
    assert len(got) == len(ref) >= 1
    assert got == ref
    one = logits_rows(run(REFBIN, args, threads="1"))
    if threads != "1":
        assert one != ref, "thread count no longer changes the reference's logits: the test lost its point"


def test_graph_compute_profile_report():
    """VSIM_GRAPH_PROFILE=1: per-op device time printed at exit with the reference's monitor row
    names (show_time_sep, monitor.c:196-262)."""
    name = sorted(e2e()["models"])[0]
    env = dict(os.environ, VSIM_GRAPH_PROFILE="1")
    out = run(GRAPH, ["-m", model_path(name), "--prompt", "1 2 3", "--n_predict", "2"], env=env)
    assert "<END|>" in out
    tail = out.split("<END|>", 1)[1]
    for row in ("COMPUTE_FORWARD_MUL_MAT_Q4_0_F32", "COMPUTE_FORWARD_MUL_MAT_F32", "COMPUTE_FORWARD_SOFT_MAX",
                "COMPUTE_FORWARD_GPTNEOX_ROPE", "COMPUTE_NODES (sum)"):
        assert row in tail, row


@pytest.mark.parametrize("name", sorted(e2e()["models"]))
def test_decode_graphs_take_the_fast_path(name):
    """Every single-token eval of the reference's loop runs as the fused decode step (one plan,
    one hipGraph replay per token); the greedy stream is still the reference's."""
    ent = e2e()["models"][name]
    prompt, want = next(iter(ent["greedy"].items()))
    env = dict(os.environ, VSIM_GRAPH_STATS="1")
    out, err = run(GRAPH, ["-m", model_path(name), "--prompt", prompt, *GREEDY], env=env, stderr=True)
    assert tokens(out) == want
    computes, fast_evals, plans = fast_stats(err)
    n_gen = len(want) - len(prompt.split())
    # the warm-up eval and the prompt batch(es) per node, every decode step (all samples but
    # the last are evaluated) on the fast path
    assert (fast_evals, plans) == (n_gen - 1, 1) and computes > fast_evals, err[-500:]


def test_interface_py_runs_the_installed_binary(tmp_path):
    """cformers/interface.py:204 spawns ../vsim-ubuntu.emax7nc from its working directory with
    the argv of interface.py:206-216 and reads the token stream after <|BEGIN> (interface.py:
    222-260).  `make -C oracle install REFROOT=...` puts the binary (the reference's own eval loop,
    its graph executor on the GPU) there; run it exactly that way and compare the sampled stream
    with the reference's (tests/golden/e2e.json, the same sampling arguments)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "vsim-ubuntu.emax7nc")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/vsim-ubuntu.emax7nc not built (make -C oracle emax7nc)")
    root = tmp_path / "vsim"
    (root / "cformers").mkdir(parents=True)
    shutil.copy(exe, root / "vsim-ubuntu.emax7nc")
    shutil.copy(os.path.join(ROOT, "vsim_amd", "_build", "libvsim_hip.so"), root / "libvsim_hip.so")
    name = "small-neox"
    ent = e2e()["models"][name]
    prompt, want = next(iter(ent["sampled"].items()))
    # interface.py's command list, in its order (top_k 20, top_p 0.95, temperature 0.85,
    # repeat_last_n 64, repeat_penalty 1.3, seed 42, n_threads 1: make_golden.py's sampling)
    command = ["../vsim-ubuntu.emax7nc", "gptneox", "-m", model_path(name), "--prompt", prompt, "--seed", "42",
               "--threads", "1", "--n_predict", "24", "--top_k", "20", "--top_p", "0.95", "--temp", "0.85",
               "--repeat_last_n", "64", "--repeat_penalty", "1.3"]
    r = subprocess.run(command, cwd=root / "cformers", capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert tokens(r.stdout) == want
