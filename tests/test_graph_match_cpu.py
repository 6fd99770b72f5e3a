"""The graph executor's decode fast path starts with a host-only recogniser (vsim_graph_match,
graph.cpp) of vsim.cpp's own single-token gptneox_eval graph (vsim.cpp:470-747).  Here it is run,
without a GPU, on every graph the reference's unmodified eval loop builds:
oracle/_ref/vsim-graphprobe is vsim.cpp compiled with -Dggml_graph_compute=probe_compute
(oracle/graph_probe.c), which shows each graph to vsim_graph_match and then computes it with the
reference's own CPU executor.  Expected: every decode graph (N = 1) matches with the n_past, the
token and the model shape of that step; prompt graphs (N > 1) and the serial-residual graph
(use_parallel_residual = 0, vsim.cpp:626-658) do not; the run's output is the reference's.
"""
import os
import re
import subprocess

import pytest

from golden_util import e2e, model_path
from vsim_amd import modelgen as mg

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PROBE = os.path.join(ROOT, "oracle", "_ref", "vsim-graphprobe")

GREEDY = ["--top_k", "1", "--top_p", "1.0", "--temp", "1.0", "--repeat_penalty", "1.0", "--seed", "42", "--threads", "1"]


def probe(path, prompt, n_predict, extra=()):
    if not os.path.exists(PROBE):
        pytest.skip("oracle/_ref/vsim-graphprobe not built (make -C oracle ref graphprobe, needs /root/reference)")
    r = subprocess.run([PROBE, "gptneox", "-m", path, "--prompt", prompt, "--n_predict", str(n_predict), *GREEDY,
                        *extra], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def parse(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("GRAPH")]
    matched = [dict(kv.split("=") for kv in ln.split()[1:]) for ln in lines if ln.startswith("GRAPHMATCH")]
    return lines, [{k: int(v) for k, v in m.items()} for m in matched]


def tokens(out):
    body = out.split("<|BEGIN>", 1)[1].split("<END|>", 1)[0]
    return [int(t) for t in re.sub(r"GRAPH\S*[^\n]*", " ", body).split()]


@pytest.mark.parametrize("name", sorted(e2e()["models"]))
def test_every_decode_graph_matches(name):
    ent = e2e()["models"][name]
    arch, hp = mg.CONFIGS[ent["config"]]
    path = model_path(name)
    prompt = next(iter(ent["greedy"]))
    n_prompt = len(prompt.split())
    out = probe(path, prompt, 24)
    lines, m = parse(out)
    # warm-up eval (4 tokens, vsim.cpp:793) and the prompt: not single-token graphs
    assert lines[0].startswith("GRAPHNOMATCH") and lines[1].startswith("GRAPHNOMATCH")
    toks = tokens(out)
    assert toks == ent["greedy"][prompt]  # the probe computes with the reference's executor
    gen = toks[n_prompt:]
    assert len(m) == len(gen) - 1 == len(lines) - 2
    for k, info in enumerate(m):
        assert info["past"] == n_prompt + k and info["token"] == gen[k]
        assert (info["layers"], info["embd"], info["head"], info["rot"], info["vocab"], info["ctx"]) == (
            hp.n_layer, hp.n_embd, hp.n_head, hp.n_rot, hp.n_vocab, 512)
        assert info["nodes"] == 1 + 42 * hp.n_layer + 4


def test_single_token_prompt_matches(tmp_path):
    """A one-token prompt is itself a decode-shaped graph (n_past 0)."""
    name = "tiny-neox"
    lines, m = parse(probe(model_path(name), "7", 3))
    assert lines[1].startswith("GRAPHMATCH") and m[0]["past"] == 0 and m[0]["token"] == 7


def test_serial_residual_graph_does_not_match(tmp_path):
    arch_s, hp = mg.CONFIGS["tiny-neox"]
    hp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, use_parallel_residual=0)
    path = str(tmp_path / "serial.bin")
    mg.write_model(path, arch_s, hp, seed=9, std=0.05)
    lines, m = parse(probe(path, "1 2 3", 4))
    assert not m and len(lines) >= 4
    assert all("parallel residual" in ln for ln in lines[2:])
