"""End-to-end parity of the device executor and the vsim-hip CLI.

GPT-NeoX: against the unmodified reference CLI's outputs (tests/golden/e2e.json):
`--return_logits` rows as printed (%.8f) and greedy / sampled token streams.
GPT-J (no reference program composes it, SURVEY.md finding 2): bit-exact against the
CPU oracle's composition of the same reference ops, logits compared as float bits.
"""
import os
import subprocess

import numpy as np
import pytest

from golden_util import e2e, fmt8, model_path, prompt_ids
from vsim_amd import hip
from vsim_amd import modelgen as mg

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CLI = os.path.join(ROOT, "vsim_amd", "_build", "vsim-hip")
MODELS = sorted(e2e()["models"])


def run_cli(args, env=None):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def last_logits(stdout):
    rows = [ln for ln in stdout.splitlines() if ln.startswith("logits:")]
    return rows[-1].split()[1:-1]


def tokens(stdout):
    return [int(t) for t in stdout.split("<|BEGIN>", 1)[1].split("<END|>", 1)[0].split()]


@pytest.mark.parametrize("name", MODELS)
def test_cli_return_logits_match_reference(name):
    ent = e2e()["models"][name]
    path = model_path(name)
    for prompt, row in ent["logits"].items():
        out = run_cli(["gptneox", "-m", path, "--prompt", prompt, "--return_logits", "--threads", "1"])
        assert last_logits(out) == row, prompt


@pytest.mark.parametrize("name", MODELS)
def test_cli_token_streams_match_reference(name):
    ent = e2e()["models"][name]
    path = model_path(name)
    for prompt, toks in ent["greedy"].items():
        out = run_cli(["gptneox", "-m", path, "--prompt", prompt, "--n_predict", "24", "--top_k", "1", "--top_p",
                       "1.0", "--temp", "1.0", "--repeat_penalty", "1.0", "--seed", "42", "--threads", "1"])
        assert tokens(out) == toks, prompt
    for prompt, toks in ent["sampled"].items():
        out = run_cli(["gptneox", "-m", path, "--prompt", prompt, "--n_predict", "24", "--top_k", "20", "--top_p",
                       "0.95", "--temp", "0.85", "--repeat_last_n", "64", "--repeat_penalty", "1.3", "--seed", "42"])
        assert tokens(out) == toks, prompt


def _decode_compare(path, arch, prompt, steps):
    """Device executor vs oracle, logits as bits, prompt batch + `steps` greedy decodes."""
    import oracle_py as O
    om = O.Model(path, arch)
    dm = hip.Model.load(path, arch)
    dm.set_mode(hip.MODE_EXACT)
    n_past = 0
    ids = list(prompt)
    lo = om.eval(0, ids)
    ld = dm.eval(0, ids)
    assert np.array_equal(lo.view(np.uint32), ld.view(np.uint32)), "prompt logits"
    n_past = len(ids)
    for s in range(steps):
        nxt = int(np.argmax(lo))
        lo = om.eval(n_past, [nxt])
        ld = dm.eval(n_past, [nxt])
        assert np.array_equal(lo.view(np.uint32), ld.view(np.uint32)), f"decode step {s}"
        n_past += 1
    dm.close()


@pytest.mark.parametrize("cfg", ["tiny-gptj", "small-gptj", "tiny-neox", "small-neox"])
def test_executor_bit_exact_vs_oracle(cfg, tmp_path):
    arch_s, hp = mg.CONFIGS[cfg]
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    path = str(tmp_path / f"{cfg}.bin")
    mg.write_model(path, arch_s, hp, seed=5, std=0.05)
    _decode_compare(path, arch, [3, 1, 4, 1, 5, 9, 2], steps=20)


def test_neox_serial_residual_vs_oracle(tmp_path):
    arch_s, hp = mg.CONFIGS["tiny-neox"]
    hp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, use_parallel_residual=0)
    path = str(tmp_path / "serial.bin")
    mg.write_model(path, arch_s, hp, seed=9, std=0.05)
    _decode_compare(path, hip.ARCH_GPTNEOX, [7, 8, 9], steps=8)


def test_fast_mode_tracks_exact(tmp_path):
    arch_s, hp = mg.CONFIGS["small-gptj"]
    path = str(tmp_path / "f.bin")
    mg.write_model(path, arch_s, hp, seed=1, std=0.05)
    m = hip.Model.load(path, hip.ARCH_GPTJ)
    m.set_mode(hip.MODE_EXACT)
    le = m.eval(0, [1, 2, 3, 4])
    m2 = hip.Model.load(path, hip.ARCH_GPTJ)
    m2.set_mode(hip.MODE_FAST)
    lf = m2.eval(0, [1, 2, 3, 4])
    cos = float(np.dot(le, lf) / (np.linalg.norm(le) * np.linalg.norm(lf)))
    assert cos > 0.95, cos


def test_bloom_fast_prefill_tracks_exact(tmp_path):
    """BLOOM's prompt layer in fast mode (fp16 MFMA GEMMs on the activation operands of
    k_act_quant_f16, GELU folded into fc_out's) stays close to exact mode (cos > 0.95)."""
    arch_s, hp = mg.CONFIGS["small-bloom"]
    path = str(tmp_path / "bpf.bin")
    mg.write_model(path, arch_s, hp, seed=6, std=0.05)
    ids = [(29 * i + 3) % hp.n_vocab for i in range(40)]
    me = hip.Model.load(path, hip.ARCH_BLOOM)
    me.set_mode(hip.MODE_EXACT)
    le = me.eval(0, ids)
    mf = hip.Model.load(path, hip.ARCH_BLOOM)
    mf.set_mode(hip.MODE_FAST)
    lf = mf.eval(0, ids)
    cos = float(np.dot(le, lf) / (np.linalg.norm(le) * np.linalg.norm(lf)))
    assert cos > 0.95, cos


@pytest.mark.parametrize("arch_name", ["small-gptj", "small-neox"])
def test_fast_prefill_deterministic(arch_name, tmp_path):
    """The fast prompt path (activations quantized straight to fp16, MFMA GEMM, MFMA
    attention) gives the same logits bits on every run: fixed-order reductions only."""
    arch_s, hp = mg.CONFIGS[arch_name]
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    path = str(tmp_path / "pfd.bin")
    mg.write_model(path, arch_s, hp, seed=4, std=0.05)
    ids = [(11 * i + 2) % hp.n_vocab for i in range(72)]
    runs = []
    for _ in range(2):
        m = hip.Model.load(path, arch)
        m.set_mode(hip.MODE_FAST)
        a = m.eval(0, ids)
        b = m.eval(len(ids), ids[:16])  # a second batch on top of the cache
        runs.append(np.concatenate([a, b]))
        m.close()
    assert np.array_equal(runs[0].view(np.uint32), runs[1].view(np.uint32))


def test_pipeline_stages_equal_single_stage(tmp_path):
    """Layer split: stage 0 = layers [0,1), stage 1 = [1,L) on one
    device, residual handed over in device memory — logits identical to one stage."""
    import torch
    arch_s, hp = mg.CONFIGS["small-neox"]
    path = str(tmp_path / "p.bin")
    mg.write_model(path, arch_s, hp, seed=2, std=0.05)
    full = hip.Model.load(path, hip.ARCH_GPTNEOX)
    s0 = hip.Model.load(path, hip.ARCH_GPTNEOX, layer_begin=0, layer_end=1)
    s1 = hip.Model.load(path, hip.ARCH_GPTNEOX, layer_begin=1, layer_end=hp.n_layer)
    ids = [5, 6, 7]
    n_past = 0
    for step in range(4):
        r = torch.empty((len(ids), hp.n_embd), dtype=torch.float32, device="cuda")
        s0.eval(n_past, ids, resid_out=r)
        lp = s1.eval(n_past, None, resid_in=r)
        lf = full.eval(n_past, ids)
        assert np.array_equal(lp.view(np.uint32), lf.view(np.uint32)), step
        n_past += len(ids)
        ids = [int(np.argmax(lf))]


def test_stage_step_needs_fresh_begin_after_eval(tmp_path):
    """vsim_model_stage_step trusts a host copy of n_past that only stage_begin sets: an eval,
    eval_argmax or generate in between moves the device n_past, so the next stage_step is
    refused (VSIM_EINVAL) until stage_begin runs again (no KV row written past n_ctx)."""
    import torch
    arch_s, hp = mg.CONFIGS["tiny-neox"]
    path = str(tmp_path / "sg.bin")
    mg.write_model(path, arch_s, hp, seed=2, std=0.05)
    m = hip.Model.load(path, hip.ARCH_GPTNEOX, n_ctx=64)
    tok = torch.zeros(1, dtype=torch.int32, device="cuda")
    m.stage_bind(tok_in=tok.data_ptr(), tok_out=tok.data_ptr())
    m.eval(0, [1, 2, 3])
    m.stage_begin(3)
    m.stage_step()
    for intervene in (lambda: m.eval(4, [5]), lambda: m.eval_argmax(5, 6), lambda: m.generate(6, 7, 2)):
        intervene()
        with pytest.raises(hip.VsimError, match="stage_begin first"):
            m.stage_step()
        m.stage_begin(8)
        m.stage_step()
    m.sync()
    m.close()


def test_kernel_counts_per_graph_kind(tmp_path):
    """kernels_per_eval after each call reports that call's own step, whichever of the four
    decode graphs (eval, eval_argmax, generate, stage step) was captured last: with the graph
    on, captured in a mixed order, each equals the count of the same call with the graph off."""
    import torch
    arch_s, hp = mg.CONFIGS["tiny-neox"]
    path = str(tmp_path / "kc.bin")
    mg.write_model(path, arch_s, hp, seed=4, std=0.05)
    m = hip.Model.load(path, hip.ARCH_GPTNEOX, n_ctx=64)
    tok = torch.zeros(1, dtype=torch.int32, device="cuda")
    m.stage_bind(tok_in=tok.data_ptr(), tok_out=tok.data_ptr())
    m.eval(0, [1, 2, 3])

    def counts(graph):
        m.set_graph(graph)
        out = {}
        m.generate(3, 4, 1)
        out["generate"] = m.info()["kernels_per_eval"]
        m.stage_begin(4)
        m.stage_step()
        out["stage"] = m.info()["kernels_per_eval"]
        m.eval_argmax(5, 6)
        out["argmax"] = m.info()["kernels_per_eval"]
        m.eval(6, [7])
        out["eval"] = m.info()["kernels_per_eval"]
        m.stage_begin(7)
        m.stage_step()
        out["stage2"] = m.info()["kernels_per_eval"]
        return out

    off, on = counts(False), counts(True)
    assert on == off, (on, off)
    assert off["argmax"] == off["eval"] + 1 and off["stage"] == off["stage2"]
    m.sync()
    m.close()


@pytest.mark.parametrize("cfg", ["small-gptj", "small-neox", "small-bloom", "small-neox-serial"])
def test_graph_replay_bit_exact_vs_oracle(cfg, tmp_path):
    """The decode step captured once in a hipGraph and replayed (n_past and the token read
    from device memory) gives the oracle's logits at every step; then the device greedy loop
    (vsim_model_generate) replays the same tokens.  The serial-residual graphs (BLOOM, GPT-NeoX
    with use_parallel_residual = 0) run their own 6-launch step (model.cpp enqueue_decode)."""
    import oracle_py as O
    serial = cfg.endswith("-serial")
    arch_s, hp = mg.CONFIGS[cfg[:-len("-serial")] if serial else cfg]
    if serial:
        hp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, use_parallel_residual=0)
    arch = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX, "bloom": hip.ARCH_BLOOM}[arch_s]
    path = str(tmp_path / f"{cfg}.bin")
    mg.write_model(path, arch_s, hp, seed=8, std=0.05)
    om = O.Model(path, arch)
    dm = hip.Model.load(path, arch)
    dm.set_mode(hip.MODE_EXACT)
    dm.set_graph(True)
    ids = [4, 8, 15, 16, 23, 42]
    lo, ld = om.eval(0, ids), dm.eval(0, ids)
    assert np.array_equal(lo.view(np.uint32), ld.view(np.uint32))
    n_past, toks = len(ids), []
    for step in range(24):
        t = int(np.argmax(lo))
        toks.append(t)
        lo, ld = om.eval(n_past, [t]), dm.eval(n_past, [t])
        assert np.array_equal(lo.view(np.uint32), ld.view(np.uint32)), step
        n_past += 1
    assert dm.info()["graph"]
    toks.append(int(np.argmax(lo)))
    assert dm.generate(len(ids) + 4, toks[4], 20) == toks[5:25]


@pytest.mark.parametrize("graph", [True, False])
def test_eval_argmax_matches_logits(graph, tmp_path):
    """The greedy step (device argmax, vsim_model_eval_argmax) returns numpy.argmax of the
    logits of the same eval: re-evaluating a position rewrites the same cache row, so
    both calls see the same state."""
    arch_s, hp = mg.CONFIGS["small-gptj"]
    path = str(tmp_path / "g.bin")
    mg.write_model(path, arch_s, hp, seed=5, std=0.05)
    m = hip.Model.load(path, hip.ARCH_GPTJ)
    m.set_graph(graph)
    lg = m.eval(0, [3, 1, 4, 1, 5])
    n_past, tok = 5, int(np.argmax(lg))
    for _ in range(12):
        lg = m.eval(n_past, [tok])
        nxt = m.eval_argmax(n_past, tok)
        assert nxt == int(np.argmax(lg))
        n_past, tok = n_past + 1, nxt


@pytest.mark.parametrize("graph", [True, False])
def test_generate_matches_stepwise_greedy(graph, tmp_path):
    """The device-resident greedy loop (vsim_model_generate) produces the tokens of the
    host-driven loop eval() + numpy.argmax."""
    arch_s, hp = mg.CONFIGS["small-gptj"]
    path = str(tmp_path / "gen.bin")
    mg.write_model(path, arch_s, hp, seed=6, std=0.05)
    a = hip.Model.load(path, hip.ARCH_GPTJ)
    b = hip.Model.load(path, hip.ARCH_GPTJ)
    a.set_graph(graph)
    b.set_graph(graph)
    prompt = [2, 7, 1, 8]
    tok = int(np.argmax(a.eval(0, prompt)))
    assert tok == int(np.argmax(b.eval(0, prompt)))
    ref, n_past, t = [], len(prompt), tok
    for _ in range(16):
        t = int(np.argmax(a.eval(n_past, [t])))
        ref.append(t)
        n_past += 1
    got = b.generate(len(prompt), tok, 10)  # in two calls: the loop resumes from (n_past, token)
    got += b.generate(len(prompt) + 10, got[-1], 6)
    assert got == ref


def test_fast_prefill_tracks_exact(tmp_path):
    """A 40-token prompt in fast mode runs the fp16 MFMA GEMM and attention (N >= 8); its
    last-row logits stay close to exact mode's (the fast path is not bit-exact: cos > 0.95,
    the same bound as the decode fast mode)."""
    arch_s, hp = mg.CONFIGS["small-gptj"]
    path = str(tmp_path / "pf.bin")
    mg.write_model(path, arch_s, hp, seed=3, std=0.05)
    ids = [(37 * i + 5) % hp.n_vocab for i in range(40)]
    me = hip.Model.load(path, hip.ARCH_GPTJ)
    me.set_mode(hip.MODE_EXACT)
    le = me.eval(0, ids)
    mf = hip.Model.load(path, hip.ARCH_GPTJ)
    mf.set_mode(hip.MODE_FAST)
    lf = mf.eval(0, ids)
    cos = float(np.dot(le, lf) / (np.linalg.norm(le) * np.linalg.norm(lf)))
    assert cos > 0.95, cos


@pytest.mark.parametrize("cfg", ["tiny-bloom", "small-bloom"])
def test_bloom_bit_exact_vs_oracle(cfg, tmp_path):
    """BLOOM: ALiBi, fused QKV, embedding LayerNorm, serial residual.
    No reference program composes the BLOOM graph (finding 2), so model-level parity is
    against the oracle's composition of reference ops; ggml_alibi itself is pinned to the
    reference's op by tests/test_oracle_golden.py::test_scale_alibi_mask_softmax."""
    arch_s, hp = mg.CONFIGS[cfg]
    path = str(tmp_path / f"{cfg}.bin")
    mg.write_model(path, arch_s, hp, seed=21, std=0.05)
    _decode_compare(path, hip.ARCH_BLOOM, [4, 8, 15, 16, 23, 42], steps=12)


def test_bloom_cli_greedy_matches_oracle(tmp_path):
    """vsim-hip bloom ...: the front-end's argv (interface.py maps BLOOM to "bloom") and the
    stdout token protocol, greedy tokens equal to the oracle's decode loop."""
    import oracle_py as O
    arch_s, hp = mg.CONFIGS["small-bloom"]
    path = str(tmp_path / "sb.bin")
    mg.write_model(path, arch_s, hp, seed=22, std=0.05)
    prompt = [3, 1, 4, 1, 5]
    out = run_cli(["bloom", "-m", path, "--prompt", " ".join(map(str, prompt)), "--n_predict", "16",
                   "--top_k", "1", "--top_p", "1.0", "--temp", "1.0", "--repeat_penalty", "1.0", "--seed", "42",
                   "--threads", "1"])
    om = O.Model(path, 2)
    want = om.generate(prompt, 16, seed=42, top_k=1, top_p=1.0, temp=1.0, repeat_penalty=1.0)
    assert tokens(out) == list(want)


def test_fast_prefill_deterministic_across_processes(tmp_path):
    """Two fast prompt evals (96 tokens, then 8 on top of the cache) in separate processes give
    the same logits bits (tools/prefill_ab.py).  In-process repeats reuse every buffer, so
    they cannot show a dependence on fresh memory; the per-layer stream-ordered operand
    allocations of an earlier prompt path did show one, in the second eval."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tool = os.path.join(root, "tools", "prefill_ab.py")
    outs = []
    for i in range(3):
        out = str(tmp_path / f"p{i}.npz")
        subprocess.run([sys.executable, tool, "--file", "--config", "small-gptj", "--n2", "8", "--out", out],
                       check=True, timeout=300)
        outs.append(out)
    for other in outs[1:]:
        subprocess.run([sys.executable, tool, "--compare", outs[0], other], check=True, timeout=120)


@pytest.mark.parametrize("arch_name,mode", [("small-gptj", "fast"), ("small-neox", "fast"), ("small-gptj", "exact"),
                                            ("small-neox", "exact")])
def test_no_kernel_reads_unwritten_memory(arch_name, mode, tmp_path):
    """Every scratch buffer and the whole KV cache filled with NaN before the first eval
    (vsim_model_debug_poison) must not change a single logit bit: no kernel of the prompt path
    (fast: activation quantize, MFMA GEMM, fp16 K/V copies, MFMA attention; exact: the general
    path) or of the decode steps reads bytes that no earlier kernel wrote.  Two prompt batches
    (the second on top of the cache, where fresh memory once changed the bits) and 12 decode
    steps."""
    arch_s, hp = mg.CONFIGS[arch_name]
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    path = str(tmp_path / "poison.bin")
    mg.write_model(path, arch_s, hp, seed=6, std=0.05)
    ids = [(13 * i + 5) % hp.n_vocab for i in range(72)]
    runs = []
    for poison in (False, True):
        m = hip.Model.load(path, arch)
        m.set_mode(hip.MODE_FAST if mode == "fast" else hip.MODE_EXACT)
        if poison:
            m.debug_poison(len(ids))
        out = [m.eval(0, ids), m.eval(len(ids), ids[:8])]
        n_past, t = len(ids) + 8, int(np.argmax(out[-1]))
        for _ in range(12):
            out.append(m.eval(n_past, [t]))
            t, n_past = int(np.argmax(out[-1])), n_past + 1
        runs.append(np.concatenate(out))
        m.close()
    assert not np.isnan(runs[1]).any()
    assert np.array_equal(runs[0].view(np.uint32), runs[1].view(np.uint32))


def test_cli_per_kernel_time_table(tmp_path):
    """VSIM_PROFILE=1: vsim-hip ends with a per-kernel device-time table, the counterpart of
    the reference's per-op table (monitor.c:196-262), and the token stream is unchanged."""
    arch_s, hp = mg.CONFIGS["small-gptj"]
    path = str(tmp_path / "prof.bin")
    mg.write_model(path, arch_s, hp, seed=9, std=0.05)
    args = ["gptj", "-m", path, "--prompt", "1 2 3 4", "--n_predict", "12", "--top_k", "1", "--seed", "1",
            "--threads", "1"]
    plain = run_cli(args)
    prof = run_cli(args, env=dict(os.environ, VSIM_PROFILE="1"))
    assert tokens(prof) == tokens(plain)
    table = prof.split("<END|>", 1)[1]
    assert "device time per kernel" in table and "COMPUTE (sum)" in table
    assert "k_layer_tail" in table and "k_gemv_solo" in table or "k_gemv" in table
