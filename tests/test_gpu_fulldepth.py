"""Bit-exact parity of the bench's own models at full depth (every layer), against the oracle.

test_gpu_fullwidth.py pins the kernels at the real widths with two layers; this file runs the
models bench.py times, with bench.py's weights (vsim_model_randomize, seed 1234, std 0.02):
  * GPT-J-6B, all 28 layers: the 5-token prompt, then 24 greedy decode steps, logits as bits
    at every step; then the device greedy loop (the bench's timed step) over the same steps;
  * pythia-12b (36 layers) and GPT-NeoXT-20B (44 layers): prompt + 8 decode steps;
  * GPT-NeoXT-20B as a 4- and an 8-stage layer split in one process (11 x 4 and 6,6,6,6,5,5,5,5
    layers, the residual handed over in device memory): the last stage's
    logits equal the oracle's.
The per-layer KV offsets il*n_ctx (vsim.cpp:555-556) and the layer loop (vsim.cpp:521-701)
are exercised at every depth; n_ctx is kept small (64) to bound the oracle's cache.
The oracle's rows are independent chains, so its thread count does not change any bit.
"""
import os

import numpy as np
import pytest

from vsim_amd import hip
from vsim_amd import modelgen as mg

pytestmark = pytest.mark.gpu

PROMPT = [50278, 12092, 2, 0, 50281]
NTH = max(1, min(16, os.cpu_count() or 1))
N_CTX = 64
BENCH_SEED = 1234  # bench.py: model.randomize(seed=1234 + rank, std=0.02), rank 0


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _hp(cfg):
    arch_s, hp = mg.CONFIGS[cfg]
    return arch_s, hp, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                            n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual)


def _bench_pair(cfg):
    import oracle_py as O
    arch_s, hp, hpd = _hp(cfg)
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    dm = hip.Model.create(arch, hpd, n_ctx=N_CTX)
    dm.randomize(seed=BENCH_SEED, std=0.02)
    om = O.Model.from_device(dm, arch_s, n_ctx=N_CTX)
    return arch_s, hp, dm, om


def _compare(dm, om, steps, label):
    lo = om.eval(0, PROMPT, nthreads=NTH)
    ld = dm.eval(0, PROMPT)
    assert np.array_equal(bits(lo), bits(ld)), f"{label}: prompt logits"
    n_past, toks = len(PROMPT), []
    for s in range(steps):
        t = int(np.argmax(lo))
        toks.append(t)
        lo = om.eval(n_past, [t], nthreads=NTH)
        ld = dm.eval(n_past, [t])
        if not np.array_equal(bits(lo), bits(ld)):
            bad = np.nonzero(bits(lo) != bits(ld))[0]
            pytest.fail(f"{label}: decode step {s} (n_past {n_past}): {bad.size} logits differ, first {bad[:5]}")
        n_past += 1
    toks.append(int(np.argmax(lo)))
    return toks


@pytest.mark.parametrize("cfg,steps", [("gpt-j-6B", 24), ("pythia-12b", 8), ("gpt-neoxt-20b", 8)])
def test_bench_model_full_depth_bit_exact(cfg, steps):
    arch_s, hp, dm, om = _bench_pair(cfg)
    dm.set_mode(hip.MODE_EXACT)
    dm.set_graph(True)
    toks = _compare(dm, om, steps, cfg)
    assert dm.info()["graph"]
    # the bench's timed step (vsim_model_generate) from the first decode position: it rewrites
    # the cache rows of the compared steps with the same values and must give the same tokens
    got = dm.generate(len(PROMPT), toks[0], steps)
    assert got == toks[1:steps + 1]
    dm.close()


def _copy_stage(full, st, arch_s, hp):
    """Copy the stage's own tensors (its layers; wte on the first stage, ln_f + lm_head on the
    last) from the whole model, through the ggml-format tensor interface."""
    mhp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, hp.use_parallel_residual)
    for name, ne, kind in mg.tensor_specs(arch_s, mhp):
        n = int(np.prod(ne))
        nbytes = n // 32 * 20 if kind == "q" else 4 * n
        if name.startswith("gpt_neox.layers."):
            li = int(name.split(".")[2])
            if not (st.layer_begin <= li < st.layer_end):
                continue
        elif name == "gpt_neox.embed_in.weight" and not st.first:
            continue
        elif name != "gpt_neox.embed_in.weight" and not st.last:
            continue
        buf = full.get_tensor(name, nbytes)
        hip.check(hip.lib().vsim_model_set_tensor(st.h, name.encode(), buf.ctypes.data, nbytes), name)


@pytest.mark.parametrize("G,split", [(4, [11, 11, 11, 11]), (8, [6, 6, 6, 6, 5, 5, 5, 5])])
def test_20b_stage_split_full_depth_bit_exact(G, split):
    """GPT-NeoXT-20B, 44 layers as G stages (the 4- and 8-GPU splits of bench.py --pipeline,
    pipeline.layer_range, here on one device): prompt + 8 decode steps through the chain of
    stages, the last stage's logits equal the oracle's whole-model logits at every step."""
    import torch
    from vsim_amd import pipeline
    arch_s, hp, dm, om = _bench_pair("gpt-neoxt-20b")
    _, _, hpd = _hp("gpt-neoxt-20b")
    spans = [pipeline.layer_range(hp.n_layer, G, g) for g in range(G)]
    stages = [hip.Model.create(hip.ARCH_GPTNEOX, hpd, n_ctx=N_CTX, layer_begin=a, layer_end=b) for a, b in spans]
    assert [s.layer_end - s.layer_begin for s in stages] == split
    for st in stages:
        _copy_stage(dm, st, arch_s, hp)
        st.set_graph(True)
    dm.close()
    bufs = [torch.empty((len(PROMPT), hp.n_embd), dtype=torch.float32, device="cuda") for _ in range(G - 1)]
    ids, n_past = list(PROMPT), 0
    for step in range(9):
        n = len(ids)
        stages[0].eval(n_past, ids, resid_out=bufs[0][:n])
        for g in range(1, G - 1):
            stages[g].eval(n_past, None, resid_in=bufs[g - 1][:n], resid_out=bufs[g][:n])
        lp = stages[G - 1].eval(n_past, None, resid_in=bufs[G - 2][:n])
        lo = om.eval(n_past, ids, nthreads=NTH)
        assert np.array_equal(bits(lp), bits(lo)), step
        n_past += n
        ids = [int(np.argmax(lo))]
    for st in stages:
        st.close()
