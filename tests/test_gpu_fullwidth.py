"""Bit-exact parity of the bench's decode path at the benchmark configs' real widths.

Two-layer models with the full dimensions and full vocabularies of GPT-J-6B, pythia-12b,
GPT-NeoXT-20B and bloom-560m: weights drawn on the device
(vsim_model_randomize), read back through vsim_model_get_tensor into the CPU oracle, so
both sides hold identical Q4_0 bytes.  A 5-token prompt (the reference's run prompt,
Makefile-ubuntu:26) and then greedy decode past P = 300 in exact mode with the hipGraph on,
logits compared as float bits at every step.  These runs go through exactly the kernels the
bench times:
  * k_gemv_solo at K = n_embd (the {fc_in, Q, K, V} batch: 28,672 x 4096 for GPT-J) and on
    the lm_head (50,400 x 4096 / 50,432 x 6144 / 250,880 x 1024);
  * k_layer_tail: fc_out (K = 4 n_embd) beside the fused attention heads (attn.hpp) at
    d = 256 / 128 / 96 / 64, KQV streamed through its 32 KB LDS tiles at P ~ 300;
  * k_ln_quant at n_embd = 4096 / 5120 / 6144, including its sequential fallback rows
    (vsim_norm_fallbacks must move).
Then the device-resident greedy loop (vsim_model_generate, the bench's timed step) is
replayed from an earlier position and must give the same tokens.
Reference semantics: imax.c:1182-1230 (dot chain), ggml.c:4246-4304 (norm), ggml.c:4495-4581
(KQ / KQV), vsim.cpp:470-747 (graph).
"""
import os

import numpy as np
import pytest

from vsim_amd import hip
from vsim_amd import modelgen as mg

pytestmark = pytest.mark.gpu

PROMPT = [50278, 12092, 2, 0, 50281]
ARCH = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX, "bloom": hip.ARCH_BLOOM}
NTH = max(1, min(16, os.cpu_count() or 1))  # the oracle's rows are independent chains: same bits


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _pair(cfg, n_layer=2, seed=7, n_ctx=512):
    import oracle_py as O
    arch_s, hp = mg.CONFIGS[cfg]
    dm = hip.Model.create(ARCH[arch_s], dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                             n_layer=n_layer, n_rot=hp.n_rot,
                                             use_parallel_residual=hp.use_parallel_residual), n_ctx=n_ctx)
    dm.randomize(seed=seed, std=0.02)
    om = O.Model.from_device(dm, arch_s, n_ctx=n_ctx)
    return arch_s, hp, dm, om


@pytest.mark.parametrize("cfg,steps", [("gpt-j-6B", 300), ("pythia-12b", 300), ("gpt-neoxt-20b", 300),
                                       ("bloom-560m", 300)])
def test_full_width_decode_bit_exact(cfg, steps):
    arch_s, hp, dm, om = _pair(cfg)
    dm.set_mode(hip.MODE_EXACT)
    dm.set_graph(True)
    fb0 = sum(hip.norm_fallbacks())
    lo = om.eval(0, PROMPT, nthreads=NTH)
    ld = dm.eval(0, PROMPT)
    assert np.array_equal(bits(lo), bits(ld)), "prompt logits"
    n_past, toks = len(PROMPT), []
    for s in range(steps):
        t = int(np.argmax(lo))
        toks.append(t)
        lo = om.eval(n_past, [t], nthreads=NTH)
        ld = dm.eval(n_past, [t])
        if not np.array_equal(bits(lo), bits(ld)):
            bad = np.nonzero(bits(lo) != bits(ld))[0]
            pytest.fail(f"{cfg}: decode step {s} (n_past {n_past}): {bad.size} logits differ, first {bad[:5]} "
                        f"oracle {lo[bad[:3]]} device {ld[bad[:3]]}")
        n_past += 1
    assert dm.info()["graph"]
    # the exact LayerNorm's sequential fallback ran inside the compared steps
    if hp.n_embd >= 4096:
        assert sum(hip.norm_fallbacks()) > fb0
    # the bench's timed step: the device greedy loop, from an earlier position (the cache rows
    # it rewrites are rewritten with the same values)
    start = 150
    got = dm.generate(len(PROMPT) + start, toks[start], 64)
    assert got == toks[start + 1:start + 65]
    dm.close()


def test_full_width_pipeline_split_bit_exact():
    """GPT-NeoXT-20B width split over two stages on one device (the layer split of
    SURVEY.md §8(e)), residual handed over in device memory: the last stage's logits equal the
    oracle's at every step."""
    import torch
    import oracle_py as O
    arch_s, hp = mg.CONFIGS["gpt-neoxt-20b"]
    hpd = dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=2, n_rot=hp.n_rot,
               use_parallel_residual=1)
    full = hip.Model.create(hip.ARCH_GPTNEOX, hpd)
    full.randomize(seed=3, std=0.02)
    om = O.Model.from_device(full, arch_s)
    s0 = hip.Model.create(hip.ARCH_GPTNEOX, hpd, layer_begin=0, layer_end=1)
    s1 = hip.Model.create(hip.ARCH_GPTNEOX, hpd, layer_begin=1, layer_end=2)
    mhp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, 2, hp.n_rot, 1)
    for st in (s0, s1):  # copy the stage's own tensors from the whole model
        for name, ne, kind in mg.tensor_specs("gptneox", mhp):
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
    for st in (s0, s1):
        st.set_graph(True)
    r = torch.empty((len(PROMPT), hp.n_embd), dtype=torch.float32, device="cuda")
    ids, n_past = list(PROMPT), 0
    for step in range(40):
        s0.eval(n_past, ids, resid_out=r[:len(ids)])
        lp = s1.eval(n_past, None, resid_in=r[:len(ids)])
        lo = om.eval(n_past, ids, nthreads=NTH)
        assert np.array_equal(bits(lp), bits(lo)), step
        n_past += len(ids)
        ids = [int(np.argmax(lo))]
