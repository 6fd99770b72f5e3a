"""Prompt batches against the oracle and at the codegen-16B shape.

* exact mode's prompt path (the general path: k_gemv_exact_rows, the op-level attention
  kernels) is bit-exact against the oracle's composition of reference ops at N = 72 and 200;
* fast mode's prompt path (activations quantized straight to fp16, MFMA GEMM, one-pass MFMA
  attention) against the same oracle, with the tolerance below: it multiplies fp16 operands
  (the Q4_0 values d*(q-8) rounded to fp16) and re-quantizes every activation to 4 bits, so a
  one-quantum flip anywhere moves the logits - the bound is on the direction of the logits
  row (cos) and on the greedy token, not on every element;
* codegen-16B width (E = 6144, H = 24, d = 256, n_rot = 64, V = 51200), one layer: exact mode
  bit-exact against the oracle at N = 64 and at the N = 2048 of BASELINE.json configs[4], where
  fast mode is held to the same oracle logits.
Reference: ggml.c:4891-5165 (Q4_0 mul_mat, INIT quantize), vsim.cpp:865-881 (prompt batches).
"""
import os

import numpy as np
import pytest

from vsim_amd import hip
from vsim_amd import modelgen as mg

pytestmark = pytest.mark.gpu

NTH = max(1, min(16, os.cpu_count() or 1))
# fast prompt vs the reference's exact composition: the bounds are set once from the recorded
# distribution profiles/r03_fast_prefill_e2e_distribution.json (tools/fast_prefill_distribution.py:
# 72 prompts of these three models at N = 72 and 288, other prompts than the ones below):
# cos min 0.9741, 5th percentile 0.9771, median 0.9884; the fast greedy token within the oracle's
# top 5 in 72 of 72, equal to the oracle's in 49 of 72 (68 %: no per-prompt top-1 bound, but at
# least 2 of each model's 4 prompts at N = 72).  The cos bound is the recorded minimum less a
# margin of 0.004 (r04: back from r03's 0.96); neither is edited after a red run.
FAST_COS_MIN = 0.97
FAST_TOP1_MIN_N72 = 2  # of 4 prompts


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def stats(a, b):
    cos = float(np.dot(a, b) / (np.linalg.norm(a) * np.linalg.norm(b)))
    maxrel = float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
    return cos, maxrel, int(np.argmax(a)) == int(np.argmax(b)), int(np.argmax(a)) in np.argsort(b)[-5:]


def _model_pair(cfg, tmp_path, seed=5):
    import oracle_py as O
    arch_s, hp = mg.CONFIGS[cfg]
    arch = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX, "bloom": hip.ARCH_BLOOM}[arch_s]
    path = str(tmp_path / f"{cfg}.bin")
    mg.write_model(path, arch_s, hp, seed=seed, std=0.05)
    return arch, hp, path, O.Model(path, arch)


@pytest.mark.parametrize("cfg", ["small-gptj", "small-neox", "small-bloom"])
@pytest.mark.parametrize("N", [72, 200])
def test_exact_prompt_bit_exact_vs_oracle(cfg, N, tmp_path):
    arch, hp, path, om = _model_pair(cfg, tmp_path)
    ids = [(29 * i + 3) % hp.n_vocab for i in range(N)]
    dm = hip.Model.load(path, arch)
    dm.set_mode(hip.MODE_EXACT)
    lo, ld = om.eval(0, ids, nthreads=NTH), dm.eval(0, ids)
    assert np.array_equal(bits(lo), bits(ld))
    # a second batch on top of the cache, then a decode step
    lo, ld = om.eval(N, ids[:9], nthreads=NTH), dm.eval(N, ids[:9])
    assert np.array_equal(bits(lo), bits(ld))
    t = int(np.argmax(lo))
    assert np.array_equal(bits(om.eval(N + 9, [t], nthreads=NTH)), bits(dm.eval(N + 9, [t])))


@pytest.mark.parametrize("cfg", ["small-gptj", "small-neox", "small-bloom"])
@pytest.mark.parametrize("N", [72, 288])  # 288: the 256 x 256-tile GEMM, weights dequantized in LDS
def test_fast_prompt_vs_oracle(cfg, N, tmp_path):
    arch, hp, path, om = _model_pair(cfg, tmp_path)
    res = []
    for seed in range(4):
        rng = np.random.default_rng(seed)
        ids = [int(v) for v in rng.integers(0, hp.n_vocab, N)]
        dm = hip.Model.load(path, arch)
        dm.set_mode(hip.MODE_FAST)
        lo, lf = om.eval(0, ids, nthreads=NTH), dm.eval(0, ids)
        dm.close()
        om2 = type(om)(path, arch)  # fresh cache for the next prompt
        om = om2
        res.append(stats(lf, lo))
    cos = [r[0] for r in res]
    top1 = sum(r[2] for r in res)
    msg = f"{cfg}: cos {['%.5f' % c for c in cos]}, max-rel {['%.3g' % r[1] for r in res]}, top-1 {top1}/4"
    print(msg)
    assert min(cos) >= FAST_COS_MIN, msg
    if N == 72:
        assert top1 >= FAST_TOP1_MIN_N72, msg
    # the greedy token: the random parity models' top logits are close and the re-quantization
    # flips of fast mode move them past each other (top-1 49/72 recorded), so the bound is the
    # oracle's top 5 (72/72 recorded)
    assert all(r[3] for r in res), msg


CODEGEN = dict(n_vocab=51200, n_embd=6144, n_head=24, n_layer=1, n_rot=64, use_parallel_residual=1)


def _codegen_pair(n_ctx):
    import oracle_py as O
    dm = hip.Model.create(hip.ARCH_GPTJ, CODEGEN, n_ctx=n_ctx)
    dm.randomize(seed=17, std=0.02)
    return dm, O


def test_codegen_width_exact_prompt_bit_exact_vs_oracle():
    dm, O = _codegen_pair(128)
    om = O.Model.from_device(dm, "gptj", n_ctx=128)
    ids = [(7919 * i + 11) % CODEGEN["n_vocab"] for i in range(64)]
    dm.set_mode(hip.MODE_EXACT)
    assert np.array_equal(bits(om.eval(0, ids, nthreads=NTH)), bits(dm.eval(0, ids)))


def test_codegen_width_prefill_n2048_vs_oracle():
    """BASELINE.json configs[4] at its own size: the 2048-token prompt through one layer of
    codegen-16B width (E = 6144, H = 24, d = 256, V = 51200).  Exact mode is bit-exact against
    the oracle (the reference's composition ggml.c:4891-5165, vsim.cpp:470-747, run at NTH
    threads); fast mode (as bench.py --prefill runs it) against the same oracle logits, under the
    recorded-distribution bound FAST_COS_MIN and the oracle's top 5 for its greedy token."""
    import time
    N = 2048
    dm, O = _codegen_pair(N + 8)
    om = O.Model.from_device(dm, "gptj", n_ctx=N + 8)
    ids = [(7919 * i + 11) % CODEGEN["n_vocab"] for i in range(N)]
    t0 = time.time()
    lo = om.eval(0, ids, nthreads=NTH)
    t_or = time.time() - t0
    dm.set_mode(hip.MODE_EXACT)
    le = dm.eval(0, ids)
    nd = int(np.count_nonzero(bits(le) != bits(lo)))
    assert nd == 0, f"exact N=2048: {nd} of {le.size} logits differ from the oracle"
    dm.set_mode(hip.MODE_FAST)
    lf = dm.eval(0, ids)  # same positions: the cache rows are rewritten
    cos, maxrel, same, top5 = stats(lf, lo)
    msg = (f"codegen-16B width, N=2048 (oracle {t_or:.1f} s at {NTH} threads): exact bit-exact; fast vs oracle "
           f"cos {cos:.5f}, max-rel {maxrel:.3g}, top-1 {'same' if same else 'differs'}, top-5 {top5}")
    print(msg)
    assert not np.isnan(lf).any()
    assert cos >= FAST_COS_MIN, msg
    assert top5, msg


GPTJ6B = dict(n_vocab=50400, n_embd=4096, n_head=16, n_layer=2, n_rot=64, use_parallel_residual=1)


def test_gptj_width_prefill_n2048():
    """GPT-J-6B width at N = 2048, fast path against exact mode on the same weights and tokens:
    the paired Q/K launch (2 x 128 tiles, one round), the half-grid split of the 128-tile V
    (transposed-copy epilogue), out-projection and fc_out GEMMs, end to end through two layers."""
    N = 2048
    dm = hip.Model.create(hip.ARCH_GPTJ, GPTJ6B, n_ctx=N + 8)
    dm.randomize(seed=29, std=0.02)
    ids = [(7919 * i + 11) % GPTJ6B["n_vocab"] for i in range(N)]
    dm.set_mode(hip.MODE_EXACT)
    le = dm.eval(0, ids)
    dm.set_mode(hip.MODE_FAST)
    lf = dm.eval(0, ids)
    lf2 = dm.eval(0, ids)
    cos, maxrel, same, _ = stats(lf, le)
    msg = f"GPT-J-6B width, N=2048: cos {cos:.5f}, max-rel {maxrel:.3g}, top-1 {'same' if same else 'differs'}"
    print(msg)
    assert not np.isnan(lf).any()
    assert np.array_equal(bits(lf), bits(lf2)), "fast prompt not deterministic"
    assert cos >= FAST_COS_MIN, msg
    dm.close()


def test_reserve_ahead_of_prompt():
    """vsim_model_reserve allocates a prompt's buffers and stream-K workspace ahead of the first
    eval: the prompt after it gives the same bits as on a model that allocates them on the way
    (fast mode, GPT-J-6B width, N = 2048: the paired Q/K launch with its hybrid split and the
    half-grid split of V), and out-of-range sizes are refused."""
    N = 2048
    ids = [(7919 * i + 11) % GPTJ6B["n_vocab"] for i in range(N)]
    out = []
    for reserve in (True, False):
        dm = hip.Model.create(hip.ARCH_GPTJ, GPTJ6B, n_ctx=N + 8)
        dm.randomize(seed=31, std=0.02)
        dm.set_mode(hip.MODE_FAST)
        if reserve:
            for bad in (0, N + 9):
                with pytest.raises(hip.VsimError):
                    dm.reserve(bad)
            dm.reserve(N)
        out.append(dm.eval(0, ids))
        dm.close()
    assert not np.isnan(out[0]).any()
    assert np.array_equal(bits(out[0]), bits(out[1]))
