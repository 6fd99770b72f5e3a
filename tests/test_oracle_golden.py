"""The CPU oracle (oracle/vsim_oracle.cpp) reproduces the reference bit-for-bit.

Fixtures come from the reference compiled from /root/reference (tests/golden/make_golden.py):
per-op vectors from its own ggml ops, end-to-end logits and token streams from its
unmodified CLI at --threads 1.  CPU only.
"""
import numpy as np
import pytest

import oracle_py as O
from golden_util import cases, e2e, fmt8, model_path, ops, prompt_ids


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_quantize_row_q4_0():
    z = ops("qrow")
    assert np.array_equal(O.quantize(z["x"]), z["y"])


@pytest.mark.parametrize("c", cases(ops("mulmat")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_mul_mat_q4_0(c):
    M, K, N = (int(v) for v in c["shape"])
    assert np.array_equal(bits(O.mul_mat(c["w"], M, K, c["x"], N)), bits(c["y"]))
    # thread count must not change the Q4_0 result (rows are independent chains)
    assert np.array_equal(bits(O.mul_mat(c["w"], M, K, c["x"], N, nthreads=5)), bits(c["y"]))


@pytest.mark.parametrize("c", cases(ops("mulmat_prompt")), ids=lambda c: "x".join(map(str, c["shape"][:3])))
def test_mul_mat_q4_0_prompt_shapes(c):
    """The reference's Q4_0 mul_mat at prompt shapes (N >= 256 tokens, K up to 4 x 6144),
    inputs regenerated from the fixture's seed (sha256 checked)."""
    import golden_util as gu
    M, K, N, seed = (int(v) for v in c["shape"])
    w, x = gu.prompt_mulmat_inputs(M, K, N, seed)
    assert gu.inputs_sha(w, x) == str(c["sha"])
    assert np.array_equal(bits(O.mul_mat(w, M, K, x, N, nthreads=8)), bits(c["y"]))


@pytest.mark.parametrize("c", cases(ops("norm")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_norm(c):
    n, r = (int(v) for v in c["shape"])
    assert np.array_equal(bits(O.norm(c["x"], n, r)), bits(c["y"]))


def test_gelu():
    z = ops("gelu")
    assert np.array_equal(bits(O.gelu(z["x"])), bits(z["y"]))


@pytest.mark.parametrize("c", cases(ops("attnsm")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_scale_mask_softmax(c):
    nc, nr, nz, n_past = (int(v) for v in c["shape"])
    y = O.attn_softmax(c["x"], nc, nr, nz, n_past, float(c["scale"][0]))
    assert np.array_equal(bits(y), bits(c["y"]))


@pytest.mark.parametrize("c", cases(ops("attnsm_alibi")), ids=lambda c: "x".join(map(str, c["shape"])))
def test_scale_alibi_mask_softmax(c):
    """ggml_alibi (ggml.c:6184-6244) in the BLOOM score path, against the reference's op."""
    nc, nr, nz, n_past = (int(v) for v in c["shape"])
    y = O.attn_softmax_alibi(c["x"], nc, nr, nz, n_past, nz, float(c["scale"][0]))
    assert np.array_equal(bits(y), bits(c["y"]))


def test_bloom_graph_runs(tmp_path):
    """The oracle's BLOOM graph (no reference program composes one: parity unpinned at the
    model level, pinned per op) loads a synthetic ggml BLOOM file (the converter's header and
    names) and decodes to finite logits."""
    from vsim_amd import modelgen as mg
    arch_s, hp = mg.CONFIGS["tiny-bloom"]
    path = str(tmp_path / "tb.bin")
    mg.write_model(path, arch_s, hp, seed=5, std=0.05)
    m = O.Model(path, 2)  # VO_ARCH_BLOOM
    lg = m.eval(0, [1, 2, 3])
    assert lg.shape == (hp.n_vocab,) and np.all(np.isfinite(lg))
    lg2 = m.eval(3, [int(np.argmax(lg))])
    assert np.all(np.isfinite(lg2)) and not np.array_equal(lg, lg2)


@pytest.mark.parametrize("style", ["neox", "gptj"])
def test_rope(style):
    for c in cases(ops("rope_" + style)):
        d, H, T, n_past, n_dims, mode = (int(v) for v in c["shape"])
        y = O.rope(style, c["x"], d, H, T, n_past, n_dims, mode)
        assert np.array_equal(bits(y), bits(c["y"])), c["shape"]


def test_kq():
    for c in cases(ops("kq")):
        d, H, nk, N = (int(v) for v in c["shape"])
        assert np.array_equal(bits(O.kq(c["a"], c["b"], d, H, nk, N)), bits(c["y"])), c["shape"]


def test_kqv():
    for c in cases(ops("kqv")):
        d, H, nk, N = (int(v) for v in c["shape"])
        assert np.array_equal(bits(O.kqv(c["a"], c["b"], d, H, nk, N)), bits(c["y"])), c["shape"]


def test_get_rows():
    z = ops("getrows")
    K = int(z["shape"][0])
    assert np.array_equal(bits(O.get_rows(z["w"], K, z["idx"])), bits(z["y"]))


MODELS = sorted(e2e()["models"])


@pytest.mark.parametrize("name", MODELS)
def test_e2e_return_logits(name):
    ent = e2e()["models"][name]
    m = O.Model(model_path(name), 0)
    for prompt, row in ent["logits"].items():
        ids = prompt_ids(prompt)
        m.eval(0, [1, 2, 3, 4, 5])  # warm-up eval (vsim.cpp:793)
        n_past, lg = 0, None
        for s in range(0, len(ids), 9):  # prompt batches of n_batch+1 = 9 (vsim.cpp:877)
            chunk = ids[s:s + 9]
            lg = m.eval(n_past, chunk)
            n_past += len(chunk)
        assert fmt8(lg) == row, prompt


@pytest.mark.parametrize("name", MODELS)
def test_e2e_token_streams(name):
    ent = e2e()["models"][name]
    m = O.Model(model_path(name), 0)
    for prompt, toks in ent["greedy"].items():
        got = m.generate(prompt_ids(prompt), 24, seed=42, top_k=1, top_p=1.0, temp=1.0, repeat_penalty=1.0)
        assert got == toks, prompt
    for prompt, toks in ent["sampled"].items():
        got = m.generate(prompt_ids(prompt), 24, seed=42, top_k=20, top_p=0.95, temp=0.85, repeat_last_n=64,
                         repeat_penalty=1.3)
        assert got == toks, prompt
