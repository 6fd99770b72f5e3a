"""Golden-fixture helpers shared by the CPU and GPU parity tests."""
from __future__ import annotations

import functools
import hashlib
import json
import os
import tempfile

import numpy as np

from vsim_amd import modelgen as mg

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def ops(name: str):
    return np.load(os.path.join(GOLDEN, f"ops_{name}.npz"))


def cases(z):
    ids = sorted({k.split("_")[0] for k in z.files})
    return [{k.split("_", 1)[1]: z[k] for k in z.files if k.startswith(c + "_")} for c in ids]


@functools.lru_cache(maxsize=None)
def e2e():
    with open(os.path.join(GOLDEN, "e2e.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=None)
def model_path(name: str) -> str:
    """Regenerate the deterministic synthetic model `name` and prove it is the file the
    reference consumed (sha256 recorded in e2e.json)."""
    ent = e2e()["models"][name]
    arch, hp = mg.CONFIGS[ent["config"]]
    d = os.path.join(tempfile.gettempdir(), "vsim_golden_models")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"{name}-{ent['sha256'][:16]}.bin")
    if not os.path.exists(path):
        mg.write_model(path + ".tmp", arch, hp, seed=ent["seed"], std=ent["std"])
        os.replace(path + ".tmp", path)
    sha = hashlib.sha256(open(path, "rb").read()).hexdigest()
    assert sha == ent["sha256"], f"regenerated {name} differs from the golden input"
    return path


def fmt8(v) -> list[str]:
    """The reference prints logits with printf("%.8f ") (vsim.cpp:828-833)."""
    return ["%.8f" % float(x) for x in np.asarray(v, np.float32)]


def prompt_ids(p: str):
    return [int(t) for t in p.split()]


# Prompt-shape Q4_0 mul_mat vectors (ops_mulmat_prompt.npz): the fixture holds the seeds and the
# reference's outputs only; the inputs are regenerated here (PCG64) and checked against the
# sha256 the generator recorded.
PROMPT_MULMAT_CASES = [  # (M rows, K, N tokens, seed): GPT-J / codegen-16B prompt widths
    (256, 4096, 256, 101), (192, 6144, 320, 102), (96, 24576, 256, 103)]


def prompt_mulmat_inputs(M, K, N, seed):
    """(Q4_0 AoS weight bytes [M][K], f32 activations [N][K]) for one case: weights N(0, 0.02)
    quantized with quantize_row_q4_0 semantics, activations N(0, 1) with exact zeros and tiny
    values mixed in (as the op goldens' activ())."""
    rng = np.random.Generator(np.random.PCG64(seed))
    w = mg.quantize_q4_0(rng.standard_normal(M * K).astype(np.float32) * np.float32(0.02))
    x = rng.standard_normal(N * K).astype(np.float32)
    x[rng.integers(0, N * K, size=N * K // 97)] = 0.0
    x[rng.integers(0, N * K, size=N * K // 61)] *= np.float32(1e-7)
    return w, x.astype(np.float32)


def inputs_sha(w, x) -> str:
    return hashlib.sha256(np.ascontiguousarray(w).tobytes() + np.ascontiguousarray(x).tobytes()).hexdigest()
