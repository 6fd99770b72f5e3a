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
