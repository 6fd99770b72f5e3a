"""The layer split of SURVEY.md §8(e) on the real HIP stages: 2, 3 and 4 ranks (separate
processes sharing this box's one GPU, gloo with host staging, tests/workers/pipeline_worker.py)
run the prompt through pipeline.pipeline_step and then greedy decode through
pipeline.decode_steps with the device-resident stage step (vsim_model_stage_step: hipGraph,
device argmax on the last stage, the token fed back to rank 0's next step).  The token
stream must equal one process running every layer (vsim_model_generate), exact mode."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from vsim_amd import hip
from vsim_amd import modelgen as mg

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
WORKER = os.path.join(ROOT, "tests", "workers", "pipeline_worker.py")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("cfg,world,graph,n_layer", [("small-neox", 2, 1, None), ("small-neox", 3, 1, 5),
                                                     ("small-neox", 4, 1, 7), ("small-gptj", 2, 1, None),
                                                     ("small-neox", 2, 0, None)])
def test_pipeline_ranks_equal_single_stage(cfg, world, graph, n_layer, tmp_path):
    arch_s, hp = mg.CONFIGS[cfg]
    if n_layer:  # more layers than ranks, uneven splits (pipeline.layer_range: 5/3 = 2, 2, 1; 7/4 = 2, 2, 2, 1)
        hp = mg.HParams(hp.n_vocab, hp.n_embd, hp.n_head, n_layer, hp.n_rot, hp.use_parallel_residual)
    arch = hip.ARCH_GPTJ if arch_s == "gptj" else hip.ARCH_GPTNEOX
    path = str(tmp_path / f"{cfg}.bin")
    mg.write_model(path, arch_s, hp, seed=11, std=0.05)
    steps = 24
    # one process, every layer
    full = hip.Model.load(path, arch)
    full.set_graph(True)
    prompt = [p % 128 for p in [50278, 12092, 2, 0, 50281]]
    t0 = int(np.argmax(full.eval(0, prompt)))
    want = [t0] + full.generate(len(prompt), t0, steps)
    full.close()
    port, out = free_port(), str(tmp_path / "tokens.json")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, WORKER, "--rank", str(r), "--world", str(world), "--port", str(port),
                               "--model", path, "--arch", str(arch), "--n-layer", str(hp.n_layer),
                               "--n-embd", str(hp.n_embd), "--steps", str(steps), "--graph", str(graph),
                               "--out", out], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=180)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("pipeline ranks timed out")
    assert all(p.returncode == 0 for p in procs), "\n".join(l[-1500:] for l in logs)
    got = json.load(open(out))["tokens"]
    assert got == want
