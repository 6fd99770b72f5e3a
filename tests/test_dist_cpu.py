"""Multi-rank paths on CPU with gloo (no GPU): the layer-split protocol of vsim_amd/pipeline.py
must give the same token stream as one rank running every layer, and the layer ranges must
tile the model.  Each rank's stage is a deterministic float32 stand-in for its layers."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vsim_amd import pipeline

E, V, L = 16, 11, 7


def _weights(nl=L):
    rng = np.random.default_rng(3)
    return (rng.standard_normal((V, E)).astype(np.float32), rng.standard_normal((nl, E, E)).astype(np.float32) * 0.3,
            rng.standard_normal((V, E)).astype(np.float32))


def _stage_fn(l0, l1, first, last, kv, nl=L):
    emb, layers, head = _weights(nl)

    def stage(n_past, ids, resid_in, resid_out):
        x = emb[np.asarray(ids)] if first else resid_in.numpy().copy()
        for l in range(l0, l1):
            # position-dependent, cache-carrying stand-in for a layer (state per rank, like the KV cache)
            kv.setdefault(l, []).append(x.sum())
            x = np.tanh(x @ layers[l] + 0.01 * (n_past + len(kv[l])))
        if last:
            return (head @ x[-1]).astype(np.float32)
        resid_out.copy_(torch.from_numpy(x.astype(np.float32)))
        return None

    return stage


def _run(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    l0, l1 = pipeline.layer_range(L, world, rank)
    stage = _stage_fn(l0, l1, rank == 0, rank == world - 1, {})
    send = (lambda t, dst: dist.send(t, dst=dst)) if world > 1 else None
    recv = (lambda t, src: dist.recv(t, src=src)) if world > 1 else None
    prompt = [1, 4, 2]
    resid = torch.zeros((len(prompt), E), dtype=torch.float32)
    tok = torch.zeros(1, dtype=torch.int64)
    toks = [pipeline.pipeline_step(rank, world, 0, prompt, stage, send, recv, resid, tok)]
    n_past = len(prompt)
    for _ in range(6):
        toks.append(pipeline.pipeline_step(rank, world, n_past, [toks[-1]], stage, send, recv, resid[:1], tok))
        n_past += 1
    if rank == 0:
        out.put(toks)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    toks = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return toks


def test_layer_ranges_tile_the_model():
    for nl in (L, 28, 36, 44):
        for world in (w for w in (1, 2, 3, 4, 7, 8) if w <= nl):
            spans = [pipeline.layer_range(nl, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == nl
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = pipeline.layer_split(nl, world)
            assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1
    # the 20B's splits of SURVEY.md §8(e)
    assert pipeline.layer_split(44, 2) == [22, 22]
    assert pipeline.layer_split(44, 4) == [11] * 4
    assert pipeline.layer_split(44, 8) == [6, 6, 6, 6, 5, 5, 5, 5]
    with pytest.raises(ValueError):
        pipeline.layer_range(L, 8, 7)  # 8 ranks for 7 layers: a rank would be empty


@pytest.mark.parametrize("world", [2, 3])
def test_pipeline_matches_single_rank(world):
    assert _stream(world) == _stream(1)


def _run_steps(rank, world, port, out, host_staged=False, nl=L):
    """pipeline.decode_steps with a stand-in stage step over bound buffers (the device-resident
    protocol of vsim_model_stage_step: token word in on rank 0, residual rows between ranks,
    argmax token word out on the last rank), after a pipeline_step prompt.  The hand-offs are
    bench.py's own transport (pipeline.make_transport): host_staged=False is the RCCL branch's
    call sequence (the tensor straight to dist.send / dist.recv), here over gloo on CPU tensors."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    first, last = rank == 0, rank == world - 1
    l0, l1 = pipeline.layer_range(nl, world, rank)
    kv = {}
    stage = _stage_fn(l0, l1, first, last, kv, nl)
    syncs = []
    send, recv = pipeline.make_transport(dist, host_staged, sync=lambda: syncs.append(1)) if world > 1 else (None, None)
    prompt = [1, 4, 2]
    resid = torch.zeros((len(prompt), E), dtype=torch.float32)
    tok = torch.zeros(1, dtype=torch.int64)
    first_tok = pipeline.pipeline_step(rank, world, 0, prompt, stage, send, recv, resid, tok)
    tok[0] = first_tok
    rin, rout = torch.zeros((1, E)), torch.zeros((1, E))
    n_past = [len(prompt)]
    toks = [first_tok]

    def step():
        logits = stage(n_past[0], [int(tok[0])] if first else None, rin, rout)
        if last:
            tok[0] = int(np.argmax(logits))
        n_past[0] += 1

    pipeline.decode_steps(rank, world, step, 6, send, recv, rin, rout, tok,
                          record=lambda i: toks.append(int(tok[0])))
    if world > 1 and not last:  # a host-staged send waits for the producing stream first
        assert bool(syncs) == host_staged
    if last:
        out.put(toks)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,host_staged", [(2, False), (3, False), (4, False), (2, True)])
def test_decode_steps_match_single_rank(world, host_staged):
    """The device-resident decode protocol gives the same stream as the per-eval one, with the
    stream-ordered (RCCL-branch) and the host-staged transports; world 4 splits 7 layers 2,2,2,1."""
    ctx = mp.get_context("spawn")

    def stream(w):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_run_steps, args=(r, w, port, q, host_staged)) for r in range(w)]
        for p in procs:
            p.start()
        toks = q.get(timeout=120)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        return toks

    assert stream(world) == stream(1) == _stream(1)


def test_decode_steps_world8_20b_split():
    """World 8 over gloo at the 20B's depth (44 layers as 6,6,6,6,5,5,5,5):
    the stream-ordered (RCCL-branch) transport's send/recv sequence through eight stand-in
    stages gives the single rank's token stream."""
    ctx = mp.get_context("spawn")

    def stream(w):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_run_steps, args=(r, w, port, q, False, 44)) for r in range(w)]
        for p in procs:
            p.start()
        toks = q.get(timeout=180)
        for p in procs:
            p.join(timeout=180)
            assert p.exitcode == 0
        return toks

    assert stream(8) == stream(1)


def test_bench_pipeline_companion_env_and_failure(monkeypatch):
    """bench.py's `pipeline_20b` companion: the child job gets a rendezvous of its own (no
    TORCHELASTIC_* agent store, MASTER_PORT + 17, the parent's rank) and a child that fails
    is reported as an error, never raised into the headline run."""
    import argparse
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    seen = {}

    class R:
        returncode = 0
        stdout = ('{"value": 1.5, "unit": "tokens/s", "n_gpus": 2, "ms_per_step": 666.7, "scaling": "strong", '
                  '"steps": 4, "config": {"parallelism": "pipeline2"}}\n')
        stderr = ""

    def fake_run(cmd, env, **kw):
        seen["cmd"], seen["env"], seen["kw"] = cmd, env, kw
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("TORCHELASTIC_USE_AGENT_STORE", "True")
    args = argparse.Namespace(mode="exact", dist_backend="nccl")
    out = bench.pipeline_companion(args, world=2, rank=0, local=0)
    assert out["value"] == 1.5 and out["n_gpus"] == 2
    env = seen["env"]
    assert not any(k.startswith("TORCHELASTIC_") for k in env)
    assert env["MASTER_PORT"] == "29517" and env["RANK"] == "0" and env["WORLD_SIZE"] == "2"
    assert "--pipeline" in seen["cmd"] and "gpt-neoxt-20b" in seen["cmd"] and seen["kw"]["timeout"] > 0
    # rank 1 returns nothing; a failing or hanging child is an error entry
    assert bench.pipeline_companion(args, world=2, rank=1, local=1) is None
    # the driver's 8-GPU run: rank 7 of 8 starts its child as rank 7 of an 8-rank job, bounded
    assert bench.pipeline_companion(args, world=8, rank=7, local=7) is None
    env = seen["env"]
    assert env["RANK"] == "7" and env["WORLD_SIZE"] == "8" and env["LOCAL_RANK"] == "7"
    assert 0 < seen["kw"]["timeout"] <= 600
    R.returncode = 3
    assert bench.pipeline_companion(args, world=2, rank=0, local=0)["error"] == "exit 3"

    def hang(cmd, env, **kw):
        raise subprocess.TimeoutExpired(cmd, kw["timeout"])

    monkeypatch.setattr(subprocess, "run", hang)
    assert "timed out" in bench.pipeline_companion(args, world=1, rank=0, local=0)["error"]
