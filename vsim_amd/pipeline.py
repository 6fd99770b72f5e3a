"""Layer-split decode protocol shared by bench.py and the CPU tests.

Rank r owns a contiguous layer range; rank 0 also owns the token embedding and the last rank
ln_f + lm_head (vsim.cpp:470-747 split at layer boundaries; with the parallel residual only
the residual row inpL crosses a boundary).  Per eval:

    rank 0:      resid = stage(n_past, tokens)            -> send resid to rank 1
    rank 0<r<G-1: recv resid from r-1; resid = stage(...) -> send to r+1
    rank G-1:    recv resid; logits = stage(...); token = argmax(logits) -> send to rank 0

so one residual send per boundary per eval plus the sampled token back to rank 0 (the
reference's loop feeds the sampled token into the next eval, vsim.cpp:860-891).

pipeline_step runs one eval through host-visible stage calls (the prompt batch);
decode_steps runs the single-token steps with the device-resident stage step, whose token
and residual stay in device buffers between the stages.
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def layer_range(n_layer: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous balanced split: the first L % G ranks hold ceil(L/G) layers, the rest
    floor(L/G) (the 20B's 44 layers as 22/22, 11 x 4, 6,6,6,6,5,5,5,5)."""
    if world > n_layer:
        raise ValueError(f"{world} ranks for {n_layer} layers leaves a rank without layers")
    base, extra = divmod(n_layer, world)
    l0 = rank * base + min(rank, extra)
    return l0, l0 + base + (1 if rank < extra else 0)


def layer_split(n_layer: int, world: int) -> list[int]:
    """Layers per rank of layer_range."""
    return [b - a for a, b in (layer_range(n_layer, world, r) for r in range(world))]


def make_transport(dist, host_staged: bool, sync: Callable | None = None):
    """(send, recv) for the stage hand-offs.

    host_staged (gloo between ranks that hold device tensors): sync() first (the producing
    stream has finished the bytes), then the tensor goes through host memory.  Otherwise
    (RCCL, bench.py --dist-backend nccl) the tensor itself is handed to dist.send / dist.recv
    with no host synchronisation: ProcessGroupNCCL orders the transfer after the work queued
    on the current stream and the current stream's later work after the transfer, so inside
    `torch.cuda.stream(ExternalStream(model.stream()))` stage step -> send -> next step stay
    stream-ordered.  The same calls on CPU tensors run over gloo (tests/test_dist_cpu.py)."""
    import torch

    def send(t, dst):
        if host_staged:
            if sync is not None:
                sync()
            dist.send(t.cpu(), dst=dst)
        else:
            dist.send(t, dst=dst)

    def recv(t, src):
        if host_staged:
            c = torch.empty(t.shape, dtype=t.dtype)
            dist.recv(c, src=src)
            t.copy_(c)
            if t.is_cuda:
                torch.cuda.current_stream().synchronize()
        else:
            dist.recv(t, src=src)

    return send, recv


def pipeline_step(rank: int, world: int, n_past: int, ids: Sequence[int],
                  stage: Callable, send: Callable, recv: Callable, resid, tok) -> int:
    """One eval of `ids` through every stage; returns the greedy next token on every rank
    that takes part in the token hand-back (rank 0 and the last rank).

    stage(n_past, ids, resid_in, resid_out) runs this rank's layers: ids on rank 0 (resid_in
    None), resid_in otherwise; it fills resid_out on every rank but the last and returns the
    logits row on the last.  send(t, dst) / recv(t, src) move a tensor; `resid` is the
    [len(ids)][E] residual buffer and `tok` a 1-element integer tensor."""
    first, last = rank == 0, rank == world - 1
    if world == 1:
        return int(np.argmax(stage(n_past, ids, None, None)))
    if first:
        stage(n_past, ids, None, resid)
        send(resid, rank + 1)
    else:
        recv(resid, rank - 1)
        out = stage(n_past, None, resid, None if last else resid)
        if not last:
            send(resid, rank + 1)
        else:
            tok[0] = int(np.argmax(out))
    if last:
        send(tok, 0)
    if first:
        recv(tok, world - 1)
    return int(tok[0])


def decode_steps(rank: int, world: int, step: Callable, n_steps: int, send: Callable, recv: Callable,
                 resid_in, resid_out, tok, record: Callable | None = None) -> None:
    """n_steps greedy decode steps through the stages with the device-resident stage step
    (vsim_model_stage_step): per step and boundary one send of the residual row, and the last
    stage's device-argmax token back to rank 0, which feeds it to its next step from the same
    device word.  Nothing crosses to the host, so with a stream-ordered transport (RCCL on the
    model's stream) the host only queues work.

    step() enqueues this rank's stage step; `tok` is the bound token word (rank 0's tok_in,
    the last rank's tok_out; one word when world == 1); record(i) runs on the last rank after
    step i (e.g. to keep the token stream)."""
    first, last = rank == 0, rank == world - 1
    for i in range(n_steps):
        if not first:
            recv(resid_in, rank - 1)
        step()
        if not last:
            send(resid_out, rank + 1)
        if last and record is not None:
            record(i)
        if world > 1:
            if last:
                send(tok, 0)
            if first:
                recv(tok, world - 1)
