#!/usr/bin/env python3
"""Headline benchmark: GPT-J-6B Q4_0 decode tokens/s on MI355X (BASELINE.json configs[1]).

A step = one decode eval of one token through the device-resident executor of
libvsim_hip.so (28 layers + lm_head, vsim.cpp:470-747 op sequence composed for GPT-J) and
the greedy pick on the device, fed to the next step (vsim_model_generate) — the reference's
decode loop (vsim.cpp:802-891) without a host round trip per token.  Synthetic random-init weights of the GPT-J-6B shapes are drawn on
the device (no checkpoints offline).  Decode starts after a 5-token prompt
(50278 12092 2 0 50281, the reference's own run prompt), so step k attends over 5+k
cached positions.

N > 1 GPUs: GPT-J-6B is below the >=12B threshold at which the north star splits layers,
so each rank decodes its own stream (replicas, weak scaling, no collective on the data
path); value = all ranks' tokens / max-over-ranks time.  `--config gpt-neoxt-20b
--pipeline` runs the 20B layer split with one RCCL send of the residual per stage; the
default run also measures that split over the same N ranks in a child job and reports it
beside the headline as `pipeline_20b` (north star: 1/2/4/8-GPU numbers for the 20B).

Prints ONE JSON line (rank 0) with `roofline` (the Q4_0 GEMV kernel: algorithmic weight
bytes / event-timed average launch) and `cpu_baseline` (the CPU oracle on the host cores: the
full 28-layer model, decode tokens timed at the job's threads and at 1 thread).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402
from vsim_amd import pipeline  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); ~6300 GB/s measured copy
PROMPT = [50278, 12092, 2, 0, 50281]
ARCHS = {"gptj": hip.ARCH_GPTJ, "gptneox": hip.ARCH_GPTNEOX, "bloom": hip.ARCH_BLOOM}
# HBM traffic of the dominant kernel, from a separate `rocprofv3 --pmc FETCH_SIZE` pass of this
# bench on the same commit (tools/gpu_round.sh) committed under profiles/; FETCH_SIZE is in KiB
# and reads half of the bytes of a 16-byte-per-lane streaming read on gfx950
# (MI355X_MICROARCH.md, HBM section), so it is doubled.
def pmc_file(mode="exact"):
    """The newest profiles/rNN_pmc_fetch_<mode>.csv (tools/gpu_round.sh), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_fetch_{mode}.csv")))
    return files[-1] if files else None


def pmc_traffic_per_launch(kernel: str, path=None, mode="exact"):
    """(mean corrected FETCH_SIZE bytes per launch of `kernel`, source file), or (None, None).
    Where one kernel serves launches of different shapes (k_gemv_solo: the per-layer batch and
    the lm_head), the launches of its most frequent grid size are taken: the per-layer one."""
    import collections
    import csv
    path = path or pmc_file(mode)
    if not path or not os.path.exists(path):
        return None, None
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") == "FETCH_SIZE" and kernel in r.get("Kernel_Name", ""):
                rows.append((r.get("Grid_Size"), float(r["Counter_Value"]) * 1024.0 * 2.0))
    if not rows:
        return None, None
    grid = collections.Counter(g for g, _ in rows).most_common(1)[0][0]
    vals = [v for g, v in rows if g == grid]
    return sum(vals) / len(vals), os.path.relpath(path, ROOT)


# The exact path's chain floor: every output row is one sequential fp32 chain of
# K/2 dependent adds (imax.c:1182-1230), and a dependent v_add_f32 takes 4.63 cycles of the
# 2.40 GHz clock (tools/chain_lat.hip, profiles/r04_chain_lat.txt).  A launch cannot end before
# its longest chain has run; chain_floor_frac = that floor / the launch's average time.
CHAIN_CYCLES_PER_ADD = 4.63
CHAIN_CLOCK_GHZ = 2.40


def chain_adds(kernel: str, E: int, F: int):
    """Dependent adds of the longest chain in one launch of `kernel` (exact-mode GEMV kernels),
    or None for kernels without a row chain."""
    if not kernel.startswith(("k_gemv_solo", "k_gemv_chain32", "k_layer_tail")):
        return None
    return (F if "fc_out" in kernel else E) // 2


def kernel_stats_file(mode="exact"):
    """The newest profiles/rNN_<mode>_kernel_stats.csv (rocprofv3 --stats, tools/gpu_round.sh)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{mode}_kernel_stats.csv")))
    return files[-1] if files else None


def rocprof_avg_us(kernel: str, mode="exact"):
    """(average duration in us of `kernel` in the newest rocprof stats of this mode, its file)."""
    import csv
    path = kernel_stats_file(mode)
    if not path:
        return None, None
    with open(path) as f:
        for r in csv.DictReader(f):
            if f"vsim::{kernel}" in r.get("Name", "") or f"vsim::{kernel}<" in r.get("Name", ""):
                return float(r["AverageNs"]) / 1e3, os.path.relpath(path, ROOT)
    return None, os.path.relpath(path, ROOT)


def roofline_from_profile(kernels, wall_s, mode, E=None, F=None):
    """The dominant kernel (most device time over the profiled steps): algorithmic bytes per
    launch / its event-timed average launch, against the HBM peak.  The aggregate over every
    profiled launch is kept under a separate key."""
    if not kernels:
        return None
    dom = max(kernels, key=lambda k: k["ms"])
    avg_ms = dom["ms"] / dom["launches"]
    bpl = dom["bytes"] / dom["launches"]
    achieved = bpl / (avg_ms * 1e-3) / 1e9
    rname = dom["name"].split()[0]
    traffic, src = pmc_traffic_per_launch(rname, mode=mode)
    tot_ms = sum(k["ms"] for k in kernels)
    tot_b = sum(k["bytes"] for k in kernels)

    def floor(k):
        n = chain_adds(k["name"], E, F) if mode == "exact" and E else None
        if n is None:
            return {}
        fl = n * CHAIN_CYCLES_PER_ADD / (CHAIN_CLOCK_GHZ * 1e3)
        return {"chain_adds": n, "chain_floor_us": round(fl, 2),
                "chain_floor_frac": round(fl / (1e3 * k["ms"] / k["launches"]), 4)}

    rp_us, rp_src = rocprof_avg_us(rname, mode)
    return {
        "bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
        "frac": round(achieved / PEAK_HBM_GBS, 4),
        "traffic": round(traffic) if traffic else None,
        "traffic_source": src,
        "kernel": dom["name"], "bytes_per_launch": round(bpl), "avg_launch_us": round(avg_ms * 1e3, 3),
        "launches": dom["launches"],
        # the same kernel's average from the newest committed rocprofv3 --stats pass (graph replay,
        # no event pair around each launch), and the frac it gives
        "rocprof_avg_us": round(rp_us, 3) if rp_us else None,
        "frac_rocprof": round(bpl / (rp_us * 1e-6) / 1e9 / PEAK_HBM_GBS, 4) if rp_us else None,
        "rocprof_source": rp_src,
        **floor(dom),
        "per_kernel": [{"kernel": k["name"], "launches": k["launches"],
                        "avg_us": round(1e3 * k["ms"] / k["launches"], 3),
                        "bytes_per_launch": round(k["bytes"] / k["launches"]),
                        "GBps": round(k["bytes"] / (k["ms"] * 1e-3) / 1e9, 1),
                        "frac": round(k["bytes"] / (k["ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                        "share_of_device_time": round(k["ms"] / tot_ms, 4), **floor(k)} for k in kernels],
        "aggregate": {"GBps": round(tot_b / (tot_ms * 1e-3) / 1e9, 1),
                      "frac": round(tot_b / (tot_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                      "device_share_of_wall": round(tot_ms * 1e-3 / wall_s, 4)},
        "note": ("exact mode: every row is the reference's sequential fp32 chain of K/2 dependent adds; "
                 "chain_floor_us is that chain alone at 4.63 cycles per add (2.4 GHz), so chain_floor_frac "
                 "says how far a kernel sits from its own chain bound and frac how far from HBM's "
                 "(DESIGN.md §4.1; the chain floor of the whole GPT-J-6B token is ~0.56 ms, ~1,800 tok/s)")
        if mode == "exact" else None,
    }


def measured_copy_gbps(nbytes=2 << 30, reps=10):
    """Device-to-device copy bandwidth on this GPU (a measured figure beside the
    8 TB/s spec): torch's copy of a 2 GiB buffer, read + write bytes / time, best of reps."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        best = max(best, 2.0 * nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del a, b
    return round(best, 1)


def metric_name(config: str) -> str:
    """BASELINE.json's metric for the headline config; the same wording for the others."""
    if config == "gpt-j-6B":
        return "decode tokens/sec GPT-J-6B Q4_0 @1 GPU; achieved HBM GB/s vs peak"
    return f"decode tokens/sec {config} Q4_0; achieved HBM GB/s vs peak"


def q4_weight_bytes(arch: str, hp: mg.HParams) -> float:
    """B_w per decode token: every Q4_0 matrix incl. lm_head, 0.625 B/w."""
    E, F, L, V = hp.n_embd, hp.n_ff, hp.n_layer, hp.n_vocab
    return 0.625 * (L * (4 * E * E + 2 * E * F) + V * E)


def host_cpu():
    """(nproc, lscpu model name, threads available to this process: the box's CPU share)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:  # the box's CPU share for this job (16 per GPU)
        avail = min(avail, int(omp))
    return os.cpu_count() or 1, model, max(1, avail)


def cpu_baseline(arch_s: str, hp: mg.HParams, n_tokens: int = 4, n_tokens_1t: int = 2):
    """CPU oracle (port of the reference path) on the host cores: the full-depth model of the
    config (every layer, synthetic weights of its shapes), a 1-token prompt, then `n_tokens`
    decode tokens timed at every thread of this job's CPU share and `n_tokens_1t` at 1 thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O
    arch = {"gptneox": 0, "gptj": 1, "bloom": 2}[arch_s]  # VO_ARCH_*
    nproc, model_name, nth = host_cpu()
    t0 = time.perf_counter()
    m = O.Model(None, arch, n_ctx=1 + n_tokens + n_tokens_1t + 1,
                synthetic=(hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, 7, 0.02))
    t_make = time.perf_counter() - t0
    m.eval(0, PROMPT[:1], nthreads=nth)
    n_past = 1

    def per_token(threads, n):
        nonlocal n_past
        t = time.perf_counter()
        for i in range(n):
            m.eval(n_past, [i + 11], nthreads=threads)
            n_past += 1
        return (time.perf_counter() - t) / n

    t_all = per_token(nth, n_tokens)
    t_one = per_token(1, n_tokens_1t)
    del m
    speed = None
    sp = sorted(glob_profiles("*_oracle_vs_ref_speed.json"))
    if sp:
        with open(sp[-1]) as f:
            speed = json.load(f)
    return {
        "value": round(1.0 / t_all, 4),
        "unit": "tokens/s",
        "cores": nth,
        "kind": "port",
        "value_1_thread": round(1.0 / t_one, 4),
        "host": {"nproc": nproc, "model_name": model_name, "threads_available_to_job": nth},
        "sample": (f"oracle/vsim_oracle.cpp (scalar restatement of imax.c:1182-1230 et al.), the full "
                   f"{hp.n_layer}-layer {arch_s} model (E={hp.n_embd}, V={hp.n_vocab}, synthetic weights, "
                   f"{t_make:.1f} s to make), 1-token prompt, then {n_tokens} decode tokens timed at {nth} "
                   f"threads: {t_all * 1e3:.1f} ms each; {n_tokens_1t} more at 1 thread: {t_one * 1e3:.1f} ms each"),
        "oracle_vs_reference_speed": ({"file": os.path.relpath(sp[-1], ROOT), "threads": speed.get("threads")}
                                      if speed else None),
    }


def glob_profiles(pattern):
    import glob
    return glob.glob(os.path.join(ROOT, "profiles", pattern))


def fast_companion(model, n_past, tok, steps):
    """The integer-dot fast mode on the same weights: throughput, and the one-step logits error
    against exact mode (each step is evaluated in both modes from the same exact KV cache;
    over many steps the error compounds through the 4-bit activation re-quantization, see
    tools/mode_drift.py), so it is a reported companion, not the headline value."""
    # (r05: 16 compared steps instead of 4, listed per step: with 4 the agreement moved between
    # 0.5 and 1.0 with the warm-up length alone -- the driver's --warmup 5 starts the comparison
    # at position 10, the default 8 at 13 -- on the same kernels, profiles/r05_fast_top1.txt)
    rel, top1 = [], []
    ncmp = 16
    for i in range(ncmp):
        model.set_mode(hip.MODE_FAST)
        lf = model.eval(n_past + i, [tok])
        model.set_mode(hip.MODE_EXACT)
        le = model.eval(n_past + i, [tok])
        rel.append(float(np.max(np.abs(lf - le)) / np.max(np.abs(le))))
        top1.append(int(np.argmax(lf) == np.argmax(le)))
        tok = int(np.argmax(le))
    n_past += ncmp
    model.set_mode(hip.MODE_FAST)
    toks = model.generate(n_past, tok, 4)  # warm-up (captures the fast-mode graph)
    n_past += 4
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.generate(n_past, toks[-1], steps)  # device greedy loop, as the exact-mode value
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    model.set_mode(hip.MODE_EXACT)
    arch_s = "gptj" if model.arch == hip.ARCH_GPTJ else "gptneox"
    hp = mg.HParams(model.n_vocab, model.n_embd, model.hp.n_head, model.hp.n_layer, model.hp.n_rot)
    gbs = q4_weight_bytes(arch_s, hp) * steps / dt / 1e9
    return {"value": round(steps / dt, 3), "unit": "tokens/s", "steps": steps,
            "weight_stream_GBps": round(gbs, 1), "frac_of_peak": round(gbs / PEAK_HBM_GBS, 4),
            "kernels": ("k_gemv_fast_epi GEMVs beside the exact attention and LayerNorm kernels (serial-residual step)"
                        if model.arch == hip.ARCH_BLOOM else
                        "k_fast_gemv (LayerNorm prologue), k_fast_tail, k_fast_oproj_join (fast_decode.hip)"),
            "one_step_max_rel_logit_err": max(rel), "one_step_top1_agree": sum(top1) / len(top1),
            "compared_from_position": n_past - ncmp - 4,
            "per_step_max_rel": [round(r, 5) for r in rel], "per_step_top1": top1,
            "parity": "not bit-exact; drifts across steps (tools/mode_drift.py)"}


def decode_companion(config, dev, steps=64, warmup=8):
    """Exact greedy decode of another BASELINE config on this GPU (BASELINE.json configs[2]:
    pythia-12b, the HBM-bound GEMV config), bounded: synthetic weights of its shapes, the same
    5-token prompt, `warmup` then `steps` timed tokens through vsim_model_generate."""
    import torch
    arch_s, hp = mg.CONFIGS[config]
    t0 = time.perf_counter()
    m = hip.Model.create(ARCHS[arch_s], dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                             n_layer=hp.n_layer, n_rot=hp.n_rot,
                                             use_parallel_residual=hp.use_parallel_residual),
                         n_ctx=len(PROMPT) + warmup + steps + 8, device=dev)
    m.randomize(seed=4321, std=0.02)
    m.set_mode(hip.MODE_EXACT)
    m.set_graph(True)
    tok = int(np.argmax(m.eval(0, PROMPT)))
    n_past = len(PROMPT)
    tok = m.generate(n_past, tok, warmup)[-1]
    n_past += warmup
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m.generate(n_past, tok, steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t1
    m.close()
    bw = q4_weight_bytes(arch_s, hp)
    return {"value": round(steps / dt, 3), "unit": "tokens/s", "steps": steps, "warmup": warmup,
            "ms_per_step": round(1e3 * dt / steps, 4), "mode": "exact",
            "weight_bytes_per_token": bw, "weight_stream_GBps": round(bw * steps / dt / 1e9, 1),
            "positions": f"{len(PROMPT) + warmup}..{len(PROMPT) + warmup + steps - 1}",
            "setup_s": round(t1 - t0, 1)}


def run_pipeline(args, world, rank, dev, dist):
    """Layer split: rank r owns a contiguous layer range (rank 0 also the
    embedding, the last rank ln_f + lm_head).  Per decode token the residual row [1][E] goes
    rank r -> r+1 (one RCCL send/recv over xGMI per boundary) and the greedy token goes back
    from the last rank to rank 0.  One token stream passes every stage in turn, so the value
    is that stream's tokens/s (strong scaling: the work per token is fixed)."""
    import torch
    arch_s, hp = mg.CONFIGS[args.config]
    arch = ARCHS[arch_s]
    L = hp.n_layer
    per = pipeline.layer_split(L, world)
    l0, l1 = pipeline.layer_range(L, world, rank)
    n_ctx = max(512, len(PROMPT) + args.warmup + args.steps + 16)
    hpd = dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=L, n_rot=hp.n_rot,
               use_parallel_residual=hp.use_parallel_residual)
    model = hip.Model.create(arch, hpd, n_ctx=n_ctx, device=dev, layer_begin=l0, layer_end=l1)
    model.randomize(seed=1234 + rank, std=0.02)
    model.set_mode(hip.MODE_EXACT if args.mode == "exact" else hip.MODE_FAST)
    model.set_graph(not args.no_graph)
    E = hp.n_embd
    host = args.dist_backend == "gloo"
    first, last = rank == 0, rank == world - 1
    rbuf = torch.empty((len(PROMPT), E), dtype=torch.float32, device="cuda")
    tokt = torch.zeros(1, dtype=torch.int64, device="cpu" if host else "cuda")
    ext = torch.cuda.ExternalStream(model.stream())

    # gloo: host-staged after the model's stream has produced the bytes; RCCL: ordered on the
    # model's stream (the current stream inside `ext`)
    send, recv = pipeline.make_transport(dist, host, sync=model.sync)

    def stage(n_past, ids, resid_in, resid_out):
        return model.eval(n_past, ids, resid_in=resid_in, resid_out=resid_out)

    # the prompt: one batched eval through the stages (general path)
    tok = pipeline.pipeline_step(rank, world, 0, PROMPT, stage, send,
                                 lambda t, src: (recv(t, src), torch.cuda.current_stream().synchronize()),
                                 rbuf[:len(PROMPT)], tokt)
    n_past = len(PROMPT)
    # decode: the device-resident stage step, bound to fixed device buffers
    tok_dev = torch.tensor([tok if tok is not None else 0], dtype=torch.int32, device="cuda")
    rin = torch.empty(E, dtype=torch.float32, device="cuda")
    rout = torch.empty(E, dtype=torch.float32, device="cuda")
    model.stage_bind(tok_in=tok_dev.data_ptr() if first else 0, resid_in=0 if first else rin.data_ptr(),
                     resid_out=0 if last else rout.data_ptr(), tok_out=tok_dev.data_ptr() if last else 0)
    model.stage_begin(n_past)
    torch.cuda.synchronize()

    def steps(n):
        with torch.cuda.stream(ext):
            pipeline.decode_steps(rank, world, model.stage_step, n, send, recv, rin, rout, tok_dev)

    steps(args.warmup)
    model.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    steps(args.steps)
    model.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = args.steps / elapsed
    bw = q4_weight_bytes(arch_s, hp)
    line = {
        "metric": metric_name(args.config),
        "value": round(value, 3), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32 (Q4_0 x Q4_0 operands)",
        "data": "synthetic (random-init weights of the config's shapes, drawn on device)",
        "config": {"workload": f"{args.config} Q4_0 decode, layers split over {world} rank(s), "
                               f"{args.steps} timed tokens after a 5-token prompt + {args.warmup} warm-up",
                   "mode": args.mode, "n_ctx": n_ctx, "parallelism": f"pipeline{world}",
                   "layers_per_rank": per, "send_bytes_per_token_per_boundary": 4 * E,
                   "backend": args.dist_backend if world > 1 else None,
                   "weight_bytes_per_token": bw, "weight_stream_GBps": round(bw * value / 1e9, 1)},
        "roofline": None, "cpu_baseline": None,
    }
    model.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def pipeline_companion(args, world, rank, local, steps=64, warmup=8, limit=300):
    """GPT-NeoXT-20B split over the same `world` ranks (run_pipeline), run as a child job of
    each rank on its own rendezvous port, so that a failure or a hang there (bounded by
    `limit`, then the child is killed) cannot take the headline measurement with it.  Rank 0
    returns the child's line, or the reason it has none."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    if world > 1:  # a store of its own: rank 0 of the child job hosts it
        env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local),
                   MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=str(int(os.environ.get("MASTER_PORT", "29500")) + 17))
    else:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            env.pop(k, None)
    cmd = [sys.executable, os.path.abspath(__file__), "--pipeline", "--config", "gpt-neoxt-20b",
           "--steps", str(steps), "--warmup", str(warmup), "--mode", args.mode,
           "--dist-backend", args.dist_backend]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=limit)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {limit} s"}
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
    if rank != 0:
        return None
    js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not js:
        return {"error": "no JSON line", "stdout_tail": r.stdout[-400:]}
    d = json.loads(js[-1])
    return {"value": d["value"], "unit": d["unit"], "n_gpus": d["n_gpus"], "ms_per_step": d["ms_per_step"],
            "scaling": d["scaling"], "steps": d["steps"], "config": d["config"]}


def prefill_companion(limit=300):
    """BASELINE.json configs[4] (codegen-16B, a 2048-token prompt on the fp16 MFMA dequant-GEMM
    path) on the driver's clock: run_prefill in a child process with `limit` seconds, three timed
    prompts after the first and one exact-mode prompt, so that a failure or a hang there cannot
    take the headline decode measurement with it.  Reports ms per prompt, TFLOP/s and the
    fraction of the dense fp16 MFMA peak, the first prompt, and the exact path's time."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK") and
           not k.startswith("TORCHELASTIC_")}
    cmd = [sys.executable, os.path.abspath(__file__), "--config", "codegen-16B", "--prefill", "2048", "--steps", "3",
           "--prefill-exact"]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=limit)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {limit} s"}
    if r.returncode != 0:
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
    js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not js:
        return {"error": "no JSON line", "stdout_tail": r.stdout[-400:]}
    d = json.loads(js[-1])
    ex = d.get("exact_mode") or {}
    return {"workload": d["config"]["workload"], "value": d["value"], "unit": d["unit"],
            "ms_per_prompt": d["ms_per_prompt"], "first_prompt_ms": d["first_prompt_ms"], "steps": d["steps"],
            "tflops": d["roofline"]["achieved"], "frac_of_dense_fp16_peak": d["roofline"]["frac"],
            "exact_mode_ms_per_prompt": ex.get("ms_per_prompt"),
            "parity": "fast prompt: per-op bound vs the reference's mul_mat, end to end cos >= 0.97 "
                      "(tests/test_gpu_prefill.py); exact prompt: bit-identical to the oracle",
            "wall_s": round(time.perf_counter() - t0, 1)}


def run_prefill(args, dev):
    """One prompt eval of args.prefill tokens (codegen-16B, N = 2048) in
    fast mode: every Q4_0 matmul on fp16 MFMA after in-LDS dequant (gemm_f16.hip: for N >= 256
    the 256 x 256-tile GEMM reading the W4T32 weights, no fp16 image), attention on the fp16
    MFMA prefill kernel, the elementwise ops fused into the GEMM epilogues or on the
    general-path kernels.  `value` is the steady state; the first prompt is reported beside it.
    --prefill-exact also times the same prompt on the exact path (the reference's fp32 chains,
    bit-identical to the oracle) and reports it as `exact_mode`."""
    import torch
    arch_s, hp = mg.CONFIGS[args.config]
    arch = ARCHS[arch_s]
    N = args.prefill
    model = hip.Model.create(arch, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                        n_layer=hp.n_layer, n_rot=hp.n_rot,
                                        use_parallel_residual=hp.use_parallel_residual),
                             n_ctx=N + 8, device=dev)
    model.randomize(seed=1234, std=0.02)
    model.set_mode(hip.MODE_FAST)
    ids = [(7919 * i + 11) % hp.n_vocab for i in range(N)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model.reserve(N)  # (the N-token scratch, the attention's key copies, the stream-K workspace)
    reserve = time.perf_counter() - t0
    t0 = time.perf_counter()
    model.eval(0, ids)  # the first prompt, reported beside the steady state
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    reps = max(1, args.steps)
    t0 = time.perf_counter()
    for _ in range(reps):
        model.eval(0, ids)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    exact = None
    if args.prefill_exact:
        model.set_mode(hip.MODE_EXACT)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.eval(0, ids)
        torch.cuda.synchronize()
        te = time.perf_counter() - t0
        model.set_mode(hip.MODE_FAST)
        exact = {"ms_per_prompt": round(te * 1e3, 1), "value": round(N / te, 1), "unit": "tokens/s",
                 "path": "exact mode: per-token fp32 chains (the reference's sumf order), bit-identical to the oracle",
                 "steps": 1}
    E, F, L, V = hp.n_embd, hp.n_ff, hp.n_layer, hp.n_vocab
    # flops as computed: every layer matmul over N tokens, the head for the last row (the
    # logits that leave the eval, vsim.cpp:736-737), causal QK^T and PV
    gemm_flops = 2.0 * N * L * (4 * E * E + 2 * E * F) + 2.0 * V * E
    attn_flops = 2.0 * 2.0 * L * E * (N * (N + 1) / 2.0)
    tflops = (gemm_flops + attn_flops) / dt / 1e12
    print(json.dumps({
        "metric": f"prefill tokens/s {args.config} Q4_0 seq={N} @1 GPU (fp16 MFMA dequant-GEMM)",
        "value": round(N / dt, 1), "unit": "tokens/s", "n_gpus": 1, "steps": reps,
        "ms_per_prompt": round(dt * 1e3, 2), "higher_is_better": True,
        "first_prompt_ms": round(first * 1e3, 2), "reserve_ms": round(reserve * 1e3, 2),
        "weight_images_GB": 0.0,  # (r03: the GEMM dequantizes the Q4_0 weights in LDS, no fp16 copies)
        "dtype": "f16 MFMA, f32 accumulate", "data": "synthetic (random-init weights, drawn on device)",
        "config": {"workload": f"{args.config} prompt eval, N={N}", "mode": "fast"},
        "roofline": {"bound": "mfma", "achieved": round(tflops, 1), "peak": 2500.0, "unit": "TFLOP/s",
                     "frac": round(tflops / 2500.0, 4), "traffic": None,
                     "flops": {"gemm": gemm_flops, "attention": attn_flops}},
        "exact_mode": exact,
    }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=248)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="gpt-j-6B", choices=["gpt-j-6B", "pythia-12b", "gpt-neoxt-20b", "bloom-560m",
                                                              "codegen-16B"])
    ap.add_argument("--mode", default="exact", choices=["exact", "fast"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-fast", action="store_true", help="skip the fast-mode companion measurement")
    ap.add_argument("--pipeline", action="store_true",
                    help="split the layers over the ranks (one residual send per stage boundary per token)")
    ap.add_argument("--prefill", type=int, default=0,
                    help="time one prompt eval of this many tokens instead of decode (fast-mode fp16 MFMA GEMM)")
    ap.add_argument("--prefill-exact", action="store_true",
                    help="with --prefill: also time the prompt once on the exact (oracle-identical) path")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: host-staged sends, for rehearsing the pipeline with ranks sharing a GPU")
    ap.add_argument("--no-pipeline-20b", action="store_true",
                    help="skip the GPT-NeoXT-20B layer-split companion measurement")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the bounded pythia-12b exact-decode companion measurement")
    ap.add_argument("--no-prefill-companion", action="store_true",
                    help="skip the bounded codegen-16B 2048-token prefill companion measurement")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    if args.pipeline:
        run_pipeline(args, world, rank, dev, dist)
        return
    if args.prefill:
        run_prefill(args, dev)
        return

    arch_s, hp = mg.CONFIGS[args.config]
    arch = ARCHS[arch_s]
    n_ctx = max(512, len(PROMPT) + args.warmup + args.steps + 96)
    model = hip.Model.create(arch, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                        n_layer=hp.n_layer, n_rot=hp.n_rot,
                                        use_parallel_residual=hp.use_parallel_residual),
                             n_ctx=n_ctx, device=dev)
    model.randomize(seed=1234 + rank, std=0.02)
    model.set_mode(hip.MODE_EXACT if args.mode == "exact" else hip.MODE_FAST)
    model.set_graph(not args.no_graph)

    logits = model.eval(0, PROMPT)
    n_past = len(PROMPT)
    tok = int(np.argmax(logits))

    def run_steps(k):
        # greedy decode kept on the device (vsim_model_generate): each step's argmax feeds
        # the next without a host round trip; the same tokens as eval() + numpy.argmax
        # (tests/test_gpu_model.py::test_generate_matches_stepwise_greedy)
        nonlocal n_past, tok
        if k:
            tok = model.generate(n_past, tok, k)[-1]
            n_past += k

    run_steps(args.warmup)
    start = (n_past, tok)  # the profile pass and the fast companion replay these positions

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    run_steps(args.steps)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # live roofline of the dominant kernel: an event pair around every launch (per kernel
    # kind, with its algorithmic bytes), over a second pass of the same decode steps
    roofline = None
    if not args.no_profile:
        n_past, tok = start
        model.set_profile(True)
        t1 = time.perf_counter()
        run_steps(args.steps)
        torch.cuda.synchronize()
        prof_wall = time.perf_counter() - t1
        kernels = model.profile_kernels()
        model.set_profile(False)
        roofline = roofline_from_profile(kernels, prof_wall, args.mode, hp.n_embd, hp.n_ff)
        if roofline is not None:
            roofline["measured_copy_GBps"] = measured_copy_gbps()
            roofline["frac_of_measured_copy"] = round(roofline["achieved"] / roofline["measured_copy_GBps"], 4)

    tokens_total = args.steps * world
    value = tokens_total / elapsed
    bw = q4_weight_bytes(arch_s, hp)
    info = model.info()
    line = {
        "metric": metric_name(args.config),
        "value": round(value, 3),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (Q4_0 x Q4_0 operands)",
        "data": "synthetic (random-init weights of the config's shapes, drawn on device)",
        "config": {"workload": f"{args.config} Q4_0 decode, {args.steps} timed tokens after a 5-token prompt "
                               f"+ {args.warmup} warm-up tokens, batch 1",
                   "mode": args.mode, "n_ctx": n_ctx, "parallelism": f"replicas{world}" if world > 1 else "single",
                   "weight_bytes_per_token": bw,
                   "weight_stream_GBps": round(bw * value / world / 1e9, 1),
                   "kernels_per_step": info["kernels_per_eval"], "graph": info["graph"]},
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_fast and args.mode == "exact":
        # (rewinds to the end of the warm-up: positions are overwritten, n_ctx bounds the rest)
        line["fast_mode"] = fast_companion(model, start[0], start[1], args.steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(arch_s, hp)
    model.close()
    if rank == 0 and world == 1 and not args.no_other_configs and args.config == "gpt-j-6B" and args.mode == "exact":
        line["other_configs"] = {"pythia-12b": decode_companion("pythia-12b", dev)}
    if rank == 0 and world == 1 and not args.no_prefill_companion and args.config == "gpt-j-6B" and args.mode == "exact":
        line["prefill_codegen16b"] = prefill_companion()
    if not args.no_pipeline_20b and args.config == "gpt-j-6B":
        if dist is not None:
            dist.barrier()
        line["pipeline_20b"] = pipeline_companion(args, world, rank, local)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
