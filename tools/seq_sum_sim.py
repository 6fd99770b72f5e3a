#!/usr/bin/env python3
"""Host simulation of the exact LayerNorm mean fallback (vsim_amd/csrc/kern.hpp seq_sum_exact):
per 256-element chunk, the chunk's own exactness certificate, exact prefix sums, speculation
from the running double sum with a TwoSum check per position, restart at the first rounding
add, in-order fallback for a chunk that fails its certificate or rounds more than CAP times.
Checks the result against the plain sequential double sum (ggml.c:4264-4270) on crafted rows,
then counts restarts and in-order chunks on rows drawn like the decode activations that fail
the whole-row certificate (the rows that take the fallback).  DESIGN.md §4.1 quotes its output.
Usage: python tools/seq_sum_sim.py [--rows 3000] [--failing 200]"""
import argparse
import math

import numpy as np

CHUNK, CAP, BIG = 256, 32, 1 << 30


def ulp_exp(f):
    """kern.hpp ulp_exp: the exponent of the ulp of a float32's binade (zero -> BIG)."""
    b = int(np.array([f], dtype=np.float32).view(np.uint32)[0]) & 0x7FFFFFFF
    if b == 0:
        return BIG
    e = b >> 23
    return -149 if e == 0 else e - 150


def certified(x):
    um = min(ulp_exp(v) for v in x)
    sa = float(np.sum(np.abs(np.asarray(x, dtype=np.float64))))
    return um == BIG or sa * (1 + 2.0 ** -30) < 2.0 ** (53 + um)


def sequential(x):
    s = 0.0
    for v in x:
        s += float(v)
    return s


def speculative(x):
    s, stats = 0.0, [0, 0]  # in-order chunks, restarts
    for c0 in range(0, len(x), CHUNK):
        ch = x[c0:c0 + CHUNK]
        vals = [float(v) for v in ch]
        b = 0
        if certified(ch):
            p = [0.0]
            for v in vals:
                p.append(p[-1] + v)  # exact under the chunk certificate
            pb = 0.0
            for _ in range(CAP + 1):
                j = None
                for jj in range(b + 1, len(vals) + 1):
                    d = p[jj] - pb
                    t = s + d
                    bb = t - s
                    er = (s - (t - bb)) + (d - bb)
                    if er != 0.0 or t != t:
                        j = jj
                        break
                if j is None:
                    s, b = s + (p[-1] - pb), len(vals)
                    break
                s, pb, b = s + (p[j] - pb), p[j], j
                stats[1] += 1
        if b < len(vals):
            stats[0] += 1
            for v in vals[b:]:
                s += v
    return s, stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=3000)
    ap.add_argument("--failing", type=int, default=200)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    bad = 0
    for t in range(a.rows):
        x = (rng.standard_normal(4096) * rng.choice([0.05, 1, 30])).astype(np.float32)
        kind = t % 5
        if kind == 1:
            x[rng.integers(0, 4096, rng.integers(1, 4))] = rng.standard_normal() * 1e-7
        if kind == 2:
            x[rng.integers(0, 4096, 50)] *= np.float32(1e-9)
        if kind == 3:
            x[rng.integers(0, 4096, 3)] = np.float32(1e30) * rng.standard_normal(3).astype(np.float32)
        if kind == 4:
            x[rng.integers(0, 4096, 5)] = np.float32(1e-40)
        r0, (r1, _) = sequential(x), speculative(x)
        bad += not (r0 == r1 or (math.isnan(r0) and math.isnan(r1)))
    print(f"crafted rows: {bad} of {a.rows} differ from the sequential sum")
    n = tried = rs = sc = 0
    while n < a.failing:
        tried += 1
        x = (rng.standard_normal(4096) * rng.choice([0.1, 1, 5])).astype(np.float32)
        if certified(x):
            continue
        n += 1
        r1, (c, r) = speculative(x)
        assert r1 == sequential(x)
        sc += c
        rs += r
    print(f"rows failing the whole-row certificate: {n / tried:.4f} of rows; per failing row "
          f"{rs / n:.3f} restarts, {sc / n:.3f} in-order chunks")


if __name__ == "__main__":
    main()
