"""Where the barrier-free chain GEMVs wait (r05 diagnostic): GPT-J-6B exact decode on the
VSIM_NB_STAMPS build (tools/build_variant.sh nbstamps Makefile 's/-fno-slp-vectorize$/& -DVSIM_NB_STAMPS/'),
then the per-workgroup s_memtime sums of the last layer's tail (fc_out tiles 0..127, the
out-projection tiles after the heads): medians per chunk (cycles of the shader clock), and the
tail's s_memrealtime timeline by role."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 64
arch_s, hp = mg.CONFIGS["gpt-j-6B"]
m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head, n_layer=hp.n_layer,
                                         n_rot=hp.n_rot, use_parallel_residual=hp.use_parallel_residual),
                     n_ctx=512, device=0)
m.randomize(seed=1234, std=0.02)
m.set_mode(hip.MODE_EXACT)
m.set_graph(True)
tok = int(np.argmax(m.eval(0, [50278, 12092, 2, 0, 50281])))
m.generate(5, tok, steps)
buf = np.zeros((2048, 32), np.uint64)
f = hip.lib().vsim_debug_nb_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert f(buf.ctypes.data, buf.nbytes) == 0
m.close()


def role(name, rows, nprod, off):
    b = buf[rows]
    nch = np.maximum(b[:, 3].astype(float), 1)
    dur = (b[:, 1] - b[:, 0]).astype(float)
    print(f"{name}: {len(rows)} workgroups, chunks {int(np.median(nch))}, position {5 + steps}")
    print(f"  consumer: {np.median(dur / nch):8.0f} cycles per chunk (p10 {np.percentile(dur / nch, 10):.0f}, "
          f"p90 {np.percentile(dur / nch, 90):.0f}), waiting for producers {np.median(b[:, 2] / nch):6.0f}")
    for k, what in enumerate(off):
        v = b[:, what[1]:what[1] + nprod].astype(float) / nch[:, None]
        print(f"  producers {what[0]:<10}: median {np.median(v):7.0f}  p90 {np.percentile(v, 90):7.0f} cycles per chunk")


role("tail fc_out tiles", np.arange(0, 128), 8, [("dma wait", 4), ("slot wait", 12), ("compute", 20)])
NA = 32  # heads x 2 workgroups (r05 ATT_SPLIT)
role("tail out-proj tiles", np.arange(128 + NA, 256 + NA), 8, [("dma wait", 4), ("slot wait", 12), ("compute", 20)])

# the last tail's timeline (s_memrealtime, 100 MHz; rows 1536 + workgroup): fc_out tiles, QKV
# workgroups (three consumers' ends), heads (count reached, end), out-projection (count, end)
nf, nq = 128, (128 if os.environ.get("VSIM_TAIL_QKV", "0") == "1" else 0)
na, no = NA, 128
tl = buf[1536:1536 + nf + nq + na + no, :8].astype(np.int64)
t0 = tl[:, 0].min()
us = lambda v: (v - t0) / 100.0  # noqa: E731


def tlrow(name, rows, cols):
    r = tl[rows]
    print(f"{name:10s} start med {np.median(us(r[:, 0])):6.2f} max {us(r[:, 0]).max():6.2f} us" +
          "".join(f" | {c} med {np.median(us(r[:, i])):6.2f} max {us(r[:, i]).max():6.2f}" for c, i in cols))


print("tail timeline (us from the first workgroup's start):")
tlrow("fc_out", np.arange(0, nf), [("dma issued", 4), ("chunk 0 landed", 5), ("chunk 0 counted", 7), ("consumer has chunk 0", 3), ("end", 2)])
if nq:
    tlrow("QKV", np.arange(nf, nf + nq), [("Q end", 1), ("K end", 2), ("V end", 3)])
tlrow("heads", np.arange(nf + nq, nf + nq + na), [("attn", 1), ("end", 2)])
tlrow("out-proj", np.arange(nf + nq + na, nf + nq + na + no), [("ready", 1), ("end", 2)])
# the heads' phases (ATT_STAMP: columns 4-7 = KQ, softmax, KQV, quantize starts; 1 = done)
hr = tl[nf + nq:nf + nq + na]
ph = buf[1536 + nf + nq:1536 + nf + nq + na, 4:8].astype(np.int64)
print("heads phases (us, medians): setup+RoPE %.2f  KQ %.2f  softmax %.2f  KQV %.2f  quantize %.2f" % (
    np.median(ph[:, 0] - hr[:, 0]) / 100, np.median(ph[:, 1] - ph[:, 0]) / 100, np.median(ph[:, 2] - ph[:, 1]) / 100,
    np.median(ph[:, 3] - ph[:, 2]) / 100, np.median(hr[:, 1] - ph[:, 3]) / 100))
# the slowest fc_out tiles (end time, consumer wait per chunk, its producers' slot wait)
fo = tl[:nf]
order = np.argsort(-fo[:, 2])
print("slowest and median fc_out tiles (index, XCD = index % 8, end us, consumer wait/chunk, producer slot wait/chunk,"
      " dma wait/chunk, consumer cycles, consumer us, GHz):")
for i in list(order[:8]) + list(order[60:64]):
    b = buf[i]
    nchk = max(int(b[3]), 1)
    cyc = float(b[1] - b[0])
    dur = (fo[i, 2] - fo[i, 0]) / 100.0
    print(f"  {i:4d} {i % 8} {us(fo[i, 2]):6.2f} {b[2] / nchk:7.0f} {np.median(b[12:20]) / nchk:7.0f} {np.median(b[4:12]) / nchk:7.0f}"
          f" {cyc:9.0f} {dur:6.2f} {cyc / dur / 1e3:5.2f}")
print("end-time quartiles:", np.percentile(us(fo[:, 2]), [0, 25, 50, 75, 100]).round(2))

# per chunk of the last tail's fc_out tiles (rows 960/1088/1216 + tile: the consumer's wait for
# chunk c, the time it asked for chunk c (its wait_ready: three batches before chunk c-1 ends), the
# time chunk c's last producer counted itself)
cw = buf[960:1088].astype(np.int64)
cs = buf[1088:1216].astype(np.int64)
if cs[:, 1].any():
    nchk = int(np.median(buf[:128, 3]))
    print("fc_out per chunk (medians over the tiles, shader cycles): c, consumer wait, asked(c) - asked(c-1)")
    for c in range(min(nchk, 32)):
        ln = np.median(cs[:, c] - cs[:, c - 1]) if c > 0 else float("nan")
        print(f"  {c:3d} {np.median(cw[:, c]):7.0f} {ln:7.0f}")
    print("fc_out producers (p, wave: dma wait, slot wait, compute per chunk; medians over tiles)")
    for p, w in enumerate([1, 2, 3, 5, 6, 7, 9, 10]):
        print(f"  p{p} w{w:2d}: {np.median(buf[:128, 4 + p] / nchk):6.0f} {np.median(buf[:128, 12 + p] / nchk):6.0f}"
              f" {np.median(buf[:128, 20 + p] / nchk):6.0f}")
if os.environ.get("NB_STAMPS_SAVE"):
    np.save(os.environ["NB_STAMPS_SAVE"], buf)
