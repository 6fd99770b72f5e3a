"""The model-file loader's checks (vsim_model_load_file), as the reference's loader makes them
(vsim.cpp:108-458: header, vocab, tensor records with names, shapes, types and sizes): a
corrupted file must be refused with VSIM_EFILE and a message naming the problem, never loaded
with transposed or garbage weights, and without leaking the half-built model."""
import ctypes
import struct

import pytest

from vsim_amd import hip
from vsim_amd import modelgen as mg

pytestmark = pytest.mark.gpu

VSIM_EFILE = -4


def records(path, arch_s, hp):
    """(header+vocab bytes, [(n_dims, name, ftype, ne, raw)])"""
    buf = open(path, "rb").read()
    off = 4 + (7 if arch_s == "gptneox" else 6) * 4 + (4 if arch_s == "gptj" else 0)
    for _ in range(hp.n_vocab):
        (ln,) = struct.unpack_from("<I", buf, off)
        off += 4 + ln
    head, recs = buf[:off], []
    while off < len(buf):
        nd, ln, ft = struct.unpack_from("<3i", buf, off)
        off += 12
        ne = list(struct.unpack_from(f"<{nd}i", buf, off))
        off += 4 * nd
        name = buf[off:off + ln].decode()
        off += ln
        n = 1
        for v in ne:
            n *= v
        nbytes = n * 4 if ft == 0 else n // 32 * 20
        recs.append([nd, name, ft, ne, buf[off:off + nbytes]])
        off += nbytes
    return head, recs


def emit(path, head, recs, truncate=0):
    out = bytearray(head)
    for nd, name, ft, ne, raw in recs:
        nb = name.encode()
        out += struct.pack("<3i", nd, len(nb), ft) + struct.pack(f"<{len(ne)}i", *ne) + nb + raw
    open(path, "wb").write(bytes(out[:len(out) - truncate] if truncate else out))


def load_rc(path, arch):
    h = ctypes.c_void_p()
    rc = hip.lib().vsim_model_load_file(path.encode(), arch, 128, 0, 0, -1, ctypes.byref(h))
    if rc == 0:
        hip.lib().vsim_model_free(h)
    return rc, hip.lib().vsim_last_error().decode()


@pytest.fixture
def base(tmp_path):
    arch_s, hp = mg.CONFIGS["tiny-neox"]
    path = str(tmp_path / "ok.bin")
    mg.write_model(path, arch_s, hp, seed=1, std=0.05)
    head, recs = records(path, arch_s, hp)
    return tmp_path, hp, head, recs


def test_valid_file_loads(base):
    tmp, hp, head, recs = base
    p = str(tmp / "same.bin")
    emit(p, head, recs)
    assert load_rc(p, hip.ARCH_GPTNEOX)[0] == 0


def test_transposed_weight_refused(base):
    tmp, hp, head, recs = base
    r = next(r for r in recs if r[1].endswith("mlp.dense_h_to_4h.weight"))
    r[3] = r[3][::-1]  # [4E, E] where [E, 4E] belongs: same byte count, wrong shape
    p = str(tmp / "t.bin")
    emit(p, head, recs)
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "wrong shape" in err, err


def test_unknown_and_missing_tensors_refused(base):
    tmp, hp, head, recs = base
    recs2 = [list(r) for r in recs]
    recs2[3][1] = "gpt_neox.layers.0.attention.bogus"
    p = str(tmp / "u.bin")
    emit(p, head, recs2)
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "unknown tensor" in err, err
    p = str(tmp / "m.bin")
    emit(p, head, recs[:-1])
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "missing" in err, err


def test_truncations_refused(base):
    tmp, hp, head, recs = base
    p = str(tmp / "tr.bin")
    emit(p, head, recs, truncate=7)
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "truncated" in err, err
    open(p, "wb").write(head[:17])
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "truncated" in err, err


def test_corrupt_records_refused(base):
    tmp, hp, head, recs = base
    recs2 = [list(r) for r in recs]
    recs2[0][0] = 5  # n_dims 5
    p = str(tmp / "c.bin")
    emit(p, head, recs2)
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "corrupt" in err, err
    recs3 = [list(r) for r in recs]
    w = next(r for r in recs3 if r[2] == 2)
    w[2] = 0  # declared F32 while the graph expects Q4_0
    w[4] = w[4] + bytes(len(w[4]) * 4 * 32 // 20 - len(w[4]))
    p = str(tmp / "ty.bin")
    emit(p, head, recs3)
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "type mismatch" in err, err


def test_f16_file_refused_with_reason(base):
    tmp, hp, head, recs = base
    h = bytearray(head)
    struct.pack_into("<i", h, 4 + 6 * 4, 1)  # f16 = 1
    p = str(tmp / "f16.bin")
    open(p, "wb").write(bytes(h))
    rc, err = load_rc(p, hip.ARCH_GPTNEOX)
    assert rc == VSIM_EFILE and "Q4_0" in err, err
