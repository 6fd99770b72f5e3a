"""Deterministic synthetic ggml model files (no checkpoints exist offline).

Writes the two on-disk formats the path reads:
  * GPT-NeoX: vsim.cpp:108-458 (header vsim.cpp:119-150, names vsim.cpp:287-346)
  * GPT-J:    convert_gptj_to_ggml.py:106-126 header + explicit vocab count,
              names of HF GPTJForCausalLM (quantize_gptj.cpp quantizes 2-D weights).
2-D ".weight" tensors are Q4_0 (20-byte blocks: fp32 d + 16 nibble bytes,
ggml.c:204-251); 1-D tensors are F32.  Values: numpy PCG64, N(0, 0.02) for matrices
and biases, 1 + N(0, 0.02) for LayerNorm gains.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

QK = 32
QBYTES = 20


def quantize_q4_0(x: np.ndarray) -> np.ndarray:
    """quantize_row_q4_0 (ggml.c:209-251) over every 32-block; returns uint8 bytes.

    Float32 arithmetic throughout, C round() = half away from zero (done in float64,
    where x*id is exact), nibble pair packing lo = q[2l], hi = q[2l+1].
    """
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, QK)
    amax = np.max(np.abs(x), axis=1)
    d = (amax / np.float32(7.0)).astype(np.float32)
    with np.errstate(divide="ignore"):
        idv = np.where(d != 0, np.float32(1.0) / d, np.float32(0.0)).astype(np.float32)
    v = (x * idv[:, None]).astype(np.float32).astype(np.float64)
    q = np.where(v >= 0, np.floor(v + 0.5), np.ceil(v - 0.5)).astype(np.int64) + 8
    q = q.astype(np.uint8)
    packed = (q[:, 0::2] | (q[:, 1::2] << 4)).astype(np.uint8)
    out = np.empty((x.shape[0], QBYTES), dtype=np.uint8)
    out[:, :4] = d.view(np.uint8).reshape(-1, 4)
    out[:, 4:] = packed
    return out.reshape(-1)


def dequantize_q4_0(b: np.ndarray, k: int) -> np.ndarray:
    """dequantize_row_q4_0 (ggml.c:301-334) for rows of k weights."""
    blk = np.asarray(b, dtype=np.uint8).reshape(-1, QBYTES)
    d = blk[:, :4].copy().view(np.float32).reshape(-1)
    qs = blk[:, 4:]
    lo = (qs & 0xF).astype(np.int32) - 8
    hi = (qs >> 4).astype(np.int32) - 8
    q = np.empty((blk.shape[0], QK), dtype=np.int32)
    q[:, 0::2] = lo
    q[:, 1::2] = hi
    return (q.astype(np.float32) * d[:, None]).astype(np.float32).reshape(-1, k)


@dataclass
class HParams:
    n_vocab: int
    n_embd: int
    n_head: int
    n_layer: int
    n_rot: int
    use_parallel_residual: int = 1
    ftype: int = 2  # 2 = Q4_0

    @property
    def n_ff(self) -> int:
        return 4 * self.n_embd


# Named configurations (dims from SURVEY.md §8 table / public HF configs)
CONFIGS = {
    "gpt-j-6B": ("gptj", HParams(50400, 4096, 16, 28, 64)),
    "pythia-12b": ("gptneox", HParams(50288, 5120, 40, 36, 32)),
    "gpt-neoxt-20b": ("gptneox", HParams(50432, 6144, 64, 44, 24)),
    "codegen-16B": ("gptj", HParams(51200, 6144, 24, 34, 64)),
    # small parity models
    "tiny-neox": ("gptneox", HParams(128, 128, 4, 2, 8)),
    "small-neox": ("gptneox", HParams(512, 512, 8, 2, 32)),
    "tiny-gptj": ("gptj", HParams(128, 128, 4, 2, 16)),
    "small-gptj": ("gptj", HParams(512, 512, 4, 2, 64)),
    # BLOOM (ALiBi, no rotary: n_rot 0; serial residual; header n_mult = 1)
    "bloom-560m": ("bloom", HParams(250880, 1024, 16, 24, 0, 0)),
    "tiny-bloom": ("bloom", HParams(128, 128, 4, 2, 0, 0)),
    "small-bloom": ("bloom", HParams(512, 512, 8, 2, 0, 0)),
}


def tensor_specs(arch: str, hp: HParams):
    """(name, ne list, kind) with kind 'q' = Q4_0 matrix, 'w' = LN gain, 'b' = bias."""
    E, V, F, L = hp.n_embd, hp.n_vocab, hp.n_ff, hp.n_layer
    s = []
    if arch == "gptneox":
        s.append(("gpt_neox.embed_in.weight", [E, V], "q"))
        s.append(("gpt_neox.final_layer_norm.weight", [E], "w"))
        s.append(("gpt_neox.final_layer_norm.bias", [E], "b"))
        s.append(("embed_out.weight", [E, V], "q"))
        for i in range(L):
            p = f"gpt_neox.layers.{i}."
            s += [
                (p + "input_layernorm.weight", [E], "w"),
                (p + "input_layernorm.bias", [E], "b"),
                (p + "post_attention_layernorm.weight", [E], "w"),
                (p + "post_attention_layernorm.bias", [E], "b"),
                (p + "attention.query.weight", [E, E], "q"),
                (p + "attention.query.bias", [E], "b"),
                (p + "attention.key.weight", [E, E], "q"),
                (p + "attention.key.bias", [E], "b"),
                (p + "attention.value.weight", [E, E], "q"),
                (p + "attention.value.bias", [E], "b"),
                (p + "attention.dense.weight", [E, E], "q"),
                (p + "attention.dense.bias", [E], "b"),
                (p + "mlp.dense_h_to_4h.weight", [E, F], "q"),
                (p + "mlp.dense_h_to_4h.bias", [F], "b"),
                (p + "mlp.dense_4h_to_h.weight", [F, E], "q"),
                (p + "mlp.dense_4h_to_h.bias", [E], "b"),
            ]
    elif arch == "gptj":
        s.append(("transformer.wte.weight", [E, V], "q"))
        for i in range(L):
            p = f"transformer.h.{i}."
            s += [
                (p + "ln_1.weight", [E], "w"),
                (p + "ln_1.bias", [E], "b"),
                (p + "attn.k_proj.weight", [E, E], "q"),
                (p + "attn.v_proj.weight", [E, E], "q"),
                (p + "attn.q_proj.weight", [E, E], "q"),
                (p + "attn.out_proj.weight", [E, E], "q"),
                (p + "mlp.fc_in.weight", [E, F], "q"),
                (p + "mlp.fc_in.bias", [F], "b"),
                (p + "mlp.fc_out.weight", [F, E], "q"),
                (p + "mlp.fc_out.bias", [E], "b"),
            ]
        s.append(("transformer.ln_f.weight", [E], "w"))
        s.append(("transformer.ln_f.bias", [E], "b"))
        s.append(("lm_head.weight", [E, V], "q"))
        s.append(("lm_head.bias", [V], "b"))
    elif arch == "bloom":  # convert_bloom_to_ggml.py:22-34 names, q|k|v rows fused
        s.append(("tok_embeddings.weight", [E, V], "q"))
        s.append(("norm.weight", [E], "w"))
        s.append(("norm.bias", [E], "b"))
        for i in range(L):
            p = f"layers.{i}."
            s += [
                (p + "attention_norm.weight", [E], "w"),
                (p + "attention_norm.bias", [E], "b"),
                (p + "attention.query_key_value.weight", [E, 3 * E], "q"),
                (p + "attention.query_key_value.bias", [3 * E], "b"),
                (p + "attention.wo.weight", [E, E], "q"),
                (p + "attention.wo.bias", [E], "b"),
                (p + "ffn_norm.weight", [E], "w"),
                (p + "ffn_norm.bias", [E], "b"),
                (p + "feed_forward.w1.weight", [E, F], "q"),
                (p + "feed_forward.w1.bias", [F], "b"),
                (p + "feed_forward.w2.weight", [F, E], "q"),
                (p + "feed_forward.w2.bias", [E], "b"),
            ]
        s.append(("output_norm.weight", [E], "w"))
        s.append(("output_norm.bias", [E], "b"))
        s.append(("output.weight", [E, V], "q"))
    else:
        raise ValueError(arch)
    return s


def gen_tensors(arch: str, hp: HParams, seed: int = 0, std: float = 0.02):
    """Yield (name, ne, ftype, raw bytes) in file order."""
    rng = np.random.Generator(np.random.PCG64(seed))
    for name, ne, kind in tensor_specs(arch, hp):
        n = int(np.prod(ne))
        vals = rng.standard_normal(n, dtype=np.float32) * np.float32(std)
        if kind == "w":
            vals = vals + np.float32(1.0)
        if kind == "q":
            yield name, ne, 2, quantize_q4_0(vals.astype(np.float32)).tobytes()
        else:
            yield name, ne, 0, vals.astype(np.float32).tobytes()


def write_model(path: str, arch: str, hp: HParams, seed: int = 0, std: float = 0.02) -> None:
    with open(path, "wb") as f:
        f.write(struct.pack("<I", 0x67676D6C))
        if arch == "gptneox":
            f.write(struct.pack("<7i", hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot,
                                hp.use_parallel_residual, hp.ftype))
        elif arch == "bloom":  # convert_bloom_to_ggml.py:79-85 (multiple_of = 1)
            f.write(struct.pack("<6i", hp.n_vocab, hp.n_embd, 1, hp.n_head, hp.n_layer, hp.ftype))
        else:
            f.write(struct.pack("<6i", hp.n_vocab, hp.n_embd, hp.n_head, hp.n_layer, hp.n_rot, hp.ftype))
            f.write(struct.pack("<i", hp.n_vocab))
        for i in range(hp.n_vocab):
            tok = f"t{i}".encode()
            f.write(struct.pack("<I", len(tok)))
            f.write(tok)
        for name, ne, ftype, raw in gen_tensors(arch, hp, seed, std):
            nb = name.encode()
            f.write(struct.pack("<3i", len(ne), len(nb), ftype))
            f.write(struct.pack(f"<{len(ne)}i", *ne))
            f.write(nb)
            f.write(raw)


def read_model(path: str, arch: str):
    """Parse a ggml file -> (hparams dict, {name: (ne, ftype, bytes)})."""
    with open(path, "rb") as f:
        buf = f.read()
    off = 0

    def i32(n=1):
        nonlocal off
        v = struct.unpack_from(f"<{n}i", buf, off)
        off += 4 * n
        return v

    magic = struct.unpack_from("<I", buf, 0)[0]
    off = 4
    if magic != 0x67676D6C:
        raise ValueError("bad magic")
    if arch == "gptneox":
        nv, ne_, nh, nl, nr, pr, ft = i32(7)
        nvv = nv
    elif arch == "bloom":
        nv, ne_, _mult, nh, nl, ft = i32(6)
        nr, pr, nvv = 0, 0, nv
    else:
        nv, ne_, nh, nl, nr, ft = i32(6)
        pr = 1
        (nvv,) = i32()
    for _ in range(nvv):
        (ln,) = struct.unpack_from("<I", buf, off)
        off += 4 + ln
    hp = HParams(nv, ne_, nh, nl, nr, pr, ft)
    tensors = {}
    while off < len(buf):
        nd, ln, ft = i32(3)
        ne = list(i32(nd))
        name = buf[off:off + ln].decode()
        off += ln
        n = int(np.prod(ne))
        nbytes = n * 4 if ft == 0 else n // QK * QBYTES
        tensors[name] = (ne, ft, buf[off:off + nbytes])
        off += nbytes
    return hp, tensors
