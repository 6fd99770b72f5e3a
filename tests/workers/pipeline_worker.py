"""One rank of the layer-split decode on the real HIP stages (tests/test_gpu_pipeline.py).

gloo between processes that share one GPU: the residual and the token are staged through
host memory (RCCL needs one GPU per rank).  The prompt goes through pipeline.pipeline_step
(general path), the decode steps through pipeline.decode_steps with the device-resident
stage step (vsim_model_stage_step: graph-captured, device argmax on the last stage).
The last rank writes the generated tokens to --out as JSON.
"""
import argparse
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vsim_amd import hip, pipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--arch", type=int, required=True)
    ap.add_argument("--n-layer", type=int, required=True)
    ap.add_argument("--n-embd", type=int, required=True)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rank, world = a.rank, a.world
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    l0, l1 = pipeline.layer_range(a.n_layer, world, rank)
    model = hip.Model.load(a.model, a.arch, layer_begin=l0, layer_end=l1)
    model.set_graph(bool(a.graph))
    first, last = rank == 0, rank == world - 1
    E = a.n_embd

    def sync():
        model.sync()
        torch.cuda.synchronize()

    # bench.py's host-staged transport (gloo: the ranks share one GPU)
    send, recv = pipeline.make_transport(dist, True, sync=sync)

    prompt = [50278, 12092, 2, 0, 50281][:5]
    prompt = [p % 128 for p in prompt]
    rbuf = torch.empty((len(prompt), E), dtype=torch.float32, device="cuda")
    tokt = torch.zeros(1, dtype=torch.int64)

    def stage(n_past, ids, resid_in, resid_out):
        return model.eval(n_past, ids, resid_in=resid_in, resid_out=resid_out)

    tok = pipeline.pipeline_step(rank, world, 0, prompt, stage, send, recv, rbuf, tokt)
    tok_dev = torch.tensor([tok], dtype=torch.int32, device="cuda")
    rin = torch.empty(E, dtype=torch.float32, device="cuda")
    rout = torch.empty(E, dtype=torch.float32, device="cuda")
    model.stage_bind(tok_in=tok_dev.data_ptr() if first else 0, resid_in=0 if first else rin.data_ptr(),
                     resid_out=0 if last else rout.data_ptr(), tok_out=tok_dev.data_ptr() if last else 0)
    model.stage_begin(len(prompt))
    toks = [tok]

    def record(i):
        model.sync()
        toks.append(int(tok_dev.item()))

    pipeline.decode_steps(rank, world, model.stage_step, a.steps, send, recv, rin, rout, tok_dev,
                          record=record if last else None)
    model.sync()
    if last:
        with open(a.out, "w") as f:
            json.dump({"tokens": toks, "prompt": prompt}, f)
    dist.barrier()
    dist.destroy_process_group()
    model.close()


if __name__ == "__main__":
    main()
