"""One rank of the engine-level data-parallel check (tests/test_dp_engine_gpu.py).

Launched as `python -m torch.distributed.run --nproc-per-node 2 ... tests/dp_engine_worker.py
<out_dir>`; both ranks run on cuda:0 over gloo (RCCL refuses two ranks on one
device), each with half of the batch, through the real Trainer.step: global
loss normaliser all-reduced before backward, Engine.backward's per-layer
hooks issuing GradBucketer's async all-reduces.  Optional second argument:
the precision ("fp32" default; "bf16" runs the weight gradients on the side
stream, so every hook issues its all-reduce from that stream).""" 
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tests.dp_engine_common import build, make_batch  # noqa: E402


def main():
    out_dir = sys.argv[1]
    precision = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from smer_music_generation_amd.train import Trainer
    m, v = build("cuda", precision)
    b = make_batch(v)
    rows = np.arange(rank * 2, rank * 2 + 2)
    bt = {k: torch.from_numpy(np.asarray(x)[rows]).to("cuda") for k, x in b.items()}
    tr = Trainer(m, v)
    assert tr.world == world
    loss = tr.step(bt)
    lt = loss.detach().clone()
    dist.all_reduce(lt)
    torch.cuda.synchronize()
    torch.save({"grad": m.flat_grad().cpu(), "loss": lt.cpu(),
                "param": m.flat_parameters().cpu()}, os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
