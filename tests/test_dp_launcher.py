"""Multi-GPU plumbing on CPU (gloo): bench.py's N-rank launcher, the
Trainer's rank-0 parameter broadcast at init and the opt-in
bf16 gradient all-reduce.  No HIP kernel runs here."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_dp_gloo import _free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_line(*extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--dry-run", "--steps", "2", "--warmup", "1"] + list(extra),
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_bench_gpus2_launches_two_ranks(wire):
    line = _bench_line("--grad-wire", wire)
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "dp2"
    assert line["params_in_sync_at_init"] is True
    assert line["allreduce_ok"] is True
    assert line["dry_run"] is True and line["value"] is None
    # both DP scalings -- weak (B per rank) and strong (the
    # global batch split over the ranks)
    modes = line["scaling_modes"]
    assert modes["weak"] == {"per_rank_batch": 32, "global_batch": 64}
    assert modes["strong"] == {"per_rank_batch": 16, "global_batch": 32}


@pytest.mark.timeout(300)
def test_bench_gpus2_strong_scaling_split():
    line = _bench_line("--global-batch", "48")
    assert line["scaling_modes"]["strong"] == {"per_rank_batch": 24, "global_batch": 48}


def _init_worker(rank, world, port, out_dir, broadcast):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smer_music_generation_amd.model import ScoreTransformer
    from smer_music_generation_amd.train import Trainer
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
    torch.manual_seed(10 + 7 * rank)  # ranks seeded differently
    m = ScoreTransformer(309, 32, 2, 2, 2, 64, 200, 0.0, 0.0)
    if rank == 0:
        torch.save(m.flat_parameters().clone(), os.path.join(out_dir, "rank0_before.pt"))
    tr = Trainer(m, v, broadcast=broadcast)
    assert tr.world == world
    torch.save({"flat": m.flat_parameters().clone(),
                "params": {k: p.detach().clone() for k, p in m.named_parameters()}},
               os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("broadcast", [True, False])
def test_trainer_init_broadcasts_rank0_params(tmp_path, broadcast):
    world = 2
    mp.spawn(_init_worker, args=(world, _free_port(), str(tmp_path), broadcast), nprocs=world,
             join=True)
    r0 = torch.load(os.path.join(tmp_path, "rank0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "rank1.pt"), weights_only=True)
    before = torch.load(os.path.join(tmp_path, "rank0_before.pt"), weights_only=True)
    assert torch.equal(r0["flat"], before)
    if broadcast:
        assert torch.equal(r0["flat"], r1["flat"])
        # the parameters are views of the flat buffer, so they moved with it
        for k, p in r1["params"].items():
            assert torch.equal(p, r0["params"][k]), k
    else:
        assert not torch.equal(r0["flat"], r1["flat"])  # the seeds really differ


def _wire_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smer_music_generation_amd.train import GradBucketer
    g = torch.Generator().manual_seed(rank)
    base = torch.randn(4096, generator=g)
    res = {}
    for name, wire in (("fp32", None), ("bf16", torch.bfloat16)):
        flat = base.clone()
        bk = GradBucketer(flat, {"a": (0, 1024), "b": (1024, 3000), "c": (3000, 4096)},
                          wire_dtype=wire)
        bk.reduce("c")
        bk.reduce("a")
        bk.finish()  # reduces "b" too
        res[name] = flat
    res["local"] = base
    torch.save(res, os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_bf16_wire_allreduce(tmp_path):
    world = 2
    mp.spawn(_wire_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rs = [torch.load(os.path.join(tmp_path, "rank%d.pt" % r), weights_only=True)
          for r in range(world)]
    exact = sum(r["local"].double() for r in rs)
    for r in rs:
        assert (r["fp32"].double() - exact).abs().max() < 1e-5
        # bf16 (8 significant bits, unit roundoff 2^-8): each rank's value is
        # rounded once and the sum once more: |err| <= 2^-7 * sum |x_r|
        bound = 2.0 ** -7 * sum(x["local"].double().abs() for x in rs) + 1e-30
        assert ((r["bf16"].double() - exact).abs() <= bound).all()
        assert r["bf16"].dtype == torch.float32
    assert torch.equal(rs[0]["bf16"], rs[1]["bf16"])
