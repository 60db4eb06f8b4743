"""Data-parallel path on CPU: 2 gloo ranks, each with half the batch.

Exercises the real DP pieces of smer_music_generation_amd.train — the
per-layer flat-buffer ranges (`layer_ranges`), the asynchronous bucketed
SUM all-reduce issued in backward order (`GradBucketer`) and the global
loss normaliser (denominator all-reduced before backward) — with the oracle
as the per-rank compute, and checks the reduced gradient equals the
single-process gradient of the concatenated batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CFG = dict(d_model=32, nhead=2, num_encoder_layers=2, num_decoder_layers=2)
F_ = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from oracle import ref_cpu
    from smer_music_generation_amd.model import ScoreTransformer
    from smer_music_generation_amd.synth import synth_training_batch
    from smer_music_generation_amd.vocab import WordVocab
    v = WordVocab(0, ['key', 'tensile', 'density', 'polyphony', 'occupation'])
    torch.manual_seed(3)
    model = ScoreTransformer(309, CFG["d_model"], CFG["nhead"], 2, 2, F_, 200, 0.0, 0.0)
    sd = {k: t.detach().clone() for k, t in model.state_dict().items()}
    b = synth_training_batch(21, v, 4, 48, 16)
    b["input"][3, 40:] = 0
    b["input_pad_mask"] = b["input"] == 0
    b["target_out"][2, 10:] = 0  # unequal non-pad counts across ranks
    return ref_cpu, model, sd, b, v


def _grads(ref_cpu, sd, b, v, rows, denom=None):
    params = {k: t.clone().requires_grad_(True) for k, t in sd.items() if k != "pos_enc.pe"}
    full = dict(params)
    full["pos_enc.pe"] = sd["pos_enc.pe"]
    sel = lambda k: torch.as_tensor(b[k][rows])  # noqa: E731
    src, tin, tout = sel("input"), sel("target_in"), sel("target_out")
    skpm, tkpm = sel("input_pad_mask"), sel("target_pad_mask")
    T = tin.shape[1]
    mask = ref_cpu.nopeek_mask(T).unsqueeze(0).repeat(src.shape[0], 1, 1)
    logits, _ = ref_cpu.forward(full, CFG, src, tin, skpm, tkpm, skpm.clone(), mask)
    w, ce_all = ref_cpu.criterion_weights(309, 8, v.control_indices, 0.8)
    y = tout.reshape(-1)
    local_denom = ce_all[y].sum()
    if denom is not None:
        denom = denom(local_denom)
    loss, _ = ref_cpu.weighted_ce(logits, tout, w, ce_all, denom=denom)
    loss.backward()
    return {k: p.grad.detach() for k, p in params.items()}, loss.detach()


def _to_flat(model, grads):
    flat = torch.zeros_like(model.flat_parameters())
    for name, g in grads.items():
        o = model._offsets[name]
        flat[o: o + g.numel()] = g.reshape(-1)
    return flat


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from smer_music_generation_amd.train import GradBucketer, layer_ranges
    ref_cpu, model, sd, b, v = _setup()
    rows = np.arange(rank * 2, rank * 2 + 2)

    def global_denom(local):
        t = local.detach().clone()
        dist.all_reduce(t)  # before backward (train.py:736-742 over the whole batch)
        return t

    grads, loss = _grads(ref_cpu, sd, b, v, rows, denom=global_denom)
    flat = _to_flat(model, grads)
    ranges = layer_ranges(model)
    bk = GradBucketer(flat, ranges)
    order = ["head"] + ["dec%d" % i for i in reversed(range(2))] + \
        ["enc%d" % i for i in reversed(range(2))] + ["embedding"]
    for name in order:
        bk.reduce(name)
    bk.finish()
    lt = loss.clone()
    dist.all_reduce(lt)
    torch.save({"flat": flat, "loss": lt}, os.path.join(out_dir, "rank%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def test_layer_ranges_cover_every_parameter():
    from smer_music_generation_amd.train import layer_ranges
    _, model, _, _, _ = _setup()
    ranges = layer_ranges(model)
    covered = np.zeros(model.flat_parameters().numel(), dtype=np.int32)
    for a, b in ranges.values():
        covered[a:b] += 1
    for name, p in model.named_parameters():
        o = model._offsets[name]
        assert (covered[o: o + p.numel()] == 1).all(), name
    assert covered.max() == 1


@pytest.mark.timeout(600)
def test_two_rank_gloo_matches_single_process(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    ref_cpu, model, sd, b, v = _setup()
    grads, loss = _grads(ref_cpu, sd, b, v, np.arange(4))
    ref_flat = _to_flat(model, grads)
    for r in range(world):
        got = torch.load(os.path.join(tmp_path, "rank%d.pt" % r), weights_only=True)
        assert abs(float(got["loss"]) - float(loss)) < 1e-5
        err = (got["flat"] - ref_flat).abs().max() / ref_flat.abs().max()
        assert err < 1e-5, err
