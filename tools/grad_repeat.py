"""Bitwise repeatability of one train step's gradients: the C4 fixture model
stepped K times at lr = 0 on the fixture batch (weights unchanged, no
dropout), every step's gradients compared with the first; prints the
parameters whose gradients differ and by how much.
    python tools/grad_repeat.py [K] [precision] [c2bench]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_prod_gpu import C4, CTRL, _fixture, prod_model  # noqa: E402


def main():
    from smer_music_generation_amd.train import Trainer
    from smer_music_generation_amd.vocab import WordVocab
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 3 and sys.argv[3] == "c2bench":
        # the bench's C2 step at full size (B 32, S 1024, T 256), dropout 0
        import bench
        from smer_music_generation_amd.synth import synth_training_batch
        args = bench.parse_args([])
        args.dropout = 0.0
        m = bench.make_model(args, dev, prec)
        v = WordVocab(0, CTRL)
        tr = Trainer(m, v, lr=0.0)
        b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
    else:
        z, meta = _fixture(os.path.join(ROOT, "tests", "golden"), "train_c4")
        m = prod_model(C4, prec, z, meta["param_names"])
        tr = Trainer(m, WordVocab(0, CTRL), lr=0.0, eos_weight=0.8)
        src = z["src"].astype(np.int64)
        tin = z["tgt_in"].astype(np.int64)
        b = {"input": src, "target_in": tin, "target_out": z["tgt_out"].astype(np.int64),
             "input_pad_mask": src == 0, "target_pad_mask": tin == 0}
    bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
    names = [n for n, _ in m.named_parameters()]
    ref = None
    bad = {}
    for k in range(K):
        tr.step(bt)
        torch.cuda.synchronize()
        g = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        if ref is None:
            ref = g
            continue
        for n in names:
            if not torch.equal(g[n], ref[n]):
                d = (g[n].float() - ref[n].float()).abs()
                rel = d.max().item() / max(ref[n].float().abs().max().item(), 1e-30)
                nd = int((d > 0).sum().item())
                bad.setdefault(n, []).append((k, nd, rel))
    out = os.environ.get("SMER_GRAD_SAVE")
    if out:  # the first step's gradients, for comparisons across processes / switches
        torch.save({n: t.cpu() for n, t in ref.items()}, out)
    cmp = os.environ.get("SMER_GRAD_CMP")
    if cmp:
        other = torch.load(cmp, weights_only=True)
        diff = [n for n in names if not torch.equal(other[n], ref[n].cpu())]
        print("vs %s: %d parameters differ (first: %s)" % (cmp, len(diff), diff[:3]))
    print("steps %d, parameters %d, differing %d" % (K, len(names), len(bad)))
    print("identical: %s" % [n for n in names if n not in bad])
    for n in names:
        if n in bad:
            print("  %-48s %s" % (n, ["step %d: %d elems, max rel %.2e" % x for x in bad[n]][:3]))


if __name__ == "__main__":
    main()
