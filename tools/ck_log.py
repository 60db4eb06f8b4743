"""Per-launch checksum log of identical train steps (repeatability probe).

Every main-stream output of Engine.backward and every side-stream weight
gradient (with its dY / X inputs re-read on the side stream after the GEMM)
is checksummed on the stream that produced it (ops.CkLog, no host sync).
Steps at lr = 0 on one batch are compared entry by entry with the first
step: the first differing main-stream entry names the victim, the side
entries around it the aggressor.
    python tools/ck_log.py [K] [c4|c2bench]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_prod_gpu import C4, CTRL, _fixture, prod_model  # noqa: E402


def describe(a, b):
    """Where two versions of a victim tensor differ: rows, 16-B chunks, values."""
    a2 = a.reshape(-1, a.shape[-1]).float().cpu()
    b2 = b.reshape(-1, b.shape[-1]).float().cpu()
    ne = (a2 != b2) & ~(torch.isnan(a2) & torch.isnan(b2))
    rows = torch.nonzero(ne.any(1)).flatten().tolist()
    print("    victim %s: %d of %d elements differ, %d of %d rows: %s"
          % (tuple(a.shape), int(ne.sum()), ne.numel(), len(rows), a2.shape[0], rows[:24]))
    epc = 16 // a.element_size()
    ab = a.reshape(-1, a.shape[-1]).cpu()
    bb = b.reshape(-1, b.shape[-1]).cpu()
    if a.element_size() == 2:
        ab, bb = ab.view(torch.int16), bb.view(torch.int16)
    else:
        ab, bb = ab.view(torch.int32), bb.view(torch.int32)
    for r in rows[:8]:
        cols = torch.nonzero(ne[r]).flatten().tolist()
        chunks = sorted(set(c // epc for c in cols))
        rel = ((b2[r] - a2[r]).abs().max() / a2[r].abs().max().clamp_min(1e-30)).item()
        print("     row %d: %d cols differ, 16-B chunks %s; max |diff| / row max |good| %.3e"
              % (r, len(cols), chunks[:16], rel))
        print("       (col, col%%8, good, bad, ulps) %s"
              % [(c, c % 8, "%.4e" % a2[r, c].item(), "%.4e" % b2[r, c].item(),
                  int(bb[r, c].item()) - int(ab[r, c].item())) for c in cols[:12]])


def main():
    from smer_music_generation_amd import ops
    from smer_music_generation_amd.train import Trainer
    from smer_music_generation_amd.vocab import WordVocab
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mode = sys.argv[2] if len(sys.argv) > 2 else "c4"
    dev = torch.device("cuda", 0)
    if mode == "c2bench":
        import bench
        from smer_music_generation_amd.synth import synth_training_batch
        args = bench.parse_args([])
        args.dropout = 0.0
        m = bench.make_model(args, dev, "bf16")
        v = WordVocab(0, CTRL)
        tr = Trainer(m, v, lr=0.0)
        b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
    else:
        z, meta = _fixture(os.path.join(ROOT, "tests", "golden"), "train_c4")
        m = prod_model(C4, "bf16", z, meta["param_names"])
        tr = Trainer(m, WordVocab(0, CTRL), lr=0.0, eos_weight=0.8)
        src = z["src"].astype(np.int64)
        tin = z["tgt_in"].astype(np.int64)
        b = {"input": src, "target_in": tin, "target_out": z["tgt_out"].astype(np.int64),
             "input_pad_mask": src == 0, "target_pad_mask": tin == 0}
    bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
    names = [n for n, _ in m.named_parameters()]
    keep = [k for k in os.environ.get("SMER_CK_KEEP", "").split(",") if k]
    log = ops.CkLog(dev, keep=keep)
    ops.CK_LOG = log
    main_stream = torch.cuda.current_stream(dev).cuda_stream
    ref = None
    ref_g = None
    for k in range(K):
        log.reset()
        tr.step(bt)
        torch.cuda.synchronize()
        vals = log.values()
        ent = [(n, "M" if s == main_stream else "S", v) for (n, s), v in zip(log.names, vals)]
        g = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        kept = dict(log.kept)
        if ref is None:
            ref, ref_g, ref_kept = ent, g, kept
            print("step 0: %d log entries" % len(ent))
            continue
        if len(ent) != len(ref):
            print("step %d: %d entries vs %d" % (k, len(ent), len(ref)))
        diff = [i for i, (a, b_) in enumerate(zip(ent, ref)) if a[2] != b_[2]]
        nbad = sum(1 for n in names if not torch.equal(g[n], ref_g[n]))
        print("step %d: %d of %d log entries differ, %d of %d parameter gradients differ"
              % (k, len(diff), len(ent), nbad, len(names)))
        if diff:
            i0 = diff[0]
            print("  first differing entry #%d %s (%s)" % (i0, ent[i0][0], ent[i0][1]))
            lo = max(0, i0 - 12)
            for i in range(lo, min(len(ent), i0 + 8)):
                print("   %s #%-4d %-3s %-18s" % ("*" if i in diff else " ", i, ent[i][1], ent[i][0]))
            fm = [i for i in diff if ent[i][1] == "M"]
            if fm:
                print("  first differing MAIN entry #%d %s" % (fm[0], ent[fm[0]][0]))
                if fm[0] in kept and fm[0] in ref_kept:
                    describe(ref_kept[fm[0]], kept[fm[0]])
            print("  differing: %s" % ", ".join("#%d %s" % (i, ent[i][0]) for i in diff[:24]))
    ops.CK_LOG = None


if __name__ == "__main__":
    main()
