"""Per-shape GEMM time inside the real C2 train step (HIP events around
every launch, bench.py's KernelTimer): where the GEMM time goes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from smer_music_generation_amd import _lib, ops
    from smer_music_generation_amd.synth import synth_training_batch
    from smer_music_generation_amd.train import Trainer
    from smer_music_generation_amd.vocab import WordVocab
    _lib.load()
    args = bench.parse_args([])
    precision = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    if len(sys.argv) > 2 and sys.argv[2] == "c4":
        args.layers, args.d_model, args.nhead, args.seq, args.tgt = 12, 768, 12, 2048, 512
    dev = torch.device("cuda", 0)
    v = WordVocab(0, bench.CTRL)
    m = bench.make_model(args, dev, precision)
    tr = Trainer(m, v, lr=1e-4)
    b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
    bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
    for _ in range(3):
        tr.step(bt)
    torch.cuda.synchronize()
    t = ops.KernelTimer()
    ops.GEMM_TIMER = t
    steps = 3
    for _ in range(steps):
        tr.step(bt)
    torch.cuda.synchronize()
    ops.GEMM_TIMER = None
    rows = sorted(t.by_shape().items(), key=lambda kv: -kv[1][1])
    tot = sum(r[1][1] for r in rows)
    print("%-40s %5s %9s %9s %7s" % ("shape", "n/st", "us/launch", "ms/step", "TF/s"))
    for tag, (n, ms, fl) in rows:
        print("%-40s %5d %9.1f %9.3f %7.0f" % (tag, n // steps, 1000 * ms / n, ms / steps,
                                               fl / (ms / 1e3) / 1e12))
    print("total GEMM ms/step %.3f" % (tot / steps))


if __name__ == "__main__":
    main()
