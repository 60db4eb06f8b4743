"""Is the C2 train step host-bound?  Enqueue time of K steps (no sync) vs
the wall time once the GPU has drained them."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from smer_music_generation_amd.synth import synth_training_batch
    from smer_music_generation_amd.train import Trainer
    from smer_music_generation_amd.vocab import WordVocab
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    v = WordVocab(0, bench.CTRL)
    m = bench.make_model(args, dev)
    tr = Trainer(m, v, lr=1e-4)
    b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
    bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
    for _ in range(3):
        tr.step(bt)
    torch.cuda.synchronize()
    K = 10
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step(bt)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("enqueue %.2f ms/step, wall %.2f ms/step" % ((t1 - t0) / K * 1e3, (t2 - t0) / K * 1e3))
    # host cost of the op wrappers alone: a tiny GPU op per call
    from smer_music_generation_amd import ops
    x = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    w = torch.zeros(64, 64, device=dev, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        ops.linear(x, w)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print("ops.linear host cost %.1f us/call" % ((t1 - t0) * 1e3))


if __name__ == "__main__":
    main()
