"""Decode-step microbenchmark for rocprofv3: R requests x S source tokens,
`n` eager (or graph-replayed) decode steps of the C2 model."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=32)
    ap.add_argument("--S", type=int, default=1000)
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--T", type=int, default=600, help="decoder cache capacity (max_tgt)")
    ap.add_argument("--precision", default=None, help="fp32 / bf16 (default: the model's)")
    a = ap.parse_args()
    from smer_music_generation_amd import _lib
    from smer_music_generation_amd.decode import DecodeSession
    _lib.load()
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    m = bench.make_model(args, dev).eval()
    with torch.no_grad():
        s = DecodeSession(m, a.R, a.S, a.T, precision=a.precision, use_graph=a.graph)
        s.prefill(list(range(a.R)), [[4] * a.S for _ in range(a.R)])
        s.step([(i, [5], 0) for i in range(a.R)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.n):
            s.step([(i, [5], k + 1) for i in range(a.R)])
        t1 = time.perf_counter()
    print("R=%d S=%d graph=%d: %.3f ms/step" % (a.R, a.S, a.graph, (t1 - t0) * 1e3 / a.n))


if __name__ == "__main__":
    main()
