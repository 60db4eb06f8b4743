"""Graph-replayed decode step, A/B in one process: one request chain per
step (SMER_DECODE_CHAINS=1) against two request halves on two graph
branches (the default), interleaved over rounds.  C2 model, R requests x S
source tokens (C2: 32 x 1000, C5: 64 x 4100).  Also checks that both
variants produce the same logits bits."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    from smer_music_generation_amd import _lib
    from smer_music_generation_amd.decode import DecodeSession
    _lib.load()
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    m = bench.make_model(args, dev).eval()
    sess = {}
    logits = {}
    with torch.no_grad():
        for v in ("1", "2"):
            os.environ["SMER_DECODE_CHAINS"] = v
            s = DecodeSession(m, R, S, 600, use_graph=True)
            g = torch.Generator().manual_seed(0)
            srcs = [torch.randint(4, 300, (S - 7 * i,), generator=g).tolist() for i in range(R)]
            s.prefill(list(range(R)), srcs)
            logits[v] = s.step([(i, [5], 0) for i in range(R)]).copy()
            sess[v] = s
        os.environ.pop("SMER_DECODE_CHAINS")
        same = (logits["1"] == logits["2"]).all()
        print("R=%d S=%d logits bit-identical across chain counts: %s" % (R, S, bool(same)))
        torch.cuda.synchronize()
        res = {"1": [], "2": []}
        for _ in range(5):
            for v, s in sess.items():
                n = 50
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(n):
                    s.graph.replay()
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) * 1e6 / n)
    for v, r in res.items():
        w = sorted(r)
        print("R=%d S=%d chains=%s: wall median %.1f min %.1f us/replay" % (R, S, v, w[len(w) // 2], w[0]))


if __name__ == "__main__":
    main()
