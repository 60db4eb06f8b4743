"""Graph-replayed decode step, A/B in one process: host issue time and wall
time per replay of the captured step, with the cross-attention query
prologue (SMER_DECODE_QLN=1) and without, interleaved over rounds (C2 model,
R requests x 1000 source tokens)."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    from smer_music_generation_amd import _lib
    from smer_music_generation_amd.decode import DecodeSession
    _lib.load()
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    m = bench.make_model(args, dev).eval()
    sess = {}
    with torch.no_grad():
        for v in ("1", "0"):  # forced on / off (default "auto": on up to 64 rows)
            os.environ["SMER_DECODE_QLN"] = v
            s = DecodeSession(m, R, 1000, 600, use_graph=True)
            s.prefill(list(range(R)), [[4] * 1000 for _ in range(R)])
            s.step([(i, [5], 0) for i in range(R)])
            sess[v] = s
        torch.cuda.synchronize()
        res = {"1": [], "0": []}
        for _ in range(5):
            for v, s in sess.items():
                n = 100
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(n):
                    s.graph.replay()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                res[v].append(((t1 - t0) * 1e6 / n, (t2 - t0) * 1e6 / n))
    for v, r in res.items():
        w = sorted(x[1] for x in r)
        print("R=%d QLN=%s: host issue %.1f us/replay, wall median %.1f min %.1f us/replay"
              % (R, v, sum(x[0] for x in r) / len(r), w[len(w) // 2], w[0]))


if __name__ == "__main__":
    main()
