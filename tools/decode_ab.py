"""Graph-replayed decode step, A/B of one environment switch in one process:
a session is captured per value of the switch (the switch is read while
the step is captured), then the replays are timed interleaved over rounds,
and the logits of the variants compared bitwise.

    python tools/decode_ab.py R S ENV_NAME VALUE_A VALUE_B
e.g. python tools/decode_ab.py 64 4096 SMER_DECODE_ODD_FIRST 1 0 (C5 shape)."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    R, S = int(sys.argv[1]), int(sys.argv[2])
    name, values = sys.argv[3], sys.argv[4:]
    from smer_music_generation_amd import _lib
    from smer_music_generation_amd.decode import DecodeSession
    _lib.load()
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    m = bench.make_model(args, dev).eval()
    sess, logits = {}, {}
    with torch.no_grad():
        for v in values:
            os.environ[name] = v
            s = DecodeSession(m, R, S, 600, use_graph=True)
            s.prefill(list(range(R)), [[4 + (i % 7)] * (S - i % 5) for i in range(R)])
            logits[v] = s.step([(i, [5], 0) for i in range(R)]).copy()
            sess[v] = s
        torch.cuda.synchronize()
        res = {v: [] for v in values}
        for _ in range(7):
            for v, s in sess.items():
                n = 100
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(n):
                    s.graph.replay()
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) * 1e6 / n)
    ref = values[0]
    for v, r in res.items():
        w = sorted(r)
        same = bool((logits[v] == logits[ref]).all())
        print("R=%d S=%d %s=%s: wall median %.1f min %.1f us/replay; logits bit-identical to %s=%s: %s"
              % (R, S, name, v, w[len(w) // 2], w[0], name, ref, same), flush=True)


if __name__ == "__main__":
    main()
