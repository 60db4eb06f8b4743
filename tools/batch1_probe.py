"""Where the batch-1 plugin call's time goes (bench.py `infill.batch1`).

    python tools/batch1_probe.py [n_requests]

Runs the bench's batch-1 workload (C2 model, fp32 decode, weighted
sampling, one `generation_all` per request) with the session set-up,
prefill, per-token step (H2D + replay + D2H) and host grammar / sampling
timed separately, then the step's kernels alone (graph replays back to
back).
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from smer_music_generation_amd import decode, generation  # noqa: E402
from smer_music_generation_amd.vocab import WordVocab  # noqa: E402

T = {"init": 0.0, "prefill": 0.0, "step": 0.0, "advance": 0.0, "n_step": 0, "n_init": 0}


def _wrap(cls, name, key, count=None):
    f = getattr(cls, name)

    def g(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        T[key] += time.perf_counter() - t
        if count:
            T[count] += 1
        return r
    setattr(cls, name, g)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    args = bench.parse_args([])
    dev = torch.device("cuda:0")
    v = WordVocab(0, bench.CTRL)
    m = bench.make_model(args, dev).eval()
    ac = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    (wev, wtr, wbr), = bench._infill_requests(1, args.seq, 8100)
    np.random.seed(1)
    generation.generation_all(m, list(wev), dev, v, None, ac, wtr, wbr)
    _wrap(decode.DecodeSession, "__init__", "init", "n_init")
    _wrap(decode.DecodeSession, "prefill", "prefill")
    _wrap(decode.DecodeSession, "step", "step", "n_step")
    _wrap(generation._Span, "advance", "advance")
    reqs = bench._infill_requests(n, args.seq, 8000)
    np.random.seed(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for ev, tr, br in reqs:
        generation.generation_all(m, list(ev), dev, v, None, ac, tr, br)
    dt = time.perf_counter() - t0
    ns = max(1, T["n_step"])
    print("batch-1: %d requests, %d tokens, %.3f s -> %.1f tokens/s, %.3f ms/token"
          % (n, T["n_step"], dt, T["n_step"] / dt, 1000 * dt / ns))
    print("  session init %.3f ms/call (first step captures the graph)" % (1000 * T["init"] / max(1, T["n_init"])))
    print("  prefill      %.3f ms/call" % (1000 * T["prefill"] / max(1, T["n_init"])))
    print("  step         %.3f ms/token (H2D + replay + D2H + sync)" % (1000 * T["step"] / ns))
    print("  advance      %.3f ms/token (host grammar + sampling)" % (1000 * T["advance"] / ns))
    other = dt - T["init"] - T["prefill"] - T["step"] - T["advance"]
    print("  other        %.3f ms/token (prepare, restore, ...)" % (1000 * other / ns))
    # the step's kernels alone
    m.set_precision("fp32")
    sess = decode.DecodeSession(m, 1, 1200, 400)
    sess.prefill([0], [np.arange(1000) % 300 + 5])
    sess.step([(0, [3], 0)])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(200):
        sess.graph.replay()
    torch.cuda.synchronize()
    print("  replay alone %.3f ms (fp32 step graph, 200 back to back)" % ((time.perf_counter() - t) / 200 * 1000))
    t = time.perf_counter()
    for i in range(200):
        sess.step([(0, [3], 1 + i)])
    print("  step call    %.3f ms (with H2D / D2H / sync, no host grammar)" % ((time.perf_counter() - t) / 200 * 1000))
    lg = np.random.randn(309).astype(np.float32)
    t = time.perf_counter()
    for _ in range(2000):
        generation.sampling(lg, v)
    print("  sampling()   %.3f ms (weighted, no flags)" % ((time.perf_counter() - t) / 2000 * 1000))


if __name__ == "__main__":
    main()
