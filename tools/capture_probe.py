"""Where the first (cold) generation_batch call's capture time goes: the
greedy decode graph (decoder step + grammar kernel) captured for three fresh
sessions in one process, with the phases of DecodeSession._capture_greedy
timed separately (eager warm step, stream capture, instantiate = first
replay), C2 model, R = 32 requests -- with the caching allocator first
filled the way a training step leaves it (torch.cuda.graph's __enter__
empties it; decode._capture does not)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    from smer_music_generation_amd import _lib
    from smer_music_generation_amd import generation as G
    from smer_music_generation_amd.vocab import WordVocab
    _lib.load()
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    m = bench.make_model(args, dev).eval()
    v = WordVocab(0, bench.CTRL)
    ac = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    junk = [torch.empty(256 << 20, dtype=torch.uint8, device=dev) for _ in range(120)]
    del junk  # ~30 GB of cached segments, as after the C2 train bench
    for rnd in range(3):
        reqs = bench._infill_requests(32, 1024 + 64 * rnd, 300 * rnd)
        G.clear_decode_sessions()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _, st = G.generation_batch(m, reqs, v, ac, greedy=True, return_stats=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        print("round %d: call %.1f ms, prefill %.1f ms, phases %s" % (
            rnd, 1e3 * (t1 - t0), 1e3 * st["prefill_s"],
            {k: round(1e3 * x, 2) for k, x in st["decode_phases_s"].items()}), flush=True)
    # the same capture twice with torch's graph API alone: a one-kernel graph
    x = torch.zeros(1024, device=dev)
    from smer_music_generation_amd.decode import _capture
    for rnd in range(2):
        junk = [torch.empty(256 << 20, dtype=torch.uint8, device=dev) for _ in range(120)]
        del junk
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = _capture(s, lambda: x.add_(1.0))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        with torch.cuda.stream(s):
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, stream=s):
                x.add_(1.0)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("full cache %d: decode._capture %.2f ms, torch.cuda.graph %.2f ms"
              % (rnd, 1e3 * (t1 - t0), 1e3 * (t2 - t1)), flush=True)
    for rnd in range(3):
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                x.add_(1.0)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("trivial graph %d: capture+instantiate %.2f ms, first replay %.2f ms"
              % (rnd, 1e3 * (t1 - t0), 1e3 * (t2 - t1)), flush=True)
    np.random.seed(0)


if __name__ == "__main__":
    main()
