"""Infill decode profile: phase split of generation_batch and the device
time of one replayed decode step (HIP events around graph.replay)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    from smer_music_generation_amd import _lib
    from smer_music_generation_amd.generation import generation_batch
    from smer_music_generation_amd.vocab import WordVocab
    from smer_music_generation_amd.decode import DecodeSession
    _lib.load()
    args = bench.parse_args([])
    dev = torch.device("cuda", 0)
    v = WordVocab(0, bench.CTRL)
    m = bench.make_model(args, dev).eval()
    ac = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
    for R in (32, 64, 128):
        reqs = bench._infill_requests(R, args.seq, 0)
        generation_batch(m, reqs[:4], v, ac, greedy=True)
        t0 = time.perf_counter()
        _, st = generation_batch(m, reqs, v, ac, greedy=True, return_stats=True)
        dt = time.perf_counter() - t0
        print("R=%d tok/s=%.0f steps=%d %s total=%.3f" % (R, st["tokens"] / dt, st["steps"],
              {k: round(st[k], 4) for k in ("prepare_s", "prefill_s", "decode_s", "step_call_s")}, dt))
        with torch.no_grad():
            s = DecodeSession(m, R, 1024, 600)
            s.prefill(list(range(R)), [[4] * 1000 for _ in range(R)])
            feeds = [(i, [5], 0) for i in range(R)]
            s.step(feeds)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(50):
                s.graph.replay()
            e1.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for k in range(50):
                s.step([(i, [5], k + 1) for i in range(R)])
            t2 = time.perf_counter()
            print("  replay device ms/step=%.3f  full step() ms=%.3f" % (e0.elapsed_time(e1) / 50,
                  (t2 - t1) * 1000 / 50))


if __name__ == "__main__":
    main()
