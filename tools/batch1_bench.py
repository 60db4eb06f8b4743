"""bench.py's batch-1 plugin line alone (infill.batch1): the default
weighted-sampling generation_all on C2-model requests, device grammar on
and off.

    python tools/batch1_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from smer_music_generation_amd import generation  # noqa: E402


def main():
    args = bench.parse_args([])
    dev = torch.device("cuda:0")
    res = {"device_grammar": bench.bench_infill_batch1(args, dev, 0)}
    orig = generation.generation_all

    def host(*a, **k):
        k["device_grammar"] = False
        return orig(*a, **k)
    generation.generation_all = host
    res["host_loop"] = bench.bench_infill_batch1(args, dev, 0)
    generation.generation_all = orig
    print(json.dumps(res))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def kernel_time():
    """The sampled grammar kernel alone (one request, C2 vocabulary), µs per
    call, and the phases of one device-grammar plugin call."""
    import numpy as np
    from smer_music_generation_amd import ops as O
    from smer_music_generation_amd.generation import grammar_tables, reject_table
    from smer_music_generation_amd.vocab import WordVocab
    dev = torch.device("cuda:0")
    v = WordVocab(0, bench.CTRL)
    V = v.vocab_size
    keep, cls = grammar_tables(v, v.density_indices)
    kt, rt, ct = (torch.from_numpy(x).to(dev) for x in (keep, reject_table(v), cls))
    np.random.seed(0)
    st0 = np.random.get_state()
    mt = torch.zeros(656, dtype=torch.int32, device=dev)
    mt[:625] = torch.from_numpy(np.concatenate([st0[1], [st0[2]]]).astype(np.uint32).view(np.int32)).to(dev)
    state = torch.tensor([[0, 4, 5, 0, 1, 0, 0, 0, 0, 0, 0, 0]], dtype=torch.int32, device=dev)
    args = [torch.randn(2, V, device=dev), state, torch.zeros(1, 16, dtype=torch.int8, device=dev), kt, rt, ct,
            torch.ones(1, dtype=torch.int32, device=dev), torch.zeros(2, dtype=torch.int64, device=dev),
            torch.zeros(4, 2, dtype=torch.int32, device=dev), torch.zeros(1, 4, dtype=torch.int32, device=dev), mt,
            torch.zeros(3, dtype=torch.int32, device=dev)]
    kw = dict(eos=v.eos_index, m0=v.char2index('m_0'), trash_pos=200)
    for _ in range(5):
        O.grammar_sample_step(*args, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        state[0, 5] = 0
        O.grammar_sample_step(*args, **kw)
    e1.record()
    torch.cuda.synchronize()
    stamps = mt[640:650].cpu().numpy().view(np.uint32).astype(np.int64)
    print(json.dumps({"stamp_deltas_cycles": np.diff(stamps).tolist()}))
    return e0.elapsed_time(e1) * 10.0  # us per call (incl. the state reset)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "kernel":
    print(json.dumps({"grammar_sample_us": kernel_time()}))


def breakdown():
    """Where a device-grammar plugin call's time goes: sessions built,
    graph captures, prefill, the device loop, the rest (host)."""
    import time
    from smer_music_generation_amd import decode
    T = {}

    def wrap(cls, name):
        f = getattr(cls, name)

        def g(*a, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            T[name] = T.get(name, 0.0) + time.perf_counter() - t
            T[name + "_n"] = T.get(name + "_n", 0) + 1
            return r
        setattr(cls, name, g)
    for n in ("__init__", "prefill", "_capture_greedy", "sampled_decode"):
        wrap(decode.DecodeSession, n)
    args = bench.parse_args([])
    dev = torch.device("cuda:0")
    r = bench.bench_infill_batch1(args, dev, 0)
    T["total_s"] = r["seconds"] + r["cold_call_s"]
    T["tokens"] = r["tokens"] + (r["cold_call_tokens"] or 0)
    print(json.dumps({k: round(v, 5) if isinstance(v, float) else v for k, v in T.items()}))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "breakdown":
    breakdown()


def lookahead_sweep():
    """The batch-1 plugin line with the device loop's lookahead (graph
    replays in flight ahead of the host's poll) at 1, 2 and 3."""
    from smer_music_generation_amd import decode
    f = decode.DecodeSession.sampled_decode
    args = bench.parse_args([])
    dev = torch.device("cuda:0")
    res = {}
    for la in (3, 1, 3, 1, 3, 1, 2):
        def g(self, *a, _la=la, **k):
            k["lookahead"] = _la
            return f(self, *a, **k)
        decode.DecodeSession.sampled_decode = g
        r = bench.bench_infill_batch1(args, dev, 0)
        res.setdefault(str(la), []).append((r["value"], r["warm_call_s_mean"]))
    decode.DecodeSession.sampled_decode = f
    print(json.dumps(res))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "lookahead":
    lookahead_sweep()


def env_sweep(name, values, rounds=2):
    """The batch-1 plugin line with a per-process switch: each value in its
    own child process (switches are read once per process), interleaved."""
    import subprocess
    res = {v: [] for v in values}
    for _ in range(rounds):
        for v in values:
            env = dict(os.environ)
            env[name] = v
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "one"], env=env,
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-2000:])
                sys.exit(out.returncode)
            res[v].append(json.loads(out.stdout.strip().splitlines()[-1])["value"])
            print(name, v, res[v][-1], flush=True)
    print(json.dumps(res))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "one":
    print(json.dumps(bench.bench_infill_batch1(bench.parse_args([]), torch.device("cuda:0"), 0)))

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "env":
    env_sweep(sys.argv[2], sys.argv[3:])
