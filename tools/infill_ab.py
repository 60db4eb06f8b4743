"""A/B of one environment switch on the decode bench lines (C2 batched
greedy infill, C5, batch-1 plugin call; bf16 unless --fp32): each value in
its own process (switches are read once per process), rounds interleaved.
    python tools/infill_ab.py ENV_NAME VALUE_A VALUE_B ... [--rounds=2] [--fp32]"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(prec):
    import torch
    import bench
    args = bench.parse_args([])
    dev = torch.device("cuda:0")
    c2 = bench.bench_infill(args, dev, 0, precision=prec)
    c5 = bench.bench_infill_c5(args, dev, 0, precision=prec)
    r = {"c2": round(c2["tokens_per_s"]), "c2_ms": round(c2["ms_per_decode_step"], 4),
         "c5": round(c5["tokens_per_s"]), "c5_ms": round(c5.get("ms_per_decode_step", 0), 4),
         "b1": bench.bench_infill_batch1(args, dev, 0)["value"]}
    print(json.dumps(r))


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "one":
    one(sys.argv[2])
elif __name__ == "__main__":
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    rounds = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--rounds=")), "2"))
    prec = "fp32" if "--fp32" in sys.argv else "bf16"
    name, values = argv[0], argv[1:]
    res = {v: [] for v in values}
    for _ in range(rounds):
        for v in values:
            env = dict(os.environ, **{name: v})
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "one", prec], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-3000:])
                sys.exit(out.returncode)
            res[v].append(json.loads(out.stdout.strip().splitlines()[-1]))
            print(name, v, res[v][-1], flush=True)
    print(json.dumps(res))
