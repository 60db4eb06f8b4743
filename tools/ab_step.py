"""A/B of one environment switch on the train step: each value in its own
process (the switches are read once per process), rounds interleaved.
    python tools/ab_step.py c2|c4|c4bf16 ENV_NAME VALUE_A VALUE_B ... [--rounds 2]
    python tools/ab_step.py c2 ENV "A=1,B=2" "A=0" ...   (several switches per value)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = [a for a in sys.argv[1:] if not a.startswith("--rounds")]
rounds = 2
for a in sys.argv[1:]:
    if a.startswith("--rounds"):
        rounds = int(a.split("=")[1])
cfg, name, values = args[0], args[1], args[2:]
res = {v: [] for v in values}
for r in range(rounds):
    for v in values:
        env = dict(os.environ)
        if name == "ENV":
            for kv in v.split(","):
                if kv:
                    k, x = kv.split("=", 1)
                    env[k] = x
        else:
            env[name] = v
        if cfg == "c2":
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "3",
                   "--no-infill", "--no-cpu", "--no-c4", "--no-c5", "--no-roofline"]
        else:
            cmd = [sys.executable, os.path.join(ROOT, "tools", "c4_step.py"),
                   "bf16" if cfg == "c4bf16" else "fp8", "4"]
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
        if out.returncode != 0:
            print(out.stdout[-2000:], out.stderr[-2000:])
            sys.exit(out.returncode)
        ms = None
        for line in out.stdout.splitlines():
            if line.startswith("{"):
                ms = json.loads(line)["ms_per_step"]
            elif "ms/step" in line:
                ms = float(line.split()[1])
        res[v].append(ms)
        print("%s %s=%s round %d: %.3f ms/step" % (cfg, name, v, r, ms), flush=True)
for v in values:
    print("%s=%s: %s" % (name, v, " ".join("%.3f" % x for x in res[v])))
