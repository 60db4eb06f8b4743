"""Write the committed profile summaries under profiles/ from a
tools/profile_round.sh run (gpurun_out/prof_<tag>/).

    python tools/refresh_profiles.py r01 [train_steps_traced]
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

from pmc_traffic import summary  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
steps = sys.argv[2] if len(sys.argv) > 2 else "12"
src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
dst = os.path.join(ROOT, "profiles")


def run(*args):
    return subprocess.run([sys.executable] + list(args), capture_output=True, text=True,
                          check=True).stdout


train = run(os.path.join(ROOT, "tools", "prof_summary.py"),
            os.path.join(src, "trace", "run_kernel_stats.csv"), steps, "30")
with open(os.path.join(dst, tag + "_train_kernel_stats.txt"), "w") as f:
    f.write("# rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 2 "
            "--no-infill --no-cpu --no-c4  with SMER_WGRAD_OVERLAP=0, i.e. weight gradients on the "
            "main stream so each kernel's duration is its own (%s steps traced: 2 warm-up + 5 timed + 5 "
            "event-timed; per-step = total/%s)\n" % (steps, steps) + train)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
            os.path.join(dst, tag + "_train_kernel_stats.csv"))

ovl = os.path.join(src, "trace_ovl", "run_kernel_stats.csv")
if os.path.exists(ovl):
    t = run(os.path.join(ROOT, "tools", "prof_summary.py"), ovl, "7", "30")
    with open(os.path.join(dst, tag + "_train_overlap_kernel_stats.txt"), "w") as f:
        f.write("# rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 2 "
                "--no-infill --no-cpu --no-c4 --no-roofline  (product path: weight gradients on "
                "a second stream, concurrent with the main chain, so kernel durations overlap; "
                "7 steps traced; per-step = total/7)\n" + t)

dec = run(os.path.join(ROOT, "tools", "prof_summary.py"),
          os.path.join(src, "dec", "run_kernel_stats.csv"), "51", "20")
with open(os.path.join(dst, tag + "_decode_kernel_stats.txt"), "w") as f:
    f.write("# rocprofv3 --kernel-trace --stats -- python3 tools/prof_decode.py --n 50 --graph "
            "(R=32, S=1000; prefill + 51 graph-replayed decode steps; per-step = total/51)\n" + dec)
shutil.copy(os.path.join(src, "dec", "run_kernel_stats.csv"),
            os.path.join(dst, tag + "_decode_kernel_stats.csv"))

fetch = os.path.join(src, "fetch", "run_counter_collection.csv")
write = os.path.join(src, "write", "run_counter_collection.csv")
with open(os.path.join(dst, tag + "_train_pmc_traffic.json"), "w") as f:
    json.dump({k[5:] if k.startswith("void ") else k: v for k, v in summary(fetch, write).items()},
              f, indent=1)
txt = run(os.path.join(ROOT, "tools", "pmc_traffic.py"), fetch, write)
with open(os.path.join(dst, tag + "_train_pmc_traffic.txt"), "w") as f:
    f.write("# rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py --steps 2 "
            "--warmup 1 --no-infill --no-cpu --no-roofline --no-c4; FETCH doubled per gfx950 "
            "correction (MI355X_MICROARCH.md HBM)\n" + txt)
print(train.splitlines()[-2:], dec.splitlines()[-2:])
