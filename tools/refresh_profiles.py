"""Write the committed profile summaries under profiles/ from a
tools/profile_round.sh run (gpurun_out/prof_<tag>/).

    python tools/refresh_profiles.py r02 [train_steps_traced]
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
# decode HBM bytes per kernel (separate FETCH / WRITE passes over 20 graph replays)
dfetch = os.path.join(src, "dec_fetch", "run_counter_collection.csv")
dwrite = os.path.join(src, "dec_write", "run_counter_collection.csv")
if os.path.exists(dfetch) and os.path.exists(dwrite):
    with open(os.path.join(dst, tag + "_decode_pmc_traffic.json"), "w") as f:
        json.dump({k[5:] if k.startswith("void ") else k: v for k, v in summary(dfetch, dwrite).items()},
                  f, indent=1)
    txt = run(os.path.join(ROOT, "tools", "pmc_traffic.py"), dfetch, dwrite)
    with open(os.path.join(dst, tag + "_decode_pmc_traffic.txt"), "w") as f:
        f.write("# rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/prof_decode.py "
                "--n 20 --graph (R=32, S=1000, incl. prefill); FETCH doubled per gfx950 correction\n" + txt)

# C4 train step, fp8 and bf16 (product path, 5 steps traced: 1 warm-up + 4)
for p in ("fp8", "bf16"):
    c = os.path.join(src, "c4_" + p, "run_kernel_stats.csv")
    if os.path.exists(c):
        t = run(os.path.join(ROOT, "tools", "prof_summary.py"), c, "5", "30")
        with open(os.path.join(dst, "%s_c4_%s_kernel_stats.txt" % (tag, p)), "w") as f:
            f.write("# rocprofv3 --kernel-trace --stats -- python3 tools/c4_step.py %s 4 (C4: 12+12 "
                    "layers d768 h12 S2048 T512 B32; weight gradients on the side stream; 5 steps "
                    "traced; per-step = total/5)\n" % p + t)

c = os.path.join(src, "c4ser", "run_kernel_stats.csv")
if os.path.exists(c):
    t = run(os.path.join(ROOT, "tools", "prof_summary.py"), c, "5", "30")
    with open(os.path.join(dst, "%s_c4_fp8_serial_kernel_stats.txt" % tag), "w") as f:
        f.write("# SMER_WGRAD_OVERLAP=0 rocprofv3 --kernel-trace --stats -- python3 tools/c4_step.py fp8 4 "
                "(C4 fp8, weight gradients serialised on the main stream: each kernel's own duration; "
                "5 steps traced; per-step = total/5)\n" + t)

# per-stream busy time of the overlapped traces (tools/stream_split.py)
for name, sub in (("train_stream_split", "trace_ovl"), ("c4_fp8_stream_split", "c4_fp8")):
    tr = os.path.join(src, sub, "run_kernel_trace.csv")
    if os.path.exists(tr):
        t = run(os.path.join(ROOT, "tools", "stream_split.py"), tr, "3")
        with open(os.path.join(dst, "%s_%s.txt" % (tag, name)), "w") as f:
            f.write("# tools/stream_split.py over the last 3 traced steps of %s (stream 0 = the dgrad "
                    "chain, stream 1 = weight gradients)\n" % sub + t)

# SQ counters (train step, weight gradients serialised) and the fp8 GEMM pair
for name, sub in (("train_pmc_sq", os.path.join("..", "pmc_" + tag, "sq.txt")),
                  ("fp8_gemm_pmc_sq", os.path.join("..", "pmc_fp8", "sq.txt"))):
    fsq = os.path.normpath(os.path.join(src, sub))
    if os.path.exists(fsq):
        shutil.copy(fsq, os.path.join(dst, "%s_%s.txt" % (tag, name)))
        js = fsq[:-4] + ".json"
        if os.path.exists(js):
            shutil.copy(js, os.path.join(dst, "%s_%s.json" % (tag, name)))
print(train.splitlines()[-2:], dec.splitlines()[-2:])
