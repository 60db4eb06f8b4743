"""A few C4 train steps in a given precision (for rocprofv3 kernel traces).
    python tools/c4_step.py fp8|bf16 [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

args = bench.parse_args([])
args.layers, args.d_model, args.nhead, args.seq, args.tgt = 12, 768, 12, 2048, 512
args.steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
args.warmup, args.roofline = 1, False
import torch  # noqa: E402
r = bench.bench_train(args, torch.device("cuda", 0), 0, 1, sys.argv[1])
print(sys.argv[1], "%.2f ms/step" % r["ms_per_step"])
