"""Run-to-run repeatability of the C4 30-step loss trajectories
(tests/test_prod_gpu.py::_c4_trajectory): each precision twice in one
process; prints the losses' largest difference between the two runs and
each run's relative deviation from the first fp32 run.
    python tools/c4_traj_repeat.py [steps] [precisions ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_prod_gpu import _c4_trajectory  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
gd = os.path.join(ROOT, "tests", "golden")
precs = sys.argv[2:] or ["fp32", "bf16", "fp8"]
runs = {p: [_c4_trajectory(gd, p, n) for _ in range(2)] for p in ["fp32"] + [p for p in precs if p != "fp32"]}
ref = runs["fp32"][0]
for p, (a, b) in runs.items():
    ra, rb = np.abs(a - ref) / ref, np.abs(b - ref) / ref
    print("%s: run-to-run max |dloss| %.3e; rel dev from fp32 max %.4f / %.4f, final %.5f / %.5f"
          % (p, np.abs(a - b).max(), ra.max(), rb.max(), ra[-1], rb[-1]), flush=True)
