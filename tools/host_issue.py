"""Host issue time of the C2 bench train step vs its GPU time: if the host
needs longer to enqueue a step than the GPU needs to run it, the step is
launch-bound (graph capture / fewer launches would pay); if not, the queue
stays full and only on-GPU dependencies leave gaps.
    python tools/host_issue.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from smer_music_generation_amd.synth import synth_training_batch  # noqa: E402
from smer_music_generation_amd.train import Trainer  # noqa: E402
from smer_music_generation_amd.vocab import WordVocab  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
args = bench.parse_args([])
v = WordVocab(0, bench.CTRL)
m = bench.make_model(args, dev)
tr = Trainer(m, v, lr=1e-4)
b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
for _ in range(3):
    tr.step(bt)
torch.cuda.synchronize()
host = []
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
e0.record()
t0 = time.perf_counter()
for _ in range(n):
    a = time.perf_counter()
    tr.step(bt)
    host.append(time.perf_counter() - a)
t_issue = time.perf_counter() - t0
e1.record()
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
gpu_ms = e0.elapsed_time(e1) / n
print("host issue per step: mean %.3f ms (min %.3f, max %.3f); all %d steps issued after %.1f ms; "
      "GPU %.3f ms per step; wall %.3f ms per step"
      % (1e3 * np.mean(host), 1e3 * min(host), 1e3 * max(host), n, 1e3 * t_issue, gpu_ms, 1e3 * t_all / n))
