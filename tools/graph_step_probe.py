"""Probe: how much of the C2 train step is launch overhead?  Times the eager
step, the host time to enqueue one step, and the same step captured in a
HIP graph (fixed seed / Adam step: a measurement only, not the product)."""
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

args = bench.parse_args([])
dev = torch.device("cuda", 0)
v = WordVocab(0, bench.CTRL)
m = bench.make_model(args, dev)
tr = Trainer(m, v, lr=1e-4)
b = synth_training_batch(1000, v, args.batch, args.seq, args.tgt)
bt = {k: torch.from_numpy(np.asarray(x)).to(dev) for k, x in b.items()}
for _ in range(3):
    tr.step(bt)
torch.cuda.synchronize()
K = 10
t0 = time.perf_counter()
for _ in range(K):
    tr.step(bt)
torch.cuda.synchronize()
print("eager ms/step %.3f" % (1000 * (time.perf_counter() - t0) / K))
enq = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.step(bt)
    enq.append(time.perf_counter() - t0)
torch.cuda.synchronize()
print("host enqueue ms/step", ["%.2f" % (1000 * e) for e in enq])
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    tr.step(bt)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    tr.step(bt)
torch.cuda.synchronize()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    g.replay()
torch.cuda.synchronize()
print("graph ms/step %.3f" % (1000 * (time.perf_counter() - t0) / K))
