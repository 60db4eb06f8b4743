"""The product infill path (generation_batch, device grammar, graph replay)
for rocprofv3: C2 workload (32 requests x ~1000-token sources), run twice."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from smer_music_generation_amd.generation import generation_batch  # noqa: E402
from smer_music_generation_amd.vocab import WordVocab  # noqa: E402

args = bench.parse_args([])
dev = torch.device("cuda", 0)
v = WordVocab(0, bench.CTRL)
m = bench.make_model(args, dev).eval()
ac = v.density_indices + v.occupation_indices + v.polyphony_indices + v.tensile_indices
reqs = bench._infill_requests(32, args.seq, 0)
for _ in range(2):
    _, st = generation_batch(m, reqs, v, ac, greedy=True, return_stats=True)
torch.cuda.synchronize()
print("steps", st["steps"], "tokens", st["tokens"])
