"""Writes the bf16 LayerNorm forward outputs (y, mean, rstd) at C2 / C4
row widths to an .npz, for comparing SMER_LN_RPW settings bit for bit
(run once per setting in separate processes)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
g0 = torch.Generator(device="cpu").manual_seed(7)
for M, N in ((32771, 512), (8192, 512), (16400, 768)):
    x = (torch.randn(M, N, generator=g0) * 3 + 1).to(torch.bfloat16).to(dev)
    g = torch.randn(N, generator=g0).to(dev)
    b = torch.randn(N, generator=g0).to(dev)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    ops.layernorm(x, g, b, y, mean, rstd)
    torch.cuda.synchronize()
    out["y%d_%d" % (M, N)] = y.view(torch.int16).cpu().numpy()
    out["m%d_%d" % (M, N)] = mean.cpu().numpy()
    out["r%d_%d" % (M, N)] = rstd.cpu().numpy()
np.savez(sys.argv[1], **out)
