"""LayerNorm forward / backward timing at the C2 (rows x 512) and C4 (rows x 768) shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(f, iters=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


for M, N in ((32768, 512), (8192, 512), (65536, 768), (16384, 768)):
    x = torch.randn(M, N, device=dev).to(torch.bfloat16)
    g = torch.randn(N, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    dx = torch.empty_like(x)
    dxd = torch.empty_like(x)
    dg = torch.zeros(N, device=dev)
    db = torch.zeros(N, device=dev)
    tf = timeit(lambda: ops.layernorm(x, g, b, y, mean, rstd))
    tb = timeit(lambda: ops.layernorm_bwd(dy, x, mean, rstd, g, dx, dx_drop=dxd, drop_p=0.1, seed=3,
                                          dgamma=dg, dbeta=db))
    q8 = torch.empty(M, N, dtype=torch.uint8, device=dev)
    qs = torch.ones(1, device=dev)
    am = torch.zeros(1, dtype=torch.int32, device=dev)
    tq = timeit(lambda: ops.layernorm_bwd(dy, x, mean, rstd, g, dx, dx_drop=dxd, drop_p=0.1, seed=3,
                                          dgamma=dg, dbeta=db, q8=q8, qs=qs, amax=am))
    print("M=%d N=%d bwd with the e4m3 gradient copy %.1f us" % (M, N, tq), flush=True)
    fb = 2 * M * N * 2 / tf / 1e3
    bb = 4 * M * N * 2 / tb / 1e3
    print("M=%d N=%d fwd %.1f us (%.0f GB/s)  bwd %.1f us (%.0f GB/s)" % (M, N, tf, fb, tb, bb), flush=True)
