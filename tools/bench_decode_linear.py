"""Decode Linear shapes (M = 2 rows per request): per-launch device time of
smer_linear_decode from graph-captured back-to-back launches (GPU).
(A split-K variant with a last-slice reduction through agent-scope atomics
measured 2.5-3.5 us slower at K = 512 and 0.3 us faster at K = 2048 and was
dropped; see DESIGN.md.)"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402


def timeit(fn, iters=50, reps=10):
    """Per-launch device time: `iters` launches captured in one HIP graph."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (iters * reps) * 1e3


bf = torch.bfloat16
shapes = [(64, n, k) for n, k in ((1536, 512), (512, 512), (2048, 512), (512, 2048), (309, 512))]
shapes += [(128, n, k) for n, k in ((1536, 512), (512, 512), (2048, 512), (512, 2048), (309, 512))]
if len(sys.argv) > 1 and sys.argv[1] == "sweep":
    shapes = [(64, n, k) for n in (64, 512, 2048) for k in (512, 1024, 2048, 4096)]
for M, N, K in shapes:
    if True:
        x = torch.randn(M, K, device="cuda").to(bf)
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(bf)
        b = torch.randn(N, device="cuda")
        res = torch.randn(M, N, device="cuda").to(bf)
        t0 = timeit(lambda: ops.linear_decode(x, w, b))
        t1 = timeit(lambda: ops.linear_decode(x, w, b, residual=res))
        print("M %3d N %4d K %4d  %6.2f us  (+residual %6.2f us)" % (M, N, K, t0, t1))
