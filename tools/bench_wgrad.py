"""wgrad (+bias) shapes of the C2 / C4 step, isolated: per-launch time.
    python tools/bench_wgrad.py [c2|c4]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


bf = torch.bfloat16
SHAPES = {
    "c2": ((512, 512, 8192), (2048, 512, 8192), (512, 2048, 8192), (1536, 512, 8192),
           (512, 512, 32768), (1024, 512, 32768), (2048, 512, 32768), (512, 2048, 32768),
           (1536, 512, 32768)),
    "c4": ((768, 768, 16384), (2304, 768, 16384), (3072, 768, 16384), (768, 3072, 16384),
           (768, 768, 65536), (1536, 768, 65536), (2304, 768, 65536), (3072, 768, 65536),
           (768, 3072, 65536)),
}
for (Mo, Nin, T) in SHAPES[sys.argv[1] if len(sys.argv) > 1 else "c2"]:
    dy = torch.randn(T, Mo, device="cuda").to(bf)
    x = torch.randn(T, Nin, device="cuda").to(bf)
    dw = torch.zeros(Mo, Nin, device="cuda")
    db = torch.zeros(Mo, device="cuda")
    t = timeit(lambda: ops.linear_wgrad(dy, x, dw, db=db))
    tb = timeit(lambda: torch.matmul(dy.t(), x))  # hipBLASLt reference point (no bias grad)
    print("wgrad M%-5d N%-5d K%-6d %8.1f us %7.1f TF   [torch/hipBLASLt %8.1f us %7.1f TF]"
          % (Mo, Nin, T, t, 2 * Mo * Nin * T / t / 1e6, tb, 2 * Mo * Nin * T / tb / 1e6), flush=True)
