"""Calibration: torch.matmul (hipBLASLt) vs smer_gemm at the C2 forward /
dgrad / wgrad shapes (plain GEMM, no epilogue), bf16.  Not a product path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
bf = torch.bfloat16


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


shapes = [("fwd QKV", 32768, 1536, 512), ("fwd FFN1", 32768, 2048, 512), ("fwd FFN2", 32768, 512, 2048),
          ("dgrad QKV", 32768, 512, 1536), ("dgrad FFN1", 32768, 512, 2048), ("dgrad FFN2", 32768, 2048, 512),
          ("dec fwd QKV", 8192, 1536, 512), ("dec fwd FFN1", 8192, 2048, 512)]
print("%-14s %6s %6s %6s %10s %10s %8s %8s" % ("shape", "M", "N", "K", "blas_us", "smer_us", "blasTF", "smerTF"))
for name, M, N, K in shapes:
    a = torch.randn(M, K, device=dev).to(bf)
    if name.startswith("dgrad"):
        w = torch.randn(K, N, device=dev).to(bf)   # dX = dY . W  (W [out=K, in=N])
        tb = timeit(lambda: torch.matmul(a, w))
        ts = timeit(lambda: ops.linear_dgrad(a, w))
    else:
        w = torch.randn(N, K, device=dev).to(bf)
        tb = timeit(lambda: torch.matmul(a, w.t()))
        ts = timeit(lambda: ops.linear(a, w))
    fl = 2.0 * M * N * K
    print("%-14s %6d %6d %6d %10.1f %10.1f %8.0f %8.0f" % (name, M, N, K, tb, ts, fl / tb / 1e6, fl / ts / 1e6),
          flush=True)
for name, M, N, K in (("wgrad QKV", 1536, 512, 32768), ("wgrad FFN1", 2048, 512, 32768),
                      ("wgrad FFN2", 512, 2048, 32768)):
    dy = torch.randn(K, M, device=dev).to(bf)
    x = torch.randn(K, N, device=dev).to(bf)
    dw = torch.zeros(M, N, device=dev)
    tb = timeit(lambda: torch.matmul(dy.t(), x))
    ts = timeit(lambda: ops.linear_wgrad(dy, x, dw, accumulate=False))
    fl = 2.0 * M * N * K
    print("%-14s %6d %6d %6d %10.1f %10.1f %8.0f %8.0f" % (name, M, N, K, tb, ts, fl / tb / 1e6, fl / ts / 1e6),
          flush=True)
