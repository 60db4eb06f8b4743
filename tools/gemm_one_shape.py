"""Run one GEMM shape N times (for rocprofv3 counter passes).
    python tools/gemm_one_shape.py fwd|fp8|dgrad|wgrad M N K [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

kind, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
bf = torch.bfloat16
if kind == "fwd":
    x = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(N, K, device="cuda").to(bf)
    b = torch.randn(N, device="cuda")
    f = lambda: ops.linear(x, w, b)  # noqa: E731
elif kind == "fp8":
    x = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(N, K, device="cuda").to(bf)
    b = torch.randn(N, device="cuda")
    x8 = torch.empty(M, K, device="cuda", dtype=torch.uint8)
    w8 = torch.empty(N, K, device="cuda", dtype=torch.uint8)
    xi, wi = torch.empty(1, device="cuda"), torch.empty(1, device="cuda")
    ops.fp8_quantize(x, x8, xi)
    ops.fp8_quantize(w, w8, wi)
    out = torch.empty(M, N, device="cuda", dtype=bf)
    f = lambda: ops.gemm_fp8(x8, xi, w8, wi, out, bias=b)  # noqa: E731
elif kind == "dgrad":
    dy = torch.randn(M, K, device="cuda").to(bf)
    w = torch.randn(K, N, device="cuda").to(bf)
    f = lambda: ops.linear_dgrad(dy, w)  # noqa: E731
else:
    dy = torch.randn(K, M, device="cuda").to(bf)
    x = torch.randn(K, N, device="cuda").to(bf)
    dw = torch.zeros(M, N, device="cuda")
    db = torch.zeros(M, device="cuda")
    f = lambda: ops.linear_wgrad(dy, x, dw, db=db, accumulate=False)  # noqa: E731
for _ in range(iters):
    f()
torch.cuda.synchronize()
