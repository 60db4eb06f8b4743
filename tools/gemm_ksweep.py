"""K sweep of the 256x256 forward GEMMs (bf16 vs fp8) at one M x N: a linear
fit of time against K splits per-tile fixed cost (prologue + epilogue) from
per-K-stage cost.   python tools/gemm_ksweep.py [M N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2304
bf = torch.bfloat16
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


print("%6s %10s %10s %10s %10s %10s" % ("K", "bf16", "bf16_nb", "fp8", "fp8_nb", "fp8_q"))
for K in (256, 512, 768, 1536, 3072):
    x = torch.randn(M, K, device=dev).to(bf)
    w = torch.randn(N, K, device=dev).to(bf)
    b = torch.randn(N, device=dev)
    out = torch.empty(M, N, device=dev, dtype=bf)
    x8 = torch.empty(M, K, device=dev, dtype=torch.uint8)
    w8 = torch.empty(N, K, device=dev, dtype=torch.uint8)
    xi, wi = torch.empty(1, device=dev), torch.empty(1, device=dev)
    ops.fp8_quantize(x, x8, xi)
    ops.fp8_quantize(w, w8, wi)
    q8 = torch.empty(M, N, device=dev, dtype=torch.uint8)
    qs = torch.ones(1, device=dev)
    am = torch.zeros(1, device=dev, dtype=torch.int32)
    t = [timeit(lambda: ops.linear(x, w, b, out=out)),
         timeit(lambda: ops.linear(x, w, None, out=out)),
         timeit(lambda: ops.gemm_fp8(x8, xi, w8, wi, out, bias=b)),
         timeit(lambda: ops.gemm_fp8(x8, xi, w8, wi, out)),
         timeit(lambda: ops.gemm_fp8_q(x8, xi, w8, wi, out, bias=b, relu=True, q8=q8, qs=qs, amax=am))]
    print("%6d " % K + " ".join("%10.1f" % v for v in t), flush=True)
