"""fp8 vs bf16 forward GEMMs at the C4 shapes (and C2), plus the cost of
the per-tensor activation quantisation."""
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
for name, M, N, K in (("C4 qkv", 65536, 2304, 768), ("C4 ffn1", 65536, 2048, 768),
                      ("C4 ffn2", 65536, 768, 2048), ("C2 ffn1", 32768, 2048, 512),
                      ("C2 ffn2", 32768, 512, 2048), ("C2 qkv", 32768, 1536, 512)):
    x = torch.randn(M, K, device="cuda").to(bf)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
    b = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=bf)
    x8 = torch.empty(M, K, device="cuda", dtype=torch.uint8)
    w8 = torch.empty(N, K, device="cuda", dtype=torch.uint8)
    xi = torch.empty(1, device="cuda")
    wi = torch.empty(1, device="cuda")
    ws = torch.empty(16, device="cuda", dtype=torch.uint8)
    ops.fp8_quantize(w, w8, wi, ws)
    tb = timeit(lambda: ops.linear(x, w, b, out=C))
    tq = timeit(lambda: ops.fp8_quantize(x, x8, xi, ws))
    tf = timeit(lambda: ops.gemm_fp8(x8, xi, w8, wi, C, bias=b))
    fl = 2.0 * M * N * K
    print("%-8s M%6d N%5d K%5d  bf16 %7.1f us %6.0f TF | fp8 %7.1f us %6.0f TF | quant x %6.1f us"
          % (name, M, N, K, tb, fl / tb / 1e6, tf, fl / tf / 1e6, tq))
