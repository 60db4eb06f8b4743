"""fp8 vs bf16 dgrad GEMMs at the C4 shapes, isolated (HIP events):
e4m3(dY) . e4m3(W^T)^T with the dgrad epilogues against ops.linear_dgrad."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = "cuda"


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
one = torch.ones(1, device=dev)
for name, M, Nin, Kout, epi in (("FFN2 dgrad", 65536, 2048, 768, "gq"), ("FFN1 dgrad", 65536, 768, 2048, "R"),
                                ("out dgrad", 65536, 768, 768, ""), ("dec out dgrad", 16384, 768, 768, ""),
                                ("dec FFN1 dgrad", 16384, 768, 2048, "R"), ("dec FFN2 dgrad", 16384, 2048, 768, "gq")):
    dy = torch.randn(M, Kout, device=dev).to(bf)
    w = torch.randn(Kout, Nin, device=dev).to(bf)
    dy8 = (dy.float().clamp(-448, 448)).to(torch.float8_e4m3fn).view(torch.uint8)
    wt8 = (w.t().contiguous().float().clamp(-448, 448)).to(torch.float8_e4m3fn).view(torch.uint8)
    kw, kw8 = {}, {}
    if "g" in epi:
        g = torch.randn(M, Nin, device=dev).to(bf)
        kw = dict(gate=g, gate_scale=1.1)
        kw8 = dict(kw)
    if "R" in epi:
        r = torch.randn(M, Nin, device=dev).to(bf)
        kw = dict(residual=r)
        kw8 = dict(kw)
    if "q" in epi:
        kw8.update(q8=torch.empty(M, Nin, dtype=torch.uint8, device=dev), qs=one,
                   amax=torch.zeros(1, dtype=torch.int32, device=dev))
    out = torch.empty(M, Nin, device=dev, dtype=bf)
    tb = timeit(lambda: ops.linear_dgrad(dy, w, out=out, **kw))
    t8 = timeit(lambda: ops.gemm_fp8_ex(dy8, one, wt8, one, out, **kw8))
    fl = 2.0 * M * Nin * Kout
    print("%-15s M%-6d N%-5d K%-5d %-3s bf16 %7.1f us %6.0f TF | fp8 %7.1f us %6.0f TF"
          % (name, M, Nin, Kout, epi, tb, fl / tb / 1e6, t8, fl / t8 / 1e6), flush=True)
