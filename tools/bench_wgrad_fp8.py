"""fp8 weight gradient vs the bf16 one at the C2 / C4 step's shapes, isolated:
per-call time of ops.linear_wgrad_fp8 (fused bias gradient; without it
beside) and of ops.linear_wgrad (bf16, fused bias).   python tools/bench_wgrad_fp8.py [c2|c4]"""
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
    "c2": ((512, 512, 32768), (1536, 512, 32768), (2048, 512, 32768), (512, 2048, 32768)),
    "c4": ((768, 768, 16384), (2304, 768, 16384), (3072, 768, 16384), (768, 3072, 16384),
           (768, 768, 65536), (1536, 768, 65536), (2304, 768, 65536), (3072, 768, 65536),
           (768, 3072, 65536)),
}
for (Mo, Nin, T) in SHAPES[sys.argv[1] if len(sys.argv) > 1 else "c4"]:
    dy = torch.randn(T, Mo, device="cuda").to(bf)
    x = torch.randn(T, Nin, device="cuda").to(bf)
    dy8 = (dy.float() * 64).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    x8 = (x.float() * 64).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    inv = torch.full((1,), 1 / 64, device="cuda")
    dw = torch.zeros(Mo, Nin, device="cuda")
    db = torch.zeros(Mo, device="cuda")
    t16 = timeit(lambda: ops.linear_wgrad(dy, x, dw, db=db))
    t8n = timeit(lambda: ops.linear_wgrad_fp8(dy8, inv, x8, inv, dw))
    t8 = timeit(lambda: ops.linear_wgrad_fp8(dy8, inv, x8, inv, dw, db=db))
    ref = (dy.float().t() @ x.float())
    dw.zero_()
    ops.linear_wgrad_fp8(dy8, inv, x8, inv, dw, accumulate=False)
    err = ((dw - ref).norm() / ref.norm()).item()
    f = 2 * Mo * Nin * T
    print("wgrad M%-5d N%-5d K%-6d bf16 %8.1f us %6.1f TF | fp8 %8.1f us %6.1f TF (%.2fx) | no bias %8.1f us"
          " | fp8 rel err %.4f" % (Mo, Nin, T, t16, f / t16 / 1e6, t8, f / t8 / 1e6, t16 / t8, t8n, err),
          flush=True)
