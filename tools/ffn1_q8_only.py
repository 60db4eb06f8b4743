"""FFN1 (C4 encoder: 65536 x 2048 x 768, bias + ReLU + dropout, e4m3 copy)
with and without its bf16 output, and the gated FFN2 dgrad (65536 x 2048 x
768) with a bf16 gate vs the e4m3 gate (smer_gemm_fp8_gate8); HIP events,
median of 20.  Also checks the two dgrads agree where the gates agree.
    python tools/ffn1_q8_only.py [M]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N, K = 2048, 768
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(3)
x8 = (torch.randn(M, K, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
w8 = (torch.randn(N, K, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
dy8 = (torch.randn(M, K, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
inv = torch.tensor([1.0 / 64], device=dev)
bias = torch.randn(N, generator=g).to(dev)
h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
hq = torch.empty(M, N, device=dev, dtype=torch.uint8)
qs = torch.tensor([0.5], device=dev)
am = torch.zeros(1, device=dev, dtype=torch.int32)


def med(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


f_c = lambda: ops.gemm_fp8_q(x8, inv, w8, inv, h, bias=bias, relu=True, drop_p=0.1, seed=7, q8=hq, qs=qs, amax=am)
f_n = lambda: ops.gemm_fp8_q(x8, inv, w8, inv, None, bias=bias, relu=True, drop_p=0.1, seed=7, q8=hq, qs=qs, amax=am)
t_c, t_n = med(f_c), med(f_n)
f_c()
hq_ref = hq.clone()
f_n()
torch.cuda.synchronize()
same = torch.equal(hq, hq_ref)
print("FFN1 %dx%dx%d fp8 + e4m3 copy: with bf16 out %.1f us, e4m3 only %.1f us (copy identical: %s)"
      % (M, N, K, t_c, t_n, same))
# gated FFN2 dgrad: dh = gate ? dy @ W2 * s : 0 ; A = dy8 [M, K], B = W2^T rows [N, K]
b8 = (torch.randn(N, K, generator=g) * 8).to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
dh1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
dh2 = torch.empty_like(dh1)
dq1 = torch.empty(M, N, device=dev, dtype=torch.uint8)
dq2 = torch.empty_like(dq1)
f_g = lambda: ops.gemm_fp8_ex(dy8, inv, b8, inv, dh1, gate=h, gate_scale=1.111, q8=dq1, qs=qs, amax=am)
f_8 = lambda: ops.gemm_fp8_gate8(dy8, inv, b8, inv, hq, 1.111, dh2, dq2, qs, am)
t_g, t_8 = med(f_g), med(f_8)
f_g()
f_8()
torch.cuda.synchronize()
open_bf = h.float() > 0
open_8 = (hq >= 1) & (hq <= 127)
agree = open_bf == open_8
eq = torch.equal(dh1[agree], dh2[agree]) and bool((dh2[~open_8] == 0).all())
print("gated dgrad %dx%dx%d: bf16 gate %.1f us, e4m3 gate %.1f us; gates differ at %d of %d; "
      "outputs equal where they agree: %s" % (M, N, K, t_g, t_8, int((~agree).sum()), agree.numel(), eq))
