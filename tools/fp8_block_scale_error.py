"""e4m3 quantisation error of an activation x weight product with per-tensor
scaling (the C4 fp8 step's delayed scaling) vs MX-style E8M0 block scales
(one power-of-two scale per 32 K-elements, the v_mfma_scale operand), on
LayerNorm-like activations with and without outlier channels (CPU, torch
float8_e4m3fn casts).

    python tools/fp8_block_scale_error.py
"""
import torch
torch.manual_seed(0)
def q_tensor(x):
    s = 448.0 / x.abs().max()
    return (x * s).to(torch.float8_e4m3fn).float() / s
def q_block(x, blk=32):
    xs = x.view(x.shape[0], -1, blk)
    am = xs.abs().amax(-1, keepdim=True).clamp_min(1e-30)
    # E8M0 scale: power of two so that amax*scale <= 448
    e = torch.floor(torch.log2(448.0 / am))
    s = torch.exp2(e)
    return ((xs * s).to(torch.float8_e4m3fn).float() / s).view_as(x)
def rel(a, b): return ((a - b).norm() / b.norm()).item()
M, K, N = 4096, 768, 768
for name, gam in (("LN out, gamma~N(1,.3)", 1 + 0.3 * torch.randn(K)),
                  ("LN out + 4 outlier channels x20", torch.cat([torch.full((4,), 20.0), 1 + 0.3 * torch.randn(K - 4)]))):
    x = torch.randn(M, K) * gam
    w = torch.randn(N, K) / K ** 0.5
    y = x @ w.t()
    for qn, q in (("per-tensor", q_tensor), ("block-32 E8M0", q_block)):
        xq, wq = q(x), q(w)
        print("%-32s %-14s act %.4f  gemm out %.4f" % (name, qn, rel(xq, x), rel(xq @ wq.t(), y)))
