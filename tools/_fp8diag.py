"""Diagnose: fp8_quantize after LayerNorm kernels (test-order dependence)."""
import sys
import torch
sys.path.insert(0, '/root/repo')
from smer_music_generation_amd import ops
dev = torch.device('cuda', 0)


def quant_check(tag):
    torch.manual_seed(0)
    M, K = 512, 768
    x = (torch.randn(M, K, device=dev) * 3).to(torch.bfloat16)
    x8 = torch.empty(M, K, device=dev, dtype=torch.uint8)
    xi = torch.empty(1, device=dev)
    ops.fp8_quantize(x, x8, xi)
    torch.cuda.synchronize()
    amax = x.float().abs().max()
    ref8 = (x.float() * (448 / amax)).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    bad = (ref8 != x8)
    rows = bad.any(1).nonzero().flatten().tolist()
    print(tag, 'agree', 1 - bad.float().mean().item(), 'bad rows', len(rows), rows[:8], flush=True)
    for i, j in bad.nonzero()[:4].tolist():
        v = x[i, j].float().item()
        print('   x', v, 'scaled', v * 448 / amax.item(), 'ref', ref8[i, j].item(), 'got', x8[i, j].item())


quant_check('fresh')
for dtype in (torch.bfloat16, torch.float32):
    for M, N in ((300, 512), (64, 768), (37, 64)):
        x = (torch.randn(M, N, device=dev) * 3 + 1).to(dtype)
        g = torch.randn(N, device=dev)
        b = torch.randn(N, device=dev)
        y = torch.empty_like(x)
        mean = torch.empty(M, device=dev)
        rstd = torch.empty(M, device=dev)
        ops.layernorm(x, g, b, y, mean, rstd)
        torch.cuda.synchronize()
        quant_check('after ln fwd %s %dx%d' % (dtype, M, N))
        dy = torch.randn(M, N, device=dev).to(dtype)
        dx = torch.empty_like(x)
        dxd = torch.empty_like(x)
        dg = torch.zeros(N, device=dev)
        db = torch.zeros(N, device=dev)
        ops.layernorm_bwd(dy, x, mean, rstd, g, dx, dx_drop=dxd, drop_p=0.2, seed=99, dgamma=dg, dbeta=db)
        torch.cuda.synchronize()
        quant_check('after ln bwd %s %dx%d' % (dtype, M, N))
