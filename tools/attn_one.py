"""One attention kernel at the C2 encoder shape, a few launches (for PMC runs).
    python tools/attn_one.py fwd|fwd_drop|bwd_drop"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "fwd_drop"
B, H, L, D = 32, 8, 1024, 64
bf = torch.bfloat16
dev = "cuda"
q = torch.randn(B * L, H * D, device=dev).to(bf)
kv = torch.randn(B * L, 2 * H * D, device=dev).to(bf)
k, v = kv[:, :H * D], kv[:, H * D:]
o = torch.empty(B * L, H * D, device=dev, dtype=bf)
lse = torch.empty(B, H, L, device=dev)
msk = ops.attn_drop_mask(B, H, L, L, dev)
p = 0.0 if which == "fwd" else 0.1
for _ in range(5):
    ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=1 / math.sqrt(D), drop_p=p, seed=1,
                 drop_mask=msk if p else None)
if which == "bwd_drop":
    do = torch.randn_like(o)
    dq = torch.empty_like(q)
    dkv = torch.empty_like(kv)
    for _ in range(5):
        ops.attn_bwd(q, k, v, o, do, lse, dq, dkv[:, :H * D], dkv[:, H * D:], B=B, H=H, Lq=L, Lk=L, D=D,
                     scale=1 / math.sqrt(D), drop_p=p, seed=1, drop_mask=msk)
torch.cuda.synchronize()
print("ok")
