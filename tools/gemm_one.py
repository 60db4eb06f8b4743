"""Run one GEMM shape N times (for rocprofv3 PMC passes).
    python tools/gemm_one.py nn|nt M N K [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

kind, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
it = int(sys.argv[5]) if len(sys.argv) > 5 else 20
bf = torch.bfloat16
A = torch.randn(M, K, device="cuda").to(bf)
B = torch.randn(N, K, device="cuda").to(bf) if kind == "nt" else torch.randn(K, N, device="cuda").to(bf)
C = torch.empty(M, N, device="cuda", dtype=bf)
for _ in range(it):
    ops.gemm(A, B, M=M, N=N, K=K, b_kcontig=(kind == "nt"), out=C)
torch.cuda.synchronize()
print("done")
