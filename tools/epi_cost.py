"""Epilogue cost of the C2 forward GEMMs: the same shape timed with no
epilogue, bias, bias+ReLU, bias+ReLU+dropout, bias+residual(+dropout)
(median of 5, interleaved), beside hipBLASLt (no epilogue)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402
from tools.gemm256s_ab import timeit  # noqa: E402

bf = torch.bfloat16
for name, M, N, K in [("ffn1", 32768, 2048, 512), ("qkv", 32768, 1536, 512), ("out", 32768, 512, 512),
                      ("ffn2", 32768, 512, 2048)]:
    A = torch.randn(M, K, device="cuda").to(bf)
    W = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
    X = torch.randn(M, N, device="cuda").to(bf)
    C = torch.empty(M, N, device="cuda", dtype=bf)
    b = torch.randn(N, device="cuda")
    cfgs = {"none": {}, "b": dict(bias=b), "br": dict(bias=b, relu=True),
            "brd": dict(bias=b, relu=True, drop_p=0.1, seed=3), "bR": dict(bias=b, residual=X),
            "bRd": dict(bias=b, residual=X, drop_p=0.1, seed=3)}
    t = {k: [] for k in list(cfgs) + ["blas"]}
    for _ in range(5):
        for k, kw in cfgs.items():
            t[k].append(timeit(lambda: ops.gemm(A, W, M=M, N=N, K=K, out=C, **kw)))
        t["blas"].append(timeit(lambda: torch.matmul(A, W.t())))
    print(name, " ".join("%s %.1f" % (k, sorted(v)[2]) for k, v in t.items()), flush=True)
