"""Median time (us) of every C2 forward / dgrad GEMM shape under the
current environment (dispatch switches read once per process), beside
hipBLASLt: run it in one process per configuration to A/B static switches.
    SMER_G256_MIN=300 python tools/shape_times.py [dec]
"dec": the decoder's shapes (M = B*T = 8192 rows) instead of the encoder's."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402
from tools.gemm256s_ab import SHAPES, timeit  # noqa: E402

bf = torch.bfloat16


def main():
    tag = " ".join("%s=%s" % (k, v) for k, v in sorted(os.environ.items()) if k.startswith("SMER_"))
    shapes = SHAPES[:9]
    if len(sys.argv) > 1 and sys.argv[1] == "dec":
        shapes = [("dec fwd qkv", 8192, 1536, 512, True, "b"), ("dec fwd out", 8192, 512, 512, True, "bRd"),
                  ("dec fwd cq", 8192, 512, 512, True, "b"), ("dec fwd ffn1", 8192, 2048, 512, True, "brd"),
                  ("dec fwd ffn2", 8192, 512, 2048, True, "bRd"),
                  ("dec dgrad ffn2", 8192, 2048, 512, False, "g"), ("dec dgrad ffn1", 8192, 512, 2048, False, "R"),
                  ("dec dgrad out", 8192, 512, 512, False, ""), ("dec dgrad qkv", 8192, 512, 1536, False, "R"),
                  ("dec dgrad cq", 8192, 512, 512, False, "R")]
    for name, M, N, K, bk, epi in shapes:
        A = torch.randn(M, K, device="cuda").to(bf)
        W = (torch.randn(N, K, device="cuda") * 0.05).to(bf)
        Wm = W if bk else W.t().contiguous()
        X = torch.randn(M, N, device="cuda").to(bf)
        C = torch.empty(M, N, device="cuda", dtype=bf)
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(N, device="cuda")
        if "r" in epi:
            kw["relu"] = True
        if "d" in epi:
            kw["drop_p"], kw["seed"] = 0.1, 3
        if "R" in epi:
            kw["residual"] = X
        if "g" in epi:
            kw["gate"] = X
        ours, blas = [], []
        for _ in range(5):
            ours.append(timeit(lambda: ops.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)))
            blas.append(timeit(lambda: torch.matmul(A, Wm.t() if bk else Wm)))
        print("%-14s %-3s ours %7.1f us | blas %7.1f us   [%s]" % (name, epi, sorted(ours)[2], sorted(blas)[2], tag),
              flush=True)
        del A, W, Wm, X, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
