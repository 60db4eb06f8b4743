"""Start-skew probe of the persistent 256x256 forward / dgrad kernels
(SMER_G256_SKEW, units of ~2k cycles for every second workgroup of an XCD)
at the C2 forward and dgrad shapes: does desynchronising the all-CU
epilogue store bursts help?  Interleaved, median of 5, both schedules
(SMER_GEMM256S=0 two-stage, =1 staggered) and hipBLASLt.
    python tools/skew_ab.py [skew values...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402
from tools.gemm256s_ab import SHAPES, timeit  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def main():
    skews = [int(x) for x in sys.argv[1:]] or [0, 2, 4, 8]
    for name, M, N, K, bk, epi in SHAPES[:9]:
        A = torch.randn(M, K, device=dev).to(bf)
        W = (torch.randn(N, K, device=dev) * 0.05).to(bf)
        Wm = W if bk else W.t().contiguous()
        X = torch.randn(M, N, device=dev).to(bf)
        C = torch.empty(M, N, device=dev, dtype=bf)
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(N, device=dev)
        if "r" in epi:
            kw["relu"] = True
        if "d" in epi:
            kw["drop_p"], kw["seed"] = 0.1, 3
        if "R" in epi:
            kw["residual"] = X
        if "g" in epi:
            kw["gate"] = X
        t = {}
        for _ in range(5):
            for flag in ("0", "1"):
                os.environ["SMER_GEMM256S"] = flag
                for sk in skews:
                    os.environ["SMER_G256_SKEW"] = str(sk)
                    t.setdefault((flag, sk), []).append(
                        timeit(lambda: ops.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)))
            t.setdefault("blas", []).append(timeit(lambda: torch.matmul(A, Wm.t() if bk else Wm)))
        os.environ.pop("SMER_G256_SKEW", None)
        os.environ.pop("SMER_GEMM256S", None)
        med = {k: sorted(v)[2] for k, v in t.items()}
        line = " | ".join("%s s%d %6.1f" % ("stag" if f == "1" else "2stg", sk, med[(f, sk)])
                          for f in ("0", "1") for sk in skews)
        print("%-11s %-3s %s | blas %6.1f us" % (name, epi, line, med["blas"]), flush=True)
        del A, W, Wm, X, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
