"""A/B of the staggered 256x256 GEMM (SMER_GEMM256S=1) against the two-stage
kernel (=0) and hipBLASLt (torch.matmul) at the C2 / C4 forward and dgrad
shapes, with the epilogue each shape has in the train step; interleaved
rounds in one process, median of 5 (us and TFLOP/s)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


SHAPES = [  # name, M, N, K, b_kcontig, epilogue
    ("fwd qkv", 32768, 1536, 512, True, "b"), ("fwd out", 32768, 512, 512, True, "bRd"),
    ("fwd ffn1", 32768, 2048, 512, True, "brd"), ("fwd ffn2", 32768, 512, 2048, True, "bRd"),
    ("fwd ckv", 32768, 6144, 512, True, "b"),
    ("dgrad ffn2", 32768, 2048, 512, False, "g"), ("dgrad ffn1", 32768, 512, 2048, False, "R"),
    ("dgrad out", 32768, 512, 512, False, ""), ("dgrad qkv", 32768, 512, 1536, False, "R"),
    ("c4 fwd qkv", 65536, 2304, 768, True, "b"), ("c4 dgrad ffn1", 65536, 768, 2048, False, "R"),
]


def main():
    rows = []
    for name, M, N, K, bk, epi in SHAPES:
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
        t = {"1": [], "0": [], "blas": []}
        for _ in range(5):
            for flag in ("1", "0"):
                os.environ["SMER_GEMM256S"] = flag
                t[flag].append(timeit(lambda: ops.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)))
            t["blas"].append(timeit(lambda: torch.matmul(A, Wm.t() if bk else Wm)))
        med = {k: sorted(v)[2] for k, v in t.items()}
        fl = 2.0 * M * N * K
        print("%-14s M%6d N%5d K%5d %-3s  stag %7.1f us %5.0f TF | two-stage %7.1f us %5.0f TF | blas %7.1f us %5.0f TF"
              % (name, M, N, K, epi, med["1"], fl / med["1"] / 1e6, med["0"], fl / med["0"] / 1e6,
                 med["blas"], fl / med["blas"] / 1e6), flush=True)
        del A, W, Wm, X, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
