"""A/B of the staggered fp8 GEMM (SMER_GEMM256S_FP8=1) against the two-stage
fp8 kernel (=0) at the C4 fp8 training shapes (encoder rows 32 x 2048,
d 768, FFN 2048), with each shape's epilogue; interleaved rounds in one
process, median of 5 (us and TFLOP/s)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16

SHAPES = [  # name, M, N, K, epilogue
    ("fwd qkv", 65536, 2304, 768, "b"), ("fwd out", 65536, 768, 768, "bRd"),
    ("fwd ffn2", 65536, 768, 2048, "bRd"), ("dgrad ffn2", 65536, 2048, 768, "g"),
    ("dgrad ffn1", 65536, 768, 2048, "R"), ("dgrad out", 65536, 768, 768, ""),
    ("dgrad qkv", 65536, 768, 2304, "R"), ("dec ffn2", 16384, 768, 2048, "bRd"),
]


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


def main():
    for name, M, N, K, epi in SHAPES:
        a8 = torch.randint(0, 255, (M, K), device=dev, dtype=torch.uint8) & 0x77
        b8 = torch.randint(0, 255, (N, K), device=dev, dtype=torch.uint8) & 0x77
        ai = torch.tensor([0.01], device=dev)
        bi = torch.tensor([0.02], device=dev)
        X = torch.randn(M, N, device=dev).to(bf)
        C = torch.empty(M, N, device=dev, dtype=bf)
        kw = {}
        if "b" in epi:
            kw["bias"] = torch.randn(N, device=dev)
        if "d" in epi:
            kw["drop_p"], kw["seed"] = 0.1, 3
        if "R" in epi:
            kw["residual"] = X
        if "g" in epi:
            kw["gate"] = X
        t = {"1": [], "0": []}
        for _ in range(5):
            for flag in ("1", "0"):
                os.environ["SMER_GEMM256S_FP8"] = flag
                fn = ops.gemm_fp8_ex if "g" in epi else ops.gemm_fp8
                t[flag].append(timeit(lambda: fn(a8, ai, b8, bi, C, **kw)))
        med = {k: sorted(v)[2] for k, v in t.items()}
        fl = 2.0 * M * N * K
        print("%-12s M%6d N%5d K%5d %-3s  stag %7.1f us %5.0f TF | two-stage %7.1f us %5.0f TF"
              % (name, M, N, K, epi, med["1"], fl / med["1"] / 1e6, med["0"], fl / med["0"] / 1e6),
              flush=True)
        del a8, b8, X, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
