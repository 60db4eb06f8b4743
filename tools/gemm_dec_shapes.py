"""The C2 decoder's forward / dgrad GEMM shapes (M = B*T = 8192 rows, d 512,
FFN 2048) with each shape's train-step epilogue: the default dispatch, the
128x128 kernel instead of the 64x128 one (SMER_GEMM64=0) and hipBLASLt
(torch, bare product); interleaved rounds, median of 5 (us and TFLOP/s).
SMER_HIP_LIB selects a variant library (tools/build_variant.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16
Mt, d, F = 8192, 512, 2048
SHAPES = [  # name, N, K, b_kcontig, epilogue
    ("fwd qkv", 3 * d, d, True, "b"), ("fwd out", d, d, True, "bRd"), ("fwd crossq", d, d, True, "b"),
    ("fwd ffn1", F, d, True, "brd"), ("fwd ffn2", d, F, True, "bRd"),
    ("dgrad ffn2", F, d, False, "g"), ("dgrad ffn1", d, F, False, "R"), ("dgrad out", d, d, False, ""),
    ("dgrad qkv", d, 3 * d, False, "R"), ("dgrad crossq", d, d, False, "R"),
]


def timeit(fn, iters=30):
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
    variants = [v for v in sys.argv[1:]] or ["default", "SMER_GEMM64=0"]
    tot = {v: 0.0 for v in variants + ["blas"]}
    for name, N, K, bk, epi in SHAPES:
        M = Mt
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
        t = {v: [] for v in variants + ["blas"]}
        for _ in range(5):
            for v in variants:
                saved = {}
                if v != "default":
                    for kv in v.split(","):
                        k_, v_ = kv.split("=")
                        saved[k_] = os.environ.get(k_)
                        os.environ[k_] = v_
                t[v].append(timeit(lambda: ops.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)))
                for k_, v_ in saved.items():
                    if v_ is None:
                        del os.environ[k_]
                    else:
                        os.environ[k_] = v_
            t["blas"].append(timeit(lambda: torch.matmul(A, Wm.t() if bk else Wm)))
        med = {k: sorted(x)[2] for k, x in t.items()}
        fl = 2.0 * M * N * K
        print("%-13s N%5d K%5d %-3s " % (name, N, K, epi) +
              " | ".join("%s %6.1f us %5.0f TF" % (k, med[k], fl / med[k] / 1e6) for k in t), flush=True)
        for k in t:
            tot[k] += med[k]
    print("sum: " + " | ".join("%s %.1f us" % (k, v) for k, v in tot.items()))


if __name__ == "__main__":
    main()
