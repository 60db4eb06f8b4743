"""Per-shape microbenchmarks of the hot kernels at the C2 shapes (GPU).

    python tools/bench_kernels.py [gemm|attn|attn_c4|all]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = "cuda"


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def bench_gemm():
    bf = torch.bfloat16
    Ms, Mt, d, F = 32768, 8192, 512, 2048
    rows = []
    shapes = [("fwd qkv enc", "nt", Ms, 3 * d, d), ("fwd ffn1 enc", "nt", Ms, F, d),
              ("fwd ffn2 enc", "nt", Ms, d, F), ("fwd out enc", "nt", Ms, d, d),
              ("dgrad ffn2 enc", "nn", Ms, F, d), ("dgrad ffn1 enc", "nn", Ms, d, F),
              ("dgrad qkv enc", "nn", Ms, d, 3 * d),
              ("wgrad ffn1 enc", "tn", F, d, Ms), ("wgrad qkv enc", "tn", 3 * d, d, Ms),
              ("wgrad out enc", "tn", d, d, Ms), ("fwd qkv dec", "nt", Mt, 3 * d, d)]
    for name, kind, M, N, K in shapes:
        if kind == "nt":
            A = torch.randn(M, K, device=dev).to(bf)
            B = torch.randn(N, K, device=dev).to(bf)
            C = torch.empty(M, N, device=dev, dtype=bf)
            bias = torch.randn(N, device=dev)
            t = timeit(lambda: ops.gemm(A, B, M=M, N=N, K=K, out=C))
            t2 = timeit(lambda: ops.gemm(A, B, M=M, N=N, K=K, out=C, bias=bias, relu=True,
                                         drop_p=0.1, seed=3))
        elif kind == "nn":
            A = torch.randn(M, K, device=dev).to(bf)
            B = torch.randn(K, N, device=dev).to(bf)
            C = torch.empty(M, N, device=dev, dtype=bf)
            R = torch.randn(M, N, device=dev).to(bf)
            t = timeit(lambda: ops.gemm(A, B, M=M, N=N, K=K, b_kcontig=False, out=C))
            t2 = timeit(lambda: ops.gemm(A, B, M=M, N=N, K=K, b_kcontig=False, out=C, residual=R))
        else:
            A = torch.randn(K, M, device=dev).to(bf)
            B = torch.randn(K, N, device=dev).to(bf)
            C = torch.zeros(M, N, device=dev)
            t = timeit(lambda: ops.gemm(A, B, M=M, N=N, K=K, a_kcontig=False, b_kcontig=False,
                                        out_f32=C, accumulate=True, dtype=bf))
            t2 = t
        fl = 2.0 * M * N * K
        # vendor library reference point (torch -> hipBLASLt), same shapes / layouts
        if kind == "nt":
            tt = timeit(lambda: torch.mm(A, B.t(), out=C))
        elif kind == "nn":
            tt = timeit(lambda: torch.mm(A, B, out=C))
        else:
            Cb = torch.empty(M, N, device=dev, dtype=bf)
            tt = timeit(lambda: torch.mm(A.t(), B, out=Cb))
        print("%-16s %s M=%6d N=%5d K=%6d  %8.1f us %7.1f TF   (epilogue: %8.1f us %7.1f TF)"
              "  [torch/hipBLASLt %7.1f TF]"
              % (name, kind, M, N, K, t, fl / t / 1e6, t2, fl / t2 / 1e6, fl / tt / 1e6))


ATTN_SHAPES = {
    "c2": (("enc self", 32, 8, 1024, 1024, False), ("dec self", 32, 8, 256, 256, True),
           ("cross", 32, 8, 256, 1024, False)),
    "c4": (("c4 enc self", 32, 12, 2048, 2048, False), ("c4 dec self", 32, 12, 512, 512, True),
           ("c4 cross", 32, 12, 512, 2048, False)),
}


def bench_attn(cfg="c2"):
    bf = torch.bfloat16
    for name, B, H, Lq, Lk, causal in ATTN_SHAPES[cfg]:
        D = 64
        q = torch.randn(B * Lq, H * D, device=dev).to(bf)
        kv = torch.randn(B * Lk, 2 * H * D, device=dev).to(bf)
        k, v = kv[:, :H * D], kv[:, H * D:]
        o = torch.empty(B * Lq, H * D, device=dev, dtype=bf)
        lse = torch.empty(B, H, Lq, device=dev)
        sc = 1 / math.sqrt(D)
        t = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D,
                                        causal=causal, scale=sc))
        msk = ops.attn_drop_mask(B, H, Lq, Lk, dev)
        tg = timeit(lambda: ops.attn_drop_mask_gen(msk, B=B, H=H, Lq=Lq, Lk=Lk, drop_p=0.1, seed=1))
        td = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D,
                                         causal=causal, scale=sc, drop_p=0.1, seed=1,
                                         drop_mask=msk, drop_mask_in=True))
        th = timeit(lambda: ops.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D,
                                         causal=causal, scale=sc, drop_p=0.1, seed=1,
                                         drop_mask=msk))
        do = torch.randn_like(o)
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        tb = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dkv[:, :H * D], dkv[:, H * D:],
                                         B=B, H=H, Lq=Lq, Lk=Lk, D=D, causal=causal, scale=sc))
        tbd = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dkv[:, :H * D], dkv[:, H * D:],
                                          B=B, H=H, Lq=Lq, Lk=Lk, D=D, causal=causal, scale=sc,
                                          drop_p=0.1, seed=1, drop_mask=msk))
        fl = 4.0 * B * H * Lq * Lk * D * (0.5 if causal else 1.0)
        print("%-9s fwd %7.1f us %6.1f TF | mask gen %6.1f | fwd+drop gen'd %7.1f (product: own %7.1f) | bwd %7.1f us "
              "%6.1f TF (2.5x fwd flops) | bwd+drop %7.1f us"
              % (name, t, fl / t / 1e6, tg, td, th, tb, 2.5 * fl / tb / 1e6, tbd))


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("gemm", "all"):
        bench_gemm()
    if which in ("attn", "all"):
        bench_attn()
    if which in ("attn_c4", "all"):
        bench_attn("c4")
