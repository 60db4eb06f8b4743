"""Decode-step kernels in isolation, each captured 50x back to back in a HIP
graph and replayed (the decode step's launch regime): per-launch time.

    python tools/bench_decode_kernels.py [R] [S]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from smer_music_generation_amd import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def graph_time(fn, reps=50, iters=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * reps)


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    M, d, F, V = 2 * R, 512, 2048, 309
    x = torch.randn(M, d, device=dev).to(bf)
    one = torch.zeros(8, device=dev)
    one_b = torch.zeros(8, device=dev, dtype=bf)
    print("R=%d M=%d S=%d" % (R, M, S))
    print("%-34s %8.2f us" % ("floor: 8-element cast", graph_time(lambda: ops.cast(one, one_b))))
    for name, N, K in (("qkv N1536 K512", 3 * d, d), ("out N512 K512", d, d),
                       ("ffn1 N2048 K512 relu", F, d), ("ffn2 N512 K2048", d, F)):
        w = torch.randn(N, K, device=dev).to(bf)
        b = torch.randn(N, device=dev)
        a = torch.randn(M, K, device=dev).to(bf)
        y = torch.empty(M, N, device=dev, dtype=bf)
        res = torch.randn(M, N, device=dev).to(bf)
        t = graph_time(lambda: ops.linear(a, w, b, out=y, relu="relu" in name,
                                          residual=res if N == d else None))
        byt = N * K * 2 + M * K * 2 + M * N * 2
        print("%-34s %8.2f us  %7.1f GB/s" % ("gemm " + name, t, byt / t / 1e3))
    wf = torch.randn(V, d, device=dev).to(bf)
    lg = torch.empty(M, V, device=dev)
    bfc = torch.randn(V, device=dev)
    print("%-34s %8.2f us" % ("gemm head N309 f32 out", graph_time(
        lambda: ops.gemm(x, wf, M=M, N=V, K=d, out_f32=lg, bias=bfc, dtype=bf))))
    g_ = torch.ones(d, device=dev)
    b_ = torch.zeros(d, device=dev)
    y = torch.empty(M, d, device=dev, dtype=bf)
    mu = torch.empty(M, device=dev)
    rs = torch.empty(M, device=dev)
    print("%-34s %8.2f us" % ("layernorm M x 512", graph_time(lambda: ops.layernorm(x, g_, b_, y, mu, rs))))
    H, D = 8, 64
    for name, nk, cap in (("self nk=100", 100, 600), ("cross nk=%d" % S, S, S)):
        req = (torch.arange(M, device=dev, dtype=torch.int32) // 2)
        nks = torch.full((M,), nk, device=dev, dtype=torch.int32)
        nks[0::2] = 1
        q = torch.randn(M, d, device=dev).to(bf)
        o = torch.empty(M, d, device=dev, dtype=bf)
        if name.startswith("self"):
            cache = torch.randn(R, cap, 2 * d, device=dev).to(bf)
            t = graph_time(lambda: ops.attn_decode(q, cache, cache.view(-1)[d:], req, nks, o, H=H,
                                                   D=D, row_stride=2 * d, req_stride=cap * 2 * d,
                                                   scale=1 / math.sqrt(D)))
        else:  # head-major memory, as DecodeSession stores it
            cache = torch.randn(R, 2, H, cap, D, device=dev).to(bf)
            t = graph_time(lambda: ops.attn_decode(q, cache, cache.view(-1)[H * cap * D:], req, nks,
                                                   o, H=H, D=D, row_stride=D,
                                                   req_stride=2 * H * cap * D,
                                                   head_stride=cap * D, scale=1 / math.sqrt(D)))
        byt = R * nk * 2 * d * 2
        print("%-34s %8.2f us  %7.1f GB/s" % ("attn_decode " + name, t, byt / t / 1e3))
    cache = torch.zeros(R, 600, 2 * d, device=dev).to(bf)
    qkv = torch.randn(M, 3 * d, device=dev).to(bf)
    pos = torch.full((M,), 5, device=dev, dtype=torch.int32)
    req = (torch.arange(M, device=dev, dtype=torch.int32) // 2)
    print("%-34s %8.2f us" % ("kv_scatter", graph_time(lambda: ops.kv_scatter(
        qkv[:, d:], cache, req, pos, row_stride=2 * d, req_stride=600 * 2 * d))))


if __name__ == "__main__":
    main()
