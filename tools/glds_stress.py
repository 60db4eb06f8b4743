"""Two-stream repeatability stress: a weight gradient on a side stream runs
concurrently with main-stream attention (forward + backward, C2 encoder
shape) and a 128x128 dgrad, N times; every output is compared bitwise with
its serial reference.  Names which kernel's outputs change under overlap.
    SMER_WGRAD_GLDS=0|1 python tools/glds_stress.py [N]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from smer_music_generation_amd import ops
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    bf = torch.bfloat16
    # side: dW (768 x 768) += dy^T x over 16384 tokens (the 128x128 kernel, split-K)
    T, Mo, Ki = 16384, 768, 768
    dy = torch.randn(T, Mo, device=dev).to(bf)
    x = torch.randn(T, Ki, device=dev).to(bf)
    ws = torch.zeros(ops.SPLITK_WS_BYTES, dtype=torch.uint8, device=dev)
    # main: attention forward + backward (B 32, H 8, L 1024, D 64) and a dgrad
    B, H, L, D = 32, 8, 1024, 64
    q, k, v = (torch.randn(B * L, H * D, device=dev).to(bf) for _ in range(3))
    do = torch.randn(B * L, H * D, device=dev).to(bf)
    g = torch.randn(B * L, 2048, device=dev).to(bf)
    w = (torch.randn(2048, H * D, device=dev) / 45).to(bf)
    kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=0.125)
    g2 = torch.randn(B * L, 2048, device=dev).to(bf)
    w2 = (torch.randn(2048, 512, device=dev) / 45).to(bf)
    xl = torch.randn(B * L, 512, device=dev).to(bf)
    mu, rs = torch.zeros(B * L, device=dev), torch.ones(B * L, device=dev)
    gam = torch.randn(512, device=dev)

    def main_work():
        o = torch.empty_like(q)
        lse = torch.empty(B * H * L, device=dev)
        ops.attn_fwd(q, k, v, o, lse, **kw)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, **kw)
        dx = ops.linear_dgrad(g, w)
        dx2 = ops.linear_dgrad(g2, w2)
        dln = torch.empty_like(xl)
        ops.layernorm_bwd(dx2, xl, mu, rs, gam, dln)
        return {"attn_o": o, "attn_dq": dq, "attn_dk": dk, "attn_dv": dv, "dgrad": dx, "dgrad256": dx2,
                "ln_bwd": dln}

    db_ref = torch.zeros(Mo, device=dev)

    def side_work(dw, db):
        ops.linear_wgrad(dy, x, dw, accumulate=False, ws=ws, db=db)

    # serial references
    ref = main_work()
    dw_ref = torch.zeros(Mo, Ki, device=dev)
    side_work(dw_ref, db_ref)
    torch.cuda.synchronize()
    side = torch.cuda.Stream(device=dev)
    bad = {}
    for it in range(n):
        dws = [torch.zeros(Mo, Ki, device=dev) for _ in range(3)]
        dbs = [torch.zeros(Mo, device=dev) for _ in range(3)]
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for dw, db in zip(dws, dbs):
                side_work(dw, db)
        outs = [main_work() for _ in range(3)]
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        for dw, db in zip(dws, dbs):
            if not torch.equal(dw, dw_ref):
                bad.setdefault("wgrad", []).append(it)
            if not torch.equal(db, db_ref):
                bad.setdefault("wgrad_bias", []).append(it)
        for o in outs:
            for name, t in o.items():
                if not torch.equal(t, ref[name]):
                    bad.setdefault(name, []).append(it)
    print("SMER_WGRAD_GLDS=%s, %d iterations: %s" % (os.environ.get("SMER_WGRAD_GLDS", "0"), n,
                                                    {k: len(v) for k, v in bad.items()} or "all bit-identical"))


if __name__ == "__main__":
    main()
