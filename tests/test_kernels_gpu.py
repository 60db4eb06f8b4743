"""Kernel-level parity of the HIP C-ABI against fp32 torch math on the GPU
(floating-point kernels: torch fp32 is the reference of the same op)."""
import math
import os

import numpy as np
import pytest
import torch

from tests.hashref import attn_keep_mask, attn_scale, drop_scale, keep_mask

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from smer_music_generation_amd import _lib as L
    L.load()
    torch.manual_seed(0)


def ops():
    from smer_music_generation_amd import ops as O
    return O


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


# ----------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (200, 309, 136), (8, 64, 64), (1000, 512, 2048)])
def test_gemm_layouts(dtype, ak, bk, M, N, K):
    O = ops()
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    Am = A if ak else A.t().contiguous()
    Bm = B if bk else B.t().contiguous()
    if not ak and M % 8:
        Am = torch.zeros(K, (M + 7) // 8 * 8, device=dev)
        Am[:, :M] = A.t()
    if not bk and N % 8:
        Bm = torch.zeros(K, (N + 7) // 8 * 8, device=dev)
        Bm[:, :N] = B.t()
    Am, Bm = Am.to(dtype), Bm.to(dtype)
    ref = A.to(dtype).float() @ B.to(dtype).float().t()
    C = torch.empty(M, N, device=dev, dtype=dtype)
    O.gemm(Am, Bm, M=M, N=N, K=K, a_kcontig=ak, b_kcontig=bk, out=C)
    Cf = torch.empty(M, N, device=dev)
    O.gemm(Am, Bm, M=M, N=N, K=K, a_kcontig=ak, b_kcontig=bk, out_f32=Cf, dtype=dtype)
    torch.cuda.synchronize()
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert rel_err(C, ref) < tol
    assert rel_err(Cf, ref) < (2e-3 if dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("M,N,K", [(256, 384, 8192), (309, 512, 4096), (1536, 512, 16384)])
def test_gemm_splitk_wgrad(M, N, K):
    """Weight-gradient shape (both operands column images, long K): the
    deterministic split-K slab path must equal the unsplit result."""
    O = ops()
    dy = torch.randn(K, (M + 7) // 8 * 8, device=dev).to(torch.bfloat16)
    x = torch.randn(K, N, device=dev).to(torch.bfloat16)
    ref = dy[:, :M].float().t() @ x.float()
    base = torch.randn(M, N, device=dev)
    out = base.clone()
    O.gemm(dy, x, M=M, N=N, K=K, a_kcontig=False, b_kcontig=False, out_f32=out, accumulate=True,
           dtype=torch.bfloat16)
    out2 = base.clone()
    O.gemm(dy, x, M=M, N=N, K=K, a_kcontig=False, b_kcontig=False, out_f32=out2, accumulate=True,
           dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert rel_err(out - base, ref) < 2e-3
    assert torch.equal(out, out2)  # deterministic


@pytest.mark.parametrize("M,N,K,acc", [(512, 512, 32768, True), (1536, 512, 8192, False),
                                       (309, 512, 4096, True), (200, 136, 96, True),
                                       (1000, 776, 32768, True), (4096, 4096, 512, False),
                                       (4096, 4096, 512, True)])
def test_gemm_wgrad_bias(M, N, K, acc):
    """Fused weight + bias gradient (split-K and unsplit, ragged M via a
    padded dy row stride) equals dy^T x and the column sums of dy.  The
    first two and the last three shapes run the 256x256 weight-gradient
    kernel (ragged 256-tiles; unsplit when the tiles alone fill the chip),
    the others the 128x128 one."""
    O = ops()
    ldm = (M + 7) // 8 * 8
    dy = torch.randn(K, ldm, device=dev).to(torch.bfloat16)
    x = torch.randn(K, N, device=dev).to(torch.bfloat16)
    dw0, db0 = torch.randn(M, N, device=dev), torch.randn(M, device=dev)
    dw, db = dw0.clone(), db0.clone()
    O.linear_wgrad(dy, x, dw, M=M, accumulate=acc, db=db)
    ref_w = dy[:, :M].float().t() @ x.float() + (dw0 if acc else 0)
    ref_b = dy[:, :M].float().sum(0) + (db0 if acc else 0)
    torch.cuda.synchronize()
    assert rel_err(dw, ref_w) < 2e-3
    assert rel_err(db, ref_b) < 2e-3
    # deterministic: a second run is bit-identical
    dw2, db2 = dw0.clone(), db0.clone()
    O.linear_wgrad(dy, x, dw2, M=M, accumulate=acc, db=db2)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("M,N,K,acc", [(512, 512, 32768, True), (1536, 512, 8192, False),
                                       (309, 512, 4096, True), (2048, 512, 32768, True),
                                       (512, 2048, 8192, False), (200, 136, 96, True)])
def test_splitk_last_arriver_equals_separate_reduce(monkeypatch, M, N, K, acc):
    """The fused split-K reduction (the tile's last-arriving slice sums the
    write-through slabs in slice order, csrc/gemm.hip splitk_tile_reduce)
    gives the same bits as the separate splitk_reduce_kernel, dW and db,
    run after run; the ticket words are left zero (a second call on the
    same workspace is still right)."""
    O = ops()
    ldm = (M + 7) // 8 * 8
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    dy = torch.randn(K, ldm, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(K, N, device=dev, generator=g).to(torch.bfloat16)
    dw0, db0 = torch.randn(M, N, device=dev, generator=g), torch.randn(M, device=dev, generator=g)
    outs = []
    for fused in ("0", "1", "1"):
        monkeypatch.setenv("SMER_SPLITK_FUSED", fused)
        dw, db = dw0.clone(), db0.clone()
        O.linear_wgrad(dy, x, dw, M=M, accumulate=acc, db=db)
        torch.cuda.synchronize()
        outs.append((dw, db))
    ref_w = dy[:, :M].float().t() @ x.float() + (dw0 if acc else 0)
    assert rel_err(outs[1][0], ref_w) < 2e-3
    for dw, db in outs[1:]:
        assert torch.equal(dw, outs[0][0]) and torch.equal(db, outs[0][1])
    ws = O.splitk_workspace(dy.device)
    assert int(ws[-64 * 1024:].view(torch.int32).abs().sum()) == 0  # tickets reset


@pytest.mark.parametrize("M,N,K,acc", [(1536, 768, 16384, True), (3072, 768, 8192, False),
                                       (2304, 768, 32768, True), (4096, 4096, 512, True)])
def test_gemm256s_wgrad_matches_reference(monkeypatch, M, N, K, acc):
    """The staggered weight-gradient kernel (SMER_WGRAD256S=1) on the 256x256
    split-K shapes: dw = dy^T x and db = column sums of dy (split and
    unsplit, accumulate on / off) against fp32 torch, deterministic, and
    against the two-stage 256x256 kernel (same k order per slice)."""
    O = ops()
    dy = torch.randn(K, M, device=dev).to(torch.bfloat16)
    x = torch.randn(K, N, device=dev).to(torch.bfloat16)
    dw0, db0 = torch.randn(M, N, device=dev), torch.randn(M, device=dev)
    ref_w = dy.float().t() @ x.float() + (dw0 if acc else 0)
    ref_b = dy.float().sum(0) + (db0 if acc else 0)
    outs = {}
    for flag in ("1", "1", "0"):
        monkeypatch.setenv("SMER_WGRAD256S", flag)
        dw, db = dw0.clone(), db0.clone()
        O.linear_wgrad(dy, x, dw, M=M, accumulate=acc, db=db)
        torch.cuda.synchronize()
        if flag in outs:
            assert torch.equal(dw, outs[flag][0]) and torch.equal(db, outs[flag][1])
        outs[flag] = (dw, db)
    dw, db = outs["1"]
    assert rel_err(dw, ref_w) < 2e-3
    assert rel_err(db, ref_b) < 2e-3
    assert rel_err(dw, outs["0"][0]) < 1e-5 and rel_err(db, outs["0"][1]) < 1e-5


@pytest.mark.parametrize("M,N,K,bk", [(8300, 2056, 512, True), (8192, 2048, 192, False),
                                      (16384, 1536, 1024, True), (8200, 2048, 256, False)])
def test_gemm256_large_m(M, N, K, bk):
    """The 256x256 kernel (>= one tile per CU) with ragged M / N tails and
    the full epilogue (bias, relu, dropout, residual) against fp32."""
    O = ops()
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    Wm = W if bk else W.t().contiguous()
    bias = torch.randn(N, device=dev)
    R = torch.randn(M, N, device=dev).to(torch.bfloat16)
    p, seed = 0.1, 7
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, bias=bias, relu=True, residual=R, drop_p=p,
           seed=seed)
    base = A.float() @ W.float().t()
    keep = torch.from_numpy(keep_mask(seed, p, M, N)).to(dev)
    ref = R.float() + torch.where(keep, torch.relu(base + bias) * drop_scale(p), torch.zeros_like(base))
    Cf = torch.empty(M, N, device=dev)
    O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out_f32=Cf)
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 2e-2
    assert rel_err(Cf, base) < 2e-3


@pytest.mark.parametrize("M,N,K,bk", [(8192, 2048, 512, False), (16384, 512, 1536, True)])
def test_gemm256_streamed_epilogue_gate(M, N, K, bk):
    """The 256x256 kernel's streamed epilogue with a ReLU-grad gate (the
    dgrad into the FFN hidden layer) and with a bare residual."""
    O = ops()
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    Wm = W if bk else W.t().contiguous()
    G = torch.randn(M, N, device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, gate=G, gate_scale=1.5)
    base = A.float() @ W.float().t()
    ref = torch.where(G.float() > 0, base * 1.5, torch.zeros_like(base))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 2e-2
    O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, residual=G)
    torch.cuda.synchronize()
    assert rel_err(C, base + G.float()) < 2e-2


@pytest.mark.parametrize("M,N,K,bk,epi", [
    (8192, 2048, 512, True, "bias_relu_drop"), (8192, 2048, 512, False, "gate"),
    (32768, 512, 2048, True, "bias_residual"), (16384, 1536, 512, True, "bias"),
    (16384, 512, 1536, False, "residual"), (8192, 512, 2048, False, "none"),
    (12288, 768, 128, True, "bias_residual")])
def test_gemm256s_matches_two_stage_kernel(monkeypatch, M, N, K, bk, epi):
    """The staggered 256x256 kernel (four k-step slots, loader / storer wave
    roles, 32-row epilogue passes) against the two-stage 256x256 kernel it
    replaces (SMER_GEMM256S=0): same k order and epilogue arithmetic, so the
    outputs are bit-identical; and against fp32.  Shapes: >= 256 whole tiles
    (one per CU and more: the persistent tile loop), K from 4 k-steps up."""
    O = ops()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(dev).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) * 0.05).to(dev).to(torch.bfloat16)
    Wm = W if bk else W.t().contiguous()
    X = torch.randn(M, N, generator=g).to(dev).to(torch.bfloat16)
    bias = torch.randn(N, generator=g).to(dev)
    kw = {}
    if "bias" in epi:
        kw["bias"] = bias
    if "relu" in epi:
        kw["relu"] = True
    if "drop" in epi:
        kw["drop_p"], kw["seed"] = 0.1, 11
    if "residual" in epi:
        kw["residual"] = X
    if "gate" in epi:
        kw["gate"], kw["gate_scale"] = X, 1.25
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("SMER_GEMM256S", flag)
        C = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, **kw)
        outs[flag] = C
    torch.cuda.synchronize()
    assert torch.equal(outs["1"], outs["0"]), (outs["1"] - outs["0"]).abs().max()
    base = A.float() @ W.float().t()
    ref = base + (bias if "bias" in epi else 0)
    if "relu" in epi:
        ref = torch.relu(ref)
    if "drop" in epi:
        keep = torch.from_numpy(keep_mask(11, 0.1, M, N)).to(dev)
        ref = torch.where(keep, ref * drop_scale(0.1), torch.zeros_like(ref))
    if "residual" in epi:
        ref = ref + X.float()
    if "gate" in epi:
        ref = torch.where(X.float() > 0, ref * 1.25, torch.zeros_like(ref))
    assert rel_err(outs["1"], ref) < 2e-2


def test_gemm_identity_asymmetric():
    O = ops()
    n = 128
    A = torch.eye(n, device=dev, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=dev).view(n, n) % 97).to(torch.bfloat16)
    C = torch.empty(n, n, device=dev, dtype=torch.float32)
    O.gemm(A, B, M=n, N=n, K=n, out_f32=C, dtype=torch.bfloat16)
    torch.cuda.synchronize()
    assert torch.equal(C, B.float().t())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(192, 256, 128), (640, 264, 136), (40, 264, 136),
                                   (64, 512, 2048), (130, 264, 1040), (2, 309, 512), (2, 512, 2048),
                                   (17, 1544, 520)])
def test_gemm_epilogue(dtype, M, N, K):
    """Skinny (M <= 256) and tiled kernels, incl. N and K tails."""
    O = ops()
    A = torch.randn(M, K, device=dev).to(dtype)
    W = torch.randn(N, K, device=dev).to(dtype)
    bias = torch.randn(N, device=dev)
    R = torch.randn(M, N, device=dev).to(dtype)
    G = torch.randn(M, N, device=dev).to(dtype)
    base = A.float() @ W.float().t()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    # bias + relu + dropout + residual
    p, seed = 0.25, 1234
    C = torch.empty(M, N, device=dev, dtype=dtype)
    O.gemm(A, W, M=M, N=N, K=K, out=C, bias=bias, relu=True, residual=R, drop_p=p, seed=seed)
    keep = torch.from_numpy(keep_mask(seed, p, M, N)).to(dev)
    ref = R.float() + torch.where(keep, torch.relu(base + bias) * drop_scale(p), torch.zeros_like(base))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < tol
    # gate (relu-backward) + fp32 accumulate
    Cf = torch.randn(M, N, device=dev)
    Cf0 = Cf.clone()
    O.gemm(A, W, M=M, N=N, K=K, out_f32=Cf, accumulate=True, gate=G, gate_scale=2.0, dtype=dtype)
    ref = Cf0 + torch.where(G.float() > 0, base * 2.0, torch.zeros_like(base))
    torch.cuda.synchronize()
    assert rel_err(Cf, ref) < (2e-3 if dtype == torch.bfloat16 else 1e-5)


# ------------------------------------------------------------ attention
def attn_ref(q, k, v, B, H, Lq, Lk, D, kpm, causal, scale, keep=None, p=0.0):
    """fp32 reference; dropout survivors scaled by the kernel's 8-bit-rate
    factor (tests/hashref.py attn_scale)."""
    qh = q.float().view(B, Lq, H, D).transpose(1, 2)
    kh = k.float().view(B, Lk, H, D).transpose(1, 2)
    vh = v.float().view(B, Lk, H, D).transpose(1, 2)
    s = (qh @ kh.transpose(-1, -2)) * scale
    mask = torch.zeros(B, 1, Lq, Lk, device=dev, dtype=torch.bool)
    if kpm is not None:
        mask |= kpm.bool().view(B, 1, 1, Lk)
    if causal:
        mask |= torch.triu(torch.ones(Lq, Lk, device=dev, dtype=torch.bool), 1)
    s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, -1)
    pr = torch.softmax(s, -1)
    if keep is not None:
        pr = torch.where(keep, pr * attn_scale(p), torch.zeros_like(pr))
    o = (pr @ vh).transpose(1, 2).reshape(B * Lq, H * D)
    return o, lse


def _attn_inputs(B, H, Lq, Lk, D, dtype, pad):
    q = torch.randn(B * Lq, H * D, device=dev).to(dtype)
    kv = torch.randn(B * Lk, 2 * H * D, device=dev).to(dtype)
    k, v = kv[:, : H * D], kv[:, H * D:]
    kpm = None
    if pad:
        kpm = torch.zeros(B, Lk, device=dev, dtype=torch.uint8)
        kpm[-1, Lk - Lk // 3:] = 1
    return q, k, v, kpm


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("Lq,Lk,causal,pad", [(128, 128, False, True), (100, 100, True, True),
                                              (64, 150, False, True), (256, 256, True, False)])
def test_attention_fwd_bwd(dtype, D, Lq, Lk, causal, pad):
    O = ops()
    B, H = 2, 3
    q, k, v, kpm = _attn_inputs(B, H, Lq, Lk, D, dtype, pad)
    scale = 1.0 / math.sqrt(D)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=dtype)
    lse = torch.empty(B, H, Lq, device=dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, kpm=kpm, causal=causal, scale=scale)
    qf, kf, vf = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ro, rlse = attn_ref(qf, kf, vf, B, H, Lq, Lk, D, kpm, causal, scale)
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 2e-5
    assert rel_err(o, ro) < tol
    assert (lse - rlse).abs().max().item() < (2e-2 if dtype == torch.bfloat16 else 1e-4)
    do = torch.randn(B * Lq, H * D, device=dev).to(dtype)
    ro.backward(do.float())
    dq = torch.empty_like(q)
    dkv = torch.empty(B * Lk, 2 * H * D, device=dev, dtype=dtype)
    dk, dv = dkv[:, : H * D], dkv[:, H * D:]
    O.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=Lq, Lk=Lk, D=D, kpm=kpm,
               causal=causal, scale=scale)
    torch.cuda.synchronize()
    tolb = 4e-2 if dtype == torch.bfloat16 else 1e-4
    assert rel_err(dq, qf.grad) < tolb
    assert rel_err(dk, kf.grad) < tolb
    assert rel_err(dv, vf.grad) < tolb


@pytest.mark.parametrize("B,H,Lq,Lk,causal", [(1, 8, 1100, 1100, False), (2, 3, 200, 333, False),
                                              (2, 2, 130, 130, True), (3, 2, 17, 70, False)])
def test_attention_f32_mfma_matches_wave_kernel(monkeypatch, B, H, Lq, Lk, causal):
    """The fp32 flash forward on the fp32 MFMA (parity-mode prefill) against
    the wave-per-query kernel and fp32 torch, incl. a fully padded sequence
    (O = 0, lse = +inf) and ragged tiles."""
    O = ops()
    D = 64
    q = torch.randn(B * Lq, H * D, device=dev) * 2
    kv = torch.randn(B * Lk, 2 * H * D, device=dev)
    k, v = kv[:, : H * D], kv[:, H * D:]
    kpm = torch.zeros(B, Lk, device=dev, dtype=torch.uint8)
    kpm[0, Lk - Lk // 4:] = 1
    if B > 1:
        kpm[-1] = 1  # a sequence with no visible key
    scale = 1.0 / math.sqrt(D)
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("SMER_ATTN_F32_MFMA", flag)
        o = torch.empty(B * Lq, H * D, device=dev)
        lse = torch.empty(B, H, Lq, device=dev)
        O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, kpm=kpm, causal=causal, scale=scale)
        torch.cuda.synchronize()
        outs[flag] = (o, lse)
    o, lse = outs["1"]
    # reference on the sequences with visible keys
    nb = B - 1 if B > 1 else B
    ro, rlse = attn_ref(q[: nb * Lq], k[: nb * Lk], v[: nb * Lk], nb, H, Lq, Lk, D, kpm[:nb], causal, scale)
    assert rel_err(o[: nb * Lq], ro) < 2e-5
    assert (lse[:nb] - rlse).abs().max().item() < 1e-4
    assert rel_err(o, outs["0"][0]) < 2e-5
    if B > 1:
        assert torch.all(o[nb * Lq:] == 0) and torch.all(torch.isinf(lse[nb:]))
        assert torch.all(outs["0"][0][nb * Lq:] == 0)


@pytest.mark.parametrize("D", [32, 64])
def test_attention_padded_keys_with_huge_scores(D):
    """Padded keys whose raw scores dwarf the valid ones: they must not leak
    into O (forward) nor produce inf/NaN in dK/dV (their rows are zero)."""
    O = ops()
    B, H, L = 2, 2, 128
    q, k, v, kpm = _attn_inputs(B, H, L, L, D, torch.bfloat16, True)
    k = k.clone()
    pad = kpm.bool().view(B, L).repeat_interleave(1, 0)
    kk = k.view(B, L, H * D)
    kk[pad] = (q.view(B, L, H * D)[pad].float() * 60.0).to(torch.bfloat16)
    o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=False, scale=0.125)
    do = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(k)
    O.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=False,
               scale=0.125, drop_p=0.1, seed=3)
    torch.cuda.synchronize()
    for t in (o, dq, dk, dv):
        assert torch.isfinite(t.float()).all()
    assert (dk.view(B, L, -1)[pad] == 0).all() and (dv.view(B, L, -1)[pad] == 0).all()
    qf, kf, vf = (t.float() for t in (q, k, v))
    ro, _ = attn_ref(qf, kf, vf, B, H, L, L, D, kpm, False, 0.125)
    assert rel_err(o, ro) < 2e-2


def _ramped_keys(q, k, B, H, L, D, ramp, top):
    """Key norms ramping over the key tiles (see the test below)."""
    g = torch.linspace(0.2, top, L, device=dev)
    if ramp == "down":
        g = g.flip(0)
    gk = g.view(1, L, 1, 1).expand(B, L, H, 1).clone()
    if ramp == "mixed":
        gk[:, :, 1::2] = g.flip(0).view(1, L, 1, 1)
    return (k.float().view(B, L, H, D) * gk).view(B * L, H * D).to(torch.bfloat16)


@pytest.mark.parametrize("D", [32, 64])
@pytest.mark.parametrize("ramp", ["up", "down", "mixed"])
@pytest.mark.parametrize("causal", [False, True])
def test_attention_deferred_max_rescale(D, ramp, causal):
    """The bf16 forward keeps a per-query reference max and rescales only
    when a tile's scores pass it by more than 2^8 (or on a query's first
    key).  N(0, 1) scores never take that branch after the first tile, so
    the key norms ramp across the 5 (ragged) key tiles: 'up' raises every
    query's max tile after tile, 'down' never moves it after the first,
    'mixed' flips the ramp per head so some rows rescale while their wave
    neighbours do not.
    (1) Moderate ramp (scores to ~17 in log2 units): forward and backward
        against the fp32 reference at the usual bf16 tolerances.
    (2) Steep ramp (scores to ~70): the forward against fp32 math on the
        operands the kernel actually multiplies -- Q pre-scaled by
        scale * log2(e) and rounded to bf16 (one extra rounding of Q, whose
        effect grows with |score|: 0.1 in lse at these scores) -- so that
        only the rescale bookkeeping is under test."""
    O = ops()
    B, H, L = 2, 4, 300
    torch.manual_seed(5)
    q, k0, v, kpm = _attn_inputs(B, H, L, L, D, torch.bfloat16, True)
    scale = 1.0 / math.sqrt(D)
    for top, qmul in ((3.0, 1.0), (5.0, 2.0)):
        k = _ramped_keys(q, k0, B, H, L, D, ramp, top)
        qq = (q.float() * qmul).to(torch.bfloat16)
        o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B, H, L, device=dev)
        O.attn_fwd(qq, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=causal, scale=scale)
        if top == 3.0:
            qf, kf, vf = (t.float().clone().requires_grad_(True) for t in (qq, k, v))
            ro, rlse = attn_ref(qf, kf, vf, B, H, L, L, D, kpm, causal, scale)
            torch.cuda.synchronize()
            assert rel_err(o, ro) < 2e-2
            assert (lse - rlse).abs().max().item() < 2e-2
            do = torch.randn(B * L, H * D, device=dev).to(torch.bfloat16)
            ro.backward(do.float())
            dq, dk, dv = torch.empty_like(qq), torch.empty_like(k), torch.empty_like(k)
            O.attn_bwd(qq, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm,
                       causal=causal, scale=scale)
            torch.cuda.synchronize()
            for a, b in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
                assert rel_err(a, b) < 4e-2
        else:
            c32 = torch.tensor(scale, dtype=torch.float32) * torch.tensor(1.4426950408889634,
                                                                          dtype=torch.float32)
            qc = (qq.float() * c32.item()).to(torch.bfloat16)
            q_eff = qc.float() * (math.log(2.0) / scale)
            ro, rlse = attn_ref(q_eff, k.float(), v.float(), B, H, L, L, D, kpm, causal, scale)
            torch.cuda.synchronize()
            assert torch.isfinite(o.float()).all()
            assert rel_err(o, ro) < 2e-2
            assert (lse - rlse).abs().max().item() < 2e-2


@pytest.mark.parametrize("causal", [False, True])
def test_attention_first_keys_far_below(causal):
    """Every query's first key tile scores far below zero (|s| * log2(e) of
    several hundred, as large un-normalised activations give) and later
    tiles above it: the first reference max then sits far below the
    initial one, and nothing may overflow on the way (no NaN / inf)."""
    O = ops()
    B, H, L, D = 2, 2, 200, 64
    torch.manual_seed(11)
    u = torch.randn(1, H * D, device=dev)
    q = (u * 6.0 + torch.randn(B * L, H * D, device=dev)).to(torch.bfloat16)
    k = torch.randn(B * L, H * D, device=dev)
    kv = k.view(B, L, H * D)
    kv[:, :64] = -u * 6.0 + 0.5 * kv[:, :64]
    k = k.to(torch.bfloat16)
    v = torch.randn(B * L, H * D, device=dev).to(torch.bfloat16)
    scale = 0.125
    o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, causal=causal, scale=scale)
    c32 = torch.tensor(scale, dtype=torch.float32) * torch.tensor(1.4426950408889634, dtype=torch.float32)
    q_eff = (q.float() * c32.item()).to(torch.bfloat16).float() * (math.log(2.0) / scale)
    ro, rlse = attn_ref(q_eff, k.float(), v.float(), B, H, L, L, D, None, causal, scale)
    torch.cuda.synchronize()
    assert torch.isfinite(o.float()).all() and torch.isfinite(lse).all()
    assert rel_err(o, ro) < 2e-2
    assert (lse - rlse).abs().max().item() < 2e-2
    do = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(k)
    O.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, causal=causal, scale=scale)
    torch.cuda.synchronize()
    for t in (dq, dk, dv):
        assert torch.isfinite(t.float()).all()


@pytest.mark.parametrize("qg2", [False, True])
def test_attention_fwd_e4m3_copy(qg2):
    """smer_attn_fwd_fp8: O and lse are the plain forward's bit for bit, the
    copy is e4m3(o * qs) (nearest-even, saturated), amax = max|o|."""
    O = ops()
    B, H, L, D = (16, 8, 512, 64) if qg2 else (2, 3, 200, 64)
    q, k, v, kpm = _attn_inputs(B, H, L, L, D, torch.bfloat16, True)
    o0 = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
    lse0 = torch.empty(B, H, L, device=dev)
    O.attn_fwd(q, k, v, o0, lse0, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, scale=0.125, drop_p=0.1, seed=9)
    o, lse = torch.empty_like(o0), torch.empty_like(lse0)
    o8 = torch.zeros(B * L, H * D, device=dev, dtype=torch.uint8)
    qs = torch.tensor([150.0], device=dev)
    amax = torch.zeros(1, dtype=torch.int32, device=dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, scale=0.125, drop_p=0.1, seed=9,
               q8=(o8, qs, amax))
    torch.cuda.synchronize()
    assert torch.equal(o, o0) and torch.equal(lse, lse0)
    want = (o.float() * 150.0).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(o8, want)
    assert amax.view(torch.float32).item() == o.float().abs().max().item()


@pytest.mark.parametrize("kg2", [False, True])
def test_attention_bwd_e4m3_copies(kg2):
    """smer_attn_bwd_fp8: the bf16 gradients are the plain backward's bit for
    bit, the e4m3 copies are e4m3(g * qs) of them (nearest-even, saturated),
    and amax holds max|g| over the three gradients (float bits)."""
    O = ops()
    B, H, L, D = (16, 8, 512, 64) if kg2 else (2, 3, 200, 64)
    q, k, v, kpm = _attn_inputs(B, H, L, L, D, torch.bfloat16, True)
    o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, scale=0.125)
    do = torch.randn_like(o)
    ref = [torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16) for _ in range(3)]
    O.attn_bwd(q, k, v, o, do, lse, *ref, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, scale=0.125,
               drop_p=0.1, seed=5)
    got = torch.empty(B * L, 3 * H * D, device=dev, dtype=torch.bfloat16)
    q8 = torch.zeros(B * L, 3 * H * D, device=dev, dtype=torch.uint8)
    qs = torch.tensor([37.0], device=dev)
    amax = torch.zeros(1, dtype=torch.int32, device=dev)
    hd = H * D
    O.attn_bwd(q, k, v, o, do, lse, got[:, :hd], got[:, hd:2 * hd], got[:, 2 * hd:], B=B, H=H, Lq=L,
               Lk=L, D=D, kpm=kpm, scale=0.125, drop_p=0.1, seed=5,
               q8=(q8[:, :hd], q8[:, hd:2 * hd], q8[:, 2 * hd:], qs, amax))
    torch.cuda.synchronize()
    for j in range(3):
        g = got[:, j * hd:(j + 1) * hd]
        assert torch.equal(g, ref[j])
        want = (g.float() * 37.0).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(q8[:, j * hd:(j + 1) * hd], want)
    m = max(t.float().abs().max().item() for t in ref)
    assert amax.view(torch.float32).item() == m
    # no bf16 gradients (the fp8 step's dQKV when both its consumers read the
    # copies): the same copies and amax alone
    q8b = torch.zeros_like(q8)
    amb = torch.zeros(1, dtype=torch.int32, device=dev)
    O.attn_bwd(q, k, v, o, do, lse, None, None, None, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, scale=0.125,
               drop_p=0.1, seed=5, q8=(q8b[:, :hd], q8b[:, hd:2 * hd], q8b[:, 2 * hd:], qs, amb))
    torch.cuda.synchronize()
    assert torch.equal(q8b, q8) and torch.equal(amb, amax)


@pytest.mark.parametrize("dtype,B,H,L,causal", [(torch.bfloat16, 2, 2, 96, True),
                                                 (torch.float32, 2, 2, 96, True),
                                                 (torch.bfloat16, 16, 8, 512, False),
                                                 (torch.bfloat16, 16, 8, 512, True)])
def test_attention_dropout(dtype, B, H, L, causal):
    """Dropout mask = tests/hashref.attn_keep_mask; the large shapes take the
    two-query-group forward (>= 512 workgroups)."""
    O = ops()
    D = 64
    p, seed = 0.1, 77
    q, k, v, kpm = _attn_inputs(B, H, L, L, D, dtype, True)
    scale = 0.125
    keep = torch.from_numpy(attn_keep_mask(seed, p, B * H * L, L)).to(dev).view(B, H, L, L)
    o = torch.empty(B * L, H * D, device=dev, dtype=dtype)
    lse = torch.empty(B, H, L, device=dev)
    mask = O.attn_drop_mask(B, H, L, L, dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=causal, scale=scale,
               drop_p=p, seed=seed, drop_mask=mask)
    qf, kf, vf = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    ro, _ = attn_ref(qf, kf, vf, B, H, L, L, D, kpm, causal, scale, keep, p)
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 2e-5
    assert rel_err(o, ro) < tol
    do = torch.randn(B * L, H * D, device=dev).to(dtype)
    ro.backward(do.float())
    dq = torch.empty_like(q)
    dk = torch.empty_like(k.contiguous())
    dv = torch.empty_like(dk)
    O.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=causal,
               scale=scale, drop_p=p, seed=seed)
    torch.cuda.synchronize()
    tolb = 4e-2 if dtype == torch.bfloat16 else 1e-4
    for a, b in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert rel_err(a, b) < tolb
    if dtype == torch.bfloat16:
        # backward reading the forward's stored keep bits == re-hashing
        dq2, dk2, dv2 = torch.empty_like(dq), torch.empty_like(dk), torch.empty_like(dv)
        O.attn_bwd(q, k, v, o, do, lse, dq2, dk2, dv2, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm,
                   causal=causal, scale=scale, drop_p=p, seed=seed, drop_mask=mask)
        torch.cuda.synchronize()
        assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)
        # forward reading keep bits the caller generated beforehand ==
        # forward with a mask buffer it fills itself == forward hashing them
        # in its loop (no buffer): same keep decisions, outputs bit for bit
        mask3 = O.attn_drop_mask(B, H, L, L, dev)
        O.attn_drop_mask_gen(mask3, B=B, H=H, Lq=L, Lk=L, drop_p=p, seed=seed)
        o3 = torch.empty_like(o)
        lse3 = torch.empty_like(lse)
        O.attn_fwd(q, k, v, o3, lse3, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=causal,
                   scale=scale, drop_p=p, seed=seed, drop_mask=mask3, drop_mask_in=True)
        o4 = torch.empty_like(o)
        lse4 = torch.empty_like(lse)
        O.attn_fwd(q, k, v, o4, lse4, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm, causal=causal,
                   scale=scale, drop_p=p, seed=seed)
        torch.cuda.synchronize()
        if not causal:  # (a causal forward skips the tiles past the diagonal)
            assert torch.equal(mask3, mask)
        assert torch.equal(o4, o) and torch.equal(lse4, lse)
        dq3, dk3, dv3 = torch.empty_like(dq), torch.empty_like(dk), torch.empty_like(dv)
        O.attn_bwd(q, k, v, o3, do, lse3, dq3, dk3, dv3, B=B, H=H, Lq=L, Lk=L, D=D, kpm=kpm,
                   causal=causal, scale=scale, drop_p=p, seed=seed, drop_mask=mask3)
        torch.cuda.synchronize()
        assert torch.equal(o3, o) and torch.equal(lse3, lse)
        assert torch.equal(dq3, dq) and torch.equal(dk3, dk) and torch.equal(dv3, dv)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_attention_weights(dtype):
    O = ops()
    B, H, Lq, Lk, D = 2, 4, 40, 72, 32
    q, k, v, kpm = _attn_inputs(B, H, Lq, Lk, D, dtype, True)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=dtype)
    lse = torch.empty(B, H, Lq, device=dev)
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, kpm=kpm, scale=0.2)
    w = torch.empty(B, Lq, Lk, device=dev)
    O.attn_weights(q, k, lse, w, B=B, H=H, Lq=Lq, Lk=Lk, D=D, kpm=kpm, scale=0.2)
    qh = q.float().view(B, Lq, H, D).transpose(1, 2)
    kh = k.float().view(B, Lk, H, D).transpose(1, 2)
    s = (qh @ kh.transpose(-1, -2)) * 0.2
    s = s.masked_fill(kpm.bool().view(B, 1, 1, Lk), float("-inf"))
    ref = torch.softmax(s, -1).mean(1)
    torch.cuda.synchronize()
    assert (w - ref).abs().max().item() < (1e-2 if dtype == torch.bfloat16 else 1e-6)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("D", [64, 32, 128, 24])
@pytest.mark.parametrize("cap", [1000, 300])
def test_decode_attention(dtype, D, cap):
    """Vectorised online-softmax kernel (D = 32/64/128; 8-wave x 4-step
    config for long caches, 4 x 2 for short) and the generic fallback
    (D = 24)."""
    O = ops()
    H, R = 4, 3
    d = H * D
    kc = torch.randn(R, cap, d, device=dev).to(dtype)
    vc = torch.randn(R, cap, d, device=dev).to(dtype)
    q = torch.randn(5, d, device=dev).to(dtype)
    row_req = torch.tensor([0, 1, 1, 2, 2], dtype=torch.int32, device=dev)
    nkeys = torch.tensor([1, 17, 18, cap, 64], dtype=torch.int32, device=dev)
    out = torch.empty(5, d, device=dev, dtype=dtype)
    O.attn_decode(q, kc, vc, row_req, nkeys, out, H=H, D=D, row_stride=d, req_stride=cap * d,
                  scale=0.125)
    torch.cuda.synchronize()
    for i in range(5):
        r, n = int(row_req[i]), int(nkeys[i])
        qh = q[i].float().view(H, 1, D)
        kh = kc[r, :n].float().view(n, H, D).transpose(0, 1)
        vh = vc[r, :n].float().view(n, H, D).transpose(0, 1)
        ref = (torch.softmax(qh @ kh.transpose(-1, -2) * 0.125, -1) @ vh).reshape(d)
        assert rel_err(out[i], ref) < (1e-2 if dtype == torch.bfloat16 else 1e-5)
    # head-major layout [R][H][cap][D] (the decode cross-attention memory),
    # filled by kv_scatter_heads from [K heads | V heads] rows
    kvh = torch.zeros(R, 2, H, cap, D, device=dev, dtype=dtype)
    rows = torch.cat([kc.view(R * cap, d), vc.view(R * cap, d)], 1).contiguous()
    rr = torch.arange(R * cap, device=dev, dtype=torch.int32) // cap
    pp = torch.arange(R * cap, device=dev, dtype=torch.int32) % cap
    if D % (8 if dtype == torch.bfloat16 else 4) == 0:
        O.kv_scatter_heads(rows, kvh, rr, pp, H=H, D=D, req_stride=2 * H * cap * D,
                           kv_stride=H * cap * D, head_stride=cap * D)
        torch.cuda.synchronize()
        assert torch.equal(kvh[:, 0].permute(0, 2, 1, 3).reshape(R, cap, d), kc)
        assert torch.equal(kvh[:, 1].permute(0, 2, 1, 3).reshape(R, cap, d), vc)
    else:
        kvh[:, 0] = kc.view(R, cap, H, D).permute(0, 2, 1, 3)
        kvh[:, 1] = vc.view(R, cap, H, D).permute(0, 2, 1, 3)
    out2 = torch.empty_like(out)
    O.attn_decode(q, kvh, kvh.view(-1)[H * cap * D:], row_req, nkeys, out2, H=H, D=D, row_stride=D,
                  req_stride=2 * H * cap * D, head_stride=cap * D, scale=0.125)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)
    # scatter
    src = torch.randn(2, d, device=dev).to(dtype)
    O.kv_scatter(src, kc, torch.tensor([2, 0], dtype=torch.int32, device=dev),
                 torch.tensor([5, cap - 1], dtype=torch.int32, device=dev), row_stride=d,
                 req_stride=cap * d)
    torch.cuda.synchronize()
    assert torch.equal(kc[2, 5], src[0]) and torch.equal(kc[0, cap - 1], src[1])


# ------------------------------------------------------------ layernorm
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
# bf16 forward: 4 rows per wave below 16384 rows (partial last workgroups), 1 above
@pytest.mark.parametrize("M,N", [(300, 512), (64, 768), (37, 64), (16387, 512), (16400, 768),
                                 (16390, 1536)])
def test_layernorm(dtype, M, N):
    O = ops()
    x = (torch.randn(M, N, device=dev) * 3 + 1).to(dtype)
    g = torch.randn(N, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    O.layernorm(x, g, b, y, mean, rstd)
    xf = x.float().clone().requires_grad_(True)
    gf, bf = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(xf, (N,), gf, bf, 1e-5)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < (1e-2 if dtype == torch.bfloat16 else 2e-6)
    dy = torch.randn(M, N, device=dev).to(dtype)
    ref.backward(dy.float())
    dx = torch.empty_like(x)
    dxd = torch.empty_like(x)
    dg = torch.zeros(N, device=dev)
    db = torch.zeros(N, device=dev)
    p, seed = 0.2, 99
    O.layernorm_bwd(dy, x, mean, rstd, g, dx, dx_drop=dxd, drop_p=p, seed=seed, dgamma=dg,
                    dbeta=db)
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert rel_err(dx, xf.grad) < tol
    keep = torch.from_numpy(keep_mask(seed, p, M, N)).to(dev)
    assert rel_err(dxd, torch.where(keep, xf.grad * drop_scale(p), torch.zeros_like(xf.grad))) < tol
    assert rel_err(dg, gf.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-5)
    assert rel_err(db, bf.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-5)


# -------------------------------------------------------------- embedding
@pytest.mark.parametrize("d", [128, 768])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding(dtype, d):
    O = ops()
    V, B, L = 309, 3, 50
    table = torch.randn(V, d, device=dev)
    pe = torch.randn(2400, d, device=dev)
    ids = torch.randint(0, V, (B, L), device=dev)
    ids[0, :20] = 7  # hot token
    out = torch.empty(B * L, d, device=dev, dtype=dtype)
    p, seed = 0.1, 5
    O.embed(ids, table, pe, out, L=L, scale=math.sqrt(d), drop_p=p, seed=seed)
    keep = torch.from_numpy(keep_mask(seed, p, B * L, d)).to(dev)
    pos = torch.arange(B * L, device=dev) % L
    ref = table[ids.view(-1)] * math.sqrt(d) + pe[pos]
    ref = torch.where(keep, ref * drop_scale(p), torch.zeros_like(ref))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < (1e-2 if dtype == torch.bfloat16 else 1e-6)
    ids2 = torch.randint(0, V, (2, 30), device=dev)
    dx0 = torch.randn(B * L, d, device=dev).to(dtype)
    dx1 = torch.randn(60, d, device=dev).to(dtype)
    dt = torch.zeros(V, d, device=dev)
    O.embed_bwd(dt, math.sqrt(d), [(ids.view(-1), dx0, p, seed), (ids2.view(-1), dx1, 0.0, 0)])
    ref = torch.zeros(V, d, device=dev)
    g0 = torch.where(keep, dx0.float() * drop_scale(p), torch.zeros_like(dx0.float()))
    ref.index_add_(0, ids.view(-1), g0)
    ref.index_add_(0, ids2.view(-1), dx1.float())
    ref *= math.sqrt(d)
    torch.cuda.synchronize()
    assert rel_err(dt, ref) < 1e-5


# ------------------------------------------------------------ loss / adam
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_weighted_ce(dtype):
    O = ops()
    R, V = 333, 309
    logits = torch.randn(R, V, device=dev) * 3
    y = torch.randint(0, V, (R,), device=dev)
    y[:10] = 0
    w = torch.rand(V, device=dev)
    w[0] = 0
    ce_all = torch.rand(V, device=dev)
    denom = torch.empty(1, device=dev)
    O.wce_denom(y, ce_all, denom)
    row = torch.empty(R, device=dev)
    loss = torch.empty(1, device=dev)
    dl = torch.empty(R, 320, device=dev, dtype=dtype)
    O.wce_fwd_bwd(logits, y, w, denom, row, loss, dl, V=V)
    lf = logits.clone().requires_grad_(True)
    ref_denom = ce_all[y].sum()
    ref = torch.nn.functional.cross_entropy(lf, y, weight=w, ignore_index=0, reduction="none")
    ref_loss = ref.sum() / ref_denom
    ref_loss.backward()
    torch.cuda.synchronize()
    assert abs(denom.item() - ref_denom.item()) < 1e-4
    assert abs(loss.item() - ref_loss.item()) < 1e-5 * max(1, abs(ref_loss.item()))
    assert rel_err(dl[:, :V], lf.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-5)


def test_adam_and_cast_and_colsum():
    O = ops()
    n = 100003
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    m = torch.randn(n, device=dev) * 0.1
    v = torch.rand(n, device=dev) * 0.1
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    O.adam(p, g, m, v, pb, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, step=3)
    mr.lerp_(g, 0.1)
    vr.mul_(0.999).addcmul_(g, g, value=0.001)
    bc1, bc2 = 1 - 0.9 ** 3, 1 - 0.999 ** 3
    pr.addcdiv_(mr, (vr.sqrt() / math.sqrt(bc2)).add_(1e-8), value=-1e-3 / bc1)
    torch.cuda.synchronize()
    assert (p - pr).abs().max().item() < 1e-6
    assert torch.equal(pb, p.to(torch.bfloat16))
    x = torch.randn(1000, 309, device=dev)
    out = torch.ones(309, device=dev)
    O.colsum(x, out, accumulate=True)
    torch.cuda.synchronize()
    assert (out - (1 + x.sum(0))).abs().max().item() < 1e-3
    xb = torch.empty(1000, 309, device=dev, dtype=torch.bfloat16)
    O.cast(x, xb)
    torch.cuda.synchronize()
    assert torch.equal(xb, x.to(torch.bfloat16))


@pytest.mark.parametrize("B,H,Lq,Lk,causal", [(2, 2, 96, 96, True), (2, 2, 80, 150, False),
                                              (16, 8, 512, 512, False)])
def test_attention_drop_mask_layout(B, H, Lq, Lk, causal):
    """The keep bits a forward with a mask buffer leaves for the backward
    (generated by attn_drop_mask_gen_kernel) equal tests/hashref.
    attn_keep_mask: u32 words [bh][q32][key tile t][lane = 16G + c], bit
    8R + 4gq + mt = (query 32*q32 + 16*gq + c, key 64t + 16mt + 4G + R)."""
    O = ops()
    D, p, seed = 64, 0.1, 99
    q, k, v, _ = _attn_inputs(B, H, Lq, Lk, D, torch.bfloat16, False)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, Lq, device=dev)
    mask = O.attn_drop_mask(B, H, Lq, Lk, dev)
    mask.zero_()
    O.attn_fwd(q, k, v, o, lse, B=B, H=H, Lq=Lq, Lk=Lk, D=D, causal=causal, scale=0.125,
               drop_p=p, seed=seed, drop_mask=mask)
    torch.cuda.synchronize()
    nq, nt = (Lq + 31) // 32, (Lk + 63) // 64
    w = mask[: B * H * nq * nt * 256].cpu().numpy().view(np.uint32).reshape(B * H, nq, nt, 4, 16)
    bits = (w[..., None] >> np.arange(32, dtype=np.uint32)) & 1          # [bh, q32, t, G, c, 32]
    bits = bits.reshape(B * H, nq, nt, 4, 16, 4, 2, 4)                   # [.., G, c, R, gq, mt]
    got = bits.transpose(0, 1, 6, 4, 2, 7, 3, 5).reshape(B * H, nq * 32, nt * 64)  # [bh, q, key]
    ref = attn_keep_mask(seed, p, B * H * Lq, Lk).reshape(B * H, Lq, Lk)
    sel = np.ones((Lq, Lk), bool) if not causal else np.tril(np.ones((Lq, Lk), bool))
    g = got[:, :Lq, :Lk].astype(bool)
    assert (g[:, sel] == ref[:, sel]).all()


# ------------------------------------------------------------ decode linear
@pytest.mark.parametrize("M,N,K", [(64, 1536, 512), (128, 512, 2048), (40, 264, 512),
                                   (256, 264, 1024)])
def test_linear_decode_kv_scatter(M, N, K):
    """Decode Linear: bias, ReLU, residual, and the K/V scatter of the
    output columns >= kv_col0 into a per-request cache."""
    O = ops()
    bf = torch.bfloat16
    x = torch.randn(M, K, device=dev).to(bf)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(bf)
    b = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(bf)
    col0 = (N // 3) // 8 * 8
    R = 5
    T = M // R + 1
    cache = torch.zeros(R, T, N - col0, device=dev, dtype=bf)
    req = torch.arange(M, device=dev, dtype=torch.int32) % R
    pos = torch.arange(M, device=dev, dtype=torch.int32) // R
    out = O.linear_decode(x, w, b, relu=True, residual=res, kv=cache, kv_req=req, kv_pos=pos,
                          kv_row_stride=N - col0, kv_req_stride=T * (N - col0), kv_col0=col0)
    ref = torch.relu(x.float() @ w.float().t() + b) + res.float()
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 2e-2
    assert torch.equal(cache[req.long(), pos.long()], out[:, col0:])


@pytest.mark.parametrize("M,N,K", [(64, 512, 512), (37, 309, 512), (128, 2048, 512), (16, 1536, 512),
                                   (24, 512, 2048)])
def test_linear_decode_ln_is_layernorm_then_linear(M, N, K):
    """The LayerNorm-prologue decode Linear == ops.layernorm then
    ops.linear_decode, bit for bit (stored LN output, GEMM output, K/V
    append), incl. ragged M / N and the fp32 logits head."""
    O = ops()
    bf = torch.bfloat16
    y = (torch.randn(M, K, device=dev) * 2 + 0.5).to(bf)
    g = torch.randn(K, device=dev)
    be = torch.randn(K, device=dev)
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(bf)
    b = torch.randn(N, device=dev)
    xln = torch.empty_like(y)
    O.layernorm(y, g, be, xln, torch.empty(M, device=dev), torch.empty(M, device=dev))
    x_out = torch.empty_like(y)
    col0 = (N // 3) // 8 * 8
    wk = (N - col0 + 7) // 8 * 8  # cache row stride (multiple of 8)
    R, T = 5, M // 5 + 1
    c1 = torch.zeros(R, T, wk, device=dev, dtype=bf)
    c2 = torch.zeros_like(c1)
    req = torch.arange(M, device=dev, dtype=torch.int32) % R
    pos = torch.arange(M, device=dev, dtype=torch.int32) // R
    kv = dict(kv_req=req, kv_pos=pos, kv_row_stride=wk, kv_req_stride=T * wk, kv_col0=col0)
    ref = O.linear_decode(xln, w, b, relu=True, kv=c1, **kv)
    got = O.linear_decode_ln(y, g, be, w, b, relu=True, x_out=x_out, kv=c2, **kv)
    lf_ref = O.linear_decode(xln, w, b, out_f32=torch.empty(M, N, device=dev))
    lf_got = O.linear_decode_ln(y, g, be, w, b, out_f32=torch.empty(M, N, device=dev))
    torch.cuda.synchronize()
    assert torch.equal(x_out, xln)
    assert torch.equal(got, ref)
    assert torch.equal(c2, c1)
    assert torch.equal(lf_got, lf_ref)


@pytest.mark.parametrize("M,N,K", [(2, 1536, 512), (2, 309, 512), (4, 2048, 512), (37, 512, 768),
                                   (64, 264, 2048)])
def test_linear_decode_f32_ln_and_kv(M, N, K):
    """fp32 decode Linears (the parity-mode decode step): the LayerNorm
    prologue stores the fp32 LayerNorm kernel's bits, the product matches
    fp32 torch, the K/V append equals the output columns."""
    O = ops()
    y = torch.randn(M, K, device=dev) * 2 + 0.5
    g, be = torch.randn(K, device=dev), torch.randn(K, device=dev)
    w = torch.randn(N, K, device=dev) / math.sqrt(K)
    b = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    xln = torch.empty_like(y)
    O.layernorm(y, g, be, xln, torch.empty(M, device=dev), torch.empty(M, device=dev))
    col0 = N // 3
    R, T = 3, M // 3 + 1
    cache = torch.zeros(R, T, N - col0, device=dev)
    req = torch.arange(M, device=dev, dtype=torch.int32) % R
    pos = torch.arange(M, device=dev, dtype=torch.int32) // R
    x_out = torch.empty_like(y)
    got = O.linear_decode_ln(y, g, be, w, b, relu=True, x_out=x_out, kv=cache, kv_req=req, kv_pos=pos,
                             kv_row_stride=N - col0, kv_req_stride=T * (N - col0), kv_col0=col0)
    lin = O.linear_decode(xln, w, b, residual=res)
    torch.cuda.synchronize()
    assert torch.equal(x_out, xln)
    ref = torch.relu(xln @ w.t() + b)
    assert rel_err(got, ref) < 1e-5
    assert torch.equal(cache[req.long(), pos.long()], got[:, col0:])
    assert rel_err(lin, xln @ w.t() + b + res) < 1e-5


@pytest.mark.parametrize("S,dm", [(300, 512), (2100, 512), (700, 768)])
def test_attn_decode_qln_is_ln_linear_attention(S, dm):
    """Decode cross attention with LN + query projection in its blocks ==
    LayerNorm -> Linear -> smer_attn_decode: the stored LN output bit for bit,
    the attention output within bf16 rounding of the query (the fused
    projection sums in a different order), incl. the pipelined long-memory
    variant and ragged key counts."""
    O = ops()
    bf = torch.bfloat16
    H, D = dm // 64, 64
    R, M = 5, 10
    y = (torch.randn(M, dm, device=dev) * 2).to(bf)
    g, be = torch.randn(dm, device=dev), torch.randn(dm, device=dev)
    wq = (torch.randn(dm, dm, device=dev) / math.sqrt(dm)).to(bf)
    bq = torch.randn(dm, device=dev) * 0.1
    cache = torch.randn(R, 2, H, S, D, device=dev).to(bf)
    req = (torch.arange(M, device=dev, dtype=torch.int32) // 2) % R
    nk = torch.tensor([1, S, 17, S - 3, 1, 64, S // 2, 5, 1, S], device=dev, dtype=torch.int32)
    kw = dict(H=H, D=D, row_stride=D, req_stride=2 * H * S * D, head_stride=S * D, scale=0.125)
    xln = torch.empty_like(y)
    O.layernorm(y, g, be, xln, torch.empty(M, device=dev), torch.empty(M, device=dev))
    q = O.linear_decode(xln, wq, bq)
    ref = torch.empty(M, dm, device=dev, dtype=bf)
    O.attn_decode(q, cache, cache.view(-1)[H * S * D:], req, nk, ref, **kw)
    got = torch.empty_like(ref)
    x_out = torch.empty_like(y)
    O.attn_decode_qln(y, g, be, wq, bq, cache, cache.view(-1)[H * S * D:], req, nk, got, x_out=x_out, **kw)
    torch.cuda.synchronize()
    assert torch.equal(x_out, xln)
    assert rel_err(got, ref) < 2e-2, rel_err(got, ref)


@pytest.mark.parametrize("S,M", [(1100, 2), (300, 6), (40, 2), (2500, 4)])
def test_attn_decode_split_f32_merge(S, M):
    """fp32 flash-decoding (8 key slices per (row, head), partials merged in
    the out-projection's prologue) == smer_attn_decode then the Linear
    (+bias, +residual), incl. rows with 1 key and slices with no key."""
    O = ops()
    H, D, dm, R = 8, 64, 512, 3
    cache = torch.randn(R, 2, H, S, D, device=dev)
    q = torch.randn(M, dm, device=dev)
    req = torch.arange(M, device=dev, dtype=torch.int32) % R
    nk = torch.tensor([S, 1, S // 3, 5, S - 1, 2][:M], device=dev, dtype=torch.int32)
    kw = dict(H=H, D=D, row_stride=D, req_stride=2 * H * S * D, head_stride=S * D, scale=0.125)
    o = torch.empty(M, dm, device=dev)
    O.attn_decode(q, cache, cache.view(-1)[H * S * D:], req, nk, o, **kw)
    w = torch.randn(dm, dm, device=dev) / math.sqrt(dm)
    b, res = torch.randn(dm, device=dev), torch.randn(M, dm, device=dev)
    ref = O.linear(o, w, b, residual=res)
    part = torch.empty(M, H, O.DEC_SPLITS, 68, device=dev)
    O.attn_decode_split_f32(q, cache, cache.view(-1)[H * S * D:], req, nk, part, **kw)
    got = O.linear_decode_merge_f32(part, w, b, M=M, residual=res)
    torch.cuda.synchronize()
    assert rel_err(got, ref) < 1e-5, rel_err(got, ref)


@pytest.mark.parametrize("S,M", [(1100, 2), (40, 2), (2500, 4)])
def test_attn_decode_split_qln_f32(S, M):
    """fp32 split decode attention with LN + query projection in its blocks
    == smer_linear_decode_ln_f32 (cross Q, x_out) -> split attention -> merge:
    the stored LN output bit for bit (same normalisation arithmetic), the
    merged output within fp32 reordering of the projection's sums; rows with
    1 key (query skipped) and slices with no key."""
    O = ops()
    H, D, dm, R = 8, 64, 512, 3
    cache = torch.randn(R, 2, H, S, D, device=dev)
    y = torch.randn(M, dm, device=dev) * 2 + 0.5
    g, be = torch.randn(dm, device=dev), torch.randn(dm, device=dev)
    wq = torch.randn(dm, dm, device=dev) / math.sqrt(dm)
    bq = torch.randn(dm, device=dev) * 0.1
    req = torch.arange(M, device=dev, dtype=torch.int32) % R
    nk = torch.tensor([S, 1, S // 3, 5][:M], device=dev, dtype=torch.int32)
    kw = dict(H=H, D=D, row_stride=D, req_stride=2 * H * S * D, head_stride=S * D, scale=0.125)
    w = torch.randn(dm, dm, device=dev) / math.sqrt(dm)
    b = torch.randn(dm, device=dev)
    xln = torch.empty_like(y)
    q = O.linear_decode_ln(y, g, be, wq, bq, x_out=xln)
    part = torch.empty(M, H, O.DEC_SPLITS, 68, device=dev)
    O.attn_decode_split_f32(q, cache, cache.view(-1)[H * S * D:], req, nk, part, **kw)
    ref = O.linear_decode_merge_f32(part, w, b, M=M, residual=xln)
    x_out = torch.full_like(y, float("nan"))
    part2 = torch.empty_like(part)
    O.attn_decode_split_qln_f32(y, g, be, wq, bq, cache, cache.view(-1)[H * S * D:], req, nk, part2,
                                x_out=x_out, **kw)
    got = O.linear_decode_merge_f32(part2, w, b, M=M, residual=x_out)
    torch.cuda.synchronize()
    assert torch.equal(x_out, xln)
    assert rel_err(got, ref) < 1e-5, rel_err(got, ref)


# ------------------------------------------------------------ fp8
def _e4m3_ref(x, amax):
    """e4m3 bytes of x * (448 / amax): f32 scale by IEEE division, f32
    product, clamp, torch's CPU float8_e4m3fn cast (nearest-even)."""
    sc = np.float32(448.0) / np.float32(amax)
    y = x.float().cpu().numpy().astype(np.float32) * sc
    return torch.from_numpy(np.clip(y, -448, 448)).to(torch.float8_e4m3fn).view(torch.uint8)


def test_gemm_fp8_exact_integer_layout():
    """fp8 MFMA fragment / output layout with exact small-integer e4m3 data
    and an asymmetric B: the kernel must reproduce A.B^T exactly."""
    O = ops()
    M, N, K = 256, 512, 384
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randint(-4, 5, (M, K), generator=g).float()
    B = torch.randint(-3, 4, (N, K), generator=g).float()
    B[:, 0] += torch.arange(N) % 5  # asymmetric
    a8 = A.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    b8 = B.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    one = torch.ones(1, device=dev)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    assert O.gemm_fp8(a8, one, b8, one, C)
    ref = A.to(torch.float8_e4m3fn).float() @ B.to(torch.float8_e4m3fn).float().t()
    torch.cuda.synchronize()
    assert torch.equal(C.float().cpu(), ref.to(torch.bfloat16).float())


@pytest.mark.parametrize("M,N,K", [(512, 768, 1280), (4608, 4096, 256), (256, 256, 3072)])
def test_gemm256s_fp8_matches_two_stage_kernel(monkeypatch, M, N, K):
    """The staggered fp8 kernel (32x32x64 block-scaled MFMA) against the
    two-stage 16x16x128 one on exact small-integer e4m3 operands: the fp32
    accumulators are exact in both, so every epilogue (scale, bias, ReLU,
    dropout, residual, ReLU gate) must agree bit for bit, and the plain
    product must equal A.B^T.  (4608, 4096) is 288 tiles: the persistent
    path with the next tile's k-steps issued under the epilogue; K = 256 is
    the 4-k-step minimum."""
    O = ops()
    g = torch.Generator(device="cpu").manual_seed(M + K)
    A = torch.randint(-4, 5, (M, K), generator=g).float()
    B = torch.randint(-3, 4, (N, K), generator=g).float()
    B[:, 0] += torch.arange(N) % 5
    a8 = A.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    b8 = B.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    ai = torch.tensor([0.0123], device=dev)
    bi = torch.tensor([0.37], device=dev)
    one = torch.ones(1, device=dev)
    bias = torch.randn(N, generator=g).to(dev)
    res = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    gate = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)

    def run(flag):
        monkeypatch.setenv("SMER_GEMM256S_FP8", flag)
        outs = []
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        assert O.gemm_fp8(a8, one, b8, one, C)
        outs.append(C)
        C = torch.empty_like(C)
        assert O.gemm_fp8(a8, ai, b8, bi, C, bias=bias, relu=True, residual=res, drop_p=0.1, seed=7)
        outs.append(C)
        C = torch.empty_like(C)
        assert O.gemm_fp8_ex(a8, ai, b8, bi, C, gate=gate, gate_scale=1.25)
        outs.append(C)
        torch.cuda.synchronize()
        return [c.cpu() for c in outs]

    new, old = run("1"), run("0")
    ref = (A.to(torch.float8_e4m3fn).float() @ B.to(torch.float8_e4m3fn).float().t()).to(torch.bfloat16)
    assert torch.equal(new[0], ref)
    for a, b in zip(new, old):
        assert torch.equal(a, b)


def test_fp8_quantize_and_gemm():
    """Per-tensor quantisation (amax + scaled e4m3 cast, matching torch's
    float8_e4m3fn rounding) and the scaled fp8 GEMM with the full epilogue
    against fp32."""
    O = ops()
    M, N, K = 512, 768, 768
    x = (torch.randn(M, K, device=dev) * 3).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    x8 = torch.empty(M, K, device=dev, dtype=torch.uint8)
    w8 = torch.empty(N, K, device=dev, dtype=torch.uint8)
    xi = torch.empty(1, device=dev)
    wi = torch.empty(1, device=dev)
    O.fp8_quantize(x, x8, xi)
    O.fp8_quantize(w, w8, wi)
    torch.cuda.synchronize()
    amax = x.float().abs().max()
    assert abs(xi.item() - amax.item() / 448) < 1e-6 * amax.item()
    # reference: the f32 scale by IEEE division (torch's `448 / t` is a
    # reciprocal times 448, 1 ulp off at times), the f32 product, torch's CPU
    # e4m3 cast (nearest-even) of the clamped value
    ref8 = _e4m3_ref(x, amax.item())
    assert torch.equal(x8.cpu(), ref8)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    assert O.gemm_fp8(x8, xi, w8, wi, C, bias=bias, relu=True, residual=res)
    ref = torch.relu(x.float() @ w.float().t() + bias) + res.float()
    torch.cuda.synchronize()
    err = ((C.float() - ref).norm() / ref.norm()).item()
    assert err < 0.05, err
    assert not O.gemm_fp8(x8[:100], xi, w8, wi, C[:100])  # outside the tiling: caller falls back


def test_fp8_quantize_rounds_nearest_even_near_midpoints():
    """amax = 15.75 puts x * (448 / amax) on or next to e4m3 midpoints for
    many bf16 x (1.4765625 * 28.444445 = 42.0 exactly, a tie -> 40; with the
    1-ulp-high scale torch's `448 / t` gives, 42.0000038 -> 44): the scale
    must be the correctly rounded quotient and the cast nearest-even."""
    O = ops()
    M, K = 256, 512
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (torch.randn(M, K, generator=g) * 3).clamp(-15.0, 15.0).to(torch.bfloat16)
    x[0, 0] = 15.75
    xd = x.to(dev)
    x8 = torch.empty(M, K, device=dev, dtype=torch.uint8)
    xi = torch.empty(1, device=dev)
    O.fp8_quantize(xd, x8, xi)
    torch.cuda.synchronize()
    assert torch.equal(x8.cpu(), _e4m3_ref(x, 15.75))


def test_fp8_quantize_segments_matches_per_tensor():
    """The batched per-step weight quantisation == one fp8_quantize per tensor
    (bit-exact bytes and scales), over tensors of different sizes / ranges."""
    O = ops()
    shapes = [(768, 256), (2304, 768), (8, 8), (1536, 768)]
    xs = [(torch.randn(*s, device=dev) * (0.01 + i)).to(torch.bfloat16) for i, s in enumerate(shapes)]
    qs = [torch.empty(s, device=dev, dtype=torch.uint8) for s in shapes]
    seg = torch.tensor([(x.data_ptr(), q.data_ptr(), x.numel()) for x, q in zip(xs, qs)],
                       dtype=torch.int64, device=dev)
    inv = torch.empty(len(xs), device=dev)
    ws = torch.empty(len(xs), device=dev, dtype=torch.int32)
    O.fp8_quantize_segments(seg, ws, inv)
    for k, x in enumerate(xs):
        q1 = torch.empty_like(qs[k])
        i1 = torch.empty(1, device=dev)
        O.fp8_quantize(x, q1, i1)
        torch.cuda.synchronize()
        assert torch.equal(q1, qs[k]), k
        assert i1.item() == inv[k].item(), k


def test_gemm_fp8_q_writes_e4m3_copy_and_amax():
    """The fp8 training forward's FFN1: besides the bf16 output, the e4m3 copy
    q8 = e4m3(out * qs) of the STORED bf16 values and max|out| folded into
    the amax slot (float bits, atomicMax over workgroups)."""
    O = ops()
    M, N, K = 512, 1024, 256
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
    x8 = torch.empty(M, K, device=dev, dtype=torch.uint8)
    w8 = torch.empty(N, K, device=dev, dtype=torch.uint8)
    xi, wi = torch.empty(1, device=dev), torch.empty(1, device=dev)
    O.fp8_quantize(x, x8, xi)
    O.fp8_quantize(w, w8, wi)
    bias = torch.randn(N, device=dev)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    q8 = torch.empty(M, N, device=dev, dtype=torch.uint8)
    qs = torch.full((1,), 37.0, device=dev)
    amax = torch.zeros(1, device=dev, dtype=torch.int32)
    assert O.gemm_fp8_q(x8, xi, w8, wi, C, bias=bias, relu=True, q8=q8, qs=qs, amax=amax)
    torch.cuda.synchronize()
    ref8 = (C.float() * 37.0).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert (ref8 == q8).float().mean().item() > 0.999
    got = amax.view(torch.float32).item()
    assert got == C.float().abs().max().item()
    ref = torch.relu(x.float() @ w.float().t() + bias)
    assert ((C.float() - ref).norm() / ref.norm()).item() < 0.05


@pytest.mark.parametrize("M,N,K,bk", [(1000, 264, 512, True), (8192, 512, 512, False),
                                      (777, 512, 1536, True)])
def test_gemm64_mid_size_epilogues(M, N, K, bk):
    """The 64x128 tile kernel (mid-size M: fewer 128x128 tiles than two per
    CU) with ragged M / N tails: bias + ReLU + dropout + residual, and a
    ReLU-grad gate."""
    O = ops()
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = torch.randn(N, K, device=dev).to(torch.bfloat16)
    Wm = W if bk else W.t().contiguous()
    bias = torch.randn(N, device=dev)
    R = torch.randn(M, N, device=dev).to(torch.bfloat16)
    p, seed = 0.1, 11
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, bias=bias, relu=True, residual=R, drop_p=p,
           seed=seed)
    base = A.float() @ W.float().t()
    keep = torch.from_numpy(keep_mask(seed, p, M, N)).to(dev)
    ref = R.float() + torch.where(keep, torch.relu(base + bias) * drop_scale(p), torch.zeros_like(base))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 2e-2
    O.gemm(A, Wm, M=M, N=N, K=K, b_kcontig=bk, out=C, gate=R, gate_scale=1.5)
    ref = torch.where(R.float() > 0, base * 1.5, torch.zeros_like(base))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 2e-2


@pytest.mark.parametrize("M,N", [(65536, 768), (20000, 1024), (40000, 2048)])
def test_layernorm_bwd_balanced_grid(M, N, monkeypatch):
    """LayerNorm backward at large M and N > 512 spreads the rows over the
    resident workgroup slots (one round): dx bit-identical to the fixed
    64-row split, dgamma / dbeta equal up to the partials' summation order,
    and both against fp32 torch."""
    O = ops()
    x = (torch.randn(M, N, device=dev) * 2 + 0.5).to(torch.bfloat16)
    g = torch.randn(N, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    O.layernorm(x, g, b, y, mean, rstd)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    res = {}
    for bal in ("1", "0"):
        monkeypatch.setenv("SMER_LN_BWD_BALANCE", bal)
        dx = torch.empty_like(x)
        dg = torch.zeros(N, device=dev)
        db = torch.zeros(N, device=dev)
        O.layernorm_bwd(dy, x, mean, rstd, g, dx, dgamma=dg, dbeta=db)
        res[bal] = (dx, dg, db)
    torch.cuda.synchronize()
    assert torch.equal(res["1"][0], res["0"][0])
    assert rel_err(res["1"][1], res["0"][1]) < 1e-5 and rel_err(res["1"][2], res["0"][2]) < 1e-5
    xf = x.float().requires_grad_(True)
    gf, bf = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xf, (N,), gf, bf, 1e-5).backward(dy.float())
    assert rel_err(res["1"][0], xf.grad) < 2e-2
    assert rel_err(res["1"][1], gf.grad) < 1e-2 and rel_err(res["1"][2], bf.grad) < 1e-2


def test_layernorm_fwd_rows_kernel_bit_identical_to_one_row_kernel(tmp_path):
    """The bf16 LayerNorm forward's rows-per-wave kernel (register arrays
    sized for the row width) returns the one-row ln_fwd_kernel's bits, for
    each rows-per-wave setting (the setting is read once per process:
    tools/ln_fwd_bits.py runs once per SMER_LN_RPW value)."""
    import subprocess
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for rpw in ("0", "1", "2", "4"):
        f = str(tmp_path / ("ln%s.npz" % rpw))
        env = dict(os.environ, SMER_LN_RPW=rpw)
        subprocess.run([sys.executable, os.path.join(root, "tools", "ln_fwd_bits.py"), f],
                       env=env, check=True, timeout=180)
        outs[rpw] = np.load(f)
    for rpw in ("1", "2", "4"):
        for k in outs["0"].files:
            assert np.array_equal(outs["0"][k], outs[rpw][k]), (rpw, k)


@pytest.mark.parametrize("M,N", [(65536, 768), (1000, 768), (16387, 640), (77, 520)])
def test_layernorm_bwd_t4_kernel(M, N, monkeypatch):
    """512 < N <= 768: the 12-columns-per-lane backward (ln_bwd_t4_kernel)
    against the two-chunk ln_bwd_kernel (SMER_LN_BWD_T4=0) and fp32 torch:
    the dropout copy zeroes exactly the same elements, dx agrees up to the
    row sums' summation order, dgamma / dbeta up to the partials' order."""
    O = ops()
    x = (torch.randn(M, N, device=dev) * 2 + 0.5).to(torch.bfloat16)
    g = torch.randn(N, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    O.layernorm(x, g, b, y, mean, rstd)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    res = {}
    for t4 in ("1", "0"):
        monkeypatch.setenv("SMER_LN_BWD_T4", t4)
        dx = torch.empty_like(x)
        dxd = torch.empty_like(x)
        dg = torch.zeros(N, device=dev)
        db = torch.zeros(N, device=dev)
        O.layernorm_bwd(dy, x, mean, rstd, g, dx, dx_drop=dxd, drop_p=0.1, seed=7, dgamma=dg, dbeta=db)
        res[t4] = (dx, dxd, dg, db)
    torch.cuda.synchronize()
    new, old = res["1"], res["0"]
    assert torch.equal(new[1] == 0, old[1] == 0)
    assert rel_err(new[0], old[0]) < 1e-2 and rel_err(new[1], old[1]) < 1e-2
    assert rel_err(new[2], old[2]) < 1e-5 and rel_err(new[3], old[3]) < 1e-5
    xf = x.float().requires_grad_(True)
    gf, bf = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xf, (N,), gf, bf, 1e-5).backward(dy.float())
    assert rel_err(new[0], xf.grad) < 2e-2
    assert rel_err(new[2], gf.grad) < 1e-2 and rel_err(new[3], bf.grad) < 1e-2


@pytest.mark.parametrize("M,N,T,acc,strided", [(256, 256, 64, False, False), (256, 512, 192, True, False),
                                               (768, 512, 4096, True, True), (2304, 768, 16384, False, False),
                                               (768, 3072, 8192, True, False)])
def test_wgrad_fp8_exact_integer_layout(M, N, T, acc, strided):
    """fp8 weight gradient (tokens-major e4m3 operands through the transposing
    8-bit LDS reads, split-K slabs, fused bias gradient) on exact small-
    integer data and power-of-two scales: every partial sum is exact in fp32,
    so dW must equal s_dy * s_x * dY^T X and db s_dy * colsum(dY) bit for bit
    (plus the old values when accumulating).
    Covers one k-step (T = 64), the 3-step prologue edge, split-K, an
    operand that is a column slice of a wider buffer, and the C4 shapes."""
    O = ops()
    g = torch.Generator(device="cpu").manual_seed(M + N + T)
    dY = torch.randint(-4, 5, (T, M), generator=g).float()
    X = torch.randint(-3, 4, (T, N), generator=g).float()
    X[:, 0] += torch.arange(T) % 5  # asymmetric
    dy8 = dY.to(torch.float8_e4m3fn).view(torch.uint8)
    if strided:  # the column slice of a wider e4m3 buffer (dQKV's copy)
        wide = torch.zeros(T, M + 256, dtype=torch.uint8)
        wide[:, 128:128 + M] = dy8
        dy8 = wide.to(dev)[:, 128:128 + M]
    else:
        dy8 = dy8.to(dev)
    x8 = X.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    si, xi = torch.tensor([0.5], device=dev), torch.tensor([0.25], device=dev)
    old = torch.randint(-8, 9, (M, N), generator=g).float()
    dw = old.to(dev) if acc else torch.full((M, N), float("nan"), device=dev)
    oldb = torch.randint(-8, 9, (M,), generator=g).float()
    db = oldb.to(dev) if acc else torch.full((M,), float("nan"), device=dev)
    assert O.linear_wgrad_fp8(dy8, si, x8, xi, dw, accumulate=acc, db=db)
    ref = (dY.t() @ X) * 0.125 + (old if acc else 0.0)
    refb = dY.sum(0) * 0.5 + (oldb if acc else 0.0)
    torch.cuda.synchronize()
    assert torch.equal(dw.cpu(), ref)
    assert torch.equal(db.cpu(), refb)
    dw2 = torch.zeros(M, N, device=dev)  # without the bias gradient: the same dW
    assert O.linear_wgrad_fp8(dy8, si, x8, xi, dw2, accumulate=False)
    torch.cuda.synchronize()
    assert torch.equal(dw2.cpu(), (dY.t() @ X) * 0.125)


def test_wgrad_fp8_declines_outside_tiling():
    O = ops()
    z = torch.zeros(64, 200, dtype=torch.uint8, device=dev)
    one = torch.ones(1, device=dev)
    dw = torch.zeros(200, 200, device=dev)
    assert not O.linear_wgrad_fp8(z, one, z, one, dw)


@pytest.mark.parametrize("mode", ["gate", "bias_relu_drop", "residual"])
def test_fp8_q8_streamed_epilogue_equals_generic(monkeypatch, mode):
    """The e4m3-copy fp8 products on the streamed epilogue (gate / residual
    rows by LDS-DMA a pass ahead, the default) against the generic epilogue
    (SMER_FP8_Q8_FAST=0).  Gate / residual: bf16 output, e4m3 copy and amax
    bit for bit.  Bias + ReLU + dropout: the streamed epilogue fuses scale
    and bias into one fma (the generic one rounds the product first), so
    the outputs agree to a bf16 ulp and the same dropout zeros; in every
    mode the copy is e4m3(out * qs) of the stored bf16 values exactly and
    amax their max |out|."""
    O = ops()
    M, N, K = 512, 768, 768
    g = torch.Generator(device="cpu").manual_seed(11)
    A = torch.randint(-4, 5, (M, K), generator=g).float()
    B = torch.randint(-3, 4, (N, K), generator=g).float()
    a8 = A.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    b8 = B.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)
    ai = torch.tensor([0.0123], device=dev)
    bi = torch.tensor([0.37], device=dev)
    X = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    qs = torch.tensor([37.0], device=dev)

    def run(flag):
        monkeypatch.setenv("SMER_FP8_Q8_FAST", flag)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        q = torch.empty(M, N, device=dev, dtype=torch.uint8)
        am = torch.zeros(1, device=dev, dtype=torch.int32)
        if mode == "gate":
            assert O.gemm_fp8_ex(a8, ai, b8, bi, C, gate=X, gate_scale=1.25, q8=q, qs=qs, amax=am)
        elif mode == "residual":
            assert O.gemm_fp8_ex(a8, ai, b8, bi, C, residual=X, q8=q, qs=qs, amax=am)
        else:
            assert O.gemm_fp8_q(a8, ai, b8, bi, C, bias=bias, relu=True, drop_p=0.1, seed=5, q8=q, qs=qs,
                                amax=am)
        torch.cuda.synchronize()
        return C.cpu(), q.cpu(), am.cpu()

    fast, gen = run("1"), run("0")
    C, q, am = fast
    want_q = (C.float() * 37.0).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(q, want_q)
    assert am.view(torch.float32).item() == C.float().abs().max().item()
    if mode == "bias_relu_drop":
        assert torch.equal(C == 0, gen[0] == 0)
        torch.testing.assert_close(C.float(), gen[0].float(), rtol=2 ** -7, atol=0)
    else:
        for a, b in zip(fast, gen):
            assert torch.equal(a, b)


def test_embed_fp8_copy_matches_embed():
    """smer_embed_fwd_fp8: the same bf16 output as smer_embed_fwd (with
    positional dropout), its e4m3 copy e4m3(out * qs) of the stored values
    and amax = max |out| (the fp8 step's first-layer QKV input)."""
    O = ops()
    V, d, B, L = 309, 512, 3, 200
    g = torch.Generator(device="cpu").manual_seed(21)
    table = torch.randn(V, d, generator=g).to(dev)
    pe = torch.randn(4096, d, generator=g).to(dev)
    ids = torch.randint(0, V, (B * L,), generator=g).to(dev)
    a = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    b = torch.empty_like(a)
    q = torch.empty(B * L, d, device=dev, dtype=torch.uint8)
    qs = torch.tensor([20.0], device=dev)
    am = torch.zeros(1, device=dev, dtype=torch.int32)
    O.embed(ids, table, pe, a, L=L, scale=22.6, drop_p=0.1, seed=5)
    O.embed_fp8(ids, table, pe, b, q, qs, am, L=L, scale=22.6, drop_p=0.1, seed=5)
    torch.cuda.synchronize()
    assert torch.equal(a.cpu(), b.cpu())
    want = (b.float().cpu() * 20.0).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(q.cpu(), want)
    assert am.cpu().view(torch.float32).item() == b.float().abs().max().item()


def test_fp8_e4m3_gate_and_copy_only_output():
    """smer_gemm_fp8_gate8 (the FFN2 dgrad gated by FFN1's e4m3 copy) equals
    smer_gemm_fp8_ex gated by the copy's dequantised bf16 values bit for bit
    (output, e4m3 copy, amax), and smer_gemm_fp8_q with a null C writes the
    same e4m3 copy and amax as with C."""
    O = ops()
    M, N, K = 512, 768, 256
    g = torch.Generator(device="cpu").manual_seed(8)
    e4 = lambda t: t.to(torch.float8_e4m3fn).view(torch.uint8).to(dev)  # noqa: E731
    a8, b8 = e4(torch.randn(M, K, generator=g) * 4), e4(torch.randn(N, K, generator=g) * 4)
    inv = torch.tensor([1.0 / 32], device=dev)
    # the gate: an e4m3 copy with zeros, negative zeros, negatives and positives
    gq = torch.randn(M, N, generator=g) * 3
    gq[torch.rand(M, N, generator=g) < 0.2] = 0.0
    gq[torch.rand(M, N, generator=g) < 0.05] = -0.0
    g8 = e4(gq)
    g_bf = g8.view(torch.float8_e4m3fn).float().mul(0.25).to(torch.bfloat16)
    qs = torch.tensor([3.0], device=dev)
    outs = []
    for use8 in (False, True):
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        q = torch.empty(M, N, device=dev, dtype=torch.uint8)
        am = torch.zeros(1, device=dev, dtype=torch.int32)
        if use8:
            assert O.gemm_fp8_gate8(a8, inv, b8, inv, g8, 1.25, out, q, qs, am)
        else:
            assert O.gemm_fp8_ex(a8, inv, b8, inv, out, gate=g_bf, gate_scale=1.25, q8=q, qs=qs, amax=am)
        outs.append((out, q, am))
    torch.cuda.synchronize()
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x.cpu(), y.cpu())
    assert int((outs[1][0] == 0).sum()) > M * N // 5  # the gate closed somewhere
    # both gated forms with a null C: the same e4m3 copy and amax alone
    for use8 in (False, True):
        q = torch.empty(M, N, device=dev, dtype=torch.uint8)
        am = torch.zeros(1, device=dev, dtype=torch.int32)
        if use8:
            assert O.gemm_fp8_gate8(a8, inv, b8, inv, g8, 1.25, None, q, qs, am)
        else:
            assert O.gemm_fp8_ex(a8, inv, b8, inv, None, gate=g_bf, gate_scale=1.25, q8=q, qs=qs, amax=am)
        torch.cuda.synchronize()
        assert torch.equal(q.cpu(), outs[1][1].cpu()) and torch.equal(am.cpu(), outs[1][2].cpu())
    # FFN1 with and without its bf16 output
    bias = torch.randn(N, generator=g).to(dev)
    res = []
    for with_c in (True, False):
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if with_c else None
        q = torch.empty(M, N, device=dev, dtype=torch.uint8)
        am = torch.zeros(1, device=dev, dtype=torch.int32)
        assert O.gemm_fp8_q(a8, inv, b8, inv, out, bias=bias, relu=True, drop_p=0.1, seed=4, q8=q, qs=qs,
                            amax=am)
        res.append((q, am))
    torch.cuda.synchronize()
    assert torch.equal(res[0][0].cpu(), res[1][0].cpu()) and torch.equal(res[0][1].cpu(), res[1][1].cpu())


@pytest.mark.parametrize("N", [768, 512])
def test_layernorm_bwd_fp8_copy_only_dropped_gradient(N):
    """smer_layernorm_bwd_fp8 with dropout and no dx_drop buffer: the same dx,
    e4m3 copy of the dropped gradient and amax as with the buffer (N = 768 runs
    the 12-column kernel, 512 the generic one)."""
    O = ops()
    M = 1024
    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.randn(M, N, generator=g).to(dev).to(torch.bfloat16)
    dy = torch.randn(M, N, generator=g).to(dev).to(torch.bfloat16)
    gamma = (torch.rand(N, generator=g) + 0.5).to(dev)
    beta = torch.zeros(N, device=dev)
    y = torch.empty_like(x)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    O.layernorm(x, gamma, beta, y, mean, rstd)
    qs = torch.tensor([40.0], device=dev)
    res = []
    for with_buf in (True, False):
        dx = torch.empty_like(x)
        dxd = torch.empty_like(x) if with_buf else None
        q = torch.empty(M, N, device=dev, dtype=torch.uint8)
        am = torch.zeros(1, device=dev, dtype=torch.int32)
        O.layernorm_bwd(dy, x, mean, rstd, gamma, dx, dx_drop=dxd, drop_p=0.1, seed=11, q8=q, qs=qs, amax=am)
        res.append((dx, q, am, dxd))
    torch.cuda.synchronize()
    for a, b in zip(res[0][:3], res[1][:3]):
        assert torch.equal(a.cpu(), b.cpu())
    want = (res[0][3].float().cpu() * 40.0).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(res[1][1].cpu(), want)
    assert not torch.equal(res[0][0].cpu(), res[0][3].cpu())  # dropout did act
