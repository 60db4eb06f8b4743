"""Tensor-level wrappers over the C-ABI (one function per entry point).

Every wrapper takes torch tensors already on the GPU, passes raw pointers,
row strides and torch's current HIP stream to libsmer_hip.so and raises
`SmerError` on a non-zero status.  There is no CPU or ATen fallback: a CPU
tensor is rejected, a missing library raises at first use.
"""
from __future__ import annotations

import torch

from ._lib import call, load

F32, BF16 = 0, 1


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return F32
    if t == torch.bfloat16:
        return BF16
    raise TypeError("unsupported dtype %s" % t)


def _p(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("smer op: tensor must be on the GPU (got %s)" % t.device)
    return t.data_ptr()


def drop_scale(p):
    """Survivor scale of every dropout site (csrc/common.h
    smer_drop_scale16): 65536 / (65536 - round(p * 65536))."""
    if p <= 0:
        return 1.0
    thr = min(65535, max(1, int(p * 65536.0 + 0.5)))
    return 65536.0 / (65536.0 - thr)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _ld(t):
    """Row stride (elements) of a 2-D view with unit column stride."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise RuntimeError("smer op: expected a 2-D row-major view, got strides %s" % (t.stride(),))
    return t.stride(0)


# ---------------------------------------------------------------------------
class KernelTimer:
    """Optional live timing of GEMM launches with HIP events on the launch
    stream (bench.py roofline): records (start, end, flops) per launch."""

    def __init__(self):
        self.records = []

    def summary(self):
        torch.cuda.synchronize()
        ms = [r[0].elapsed_time(r[1]) for r in self.records]
        fl = [r[2] for r in self.records]
        return {"launches": len(ms), "total_ms": float(sum(ms)), "flops": float(sum(fl))}

    def by_shape(self):
        """{tag: (launches, total_ms, flops)} over the recorded launches."""
        torch.cuda.synchronize()
        out = {}
        for r in self.records:
            tag = r[3] if len(r) > 3 else "?"
            n, t, f = out.get(tag, (0, 0.0, 0.0))
            out[tag] = (n + 1, t + r[0].elapsed_time(r[1]), f + r[2])
        return out


GEMM_TIMER = None  # set to a KernelTimer to instrument smer_gemm launches


def gemm(A, B, *, M, N, K, a_kcontig=True, b_kcontig=True, out=None, out_f32=None,
         accumulate=False, bias=None, alpha=1.0, relu=False, residual=None, gate=None,
         gate_scale=1.0, drop_p=0.0, seed=0, dtype=None):
    """out (+)= epilogue(alpha * op(A) op(B)^T); see include/smer_hip.h."""
    dt = dtype_code(dtype if dtype is not None else A.dtype)
    timer = GEMM_TIMER
    if timer is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    _gemm_call(dt, A, B, M, N, K, a_kcontig, b_kcontig, out, out_f32, accumulate, bias, alpha,
               relu, residual, gate, gate_scale, drop_p, seed)
    if timer is not None:
        ev1.record()
        epi = "".join(c for c, on in (("b", bias is not None), ("r", relu), ("d", drop_p > 0),
                                      ("R", residual is not None), ("g", gate is not None),
                                      ("f", out_f32 is not None), ("+", accumulate)) if on)
        tag = "%s%s M%d N%d K%d %s" % ("n" if a_kcontig else "t", "t" if b_kcontig else "n",
                                        M, N, K, epi)
        timer.records.append((ev0, ev1, 2.0 * M * N * K, tag))


class CkLog:
    """Repeatability probe (tools/ck_log.py): an order-independent checksum
    of a tensor taken on the current stream into a preallocated device log,
    no host sync, no allocation per entry.  Engine.backward calls `ck()` after
    each launch when `ops.CK_LOG` is set; not used on the product path."""

    PARTS = 64

    def __init__(self, device, n=4096, keep=()):
        self.buf = torch.zeros(n * self.PARTS, dtype=torch.int64, device=device)
        self.n = n
        self.names = []
        self.keep = tuple(keep)  # name substrings whose tensors are also cloned
        self.kept = {}

    def add(self, name, t):
        i = len(self.names)
        if i >= self.n:
            return
        if t.dim() == 1:
            rows, row_b, ld_b = 1, t.numel() * t.element_size(), t.numel() * t.element_size()
        else:
            t2 = t.reshape(-1, t.shape[-1]) if t.dim() > 2 else t
            rows, row_b, ld_b = t2.shape[0], t2.shape[1] * t2.element_size(), _ld(t2) * t2.element_size()
        self.names.append((name, torch.cuda.current_stream(t.device).cuda_stream))
        call("smer_debug_checksum", _p(t), rows, row_b, ld_b, self.buf.data_ptr() + i * self.PARTS * 8,
             self.PARTS, _stream())
        if any(k in name for k in self.keep):
            self.kept[i] = t.clone()

    def values(self):
        import numpy as np
        v = self.buf.view(self.n, self.PARTS)[:len(self.names)].cpu().numpy().view(np.uint64)
        return [int(x) for x in v.sum(axis=1, dtype=np.uint64)]

    def reset(self):
        self.buf.zero_()
        self.names = []
        self.kept = {}


CK_LOG = None


def ck(name, t):
    if CK_LOG is not None and t is not None:
        CK_LOG.add(name, t)


_SPLITK_WS = {}
SPLITK_WS_BYTES = 64 << 20


def splitk_workspace(device):
    """Persistent per-device split-K slab buffer (stream-ordered reuse)."""
    ws = _SPLITK_WS.get(device)
    if ws is None:
        ws = torch.zeros(SPLITK_WS_BYTES, dtype=torch.uint8, device=device)  # its tail: split-K tickets, zero
        _SPLITK_WS[device] = ws
    return ws


def _gemm_call(dt, A, B, M, N, K, a_kcontig, b_kcontig, out, out_f32, accumulate, bias, alpha,
               relu, residual, gate, gate_scale, drop_p, seed):
    ws = None
    if out_f32 is not None and out is None and bias is None and residual is None and gate is None:
        ws = splitk_workspace(A.device)
    call("smer_gemm", dt, int(a_kcontig), int(b_kcontig), M, N, K, _p(A), _ld(A), _p(B), _ld(B),
         _p(bias), float(alpha), int(relu), _p(residual),
         _ld(residual) if residual is not None else 0, _p(gate),
         _ld(gate) if gate is not None else 0, float(gate_scale), float(drop_p),
         int(seed) & 0xFFFFFFFF, _p(out), _ld(out) if out is not None else 0, _p(out_f32),
         _ld(out_f32) if out_f32 is not None else 0, int(accumulate), _p(ws),
         ws.numel() if ws is not None else 0, _stream())


def linear(x, w, bias=None, *, out=None, out_f32=None, accumulate=False, relu=False,
           residual=None, drop_p=0.0, seed=0):
    """y = x @ w^T (+bias ...): x [M,K], w [N,K]."""
    M, K = x.shape
    N = w.shape[0]
    if out is None and out_f32 is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    gemm(x, w, M=M, N=N, K=K, out=out, out_f32=out_f32, accumulate=accumulate, bias=bias,
         relu=relu, residual=residual, drop_p=drop_p, seed=seed, dtype=x.dtype)
    return out if out is not None else out_f32


def linear_dgrad(dy, w, *, K=None, out=None, residual=None, gate=None, gate_scale=1.0,
                 out_f32=None, accumulate=False):
    """dx = dy @ w: dy [M,N_out], w [N_out, K_in] -> [M, K_in]."""
    M = dy.shape[0]
    Kc = K if K is not None else w.shape[0]
    Nin = w.shape[1]
    if out is None and out_f32 is None:
        out = torch.empty(M, Nin, device=dy.device, dtype=dy.dtype)
    gemm(dy, w, M=M, N=Nin, K=Kc, a_kcontig=True, b_kcontig=False, out=out, out_f32=out_f32,
         accumulate=accumulate, residual=residual, gate=gate, gate_scale=gate_scale,
         dtype=dy.dtype)
    return out if out is not None else out_f32


def linear_wgrad(dy, x, dw, *, M=None, accumulate=True, db=None, ws=None, max_wg=0):
    """dw (+)= dy^T @ x: dy [T, M_out(ld)], x [T, K_in] -> dw fp32 [M_out, K_in];
    db (+)= column sums of dy when given (bf16: fused into the GEMM).  `ws`:
    split-K slab buffer (default: the per-device one; a second stream running
    wgrads concurrently passes its own).  max_wg > 0 caps the persistent
    weight-gradient grid (smer_gemm_wgrad_bias_ex: leave CUs to a concurrent
    stream)."""
    T = dy.shape[0]
    Mo = M if M is not None else dy.shape[1]
    if db is not None and dy.dtype == torch.bfloat16:
        if ws is None:
            ws = splitk_workspace(dy.device)
        timer = GEMM_TIMER
        if timer is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        call("smer_gemm_wgrad_bias_ex", BF16, Mo, x.shape[1], T, _p(dy), _ld(dy), _p(x), _ld(x),
             _p(dw), _ld(dw), int(accumulate), _p(db), int(accumulate), _p(ws), ws.numel(),
             int(max_wg), _stream())
        if timer is not None:
            ev1.record()
            timer.records.append((ev0, ev1, 2.0 * Mo * x.shape[1] * T,
                                  "wgrad+bias M%d N%d K%d" % (Mo, x.shape[1], T)))
        return
    gemm(dy, x, M=Mo, N=x.shape[1], K=T, a_kcontig=False, b_kcontig=False, out_f32=dw,
         accumulate=accumulate, dtype=dy.dtype)
    if db is not None:
        colsum(dy, db, N=Mo, accumulate=accumulate)


# ---------------------------------------------------------------------------
def attn_drop_mask(B, H, Lq, Lk, device):
    """Buffer for the forward's attention-dropout keep bits (read by attn_bwd)."""
    n = load().smer_attn_drop_mask_bytes(B, H, Lq, Lk)
    return torch.empty(max(16, n), dtype=torch.uint8, device=device)


_WARNED_P = set()


def attn_drop_rate(p):
    """Realised attention-probability dropout rate: the attention kernels
    draw keep decisions at 1/128 granularity (csrc/common.h smer_attn_thr7:
    round(128 p) clamped to [1, 127]), survivors scaled exactly for it."""
    if p <= 0:
        return 0.0
    return min(127, max(1, int(p * 128.0 + 0.5))) / 128.0


def _check_attn_p(p):
    r = attn_drop_rate(p)
    if p > 0 and abs(r - p) > 0.1 * p and p not in _WARNED_P:
        import warnings
        _WARNED_P.add(p)
        warnings.warn("attention dropout p=%g is realised as %g (1/128 granularity of the "
                      "attention kernels); activation dropout sites keep p to 1/65536" % (p, r))


def attn_fwd(q, k, v, o, lse, *, B, H, Lq, Lk, D, kpm=None, causal=False, scale, drop_p=0.0,
             seed=0, drop_mask=None, drop_mask_in=False, q8=None):
    """drop_mask: keep-bit buffer the forward fills (hashing) for the
    backward, or, with drop_mask_in, reads (from attn_drop_mask_gen).
    q8 (bf16): (o8, qs, amax) -- the e4m3 copy e4m3(o * qs[0]) of the output,
    max|o| folded into amax (smer_attn_fwd_fp8)."""
    _check_attn_p(drop_p)
    if q8 is not None:
        if dtype_code(q.dtype) != BF16:
            raise RuntimeError("attn_fwd: the e4m3 copy needs bf16")
        o8, qs, amax = q8
        call("smer_attn_fwd_fp8", B, H, Lq, Lk, D, _p(q), _ld(q), _p(k), _ld(k), _p(v), _ld(v), _p(o),
             _ld(o), _p(lse), _p(kpm), int(causal), float(scale), float(drop_p), int(seed) & 0xFFFFFFFF,
             _p(drop_mask), int(bool(drop_mask_in)), _p(o8), _ld(o8), _p(qs), _p(amax), _stream())
        return
    call("smer_attn_fwd", dtype_code(q.dtype), B, H, Lq, Lk, D, _p(q), _ld(q), _p(k), _ld(k),
         _p(v), _ld(v), _p(o), _ld(o), _p(lse), _p(kpm), int(causal), float(scale),
         float(drop_p), int(seed) & 0xFFFFFFFF, _p(drop_mask), int(bool(drop_mask_in)), _stream())


def attn_drop_mask_gen(mask, *, B, H, Lq, Lk, drop_p, seed):
    call("smer_attn_drop_mask_gen", B, H, Lq, Lk, float(drop_p), int(seed) & 0xFFFFFFFF,
         _p(mask), _stream())


def attn_bwd(q, k, v, o, do, lse, dq, dk, dv, *, B, H, Lq, Lk, D, kpm=None, causal=False,
             scale, drop_p=0.0, seed=0, drop_mask=None, q8=None):
    """q8 (bf16): (dq8, dk8, dv8, qs, amax) -- e4m3 copies of the gradients
    (uint8 views shaped like dq / dk / dv; dq8 or dk8 + dv8 may be None)
    scaled by qs[0], max|g| folded into amax (smer_attn_bwd_fp8); a gradient
    with a copy may then be None itself (dk with dv): the copy alone."""
    lib = load()
    dt = dtype_code(q.dtype)
    nbytes = lib.smer_attn_bwd_workspace(dt, B, H, Lq, Lk)
    ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=q.device)
    if q8 is not None:
        if dt != BF16:
            raise RuntimeError("attn_bwd: e4m3 copies need bf16")
        dq8, dk8, dv8, qs, amax = q8
        ld8 = lambda t: _ld(t) if t is not None else 0  # noqa: E731
        call("smer_attn_bwd_fp8", B, H, Lq, Lk, D, _p(q), _ld(q), _p(k), _ld(k), _p(v), _ld(v),
             _p(o), _ld(o), _p(do), _ld(do), _p(lse), _p(kpm), int(causal), float(scale),
             float(drop_p), int(seed) & 0xFFFFFFFF, _p(dq), ld8(dq), _p(dk), ld8(dk), _p(dv),
             ld8(dv), _p(ws), nbytes, _p(drop_mask), _p(dq8), ld8(dq8), _p(dk8), ld8(dk8),
             _p(dv8), ld8(dv8), _p(qs), _p(amax), _stream())
        return
    call("smer_attn_bwd", dt, B, H, Lq, Lk, D, _p(q), _ld(q), _p(k), _ld(k), _p(v), _ld(v),
         _p(o), _ld(o), _p(do), _ld(do), _p(lse), _p(kpm), int(causal), float(scale),
         float(drop_p), int(seed) & 0xFFFFFFFF, _p(dq), _ld(dq), _p(dk), _ld(dk), _p(dv),
         _ld(dv), _p(ws), nbytes, _p(drop_mask), _stream())


def attn_weights(q, k, lse, out, *, B, H, Lq, Lk, D, kpm=None, causal=False, scale):
    call("smer_attn_weights", dtype_code(q.dtype), B, H, Lq, Lk, D, _p(q), _ld(q), _p(k),
         _ld(k), _p(lse), _p(kpm), int(causal), float(scale), _p(out), _stream())


def attn_decode(q, kcache, vcache, row_req, row_nkeys, out, *, H, D, row_stride, req_stride,
                scale, head_stride=0):
    call("smer_attn_decode", dtype_code(q.dtype), q.shape[0], H, D, _p(q), _ld(q), _p(kcache),
         _p(vcache), int(row_stride), int(req_stride), int(head_stride), _p(row_req),
         _p(row_nkeys), _p(out), _ld(out), float(scale), _stream())


def attn_decode_qln(y, gamma, beta, wq, bq, kcache, vcache, row_req, row_nkeys, out, *, H, D,
                    row_stride, req_stride, scale, head_stride=0, x_out=None, eps=1e-5):
    """Decode cross attention whose query is LayerNorm(y) . wq^T + bq, both
    computed in the attention block (see smer_hip.h); x_out <- LayerNorm(y)."""
    M, dm = y.shape
    call("smer_attn_decode_qln", M, H, D, _p(y), _ld(y), _p(gamma), _p(beta), float(eps), _p(wq),
         _ld(wq), _p(bq), _p(x_out), _ld(x_out) if x_out is not None else 0, dm, _p(kcache),
         _p(vcache), int(row_stride), int(req_stride), int(head_stride), _p(row_req),
         _p(row_nkeys), _p(out), _ld(out), float(scale), _stream())


DEC_SPLITS = 8  # key slices of attn_decode_split_f32 (csrc DEC_NS)


def attn_decode_split_f32(q, kcache, vcache, row_req, row_nkeys, part, *, H, D, row_stride, req_stride,
                          scale, head_stride=0):
    """fp32 decode attention over 8 key slices per (row, head): partial
    records part [rows, H, 8, 68] (see smer_hip.h)."""
    call("smer_attn_decode_split_f32", q.shape[0], H, D, _p(q), _ld(q), _p(kcache), _p(vcache),
         int(row_stride), int(req_stride), int(head_stride), _p(row_req), _p(row_nkeys), _p(part),
         float(scale), _stream())


def attn_decode_split_qln_f32(y, gamma, beta, wq, bq, kcache, vcache, row_req, row_nkeys, part, *, H, D,
                              row_stride, req_stride, scale, head_stride=0, x_out=None, eps=1e-5):
    """attn_decode_split_f32 whose query is LayerNorm(y) . wq^T + bq, both
    computed in the attention blocks (fp32, d_model 512); x_out <- LayerNorm(y)."""
    M, dm = y.shape
    call("smer_attn_decode_split_qln_f32", M, H, D, _p(y), _ld(y), _p(gamma), _p(beta), float(eps), _p(wq),
         _ld(wq), _p(bq), _p(x_out), _ld(x_out) if x_out is not None else 0, dm, _p(kcache), _p(vcache),
         int(row_stride), int(req_stride), int(head_stride), _p(row_req), _p(row_nkeys), _p(part),
         float(scale), _stream())


def linear_decode_merge_f32(part, w, bias=None, *, M, residual=None, relu=False, out=None):
    """out = merge(part) @ w^T + bias (+relu) (+residual), fp32; merge()
    combines attn_decode_split_f32's slices into the attention output rows."""
    N, K = w.shape
    if out is None:
        out = torch.empty(M, N, device=w.device, dtype=torch.float32)
    call("smer_linear_decode_merge_f32", M, N, K, _p(part), _p(w), _ld(w), _p(bias), int(bool(relu)),
         _p(residual), _ld(residual) if residual is not None else 0, _p(out), _ld(out), None, 0, _stream())
    return out


def kv_scatter_heads(src, cache, row_req, row_pos, *, H, D, req_stride, kv_stride, head_stride):
    """Rows of [K heads | V heads] into a head-major cache (see smer_hip.h)."""
    if src.shape[1] != 2 * H * D:
        raise RuntimeError("kv_scatter_heads: src must have 2*H*D columns")
    call("smer_kv_scatter_heads", dtype_code(src.dtype), src.shape[0], H, D, _p(src), _ld(src),
         _p(cache), int(req_stride), int(kv_stride), int(head_stride), _p(row_req), _p(row_pos),
         _stream())


def kv_scatter(src, cache, row_req, row_pos, *, row_stride, req_stride):
    call("smer_kv_scatter", dtype_code(src.dtype), src.shape[0], src.shape[1], _p(src), _ld(src),
         _p(cache), int(row_stride), int(req_stride), _p(row_req), _p(row_pos), _stream())


def linear_decode(x, w, bias=None, *, relu=False, residual=None, out=None, out_f32=None, kv=None,
                  kv_req=None, kv_pos=None, kv_row_stride=0, kv_req_stride=0, kv_col0=0):
    """Decode-step Linear (bf16, M <= 256; fp32, M <= 64): out = x @ w^T +
    bias (+relu) (+residual); output columns >= kv_col0 are also appended to
    the K/V cache `kv` at (kv_req[m], kv_pos[m])."""
    M, K = x.shape
    N = w.shape[0]
    if out is None and out_f32 is None:
        out = torch.empty(M, N, device=x.device, dtype=x.dtype)
    fn = "smer_linear_decode_f32" if x.dtype == torch.float32 else "smer_linear_decode"
    call(fn, M, N, K, _p(x), _ld(x), _p(w), _ld(w), _p(bias), int(bool(relu)),
         _p(residual), _ld(residual) if residual is not None else 0, _p(out),
         _ld(out) if out is not None else 0, _p(out_f32), _ld(out_f32) if out_f32 is not None else 0,
         _p(kv), int(kv_row_stride), int(kv_req_stride), _p(kv_req), _p(kv_pos), int(kv_col0),
         _stream())
    return out if out is not None else out_f32


def linear_decode_ln(y, gamma, beta, w, bias=None, *, x_out=None, eps=1e-5, relu=False,
                     residual=None, out=None, out_f32=None, kv=None, kv_req=None, kv_pos=None,
                     kv_row_stride=0, kv_req_stride=0, kv_col0=0):
    """linear_decode(LayerNorm(y), w, ...): the LayerNorm fused into the
    Linear's prologue (bit-identical to ops.layernorm); x_out receives LN(y)."""
    M, K = y.shape
    N = w.shape[0]
    if out is None and out_f32 is None:
        out = torch.empty(M, N, device=y.device, dtype=y.dtype)
    fn = "smer_linear_decode_ln_f32" if y.dtype == torch.float32 else "smer_linear_decode_ln"
    call(fn, M, N, K, _p(y), _ld(y), _p(gamma), _p(beta), float(eps), _p(x_out),
         _ld(x_out) if x_out is not None else 0, _p(w), _ld(w), _p(bias), int(bool(relu)),
         _p(residual), _ld(residual) if residual is not None else 0, _p(out),
         _ld(out) if out is not None else 0, _p(out_f32), _ld(out_f32) if out_f32 is not None else 0,
         _p(kv), int(kv_row_stride), int(kv_req_stride), _p(kv_req), _p(kv_pos), int(kv_col0),
         _stream())
    return out if out is not None else out_f32


# ---------------------------------------------------------------------------
def fp8_quantize(x, q, inv_scale, workspace=None):
    """q (uint8 e4m3 bits, same shape as x) = e4m3(x * 448 / amax|x|);
    inv_scale (1-element fp32, device) = amax / 448."""
    rows, cols = x.shape
    if workspace is None:
        workspace = torch.empty(16, dtype=torch.uint8, device=x.device)
    call("smer_fp8_quantize", rows, cols, _p(x), _ld(x), _p(q), _ld(q), _p(workspace),
         _p(inv_scale), _stream())
    return q


def fp8_quantize_segments(seg, amax_ws, inv, blocks_per_seg=64):
    """Batched fp8_quantize: seg int64 [nseg, 3] on the device = (src bf16
    ptr, dst uint8 ptr, n); inv fp32 [nseg] <- amax / 448 per tensor."""
    n = seg.shape[0]
    if amax_ws.numel() < n or inv.numel() < n:
        raise ValueError("fp8_quantize_segments: workspace / inv smaller than nseg")
    call("smer_fp8_quantize_segments", n, _p(seg), _p(amax_ws), _p(inv), int(blocks_per_seg),
         _stream())


def fp8_quantize_segments_t(seg, amax_ws, inv, blocks_per_seg=64):
    """Batched transposing e4m3 quantisation: seg int64 [nseg, 4] on the
    device = (src bf16 ptr [rows, cols], dst uint8 ptr [cols, rows], rows,
    cols), rows / cols multiples of 64; inv fp32 [nseg] <- amax / 448."""
    n = seg.shape[0]
    if amax_ws.numel() < n or inv.numel() < n:
        raise ValueError("fp8_quantize_segments_t: workspace / inv smaller than nseg")
    call("smer_fp8_quantize_segments_t", n, _p(seg), _p(amax_ws), _p(inv), int(blocks_per_seg),
         _stream())


def gemm_fp8_ex(a8, a_inv, b8, b_inv, out, *, bias=None, residual=None, gate=None, gate_scale=1.0,
                q8=None, qs=None, amax=None):
    """out[M,N] bf16 = a_inv*b_inv * a8 @ b8^T (+ bias) (+ residual | ReLU gate:
    out = gate > 0 ? v * gate_scale : 0), optionally with the e4m3 copy of out
    (q8 = e4m3(out * qs), max|out| folded into amax).  The fp8 backward's
    dgrad products; out may be None beside q8 (the e4m3 copy alone, streamed
    epilogue).  Returns False (nothing launched) outside the tiling."""
    M, K = a8.shape
    N = b8.shape[0]
    if M % 256 or N % 256 or K % 128:
        return False
    timer = GEMM_TIMER
    if timer is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    call("smer_gemm_fp8_ex", M, N, K, _p(a8), _ld(a8), _p(b8), _ld(b8), _p(a_inv), _p(b_inv),
         _p(bias), 0, _p(residual), _ld(residual) if residual is not None else 0, _p(gate),
         _ld(gate) if gate is not None else 0, float(gate_scale), 0.0, 0, _p(out), _ld(out) if out is not None else 0, _p(q8),
         _ld(q8) if q8 is not None else 0, _p(qs), _p(amax), _stream())
    if timer is not None:
        ev1.record()
        timer.records.append((ev0, ev1, 2.0 * M * N * K, "fp8 dgrad M%d N%d K%d%s" % (
            M, N, K, " g" if gate is not None else " R" if residual is not None else "")))
    return True


def linear_wgrad_fp8(dy8, dy_inv, x8, x_inv, dw, *, accumulate=True, db=None, ws=None, max_wg=0):
    """dw fp32 [M, N] (+)= dy_inv*x_inv * dy8^T @ x8 from the tokens-major
    e4m3 copies dy8 [T, M] and x8 [T, N] (precision "fp8" weight gradients),
    db (+)= dy_inv * column sums of dy8 when given.  Returns False (nothing
    launched) outside the kernel's tiling (M, N % 256, T % 64)."""
    T, M = dy8.shape
    N = x8.shape[1]
    if M % 256 or N % 256 or T % 64 or x8.shape[0] != T or tuple(dw.shape) != (M, N):
        return False
    if ws is None:
        ws = splitk_workspace(dy8.device)
    timer = GEMM_TIMER
    if timer is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    call("smer_gemm_wgrad_fp8", M, N, T, _p(dy8), _ld(dy8), _p(x8), _ld(x8), _p(dy_inv), _p(x_inv), _p(dw),
         _ld(dw), int(accumulate), _p(db), int(accumulate), _p(ws), ws.numel(), int(max_wg), _stream())
    if timer is not None:
        ev1.record()
        timer.records.append((ev0, ev1, 2.0 * M * N * T, "fp8 wgrad M%d N%d K%d" % (M, N, T)))
    return True


def gemm_fp8(a8, a_inv, b8, b_inv, out, *, bias=None, relu=False, residual=None, drop_p=0.0,
             seed=0):
    """out[M,N] bf16 = a_inv*b_inv * a8 @ b8^T (+ epilogue).  Returns False
    (nothing launched) when the shape is outside the fp8 kernel's tiling."""
    M, K = a8.shape
    N = b8.shape[0]
    if M % 256 or N % 256 or K % 128:
        return False
    timer = GEMM_TIMER
    if timer is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    call("smer_gemm_fp8", M, N, K, _p(a8), _ld(a8), _p(b8), _ld(b8), _p(a_inv), _p(b_inv),
         _p(bias), int(bool(relu)), _p(residual), _ld(residual) if residual is not None else 0,
         float(drop_p), int(seed) & 0xFFFFFFFF, _p(out), _ld(out), _stream())
    if timer is not None:
        ev1.record()
        timer.records.append((ev0, ev1, 2.0 * M * N * K, "fp8 M%d N%d K%d%s" % (
            M, N, K, " R" if residual is not None else "")))
    return True


def gemm_fp8_gate8(a8, a_inv, b8, b_inv, gate8, gate_scale, out, q8, qs, amax):
    """out[M,N] bf16 = gate8 > 0 ? a_inv*b_inv * (a8 @ b8^T) * gate_scale : 0
    with the gate read from an e4m3 copy (bytes 1..127 open), plus the e4m3
    copy of out: the fp8 step's FFN2 dgrad when FFN1 kept only its e4m3
    output.  Returns False (nothing launched) outside the tiling."""
    M, K = a8.shape
    N = b8.shape[0]
    if M % 256 or N % 256 or K % 128:
        return False
    timer = GEMM_TIMER
    if timer is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    call("smer_gemm_fp8_gate8", M, N, K, _p(a8), _ld(a8), _p(b8), _ld(b8), _p(a_inv), _p(b_inv),
         _p(gate8), _ld(gate8), float(gate_scale), _p(out), _ld(out) if out is not None else 0, _p(q8), _ld(q8),
         _p(qs), _p(amax),
         _stream())
    if timer is not None:
        ev1.record()
        timer.records.append((ev0, ev1, 2.0 * M * N * K, "fp8 dgrad M%d N%d K%d g8" % (M, N, K)))
    return True


def gemm_fp8_q(a8, a_inv, b8, b_inv, out, *, bias=None, relu=False, residual=None, drop_p=0.0,
               seed=0, q8=None, qs=None, amax=None):
    """gemm_fp8 plus an e4m3 copy of `out` (q8 = e4m3(out * qs), max|out| folded
    into amax): the fp8 training forward's FFN1 (its output feeds FFN2).
    out=None: the e4m3 copy alone (streamed epilogue, SMER_FP8_Q8_FAST)."""
    M, K = a8.shape
    N = b8.shape[0]
    if M % 256 or N % 256 or K % 128:
        return False
    timer = GEMM_TIMER
    if timer is not None:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    call("smer_gemm_fp8_q", M, N, K, _p(a8), _ld(a8), _p(b8), _ld(b8), _p(a_inv), _p(b_inv),
         _p(bias), int(bool(relu)), _p(residual), _ld(residual) if residual is not None else 0,
         float(drop_p), int(seed) & 0xFFFFFFFF, _p(out), _ld(out) if out is not None else 0, _p(q8),
         _ld(q8) if q8 is not None else 0, _p(qs), _p(amax), _stream())
    if timer is not None:
        ev1.record()
        timer.records.append((ev0, ev1, 2.0 * M * N * K, "fp8q M%d N%d K%d" % (M, N, K)))
    return True


def layernorm_fp8(x, gamma, beta, y, mean, rstd, q8, qs, amax, eps=1e-5):
    """bf16 LayerNorm that also writes the e4m3 copy of y (delayed scaling)."""
    M, N = x.shape
    call("smer_layernorm_fwd_fp8", M, N, _p(x), _ld(x), _p(gamma), _p(beta), float(eps), _p(y),
         _ld(y), _p(mean), _p(rstd), _p(q8), _ld(q8), _p(qs), _p(amax), _stream())


def fp8_scales(amax_prev, qs, inv, amax_next):
    call("smer_fp8_scales", amax_prev.numel(), _p(amax_prev), _p(qs), _p(inv), _p(amax_next),
         _stream())


def grammar_greedy_step(logits, state, targets, keep, cls, src_len, ids, meta, out_tok, alive, *,
                        eos, m0, trash_pos, max_span=100, ring=None):
    """alive: int32 [1] live count (zeroed per step by a memset), or, with
    `ring` (pinned host int32 [n]), int32 [3] control words zeroed once: the
    step's live count lands in ring[step % n] with no per-step memset or copy."""
    R, nst = state.shape
    V = keep.shape[1]
    for t, dt in ((state, torch.int32), (targets, torch.int8), (keep, torch.uint8),
                  (cls, torch.uint8), (src_len, torch.int32), (ids, torch.int64),
                  (meta, torch.int32), (out_tok, torch.int32), (alive, torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise RuntimeError("grammar_greedy_step: expected contiguous %s" % dt)
    if logits.shape[0] < 2 * R or ids.shape[0] != 2 * R or meta.shape != (4, 2 * R) or \
            targets.shape[0] != R or keep.shape[0] != 13 or cls.shape[0] != V or src_len.shape[0] != R:
        raise RuntimeError("grammar_greedy_step: shape mismatch")
    if ring is not None:
        if ring.dtype != torch.int32 or not ring.is_pinned() or alive.numel() < 3:
            raise RuntimeError("grammar_greedy_step: ring must be pinned int32, alive int32 [3]")
        call("smer_grammar_greedy_step_ring", R, V, _p(logits), _ld(logits), _p(state), nst,
             _p(targets), targets.shape[1], _p(keep), _p(cls), int(eos), int(m0), int(trash_pos),
             int(max_span), _p(src_len), _p(ids), _p(meta), _p(out_tok), out_tok.shape[1],
             _p(alive), ring.data_ptr(), ring.numel(), _stream())  # pinned host memory
        return
    call("smer_grammar_greedy_step", R, V, _p(logits), _ld(logits), _p(state), nst, _p(targets),
         targets.shape[1], _p(keep), _p(cls), int(eos), int(m0), int(trash_pos), int(max_span),
         _p(src_len), _p(ids), _p(meta), _p(out_tok), out_tok.shape[1], _p(alive), _stream())


def grammar_sample_step(logits, state, targets, keep, reject, cls, src_len, ids, meta, out_tok, mt,
                        ctl, *, eos, m0, trash_pos, max_span=100, ring=None):
    """The sampled grammar step (smer_grammar_sample_step): mt uint32 [625]
    (numpy MT19937 key + position, updated in place), ctl int32 [3]; with
    `ring` (pinned host int32 [n]) the live count lands in ring[step % n],
    else in ctl[0]."""
    R, nst = state.shape
    V = keep.shape[1]
    for t, dt in ((state, torch.int32), (targets, torch.int8), (keep, torch.uint8),
                  (reject, torch.uint8), (cls, torch.uint8), (src_len, torch.int32),
                  (ids, torch.int64), (meta, torch.int32), (out_tok, torch.int32),
                  (mt, torch.int32), (ctl, torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise RuntimeError("grammar_sample_step: expected contiguous %s" % dt)
    if logits.shape[0] < 2 * R or ids.shape[0] != 2 * R or meta.shape != (4, 2 * R) or \
            targets.shape[0] != R or keep.shape[0] != 13 or reject.shape != keep.shape or \
            cls.shape[0] != V or src_len.shape[0] != R or mt.numel() < 625 or ctl.numel() < 3:
        raise RuntimeError("grammar_sample_step: shape mismatch")
    if ring is not None and (ring.dtype != torch.int32 or not ring.is_pinned()):
        raise RuntimeError("grammar_sample_step: ring must be pinned int32")
    call("smer_grammar_sample_step", R, V, _p(logits), _ld(logits), _p(state), nst, _p(targets),
         targets.shape[1], _p(keep), _p(reject), _p(cls), int(eos), int(m0), int(trash_pos),
         int(max_span), _p(src_len), _p(ids), _p(meta), _p(out_tok), out_tok.shape[1], _p(mt),
         _p(ctl), ring.data_ptr() if ring is not None else None, ring.numel() if ring is not None else 0,
         _stream())


# ---------------------------------------------------------------------------
def layernorm(x, gamma, beta, y, mean, rstd, eps=1e-5):
    M, N = x.shape
    call("smer_layernorm_fwd", dtype_code(x.dtype), M, N, _p(x), _ld(x), _p(gamma), _p(beta),
         float(eps), _p(y), _ld(y), _p(mean), _p(rstd), _stream())


def layernorm_bwd(dy, x, mean, rstd, gamma, dx, *, dx_drop=None, drop_p=0.0, seed=0,
                  dgamma=None, dbeta=None, accumulate=True, param_stream=None, q8=None, qs=None,
                  amax=None):
    """param_stream: run the dgamma / dbeta column reduction on that stream
    (after this stream's LayerNorm kernel), off the dgrad chain.  q8 (bf16
    only): also the e4m3 copy e4m3(g * qs) of the gradient g that feeds the
    next dgrad (the dropped gradient when drop_p > 0, else dx), max|g| folded
    into amax; with q8, drop_p > 0 and no dx_drop that gradient exists only
    as its copy."""
    lib = load()
    M, N = x.shape
    nbytes = lib.smer_layernorm_bwd_workspace(M, N) if (dgamma is not None or dbeta is not None) else 0
    ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=x.device)
    if q8 is not None:
        if x.dtype != torch.bfloat16 or dy.dtype != torch.bfloat16:
            raise RuntimeError("layernorm_bwd: the e4m3 copy needs bf16 dy and x")
        partial = param_stream is not None and nbytes > 0
        call("smer_layernorm_bwd_fp8", M, N, _p(dy), _ld(dy), _p(x), _ld(x), _p(mean), _p(rstd),
             _p(gamma), _p(dx), _ld(dx), _p(dx_drop), _ld(dx_drop) if dx_drop is not None else 0,
             float(drop_p), int(seed) & 0xFFFFFFFF, _p(q8), _ld(q8), _p(qs), _p(amax),
             _p(None if partial else dgamma), _p(None if partial else dbeta), int(accumulate),
             _p(ws), nbytes, int(partial), _stream())
        if partial:
            param_stream.wait_stream(torch.cuda.current_stream(x.device))
            with torch.cuda.stream(param_stream):
                call("smer_layernorm_param_reduce", M, N, _p(ws), nbytes, _p(dgamma), _p(dbeta),
                     int(accumulate), _stream())
            ws.record_stream(param_stream)
        return
    if param_stream is not None and nbytes:
        call("smer_layernorm_bwd_partials", dtype_code(x.dtype), M, N, _p(dy), _ld(dy),
             int(dy.dtype == torch.float32 and x.dtype != torch.float32), _p(x), _ld(x), _p(mean),
             _p(rstd), _p(gamma), _p(dx), _ld(dx), _p(dx_drop),
             _ld(dx_drop) if dx_drop is not None else 0, float(drop_p), int(seed) & 0xFFFFFFFF,
             _p(ws), nbytes, _stream())
        param_stream.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(param_stream):
            call("smer_layernorm_param_reduce", M, N, _p(ws), nbytes, _p(dgamma), _p(dbeta),
                 int(accumulate), _stream())
        ws.record_stream(param_stream)
        return
    call("smer_layernorm_bwd", dtype_code(x.dtype), M, N, _p(dy), _ld(dy),
         int(dy.dtype == torch.float32 and x.dtype != torch.float32), _p(x), _ld(x), _p(mean),
         _p(rstd), _p(gamma), _p(dx), _ld(dx), _p(dx_drop),
         _ld(dx_drop) if dx_drop is not None else 0, float(drop_p), int(seed) & 0xFFFFFFFF,
         _p(dgamma), _p(dbeta), int(accumulate), _p(ws), nbytes, _stream())


def embed(ids, table, pe, out, *, L=0, positions=None, scale, drop_p=0.0, seed=0):
    n_tok = ids.numel()
    d = table.shape[1]
    call("smer_embed_fwd", dtype_code(out.dtype), n_tok, d, _p(ids), _p(positions), int(L),
         _p(table), _p(pe), float(scale), float(drop_p), int(seed) & 0xFFFFFFFF, _p(out),
         _ld(out), _stream())


def embed_fp8(ids, table, pe, out, q8, qs, amax, *, L=0, positions=None, scale, drop_p=0.0, seed=0):
    """embed (bf16 out) plus the e4m3 copy q8 = e4m3(out * qs), max |out|
    folded into amax (the fp8 step's first-layer QKV input)."""
    n_tok = ids.numel()
    d = table.shape[1]
    call("smer_embed_fwd_fp8", n_tok, d, _p(ids), _p(positions), int(L), _p(table), _p(pe), float(scale),
         float(drop_p), int(seed) & 0xFFFFFFFF, _p(out), _ld(out), _p(q8), _ld(q8), _p(qs), _p(amax), _stream())


def embed_bwd(dtable, scale, segs):
    """segs: list of up to two (ids int64 [n], dx [n, d], drop_p, seed)."""
    lib = load()
    V, d = dtable.shape
    segs = list(segs) + [(None, None, 0.0, 0)] * (2 - len(segs))
    (i0, x0, p0, s0), (i1, x1, p1, s1) = segs
    n0 = i0.numel() if i0 is not None else 0
    n1 = i1.numel() if i1 is not None else 0
    dt = dtype_code((x0 if x0 is not None else x1).dtype)
    nbytes = lib.smer_embed_bwd_workspace(V, d, n0 + n1)
    ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=dtable.device)
    call("smer_embed_bwd", dt, V, d, float(scale), _p(i0), _p(x0),
         _ld(x0) if x0 is not None else 0, n0, float(p0), int(s0) & 0xFFFFFFFF, _p(i1), _p(x1),
         _ld(x1) if x1 is not None else 0, n1, float(p1), int(s1) & 0xFFFFFFFF, _p(dtable),
         _p(ws), nbytes, _stream())


def wce_denom(y, ce_all, denom):
    call("smer_wce_denom", y.numel(), _p(y), _p(ce_all), _p(denom), _stream())


def wce_fwd_bwd(logits, y, w, denom, row_loss, loss_out=None, dlogits=None, *, V=None,
                grad_scale=1.0):
    R = logits.shape[0]
    Vv = V if V is not None else logits.shape[1]
    dt = dtype_code(dlogits.dtype) if dlogits is not None else F32
    call("smer_wce_fwd_bwd", dt, R, Vv, _p(logits), _ld(logits), _p(y), _p(w), _p(denom),
         _p(row_loss), _p(loss_out), _p(dlogits), _ld(dlogits) if dlogits is not None else 0,
         float(grad_scale), _stream())


def argmax_accuracy(logits, y, cls, ncls, pad, counts):
    """counts[2c], counts[2c+1] += rows / argmax hits of token class c (and
    the total in the last pair) over the rows whose target is not `pad`
    (smer_argmax_accuracy; train.py:988-1034)."""
    R, V = logits.shape
    if y.dtype != torch.int64 or cls.dtype != torch.int32 or counts.dtype != torch.int32:
        raise TypeError("argmax_accuracy: int64 targets, int32 class table and counts")
    if counts.numel() < 2 * ncls + 2:
        raise ValueError("argmax_accuracy: counts needs 2 * ncls + 2 entries")
    call("smer_argmax_accuracy", R, V, _p(logits), _ld(logits), _p(y), _p(cls), int(ncls), int(pad),
         _p(counts), _stream())


def adam(p, g, m, v, p_bf16, *, lr, b1, b2, eps, step):
    import math
    bc1 = 1.0 - b1 ** step
    bc2s = math.sqrt(1.0 - b2 ** step)
    call("smer_adam", p.numel(), _p(p), _p(g), _p(m), _p(v), _p(p_bf16), float(lr), float(b1),
         float(b2), float(eps), float(bc1), float(bc2s), _stream())


def cast(src, dst):
    assert src.numel() == dst.numel()
    call("smer_cast", dtype_code(src.dtype), dtype_code(dst.dtype), src.numel(), _p(src),
         _p(dst), _stream())


def cast2d(src, dst, *, rows=None, cols=None):
    r = rows if rows is not None else src.shape[0]
    c = cols if cols is not None else src.shape[1]
    call("smer_cast2d", dtype_code(src.dtype), dtype_code(dst.dtype), r, c, _p(src), _ld(src),
         _p(dst), _ld(dst), _stream())


def colsum(x, out, *, N=None, accumulate=True):
    lib = load()
    M = x.shape[0]
    Nn = N if N is not None else x.shape[1]
    nbytes = lib.smer_colsum_workspace(M, Nn)
    ws = torch.empty(max(1, nbytes), dtype=torch.uint8, device=x.device)
    call("smer_colsum", dtype_code(x.dtype), M, Nn, _p(x), _ld(x), _p(out), int(accumulate),
         _p(ws), nbytes, _stream())
