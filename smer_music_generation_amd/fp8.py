"""fp8 (OCP e4m3) training forward with delayed per-tensor scaling.

BASELINE.json configs[3] (C4) asks for fp8 MFMA GEMMs on CDNA4.  In the
`precision="fp8"` mode the forward contractions whose input comes from a
LayerNorm run on the block-scaled fp8 MFMA (`smer_gemm_fp8`): the QKV
in-projections of layers >= 1, FFN1, the decoder's cross-attention Q and the
stacked cross-attention K/V of the memory (`transformer.py:389,393,459,463,
467`); FFN2, whose input FFN1 writes in e4m3 beside its bf16 output
(engine.FP8_FFN2, on since round 6), and the attention
out-projections, whose input the attention forward writes in e4m3 beside O
(FP8_ATTN_OUT).  The vocab head stays bf16; master weights fp32, working
weights bf16.

Backward (FP8_DGRAD): the dgrad products whose input gradient comes from a
LayerNorm backward, the FFN2 dgrad or the attention backward run as
e4m3(dY) . e4m3(W^T)^T on the same kernel: FFN2 dgrad (ReLU gate in the
epilogue, writing the e4m3 copy of dh), FFN1 dgrad (residual), the attention
out-projection dgrads, and the QKV / cross-Q dgrads (the attention
backward kernels write dQ / dK / dV's e4m3 copies, round 3).  Producers
write the gradient's e4m3 copy beside its bf16 output; scales are delayed
like the forward's (the amax recorded in step t - 1), so a backward site
switches to fp8 once it has one step of history (the first step's backward
is bf16).  W^T copies are quantised with the forward copies, once per
optimizer step.  The memory dgrad (K = 12 * 2d) reads one e4m3 copy of
every layer's cross-attention dK | dV under a single scale site (shared with
the cross dQ copies).  Weight gradients (FP8_WGRAD, round 6): dW =
e4m3(dY)^T e4m3(X) wherever both copies exist (all but the first layers'
QKV, and FFN2's without engine.FP8_FFN2), through the
transposing 8-bit LDS reads of smer_gemm_wgrad_fp8; the bias gradient from
the same e4m3 dY.

Scaling (no standalone quantise pass over activations):
  * every producer (LayerNorm, the FFN1 epilogue) writes an e4m3 copy
    q = e4m3(y * qs) beside its bf16 output and folds max|y| into an amax
    slot of this forward (atomicMax on float bits);
  * qs for forward t comes from the amax recorded in forward t-1
    (`smer_fp8_scales`: qs = 448 / amax, inv = amax / 448); a site with no
    recorded amax yet (the first forward) still writes its copy and amax but
    its consumer GEMM runs bf16 (`record_fwd`), as the backward sites do;
  * weights are quantised once per optimizer step (current scaling: amax of
    the new weights, then the cast), all of them in one batched call
    (`smer_fp8_quantize_segments`: a memset + 2 launches per step), into
    persistent e4m3 buffers, and reused until the next update.
"""
from __future__ import annotations

import os

import torch

from . import ops

N_SITES = 512
# fp8 backward dgrads (SMER_FP8_DGRAD=0: bf16 backward, A/B and tests)
FP8_DGRAD = os.environ.get("SMER_FP8_DGRAD", "1") != "0"
# ... including the QKV / cross-Q dgrads fed by the attention backward
# (SMER_FP8_ATTN_DGRAD=0: those stay bf16, A/B)
FP8_ATTN_DGRAD = os.environ.get("SMER_FP8_ATTN_DGRAD", "1") != "0"
# fp8 attention out-projections in the forward: the attention kernel writes
# the e4m3 copy of its output (SMER_FP8_ATTN_OUT=0: bf16, A/B)
FP8_ATTN_OUT = os.environ.get("SMER_FP8_ATTN_OUT", "1") != "0"
# fp8 weight gradients dW = e4m3(dY)^T e4m3(X) (and db from the same e4m3
# dY) wherever both copies exist: the backward's dY copies above and the
# forward's X copies (LayerNorm outputs, attention outputs, FFN1's output
# with engine.FP8_FFN2) (SMER_FP8_WGRAD=0: bf16 weight gradients, A/B)
FP8_WGRAD = os.environ.get("SMER_FP8_WGRAD", "1") != "0"

# forward contraction groups that run on the fp8 MFMA (tests / tools switch
# groups off to measure each one's numerical effect): "qkv" self-attention
# in-projections, "cross" the cross-attention Q and stacked K/V projections,
# "ffn" FFN1 (and FFN2 with engine.FP8_FFN2), "out" the attention
# out-projections (with FP8_ATTN_OUT)
FWD_GROUPS = set(g for g in os.environ.get("SMER_FP8_FWD", "qkv,cross,ffn,out").split(",") if g)


def fwd_group(wname):
    """Forward group of an fp8 weight name (see gemm_weights)."""
    tail = wname.split(".")[-1]
    if tail in ("in", "sa"):
        return "qkv"
    if tail in ("cq", "ckv") or wname == "ckv":
        return "cross"
    if tail in ("l1", "l2"):
        return "ffn"
    return "out"


class Fp8Forward:
    def __init__(self, engine, device):
        self.eng = engine
        self.dev = device
        self.sites = {}
        self.amax = [torch.zeros(N_SITES, dtype=torch.int32, device=device) for _ in range(2)]
        self.qs = torch.ones(N_SITES, device=device)
        self.inv = torch.ones(N_SITES, device=device)
        self.t = 0
        self.cur = self.amax[1]
        # amax sink of eval / no-grad forwards: written, never turned into scales
        self._eval_amax = torch.zeros(N_SITES, dtype=torch.int32, device=device)
        self.trained = False
        self._wkey = None
        self._w = {}
        self._wbuf = {}       # name -> (e4m3 buffer, inv view), persistent
        self._seg = None      # (key, device seg table, amax workspace, inv)
        self._wt = {}         # name -> (e4m3 W^T buffer, inv view), persistent
        self._segt = None
        self._bwd_recorded = set()  # backward sites whose amax this step records
        self.bwd_ready = set()      # ... recorded in an earlier step: scales valid
        self._fwd_recorded = set()  # forward site indices whose amax this forward records
        self.fwd_ready = set()      # ... recorded by an earlier calibrating forward

    def begin(self, W=None, training=True):
        """Start a forward: this forward's scales from the previous one's
        amax; after a weight update, re-quantise every fp8 weight of W.
        Once a training forward has run, only training forwards advance the
        scale history: an eval / no-grad forward (validation) reuses the
        current scales and records its amax into a sink that never feeds a
        scale.  Before the first training forward (an inference-only model)
        every forward advances it, which calibrates the scales.
        A non-finite activation makes its site's amax +inf (the producers map
        NaN to inf in the amax and pass NaN through the e4m3 cast), so
        `finite()` turns false after a diverged forward."""
        calibrate = training or not self.trained
        self.trained = self.trained or training
        if calibrate:
            self.bwd_ready |= self._bwd_recorded
            self._bwd_recorded = set()
            self.fwd_ready |= self._fwd_recorded
            self._fwd_recorded = set()
            prev, nxt = self.amax[self.t % 2], self.amax[(self.t + 1) % 2]
            ops.fp8_scales(prev, self.qs, self.inv, nxt)
            self.cur = nxt
            self.t += 1
        else:
            self.cur = self._eval_amax
        if W is not None and self.eng._wgen != self._wkey:
            self._quantize_weights(W)

    @staticmethod
    def gemm_weights(W):
        """(name, bf16 weight) of every GEMM that runs on the fp8 MFMA."""
        out = []
        for i, L in enumerate(W.enc):
            out += [("enc%d.in" % i, L.in_w), ("enc%d.l1" % i, L.l1_w), ("enc%d.l2" % i, L.l2_w)]
            if FP8_ATTN_OUT:
                out.append(("enc%d.out" % i, L.out_w))
        for i, L in enumerate(W.dec):
            out += [("dec%d.sa" % i, L.sa_w), ("dec%d.cq" % i, L.cq_w), ("dec%d.l1" % i, L.l1_w),
                    ("dec%d.l2" % i, L.l2_w)]
            if FP8_ATTN_OUT:
                out += [("dec%d.sao" % i, L.sa_ow), ("dec%d.cao" % i, L.ca_ow)]
        if getattr(W, "ckv_all", None) is not None:
            out.append(("ckv", W.ckv_all))
        return out

    @staticmethod
    def dgrad_weights(W):
        """(name, bf16 weight [out, in]) of every dgrad that runs on the fp8
        MFMA (as e4m3(dY) . e4m3(W^T)^T)."""
        out = []
        for i, L in enumerate(W.enc):
            out += [("enc%d.in" % i, L.in_w), ("enc%d.out" % i, L.out_w), ("enc%d.l1" % i, L.l1_w),
                    ("enc%d.l2" % i, L.l2_w)]
        for i, L in enumerate(W.dec):
            out += [("dec%d.sa" % i, L.sa_w), ("dec%d.sao" % i, L.sa_ow), ("dec%d.cq" % i, L.cq_w),
                    ("dec%d.cao" % i, L.ca_ow), ("dec%d.l1" % i, L.l1_w), ("dec%d.l2" % i, L.l2_w)]
        if getattr(W, "ckv_all", None) is not None:
            out.append(("ckv", W.ckv_all))
        return out

    def _quantize_weights_t(self, W):
        ws = [(n, w) for n, w in self.dgrad_weights(W)
              if w.is_contiguous() and w.dim() == 2 and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0]
        key = tuple((n, w.data_ptr(), tuple(w.shape)) for n, w in ws)
        if self._segt is None or self._segt[0] != key:
            rows = []
            for n, w in ws:
                buf = self._wt.get(n)
                if buf is None or buf[0].shape != (w.shape[1], w.shape[0]):
                    buf = (torch.empty(w.shape[1], w.shape[0], dtype=torch.uint8, device=self.dev), None)
                rows.append((w.data_ptr(), buf[0].data_ptr(), w.shape[0], w.shape[1]))
                self._wt[n] = buf
            host = torch.tensor(rows, dtype=torch.int64).pin_memory() if rows else None
            seg = (torch.empty_like(host, device=self.dev).copy_(host, non_blocking=True)
                   if rows else None)
            inv = torch.ones(max(1, len(ws)), device=self.dev)
            amax_ws = torch.zeros(max(1, len(ws)), dtype=torch.int32, device=self.dev)
            self._segt = (key, seg, amax_ws, inv, host)
            self._wt = {n: (self._wt[n][0], inv[k:k + 1]) for k, (n, _) in enumerate(ws)}
        _, seg, amax_ws, inv, _ = self._segt
        if seg is not None:
            ops.fp8_quantize_segments_t(seg, amax_ws, inv)

    def weight_t(self, name):
        """(e4m3 W^T, inv scale) of a dgrad weight, or None."""
        return self._wt.get(name)

    def record_bwd(self, name):
        """A backward producer wrote site `name`'s amax this step."""
        self._bwd_recorded.add(name)

    def record_fwd(self, i):
        """A forward producer wrote site i's amax into this forward's slot.
        Returns whether site i's scale is delayed-scaling valid now, i.e. an
        earlier calibrating forward recorded its amax.  A site without that
        history (the first training forward, a new site) feeds a bf16 GEMM
        instead of its e4m3 copy: no forward contraction ever runs on the
        unit scale (qs = 1) of a site whose range was never measured."""
        if self.cur is not self._eval_amax:
            self._fwd_recorded.add(i)
        return i in self.fwd_ready

    def _quantize_weights(self, W):
        ws = [(n, w) for n, w in self.gemm_weights(W) if w.is_contiguous() and w.numel() % 8 == 0]
        key = tuple((n, w.data_ptr(), w.numel()) for n, w in ws)
        if self._seg is None or self._seg[0] != key:
            rows = []
            for n, w in ws:
                buf = self._wbuf.get(n)
                if buf is None or buf.shape != w.shape:
                    buf = torch.empty(w.shape, dtype=torch.uint8, device=self.dev)
                    self._wbuf[n] = buf
                rows.append((w.data_ptr(), buf.data_ptr(), w.numel()))
            host = torch.tensor(rows, dtype=torch.int64).pin_memory()
            seg = torch.empty_like(host, device=self.dev).copy_(host, non_blocking=True)
            inv = torch.ones(len(ws), device=self.dev)
            amax_ws = torch.zeros(len(ws), dtype=torch.int32, device=self.dev)
            self._seg = (key, seg, amax_ws, inv, host)
        _, seg, amax_ws, inv, _ = self._seg
        ops.fp8_quantize_segments(seg, amax_ws, inv)
        self._w = {n: (self._wbuf[n], inv[k:k + 1]) for k, (n, _) in enumerate(ws)}
        if FP8_DGRAD:
            self._quantize_weights_t(W)
        self._wkey = self.eng._wgen

    def finite(self):
        """Device bool: every amax of the last training forward is finite
        (the bits of +inf / NaN sort above every finite float)."""
        last = self.amax[self.t % 2]
        return (last < 0x7F800000).all()

    def site(self, name):
        i = self.sites.get(name)
        if i is None:
            i = len(self.sites)
            if i >= N_SITES:
                raise RuntimeError("fp8: more than %d scaled activations" % N_SITES)
            self.sites[name] = i
        return i

    def qs_of(self, i):
        return self.qs[i:i + 1]

    def inv_of(self, i):
        return self.inv[i:i + 1]

    def amax_of(self, i):
        return self.cur[i:i + 1]

    def weight(self, name, w):
        """(e4m3 copy, inv scale) of a bf16 working weight, refreshed whenever
        the engine's weights change (after every optimizer step)."""
        key = self.eng._wgen
        if key != self._wkey:
            self._w = {}
            self._wkey = key
        hit = self._w.get(name)
        if hit is None or hit[0].shape != w.shape:
            q = torch.empty(w.shape, dtype=torch.uint8, device=w.device)
            inv = torch.empty(1, device=w.device)
            ops.fp8_quantize(w, q, inv)
            hit = (q, inv)
            self._w[name] = hit
        return hit


def eligible(M, N, K):
    """Shapes the fp8 MFMA kernel tiles (256 x 256 outputs, 128-deep K)."""
    return M % 256 == 0 and N % 256 == 0 and K % 128 == 0
