"""KV-cached, batched incremental decoder for the infill loop.

The reference re-runs the whole encoder over S source tokens and the whole
decoder over the t-token prefix for EVERY generated token
(`generation.py:542-545` -> `model_generate`, `generation.py:209-225`).
Here, per request:
  * prefill: the encoder runs once; every decoder layer's cross-attention
    K/V of the memory (`transformer.py:463`) is computed once into a cache;
  * step: only the new token(s) go through the decoder; their self-attention
    K/V are appended to a per-layer cache that persists ACROSS spans (the
    prefix accumulates, `generation.py:686`), positions continue.
Mathematically identical to the full recompute (causal attention: earlier
positions never see later tokens); fp32 mode reproduces the reference logits
to ~1e-6 and its greedy token ids exactly.

Fixed-shape step: every request owns TWO row slots per step (a feed is one
token, or two right after a control span: the control token + the next
m_0).  Unused slots are dummies that write their K/V into a reserved trash
position (Tmax-1, never attended).  The step shape is therefore constant and
is captured ONCE into a HIP graph (torch.cuda.CUDAGraph drives stream
capture; every kernel is a libsmer_hip.so launch on the captured stream) and
replayed per token: one H2D of the row table, one replay, one D2H.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from . import ops


def _capture(stream, fn):
    """Capture fn()'s launches on `stream` into a HIP graph.  Not the
    torch.cuda.graph context manager: its __enter__ empties the caching
    allocator (hipFree of every cached segment -- 40-140 ms after a training
    step had filled the cache, the whole cold-call capture cost in the
    round-3 bench), which a decode step allocating a few small buffers in
    the graph's private pool does not need."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        g.capture_begin()
        try:
            fn()
        finally:
            g.capture_end()
    return g


class DecodeSession:
    def __init__(self, model, max_requests, max_src, max_tgt, precision=None, use_graph=True):
        if precision is not None:
            model.set_precision(precision)
        self.model = model
        self.eng = model.engine
        eng = self.eng
        self.dt = eng.act_dtype()
        dev = model.flat_parameters().device
        if dev.type != "cuda":
            raise RuntimeError("DecodeSession needs the model on a ROCm GPU")
        self.dev = dev
        self.R, self.Smax = int(max_requests), int(max_src)
        self.Tmax = int(max_tgt) + 1  # + trash slot
        d = eng.d
        self.d = d
        if max(self.Smax, self.Tmax) > model.pos_enc.pe.shape[0]:
            model.pos_enc.extend(max(self.Smax, self.Tmax))
        self.self_kv = [torch.zeros(self.R, self.Tmax, 2 * d, dtype=self.dt, device=dev)
                        for _ in range(eng.n_dec)]
        # cross-attention memory, head-major [R, K|V, H, Smax, D]: each
        # (request, head) streams one contiguous key run per decode step
        H, D = eng.H, eng.D
        self.cross_kv = [torch.zeros(self.R, 2, H, self.Smax, D, dtype=self.dt, device=dev)
                         for _ in range(eng.n_dec)]
        self.src_len = np.zeros(self.R, dtype=np.int64)
        self.W = eng.weights(self.dt)
        # static step buffers: 2 slots per request
        M = 2 * self.R
        self.M = M
        self.ids_t = torch.zeros(M, dtype=torch.int64, device=dev)
        self.meta_t = torch.zeros(4, M, dtype=torch.int32, device=dev)
        self.ids_h = torch.zeros(M, dtype=torch.int64).pin_memory()
        self.meta_h = torch.zeros(4, M, dtype=torch.int32).pin_memory()
        self.logits_h = torch.zeros(M, eng.V, dtype=torch.float32).pin_memory()
        self.use_graph = use_graph
        self.graph = None
        # step(): the row-table H2D and logits D2H copies inside the step graph
        self._graph_copies = os.environ.get("SMER_DECODE_GRAPH_COPY", "1") == "1"
        self.logits_t = None
        # the positional table the captured graphs address (pos_enc.extend()
        # by a later session reallocates it: _pe_guard drops stale graphs)
        self._pe_ptr = model.pos_enc.pe.data_ptr()

    def _pe_guard(self):
        """Drop the captured step / greedy graphs when the model's
        positional table moved since they were captured (another session's
        pos_enc.extend() freed the buffer they read)."""
        ptr = self.model.pos_enc.pe.data_ptr()
        if ptr != self._pe_ptr:
            self.graph = None
            self._greedy = None
            self._pe_ptr = ptr

    def refresh_weights(self):
        self.W = self.eng.weights(self.dt)
        self.graph = None

    # ------------------------------------------------------------------
    def prefill(self, slots, srcs):
        """Encode `srcs` (list of 1-D int arrays) into request `slots`."""
        eng, W, dt, dev, d = self.eng, self.W, self.dt, self.dev, self.d
        H, D = eng.H, eng.D
        B = len(slots)
        lens = [len(s) for s in srcs]
        S = max(lens)
        if S > self.Smax:
            raise ValueError("source length %d exceeds session max_src %d" % (S, self.Smax))
        src = np.zeros((B, S), dtype=np.int64)
        for b, s in enumerate(srcs):
            src[b, :len(s)] = np.asarray(s, dtype=np.int64)
        src_t = torch.from_numpy(src).to(dev)
        kpm = None
        if min(lens) != S:
            kpm = torch.from_numpy((np.arange(S)[None, :] >= np.array(lens)[:, None]).astype(np.uint8)).to(dev)
        pe = self.model.pos_enc.pe
        pe2 = pe.view(pe.shape[0], pe.shape[2])
        x = torch.empty(B * S, d, dtype=dt, device=dev)
        ops.embed(src_t.view(-1), W.emb, pe2, x, L=S, scale=math.sqrt(d))
        scale = 1.0 / math.sqrt(D)
        for L in W.enc:
            qkv = ops.linear(x, L.in_w, L.in_b)
            o = torch.empty(B * S, d, dtype=dt, device=dev)
            lse = torch.empty(B, H, S, device=dev)
            ops.attn_fwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, lse, B=B, H=H, Lq=S,
                         Lk=S, D=D, kpm=kpm, causal=False, scale=scale)
            y1 = ops.linear(o, L.out_w, L.out_b, residual=x)
            x1, _, _ = eng._ln(y1, L.n1, dt)
            h = ops.linear(x1, L.l1_w, L.l1_b, relu=True)
            y2 = ops.linear(h, L.l2_w, L.l2_b, residual=x1)
            x, _, _ = eng._ln(y2, L.n2, dt)
        mem, _, _ = eng._ln(x, W.enc_norm, dt)
        # all B*S memory rows go to the caches (rows past a source's length
        # land beyond its src_len and are never attended)
        req = np.repeat(np.asarray(slots, dtype=np.int32), S)
        pos = np.tile(np.arange(S, dtype=np.int32), B)
        req_t = torch.from_numpy(req).to(dev)
        pos_t = torch.from_numpy(pos).to(dev)
        for li, L in enumerate(W.dec):
            kvc = ops.linear(mem, L.ckv_w, L.ckv_b)
            ops.kv_scatter_heads(kvc, self.cross_kv[li], req_t, pos_t, H=H, D=D,
                                 req_stride=2 * H * self.Smax * D, kv_stride=H * self.Smax * D,
                                 head_stride=self.Smax * D)
        for b, s in enumerate(slots):
            self.src_len[s] = lens[b]

    # ------------------------------------------------------------------
    def _run(self):
        """The fixed-shape decoder step on the static buffers."""
        eng, W, dt, dev, d = self.eng, self.W, self.dt, self.dev, self.d
        H, D, M = eng.H, eng.D, self.M
        pos_t, req_t, nks_t, nkc_t = self.meta_t[0], self.meta_t[1], self.meta_t[2], self.meta_t[3]
        pe = self.model.pos_enc.pe
        pe2 = pe.view(pe.shape[0], pe.shape[2])
        x = torch.empty(M, d, dtype=dt, device=dev)
        ops.embed(self.ids_t, W.emb, pe2, x, positions=pos_t, scale=math.sqrt(d))
        scale = 1.0 / math.sqrt(D)
        sstride = self.Tmax * 2 * d
        cstride = 2 * H * self.Smax * D
        # the fused fp32 layers need the LayerNorm-prologue Linear's limits
        # (K = d_model a multiple of 8, at most 2048); other widths unfused
        if (dt == torch.float32 and M <= 64 and d % 8 == 0 and d <= 2048
                and os.environ.get("SMER_DECODE_F32_FUSED", "1") == "1"):
            if self.logits_t is None:
                self.logits_t = torch.empty(M, eng.V, device=dev)
            self._run_fused_layers_f32(x, scale, sstride, cstride)
            return
        fused = dt == torch.bfloat16
        if fused:
            if self.logits_t is None:
                self.logits_t = torch.empty(M, eng.V, device=dev)
            chains = self._chains()
            if chains == 1:
                self._run_fused_layers(x, scale, sstride, cstride, 0, M)
                return
            # Two independent request halves on two streams (graph branches),
            # meant to overlap one half's HBM-bound cross attention with the
            # other half's latency-bound Linears.  Every kernel computes a row
            # the same way whatever rows share its launch (logits bit-identical
            # either way).
            h = 2 * (self.R // 2)
            main = torch.cuda.current_stream(dev)
            side = self._side_stream()
            side.wait_stream(main)
            self._run_fused_layers(x, scale, sstride, cstride, 0, h)
            with torch.cuda.stream(side):
                self._run_fused_layers(x, scale, sstride, cstride, h, M)
            main.wait_stream(side)
            return
        for li, L in enumerate(W.dec):
            cache = self.self_kv[li]
            qkv = ops.linear(x, L.sa_w, L.sa_b)
            ops.kv_scatter(qkv[:, d:], cache, req_t, pos_t, row_stride=2 * d, req_stride=sstride)
            o = torch.empty(M, d, dtype=dt, device=dev)
            ops.attn_decode(qkv[:, :d], cache, cache.view(-1)[d:], req_t, nks_t, o, H=H, D=D,
                            row_stride=2 * d, req_stride=sstride, scale=scale)
            y1 = ops.linear(o, L.sa_ow, L.sa_ob, residual=x)
            x1, _, _ = eng._ln(y1, L.n1, dt)
            qc = ops.linear(x1, L.cq_w, L.cq_b)
            cc = self.cross_kv[li]
            oc = torch.empty(M, d, dtype=dt, device=dev)
            ops.attn_decode(qc, cc, cc.view(-1)[H * self.Smax * D:], req_t, nkc_t, oc, H=H, D=D,
                            row_stride=D, req_stride=cstride, head_stride=self.Smax * D,
                            scale=scale)
            y2 = ops.linear(oc, L.ca_ow, L.ca_ob, residual=x1)
            x2, _, _ = eng._ln(y2, L.n2, dt)
            h = ops.linear(x2, L.l1_w, L.l1_b, relu=True)
            y3 = ops.linear(h, L.l2_w, L.l2_b, residual=x2)
            x, _, _ = eng._ln(y3, L.n3, dt)
        out, _, _ = eng._ln(x, W.dec_norm, dt)
        logits = torch.empty(M, eng.V, device=dev) if self.logits_t is None else self.logits_t
        ops.gemm(out, W.fc_w, M=M, N=eng.V, K=d, out_f32=logits, bias=W.fc_b, dtype=dt)
        self.logits_t = logits

    def _chains(self):
        """Request chains per decode step.  SMER_DECODE_CHAINS=2 splits the
        requests into two halves on two graph branches; measured slower
        (C2 364 vs 326 us per replay, C5 888 vs 871: tools/decode_chain_probe.py),
        so one chain is the default."""
        if self.R < 2:
            return 1
        return 2 if os.environ.get("SMER_DECODE_CHAINS", "1") == "2" else 1

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.dev)
        return self._side

    def _run_fused_layers(self, x, scale, sstride, cstride, r0, r1):
        """bf16 decoder step with every post-norm LayerNorm fused into the
        prologue of the Linear that consumes it (ops.linear_decode_ln: LN1 ->
        cross Q, LN2 -> FFN1, LN3 -> next layer's QKV, final norm -> vocab
        head; the LN output is also stored as the next residual), the cross
        query projection computed inside the cross-attention blocks, and the
        new K/V appended by the QKV epilogue: 7 launches per layer (11 in
        round 1)."""
        eng, W, dt, dev, d = self.eng, self.W, self.dt, self.dev, self.d
        H, D, M = eng.H, eng.D, r1 - r0
        pos_t, req_t, nks_t, nkc_t = (self.meta_t[0, r0:r1], self.meta_t[1, r0:r1],
                                      self.meta_t[2, r0:r1], self.meta_t[3, r0:r1])
        x = x[r0:r1]
        # The in-attention query projection re-reads the head's Wq slice per
        # (row, head) block: 329 vs 342 us per replayed step at R = 32, 484
        # vs 480 at R = 64 (tools/decode_host_probe.py).  It rounds q in a
        # different order than the Linear, so the choice must not depend on
        # the batch (a request's tokens may not depend on its batch-mates):
        # on whenever the shape allows it.
        self._qln = D == 64 and d in (512, 768, 1024) and os.environ.get("SMER_DECODE_QLN", "1") == "1"
        y_prev = n_prev = None
        for li, L in enumerate(W.dec):
            cache = self.self_kv[li]
            kv = dict(kv=cache, kv_req=req_t, kv_pos=pos_t, kv_row_stride=2 * d,
                      kv_req_stride=sstride, kv_col0=d)
            if y_prev is None:  # layer 0: x is the embedding (no norm in front)
                qkv = ops.linear_decode(x, L.sa_w, L.sa_b, **kv)
            else:
                x = torch.empty(M, d, dtype=dt, device=dev)
                qkv = ops.linear_decode_ln(y_prev, n_prev[0], n_prev[1], L.sa_w, L.sa_b, x_out=x, **kv)
            o = torch.empty(M, d, dtype=dt, device=dev)
            ops.attn_decode(qkv[:, :d], cache, cache.view(-1)[d:], req_t, nks_t, o, H=H, D=D,
                            row_stride=2 * d, req_stride=sstride, scale=scale)
            y1 = ops.linear(o, L.sa_ow, L.sa_ob, residual=x)
            x1 = torch.empty(M, d, dtype=dt, device=dev)
            cc = self.cross_kv[li]
            oc = torch.empty(M, d, dtype=dt, device=dev)
            if self._qln:  # LN1 + cross Q inside the cross-attention blocks
                ops.attn_decode_qln(y1, L.n1[0], L.n1[1], L.cq_w, L.cq_b, cc,
                                    cc.view(-1)[H * self.Smax * D:], req_t, nkc_t, oc, H=H, D=D,
                                    row_stride=D, req_stride=cstride, head_stride=self.Smax * D,
                                    scale=scale, x_out=x1)
            else:
                qc = ops.linear_decode_ln(y1, L.n1[0], L.n1[1], L.cq_w, L.cq_b, x_out=x1)
                ops.attn_decode(qc, cc, cc.view(-1)[H * self.Smax * D:], req_t, nkc_t, oc, H=H, D=D,
                                row_stride=D, req_stride=cstride, head_stride=self.Smax * D,
                                scale=scale)
            y2 = ops.linear(oc, L.ca_ow, L.ca_ob, residual=x1)
            x2 = torch.empty(M, d, dtype=dt, device=dev)
            h = ops.linear_decode_ln(y2, L.n2[0], L.n2[1], L.l1_w, L.l1_b, relu=True, x_out=x2)
            y_prev = ops.linear(h, L.l2_w, L.l2_b, residual=x2)
            n_prev = L.n3
        x, _, _ = eng._ln(y_prev, n_prev, dt)  # last LN3; the final norm feeds the head below
        ops.linear_decode_ln(x, W.dec_norm[0], W.dec_norm[1], W.fc_w, W.fc_b,
                             out_f32=self.logits_t[r0:r1])

    def _run_fused_layers_f32(self, x, scale, sstride, cstride):
        """fp32 (parity-mode) decoder step, 8 launches per layer instead of 12:
        the post-norm LayerNorms run in the prologue of the Linear that
        consumes them (ops.linear_decode_ln: LN3 -> next QKV, LN1 -> cross Q,
        LN2 -> FFN1, final norm -> vocab head; the LN output also stored as
        the next residual, the LayerNorm kernel's bits) and the QKV epilogue
        appends the new K/V to the cache (no kv_scatter launch).  Every
        operand fp32; the attention and the plain Linears as in _run."""
        eng, W, dt, dev, d = self.eng, self.W, self.dt, self.dev, self.d
        H, D, M = eng.H, eng.D, self.M
        pos_t, req_t, nks_t, nkc_t = self.meta_t[0], self.meta_t[1], self.meta_t[2], self.meta_t[3]
        # cross attention as flash-decoding (8 key slices per (row, head),
        # merged in the out-projection's prologue): the unsplit form runs
        # 2 * R * H blocks, 16 at batch 1
        self._split_f32 = D == 64 and d <= 2048 and os.environ.get("SMER_DECODE_SPLIT_F32", "1") == "1"
        # few rows (batch 1-2): LN1 + the cross-attention query projection
        # computed inside the split attention blocks (one launch fewer per
        # layer; each block re-reads its head's 128 KB of Wq from L2, so not
        # for many rows)
        qln = self._split_f32 and d == 512 and M <= 4 and os.environ.get("SMER_DECODE_QLN_F32", "1") == "1"
        y_prev = n_prev = None
        for li, L in enumerate(W.dec):
            cache = self.self_kv[li]
            kv = dict(kv=cache, kv_req=req_t, kv_pos=pos_t, kv_row_stride=2 * d,
                      kv_req_stride=sstride, kv_col0=d)
            if y_prev is None:  # layer 0: x is the embedding (no norm in front)
                qkv = ops.linear_decode(x, L.sa_w, L.sa_b, **kv)
            else:
                x = torch.empty(M, d, dtype=dt, device=dev)
                qkv = ops.linear_decode_ln(y_prev, n_prev[0], n_prev[1], L.sa_w, L.sa_b, x_out=x, **kv)
            # (the self attention stays unsplit: its <= ~400-key caches
            # measured 0.306 vs 0.296 ms per step split)
            o = torch.empty(M, d, dtype=dt, device=dev)
            ops.attn_decode(qkv[:, :d], cache, cache.view(-1)[d:], req_t, nks_t, o, H=H, D=D,
                            row_stride=2 * d, req_stride=sstride, scale=scale)
            y1 = ops.linear(o, L.sa_ow, L.sa_ob, residual=x)
            x1 = torch.empty(M, d, dtype=dt, device=dev)
            cc = self.cross_kv[li]
            if qln:
                part = torch.empty(M, H, ops.DEC_SPLITS, 68, device=dev)
                ops.attn_decode_split_qln_f32(y1, L.n1[0], L.n1[1], L.cq_w, L.cq_b, cc,
                                              cc.view(-1)[H * self.Smax * D:], req_t, nkc_t, part, H=H, D=D,
                                              row_stride=D, req_stride=cstride, head_stride=self.Smax * D,
                                              scale=scale, x_out=x1)
                y2 = ops.linear_decode_merge_f32(part, L.ca_ow, L.ca_ob, M=M, residual=x1)
            elif self._split_f32:  # 8 key slices per (row, head), merged by the out-projection
                qc = ops.linear_decode_ln(y1, L.n1[0], L.n1[1], L.cq_w, L.cq_b, x_out=x1)
                part = torch.empty(M, H, ops.DEC_SPLITS, 68, device=dev)
                ops.attn_decode_split_f32(qc, cc, cc.view(-1)[H * self.Smax * D:], req_t, nkc_t, part, H=H,
                                          D=D, row_stride=D, req_stride=cstride, head_stride=self.Smax * D,
                                          scale=scale)
                y2 = ops.linear_decode_merge_f32(part, L.ca_ow, L.ca_ob, M=M, residual=x1)
            else:
                qc = ops.linear_decode_ln(y1, L.n1[0], L.n1[1], L.cq_w, L.cq_b, x_out=x1)
                oc = torch.empty(M, d, dtype=dt, device=dev)
                ops.attn_decode(qc, cc, cc.view(-1)[H * self.Smax * D:], req_t, nkc_t, oc, H=H, D=D,
                                row_stride=D, req_stride=cstride, head_stride=self.Smax * D, scale=scale)
                y2 = ops.linear(oc, L.ca_ow, L.ca_ob, residual=x1)
            x2 = torch.empty(M, d, dtype=dt, device=dev)
            h = ops.linear_decode_ln(y2, L.n2[0], L.n2[1], L.l1_w, L.l1_b, relu=True, x_out=x2)
            y_prev = ops.linear(h, L.l2_w, L.l2_b, residual=x2)
            n_prev = L.n3
        x, _, _ = eng._ln(y_prev, n_prev, dt)  # last LN3; the final norm feeds the head below
        ops.linear_decode_ln(x, W.dec_norm[0], W.dec_norm[1], W.fc_w, W.fc_b, out_f32=self.logits_t)

    def _ensure_graph(self):
        if self.graph is not None or not self.use_graph:
            return
        # warm up eagerly once (allocator, library load), then capture; the
        # step graph also holds the row-table H2D copies and the logits D2H
        # copy (memcpy nodes: no separate copy launches per token)
        self._run()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        if self._graph_copies:
            self.graph = _capture(s, self._run_with_copies)
        else:
            self.graph = _capture(s, self._run)
        torch.cuda.current_stream().wait_stream(s)

    def _run_with_copies(self):
        self.ids_t.copy_(self.ids_h, non_blocking=True)
        self.meta_t.copy_(self.meta_h, non_blocking=True)
        self._run()
        self.logits_h.copy_(self.logits_t, non_blocking=True)

    def _load_feeds(self, feeds, copy=True):
        """Host-built step rows: feeds = [(slot, new_token_ids (1 or 2),
        first_position)]; every other row is a dummy into the trash slot.
        Returns the rows of each feed's last token.  copy=False: the pinned
        host rows only (the captured step graph copies them itself)."""
        Tm = self.Tmax
        ids = self.ids_h.numpy()
        meta = self.meta_h.numpy()
        ids[:] = 0
        slots = np.arange(self.M, dtype=np.int32) // 2
        meta[0] = Tm - 1           # dummy rows -> trash position
        meta[1] = slots
        meta[2] = 1                # dummy rows attend one key
        meta[3] = 1
        last = []
        for slot, toks, p0 in feeds:
            n = len(toks)
            if n > 2:
                raise ValueError("a feed carries at most 2 new tokens")
            if p0 + n > Tm - 1:
                raise ValueError("decoder prefix exceeds session max_tgt %d" % (Tm - 1))
            r0 = 2 * slot + (2 - n)
            for k in range(n):
                ids[r0 + k] = int(toks[k])
                meta[0, r0 + k] = p0 + k
                meta[2, r0 + k] = p0 + k + 1
                meta[3, r0 + k] = max(int(self.src_len[slot]), 1)
            last.append(2 * slot + 1)
        if copy:
            self.ids_t.copy_(self.ids_h, non_blocking=True)
            self.meta_t.copy_(self.meta_h, non_blocking=True)
        return last

    def step(self, feeds):
        """feeds: list of (slot, new_token_ids (1 or 2), first_position).
        Returns fp32 logits [len(feeds), V] (numpy) of each feed's LAST new
        token.  Slots not fed this step are dummies."""
        self._pe_guard()
        if self.use_graph:
            # the first call's eager warm-up reads the device row tables
            first = self.graph is None
            last = self._load_feeds(feeds, copy=first or not self._graph_copies)
            self._ensure_graph()
            self.graph.replay()
            if not self._graph_copies:
                self.logits_h.copy_(self.logits_t, non_blocking=True)
            torch.cuda.current_stream().synchronize()
            return self.logits_h.numpy()[last]
        last = self._load_feeds(feeds)
        self._run()
        self.logits_h.copy_(self.logits_t, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return self.logits_h.numpy()[last]

    # ------------------------------------------------------------------
    # greedy decode with the grammar on device (csrc/decode_ops.hip)
    # ------------------------------------------------------------------
    N_STATE = 12

    def _capture_greedy(self, st, tg, keep, cls, cap, nm, eos, m0, lookahead, max_span, use_ring,
                        sample=False):
        """Persistent grammar buffers + the captured (decoder step + grammar)
        graph, reused by later greedy_decode calls of the same shapes."""
        dev = self.dev
        self.g_state = torch.from_numpy(st).to(dev)
        self.g_targets = torch.from_numpy(tg).to(dev)
        self.g_keep = torch.from_numpy(np.ascontiguousarray(keep, dtype=np.uint8)).to(dev)
        self.g_cls = torch.from_numpy(np.ascontiguousarray(cls, dtype=np.uint8)).to(dev)
        self.g_srclen = torch.from_numpy(self.src_len.astype(np.int32)).to(dev)
        self.g_out = torch.zeros(self.R, cap, dtype=torch.int32, device=dev)
        # live counts: the step's grammar kernel publishes its count into a
        # pinned host ring itself (no per-step memset / D2H copy between the
        # replays); SMER_GRAMMAR_RING=0: memset + copy per step (A/B)
        ring = torch.zeros(2 * lookahead + 2, dtype=torch.int32).pin_memory()
        rv = ring.numpy()
        self.g_alive = torch.zeros(3 if use_ring else 1, dtype=torch.int32, device=dev)
        gargs = dict(eos=eos, m0=m0, trash_pos=self.Tmax - 1, max_span=max_span,
                     ring=ring if use_ring else None)

        def grammar():
            if sample:
                ops.grammar_sample_step(self.logits_t, self.g_state, self.g_targets, self.g_keep,
                                        self.g_reject, self.g_cls, self.g_srclen, self.ids_t,
                                        self.meta_t, self.g_out, self.g_mt, self.g_alive, **gargs)
                return
            ops.grammar_greedy_step(self.logits_t, self.g_state, self.g_targets, self.g_keep,
                                    self.g_cls, self.g_srclen, self.ids_t, self.meta_t, self.g_out,
                                    self.g_alive, **gargs)

        # warm the decoder step eagerly (dummy rows only), then capture
        # step + grammar; the grammar kernel never runs outside the graph
        t_a = time.perf_counter()
        self._load_feeds([])
        self._run()
        torch.cuda.synchronize()
        t_b = time.perf_counter()
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        g = _capture(gs, lambda: (self._run(), grammar()))
        torch.cuda.current_stream().wait_stream(gs)
        torch.cuda.synchronize()
        t_c = time.perf_counter()
        return g, ring, rv, t_a, t_b, t_c

    def sampled_decode(self, spans, keep, reject, cls, *, eos, m0, lookahead=3, max_span=100):
        """The sampled infill loop (the reference's default weighted_sampling
        with its redraws) on device: each step is one replay of the captured
        decoder step + csrc/decode_ops.hip grammar_sample_kernel, which draws
        from numpy's global MT19937 stream -- its state is handed to the
        device here and handed back to np.random afterwards, so the host
        stream continues exactly as if the host had drawn.  Returns
        (per-request emitted ids, steps, error flags, per-request redraw
        failure flags)."""
        if all(sp.done for sp in spans):  # nothing to draw: np.random stays untouched
            return [[] for _ in spans], 0, np.zeros(len(spans), dtype=np.int32), [[] for _ in spans]
        st0 = np.random.get_state()
        if st0[0] != "MT19937":
            raise RuntimeError("sampled_decode: np.random is not MT19937")
        mt_h = np.empty(625, dtype=np.uint32)
        mt_h[:624] = st0[1]
        mt_h[624] = int(st0[2])
        res = self._grammar_decode(spans, keep, cls, eos=eos, m0=m0, lookahead=lookahead,
                                   max_span=max_span, sample=(reject, mt_h))
        m = self.g_mt.cpu().numpy().view(np.uint32)
        np.random.set_state(("MT19937", m[:624].copy(), int(m[624]), st0[3], st0[4]))
        ids, steps, err, step_ms = res
        fails = [[(x >> 16) & 1 for x in q] for q in ids]
        return [[x & 0xFFFF for x in q] for q in ids], steps, err, fails

    def greedy_decode(self, spans, keep, cls, *, eos, m0, lookahead=3, max_span=100):
        return self._grammar_decode(spans, keep, cls, eos=eos, m0=m0, lookahead=lookahead,
                                    max_span=max_span)

    def _grammar_decode(self, spans, keep, cls, *, eos, m0, lookahead=3, max_span=100, sample=None):
        """Run the greedy infill loop of `spans` (generation._Span, one per
        request slot 0..len-1, freshly started, sources prefilled) entirely
        on device: each step is one replay of the captured decoder step +
        grammar kernel; the host only polls the live count, `lookahead`
        steps behind.  Returns (per-request emitted ids, steps, error flags);
        the caller replays the ids through its host spans."""
        R = len(spans)
        if R > self.R:
            raise ValueError("more spans than session slots")
        self._pe_guard()
        dev = self.dev
        # mask-target table capacity: a power of two >= 16, so calls whose
        # requests have different mask counts replay the same captured graph
        # (a capture costs ~10 ms; the kernels read the table by its row
        # stride, which is the capacity)
        need = max(1, max(s.n_masks for s in spans))
        nm = 16
        while nm < need:
            nm *= 2
        cap = self.Tmax
        st = np.zeros((self.R, self.N_STATE), dtype=np.int32)
        tg = np.zeros((self.R, nm), dtype=np.int8)
        from .generation import _target_code  # late import: generation imports decode
        feeds = []
        for r, sp in enumerate(spans):
            st[r, 2] = 1                      # this_in = [m_0]
            st[r, 4] = sp.n_masks
            st[r, 5] = 1 if sp.done else 0
            st[r, 6] = int(bool(sp.no_whole))
            for k, t in enumerate(sp.mask_target[:nm]):
                tg[r, k] = _target_code(t)
            if not sp.done:
                st[r, 0] = 1                  # m_0 is fed at position 0 below
                feeds.append((r, [m0], 0))
        st[R:, 5] = 1
        if not feeds:
            return [[] for _ in range(R)], 0, np.zeros(R, dtype=np.int32), []
        use_ring = os.environ.get("SMER_GRAMMAR_RING", "1") != "0" or sample is not None
        gkey = (nm, int(max_span), int(eos), int(m0), int(lookahead), use_ring, keep.shape, cls.shape,
                sample is not None)
        gc = getattr(self, "_greedy", None)
        if sample is not None:
            reject_t = torch.from_numpy(np.ascontiguousarray(sample[0], dtype=np.uint8))
            mt_t = torch.from_numpy(sample[1].view(np.int32))
            if getattr(self, "g_mt", None) is None:
                self.g_mt = torch.zeros(625, dtype=torch.int32, device=dev)
            if getattr(self, "g_reject", None) is None or tuple(self.g_reject.shape) != tuple(keep.shape):
                # (a captured graph keyed on another keep shape is never replayed for this one)
                self.g_reject = torch.zeros(keep.shape, dtype=torch.uint8, device=dev)
            self.g_mt.copy_(mt_t)
            self.g_reject.copy_(reject_t)
        if gc is not None and gc["key"] == gkey:
            # the captured step + grammar graph of an earlier call with the
            # same shapes: refresh its persistent inputs in place and replay
            t_a = t_b = time.perf_counter()
            self.eng.weights(self.dt)  # re-casts the bf16 weights in place if they moved
            self.g_state.copy_(torch.from_numpy(st))
            self.g_targets.copy_(torch.from_numpy(tg))
            self.g_keep.copy_(torch.from_numpy(np.ascontiguousarray(keep, dtype=np.uint8)))
            self.g_cls.copy_(torch.from_numpy(np.ascontiguousarray(cls, dtype=np.uint8)))
            self.g_srclen.copy_(torch.from_numpy(self.src_len.astype(np.int32)))
            self.g_out.zero_()
            self.g_alive.zero_()
            g, ring = gc["graph"], gc["ring"]
            ring.zero_()
            rv = ring.numpy()
            torch.cuda.synchronize()
            t_c = time.perf_counter()
        else:
            g, ring, rv, t_a, t_b, t_c = self._capture_greedy(st, tg, keep, cls, cap, nm, eos, m0,
                                                             lookahead, max_span, use_ring,
                                                             sample is not None)
            self._greedy = {"key": gkey, "graph": g, "ring": ring}
        self._load_feeds(feeds)
        max_steps = max([s.n_masks for s in spans] + [0]) * (max_span + 1) + 2
        inflight = []
        events = []
        steps = None
        issued = 0
        ev_start = torch.cuda.Event(enable_timing=True)
        ev_start.record()
        while steps is None:
            if len(inflight) > lookahead or (issued >= max_steps and inflight):
                j, ev, slot = inflight.pop(0)
                ev.synchronize()
                if rv[slot] == 0:
                    steps = j + 1
                    break
                continue
            if issued >= max_steps:
                raise RuntimeError("greedy_decode: no convergence within %d steps" % max_steps)
            g.replay()
            slot = issued % len(rv)
            if not use_ring:
                ring[slot:slot + 1].copy_(self.g_alive, non_blocking=True)
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            events.append(ev)
            inflight.append((issued, ev, slot))
            issued += 1
        torch.cuda.synchronize()
        t_d = time.perf_counter()
        # host seconds of this call's phases (bench / probes)
        self.phase_s = {"warm_s": t_b - t_a, "capture_s": t_c - t_b, "loop_s": t_d - t_c}
        st = self.g_state.cpu().numpy()
        out = self.g_out.cpu().numpy()
        ids = [out[r, :min(int(st[r, 7]), cap)].tolist() for r in range(R)]
        step_ms = [ev_start.elapsed_time(e) for e in events[:steps]]
        return ids, steps, st[:R, 8].copy(), step_ms
