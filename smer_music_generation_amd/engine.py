"""Forward / backward schedule of the SMER encoder-decoder on gfx950 kernels.

Layout: activations are batch-major token rows [B*L, d] (row = b*L + i)
instead of the reference's seq-first [L, B, d] — the per-token math of
`transformer.py:378-470` is unchanged, only the row order differs, and
rows of one sequence are contiguous for the attention tiles.

Every op is a libsmer_hip.so call (see ops.py); torch provides tensors
(memory), the stream and autograd plumbing only.

Per encoder layer (transformer.py:389-395):
    qkv = x Wqkv^T + b                       smer_gemm
    o   = softmax(q k^T / sqrt(dh) + kpm) v  smer_attn_fwd   (dropout on P)
    y1  = x + drop(o Wo^T + bo)              smer_gemm (residual + dropout epilogue)
    x1  = LN1(y1)                            smer_layernorm_fwd
    h   = drop(relu(x1 W1^T + b1))           smer_gemm
    y2  = x1 + drop(h W2^T + b2)             smer_gemm
    x2  = LN2(y2)
Decoder layers add the causal self-attention and the cross-attention
(transformer.py:459-469); the final norms and the vocab head follow
(transformer.py:274-275, 329-330, model.py:106).
"""
from __future__ import annotations

import math
import os

import torch

from . import ops

_SITE = {"pe_src": 1, "pe_tgt": 2}


def _site(kind, layer, which):
    return 16 + (layer * 16 + which) * 2 + (0 if kind == "enc" else 1)


class _W:
    pass


# fp8 mode: FFN1 also writes the e4m3 copy of its ReLU output so that FFN2
# runs on the fp8 MFMA too, forward and weight gradient.  Round 2 measured
# that extra 1-byte stream costing the FFN1 epilogue more than FFN2 gained
# (the e4m3-copy products then ran the generic epilogue, one dependent HBM
# round trip per pass); round 6 moved them to the streamed epilogue and
# made the weight gradients fp8: C4 78.24-78.31 -> 77.74-77.76 ms.
# SMER_FP8_FFN2=0: FFN1 with a bf16 output only, FFN2 bf16 (A/B).
FP8_FFN2 = os.environ.get("SMER_FP8_FFN2", "1") == "1"
# SMER_FP8_EMBED=1: the embedding also writes an e4m3 copy so that the first
# encoder / decoder layers' QKV projections (forward, weight gradient) run
# fp8 too.  Off: C4 79.54 vs 79.37 ms mean over 7 interleaved runs (noise
# level) while the largest per-parameter gradient error of the C4 fp8 test
# rose 0.564 -> 0.641 (decoder layer 0's norm1; bound 0.65).
FP8_EMBED = os.environ.get("SMER_FP8_EMBED", "0") == "1"
# SMER_FP8_H8=1: once FFN1's e4m3 copy feeds FFN2 (its site has a scale
# history), FFN1 writes that copy alone, and the FFN2 dgrad takes its ReLU /
# dropout gate from the copy (smer_gemm_fp8_gate8) and writes only dh's e4m3
# copy when FFN1's weight gradient and dgrad both read it: no bf16 [tokens, F]
# tensor is written or read back (C4 79.43 -> 78.17 ms).  Likewise the
# LayerNorm backward's dropped gradients and the attention backward's dQKV,
# cross dQ and memory dK|dV (all: C4 78.70 -> 76.12 ms).  Needs the streamed
# e4m3-copy epilogue.
FP8_H8 = (os.environ.get("SMER_FP8_H8", "1") == "1"
          and os.environ.get("SMER_FP8_Q8_FAST", "1") != "0")


# Persistent-grid cap of the weight gradients on the side stream (workgroups;
# 0 = the whole chip): they then leave the other CUs to the dgrad /
# attention-backward chain (SMER_WGRAD_SIDE_CAP)
_WGRAD_SIDE_CAP = int(os.environ.get("SMER_WGRAD_SIDE_CAP", "0"))
# the same cap for the fp8 weight gradients only (SMER_WGRAD_FP8_CAP; -1 =
# SMER_WGRAD_SIDE_CAP's value).  192 of 256 CUs: C4 fp8 76.24 -> 75.45 ms
# (uncapped / 160 / 192 / 224: 76.24 / 76.18 / 75.45 / 76.28, 3 runs each)
_WGRAD_FP8_CAP = int(os.environ.get("SMER_WGRAD_FP8_CAP", "192"))
# attention-dropout keep words generated up front on a second stream
# (SMER_ATTN_MASK_PREGEN=1)
_ATTN_MASK_PREGEN = os.environ.get("SMER_ATTN_MASK_PREGEN", "0") == "1"


class Engine:
    def __init__(self, model):
        self.m = model
        self.d = model.d_model
        self.H = model.nhead
        self.D = self.d // self.H
        self.F = model.dim_feedforward
        self.V = model.vocab_size
        self.Vp = (self.V + 63) // 64 * 64
        self.n_enc = model.num_encoder_layers
        self.n_dec = model.num_decoder_layers
        self._bf16 = None
        self._bf16_version = None
        self._fc_pad = None
        self._wgen = 0          # bumped whenever the working weights are rewritten
        self._ckv_all = None    # (key, W [L*2d, d], b [L*2d]) stacked cross-attn K/V projections
        self._side = {}         # device -> (wgrad stream, its split-K workspace)
        self._mstream = {}      # device -> attention-mask generator stream
        self._fp8 = None        # fp8.Fp8Forward (precision "fp8")

    # ------------------------------------------------------------------
    def act_dtype(self):
        return torch.float32 if self.m.precision == "fp32" else torch.bfloat16

    def _weights_flat(self, dt):
        flat = self.m.flat_parameters()
        if dt == torch.float32:
            return flat
        ver = self._version_key()
        if self._bf16 is None or self._bf16.numel() != flat.numel() or self._bf16_version != ver:
            if self._bf16 is None or self._bf16.numel() != flat.numel():
                self._bf16 = torch.empty(flat.numel(), dtype=torch.bfloat16, device=flat.device)
            ops.cast(flat, self._bf16)
            self._fc_pad = None
            self._bf16_version = ver
            self._wgen += 1
        return self._bf16

    def _version_key(self):
        # parameters are .data-views of the flat buffer; in-place updates by
        # any optimizer bump the per-parameter version counters
        flat = self.m.flat_parameters()
        return (flat.data_ptr(), flat._version, sum(p._version for p in self.m.parameters()))

    def mark_bf16_fresh(self):
        """Called by the fused Adam, which rewrites the bf16 copy itself."""
        self._bf16_version = self._version_key()
        self._fc_pad = None
        self._wgen += 1

    def mark_params_updated(self):
        """The fp32 master was rewritten through a raw pointer (fused Adam):
        torch's version counters did not move, so invalidate every cached
        derivative of the weights (bf16 copy, stacked cross-attention K/V)."""
        self._bf16_version = None
        self._fc_pad = None
        self._wgen += 1

    def weights(self, dt):
        """Per-layer views of the working weights (bf16 copy or fp32 master);
        biases / norms always fp32 master."""
        work = self._weights_flat(dt)
        master = self.m.flat_parameters()
        off = self.m._offsets
        d, F, V = self.d, self.F, self.V

        def wv(name, shape):
            o = off[name]
            return work[o: o + math.prod(shape)].view(shape)

        def mv(name, n):
            o = off[name]
            return master[o: o + n]

        W = _W()
        W.emb = mv("embedding.weight", V * d).view(V, d)
        W.enc, W.dec = [], []
        for i in range(self.n_enc):
            p = "transformer.encoder.layers.%d" % i
            L = _W()
            L.in_w, L.in_b = wv(p + ".self_attn.in_proj_weight", (3 * d, d)), mv(p + ".self_attn.in_proj_bias", 3 * d)
            L.out_w, L.out_b = wv(p + ".self_attn.out_proj.weight", (d, d)), mv(p + ".self_attn.out_proj.bias", d)
            L.l1_w, L.l1_b = wv(p + ".linear1.weight", (F, d)), mv(p + ".linear1.bias", F)
            L.l2_w, L.l2_b = wv(p + ".linear2.weight", (d, F)), mv(p + ".linear2.bias", d)
            L.n1 = (mv(p + ".norm1.weight", d), mv(p + ".norm1.bias", d))
            L.n2 = (mv(p + ".norm2.weight", d), mv(p + ".norm2.bias", d))
            W.enc.append(L)
        W.enc_norm = (mv("transformer.encoder.norm.weight", d), mv("transformer.encoder.norm.bias", d))
        for i in range(self.n_dec):
            p = "transformer.decoder.layers.%d" % i
            L = _W()
            L.sa_w, L.sa_b = wv(p + ".self_attn.in_proj_weight", (3 * d, d)), mv(p + ".self_attn.in_proj_bias", 3 * d)
            L.sa_ow, L.sa_ob = wv(p + ".self_attn.out_proj.weight", (d, d)), mv(p + ".self_attn.out_proj.bias", d)
            ca = wv(p + ".multihead_attn.in_proj_weight", (3 * d, d))
            cb = mv(p + ".multihead_attn.in_proj_bias", 3 * d)
            L.cq_w, L.cq_b, L.ckv_w, L.ckv_b = ca[:d], cb[:d], ca[d:], cb[d:]
            L.ca_ow, L.ca_ob = wv(p + ".multihead_attn.out_proj.weight", (d, d)), mv(p + ".multihead_attn.out_proj.bias", d)
            L.l1_w, L.l1_b = wv(p + ".linear1.weight", (F, d)), mv(p + ".linear1.bias", F)
            L.l2_w, L.l2_b = wv(p + ".linear2.weight", (d, F)), mv(p + ".linear2.bias", d)
            L.n1 = (mv(p + ".norm1.weight", d), mv(p + ".norm1.bias", d))
            L.n2 = (mv(p + ".norm2.weight", d), mv(p + ".norm2.bias", d))
            L.n3 = (mv(p + ".norm3.weight", d), mv(p + ".norm3.bias", d))
            W.dec.append(L)
        W.dec_norm = (mv("transformer.decoder.norm.weight", d), mv("transformer.decoder.norm.bias", d))
        W.fc_w = wv("fc.weight", (V, d))
        W.fc_b = mv("fc.bias", V)
        # vocab head padded to Vp rows (zero rows) for the K = V dgrad
        if self._fc_pad is None or self._fc_pad.dtype != dt or self._fc_pad.device != work.device:
            self._fc_pad = torch.zeros(self.Vp, d, dtype=dt, device=work.device)
        ops.cast(W.fc_w.reshape(-1), self._fc_pad[:V].reshape(-1))
        W.fc_pad = self._fc_pad
        # The decoder's cross-attention K/V projections all read the encoder
        # memory: stacked [L*2d, d] they run as ONE GEMM in the forward
        # (memory -> every layer's K|V) and ONE dgrad GEMM (K = L*2d) in the
        # backward instead of L each.  Rebuilt when the weights change.
        key = (dt, work.data_ptr(), self._wgen, self._version_key())
        if self.n_dec and (self._ckv_all is None or self._ckv_all[0] != key):
            n2 = 2 * d
            if os.environ.get("SMER_CKV_REUSE", "1") == "1" and self._ckv_all is not None and self._ckv_all[1].dtype == dt and \
                    self._ckv_all[1].device == work.device and self._ckv_all[1].shape[0] == self.n_dec * n2:
                wall, ball = self._ckv_all[1], self._ckv_all[2]  # rewritten in place (stable pointers)
            else:
                wall = torch.empty(self.n_dec * n2, d, dtype=dt, device=work.device)
                ball = torch.empty(self.n_dec * n2, device=work.device)
            for i, L in enumerate(W.dec):
                ops.cast2d(L.ckv_w, wall[i * n2:(i + 1) * n2])
                ops.cast(L.ckv_b, ball[i * n2:(i + 1) * n2])
            self._ckv_all = (key, wall, ball)
        if self.n_dec:
            W.ckv_all, W.ckv_b_all = self._ckv_all[1], self._ckv_all[2]
        return W

    def grad_views(self):
        g = self.m.flat_grad()
        off = self.m._offsets
        d, F, V = self.d, self.F, self.V

        def gv(name, shape):
            o = off[name]
            return g[o: o + math.prod(shape)].view(shape)

        G = _W()
        G.emb = gv("embedding.weight", (V, d))
        G.enc, G.dec = [], []
        for i in range(self.n_enc):
            p = "transformer.encoder.layers.%d" % i
            L = _W()
            L.in_w, L.in_b = gv(p + ".self_attn.in_proj_weight", (3 * d, d)), gv(p + ".self_attn.in_proj_bias", (3 * d,))
            L.out_w, L.out_b = gv(p + ".self_attn.out_proj.weight", (d, d)), gv(p + ".self_attn.out_proj.bias", (d,))
            L.l1_w, L.l1_b = gv(p + ".linear1.weight", (F, d)), gv(p + ".linear1.bias", (F,))
            L.l2_w, L.l2_b = gv(p + ".linear2.weight", (d, F)), gv(p + ".linear2.bias", (d,))
            L.n1 = (gv(p + ".norm1.weight", (d,)), gv(p + ".norm1.bias", (d,)))
            L.n2 = (gv(p + ".norm2.weight", (d,)), gv(p + ".norm2.bias", (d,)))
            G.enc.append(L)
        G.enc_norm = (gv("transformer.encoder.norm.weight", (d,)), gv("transformer.encoder.norm.bias", (d,)))
        for i in range(self.n_dec):
            p = "transformer.decoder.layers.%d" % i
            L = _W()
            L.sa_w, L.sa_b = gv(p + ".self_attn.in_proj_weight", (3 * d, d)), gv(p + ".self_attn.in_proj_bias", (3 * d,))
            L.sa_ow, L.sa_ob = gv(p + ".self_attn.out_proj.weight", (d, d)), gv(p + ".self_attn.out_proj.bias", (d,))
            ca = gv(p + ".multihead_attn.in_proj_weight", (3 * d, d))
            cb = gv(p + ".multihead_attn.in_proj_bias", (3 * d,))
            L.cq_w, L.cq_b, L.ckv_w, L.ckv_b = ca[:d], cb[:d], ca[d:], cb[d:]
            L.ca_ow, L.ca_ob = gv(p + ".multihead_attn.out_proj.weight", (d, d)), gv(p + ".multihead_attn.out_proj.bias", (d,))
            L.l1_w, L.l1_b = gv(p + ".linear1.weight", (F, d)), gv(p + ".linear1.bias", (F,))
            L.l2_w, L.l2_b = gv(p + ".linear2.weight", (d, F)), gv(p + ".linear2.bias", (d,))
            L.n1 = (gv(p + ".norm1.weight", (d,)), gv(p + ".norm1.bias", (d,)))
            L.n2 = (gv(p + ".norm2.weight", (d,)), gv(p + ".norm2.bias", (d,)))
            L.n3 = (gv(p + ".norm3.weight", (d,)), gv(p + ".norm3.bias", (d,)))
            G.dec.append(L)
        G.dec_norm = (gv("transformer.decoder.norm.weight", (d,)), gv("transformer.decoder.norm.bias", (d,)))
        G.fc_w = gv("fc.weight", (V, d))
        G.fc_b = gv("fc.bias", (V,))
        return G

    # ------------------------------------------------------------------
    def _ln(self, x, wb, dt):
        M = x.shape[0]
        y = torch.empty_like(x)
        mean = torch.empty(M, device=x.device)
        rstd = torch.empty(M, device=x.device)
        ops.layernorm(x, wb[0], wb[1], y, mean, rstd)
        return y, mean, rstd

    # ---- fp8 forward helpers (precision "fp8"; see fp8.py) --------------
    def _ln_q(self, f8, x, wb, dt, site):
        """LayerNorm; with f8, also the e4m3 copy of y for an fp8 GEMM.
        Returns (y, mean, rstd, (y8, site index) or None)."""
        if f8 is None or site is None:
            return self._ln(x, wb, dt) + (None,)
        M, N = x.shape
        y = torch.empty_like(x)
        mean = torch.empty(M, device=x.device)
        rstd = torch.empty(M, device=x.device)
        si = f8.site(site)
        q = torch.empty(M, N, dtype=torch.uint8, device=x.device)
        ops.layernorm_fp8(x, wb[0], wb[1], y, mean, rstd, q, f8.qs_of(si), f8.amax_of(si))
        # no amax history yet: the copy only records this forward's range
        return y, mean, rstd, ((q, si) if f8.record_fwd(si) else None)

    @staticmethod
    def _embed_q(f8, ids, table, pe, out, L, scale, p, seed, site):
        """Embedding + PE; with f8 also its e4m3 copy for the first layer's
        QKV projection: returns (copy, site) or None (as _ln_q)."""
        if f8 is None or not FP8_EMBED or out.dtype != torch.bfloat16:
            ops.embed(ids, table, pe, out, L=L, scale=scale, drop_p=p, seed=seed)
            return None
        si = f8.site(site)
        q = torch.empty(out.shape, dtype=torch.uint8, device=out.device)
        ops.embed_fp8(ids, table, pe, out, q, f8.qs_of(si), f8.amax_of(si), L=L, scale=scale, drop_p=p, seed=seed)
        return (q, si) if f8.record_fwd(si) else None

    @staticmethod
    def _deq8(hq, f8):
        """bf16 values of an e4m3 copy (q, site) (a bf16 fallback's input
        when FFN1 kept only its copy; not on the fp8 step's path)."""
        return (hq[0].view(torch.float8_e4m3fn).float() * f8.inv_of(hq[1])).to(torch.bfloat16)

    @staticmethod
    def _ffn2_fp8(f8, M, w2, name):
        """Whether FFN2 (w2 [d, F]) runs on the fp8 MFMA whenever its input
        has a usable e4m3 copy (then FFN1 may write that copy alone)."""
        if f8 is None:
            return False
        from .fp8 import FWD_GROUPS, eligible, fwd_group
        return eligible(M, w2.shape[0], w2.shape[1]) and fwd_group(name) in FWD_GROUPS

    @staticmethod
    def _attn_q8(f8, o, site, D):
        """fp8 forward: (q8 argument of ops.attn_fwd, (e4m3 copy of o, site)
        or None) so that the out-projection reads the attention output in
        e4m3.  The copy instance is built for head dim 64 only; other head
        dims keep bf16 out-projections."""
        from .fp8 import FP8_ATTN_OUT
        if f8 is None or not FP8_ATTN_OUT or D != 64:
            return None, None
        si = f8.site(site)
        q = torch.empty(o.shape, dtype=torch.uint8, device=o.device)
        return (q, f8.qs_of(si), f8.amax_of(si)), ((q, si) if f8.record_fwd(si) else None)

    def _lin(self, f8, x, xq, wname, w, b, q_site=None, q_only=False, **epi):
        """x @ w^T + epilogue: on the fp8 MFMA when x has an e4m3 copy xq and
        the shape tiles, else bf16.  q_site: also write the e4m3 copy of the
        output (returns (out, (q, site)) — (out, None) when the FFN2 input
        copy is disabled, see FP8_FFN2).  q_only: the consumer runs fp8
        whenever the copy is usable, so then only the copy is written and out
        is None (FP8_H8)."""
        M, K = (x if x is not None else xq[0]).shape  # (x None: only the e4m3 copy exists)
        N = w.shape[0]
        adt, adev = (x.dtype, x.device) if x is not None else (torch.bfloat16, xq[0].device)
        if q_site is not None and not FP8_FFN2:
            return self._lin(f8, x, xq, wname, w, b, **epi), None
        if f8 is not None and xq is not None:
            from .fp8 import FWD_GROUPS, eligible, fwd_group
            if eligible(M, N, K) and epi.get("gate") is None and fwd_group(wname) in FWD_GROUPS:
                w8, winv = f8.weight(wname, w)
                if q_site is not None:
                    si = f8.site(q_site)
                    out = None if (q_only and FP8_H8 and si in f8.fwd_ready) else \
                        torch.empty(M, N, dtype=adt, device=adev)
                    q = torch.empty(M, N, dtype=torch.uint8, device=adev)
                    ops.gemm_fp8_q(xq[0], f8.inv_of(xq[1]), w8, winv, out, bias=b, q8=q,
                                   qs=f8.qs_of(si), amax=f8.amax_of(si), **epi)
                    return out, ((q, si) if f8.record_fwd(si) else None)
                out = torch.empty(M, N, dtype=adt, device=adev)
                ops.gemm_fp8(xq[0], f8.inv_of(xq[1]), w8, winv, out, bias=b, **epi)
                return out
        if x is None:
            raise RuntimeError("engine: %s has only an e4m3 input but did not run fp8" % wname)
        out = ops.linear(x, w, b, **epi)
        return (out, None) if q_site is not None else out

    def forward(self, src, tgt, src_kpm, tgt_kpm, mem_kpm, *, training, need_weights, save,
                seed=0):
        """Returns (logits fp32 [B*T, V], weights [L,B,T,S] or None, ctx)."""
        m = self.m
        dt = self.act_dtype()
        dev = src.device
        B, S = src.shape
        T = tgt.shape[1]
        d, H, D = self.d, self.H, self.D
        scale = 1.0 / math.sqrt(D)
        p_pos = float(m.pos_dropout) if training else 0.0
        p_tr = float(m.trans_dropout) if training else 0.0
        W = self.weights(dt)
        pe = m.pos_enc.pe
        if max(S, T) > pe.shape[0]:
            raise RuntimeError("sequence length %d exceeds max_seq_length %d" % (max(S, T), pe.shape[0]))
        pe2 = pe.view(pe.shape[0], pe.shape[2])
        src_ids = src.reshape(-1).contiguous().long()
        tgt_ids = tgt.reshape(-1).contiguous().long()
        skpm = src_kpm.to(torch.uint8).contiguous() if src_kpm is not None else None
        tkpm = tgt_kpm.to(torch.uint8).contiguous() if tgt_kpm is not None else None
        mkpm = mem_kpm.to(torch.uint8).contiguous() if mem_kpm is not None else None
        sd = lambda site: (seed * 1000003 + site) & 0xFFFFFFFF  # noqa: E731
        ctx = _W()
        ctx.B, ctx.S, ctx.T, ctx.dt, ctx.p_pos, ctx.p_tr, ctx.seed = B, S, T, dt, p_pos, p_tr, seed
        ctx.src_ids, ctx.tgt_ids, ctx.skpm, ctx.tkpm, ctx.mkpm = src_ids, tgt_ids, skpm, tkpm, mkpm
        ctx.enc, ctx.dec = [], []
        # fp8: the e4m3 copies of each layer's weight-gradient inputs X (None
        # where a site has no copy / no scale history yet)
        ctx.enc_q, ctx.dec_q = [], []
        # attention-dropout keep bits written by the forward, read by backward
        ctx.masks = {}
        keep_mask = save and p_tr > 0 and dt == torch.bfloat16

        # SMER_ATTN_MASK_PREGEN=1: every attention site's keep words are
        # generated up front on a second stream (VALU-only, beside the
        # forward's GEMMs) and the forwards read them instead of hashing
        pregen = {}
        if keep_mask and _ATTN_MASK_PREGEN:
            ms = self._mask_stream(dev)
            ms.wait_stream(torch.cuda.current_stream(dev))
            sites = [(("enc", i), S, S, sd(_site("enc", i, 0))) for i in range(self.n_enc)]
            for i in range(self.n_dec):
                sites += [(("dec", i), T, T, sd(_site("dec", i, 0))), (("cross", i), T, S, sd(_site("dec", i, 2)))]
            bufs = [ops.attn_drop_mask(B, H, Lq, Lk, dev) for _, Lq, Lk, _ in sites]  # main-stream blocks
            with torch.cuda.stream(ms):
                for (key, Lq, Lk, sdv), m_ in zip(sites, bufs):
                    ops.attn_drop_mask_gen(m_, B=B, H=H, Lq=Lq, Lk=Lk, drop_p=p_tr, seed=sdv)
                    ev = torch.cuda.Event()
                    ev.record(ms)
                    pregen[key] = (m_, ev)
            for m_ in bufs:
                m_.record_stream(ms)

        def amask(key, Lq, Lk):
            if not keep_mask:
                return None
            if key in pregen:
                m_, ev = pregen[key]
                torch.cuda.current_stream(dev).wait_event(ev)
                ctx.masks[key] = m_
                return m_
            m_ = ops.attn_drop_mask(B, H, Lq, Lk, dev)
            ctx.masks[key] = m_
            return m_

        f8 = None
        if m.precision == "fp8":
            if self._fp8 is None:
                from .fp8 import Fp8Forward
                self._fp8 = Fp8Forward(self, dev)
            f8 = self._fp8
            f8.begin(W, training=training)
        ctx.f8 = f8 if (training and save) else None
        x = torch.empty(B * S, d, dtype=dt, device=dev)
        # xq: e4m3 copy of each layer's input x (fp8 mode)
        xq = self._embed_q(f8, src_ids, W.emb, pe2, x, S, math.sqrt(d), p_pos, sd(_SITE["pe_src"]), "emb.src")
        for i, L in enumerate(W.enc):
            xq_in = xq
            qkv = self._lin(f8, x, xq, "enc%d.in" % i, L.in_w, L.in_b)
            o = torch.empty(B * S, d, dtype=dt, device=dev)
            lse = torch.empty(B, H, S, device=dev)
            q8, oq = self._attn_q8(f8, o, "enc%d.o" % i, D)
            ops.attn_fwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, lse, B=B, H=H, Lq=S, Lk=S,
                         D=D, kpm=skpm, causal=False, scale=scale, drop_p=p_tr, seed=sd(_site("enc", i, 0)),
                         drop_mask=amask(("enc", i), S, S), drop_mask_in=bool(pregen), q8=q8)
            y1 = self._lin(f8, o, oq, "enc%d.out" % i, L.out_w, L.out_b, residual=x, drop_p=p_tr,
                           seed=sd(_site("enc", i, 1)))
            x1, m1, r1, x1q = self._ln_q(f8, y1, L.n1, dt, "enc%d.ln1" % i)
            h, hq = self._lin(f8, x1, x1q, "enc%d.l1" % i, L.l1_w, L.l1_b, q_site="enc%d.h" % i,
                              q_only=self._ffn2_fp8(f8, B * S, L.l2_w, "enc%d.l2" % i),
                              relu=True, drop_p=p_tr, seed=sd(_site("enc", i, 2)))
            y2 = self._lin(f8, h, hq, "enc%d.l2" % i, L.l2_w, L.l2_b, residual=x1, drop_p=p_tr,
                           seed=sd(_site("enc", i, 3)))
            x2, m2, r2, xq = self._ln_q(f8, y2, L.n2, dt,
                                        "enc%d.ln2" % i if i + 1 < self.n_enc else None)
            if save:
                ctx.enc.append((x, qkv, o, lse, y1, m1, r1, x1, h, y2, m2, r2))
                ctx.enc_q.append((xq_in, oq, x1q, hq))
            x = x2
        mem, me, re, memq = self._ln_q(f8, x, W.enc_norm, dt, "mem")
        ctx.enc_last = (x, me, re)
        ctx.mem = mem
        ctx.memq = memq

        y = torch.empty(B * T, d, dtype=dt, device=dev)
        yq0 = self._embed_q(f8, tgt_ids, W.emb, pe2, y, T, math.sqrt(d), p_pos, sd(_SITE["pe_tgt"]), "emb.tgt")
        wts = torch.empty(self.n_dec, B, T, S, device=dev) if need_weights else None
        # every decoder layer's cross-attention K|V of the memory, one GEMM
        kvc_all = self._lin(f8, mem, memq, "ckv", W.ckv_all, W.ckv_b_all) if self.n_dec else None
        yq = yq0
        for i, L in enumerate(W.dec):
            yq_in = yq
            qkv = self._lin(f8, y, yq, "dec%d.sa" % i, L.sa_w, L.sa_b)
            o = torch.empty(B * T, d, dtype=dt, device=dev)
            lse = torch.empty(B, H, T, device=dev)
            q8, oq = self._attn_q8(f8, o, "dec%d.o" % i, D)
            ops.attn_fwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, lse, B=B, H=H, Lq=T, Lk=T,
                         D=D, kpm=tkpm, causal=True, scale=scale, drop_p=p_tr, seed=sd(_site("dec", i, 0)),
                         drop_mask=amask(("dec", i), T, T), drop_mask_in=bool(pregen), q8=q8)
            y1 = self._lin(f8, o, oq, "dec%d.sao" % i, L.sa_ow, L.sa_ob, residual=y, drop_p=p_tr,
                           seed=sd(_site("dec", i, 1)))
            x1, m1, r1, x1q = self._ln_q(f8, y1, L.n1, dt, "dec%d.ln1" % i)
            qc = self._lin(f8, x1, x1q, "dec%d.cq" % i, L.cq_w, L.cq_b)
            kvc = kvc_all[:, i * 2 * d:(i + 1) * 2 * d]
            oc = torch.empty(B * T, d, dtype=dt, device=dev)
            lsec = torch.empty(B, H, T, device=dev)
            q8, ocq = self._attn_q8(f8, oc, "dec%d.oc" % i, D)
            ops.attn_fwd(qc, kvc[:, :d], kvc[:, d:], oc, lsec, B=B, H=H, Lq=T, Lk=S, D=D, kpm=mkpm,
                         causal=False, scale=scale, drop_p=p_tr, seed=sd(_site("dec", i, 2)),
                         drop_mask=amask(("cross", i), T, S), drop_mask_in=bool(pregen), q8=q8)
            if need_weights:
                ops.attn_weights(qc, kvc[:, :d], lsec, wts[i], B=B, H=H, Lq=T, Lk=S, D=D, kpm=mkpm,
                                 scale=scale)
            y2 = self._lin(f8, oc, ocq, "dec%d.cao" % i, L.ca_ow, L.ca_ob, residual=x1, drop_p=p_tr,
                           seed=sd(_site("dec", i, 3)))
            x2, m2, r2, x2q = self._ln_q(f8, y2, L.n2, dt, "dec%d.ln2" % i)
            h, hq = self._lin(f8, x2, x2q, "dec%d.l1" % i, L.l1_w, L.l1_b, q_site="dec%d.h" % i,
                              q_only=self._ffn2_fp8(f8, B * T, L.l2_w, "dec%d.l2" % i),
                              relu=True, drop_p=p_tr, seed=sd(_site("dec", i, 4)))
            y3 = self._lin(f8, h, hq, "dec%d.l2" % i, L.l2_w, L.l2_b, residual=x2, drop_p=p_tr,
                           seed=sd(_site("dec", i, 5)))
            x3, m3, r3, yq = self._ln_q(f8, y3, L.n3, dt,
                                        "dec%d.ln3" % i if i + 1 < self.n_dec else None)
            if save:
                ctx.dec.append((y, qkv, o, lse, y1, m1, r1, x1, qc, kvc, oc, lsec, y2, m2, r2, x2,
                                h, y3, m3, r3))
                ctx.dec_q.append((yq_in, oq, x1q, ocq, x2q, hq))
            y = x3
        out, mo, ro = self._ln(y, W.dec_norm, dt)
        ctx.dec_last = (y, mo, ro)
        ctx.dec_out = out
        logits = torch.empty(B * T, self.V, device=dev)
        ops.gemm(out, W.fc_w, M=B * T, N=self.V, K=d, out_f32=logits, bias=W.fc_b, dtype=dt)
        return logits, wts, ctx

    # ------------------------------------------------------------------
    def _mask_stream(self, dev):
        ms = self._mstream.get(dev)
        if ms is None:
            ms = self._mstream[dev] = torch.cuda.Stream(device=dev)
        return ms

    def _wgrad_stream(self, dev, dt):
        """Weight gradients run on a second HIP stream, overlapping the
        dgrad / attention-backward chain on the main stream (they only feed
        the optimizer).  bf16 only; SMER_WGRAD_OVERLAP=0 serialises."""
        if dt != torch.bfloat16 or os.environ.get("SMER_WGRAD_OVERLAP", "1") == "0":
            return None
        side = self._side.get(dev)
        if side is None:
            side = (torch.cuda.Stream(device=dev),
                    torch.zeros(ops.SPLITK_WS_BYTES, dtype=torch.uint8, device=dev))  # zero split-K tickets
            self._side[dev] = side
        return side

    @staticmethod
    def _wgrad(side, dy, x, gw, q8=None, **kw):
        """dW (+ db) of one Linear, on the side stream when there is one.
        q8 = (dy e4m3, its inv scale, x e4m3, its inv scale): the fp8 weight
        gradient (smer_gemm_wgrad_fp8), bf16 when its shape does not tile."""
        def run(ws, cap):
            if q8 is not None and ops.linear_wgrad_fp8(q8[0], q8[1], q8[2], q8[3], gw, db=kw.get("db"),
                                                       accumulate=kw.get("accumulate", True), ws=ws,
                                                       max_wg=cap if (_WGRAD_FP8_CAP < 0 or ws is None)
                                                       else _WGRAD_FP8_CAP):
                return
            if x is None or dy is None:
                raise RuntimeError("engine: fp8 weight gradient declined with no bf16 input")
            ops.linear_wgrad(dy, x, gw, ws=ws, max_wg=cap, **kw)
        if side is None:
            run(None, 0)
            return
        stream, ws = side
        stream.wait_stream(torch.cuda.current_stream(side[1].device))
        with torch.cuda.stream(stream):
            run(ws, _WGRAD_SIDE_CAP)
            if ops.CK_LOG is not None:
                ops.ck("S:dW", gw)
                ops.ck("S:db", kw.get("db"))
                ops.ck("S:dy", dy)
                ops.ck("S:x", x)
        # temporaries freed on the main stream must not be reused before the
        # side stream has read them
        for t in (dy, x):
            if t is not None:
                t.record_stream(stream)
        if q8 is not None:
            q8[0].record_stream(stream)
            q8[2].record_stream(stream)

    @staticmethod
    def _join(side):
        if side is not None:
            torch.cuda.current_stream(side[0].device).wait_stream(side[0])

    @staticmethod
    def _hook(side, hook, name):
        """A layer's gradients are final: call hook(name) (GradBucketer issues
        that range's all-reduce).  With the weight-gradient stream, every
        gradient write of a layer range is queued on it (weight / bias
        gradients and the LayerNorm parameter reductions), so the hook runs
        with that stream current: the collective waits for the side stream
        only and the main stream's dgrad chain never joins it mid-backward
        (the overlap survives under DP).  The main stream joins once, at the
        end of backward."""
        if side is None:
            hook(name)
            return
        with torch.cuda.stream(side[0]):
            hook(name)

    def backward(self, ctx, dlog_pad, hook=None):
        """dlog_pad: [B*T, Vp] activation dtype (cols >= V zero).  Accumulates
        every parameter gradient into the flat grad buffer.  `hook(name)` is
        called after each layer's grads are final (DP bucket overlap)."""
        m = self.m
        dt = ctx.dt
        dev = dlog_pad.device
        B, S, T = ctx.B, ctx.S, ctx.T
        d, H, D, V = self.d, self.H, self.D, self.V
        scale = 1.0 / math.sqrt(D)
        p_tr = ctx.p_tr
        sd = lambda site: (ctx.seed * 1000003 + site) & 0xFFFFFFFF  # noqa: E731
        W = self.weights(dt)
        G = self.grad_views()
        Mt, Ms = B * T, B * S

        from .fp8 import FP8_ATTN_DGRAD, FP8_DGRAD, eligible
        f8 = ctx.f8 if FP8_DGRAD else None

        def ln_bwd(g_in, y_, mu, rs, wb, dx_, dxd_, seed_, gw, site):
            """LayerNorm backward; in fp8 mode also the e4m3 copy of the gradient
            feeding the next dgrad: returns (q8, site) once the site's scale has
            a step of history, else None."""
            kw = dict(dx_drop=dxd_ if p_tr > 0 else None, drop_p=p_tr, seed=seed_, dgamma=gw[0],
                      dbeta=gw[1], param_stream=ps)
            if f8 is None:
                ops.layernorm_bwd(g_in, y_, mu, rs, wb[0], dx_, **kw)
                if ops.CK_LOG is not None:
                    ops.ck("M:ln_in.g", g_in)
                    ops.ck("M:ln_in.y", y_)
                    ops.ck("M:ln_in.mu", mu)
                    ops.ck("M:ln_in.rs", rs)
                return None
            si = f8.site(site)
            q = torch.empty(y_.shape, dtype=torch.uint8, device=dev)
            ops.layernorm_bwd(g_in, y_, mu, rs, wb[0], dx_, q8=q, qs=f8.qs_of(si), amax=f8.amax_of(si), **kw)
            f8.record_bwd(site)
            return (q, si) if site in f8.bwd_ready else None

        def attn_q8(shape, site, parts):
            """e4m3 copy buffer of an attention-backward gradient [rows, cols]
            and the q8 argument of ops.attn_bwd; parts: column slices (dq, dk,
            dv) of the copy, None for a gradient without one.  Returns
            (q8 arg, gq for dgrad or None)."""
            if f8 is None or not FP8_ATTN_DGRAD:
                return None, None
            si = f8.site(site)
            buf = torch.empty(shape, dtype=torch.uint8, device=dev)
            views = [None if p is None else buf[:, p[0]:p[1]] for p in parts]
            f8.record_bwd(site)
            return (views[0], views[1], views[2], f8.qs_of(si), f8.amax_of(si)), \
                ((buf, si) if site in f8.bwd_ready else None)

        def dgrad(gq, g, wname, w, q_site=None, q_only=False, **epi):
            """g @ w; on the fp8 MFMA (e4m3(g) . e4m3(w^T)^T) when g has a usable
            e4m3 copy gq (g may then be None: only the copy exists).  q_site:
            also the e4m3 copy of the output; q_only: only that copy once it is
            usable (the bf16 output is then None, FP8_H8)."""
            M = (g if g is not None else gq[0]).shape[0]
            if gq is not None:
                wt = f8.weight_t(wname)
                if wt is not None and eligible(M, w.shape[1], w.shape[0]):
                    out = None if (q_only and q_site is not None and q_site in f8.bwd_ready) else \
                        torch.empty(M, w.shape[1], dtype=dt, device=dev)
                    if q_site is None:
                        if ops.gemm_fp8_ex(gq[0], f8.inv_of(gq[1]), wt[0], wt[1], out, **epi):
                            return out, None
                    else:
                        si = f8.site(q_site)
                        q = torch.empty(M, w.shape[1], dtype=torch.uint8, device=dev)
                        if ops.gemm_fp8_ex(gq[0], f8.inv_of(gq[1]), wt[0], wt[1], out, q8=q,
                                           qs=f8.qs_of(si), amax=f8.amax_of(si), **epi):
                            f8.record_bwd(q_site)
                            return out, ((q, si) if q_site in f8.bwd_ready else None)
            # bf16 (also whenever the fp8 kernel declined the shape: nothing launched)
            if g is None:
                raise RuntimeError("engine: %s dgrad has only an e4m3 input but did not run fp8" % wname)
            return ops.linear_dgrad(g, w, **epi), None

        # vocab head
        side = self._wgrad_stream(dev, dt)
        ps = side[0] if side is not None else None  # LayerNorm dgamma / dbeta reductions too
        wg_ = lambda *a, **kw: self._wgrad(side, *a, **kw)  # noqa: E731
        from .fp8 import FP8_WGRAD
        f8w = ctx.f8 if FP8_WGRAD else None

        def wg(dy_, x_, gw, dyq=None, xq=None, **kw):
            """weight gradient; on the fp8 MFMA when both operands have a
            usable e4m3 copy ((tensor, site) pairs)"""
            if f8w is not None and dyq is not None and xq is not None:
                kw["q8"] = (dyq[0], f8w.inv_of(dyq[1]), xq[0], f8w.inv_of(xq[1]))
            wg_(dy_, x_, gw, **kw)
        def ffn2_bwd(dyq, dyd, name, w2, GL, h, hq, q_site, xq1, name1):
            """FFN2's weight gradient and gated dgrad (returns dh, its e4m3
            copy).  h None: FFN1 kept only its e4m3 copy hq (FP8_H8); the gate
            then comes from the copy (smer_gemm_fp8_gate8), and bf16 values
            are rebuilt from it only where a bf16 fallback needs them.  dh
            itself is written only as its e4m3 copy when both of its
            consumers (FFN1's weight gradient with FFN1's input copy xq1, and
            FFN1's dgrad, weight name1) will read that copy."""
            gs = ops.drop_scale(p_tr)
            Mr = (dyd if dyd is not None else dyq[0]).shape[0]
            q_only = (FP8_H8 and f8 is not None and f8w is not None and xq1 is not None
                      and f8.weight_t(name1) is not None and eligible(Mr, w2.shape[0], w2.shape[1]))
            if h is None and not (f8 is not None and f8w is not None and dyq is not None
                                  and f8.weight_t(name) is not None):
                h = self._deq8(hq, ctx.f8)
            wg(dyd, h, GL.l2_w, dyq, hq, db=GL.l2_b)
            if h is not None:
                return dgrad(dyq, dyd, name, w2, q_site=q_site, q_only=q_only, gate=h, gate_scale=gs)
            wt = f8.weight_t(name)
            si = f8.site(q_site)
            M, N = Mr, w2.shape[1]
            out = None if (q_only and q_site in f8.bwd_ready) else torch.empty(M, N, dtype=dt, device=dev)
            q = torch.empty(M, N, dtype=torch.uint8, device=dev)
            if not ops.gemm_fp8_gate8(dyq[0], f8.inv_of(dyq[1]), wt[0], wt[1], hq[0], gs, out, q,
                                      f8.qs_of(si), f8.amax_of(si)):
                raise RuntimeError("engine: %s e4m3-gated dgrad declined its shape" % name)
            f8.record_bwd(q_site)
            return out, ((q, si) if q_site in f8.bwd_ready else None)

        def q_only_grad(xq_, name, w, site, dropped=True):
            """Whether the output gradient of Linear `name` (weight w [N, K],
            input copy xq_) may exist only as its e4m3 copy: its weight
            gradient and dgrad both read that copy (the LayerNorm backward's
            dropped gradient, dropped=True, or the attention backward's dQKV
            then is not written in bf16, FP8_H8)."""
            M = ctx.B * (ctx.S if name.startswith("enc") else ctx.T)
            return (FP8_H8 and (p_tr > 0 or not dropped) and f8 is not None and f8w is not None and xq_ is not None
                    and site in f8.bwd_ready and f8.weight_t(name) is not None
                    and eligible(M, w.shape[1], w.shape[0]) and w.shape[0] % 256 == 0 and M % 64 == 0)

        def dgrad_in(y_, xq_, name, w, site):
            """The LayerNorm backward's dropped-gradient buffer (None: copy only)."""
            if p_tr == 0:
                return None
            return None if q_only_grad(xq_, name, w, site) else torch.empty_like(y_)

        ops.ck("M:dlog", dlog_pad)
        wg(dlog_pad, ctx.dec_out, G.fc_w, M=V, db=G.fc_b)
        g_out = ops.linear_dgrad(dlog_pad, W.fc_pad, K=self.Vp)
        ck = ops.ck
        ck("M:g_out", g_out)
        # final decoder norm
        y_last, mo, ro = ctx.dec_last
        dy = torch.empty_like(y_last)
        ops.layernorm_bwd(g_out, y_last, mo, ro, W.dec_norm[0], dy, dgamma=G.dec_norm[0],
                          dbeta=G.dec_norm[1], param_stream=ps)
        ck("M:dy_final", dy)
        if hook:
            self._hook(side, hook, "head")
        # every layer's dK|dV of the memory lands in one [Ms, L*2d] buffer:
        # one dgrad GEMM (K = L*2d) after the decoder loop gives dmemory
        # fp8: one e4m3 copy of it (and of each layer's cross dQ) under one
        # scale site, so the memory dgrad runs on the fp8 MFMA as well; with
        # FP8_H8 and every consumer on the copy (each layer's K/V weight
        # gradient, the memory dgrad) the bf16 buffer is not written at all
        cross8 = None
        if f8 is not None and FP8_ATTN_DGRAD and self.n_dec:
            cross8 = (f8.site("b.cross"), torch.empty(Ms, self.n_dec * 2 * d, dtype=torch.uint8, device=dev))
        kv_q_only = (cross8 is not None and FP8_H8 and f8w is not None and "b.cross" in f8.bwd_ready
                     and ctx.memq is not None and f8.weight_t("ckv") is not None
                     and eligible(Ms, d, self.n_dec * 2 * d) and (2 * d) % 256 == 0 and Ms % 64 == 0)
        dkvc_all = None if kv_q_only else torch.empty(Ms, self.n_dec * 2 * d, dtype=dt, device=dev)
        for i in reversed(range(self.n_dec)):
            L, GL = W.dec[i], G.dec[i]
            (y_in, qkv, o, lse, y1, m1, r1, x1, qc, kvc, oc, lsec, y2, m2, r2, x2, h, y3, m3,
             r3) = ctx.dec[i]
            yq_in, oq, x1q, ocq, x2q, hq = ctx.dec_q[i]
            # FFN block: x3 = LN3(x2 + drop(W2 drop(relu(W1 x2))))
            dy3 = torch.empty_like(y3)
            dy3d = dgrad_in(y3, hq, "dec%d.l2" % i, L.l2_w, "b.dec%d.ln3" % i) if p_tr > 0 else dy3
            dy3q = ln_bwd(dy, y3, m3, r3, L.n3, dy3, dy3d, sd(_site("dec", i, 5)), GL.n3, "b.dec%d.ln3" % i)
            ck("M:dec%d.dy3" % i, dy3d)
            dh, dhq = ffn2_bwd(dy3q, dy3d, "dec%d.l2" % i, L.l2_w, GL, h, hq, "b.dec%d.dh" % i, x2q,
                               "dec%d.l1" % i)
            ck("M:dec%d.dh" % i, dh)
            wg(dh, x2, GL.l1_w, dhq, x2q, db=GL.l1_b)
            dx2, _ = dgrad(dhq, dh, "dec%d.l1" % i, L.l1_w, residual=dy3)
            ck("M:dec%d.dx2" % i, dx2)
            # cross-attention block: x2 = LN2(x1 + drop(Wo attn(q(x1), kv(mem))))
            dy2 = torch.empty_like(y2)
            dy2d = dgrad_in(y2, ocq, "dec%d.cao" % i, L.ca_ow, "b.dec%d.ln2" % i) if p_tr > 0 else dy2
            dy2q = ln_bwd(dx2, y2, m2, r2, L.n2, dy2, dy2d, sd(_site("dec", i, 3)), GL.n2, "b.dec%d.ln2" % i)
            ck("M:dec%d.dy2" % i, dy2d)
            wg(dy2d, oc, GL.ca_ow, dy2q, ocq, db=GL.ca_ob)
            doc, _ = dgrad(dy2q, dy2d, "dec%d.cao" % i, L.ca_ow)
            ck("M:dec%d.doc" % i, doc)
            dqc = None if (cross8 is not None and q_only_grad(x1q, "dec%d.cq" % i, L.cq_w, "b.cross",
                                                              dropped=False)) else \
                torch.empty(Mt, d, dtype=dt, device=dev)
            dkvc = dkvc_all[:, i * 2 * d:(i + 1) * 2 * d] if dkvc_all is not None else None
            q8c, dqcq = None, None
            if cross8 is not None:
                si, dkvc8 = cross8
                dqc8 = torch.empty(Mt, d, dtype=torch.uint8, device=dev)
                q8c = (dqc8, dkvc8[:, i * 2 * d:i * 2 * d + d], dkvc8[:, i * 2 * d + d:(i + 1) * 2 * d],
                       f8.qs_of(si), f8.amax_of(si))
                f8.record_bwd("b.cross")
                dqcq = (dqc8, si) if "b.cross" in f8.bwd_ready else None
            ops.attn_bwd(qc, kvc[:, :d], kvc[:, d:], oc, doc, lsec, dqc,
                         dkvc[:, :d] if dkvc is not None else None, dkvc[:, d:] if dkvc is not None else None,
                         B=B, H=H, Lq=T, Lk=S, D=D, kpm=ctx.mkpm, causal=False, scale=scale,
                         drop_p=p_tr, seed=sd(_site("dec", i, 2)), drop_mask=ctx.masks.get(("cross", i)),
                         q8=q8c)
            ck("M:dec%d.dqc" % i, dqc)
            ck("M:dec%d.dkvc" % i, dkvc)
            wg(dqc, x1, GL.cq_w, dqcq, x1q, db=GL.cq_b)
            dkvcq = None
            if cross8 is not None and "b.cross" in f8.bwd_ready:
                dkvcq = (cross8[1][:, i * 2 * d:(i + 1) * 2 * d], cross8[0])
            wg(dkvc, ctx.mem, GL.ckv_w, dkvcq, ctx.memq, db=GL.ckv_b)
            dx1, _ = dgrad(dqcq, dqc, "dec%d.cq" % i, L.cq_w, residual=dy2)
            ck("M:dec%d.dx1" % i, dx1)
            # self-attention block
            dy1 = torch.empty_like(y1)
            dy1d = dgrad_in(y1, oq, "dec%d.sao" % i, L.sa_ow, "b.dec%d.ln1" % i) if p_tr > 0 else dy1
            dy1q = ln_bwd(dx1, y1, m1, r1, L.n1, dy1, dy1d, sd(_site("dec", i, 1)), GL.n1, "b.dec%d.ln1" % i)
            ck("M:dec%d.dy1" % i, dy1d)
            wg(dy1d, o, GL.sa_ow, dy1q, oq, db=GL.sa_ob)
            do, _ = dgrad(dy1q, dy1d, "dec%d.sao" % i, L.sa_ow)
            ck("M:dec%d.do" % i, do)
            q8s, dqkvq = attn_q8((Mt, 3 * d), "b.dec%d.dqkv" % i, [(0, d), (d, 2 * d), (2 * d, 3 * d)])
            dqkv = None if (q8s is not None and q_only_grad(yq_in, "dec%d.sa" % i, L.sa_w, "b.dec%d.dqkv" % i,
                                                            dropped=False)) else \
                torch.empty(Mt, 3 * d, dtype=dt, device=dev)
            dq_, dk_, dv_ = (None, None, None) if dqkv is None else \
                (dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:])
            ops.attn_bwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, do, lse, dq_,
                         dk_, dv_, B=B, H=H, Lq=T, Lk=T, D=D,
                         kpm=ctx.tkpm, causal=True, scale=scale, drop_p=p_tr,
                         seed=sd(_site("dec", i, 0)), drop_mask=ctx.masks.get(("dec", i)), q8=q8s)
            ck("M:dec%d.dqkv" % i, dqkv)
            wg(dqkv, y_in, GL.sa_w, dqkvq, yq_in, db=GL.sa_b)
            dy, _ = dgrad(dqkvq, dqkv, "dec%d.sa" % i, L.sa_w, residual=dy1)
            ck("M:dec%d.dy" % i, dy)
            if hook:
                self._hook(side, hook, "dec%d" % i)
        d_tgt = dy
        if self.n_dec:
            if kv_q_only or (cross8 is not None and "b.cross" in f8.bwd_ready and f8.weight_t("ckv") is not None
                             and eligible(Ms, d, self.n_dec * 2 * d)):
                # bf16 output (the bf16 path sums into fp32): its rounding,
                # unit roundoff 2^-9, is far below the e4m3 operands' 2^-4
                dmem, _ = dgrad((cross8[1], cross8[0]), dkvc_all, "ckv", W.ckv_all)
            else:
                dmem = ops.linear_dgrad(dkvc_all, W.ckv_all, out_f32=torch.empty(Ms, d, device=dev))
        else:
            dmem = torch.zeros(Ms, d, device=dev)
        ck("M:dmem", dmem)
        # encoder
        x_last, me, re = ctx.enc_last
        dx = torch.empty_like(x_last)
        ops.layernorm_bwd(dmem, x_last, me, re, W.enc_norm[0], dx, dgamma=G.enc_norm[0],
                          dbeta=G.enc_norm[1], param_stream=ps)
        for i in reversed(range(self.n_enc)):
            L, GL = W.enc[i], G.enc[i]
            (x_in, qkv, o, lse, y1, m1, r1, x1, h, y2, m2, r2) = ctx.enc[i]
            xq_in, oq, x1q, hq = ctx.enc_q[i]
            dy2 = torch.empty_like(y2)
            dy2d = dgrad_in(y2, hq, "enc%d.l2" % i, L.l2_w, "b.enc%d.ln2" % i) if p_tr > 0 else dy2
            dy2q = ln_bwd(dx, y2, m2, r2, L.n2, dy2, dy2d, sd(_site("enc", i, 3)), GL.n2, "b.enc%d.ln2" % i)
            ck("M:enc%d.dy2" % i, dy2d)
            dh, dhq = ffn2_bwd(dy2q, dy2d, "enc%d.l2" % i, L.l2_w, GL, h, hq, "b.enc%d.dh" % i, x1q,
                               "enc%d.l1" % i)
            ck("M:enc%d.dh" % i, dh)
            wg(dh, x1, GL.l1_w, dhq, x1q, db=GL.l1_b)
            dx1, _ = dgrad(dhq, dh, "enc%d.l1" % i, L.l1_w, residual=dy2)
            ck("M:enc%d.dx1" % i, dx1)
            dy1 = torch.empty_like(y1)
            dy1d = dgrad_in(y1, oq, "enc%d.out" % i, L.out_w, "b.enc%d.ln1" % i) if p_tr > 0 else dy1
            dy1q = ln_bwd(dx1, y1, m1, r1, L.n1, dy1, dy1d, sd(_site("enc", i, 1)), GL.n1, "b.enc%d.ln1" % i)
            ck("M:enc%d.dy1" % i, dy1d)
            wg(dy1d, o, GL.out_w, dy1q, oq, db=GL.out_b)
            do, _ = dgrad(dy1q, dy1d, "enc%d.out" % i, L.out_w)
            ck("M:enc%d.do" % i, do)
            q8s, dqkvq = attn_q8((Ms, 3 * d), "b.enc%d.dqkv" % i, [(0, d), (d, 2 * d), (2 * d, 3 * d)])
            dqkv = None if (q8s is not None and q_only_grad(xq_in, "enc%d.in" % i, L.in_w, "b.enc%d.dqkv" % i,
                                                            dropped=False)) else \
                torch.empty(Ms, 3 * d, dtype=dt, device=dev)
            dq_, dk_, dv_ = (None, None, None) if dqkv is None else \
                (dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:])
            ops.attn_bwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, do, lse, dq_,
                         dk_, dv_, B=B, H=H, Lq=S, Lk=S, D=D,
                         kpm=ctx.skpm, causal=False, scale=scale, drop_p=p_tr,
                         seed=sd(_site("enc", i, 0)), drop_mask=ctx.masks.get(("enc", i)), q8=q8s)
            ck("M:enc%d.dqkv" % i, dqkv)
            wg(dqkv, x_in, GL.in_w, dqkvq, xq_in, db=GL.in_b)
            dx, _ = dgrad(dqkvq, dqkv, "enc%d.in" % i, L.in_w, residual=dy1)
            ck("M:enc%d.dx" % i, dx)
            if hook:
                self._hook(side, hook, "enc%d" % i)
        # shared embedding (model.py:76): both streams scatter into one table
        ops.embed_bwd(G.emb, math.sqrt(d), [(ctx.src_ids, dx, ctx.p_pos, sd(_SITE["pe_src"])),
                                            (ctx.tgt_ids, d_tgt, ctx.p_pos, sd(_SITE["pe_tgt"]))])
        self._join(side)
        if hook:
            hook("embedding")


# ----------------------------------------------------------------------
# autograd entry used by ScoreTransformer.forward
# ----------------------------------------------------------------------
class ScoreTransformerFunction(torch.autograd.Function):
    @staticmethod
    def forward(fctx, anchor, model, need_grad, src, tgt, src_kpm, tgt_kpm, mem_kpm, tgt_mask):
        eng = model.engine
        if not src.is_cuda:
            raise RuntimeError("the SMER engine runs on the GPU: move the model and inputs to "
                               "a ROCm device first")
        training = model.training and (model.pos_dropout > 0 or model.trans_dropout > 0)
        seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if training else 0
        logits, wts, ctx = eng.forward(src, tgt, src_kpm, tgt_kpm, mem_kpm,
                                       training=model.training, need_weights=model.need_weights,
                                       save=need_grad, seed=seed)
        fctx.eng = eng
        fctx.ctx = ctx
        fctx.model = model
        B, T = tgt.shape
        out = logits.view(B, T, eng.V)
        w = wts.permute(1, 0, 2, 3) if wts is not None else None
        if w is not None:
            fctx.mark_non_differentiable(w)
        return out, w

    @staticmethod
    def backward(fctx, dlogits, dweights):
        eng = fctx.eng
        ctx = fctx.ctx
        B, T = ctx.B, ctx.T
        dl = torch.zeros(B * T, eng.Vp, dtype=ctx.dt, device=dlogits.device)
        ops.cast2d(dlogits.reshape(B * T, eng.V).contiguous().float(), dl, cols=eng.V)
        eng.backward(ctx, dl)
        fctx.ctx = None
        return (None,) * 9
