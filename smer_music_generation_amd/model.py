"""Drop-in `ScoreTransformer` (reference `model.py:59-125`, `transformer.py`).

Same constructor, forward signature, return tuple, parameter names and
state_dict keys as the reference.  Underneath, every
parameter is a view into ONE flat fp32 buffer (so the fused Adam, the bf16
working copy and the data-parallel gradient buckets are single contiguous
streams) and `forward` runs the hand-written gfx950 kernels of
libsmer_hip.so through `engine.Engine` — there is no ATen compute path.

Initialisation replays the reference constructor's RNG consumption in the
same order (embedding normal_, MHA out_proj Linear + xavier in_proj,
FFN Linears, Transformer._reset_parameters xavier_uniform_, fc Linear), so
`torch.manual_seed(s); ScoreTransformer(...)` yields the reference weights.
"""
from __future__ import annotations

import copy
import math

import torch
from torch import nn
from torch.nn import init

from . import engine as _engine


def param_spec(vocab_size, d_model, dim_feedforward, n_enc, n_dec):
    """Ordered (name, shape) of all parameters = reference named_parameters()."""
    V, d, F = vocab_size, d_model, dim_feedforward
    out = [("embedding.weight", (V, d))]

    def mha(p):
        return [(p + ".in_proj_weight", (3 * d, d)), (p + ".in_proj_bias", (3 * d,)),
                (p + ".out_proj.weight", (d, d)), (p + ".out_proj.bias", (d,))]

    def ffn(p):
        return [(p + ".linear1.weight", (F, d)), (p + ".linear1.bias", (F,)),
                (p + ".linear2.weight", (d, F)), (p + ".linear2.bias", (d,))]

    def ln(p):
        return [(p + ".weight", (d,)), (p + ".bias", (d,))]

    for i in range(n_enc):
        p = "transformer.encoder.layers.%d" % i
        out += mha(p + ".self_attn") + ffn(p) + ln(p + ".norm1") + ln(p + ".norm2")
    out += ln("transformer.encoder.norm")
    for i in range(n_dec):
        p = "transformer.decoder.layers.%d" % i
        out += mha(p + ".self_attn") + mha(p + ".multihead_attn") + ffn(p)
        out += ln(p + ".norm1") + ln(p + ".norm2") + ln(p + ".norm3")
    out += ln("transformer.decoder.norm")
    out += [("fc.weight", (V, d)), ("fc.bias", (V,))]
    return out


# --------------------------------------------------------------------------
# module tree mirroring the reference names
# --------------------------------------------------------------------------
class _Linear(nn.Module):
    def __init__(self, fan_in, fan_out):
        super().__init__()
        self.in_features, self.out_features = fan_in, fan_out
        self.weight = nn.Parameter(torch.empty(fan_out, fan_in))
        self.bias = nn.Parameter(torch.empty(fan_out))
        # nn.Linear.reset_parameters
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
        init.uniform_(self.bias, -bound, bound)


class MultiheadAttention(nn.Module):
    """Parameter holder with torch.nn.MultiheadAttention's names and init
    (in_proj_weight/bias packed, out_proj); compute lives in the engine."""

    def __init__(self, embed_dim, num_heads, dropout=0.0):
        super().__init__()
        self.embed_dim, self.num_heads, self.dropout = embed_dim, num_heads, dropout
        self.head_dim = embed_dim // num_heads
        if self.head_dim * num_heads != embed_dim:
            raise AssertionError("embed_dim must be divisible by num_heads")
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        self.out_proj = _Linear(embed_dim, embed_dim)
        init.xavier_uniform_(self.in_proj_weight)
        init.constant_(self.in_proj_bias, 0.0)
        init.constant_(self.out_proj.bias, 0.0)


class LayerNorm(nn.Module):
    def __init__(self, d, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))


class TransformerEncoderLayer(nn.Module):
    """`transformer.py:337-396` (post-LN)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu"):
        super().__init__()
        if activation != "relu":
            raise NotImplementedError("only relu is on the hot path (transformer.py:477-483)")
        self.self_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.linear1 = _Linear(d_model, dim_feedforward)
        self.dropout_p = dropout
        self.linear2 = _Linear(dim_feedforward, d_model)
        self.norm1 = LayerNorm(d_model)
        self.norm2 = LayerNorm(d_model)


class TransformerDecoderLayer(nn.Module):
    """`transformer.py:399-470` (post-LN, self + cross attention)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu"):
        super().__init__()
        if activation != "relu":
            raise NotImplementedError("only relu is on the hot path (transformer.py:477-483)")
        self.self_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.multihead_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.linear1 = _Linear(d_model, dim_feedforward)
        self.dropout_p = dropout
        self.linear2 = _Linear(dim_feedforward, d_model)
        self.norm1 = LayerNorm(d_model)
        self.norm2 = LayerNorm(d_model)
        self.norm3 = LayerNorm(d_model)


class _Stack(nn.Module):
    def __init__(self, layer, n, d_model):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(n)])
        self.num_layers = n
        self.norm = LayerNorm(d_model)


class Transformer(nn.Module):
    """`transformer.py:16-142` parameter tree + _reset_parameters."""

    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, activation="relu"):
        super().__init__()
        enc_layer = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation)
        self.encoder = _Stack(enc_layer, num_encoder_layers, d_model)
        dec_layer = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation)
        self.decoder = _Stack(dec_layer, num_decoder_layers, d_model)
        for p in self.parameters():  # transformer.py:137-142
            if p.dim() > 1:
                init.xavier_uniform_(p)
        self.d_model = d_model
        self.nhead = nhead


class _Embedding(nn.Module):
    def __init__(self, num, dim):
        super().__init__()
        self.num_embeddings, self.embedding_dim = num, dim
        self.weight = nn.Parameter(torch.empty(num, dim))
        init.normal_(self.weight)


def sinusoid_table(max_len, d_model):
    """`model.py:113-121` ([max_len, 1, d])."""
    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
    div = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div)
    pe[:, 1::2] = torch.cos(position * div)
    return pe.unsqueeze(0).transpose(0, 1)


class PositionalEncoding(nn.Module):
    """`model.py:110-125`; accepts a checkpoint `pe` of any max_len (rows
    are position-wise identical; SURVEY.md §5 long-context note)."""

    def __init__(self, d_model, dropout=0.1, max_len=100):
        super().__init__()
        self.p = dropout
        self.register_buffer("pe", sinusoid_table(max_len, d_model))

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        key = prefix + "pe"
        if key in state_dict and state_dict[key].shape != self.pe.shape:
            src = state_dict[key]
            n = min(src.shape[0], self.pe.shape[0])
            fixed = self.pe.clone()
            fixed[:n] = src[:n].to(fixed.dtype)
            state_dict = dict(state_dict)
            state_dict[key] = fixed
        return super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def extend(self, max_len):
        if max_len > self.pe.shape[0]:
            self.pe = sinusoid_table(max_len, self.pe.shape[2]).to(self.pe.device)


class ScoreTransformer(nn.Module):
    """`model.py:59-106`.

    Extra keyword-only knobs (reference defaults preserved):
      precision: 'bf16' (MFMA path, default), 'fp32' (parity path) or 'fp8'
        (the QKV / FFN / cross-attention forward contractions on the e4m3
        MFMA with delayed per-tensor scaling, everything else bf16; fp8.py)
      need_weights: return the head-averaged cross-attention weights
        [B, L, T, S] like the reference (default True); False returns None.
    """

    def __init__(self, vocab_size, d_model, nhead, num_encoder_layers, num_decoder_layers,
                 dim_feedforward, max_seq_length, pos_dropout, trans_dropout, *,
                 precision="bf16", need_weights=True):
        super().__init__()
        self.d_model = d_model
        self.embedding = _Embedding(vocab_size, d_model)
        self.pos_enc = PositionalEncoding(d_model, pos_dropout, max_seq_length)
        self.transformer = Transformer(d_model, nhead, num_encoder_layers, num_decoder_layers,
                                       dim_feedforward, trans_dropout)
        self.fc = _Linear(d_model, vocab_size)
        self.vocab_size = vocab_size
        self.nhead = nhead
        self.dim_feedforward = dim_feedforward
        self.num_encoder_layers = num_encoder_layers
        self.num_decoder_layers = num_decoder_layers
        self.pos_dropout = pos_dropout
        self.trans_dropout = trans_dropout
        self.need_weights = need_weights
        self.precision = precision
        self._spec = param_spec(vocab_size, d_model, dim_feedforward, num_encoder_layers,
                                num_decoder_layers)
        self._engine = None
        self._flatten()

    # ---- flat parameter storage ---------------------------------------
    def _flatten(self):
        """Rebind every parameter as a view of one flat fp32 buffer (64-elem
        aligned slots) on the parameters' current device."""
        params = dict(self.named_parameters())
        dev = params["embedding.weight"].device
        offs, cur = {}, 0
        for name, shape in self._spec:
            offs[name] = cur
            cur += (math.prod(shape) + 63) // 64 * 64
        flat = torch.zeros(cur, dtype=torch.float32, device=dev)
        for name, shape in self._spec:
            p = params[name]
            n = p.numel()
            flat[offs[name]: offs[name] + n].copy_(p.data.reshape(-1).float())
            p.data = flat[offs[name]: offs[name] + n].view(shape)
        self._flat = flat
        self._offsets = offs
        self._grad_flat = None
        self._engine = None

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        if hasattr(self, "_spec"):
            self._flatten()
        return out

    def flat_parameters(self):
        return self._flat

    def flat_grad(self):
        """Flat fp32 gradient buffer; every parameter's .grad is a view."""
        if self._grad_flat is None or self._grad_flat.device != self._flat.device:
            self._grad_flat = torch.zeros_like(self._flat)
        g = self._grad_flat
        named = list(self.named_parameters())
        if all(p.grad is None for _, p in named):
            g.zero_()
            for name, p in named:
                o = self._offsets[name]
                p.grad = g[o: o + p.numel()].view(p.shape)
            return g
        for name, p in named:
            o = self._offsets[name]
            want = g[o: o + p.numel()].view(p.shape)
            if p.grad is None or p.grad.data_ptr() != want.data_ptr():
                if p.grad is not None:
                    want.copy_(p.grad)
                else:
                    want.zero_()
                p.grad = want
        return g

    def set_precision(self, precision):
        assert precision in ("bf16", "fp32", "fp8")
        self.precision = precision
        return self

    @property
    def engine(self):
        if self._engine is None:
            self._engine = _engine.Engine(self)
        return self._engine

    def _check_causal(self, tgt_mask, T):
        """The engine's decoder self-attention is causal by construction, the
        only mask the reference ever passes (`train.py:715`,
        `generation.py:214`; only tgt_mask[0] is used, `model.py:95`).  Any
        other mask (or none, which the reference would treat as
        unmasked) raises instead of silently computing something else.
        Checked once per mask tensor (keyed by storage and version)."""
        if tgt_mask is None:
            raise RuntimeError("tgt_mask=None (unmasked decoder self-attention) is not supported: "
                               "pass the causal nopeek mask (gen_nopeek_mask)")
        m = tgt_mask[0] if tgt_mask.dim() == 3 else tgt_mask
        if tuple(m.shape) != (T, T):
            raise RuntimeError("tgt_mask must be [T, T] or [B, T, T] with T=%d, got %s"
                               % (T, tuple(tgt_mask.shape)))
        key = (m.data_ptr(), m._version, T, str(m.device), m.dtype)
        if getattr(self, "_causal_ok", None) == key:
            return
        upper = torch.ones(T, T, dtype=torch.bool, device=m.device).triu(1)
        if m.dtype == torch.bool:
            ok = torch.equal(m, upper)
        else:
            mf = m.float()
            ok = bool(torch.all(torch.isneginf(mf[upper])).item()) and \
                bool(torch.all(mf[~upper] == 0).item())
        if not ok:
            raise RuntimeError("tgt_mask is not the causal nopeek mask: the engine only computes "
                               "causal decoder self-attention (the reference's only mask)")
        self._causal_ok = key

    # ---- reference forward ---------------------------------------------
    def forward(self, src, tgt, src_key_padding_mask, tgt_key_padding_mask,
                memory_key_padding_mask, tgt_mask):
        """`model.py:85-106`: returns (logits [B,T,V] fp32, cross-attention
        weights [B, L, T, S] or None).  tgt_mask must be the causal nopeek
        mask (`train.py:1356-1369`); only tgt_mask[0] is used (`model.py:95`)."""
        if src.size(0) != tgt.size(0):
            raise RuntimeError("the batch number of src and tgt must be equal")
        self._check_causal(tgt_mask, tgt.size(1))
        need_grad = torch.is_grad_enabled() and self.embedding.weight.requires_grad
        return _engine.ScoreTransformerFunction.apply(
            self.embedding.weight, self, need_grad, src, tgt, src_key_padding_mask, tgt_key_padding_mask,
            memory_key_padding_mask, tgt_mask)
