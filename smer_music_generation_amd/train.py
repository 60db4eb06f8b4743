"""Fused training step: forward -> weighted CE -> backward -> (RCCL) -> Adam.

Restates the reference step (`train.py:702-797`) with the same criteria
(`train.py:555-642`), the same normaliser (`train.py:736-742`) and torch
Adam semantics (`train.py:264`), as one stream of gfx950 kernels:

  * the 7-12 CrossEntropyLoss(weight=w_c, ignore_index=0, reduction='none')
    criteria sum to ONE weighted CE with w = sum_c w_c (the classes are
    disjoint), normalised by sum_i ce_weight_all[y_i] -> smer_wce_*;
  * data parallel (new; the reference is single-device): one
    process per GPU; the scalar denominator is all-reduced BEFORE backward,
    so SUM-reduced gradients equal the single-process gradient of the
    concatenated batch; per-layer gradient slices of the flat buffer are
    all-reduced asynchronously (RCCL over xGMI) as soon as backward has
    produced them, overlapping the remaining backward kernels;
  * Adam on the flat fp32 master buffer also refreshes the bf16 working copy.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from . import ops

CRITERIA = ["meta", "time_signature", "program", "tempo", "structure", "pitch", "duration",
            "tensile", "key", "density", "occupation", "polyphony"]


def criterion_vectors(vocab, eos_weight, device="cpu"):
    """(per-criterion weight vectors, ce_weight_all) exactly as train.py:555-642."""
    V = vocab.vocab_size
    w = {}
    meta = torch.zeros(V)
    meta[1] = eos_weight
    w["meta"] = meta
    for name, (a, b) in (("structure", (3, 7)), ("time_signature", (7, 11)), ("tempo", (11, 18)),
                         ("program", (18, 146)), ("pitch", (146, 234)),
                         ("duration", (234, 234 + len(vocab.duration_indices)))):
        t = torch.zeros(V)
        t[a:b] = 1
        w[name] = t
    for name in ("key", "tensile", "density", "polyphony", "occupation"):
        if name in vocab.control_indices:
            idx = vocab.control_indices[name]
            t = torch.zeros(V)
            t[idx[0]: idx[-1] + 1] = 1
            w[name] = t
    ce_all = torch.ones(V)
    ce_all[0] = 0
    ce_all[2] = 0
    ce_all[-1] = 0
    ce_all[1] = eos_weight
    return {k: v.to(device) for k, v in w.items()}, ce_all.to(device)


class GradBucketer:
    """Asynchronous SUM all-reduce of contiguous slices of a flat gradient
    buffer, issued in backward order (works with nccl=RCCL and gloo)."""

    def __init__(self, flat_grad, ranges, group=None):
        self.flat = flat_grad
        self.ranges = ranges  # name -> (start, end)
        self.group = group
        self.pending = []
        self.done = set()

    def reduce(self, name):
        if name in self.done or name not in self.ranges:
            return
        a, b = self.ranges[name]
        self.pending.append(dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM,
                                            group=self.group, async_op=True))
        self.done.add(name)

    def finish(self):
        for name in self.ranges:
            self.reduce(name)
        for w in self.pending:
            w.wait()
        self.pending = []
        self.done = set()


def layer_ranges(model):
    """Contiguous flat-buffer range per backward hook name (see
    Engine.backward): head = decoder final norm + fc, dec{i}, enc{i} (the
    last encoder layer also owns the encoder final norm), embedding."""
    off = model._offsets
    spec = model._spec
    order = [n for n, _ in spec]
    ends = {}
    for i, (n, shp) in enumerate(spec):
        ends[n] = off[n] + (math.prod(shp) + 63) // 64 * 64
    total = model.flat_parameters().numel()

    def rng(prefix_list):
        names = [n for n in order if any(n.startswith(p) for p in prefix_list)]
        return (min(off[n] for n in names), max(ends[n] for n in names))

    r = {"embedding": rng(["embedding."])}
    n_enc, n_dec = model.num_encoder_layers, model.num_decoder_layers
    for i in range(n_enc):
        pre = ["transformer.encoder.layers.%d." % i]
        if i == n_enc - 1:
            pre.append("transformer.encoder.norm.")
        r["enc%d" % i] = rng(pre)
    for i in range(n_dec):
        r["dec%d" % i] = rng(["transformer.decoder.layers.%d." % i])
    a, _ = rng(["transformer.decoder.norm."])
    r["head"] = (a, total)
    return r


class Trainer:
    """One optimizer step per `step(batch)`; DP across the default process
    group when torch.distributed is initialised (world_size > 1)."""

    def __init__(self, model, vocab, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, eos_weight=0.8,
                 group=None):
        self.model = model
        self.vocab = vocab
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        dev = model.flat_parameters().device
        w, ce_all = criterion_vectors(vocab, eos_weight, dev)
        self.crit_w = w
        self.w_total = sum(w.values())
        self.ce_all = ce_all
        n = model.flat_parameters().numel()
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        self.t = 0
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self._ranges = layer_ranges(model)
        self._seed = 1

    def set_eos_weight(self, eos_weight):
        """Pretrain -> finetune switch (train.py:670-676)."""
        self.crit_w["meta"][1] = eos_weight
        self.w_total = sum(self.crit_w.values())
        self.ce_all[1] = eos_weight

    def step(self, batch, return_parts=False):
        """batch: dict of device tensors input/target_in/target_out/
        input_pad_mask/target_pad_mask (dataset.py:856-862).  Returns the
        (local-share) loss as a device scalar; no host sync."""
        model = self.model
        eng = model.engine
        model.train()
        src, tin, tout = batch["input"], batch["target_in"], batch["target_out"]
        skpm, tkpm = batch["input_pad_mask"], batch["target_pad_mask"]
        B, T = tin.shape
        dropout = model.pos_dropout > 0 or model.trans_dropout > 0
        seed = 0
        if dropout:
            self._seed = (self._seed * 1103515245 + 12345) & 0x7FFFFFFF
            seed = self._seed
        logits, _, ctx = eng.forward(src, tin, skpm, tkpm, skpm, training=True,
                                     need_weights=False, save=True, seed=seed)
        y = tout.reshape(-1).contiguous().long()
        denom = torch.empty(1, device=logits.device)
        ops.wce_denom(y, self.ce_all, denom)
        if self.world > 1:
            dist.all_reduce(denom, group=self.group)
        dlog = torch.zeros(B * T, eng.Vp, dtype=ctx.dt, device=logits.device)
        row_loss = torch.empty(B * T, device=logits.device)
        loss = torch.empty(1, device=logits.device)
        ops.wce_fwd_bwd(logits, y, self.w_total, denom, row_loss, loss, dlog, V=eng.V)
        grad = model.flat_grad()
        grad.zero_()
        hook = None
        bucketer = None
        if self.world > 1:
            bucketer = GradBucketer(grad, self._ranges, self.group)
            hook = bucketer.reduce
        eng.backward(ctx, dlog, hook=hook)
        if bucketer is not None:
            bucketer.finish()
        self.t += 1
        work = eng._bf16 if eng.act_dtype() == torch.bfloat16 and eng._bf16 is not None else None
        ops.adam(model.flat_parameters(), grad, self.m, self.v, work, lr=self.lr, b1=self.b1,
                 b2=self.b2, eps=self.eps, step=self.t)
        if work is not None:
            eng.mark_bf16_fresh()
        else:
            eng._bf16_version = None
        if return_parts:
            return loss, self.loss_parts(row_loss, y, denom)
        return loss

    def loss_parts(self, row_loss, y, denom):
        """Per-criterion losses for logging (train.py:788-797), on device."""
        out = {}
        for name in CRITERIA:
            if name in self.crit_w:
                sel = self.crit_w[name][y] > 0
                out[name] = (row_loss * sel).sum() / denom[0]
        return out
