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
import os

import numpy as np
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
    buffer, issued in backward order (works with nccl=RCCL and gloo).

    wire_dtype=torch.bfloat16 (opt-in; fp32 is the parity default) sends each
    slice as bf16: the slice is cast into a persistent bf16 shadow on the
    compute stream, that shadow is all-reduced (half the xGMI bytes: 89 MB
    instead of 178 MB per C2 step), and the sum is widened back
    into the fp32 slice once the collective has finished.  Summation then
    happens in bf16 inside RCCL, so results differ from the fp32 reduction
    by bf16 rounding of the per-rank gradients and of the partial sums."""

    def __init__(self, flat_grad, ranges, group=None, wire_dtype=None):
        self.flat = flat_grad
        self.ranges = ranges  # name -> (start, end)
        self.group = group
        self.pending = []
        self.done = set()
        self.wire_dtype = wire_dtype if wire_dtype not in (None, flat_grad.dtype) else None
        self.shadow = (torch.empty_like(flat_grad, dtype=self.wire_dtype)
                       if self.wire_dtype is not None else None)

    def reduce(self, name):
        if name in self.done or name not in self.ranges:
            return
        a, b = self.ranges[name]
        if self.shadow is None:
            buf = self.flat[a:b]
        else:
            buf = self.shadow[a:b]
            buf.copy_(self.flat[a:b])
        self.pending.append((a, b, dist.all_reduce(buf, op=dist.ReduceOp.SUM,
                                                   group=self.group, async_op=True)))
        self.done.add(name)

    def finish(self):
        for name in self.ranges:
            self.reduce(name)
        for a, b, w in self.pending:
            w.wait()
            if self.shadow is not None:
                self.flat[a:b].copy_(self.shadow[a:b])
        self.pending = []
        self.done = set()


def broadcast_parameters(model, group=None):
    """every rank starts from rank 0's parameters.  The flat fp32
    master is one tensor, so this is a single broadcast; the bf16 working copy
    and every derived weight cache are invalidated afterwards.  The reference
    builds and initialises its model per process (train.py:257-264); without
    this, DP correctness would rest on every rank seeding identically."""
    flat = model.flat_parameters()
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(flat.data, src=src, group=group)
    if hasattr(model, "engine"):
        model.engine.mark_params_updated()


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


class FusedAdam(torch.optim.Optimizer):
    """`torch.optim.Adam`'s state and param_groups over the Trainer's flat
    moment buffers (train.py:264 builds `Adam(model.parameters(), lr)`).

    The update itself is the Trainer's fused kernel; this object exists so
    that the reference's surrounding code works unchanged:
      * `state_dict()` / `load_state_dict()` in torch Adam's format, so a
        reference checkpoint's `optimizer_state_dict` (train.py:266-303,
        970-971) resumes here and ours resumes in torch Adam;
      * `param_groups[0]['lr']` is read every step, so
        `ReduceLROnPlateau(trainer.optimizer, ...)` (train.py:663-664, 939)
        drives the fused step.
    Per-parameter `exp_avg` / `exp_avg_sq` are views of the flat buffers."""

    def __init__(self, model, m, v, lr, betas, eps):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=0, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False,
                        fused=None, decoupled_weight_decay=False)
        super().__init__(list(model.parameters()), defaults)
        self._m, self._v = m, v
        self._views = []
        for name, p in model.named_parameters():
            o = model._offsets[name]
            n = p.numel()
            self._views.append((p, m[o: o + n].view(p.shape), v[o: o + n].view(p.shape)))
        self.t = 0

    def step(self, closure=None):
        raise RuntimeError("FusedAdam is stepped by Trainer.step (fused kernel)")

    def zero_grad(self, set_to_none=False):
        for p, _, _ in self._views:
            if p.grad is not None:
                p.grad.zero_()

    def state_dict(self):
        state = {}
        if self.t > 0:
            for i, (_, ma, va) in enumerate(self._views):
                state[i] = {"step": torch.tensor(float(self.t)), "exp_avg": ma.detach().clone(),
                            "exp_avg_sq": va.detach().clone()}
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(self._views)))
            groups.append(d)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(self._views):
            raise ValueError("optimizer state has %d groups / %s params, expected 1 / %d"
                             % (len(groups), [len(g["params"]) for g in groups], len(self._views)))
        for k in ("lr", "betas", "eps", "weight_decay", "amsgrad"):
            if k in groups[0]:
                self.param_groups[0][k] = groups[0][k]
        if self.param_groups[0].get("weight_decay", 0) or self.param_groups[0].get("amsgrad"):
            raise ValueError("FusedAdam implements Adam without weight decay / amsgrad (train.py:264)")
        st = state_dict["state"]
        steps = set()
        order = groups[0]["params"]
        for slot, pid in enumerate(order):
            s = st.get(pid)
            _, ma, va = self._views[slot]
            if s is None:
                ma.zero_()
                va.zero_()
                steps.add(0)
                continue
            ma.copy_(s["exp_avg"].reshape(ma.shape).to(ma.device, ma.dtype))
            va.copy_(s["exp_avg_sq"].reshape(va.shape).to(va.device, va.dtype))
            steps.add(int(float(s["step"])))
        if len(steps) > 1:
            raise ValueError("per-parameter Adam steps differ %s; the fused step shares one" % steps)
        self.t = steps.pop() if steps else 0


class Trainer:
    """One optimizer step per `step(batch)`; DP across the default process
    group when torch.distributed is initialised (world_size > 1)."""

    def __init__(self, model, vocab, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, eos_weight=0.8,
                 group=None, grad_wire_dtype=None, broadcast=True, dp=None):
        """grad_wire_dtype: None / torch.float32 (default, parity) or
        torch.bfloat16 for the DP gradient all-reduce (see GradBucketer).
        broadcast: under DP, copy rank 0's parameters to every rank here.
        dp: run the data-parallel path (normaliser all-reduce, per-layer
        bucketed gradient all-reduces issued from the backward hooks) --
        default: when the process group has more than one rank; True also
        at world size 1 (the real RCCL calls and stream ordering on one GPU)."""
        self.model = model
        self.vocab = vocab
        dev = model.flat_parameters().device
        w, ce_all = criterion_vectors(vocab, eos_weight, dev)
        self.crit_w = w
        self.w_total = sum(w.values())
        self.ce_all = ce_all
        n = model.flat_parameters().numel()
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        self.optimizer = FusedAdam(model, self.m, self.v, lr, betas, eps)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        if dp and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("Trainer(dp=True) needs an initialised torch.distributed process group")
        self.dp = self.world > 1 if dp is None else bool(dp)
        self._ranges = layer_ranges(model)
        self._seed = 1
        self.grad_wire_dtype = grad_wire_dtype
        self._bucketer = None
        if self.dp and broadcast:
            broadcast_parameters(model, group)

    # hyper-parameters live in the optimizer's param group (schedulers edit it)
    @property
    def lr(self):
        return self.optimizer.param_groups[0]["lr"]

    @lr.setter
    def lr(self, value):
        self.optimizer.param_groups[0]["lr"] = float(value)

    @property
    def t(self):
        return self.optimizer.t

    @t.setter
    def t(self, value):
        self.optimizer.t = int(value)

    def state_dict(self):
        """torch Adam format (`optimizer_state_dict` of train.py:970-971)."""
        return self.optimizer.state_dict()

    def load_state_dict(self, state_dict):
        self.optimizer.load_state_dict(state_dict)
        self.model.engine.mark_params_updated()  # weights may have been reloaded too

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
        if self.dp:
            dist.all_reduce(denom, group=self.group)
        dlog = torch.zeros(B * T, eng.Vp, dtype=ctx.dt, device=logits.device)
        row_loss = torch.empty(B * T, device=logits.device)
        loss = torch.empty(1, device=logits.device)
        ops.wce_fwd_bwd(logits, y, self.w_total, denom, row_loss, loss, dlog, V=eng.V)
        grad = model.flat_grad()
        grad.zero_()
        hook = None
        bucketer = None
        self.t += 1
        work = eng._bf16 if eng.act_dtype() == torch.bfloat16 and eng._bf16 is not None else None
        g = self.optimizer.param_groups[0]
        flat = model.flat_parameters()

        def adam(a=None, b=None):
            sl = slice(a, b)
            ops.adam(flat[sl], grad[sl], self.m[sl], self.v[sl], work[sl] if work is not None else None,
                     lr=g["lr"], b1=g["betas"][0], b2=g["betas"][1], eps=g["eps"], step=self.t)
        stepped = None
        if self.dp:
            if self._bucketer is None or self._bucketer.flat is not grad:
                # persistent: the bf16 shadow is allocated once
                self._bucketer = GradBucketer(grad, self._ranges, self.group,
                                              wire_dtype=self.grad_wire_dtype)
            bucketer = self._bucketer
            hook = bucketer.reduce
        elif os.environ.get("SMER_ADAM_OVERLAP", "1") != "0":
            # Adam of each layer range as soon as its gradients are final: the
            # hook runs with the weight-gradient stream current, which first
            # waits for everything the main stream has queued (that layer's
            # dgrads still read its working weights); elementwise, so the
            # result is the same bits as one Adam over the flat buffers
            main = torch.cuda.current_stream(flat.device)
            stepped = set()

            def hook(name):
                if name not in self._ranges or name == "embedding":
                    return
                torch.cuda.current_stream(flat.device).wait_stream(main)
                adam(*self._ranges[name])
                stepped.add(name)
        eng.backward(ctx, dlog, hook=hook)
        if bucketer is not None:
            bucketer.finish()
        if stepped is None:
            adam()
        else:  # the ranges no hook stepped (the embedding), on the main stream
            for name, (a, b) in self._ranges.items():
                if name not in stepped:
                    adam(a, b)
        if work is not None:
            eng.mark_bf16_fresh()
        else:
            eng.mark_params_updated()
        if return_parts:
            return loss, self.loss_parts(row_loss, y, denom)
        return loss

    def _class_table(self, dev):
        """int32 [V] token class id of every vocabulary index (vocab
        get_token_classes), the class names in id order."""
        ct = getattr(self, "_cls", None)
        if ct is None or ct[0].device != dev:
            v = self.vocab
            names = sorted(set(v.token_class_ranges.values()))
            ids = {n: i for i, n in enumerate(names)}
            # -1: an index with no token class (the reference's `accuracy`
            # raises KeyError on such a target and validate() skips the batch)
            tab = torch.tensor([ids.get(v.token_class_ranges.get(i), -1) for i in range(v.vocab_size)],
                               dtype=torch.int32)
            ct = self._cls = (tab.to(dev), names)
        return ct

    def eval_step(self, batch):
        """The validation pass of one batch (train.py:1037-1195 `validate`
        body + `accuracy`, train.py:988-1034) on device, no backward: eval
        forward (no dropout), the fused criteria (no gradient written) and the
        argmax accuracy counts.  Returns (loss, {criterion: loss}, counts)
        as device tensors, no host sync; counts int32 [2 * n_classes + 2]
        (rows, hits per token class in `accuracy_from_counts`' class order,
        then the total)."""
        model = self.model
        eng = model.engine
        was_training = model.training
        model.eval()
        src, tin, tout = batch["input"], batch["target_in"], batch["target_out"]
        skpm, tkpm = batch["input_pad_mask"], batch["target_pad_mask"]
        B, T = tin.shape
        try:
            with torch.no_grad():
                logits, _, _ = eng.forward(src, tin, skpm, tkpm, skpm, training=False,
                                           need_weights=False, save=False, seed=0)
                y = tout.reshape(-1).contiguous().long()
                denom = torch.empty(1, device=logits.device)
                ops.wce_denom(y, self.ce_all, denom)
                row_loss = torch.empty(B * T, device=logits.device)
                loss = torch.empty(1, device=logits.device)
                ops.wce_fwd_bwd(logits, y, self.w_total, denom, row_loss, loss, None, V=eng.V)
                parts = self.loss_parts(row_loss, y, denom)
                cls, names = self._class_table(logits.device)
                counts = torch.zeros(2 * len(names) + 2, dtype=torch.int32, device=logits.device)
                ops.argmax_accuracy(logits, y, cls, len(names), self.vocab.pad_index, counts)
        finally:
            if was_training:
                model.train()
        return loss, parts, counts

    def accuracy_from_counts(self, counts):
        """{token class: accuracy, 'total': accuracy} as train.py:1022-1026
        forms it (a class with no target rows keeps 0)."""
        _, names = self._class_table(self.model.flat_parameters().device)
        c = counts.detach().to("cpu").numpy().astype(np.int64)
        out = {}
        for i, n in enumerate(names + ["total"]):
            out[n] = float(c[2 * i + 1]) / float(c[2 * i]) if c[2 * i] else 0
        return out

    def loss_parts(self, row_loss, y, denom):
        """Per-criterion losses for logging (train.py:788-797), on device."""
        out = {}
        for name in CRITERIA:
            if name in self.crit_w:
                sel = self.crit_w[name][y] > 0
                out[name] = (row_loss * sel).sum() / denom[0]
        return out


def validate(valid_loader, trainer, device=None):
    """`validate` (train.py:1037-1195) over a loader of collated batches
    (dataset.py:856-862 keys) with the fused device pass: per batch the
    criteria and the accuracy counts stay on device; the dictionaries are
    averaged over batches as the reference averages them (per-batch loss and
    per-batch class accuracy, each divided by the number of batches).
    Returns (total_loss, total_accuracy)."""
    dev = device or trainer.model.flat_parameters().device
    total_loss, total_acc, steps = {}, {}, 0
    for data in iter(valid_loader):
        bt = {k: (torch.as_tensor(np.asarray(data[k])) if not torch.is_tensor(data[k]) else data[k]).to(dev)
              for k in ("input", "target_in", "target_out", "input_pad_mask", "target_pad_mask")}
        loss, parts, counts = trainer.eval_step(bt)
        steps += 1
        total_loss["total"] = total_loss.get("total", 0.0) + float(loss.item())
        for k, v in parts.items():
            total_loss[k] = total_loss.get(k, 0.0) + float(v.item())
        for k, v in trainer.accuracy_from_counts(counts).items():
            total_acc[k] = total_acc.get(k, 0.0) + v
    for d in (total_loss, total_acc):
        for k in d:
            d[k] /= max(steps, 1)
    return total_loss, total_acc
