"""Generate the golden vectors that pin the oracle and the engine.

RUN ONLY IN THE BUILD CONTAINER (needs /root/reference; never runs on the GPU
box).  Imports the reference's own modules — `model.py`, `transformer.py`,
`vocab.py`, `generation.py` (absent MIDI/log libraries stubbed as empty
modules) — runs them on deterministic inputs and writes data
only (inputs + expected outputs) into tests/golden/.  `train.py` cannot be
imported (wandb login at import, `train.py:23-25`), so its criteria are
re-issued here exactly as `train.py:555-642,726-780` call them.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import logging
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(OUT, "..", ".."))
sys.path.insert(0, REF)
for _m in ("pretty_midi", "music21", "coloredlogs"):
    sys.modules.setdefault(_m, types.ModuleType(_m))

import model as ref_model          # noqa: E402  (reference)
import vocab as ref_vocab          # noqa: E402  (reference)
import generation as ref_gen       # noqa: E402  (reference)

from smer_music_generation_amd.synth import synth_events  # noqa: E402  (our data generator)

CTRL = ['key', 'tensile', 'density', 'polyphony', 'occupation']
MICRO = dict(d_model=64, nhead=2, num_encoder_layers=2, num_decoder_layers=2,
             dim_feedforward=128, max_seq_length=2400)


def vocab_golden():
    out = {}
    for mode in (0, 1):
        for cl in ([], CTRL, ['key', 'density']):
            v = ref_vocab.WordVocab(mode, cl)
            rec = {"char2idx": v._char2idx, "vocab_size": v.vocab_size,
                   "token_class_ranges": {str(k): c for k, c in v.token_class_ranges.items()},
                   "name_to_tokens": v.name_to_tokens, "control_tokens": v.control_tokens,
                   "control_indices": v.control_indices, "class_names": sorted(v.class_names)}
            for a in ("structure_indices", "pitch_indices", "mask_indices", "duration_indices",
                      "duration_only_indices", "program_indices", "tempo_indices",
                      "time_signature_indices", "rest_indices", "sep_indices"):
                rec[a] = getattr(v, a)
            if mode == 0:
                rec["continue_index"] = v.continue_index
            out["%d|%s" % (mode, ",".join(cl))] = rec
    with open(os.path.join(OUT, "vocab_golden.json"), "w") as f:
        json.dump(out, f, sort_keys=True)


def build_model(seed=0):
    torch.manual_seed(seed)
    v = ref_vocab.WordVocab(0, CTRL)
    m = ref_model.ScoreTransformer(v.vocab_size, MICRO["d_model"], MICRO["nhead"],
                                   MICRO["num_encoder_layers"], MICRO["num_decoder_layers"],
                                   MICRO["dim_feedforward"], MICRO["max_seq_length"], 0.0, 0.0)
    for p in m.parameters():  # train.py:261-263
        if p.dim() > 1:
            torch.nn.init.xavier_normal_(p)
    return v, m


def gen_nopeek_mask(length):  # train.py:1356-1369 (same as generation.py:193)
    return ref_gen.gen_nopeek_mask(length)


def forward_and_train_golden():
    v, m = build_model(0)
    m.eval()
    rng = np.random.default_rng(7)
    B, S, T = 2, 48, 16
    src = rng.integers(3, 300, size=(B, S)).astype(np.int64)
    tin = rng.integers(3, 300, size=(B, T)).astype(np.int64)
    tout = rng.integers(1, 309, size=(B, T)).astype(np.int64)
    tin[:, 0] = 2
    src[1, 40:] = 0
    tin[1, 12:] = 0
    tout[1, 12:] = 0
    tout[0, 5] = 2      # mask id: weight 0 in the denominator
    tout[0, 9] = 308    # unk
    tout[0, 3] = 1      # eos
    skpm = src == 0
    tkpm = tin == 0
    src_t, tin_t, tout_t = map(torch.as_tensor, (src, tin, tout))
    skpm_t, tkpm_t = torch.as_tensor(skpm), torch.as_tensor(tkpm)
    mask = gen_nopeek_mask(T).unsqueeze(0).repeat(B, 1, 1)
    logits, attn = m(src_t, tin_t, skpm_t, tkpm_t, skpm_t.clone(), mask)

    # criteria exactly as train.py:555-642 builds them (pretraining: eos_weight 0.8)
    dev = "cpu"
    eos_weight = 0.8
    V = v.vocab_size
    CE = torch.nn.CrossEntropyLoss
    meta_weight = torch.zeros(V, device=dev)
    meta_weight[1] = eos_weight
    ce_weight_all = torch.ones(V, device=dev)
    ce_weight_all[0] = 0
    ce_weight_all[2] = 0
    ce_weight_all[-1] = 0
    ce_weight_all[1] = eos_weight

    def rng_w(a, b):
        w = torch.zeros(V)
        w[a:b] = 1
        return w
    crit = {"meta": CE(ignore_index=0, weight=meta_weight, reduction='none'),
            "structure": CE(ignore_index=0, weight=rng_w(3, 7), reduction='none'),
            "time_signature": CE(ignore_index=0, weight=rng_w(7, 11), reduction='none'),
            "tempo": CE(ignore_index=0, weight=rng_w(11, 18), reduction='none'),
            "program": CE(ignore_index=0, weight=rng_w(18, 146), reduction='none'),
            "pitch": CE(ignore_index=0, weight=rng_w(146, 234), reduction='none'),
            "duration": CE(ignore_index=0, weight=rng_w(234, 234 + len(v.duration_indices)),
                           reduction='none')}
    for name in ('key', 'tensile', 'density', 'polyphony', 'occupation'):
        idx = v.control_indices[name]
        crit[name] = CE(ignore_index=0, weight=rng_w(idx[0], idx[-1] + 1), reduction='none')
    x = logits.reshape(-1, V)
    y = tout_t.reshape(-1)
    denom = ce_weight_all[y].sum()
    parts = {}
    order = ["meta", "time_signature", "program", "tempo", "structure", "pitch", "duration",
             "tensile", "key", "density", "occupation", "polyphony"]  # train.py:734-780
    loss = None
    for name in order:
        l = torch.sum(crit[name](x, y)) / denom
        parts[name] = float(l)
        loss = l if loss is None else loss + l
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    opt.zero_grad()
    loss.backward()
    sd0 = {k: t.detach().clone() for k, t in m.state_dict().items()}
    grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
    opt.step()
    sd1 = {k: t.detach().clone() for k, t in m.state_dict().items()}

    arrays = {"src": src, "tgt_in": tin, "tgt_out": tout, "src_kpm": skpm, "tgt_kpm": tkpm,
              "logits": logits.detach().numpy(), "attn": attn.detach().numpy(),
              "loss": np.float32(loss.detach()), "denom": np.float32(denom),
              "pe_head": sd0["pos_enc.pe"][:64, 0].numpy()}
    for k, t in sd0.items():
        if k != "pos_enc.pe":
            arrays["w/" + k] = t.numpy()
    for k, t in grads.items():
        arrays["g/" + k] = t.numpy()
    for k in ("fc.weight", "embedding.weight", "transformer.encoder.layers.0.self_attn.in_proj_weight",
              "transformer.decoder.layers.1.linear2.bias", "transformer.decoder.norm.weight"):
        arrays["adam1/" + k] = sd1[k].numpy()
    np.savez_compressed(os.path.join(OUT, "forward_train_micro.npz"), **arrays)
    meta = {"config": MICRO, "vocab": [0, CTRL], "eos_weight": eos_weight, "parts": parts,
            "torch": torch.__version__, "dropout": 0.0, "lr": 1e-4,
            "note": "reference ScoreTransformer eval(), seed 0, xavier_normal re-init"}
    with open(os.path.join(OUT, "forward_train_micro.json"), "w") as f:
        json.dump(meta, f, indent=1)
    return v, m


def sampling_mask_golden(v):
    """Allowed-id sets of `sampling` per flag combination (generation.py:41-88)."""
    captured = []
    orig = ref_gen.softmax_with_temperature

    def cap(logits, temperature):
        captured.append(np.array(logits))
        return orig(logits, temperature)
    ref_gen.softmax_with_temperature = cap
    combos = [dict(no_rest=True, no_sep=True, no_eos=True, no_whole_duration=True, no_control=True),
              dict(no_rest=True, no_sep=True, no_duration=True, no_continue=True, no_eos=True,
                   no_control=True),
              dict(no_rest=True, no_sep=True, no_continue=True, no_whole_duration=True, no_eos=True,
                   no_control=True),
              dict(no_rest=True, no_sep=True, no_continue=True, no_whole_duration=False,
                   no_eos=True, no_control=True),
              dict(no_pitch=True, no_rest=True, no_sep=True, no_continue=True,
                   no_whole_duration=True, no_eos=True, no_control=True),
              dict(is_density=True), dict(is_occupation=True), dict(is_polyphony=True),
              dict(is_tensile=True), dict(no_duration=True, no_control=True),
              dict(no_whole_duration=True, no_control=True),
              dict(no_whole_duration=False, no_control=True)]
    out = []
    np.random.seed(0)
    for c in combos:
        captured.clear()
        ref_gen.sampling(torch.arange(v.vocab_size, dtype=torch.float32) / 100.0, v, **c)
        keep = (captured[0] != -100)
        out.append({"flags": c, "allowed": np.nonzero(keep)[0].tolist()})
    ref_gen.softmax_with_temperature = orig
    with open(os.path.join(OUT, "sampling_masks.json"), "w") as f:
        json.dump(out, f)


def infill_golden(v, m):
    """generation_all on synthetic plugin-format events: greedy (weighted_sampling
    patched to argmax) and seeded sampling."""
    m.eval()
    logger = logging.getLogger("golden")
    all_controls = v.density_indices + v.occupation_indices + v.polyphony_indices + \
        v.tensile_indices
    cases = [dict(seed=0, n_bars=4, n_tracks=2, tracks=[1], bars=[1, 2]),
             dict(seed=1, n_bars=3, n_tracks=3, tracks=[0, 2], bars=[0]),
             dict(seed=2, n_bars=4, n_tracks=3, tracks=[2], bars=[3])]
    recs = []
    orig_ws = ref_gen.weighted_sampling
    orig_mg = ref_gen.model_generate
    for mode in ("greedy", "sample"):
        for c in cases:
            events = synth_events(c["seed"], c["n_bars"], c["n_tracks"])
            calls = []

            def mg(model, src, tgt, device, return_weights=False):
                calls.append(list(tgt))
                return orig_mg(model, src, tgt, device, return_weights)
            ref_gen.model_generate = mg
            if mode == "greedy":
                ref_gen.weighted_sampling = lambda probs: int(np.argmax(probs))
            else:
                ref_gen.weighted_sampling = orig_ws
                np.random.seed(1234 + c["seed"])
            ev_in = list(events)
            res = ref_gen.generation_all(m, list(events), "cpu", v, logger, all_controls,
                                         c["tracks"], c["bars"])
            ref_gen.model_generate = orig_mg
            ref_gen.weighted_sampling = orig_ws
            restored, mtn, mbn = res
            recs.append({"mode": mode, "case": c, "events": ev_in,
                         "restored": [str(x) for x in restored], "mask_track_names": mtn,
                         "mask_bar_names": mbn, "n_calls": len(calls),
                         "final_prefix": calls[-1], "prefix_lengths": [len(x) for x in calls]})
    with open(os.path.join(OUT, "infill_micro.json"), "w") as f:
        json.dump({"all_controls": all_controls, "cases": recs}, f, default=int)


def mask_golden(v):
    recs = []
    for seed, nb, nt, tracks, bars in ((3, 4, 2, [0], [0, 3]), (4, 2, 3, [1, 2], [1]),
                                       (5, 3, 1, [0], [2])):
        events = synth_events(seed, nb, nt)
        toks, mtn, mbn = ref_gen.mask_bar_and_track(events, v, tracks, bars)
        recs.append({"events": events, "tracks": tracks, "bars": bars,
                     "tokens": [int(t) for t in toks], "mask_track_names": mtn,
                     "mask_bar_names": mbn})
    with open(os.path.join(OUT, "mask_bar_and_track.json"), "w") as f:
        json.dump(recs, f, default=int)


if __name__ == "__main__":
    torch.set_num_threads(8)
    vocab_golden()
    v, _ = forward_and_train_golden()
    sampling_mask_golden(v)
    mask_golden(v)
    _, m0 = build_model(0)  # fresh (pre-Adam) weights = the w/ arrays of the npz
    infill_golden(v, m0)
    print("golden written to", OUT)
