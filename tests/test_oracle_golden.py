"""Pin the oracle (and the host wire/vocab layer) to the reference's own
outputs captured in tests/golden/ (see tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ref_cpu
from smer_music_generation_amd import wire
from smer_music_generation_amd.vocab import WordVocab

CTRL = ['key', 'tensile', 'density', 'polyphony', 'occupation']


def _load(golden_dir):
    z = np.load(os.path.join(golden_dir, "forward_train_micro.npz"))
    meta = json.load(open(os.path.join(golden_dir, "forward_train_micro.json")))
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    return z, meta, sd


def test_vocab_matches_reference(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "vocab_golden.json")))
    for key, rec in g.items():
        mode, cl = key.split("|")
        v = WordVocab(int(mode), [c for c in cl.split(",") if c])
        assert v._char2idx == rec["char2idx"]
        assert v.vocab_size == rec["vocab_size"]
        assert {str(k): c for k, c in v.token_class_ranges.items()} == rec["token_class_ranges"]
        assert v.name_to_tokens == rec["name_to_tokens"]
        assert v.control_tokens == rec["control_tokens"]
        assert v.control_indices == rec["control_indices"]
        assert sorted(v.class_names) == rec["class_names"]
        for a in ("structure_indices", "pitch_indices", "mask_indices", "duration_indices",
                  "duration_only_indices", "program_indices", "tempo_indices",
                  "time_signature_indices", "rest_indices", "sep_indices"):
            assert getattr(v, a) == rec[a], a
        if int(mode) == 0:
            assert v.continue_index == rec["continue_index"]


def test_pe_matches_reference(golden_dir):
    z, meta, _ = _load(golden_dir)
    pe = ref_cpu.pe_table(64, meta["config"]["d_model"])[:, 0].numpy()
    np.testing.assert_allclose(pe, z["pe_head"], rtol=0, atol=1e-6)


def test_oracle_forward_matches_reference(golden_dir):
    z, meta, sd = _load(golden_dir)
    cfg = dict(meta["config"])
    src, tin = torch.from_numpy(z["src"]), torch.from_numpy(z["tgt_in"])
    skpm, tkpm = torch.from_numpy(z["src_kpm"]), torch.from_numpy(z["tgt_kpm"])
    T = tin.shape[1]
    mask = ref_cpu.nopeek_mask(T).unsqueeze(0).repeat(src.shape[0], 1, 1)
    with torch.no_grad():
        logits, attn = ref_cpu.forward(sd, cfg, src, tin, skpm, tkpm, skpm.clone(), mask)
    np.testing.assert_allclose(logits.numpy(), z["logits"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(attn.numpy(), z["attn"], rtol=0, atol=1e-6)


def test_oracle_loss_grads_adam_match_reference(golden_dir):
    z, meta, sd = _load(golden_dir)
    cfg = dict(meta["config"])
    v = WordVocab(0, CTRL)
    batch = {"input": z["src"], "target_in": z["tgt_in"], "target_out": z["tgt_out"],
             "input_pad_mask": z["src_kpm"], "target_pad_mask": z["tgt_kpm"]}
    loss, parts, grads, _ = ref_cpu.train_step(sd, cfg, batch, v.control_indices,
                                               meta["eos_weight"], len(v.duration_indices))
    assert abs(float(loss) - float(z["loss"])) <= 1e-6 * max(1.0, abs(float(z["loss"])))
    for k, val in meta["parts"].items():
        assert abs(parts[k] - val) <= 1e-6 * max(1.0, abs(val)), k
    for k in grads:
        ref = z["g/" + k]
        np.testing.assert_allclose(grads[k].numpy(), ref, rtol=1e-4,
                                   atol=1e-6 * max(1.0, np.abs(ref).max()), err_msg=k)
    params = {k: t.clone() for k, t in sd.items()}
    m = {k: torch.zeros_like(t) for k, t in params.items()}
    s = {k: torch.zeros_like(t) for k, t in params.items()}
    ref_cpu.adam_step(params, grads, m, s, 1, lr=meta["lr"])
    for k in z.files:
        if k.startswith("adam1/"):
            np.testing.assert_allclose(params[k[6:]].numpy(), z[k], rtol=0, atol=2e-7, err_msg=k)


def test_sampling_masks_match_reference(golden_dir):
    v = WordVocab(0, CTRL)
    for rec in json.load(open(os.path.join(golden_dir, "sampling_masks.json"))):
        keep = ref_cpu.allowed_mask(v, **rec["flags"])
        assert np.nonzero(keep)[0].tolist() == rec["allowed"], rec["flags"]


def test_mask_bar_and_track_matches_reference(golden_dir):
    v = WordVocab(0, CTRL)
    for rec in json.load(open(os.path.join(golden_dir, "mask_bar_and_track.json"))):
        toks, mtn, mbn = wire.mask_bar_and_track(list(rec["events"]), v, rec["tracks"], rec["bars"])
        assert toks.tolist() == rec["tokens"]
        assert mtn == rec["mask_track_names"] and mbn == rec["mask_bar_names"]


@pytest.mark.parametrize("mode", ["greedy", "sample"])
def test_oracle_infill_matches_reference(golden_dir, mode):
    z, meta, sd = _load(golden_dir)
    sd["pos_enc.pe"] = ref_cpu.pe_table(2400, meta["config"]["d_model"])
    cfg = dict(meta["config"])
    v = WordVocab(0, CTRL)
    g = json.load(open(os.path.join(golden_dir, "infill_micro.json")))
    fn = ref_cpu.full_recompute_logits_fn(sd, cfg)
    for rec in g["cases"]:
        if rec["mode"] != mode:
            continue
        c = rec["case"]
        events = list(rec["events"])
        target, tracks = wire.mask_targets(events, c["tracks"], c["bars"])
        src, mtn, mbn = wire.mask_bar_and_track(events, v, tracks, c["bars"])
        ts = events[0]
        no_whole = not (int(ts[0]) >= 4 and int(ts[2]) == 4)
        if mode == "sample":
            np.random.seed(1234 + c["seed"])
        trace = []
        total, tgt_inp = ref_cpu.infill(fn, src, target, v, g["all_controls"], no_whole,
                                        greedy=(mode == "greedy"), trace=trace)
        assert trace == rec["prefix_lengths"]
        src_tok = [v.index2char(int(t)) for t in src]
        restored = wire.restore_marked_input(src_tok, total)
        assert [str(x) for x in restored] == rec["restored"]
        assert (mtn, mbn) == (rec["mask_track_names"], rec["mask_bar_names"])
