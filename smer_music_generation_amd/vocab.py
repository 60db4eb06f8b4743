"""SMER token vocabulary — the token-id interface the engine keeps.

Mirrors `WordVocab` of the reference (`vocab.py:114-338`, identical copy in
`vocab_control.py`): same constructor ``WordVocab(mode, control_list)``, same
ids, same index lists and class maps, pickle-compatible save/load.  The id
layout for mode 0 (SMER) is 309 tokens, independent of ``control_list``
(SURVEY.md Appendix A); mode 1 (REMI-style step tokens) is 349 tokens.

The token groups are built here from their definitions (reference
`vocab.py:20-112`), in the order the reference concatenates them
(`vocab.py:129-138`): specials, mask, structure, song tokens, note tokens,
then density / polyphony / occupation / key / tensile / unk.
"""
from __future__ import annotations

import pickle

import numpy as np

# ---- token groups (reference vocab.py:20-112) --------------------------------
PAD, EOS = "<pad>", "<eos>"
MASK_TOKENS = ["m_0"]
TIME_SIGNATURES = ["4/4", "3/4", "2/4", "6/8"]
PROGRAMS = ["i_%d" % n for n in range(128)]
TEMPOS = ["t_%d" % n for n in range(7)]
TRACKS = ["track_%d" % n for n in range(3)]
STRUCTURE = ["bar"] + TRACKS
SONG = TIME_SIGNATURES + TEMPOS + PROGRAMS
REST, SEP, CONTINUE = "rest", "sep", "continue"
STEPS = ["e_%d" % n for n in range(16)]
DURATION_MULTI = ["whole", "half", "quarter", "eighth", "sixteenth"]
DURATION_SINGLE = ["n_%d" % n for n in range(1, 33)]
PITCHES = ["p_%d" % n for n in range(21, 109)]
KEY_NAMES = ["C major", "G major", "D major", "A major", "E major", "B major",
             "F major", "B- major", "E- major", "A- major", "D- major", "G- major",
             "A minor", "E minor", "B minor", "F# minor", "C# minor", "G# minor",
             "D minor", "G minor", "C minor", "F minor", "B- minor", "E- minor"]
KEYS = ["k_%d" % n for n in range(len(KEY_NAMES))]
KEY_TO_TOKEN = {name: "k_%d" % i for i, name in enumerate(KEY_NAMES)}
TOKEN_TO_KEY = {v: k for k, v in KEY_TO_TOKEN.items()}
DENSITY = ["d_%d" % n for n in range(10)]
OCCUPATION = ["o_%d" % n for n in range(10)]
POLYPHONY = ["y_%d" % n for n in range(10)]
TENSILE = ["s_%d" % n for n in range(12)]
UNK = ["unk"]

# control groups a run may enable (train.py:1393-1407 control_number map)
ALL_CONTROLS = ["key", "tensile", "density", "polyphony", "occupation"]
_CONTROL_GROUPS = {"key": KEYS, "density": DENSITY, "occupation": OCCUPATION,
                   "polyphony": POLYPHONY, "tensile": TENSILE}


class WordVocab(object):
    """Token <-> id map with the reference's attribute surface (`vocab.py:114`)."""

    def __init__(self, mode, control_list):
        mode = int(mode)
        if mode == 0:
            durations_only = list(DURATION_MULTI)
            duration_group = durations_only + [REST, SEP, CONTINUE]
        else:
            durations_only = list(DURATION_SINGLE)
            duration_group = STEPS + durations_only
        self.mode = mode
        basic = [PAD, EOS] + MASK_TOKENS + STRUCTURE + SONG + PITCHES + duration_group
        ordered = basic + DENSITY + POLYPHONY + OCCUPATION + KEYS + TENSILE + UNK

        self.pad_index = 0
        self.eos_index = 1
        self.char_lst = ordered
        self.basic_tokens = basic
        self.corrupt_tokens = list(UNK)
        self._char2idx = {}
        for tok in ordered:
            self._char2idx.setdefault(tok, len(self._char2idx))
        self._idx2char = {i: t for t, i in self._char2idx.items()}
        print('vocab size: %d' % self.vocab_size)

        ids = lambda toks: [self._char2idx[t] for t in toks]
        self.structure_indices = ids(STRUCTURE)
        self.pitch_indices = ids(PITCHES)
        self.mask_indices = ids(MASK_TOKENS)
        self.duration_indices = ids(duration_group)
        self.duration_only_indices = ids(durations_only)
        self.program_indices = ids(PROGRAMS)
        self.tempo_indices = ids(TEMPOS)
        self.time_signature_indices = ids(TIME_SIGNATURES)
        self.rest_indices = ids([REST]) if mode == 0 else []
        self.sep_indices = ids([SEP]) if mode == 0 else []
        if mode == 0:
            self.continue_index = self._char2idx[CONTINUE]
        else:
            self.step_indices = ids(STEPS)

        self.token_class_ranges = {}
        self.name_to_tokens = {}
        self.control_indices = {}
        self.control_tokens = []
        # class registration order follows the reference (vocab.py:186-236):
        # program, rest, sep, tempo, time_signature, structure, pitch, duration
        for cname, idxs in (("program", self.program_indices), ("rest", self.rest_indices),
                            ("sep", self.sep_indices), ("tempo", self.tempo_indices),
                            ("time_signature", self.time_signature_indices),
                            ("structure", self.structure_indices), ("pitch", self.pitch_indices),
                            ("duration", self.duration_indices)):
            self._register_class(cname, idxs)
        self.token_class_ranges[self.eos_index] = 'eos'
        self.token_class_ranges[self.vocab_size - 1] = 'unk'
        self.name_to_tokens['eos'] = EOS

        for cname in ("key", "density", "occupation", "polyphony", "tensile"):
            if cname not in control_list:
                continue
            idxs = ids(_CONTROL_GROUPS[cname])
            setattr(self, cname + "_indices", idxs)
            self.control_indices[cname] = idxs
            self._register_class(cname, idxs)
            self.control_tokens.extend(self.name_to_tokens[cname])
        self.class_names = set(self.token_class_ranges.values())

    def _register_class(self, cname, idxs):
        for i in idxs:
            self.token_class_ranges[i] = cname
            self.name_to_tokens.setdefault(cname, []).append(self._idx2char[i])

    # --- reference accessors (vocab.py:312-329) ---
    def char2index(self, token):
        if token not in self._char2idx:
            print('invalid')
        return self._char2idx.get(token)

    def index2char(self, idxs):
        return self._idx2char.get(idxs)

    def get_token_classes(self, idx):
        return self.token_class_ranges[idx]

    @property
    def vocab_size(self):
        return len(self._char2idx)

    def save_vocab(self, vocab_path):
        with open(vocab_path, "wb") as f:
            pickle.dump(self, f)

    @staticmethod
    def load_vocab(vocab_path: str) -> 'WordVocab':
        with open(vocab_path, "rb") as f:
            return pickle.load(f)


def control_list_for(control_number: int):
    """`train.py:1393-1407`: CLI control_number -> control_list."""
    return {0: [], 1: ['key', 'tensile'], 2: ['key', 'density'], 3: ['key', 'polyphony'],
            4: ['key', 'occupation'],
            5: ['key', 'tensile', 'density', 'polyphony', 'occupation']}[int(control_number)]


def id_masks(vocab: WordVocab):
    """Boolean [V] masks per token class, used by the vectorised sampler."""
    V = vocab.vocab_size
    out = {}
    for name in ("pitch_indices", "duration_only_indices", "rest_indices", "sep_indices",
                 "program_indices", "structure_indices", "time_signature_indices",
                 "tempo_indices"):
        m = np.zeros(V, dtype=bool)
        m[getattr(vocab, name)] = True
        out[name] = m
    for cname in ("density", "occupation", "polyphony", "tensile"):
        m = np.zeros(V, dtype=bool)
        idx = getattr(vocab, cname + "_indices", None)
        if idx is not None:
            m[idx] = True
        out[cname] = m
    return out
