"""Infill call surface of the plugin (reference `generation.py`).

Same names, signatures, return values and error behaviour as the
reference: `model_generate` (209-225), `generation_all` (468-696),
`sampling` (41-95), `softmax_with_temperature` (28-30), `weighted_sampling`
(33-38), `nucleus` (11-25), `gen_nopeek_mask` (193-206), plus the wire
helpers (`mask_bar_and_track`, `restore_marked_input`, `fill_empty_bars`,
`change_controls`) and the north-star alias `infill = generation_all`.

Differences, all opt-in keywords with reference defaults:
  * `generation_all(..., use_kv_cache=True)`: decode through the KV-cached
    `DecodeSession` (one encoder pass per request) instead of re-running the
    full model per token; `use_kv_cache=False` is the reference algorithm.
  * `greedy=False`: True replaces `weighted_sampling` by argmax.
  * `generation_all(..., precision="fp32")`: the plugin call decodes in
    fp32 whatever precision the model trains in (bit-exact ids); None
    decodes at the model's own precision.
  * `generation_batch(...)`: many requests decoded in lockstep.
The grammar state machine, the -100 logit masking, the float64 softmax and
the numpy RNG consumption are the reference's, so with the same
`np.random` state the same token ids come out.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .decode import DecodeSession
from .durations import durations_for_events
from .wire import (change_controls, fill_empty_bars, mask_bar_and_track,  # noqa: F401
                   mask_targets, restore_marked_input)


# --------------------------------------------------------------------------
# sampling (generation.py:11-95)
# --------------------------------------------------------------------------
def nucleus(probs, p):
    probs /= (sum(probs) + 1e-5)
    sorted_probs = np.sort(probs)[::-1]
    sorted_index = np.argsort(probs)[::-1]
    csum = np.cumsum(sorted_probs)
    after = csum > p
    if sum(after) > 0:
        cand = sorted_index[:np.where(after)[0][0] + 1]
    else:
        cand = sorted_index[:]
    cp = np.array([probs[i] for i in cand])
    cp /= sum(cp)
    return np.random.choice(cand, size=1, p=cp)[0]


def softmax_with_temperature(logits, temperature):
    e = np.exp(logits / temperature)
    return e / np.sum(e)


def weighted_sampling(probs):
    # the reference's builtin sum() adds left to right from 0: the last
    # element of the (sequential) cumulative sum is that number exactly, in
    # 1/12 of the time; probs[argsort] holds np.sort's values (ties are
    # equal values), so one sort serves both.  `probs` is float64 here
    # (sampling() widens the logits before the softmax), so builtin sum()
    # adds float64 scalars under NumPy 1.x and 2.x alike: no promotion-rule
    # dependence; a float32 input is rejected rather than silently diverging
    if probs.dtype != np.float64:
        raise TypeError("weighted_sampling expects float64 probabilities")
    probs /= np.add.accumulate(probs)[-1]
    sorted_index = np.argsort(probs)[::-1]
    return _choice1(sorted_index, probs[sorted_index])


def _choice1(a, p):
    """np.random.choice(a, size=1, p=p)[0] on the global RandomState, without
    its argument checks (a third of the per-token host time): NumPy's legacy
    `RandomState.choice` with replacement draws ONE `random_sample` and
    returns a[searchsorted(cdf / cdf[-1], u, side='right')], so the same
    uniform gives the same index and leaves the same generator state.  Any
    input its checks would reject (a negative or NaN entry, a sum off 1)
    goes to np.random.choice itself, so the errors are NumPy's own
    (tests/test_sampling.py compares the two on seeded streams)."""
    cdf = np.cumsum(p)
    total = cdf[-1]
    if not (abs(total - 1.0) <= 1e-9) or not (p >= 0.0).all():
        return np.random.choice(a, size=1, p=p)[0]
    cdf /= total
    u = np.random.random_sample(1)
    return a[cdf.searchsorted(u, side='right')][0]


_FLAG_NAMES = ("no_pitch", "no_duration", "no_rest", "no_whole_duration", "no_eos",
               "no_continue", "no_sep", "is_density", "is_polyphony", "is_occupation",
               "is_tensile", "no_control")
_MASK_CACHE = {}


def allowed_ids(vocab, **flags):
    """Boolean [V]: logits `sampling` keeps (others become -100).  The
    reference's `no_control` test (`i in dict.values()`) never matches
    (SURVEY Q1), so it is a no-op here too."""
    key = (id(vocab),) + tuple(map(bool, map(flags.get, _FLAG_NAMES)))
    hit = _MASK_CACHE.get(key)
    if hit is not None:
        return hit
    V = vocab.vocab_size
    keep = np.ones(V, dtype=bool)
    g = flags.get
    if g("no_pitch"):
        keep[vocab.pitch_indices] = False
    if g("no_duration"):
        keep[vocab.duration_only_indices] = False
    if g("no_continue"):
        keep[vocab.continue_index] = False
    if g("no_rest"):
        keep[vocab.rest_indices] = False
    if g("no_sep"):
        keep[vocab.sep_indices] = False
    if g("no_whole_duration"):
        keep[vocab.duration_only_indices[0]] = False
    if g("no_eos"):
        keep[vocab.eos_index] = False
    for flag, attr in (("is_density", "density_indices"), ("is_occupation", "occupation_indices"),
                       ("is_polyphony", "polyphony_indices"), ("is_tensile", "tensile_indices")):
        if g(flag):
            only = np.zeros(V, dtype=bool)
            only[getattr(vocab, attr)] = True
            keep &= only
    keep[vocab.program_indices + vocab.structure_indices + vocab.time_signature_indices +
         vocab.tempo_indices] = False
    keep.setflags(write=False)
    _MASK_CACHE[key] = keep
    return keep


def sampling(logit, vocab, p=None, t=1.0, greedy=False, **flags):
    """`generation.py:41-95` with vectorised masking."""
    if isinstance(logit, torch.Tensor):
        logit = logit.squeeze().detach().cpu().numpy()
    lg = np.where(allowed_ids(vocab, **flags), np.asarray(logit, dtype=np.float32).astype(np.float64),
                  -100.0)
    probs = softmax_with_temperature(lg, t)
    if greedy:
        return int(np.argmax(probs))
    if p is not None:
        return nucleus(probs, p)
    return weighted_sampling(probs)


def gen_nopeek_mask(length):
    m = (torch.triu(torch.ones(length, length)) == 1).transpose(0, 1)
    return m.float().masked_fill(m == 0, float("-inf")).masked_fill(m == 1, 0.0)


def model_generate(model, src, tgt, device, return_weights=False):
    """`generation.py:209-225`: batch-1 full forward; logits [t, V] on CPU."""
    src = torch.as_tensor(src).clone().detach().unsqueeze(0).long().to(device)
    tgt = torch.tensor(tgt).unsqueeze(0).to(device)
    mask = gen_nopeek_mask(tgt.shape[1]).unsqueeze(0).to(device)
    with torch.no_grad():
        out, w = model.forward(src, tgt, src_key_padding_mask=None, tgt_key_padding_mask=None,
                               memory_key_padding_mask=None, tgt_mask=mask)
    if return_weights:
        return out.squeeze(0).to("cpu"), (w.squeeze(0).to("cpu") if w is not None else None)
    return out.squeeze(0).to("cpu")


# --------------------------------------------------------------------------
# the per-span grammar state machine (generation.py:528-687)
# --------------------------------------------------------------------------
N_GRAMMAR_STATES = 13


def _target_code(tc):
    """Control target of a mask: 'r' 0, 'd' 1, 'o' 2, 'p' 3, anything else
    't' 4 (the reference's `else: is_tensile`, generation.py:575-583)."""
    return {'r': 0, 'd': 1, 'o': 2, 'p': 3}.get(tc, 4)


_SPEC_CACHE = {}


def grammar_spec(v, code):
    """(sampling flags, redraw check, failure message) of grammar state
    `code`, built once per (vocab, code) (the per-token host replay of the
    device decode calls this for every emitted id)."""
    key = (id(v), code)
    hit = _SPEC_CACHE.get(key)
    if hit is None or hit[0] is not v:
        hit = (v, _grammar_spec(v, code))
        _SPEC_CACHE[key] = hit
    return hit[1]


def _grammar_spec(v, code):
    """(sampling flags, redraw check, failure message) of grammar state
    `code` (generation.py:549-630):
    0 sep, 1 continue, 2/3 pitch, 4/5 rest (+no_whole), 6-9 first token of a
    d/o/p/t control span, 10 first token of a note span, 11/12 free."""
    if code == 0:
        return (dict(no_rest=True, no_sep=True, no_eos=True, no_whole_duration=True,
                     no_control=True),
                lambda i: i in v.rest_indices or i == v.eos_index or
                i == v.duration_only_indices[0], "in sep failed")
    if code == 1:
        return (dict(no_rest=True, no_sep=True, no_duration=True, no_continue=True,
                     no_eos=True, no_control=True),
                lambda i: i not in v.pitch_indices, 'in continue failed')
    if code in (2, 3):
        return (dict(no_rest=True, no_sep=True, no_continue=True,
                     no_whole_duration=code == 3, no_eos=True, no_control=True),
                lambda i: i not in v.duration_only_indices and i not in v.pitch_indices,
                'in pitch failed')
    if code in (4, 5):
        return (dict(no_pitch=True, no_rest=True, no_sep=True, no_continue=True,
                     no_whole_duration=code == 5, no_eos=True, no_control=True),
                lambda i: i not in v.duration_only_indices, 'in rest failed')
    if 6 <= code <= 9:
        return {('is_density', 'is_occupation', 'is_polyphony', 'is_tensile')[code - 6]: True}, None, ''
    if code == 10:
        return (dict(no_duration=True, no_control=True),
                lambda i: i in v.duration_only_indices, 'start failed')
    return dict(no_whole_duration=code == 12, no_control=True), None, ''


def grammar_tables(vocab, all_controls):
    """Device tables of the greedy grammar kernel: keep uint8 [13, V]
    (allowed_ids of every state) and token classes cls uint8 [V]
    (1 continue, 2 pitch, 4 duration-only, 8 'sep', 16 'rest', 32 control)."""
    V = vocab.vocab_size
    keep = np.stack([allowed_ids(vocab, **grammar_spec(vocab, c)[0])
                     for c in range(N_GRAMMAR_STATES)]).astype(np.uint8)
    cls = np.zeros(V, dtype=np.uint8)
    if getattr(vocab, "continue_index", None) is not None:
        cls[vocab.continue_index] |= 1
    cls[vocab.pitch_indices] |= 2
    cls[vocab.duration_only_indices] |= 4
    for i in range(V):
        ch = vocab.index2char(i)
        if ch == 'sep':
            cls[i] |= 8
        if ch == 'rest':
            cls[i] |= 16
    cls[[int(c) for c in all_controls]] |= 32
    return keep, cls


class _Span:
    """Decoding state of one request: mask index, span tokens, grammar flags."""

    def __init__(self, vocab, src, mask_target, all_controls, no_whole, greedy, logger):
        self.v = vocab
        self.src = src
        self.mask_target = mask_target
        self.all_controls = set(int(c) for c in all_controls)
        self.no_whole = no_whole
        self.greedy = greedy
        self.logger = logger
        self.m0 = vocab.char2index('m_0')
        self.eos = vocab.char2index('<eos>')
        self._pitch = frozenset(vocab.pitch_indices)
        self._dur = frozenset(vocab.duration_only_indices)
        self.n_masks = int(np.sum(np.asarray(src) == self.m0))
        self.mask_idx = 0
        self.tgt_inp = []
        self.total = []
        self.done = self.n_masks == 0
        self._start_span()

    def _start_span(self):
        self.this_in = [self.m0]
        self.this_ev = ['m_0']
        self.in_pitch = self.in_rest = self.in_sep = self.in_continue = False

    def prefix(self):
        return self.tgt_inp + self.this_in

    def _draw(self, logit, check, failmsg, flags):
        idx = sampling(logit, self.v, greedy=self.greedy, **flags)
        if check is None:
            return idx
        n = 0
        while check(idx):
            idx = sampling(logit, self.v, greedy=self.greedy, **flags)
            n += 1
            if n > 10:
                if self.logger is not None:
                    self.logger.info(failmsg)
                break
        return idx

    def state_code(self):
        """Grammar state of the current prefix (generation.py:549-630), the
        code csrc/decode_ops.hip grammar_state() computes on device."""
        nw = int(bool(self.no_whole))
        if self.in_sep:
            return 0
        if self.in_continue:
            return 1
        if self.in_pitch:
            return 2 + nw
        if self.in_rest:
            return 4 + nw
        if len(self.this_in) == 1:
            tc = _target_code(self.mask_target[self.mask_idx])
            return 10 if tc == 0 else 5 + tc
        return 11 + nw

    def spec(self):
        """(sampling flags, redraw check, failure message) of the current
        grammar state (generation.py:549-630)."""
        return grammar_spec(self.v, self.state_code())

    def advance(self, logit):
        """Consume the logits of the current prefix's last position."""
        flags, check, failmsg = self.spec()
        return self.commit(self._draw(logit, check, failmsg, flags))

    def commit_greedy(self, idx, check, failmsg):
        """Greedy draw already taken (argmax over the masked logits): the
        reference's redraw loop would re-draw the same id 11 times."""
        if self.logger is not None and check is not None and check(int(idx)):
            self.logger.info(failmsg)
        return self.commit(idx)

    def commit_all(self, seq):
        """commit() over a whole emitted id sequence when nothing reads the
        grammar flags between its ids (the device greedy grammar with no
        redraw logger): the same tgt_inp / total / mask_idx / done, without
        the per-token flag updates (only spec() reads them, and a finished
        request never calls it again)."""
        i2c = self.v.index2char
        eos, ctrl = self.eos, self.all_controls
        this_in, this_ev = self.this_in, self.this_ev
        for idx in seq:
            if idx in ctrl:
                this_in += [idx, eos]
                this_ev += [i2c(idx), '<eos>']
            else:
                this_in.append(idx)
                this_ev.append(i2c(idx))
            if this_in[-1] == eos or len(this_in) >= 100:
                self.tgt_inp.extend(this_in[:-1])
                self.total.extend(this_ev[:-1])
                self.mask_idx += 1
                if self.mask_idx >= self.n_masks:
                    self.done = True
                else:
                    self._start_span()
                    this_in, this_ev = self.this_in, self.this_ev

    def commit(self, idx):
        v = self.v
        idx = int(idx)
        ev = v.index2char(idx)
        if idx == v.continue_index:
            self.in_continue, self.in_sep = True, False
        if idx in self._pitch:
            self.in_pitch, self.in_sep, self.in_continue = True, False, False
        if idx in self._dur:
            self.in_rest, self.in_pitch = False, False
        if ev == 'sep':
            self.in_sep = True
        if ev == 'rest':
            self.in_rest = True
        if idx in self.all_controls:
            self.this_in += [idx, self.eos]
            self.this_ev += [ev, '<eos>']
        else:
            self.this_in.append(idx)
            self.this_ev.append(ev)
        if self.this_in[-1] == self.eos or len(self.this_in) >= 100:
            self.tgt_inp.extend(self.this_in[:-1])
            self.total.extend(self.this_ev[:-1])
            self.mask_idx += 1
            if self.mask_idx >= self.n_masks:
                self.done = True
            else:
                self._start_span()
        return idx


def _src_tokens(vocab, src):
    """[vocab.index2char(int(t)) for t in src] (generation.py:685) through
    one dict lookup per id instead of a method call and an int() each."""
    table = getattr(vocab, "_idx2char", None)
    get = table.get if isinstance(table, dict) else vocab.index2char
    return list(map(get, src.tolist() if hasattr(src, "tolist") else list(src)))


def _prepare(events, vocab, tracks_to_generate, bars_to_generate):
    """generation.py:470-516: duration tables, mask targets, masked src."""
    name_to_time, time_to_name, times, bar_duration = durations_for_events(events)
    n_bars = events.count('bar') if isinstance(events, list) else sum(1 for e in events if e == 'bar')
    target, tracks = mask_targets(events, tracks_to_generate, bars_to_generate)
    if bars_to_generate[-1] >= n_bars:
        events = fill_empty_bars(events, bars_to_generate[-1] - n_bars + 1, bar_duration,
                                 time_to_name, times)
    src, mtn, mbn = mask_bar_and_track(events, vocab, tracks, bars_to_generate)
    no_whole = not (int(events[0][0]) >= 4 and int(events[0][2]) == 4)
    return src, mtn, mbn, target, no_whole


class _Precision:
    """Run a block at another arithmetic precision of the model, restoring
    the model's own afterwards (the plugin call decodes in fp32 whatever
    precision the model trains in)."""

    def __init__(self, model, precision):
        self.model, self.want = model, precision
        self.prev = None

    def __enter__(self):
        if self.want is not None and self.want != self.model.precision:
            self.prev = self.model.precision
            self.model.set_precision(self.want)
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            self.model.set_precision(self.prev)
        return False


def generation_all(model, events, device, vocab, logger, all_controls, tracks_to_generate,
                   bars_to_generate, *, greedy=False, use_kv_cache=True, stats=None,
                   precision="fp32", warm=True, device_grammar=True):
    """`generation.py:468-696`.  Returns (restored '<U9' tokens,
    mask_track_names, mask_bar_names) or None (nothing masked / on error,
    after printing it, as the reference does).  `stats` (a dict, opt-in)
    receives the number of decode steps (= tokens drawn).
    warm: decode on this model's cached batch-1 session (KV caches and the
    captured step graph kept across calls, as in generation_batch); False
    builds a private session freed after the call.  A warm session is not
    re-entrant: concurrent calls on one model (threads) would share its
    caches and graph, so serialise them or pass warm=False.
    precision: arithmetic of this call's decode.  "fp32" (default) gives
    the reference's token ids bit for bit (north_star: bit-exact greedy ids;
    sampled ids are the same draws of the same numpy stream) whatever
    precision the model trains in; None decodes at the model's own precision
    (bf16 for a default-constructed model: faster, ids may differ at
    near-ties); the batched serving API `generation_batch` keeps None.
    device_grammar: (KV-cached path) run the grammar and the draws on the
    device inside the captured decode step -- greedy argmax, or the default
    weighted sampling on numpy's MT19937 stream handed to the device and back
    (csrc/decode_ops.hip grammar_sample_kernel) -- with no host round trip
    per token; False keeps the per-token host loop."""
    with _Precision(model, precision):
        return _generation_all(model, events, device, vocab, logger, all_controls,
                               tracks_to_generate, bars_to_generate, greedy, use_kv_cache, stats,
                               warm, device_grammar)


_REJECT_CACHE = {}


def reject_table(vocab):
    """uint8 [13, V]: the redraw checks of the grammar states
    (generation.py:556-615; grammar_spec's check), 1 = redraw."""
    hit = _REJECT_CACHE.get(id(vocab))
    if hit is not None and hit[0] is vocab:
        return hit[1]
    V = vocab.vocab_size
    rej = np.zeros((N_GRAMMAR_STATES, V), dtype=np.uint8)
    for c in range(N_GRAMMAR_STATES):
        chk = grammar_spec(vocab, c)[1]
        if chk is not None:
            rej[c] = [bool(chk(i)) for i in range(V)]
    _REJECT_CACHE[id(vocab)] = (vocab, rej)
    return rej


def _sampled_on_device(sess, st, vocab, all_controls, logger):
    """One request's sampled span loop on device (DecodeSession.
    sampled_decode), then the emitted ids replayed through the host span
    (event lists, the redraw-failure log lines).  Returns the steps, or None
    when a row's probabilities missed 1 by more than 1e-9 (np.random.choice
    territory): the RNG is then rewound and the caller decodes on the host."""
    keep, cls = grammar_tables(vocab, all_controls)
    rng0 = np.random.get_state()
    seqs, steps, err, fails = sess.sampled_decode([st], keep, reject_table(vocab), cls,
                                                  eos=vocab.eos_index, m0=vocab.char2index('m_0'))
    if err[0] & 2:
        np.random.set_state(rng0)
        return None
    if err[0] & 1:
        raise ValueError("decoder prefix exceeds session max_tgt %d" % (sess.Tmax - 1))
    for idx, fail in zip(seqs[0], fails[0]):
        if fail and logger is not None:
            logger.info(st.spec()[2])
        st.commit(idx)
    if not st.done:
        raise RuntimeError("device grammar and host replay disagree")
    return len(seqs[0])


def _generation_all(model, events, device, vocab, logger, all_controls, tracks_to_generate,
                    bars_to_generate, greedy, use_kv_cache, stats, warm=True, device_grammar=True):
    try:
        src, mtn, mbn, target, no_whole = _prepare(events, vocab, tracks_to_generate,
                                                   bars_to_generate)
        st = _Span(vocab, src, target, all_controls, no_whole, greedy, logger)
        if st.n_masks == 0:
            return None
        model.eval()
        with torch.no_grad():
            steps = 0
            if use_kv_cache:
                # the warm batch-1 session of this model and precision: KV
                # caches, step buffers and the captured step graph persist
                # across plugin calls (same rules as generation_batch's)
                sess = _batch_session(model, 1, len(src), max(128, 100 * st.n_masks + 8), None,
                                      warm=warm)
                sess.prefill([0], [src])
                if device_grammar and not greedy and vocab.vocab_size <= 512:
                    n = _sampled_on_device(sess, st, vocab, all_controls, logger)
                    if n is not None:
                        steps = n
                    else:  # fresh span, same RNG start: the host loop below
                        st = _Span(vocab, src, target, all_controls, no_whole, greedy, logger)
                        sess.prefill([0], [src])
                fed = 0
                while not st.done:
                    pre = st.prefix()
                    logit = sess.step([(0, pre[fed:], fed)])[0]
                    fed = len(pre)
                    st.advance(logit)
                    steps += 1
            else:
                src_t = torch.tensor(src)
                while not st.done:
                    out = model_generate(model, src_t, st.prefix(), device)
                    st.advance(out[-1].numpy())
                    steps += 1
            if stats is not None:
                stats["steps"] = steps
        return restore_marked_input(_src_tokens(vocab, src), st.total), mtn, mbn
    except Exception as e:  # reference behaviour (generation.py:695-696)
        print(e)


infill = generation_all


# Warm decode sessions of generation_batch, one per (model, precision, R),
# at most two kept: the KV caches, step buffers and the captured step +
# grammar graph persist across calls (a serving process keeps them; capturing
# costs ~10 ms at C2).  A cached session is reused when the call's sources and
# prefix fit AND its cache capacities fall in the same decode-attention
# variant class as a fresh session's would (>= 512 key rows: 8-wave blocks;
# the kernels pick by capacity, and the variants sum in different orders), so
# reuse never changes a token.
_BATCH_SESSIONS = {}


def clear_decode_sessions(model=None):
    """Drop the warm decode sessions of `model` (all models when None),
    releasing their KV caches and captured graphs; the next
    generation_batch call builds a fresh session."""
    for key in [k for k, s in _BATCH_SESSIONS.items() if model is None or s.model is model]:
        del _BATCH_SESSIONS[key]


def _plugin_capacity(Smax, Tmax):
    """Capacities of a warm batch-1 (plugin) session: rounded up to powers of
    two (>= 128), so consecutive calls on sources / mask counts of similar
    size reuse one session and its captured graphs instead of rebuilding
    them (a rebuild + capture costs ~6 ms, 1/4 of a typical call); a fresh
    session for the same request rounds the same way.  The rounding never
    carries a capacity across 512 rows, where the decode attention switches
    to its 8-wave variant (another summation order), so warm and cold
    sessions give the same logits.  Tmax excludes the trash slot (the cache
    holds Tmax + 1 rows)."""
    S0, T0 = int(Smax), int(Tmax)
    S = 1 << max(7, (S0 - 1).bit_length())
    if S0 < 512:
        S = min(S, 511)
    T = (1 << max(7, T0.bit_length())) - 1
    if T0 + 1 < 512:
        T = min(T, 510)
    return S, T


def _batch_session(model, R, Smax, Tmax, precision, exact_tmax=False, warm=True):
    """A decode session for this call.  A cached one is reused only when it
    still addresses the model's current weight buffers (moving the model
    re-flattens them) and, for an explicit max_tgt, has exactly that
    capacity (so the 'prefix exceeds max_tgt' error depends on this call's
    arguments alone; the auto-sized capacity 100 * n_masks + 8 can never be
    exceeded).  Before reuse the working weights are re-synchronised with the
    fp32 master in place (a load_state_dict or an optimizer step since the
    last call), so prefill and the captured step read current weights."""
    if precision is not None:
        model.set_precision(precision)
    if not warm:
        return DecodeSession(model, R, Smax, Tmax)
    if R == 1 and not exact_tmax:
        Smax, Tmax = _plugin_capacity(Smax, Tmax)
    key = (id(model), model.precision, R)
    s = _BATCH_SESSIONS.get(key)
    fits = (s is not None and s.model is model and s.Smax >= Smax and s.Tmax >= Tmax + 1
            and (s.Tmax == Tmax + 1 or not exact_tmax)
            and (s.Smax >= 512) == (Smax >= 512) and (s.Tmax >= 512) == (Tmax + 1 >= 512))
    if fits:
        W = s.eng.weights(s.dt)  # re-casts in place when the master moved
        if W.fc_w.data_ptr() == s.W.fc_w.data_ptr() and W.emb.data_ptr() == s.W.emb.data_ptr():
            s.W = W
            s.src_len[:] = 0
            return s
    s = DecodeSession(model, R, Smax, Tmax)
    _BATCH_SESSIONS.pop(key, None)
    while len(_BATCH_SESSIONS) >= 2:
        _BATCH_SESSIONS.pop(next(iter(_BATCH_SESSIONS)))
    _BATCH_SESSIONS[key] = s
    return s


def generation_batch(model, requests, vocab, all_controls, *, greedy=True, logger=None,
                     max_tgt=None, precision=None, return_stats=False, device_grammar=True,
                     warm=True):
    """Decode many infill requests in lockstep on one KV-cached session.

    requests: list of (events, tracks_to_generate, bars_to_generate).
    Greedy decoding runs the grammar on device (`device_grammar`, the
    default): the step graph ends in the grammar kernel that picks every
    request's token and writes the next step's feed, so steps replay back
    to back; the emitted ids are then replayed through the host `_Span`s,
    which rebuild exactly the reference's event lists (and log the
    reference's redraw failures).  `device_grammar=False` (or sampling)
    keeps the per-step host loop.
    warm: reuse (and keep) this model's cached decode session, as a serving
    process would; False builds a private session freed after the call
    (see also clear_decode_sessions).
    Returns a list of (restored, mask_track_names, mask_bar_names) (None
    where nothing was masked), and optionally {'tokens', 'steps'}."""
    t0 = time.perf_counter()
    preps = [_prepare(list(ev), vocab, tr, br) for ev, tr, br in requests]
    spans = [_Span(vocab, p[0], p[3], all_controls, p[4], greedy, logger) for p in preps]
    R = len(requests)
    Smax = max(len(p[0]) for p in preps)
    Tmax = max_tgt or max(128, 100 * max(s.n_masks for s in spans) + 8)
    model.eval()
    tokens = steps = 0
    with torch.no_grad():
        sess = _batch_session(model, R, Smax, Tmax, precision, exact_tmax=max_tgt is not None,
                              warm=warm)
        t1 = time.perf_counter()
        sess.prefill(list(range(R)), [p[0] for p in preps])
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t_dev = 0.0
        fed = [0] * R
        latency = None
        kv_reads = None
        if greedy and device_grammar:
            keep, cls = grammar_tables(vocab, all_controls)
            m0 = vocab.char2index('m_0')
            ts = time.perf_counter()
            seqs, steps, err, step_ms = sess.greedy_decode(spans, keep, cls, eos=vocab.eos_index,
                                                           m0=m0)
            t_dev = time.perf_counter() - ts
            # completion time of each request from the call's start: host
            # preparation + prefill, then the GPU end time of its last step
            latency = [(ts - t0) + (step_ms[len(q) - 1] / 1000.0 if q else 0.0) for q in seqs]
            if np.any(err):
                raise ValueError("decoder prefix exceeds session max_tgt %d" % (sess.Tmax - 1))
            # key rows the decode steps attended to (SURVEY §8d infill bytes):
            # request r's i-th step reads its S_r memory rows and i+1 prefix rows
            kv_reads = int(sum(len(q) * len(p[0]) + len(q) * (len(q) + 1) // 2
                               for q, p in zip(seqs, preps)))
            for sp, seq in zip(spans, seqs):
                if logger is None:  # no redraw report to log: commit only
                    sp.commit_all(seq)
                else:
                    for idx in seq:
                        _, chk, msg = sp.spec()
                        sp.commit_greedy(idx, chk, msg)
                if not sp.done:
                    raise RuntimeError("device grammar and host replay disagree")
                tokens += len(seq)
        while True:
            live = [i for i in range(R) if not spans[i].done]
            if not live:
                break
            feeds = []
            for i in live:
                pre = spans[i].prefix()
                feeds.append((i, pre[fed[i]:], fed[i]))
                fed[i] = len(pre)
            ts = time.perf_counter()
            lg = sess.step(feeds)
            t_dev += time.perf_counter() - ts
            if greedy:
                # one masked argmax over all live rows (same ids as the
                # per-row float64 softmax argmax: exp/normalise is monotone)
                specs = [spans[i].spec() for i in live]
                keep = np.stack([allowed_ids(vocab, **f) for f, _, _ in specs])
                ids = np.argmax(np.where(keep, lg, np.float32(-100.0)), axis=1)
                for k, i in enumerate(live):
                    spans[i].commit_greedy(ids[k], specs[k][1], specs[k][2])
            else:
                for k, i in enumerate(live):
                    spans[i].advance(lg[k])
            tokens += len(live)
            steps += 1
    out = []
    for p, st in zip(preps, spans):
        if st.n_masks == 0:
            out.append(None)
            continue
        out.append((restore_marked_input(_src_tokens(vocab, p[0]), st.total), p[1], p[2]))
    if return_stats:
        t3 = time.perf_counter()
        return out, {"tokens": tokens, "steps": steps, "prepare_s": t1 - t0,
                     "prefill_s": t2 - t1, "decode_s": t3 - t2, "step_call_s": t_dev,
                     "request_latency_s": latency, "kv_row_reads": kv_reads,
                     "generated": [list(st.total) for st in spans],
                     "decode_phases_s": dict(getattr(sess, "phase_s", {}))}
    return out
