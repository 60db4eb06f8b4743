// Host-side inner loop of the SMER pretraining span masking:
// reference dataset.py:166-311 (`ParallelLanguageDataset.random_word`), on
// token ids, drawing from a replica of CPython's `random` generator so the
// stream (and every masking decision) is the reference's.  See
// include/smer_data.h.  Built with g++ into libsmer_data.so (no GPU code).
#include "smer_data.h"

#include <cstddef>
#include <cstdint>
#include <vector>

namespace {

// MT19937 (Matsumoto & Nishimura 1998), state layout as CPython keeps it:
// 624 words + the next-word index; random() = 53-bit double from two words
// (a >> 5, b >> 6), as CPython's random_random.
struct Mt {
  uint32_t s[624];
  uint32_t i;

  void twist() {
    constexpr uint32_t A = 0x9908b0dfu, HI = 0x80000000u, LO = 0x7fffffffu;
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (s[k] & HI) | (s[(k + 1) % 624] & LO);
      s[k] = s[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? A : 0u);
    }
    i = 0;
  }
  uint32_t next() {
    if (i >= 624) twist();
    uint32_t y = s[i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  double random() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
};

inline void load(Mt& g, const uint32_t* mt) {
  for (int k = 0; k < 624; ++k) g.s[k] = mt[k];
  g.i = mt[624];
}
inline void store(const Mt& g, uint32_t* mt) {
  for (int k = 0; k < 624; ++k) mt[k] = g.s[k];
  mt[624] = g.i;
}

}  // namespace

extern "C" void smer_mt_random(uint32_t* mt, int n, double* out) {
  Mt g;
  load(g, mt);
  for (int k = 0; k < n; ++k) out[k] = g.random();
  store(g, mt);
}

extern "C" int smer_span_mask(uint32_t* mt, int n_events, const int32_t* ids, const int64_t* off,
                              const uint8_t* tok_class, int vocab_size, int control_mode,
                              int32_t corrupt_id, int32_t mask_id, int32_t eos_id, double total_ratio,
                              double thr15, int32_t* tokens, int32_t* dec_in, int32_t* dec_tgt,
                              int64_t* lens) {
  if (n_events < 0 || !mt || (n_events > 0 && (!ids || !off || !tok_class || !lens))) return -1;
  for (int e = 0; e < n_events; ++e)
    for (int64_t p = off[e]; p < off[e + 1]; ++p)
      if (ids[p] < 0 || ids[p] >= vocab_size) return -1;
  Mt g;
  load(g, mt);
  std::vector<int32_t> w;  // the event copy with its corrupted controls
  int64_t nt = 0, ni = 0, no = 0;
  const int span_len[3] = {3, 1, 2};
  for (int e = 0; e < n_events; ++e) {
    const int32_t* src = ids + off[e];
    const int64_t n = off[e + 1] - off[e];
    w.assign(src, src + n);
    // corruption: one draw per control position, in order (dataset.py:
    // 205-231); mode 1 counts a run of controls from a control whose
    // predecessor is a track / bar token until the next non-control
    bool run = false;
    for (int64_t p = 0; p < n; ++p) {
      const bool ctl = tok_class[src[p]] & SMER_TOK_CONTROL;
      bool corruptible = ctl;
      if (control_mode != 0) {
        if (!ctl) run = false;
        else if (p > 0 && (tok_class[src[p - 1]] & SMER_TOK_TRACK_OR_BAR)) run = true;
        corruptible = ctl && run;
      }
      if (corruptible && g.random() < .05) w[p] = corrupt_id;
    }
    // span loop (dataset.py:241-288): a span of 3 / 1 / 2 tokens by the
    // first draw (< .5 / in (.5, .75) / otherwise), kept by a second draw
    // (< thr15) when it fits; else the token passes through unmasked
    int64_t sp = 0, kt = 0, ki = 0, ko = 0;
    double ratio = 0.0;
    while (ratio < total_ratio && sp < n) {
      const double p = g.random();
      const int len = p < 0.5 ? span_len[0] : (0.5 < p && p < 0.75) ? span_len[1] : span_len[2];
      int L = 0;
      if (sp + len <= n && g.random() < thr15) L = len;
      if (L) {
        tokens[nt + kt++] = mask_id;
        ratio += (double)L / (double)n;
        dec_in[ni + ki++] = mask_id;
        for (int k = 0; k < L; ++k) {
          dec_in[ni + ki++] = w[sp + k];
          dec_tgt[no + ko++] = w[sp + k];
        }
        dec_tgt[no + ko++] = eos_id;
        sp += L;
      } else {
        tokens[nt + kt++] = w[sp++];
      }
    }
    while (sp < n) tokens[nt + kt++] = w[sp++];
    lens[3 * e] = kt;
    lens[3 * e + 1] = ki;
    lens[3 * e + 2] = ko;
    nt += kt;
    ni += ki;
    no += ko;
  }
  store(g, mt);
  return 0;
}
