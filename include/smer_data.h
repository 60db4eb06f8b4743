/* smer_data.h — host-side C ABI of the SMER training-data pipeline (SURVEY
 * §8 row f3).  Host code only (libsmer_data.so, built with g++): the
 * per-token inner loop of the reference's pretraining span masking,
 * `ParallelLanguageDataset.random_word` (reference dataset.py:166-311), with
 * the exact random stream of CPython's `random` module (MT19937).
 *
 * The caller passes the generator state as CPython's random.getstate()[1]
 * holds it (624 state words + the index) and gets it back advanced by exactly
 * the draws the reference loop would have made, so Python-side draws before
 * (index choice, shuffle) and after continue the same stream.
 */
#ifndef SMER_DATA_H
#define SMER_DATA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Token classes, one byte per vocabulary id (tok_class[id]). */
#define SMER_TOK_CONTROL 1u      /* in vocab.control_tokens */
#define SMER_TOK_TRACK_OR_BAR 2u /* 'track_<d>...' or 'bar' */

/* Span-mask n_events events (token ids, event e = ids[off[e]:off[e+1]]).
 * Per event, reference dataset.py:179-296:
 *   1. control positions (control_mode 0: every control token, dataset.py:
 *      219-227; 1: bar_control_at_end — runs of controls that directly follow
 *      a track / bar token, dataset.py:185-217) are corrupted to corrupt_id
 *      with probability .05 each (one random() per position);
 *   2. the span loop: spans of 3 / 1 / 2 tokens chosen with probability
 *      .5 / .25 / .25 and kept with probability thr15 (= total_ratio /
 *      dot([.5,.25,.25],[3,1,2]) * 1.5, computed by the caller) until the
 *      masked fraction reaches total_ratio.
 * Outputs, concatenated in event order: tokens (<= n ids), dec_in and
 * dec_tgt (each <= 2n ids); lens[3e..3e+2] = their per-event lengths (an
 * event whose dec_in is empty is still reported, with its lengths).
 * mt: 625 uint32 (624 words + index), read and written back.
 * Returns 0, or -1 on bad arguments (an id outside [0, vocab_size)). */
int smer_span_mask(uint32_t* mt, int n_events, const int32_t* ids, const int64_t* off,
                   const uint8_t* tok_class, int vocab_size, int control_mode, int32_t corrupt_id,
                   int32_t mask_id, int32_t eos_id, double total_ratio, double thr15,
                   int32_t* tokens, int32_t* dec_in, int32_t* dec_tgt, int64_t* lens);

/* n draws of CPython's random.random() from state mt (test hook). */
void smer_mt_random(uint32_t* mt, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif
