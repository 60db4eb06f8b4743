// Device-side greedy infill grammar: the per-token host loop of
// generation.py:528-687 (grammar flags -> sampling mask -> argmax -> commit
// -> next prefix) as one kernel appended to the captured decode step, so a
// batch of requests decodes for many steps without a host round trip.
//
// Per request r the step's logits row is `logits[(2r+1) * ldl]` (the last
// fed token of the request's two step slots, decode.py).  The kernel
//   1. derives the grammar state code from the request's flags
//      (_Span.spec, generation.py:549-630) -> keep[state][V] mask table,
//   2. takes argmax over where(keep, logit, -100) (first index on ties, as
//      np.argmax over the reference's float64 softmax of the same masked
//      row: exp / normalise is monotone),
//   3. commits the id (_Span.commit, generation.py:632-687): flag updates,
//      control -> [id, eos], span end on eos / 100 tokens, next mask index,
//   4. writes the next step's feed (ids + meta rows 2r, 2r+1) and appends
//      the id to out_tok[r].
// One wave per request (latency-bound: a few dependent loads per request,
// all requests in parallel).  The number of requests still live after the
// step is counted into *alive, which the kernel's caller zeroes first
// (smer_grammar_greedy_step issues the memset on the same stream).
#include "common.h"

namespace {
constexpr int ST_POS = 0, ST_FLAGS = 1, ST_LEN = 2, ST_MIDX = 3, ST_NMASK = 4, ST_DONE = 5,
              ST_NOWHOLE = 6, ST_COUNT = 7, ST_ERR = 8;
constexpr int F_SEP = 1, F_CONT = 2, F_PITCH = 4, F_REST = 8;
// token class bits (host builds cls[V] from the vocab)
constexpr int C_CONT = 1, C_PITCH = 2, C_DUR = 4, C_SEPSTR = 8, C_RESTSTR = 16, C_CTRL = 32;
}  // namespace

__device__ __forceinline__ int grammar_state(int flags, int len, int target, int no_whole) {
  if (flags & F_SEP) return 0;
  if (flags & F_CONT) return 1;
  if (flags & F_PITCH) return 2 + no_whole;
  if (flags & F_REST) return 4 + no_whole;
  if (len == 1) return target == 0 ? 10 : 5 + target;  // 'r' -> 10; d,o,p,t -> 6..9
  return 11 + no_whole;
}

// RING: no memset / host copy per step.  ctl = {live count, tickets, step}
// (device, zeroed once by the caller); every request's block takes a ticket
// after adding itself to the live count, and the step's last block publishes
// the count to ring[step % ring_n] (host-visible pinned memory) and resets
// ctl for the next step.  The host reads the slot after the step's event.
__device__ __forceinline__ void grammar_ring_ticket(int32_t* ctl, int32_t* ring, int ring_n, int R) {
  const int t = __hip_atomic_fetch_add(&ctl[1], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (t == R - 1) {
    const int a = __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const int s = __hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ring[s % ring_n], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&ctl[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctl[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctl[2], s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <bool RING>
__global__ __launch_bounds__(64) void grammar_greedy_kernel(
    int R, int V, const float* __restrict__ logits, long ldl, int32_t* __restrict__ state,
    int nst, const int8_t* __restrict__ targets, int max_masks, const uint8_t* __restrict__ keep,
    const uint8_t* __restrict__ cls, int eos, int m0, int trash_pos, int max_span,
    const int32_t* __restrict__ src_len, int64_t* __restrict__ ids, int32_t* __restrict__ meta,
    int M, int32_t* __restrict__ out_tok, int cap, int32_t* __restrict__ alive,
    int32_t* __restrict__ ring, int ring_n) {
  // one wave per request; the whole state vector is read in one load
  // (lane k <- st[k]) alongside the logits row, then broadcast
  const int r = blockIdx.x, lane = threadIdx.x;
  int32_t* st = state + (long)r * nst;
  const int sv = lane < nst ? st[lane] : 0;
  const float* lr = logits + (long)(2 * r + 1) * ldl;
  float lg[5];
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int i = lane + 64 * u;
    lg[u] = i < V ? lr[i] : -INFINITY;
  }
  const int done0 = __shfl(sv, ST_DONE, 64);
  if (done0) {  // wave-uniform
    if (RING && lane == 0) grammar_ring_ticket(alive, ring, ring_n, R);
    return;
  }
  const int flags = __shfl(sv, ST_FLAGS, 64), len = __shfl(sv, ST_LEN, 64),
            midx = __shfl(sv, ST_MIDX, 64), nmask = __shfl(sv, ST_NMASK, 64),
            nowhole = __shfl(sv, ST_NOWHOLE, 64), cnt = __shfl(sv, ST_COUNT, 64),
            pos = __shfl(sv, ST_POS, 64);
  const int code = grammar_state(flags, len, targets[(long)r * max_masks + midx], nowhole);
  const uint8_t* kp = keep + (long)code * V;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int u = 0; u < (V + 63) / 64 && u < 5; ++u) {
    const int i = lane + 64 * u;
    if (i < V) {
      const float x = kp[i] ? lg[u] : -100.f;
      if (x > best || bi == 0x7fffffff) { best = x; bi = i; }  // ascending i: first max kept
    }
  }
  for (int i = lane + 320; i < V; i += 64) {  // V > 320 (not the SMER vocab)
    const float x = kp[i] ? lr[i] : -100.f;
    if (x > best || bi == 0x7fffffff) { best = x; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane != 0) return;
  const int idx = bi;
  const int c = cls[idx];
  int f = flags;
  if (c & C_CONT) f = (f | F_CONT) & ~F_SEP;
  if (c & C_PITCH) f = (f | F_PITCH) & ~(F_SEP | F_CONT);
  if (c & C_DUR) f &= ~(F_REST | F_PITCH);
  if (c & C_SEPSTR) f |= F_SEP;
  if (c & C_RESTSTR) f |= F_REST;
  if (cnt < cap) out_tok[(long)r * cap + cnt] = idx;
  st[ST_COUNT] = cnt + 1;
  int feed[2], nf;
  bool end;
  if (c & C_CTRL) {  // this_in += [idx, eos]: the span ends
    end = true; feed[0] = idx; feed[1] = m0; nf = 2;
  } else if (idx == eos || len + 1 >= max_span) {  // last token dropped, m_0 takes its place
    end = true; feed[0] = m0; nf = 1;
  } else {
    end = false; feed[0] = idx; nf = 1;
  }
  bool done = false;
  int nlen = len + 1, nmidx = midx;
  if (end) {
    nmidx = midx + 1;
    if (nmidx >= nmask) {
      done = true;
      nf = 0;  // nothing more to feed
    } else {
      f = 0;
      nlen = 1;
    }
  }
  st[ST_MIDX] = nmidx;
  st[ST_LEN] = nlen;
  st[ST_FLAGS] = f;
  if (!done && pos + nf > trash_pos) {  // decoder prefix would overrun the cache
    st[ST_ERR] = 1;
    done = true;
  }
  // next step's rows 2r (first) and 2r+1 (last): dummies unless fed
  const int skv = max(src_len[r], 1);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = 2 * r + k;
    const int j = k - (2 - nf);  // index into feed for this row (row 2r+1 carries the last)
    const bool real = !done && j >= 0;
    ids[row] = real ? feed[j] : 0;
    meta[row] = real ? pos + j : trash_pos;
    meta[M + row] = r;
    meta[2 * M + row] = real ? pos + j + 1 : 1;
    meta[3 * M + row] = real ? skv : 1;
  }
  if (done) {
    st[ST_DONE] = 1;
  } else {
    st[ST_POS] = pos + nf;
    if (RING) __hip_atomic_fetch_add(&alive[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else atomicAdd(alive, 1);  // integer count: order-independent
  }
  if (RING) grammar_ring_ticket(alive, ring, ring_n, R);
}

extern "C" int smer_grammar_greedy_step(int R, int V, const float* logits, long ldl,
                                        int32_t* state, int nst, const int8_t* targets,
                                        int max_masks, const uint8_t* keep, const uint8_t* cls,
                                        int eos, int m0, int trash_pos, int max_span,
                                        const int32_t* src_len, int64_t* ids, int32_t* meta,
                                        int32_t* out_tok, int cap, int32_t* alive,
                                        smer_stream_t stream) {
  SMER_REQUIRE(R > 0 && V > 0 && nst >= 9 && max_masks > 0 && cap > 0, "smer_grammar_greedy_step: sizes");
  SMER_REQUIRE(ldl >= V, "smer_grammar_greedy_step: logits row stride");
  SMER_REQUIRE(logits && state && targets && keep && cls && src_len && ids && meta && out_tok && alive,
               "smer_grammar_greedy_step: null pointer");
  SMER_REQUIRE(eos >= 0 && eos < V && m0 >= 0 && m0 < V && trash_pos > 0 && max_span > 1,
               "smer_grammar_greedy_step: token ids");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(alive, 0, sizeof(int32_t), s) != hipSuccess)
    return smer_set_error(SMER_ERR_HIP, "smer_grammar_greedy_step: memset");
  hipLaunchKernelGGL(grammar_greedy_kernel<false>, dim3(R), dim3(64), 0, s, R, V,
                     logits, ldl, state, nst, targets, max_masks, keep, cls, eos, m0, trash_pos,
                     max_span, src_len, ids, meta, 2 * R, out_tok, cap, alive, nullptr, 0);
  SMER_CHECK_LAUNCH("smer_grammar_greedy_step");
  return SMER_OK;
}

extern "C" int smer_grammar_greedy_step_ring(int R, int V, const float* logits, long ldl,
                                             int32_t* state, int nst, const int8_t* targets,
                                             int max_masks, const uint8_t* keep, const uint8_t* cls,
                                             int eos, int m0, int trash_pos, int max_span,
                                             const int32_t* src_len, int64_t* ids, int32_t* meta,
                                             int32_t* out_tok, int cap, int32_t* ctl,
                                             int32_t* ring, int ring_n, smer_stream_t stream) {
  SMER_REQUIRE(R > 0 && V > 0 && nst >= 9 && max_masks > 0 && cap > 0 && ring_n > 0,
               "smer_grammar_greedy_step_ring: sizes");
  SMER_REQUIRE(ldl >= V, "smer_grammar_greedy_step_ring: logits row stride");
  SMER_REQUIRE(logits && state && targets && keep && cls && src_len && ids && meta && out_tok && ctl && ring,
               "smer_grammar_greedy_step_ring: null pointer");
  SMER_REQUIRE(eos >= 0 && eos < V && m0 >= 0 && m0 < V && trash_pos > 0 && max_span > 1,
               "smer_grammar_greedy_step_ring: token ids");
  // the ring is pinned host memory: its device-side address
  void* dring = nullptr;
  if (hipHostGetDevicePointer(&dring, ring, 0) != hipSuccess || dring == nullptr) {
    (void)hipGetLastError();
    dring = ring;
  }
  hipLaunchKernelGGL(grammar_greedy_kernel<true>, dim3(R), dim3(64), 0, (hipStream_t)stream, R, V,
                     logits, ldl, state, nst, targets, max_masks, keep, cls, eos, m0, trash_pos,
                     max_span, src_len, ids, meta, 2 * R, out_tok, cap, ctl, (int32_t*)dring, ring_n);
  SMER_CHECK_LAUNCH("smer_grammar_greedy_step_ring");
  return SMER_OK;
}
