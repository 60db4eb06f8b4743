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

// Commit id `idx` of request r (_Span.commit, generation.py:632-687): flag
// updates, control -> [id, eos], span end on eos / max_span tokens, next
// mask index; writes the next step's feed (rows 2r, 2r+1) and appends the
// id to out_tok[r] (bit 16: the redraw loop gave up on this draw).
// Returns whether the request is still live.  Lane 0 only.
__device__ bool grammar_commit(int r, int idx, bool fail, int flags, int len, int midx, int nmask, int cnt,
                               int pos, int32_t* st, const uint8_t* cls, int eos, int m0, int trash_pos,
                               int max_span, const int32_t* src_len, int64_t* ids, int32_t* meta, int M,
                               int32_t* out_tok, int cap) {
  const int c = cls[idx];
  int f = flags;
  if (c & C_CONT) f = (f | F_CONT) & ~F_SEP;
  if (c & C_PITCH) f = (f | F_PITCH) & ~(F_SEP | F_CONT);
  if (c & C_DUR) f &= ~(F_REST | F_PITCH);
  if (c & C_SEPSTR) f |= F_SEP;
  if (c & C_RESTSTR) f |= F_REST;
  if (cnt < cap) out_tok[(long)r * cap + cnt] = idx | (fail ? 0x10000 : 0);
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
    st[ST_ERR] |= 1;
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
  if (done) st[ST_DONE] = 1;
  else st[ST_POS] = pos + nf;
  return !done;
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
  const bool l = grammar_commit(r, bi, false, flags, len, midx, nmask, cnt, pos, st, cls, eos, m0,
                                trash_pos, max_span, src_len, ids, meta, M, out_tok, cap);
  if (l) {
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

// ---------------------------------------------------------------------------
// Device-side sampled infill grammar (the plugin's default path,
// generation.py:33-95 + 528-687): the reference's float64 softmax of the
// masked logits, `weighted_sampling`'s normalisation and descending sort,
// `np.random.choice`'s cdf / searchsorted, and the redraw loop, consuming the
// numpy legacy MT19937 stream (`random_sample`: two 32-bit outputs per
// uniform) handed over from np.random.get_state() and back by the caller.
// One block (one wave) walks the requests in order, as the host loop draws
// them.  Arithmetic order (host equivalents):
//   S = np.sum(e): numpy's pairwise summation (8 accumulators, blocks of 128,
//       tests/test_sampling.py pins the replica against numpy itself);
//   T = np.add.accumulate(p)[-1], cdf = np.cumsum(p_sorted): sequential;
//   u = (a >> 5, b >> 6) -> (a * 2^26 + b) / 2^53, idx = first cdf > u.
// exp is the device's float64 exp (within 1 ulp of numpy's; a draw could
// differ only if u fell within that distance of a cdf step), and exact ties
// between probabilities sort by descending index, the order a stable argsort
// reversed gives (numpy's introsort order for equal float32 logits is
// implementation-defined): documented in DESIGN.md.
// ---------------------------------------------------------------------------
namespace {
constexpr int SMX = 512;  // vocabulary slots of the sort (V <= 512)

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
// numpy's mt19937_gen over the LDS key, by the whole wave: each range's
// reads all happen before its writes (the sequential loop reads key[i + 1]
// before rewriting it), ranges in the order whose inputs they need
__device__ void mt_twist(uint32_t* key, int lane) {
  auto mix = [](uint32_t ki, uint32_t ki1, uint32_t km) {
    const uint32_t y = (ki & 0x80000000u) | (ki1 & 0x7fffffffu);
    return km ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  };
  const int lo[3] = {0, 227, 454}, hi[3] = {227, 454, 623};
  const int off[3] = {397, -227, -227};
  for (int ph = 0; ph < 3; ++ph) {
    uint32_t nv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = lo[ph] + lane + 64 * u;
      nv[u] = i < hi[ph] ? mix(key[i], key[i + 1], key[i + off[ph]]) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = lo[ph] + lane + 64 * u;
      if (i < hi[ph]) key[i] = nv[u];
    }
    __syncthreads();
  }
  uint32_t last = mix(key[623], key[0], key[396]);
  __syncthreads();
  if (lane == 0) key[623] = last;
  __syncthreads();
}
__device__ __forceinline__ uint32_t mt_next(uint32_t* key, int& pos, int lane) {
  if (pos >= 624) {  // wave-uniform
    mt_twist(key, lane);
    pos = 0;
  }
  return mt_temper(key[pos++]);
}
// numpy legacy random_sample
__device__ __forceinline__ double mt_uniform(uint32_t* key, int& pos, int lane) {
  const int32_t a = (int32_t)(mt_next(key, pos, lane) >> 5);
  const int32_t b = (int32_t)(mt_next(key, pos, lane) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
// numpy's pairwise_sum (loops_utils.h.src) for one contiguous block
__device__ double np_pairwise_leaf(const double* a, int n) {
  if (n < 8) {
    double r = 0.;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = a[i + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += x[j];
  }
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}
template <int DEPTH>
__device__ double np_pairwise(const double* a, int n) {
  if constexpr (DEPTH == 0) {
    return np_pairwise_leaf(a, n);
  } else {
    if (n <= 128) return np_pairwise_leaf(a, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise<DEPTH - 1>(a, n2) + np_pairwise<DEPTH - 1>(a + n2, n - n2);
  }
}
// sequential left-to-right sum of a[0..n) from 0 (np.add.accumulate's last
// element, builtin sum()); LDS loads issued 8 at a time ahead of their adds
__device__ double seq_sum(const double* a, int n) {
  double t = 0.;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = a[i + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) t += x[j];
  }
  for (; i < n; ++i) t += a[i];
  return t;
}
// c[i] = a[0] + ... + a[i], sequential (np.cumsum); returns c[n - 1].  A
// batch's 8 sums are formed before its 8 stores (a store right behind each
// add stalled on it: 25.7 vs 13.6 cycles per element for the plain sum)
__device__ double seq_cumsum(const double* a, double* c, int n) {
  double t = 0.;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    double x[8], r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = a[i + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      t += x[j];
      r[j] = t;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) c[i + j] = r[j];
  }
  for (; i < n; ++i) {
    t += a[i];
    c[i] = t;
  }
  return t;
}
// value of lane ^ X (X a power of two < 64): DPP for 1 and 2, swizzle
// (no LDS traffic) within 32-lane halves for 4-16, the half swap for 32
template <int X>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (X == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (X == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (X < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (X << 10) | 0x1F);
  else {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (__lane_id() < 32) ? r[1] : r[0];
  }
}
template <int X>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v) {
  return ((uint64_t)lane_xor<X>((uint32_t)(v >> 32)) << 32) | lane_xor<X>((uint32_t)v);
}

// bitonic sort, descending, of 64 E keys held E per lane (element s = lane
// * E + e): partners at distance >= E sit in lane ^ (dist / E), nearer ones
// in the same lane
template <int E>
__device__ __forceinline__ void sort_desc(uint64_t (&kv)[E], int lane) {
#pragma unroll
  for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      if (jj >= E) {
        const int lx = jj / E;
        const bool lower = (lane & lx) == 0;
#pragma unroll
        for (int j = 0; j < E; ++j) {
          const int e = lane * E + j;
          const bool desc = (e & k) == 0;
          uint64_t o;
          switch (lx) {
            case 1: o = lane_xor64<1>(kv[j]); break;
            case 2: o = lane_xor64<2>(kv[j]); break;
            case 4: o = lane_xor64<4>(kv[j]); break;
            case 8: o = lane_xor64<8>(kv[j]); break;
            case 16: o = lane_xor64<16>(kv[j]); break;
            default: o = lane_xor64<32>(kv[j]); break;
          }
          const uint64_t mx = kv[j] > o ? kv[j] : o, mn = kv[j] > o ? o : kv[j];
          kv[j] = (lower == desc) ? mx : mn;
        }
      } else {
#pragma unroll
        for (int j = 0; j < E; ++j) {
          if (j & jj) continue;
          const int e = lane * E + j;
          const bool desc = (e & k) == 0;
          const uint64_t a0 = kv[j], a1 = kv[j | jj];
          const bool sw = desc ? a1 > a0 : a0 > a1;
          kv[j] = sw ? a1 : a0;
          kv[j | jj] = sw ? a0 : a1;
        }
      }
    }
  }
}

// fast path of the sampler: sort the first 64 E compacted keys (E per lane)
// and gather the p of sort positions < NA into sp
template <int E>
__device__ __forceinline__ void fast_sort_gather(const uint64_t* kA, int lane, int NA, int (&sidx)[8], double* sp,
                                                 const double* pe) {
  uint64_t k[E];
#pragma unroll
  for (int e = 0; e < E; ++e) k[e] = kA[lane * E + e];
  sort_desc<E>(k, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int s = lane * E + e;
    sidx[e] = (int)(uint32_t)k[e];
    if (s < NA) sp[s] = pe[sidx[e]];
  }
}

// np.sum's pairwise order over a[0..n) with the leaves' eight accumulator
// chains summed by separate lanes: lane 8L + j runs chain j of leaf L (the
// leaves are the blocks of <= 128 the recursion stops at, in order), lane 0
// then adds each leaf's tree and remainder and the leaves in the recursion's
// order -- the same additions in the same order as numpy's one thread
// leaf blocks of numpy's pairwise recursion over [a0, a0 + n) into lv
// (start, length pairs; lv[16] = count)
template <int DEPTH>
__device__ void pw_split(int* lv, int a0, int n) {
  if (DEPTH == 0 || n <= 128) {
    const int q = lv[16];
    lv[2 * q] = a0;
    lv[2 * q + 1] = n;
    lv[16] = q + 1;
    return;
  }
  if constexpr (DEPTH > 0) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    pw_split<DEPTH - 1>(lv, a0, n2);
    pw_split<DEPTH - 1>(lv, a0 + n2, n - n2);
  }
}
template <int DEPTH>
__device__ double pw_combine(const double* leafsum, int& li, int n) {
  if (DEPTH == 0 || n <= 128) return leafsum[li++];
  if constexpr (DEPTH > 0) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    const double x = pw_combine<DEPTH - 1>(leafsum, li, n2);
    return x + pw_combine<DEPTH - 1>(leafsum, li, n - n2);
  }
  return 0.;
}
// all 64 lanes call; scratch: 72 doubles of LDS, lv: 17 ints of LDS
__device__ double np_pairwise_par(const double* a, int n, double* scratch, int* lv, int lane) {
  if (lane == 0) {
    lv[16] = 0;
    pw_split<3>(lv, 0, n);
  }
  __syncthreads();
  const int nl = lv[16];
  const int leaf = lane >> 3, j = lane & 7;
  double r = 0.;
  if (leaf < nl && lv[2 * leaf + 1] >= 8) {
    const double* b = a + lv[2 * leaf];
    const int len = lv[2 * leaf + 1];
    const int m = len - len % 8;
    r = b[j];
    for (int i = 8; i < m; i += 8) r += b[i + j];
  }
  scratch[lane] = r;
  __syncthreads();
  double res = 0.;
  if (lane == 0) {
    for (int q = 0; q < nl; ++q) {
      const double* b = a + lv[2 * q];
      const int len = lv[2 * q + 1];
      double t;
      int i;
      if (len < 8) {
        t = 0.;
        i = 0;
      } else {
        const double* rr = scratch + 8 * q;
        t = ((rr[0] + rr[1]) + (rr[2] + rr[3])) + ((rr[4] + rr[5]) + (rr[6] + rr[7]));
        i = len - len % 8;
      }
      for (; i < len; ++i) t += b[i];
      scratch[64 + q] = t;
    }
    int li = 0;
    res = pw_combine<3>(scratch + 64, li, n);
  }
  __syncthreads();
  return res;
}

// sort position: larger probability first; equal probabilities by
// descending index
__device__ __forceinline__ bool before(double pa, int ia, double pb, int ib) {
  return pa > pb || (pa == pb && ia > ib);
}
}  // namespace

// order-preserving uint32 image of a float (larger float, larger image)
__device__ __forceinline__ uint32_t f32_ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

#ifndef SMER_SAMPLE_STAMPS
#define SMER_SAMPLE_STAMPS 0  // tools/build_variant.sh ... -DSMER_SAMPLE_STAMPS=1: phase clocks in mt[640..]
#endif
#define SSTAMP(k) do { if (SMER_SAMPLE_STAMPS && lane == 0) mt[640 + (k)] = (uint32_t)__builtin_amdgcn_s_memtime(); } while (0)

template <bool RING>
__global__ __launch_bounds__(64) void grammar_sample_kernel(
    int R, int V, const float* __restrict__ logits, long ldl, int32_t* __restrict__ state, int nst,
    const int8_t* __restrict__ targets, int max_masks, const uint8_t* __restrict__ keep,
    const uint8_t* __restrict__ reject, const uint8_t* __restrict__ cls, int eos, int m0, int trash_pos,
    int max_span, const int32_t* __restrict__ src_len, int64_t* __restrict__ ids,
    int32_t* __restrict__ meta, int M, int32_t* __restrict__ out_tok, int cap,
    int32_t* __restrict__ alive, int32_t* __restrict__ ring, int ring_n, uint32_t* __restrict__ mt) {
  // one wave; element i of a row lives in lane i / 8, slot i % 8
  __shared__ uint32_t key[624];
  __shared__ double pe[SMX];   // e, then p by vocabulary index
  __shared__ double sp[SMX];   // p in sort order, then the normalised cdf
  __shared__ uint64_t kA[SMX];  // fast path: the compacted keys of set A
  __shared__ double bc[2];
  __shared__ int pwl[17];
  __shared__ __attribute__((aligned(16))) uint8_t tk[13 * SMX], tr[13 * SMX];  // keep / reject tables
  __shared__ uint8_t tcls[SMX];
  const int lane = threadIdx.x;
  SSTAMP(0);
  // every input load of the step in one batch (one memory latency, not a
  // chain of them): the MT key, the grammar tables, the first request
  {
    uint32_t kw[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) kw[u] = lane + 64 * u < 624 ? mt[lane + 64 * u] : 0u;
    // the tables as 4-B words where whole (any 4-B alignment of the bases
    // is the caller's: torch allocations are), the tail bytes one by one
    const int nt = 13 * V, nw = ((((uintptr_t)keep | (uintptr_t)reject) & 3) == 0) ? nt / 4 : 0;
    constexpr int WPL = 13 * SMX / 4 / 64;  // words per lane
    uint32_t bk[WPL], br[WPL];
#pragma unroll
    for (int u = 0; u < WPL; ++u) {
      const int w = lane + 64 * u;
      bk[u] = w < nw ? reinterpret_cast<const uint32_t*>(keep)[w] : 0u;
      br[u] = w < nw ? reinterpret_cast<const uint32_t*>(reject)[w] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 10; ++u)
      if (lane + 64 * u < 624) key[lane + 64 * u] = kw[u];
#pragma unroll
    for (int u = 0; u < WPL; ++u) {
      reinterpret_cast<uint32_t*>(tk)[lane + 64 * u] = bk[u];
      reinterpret_cast<uint32_t*>(tr)[lane + 64 * u] = br[u];
    }
    for (int i = 4 * nw + lane; i < nt; i += 64) {
      tk[i] = keep[i];
      tr[i] = reject[i];
    }
    for (int i = lane; i < V; i += 64) tcls[i] = cls[i];
  }
  // a request's state row, mask targets and logits (indices clamped, not
  // guarded: a guarded load waits right behind itself); request 0's with the
  // batch above, request r + 1's under request r's work
  auto fetch = [&](int r, int& sv, int& tgv, float (&lg)[8]) {
    const int rr = min(r, R - 1);
    sv = state[(long)rr * nst + min(lane, nst - 1)];
    tgv = (int)targets[(long)rr * max_masks + min(lane, max_masks - 1)];
    const float* lr = logits + (long)(2 * rr + 1) * ldl;
#pragma unroll
    for (int j = 0; j < 8; ++j) lg[j] = lr[min(lane * 8 + j, V - 1)];
  };
  int sv_n, tgv_n;
  float lg_n[8];
  fetch(0, sv_n, tgv_n, lg_n);
  int pos = (int)mt[624];
  __syncthreads();
  SSTAMP(1);
  int live = 0;
  for (int r = 0; r < R; ++r) {
    int32_t* st = state + (long)r * nst;
    const int sv = sv_n, tgv = tgv_n;
    float lg8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) lg8[j] = lg_n[j];
    fetch(r + 1, sv_n, tgv_n, lg_n);
    if (__shfl(sv, ST_DONE, 64)) continue;  // wave-uniform
    const int flags = __shfl(sv, ST_FLAGS, 64), len = __shfl(sv, ST_LEN, 64),
              midx = __shfl(sv, ST_MIDX, 64), nmask = __shfl(sv, ST_NMASK, 64),
              nowhole = __shfl(sv, ST_NOWHOLE, 64), cnt = __shfl(sv, ST_COUNT, 64),
              pos_t = __shfl(sv, ST_POS, 64);
    const int tgt = midx < 64 ? __shfl(tgv, midx, 64) : (int)targets[(long)r * max_masks + midx];
    const int code = grammar_state(flags, len, tgt, nowhole);
    const uint8_t* kp = tk + code * V;
    const uint8_t* rj = tr + code * V;
    // e = exp(where(keep, float64(logit), -100.0)); sort keys: the masked
    // float32 logit's order image (the probabilities' order: exp and the two
    // normalisations are monotone and keep distinct float32 inputs distinct)
    // above the index (ties: larger index first)
    uint64_t kv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane * 8 + j;
      const float x = (i < V && kp[i]) ? lg8[j] : -100.f;
      kv[j] = i < V ? ((uint64_t)f32_ord(x) << 32) | (uint32_t)i : 0ull;
      pe[i] = i < V ? exp((double)x) : 0.;
    }
    __syncthreads();
    SSTAMP(2);
    {
      const double t = np_pairwise_par(pe, V, sp, pwl, lane);
      if (lane == 0) bc[0] = t;
    }
    __syncthreads();
    const double S = bc[0];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane * 8 + j;
      if (i < V) pe[i] = pe[i] / S;
    }
    __syncthreads();
    SSTAMP(3);
    if (lane == 0) bc[1] = seq_sum(pe, V);
    __syncthreads();
    SSTAMP(4);
    const double T = bc[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane * 8 + j;
      if (i < V) pe[i] = pe[i] / T;
    }
    // The sort order, the sorted p and the cdf.  Fast path: the elements
    // with x > -100 (set A: kept logits) sorted alone on a 64 / 128 / 256-key
    // network; the rest all equal -100 (masked, or kept at exactly -100: set
    // B, one shared p) and follow in descending index order, and when some
    // kept logit is >= -60 their p is below 2^-54 of A's sum, so adding them
    // leaves every cdf value past A at t_A: the cdf of A ends at t_A / t_A =
    // 1.0 exactly, every draw u < 1 lands in A, and B is never needed.  Any
    // kept logit below -100, none >= -60, no A, or a pB check that fails
    // takes the full 512-key path (numpy's arithmetic either way).
    double cd[8];
    int sidx[8];
    double total;
    bool fast;
    {
      uint32_t am = 0u;
      bool c_any = false, hi = false;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = lane * 8 + j;
        const float x = (i < V && kp[i]) ? lg8[j] : -100.f;
        if (i < V && x > -100.f) am |= 1u << j;
        if (i < V && x < -100.f) c_any = true;
        if (i < V && x >= -60.f) hi = true;
      }
      fast = !__any(c_any) && __any(hi) && __any(am != 0u);
      if (fast) {
        // compact A's keys into LDS (prefix over lanes), pad to the network size
        int incl = __popc(am);
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int t = __shfl_up(incl, d, 64);
          if (lane >= d) incl += t;
        }
        const int NA = __shfl(incl, 63, 64);
        int pos = incl - __popc(am);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (am & (1u << j)) kA[pos++] = kv[j];
        const int E = NA <= 64 ? 1 : NA <= 128 ? 2 : NA <= 256 ? 4 : 8;
        for (int q = NA + lane; q < 64 * E; q += 64) kA[q] = 0ull;  // below every key
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j) { cd[j] = -1.0; sidx[j] = 0; }
        if (E == 1) fast_sort_gather<1>(kA, lane, NA, sidx, sp, pe);
        else if (E == 2) fast_sort_gather<2>(kA, lane, NA, sidx, sp, pe);
        else if (E == 4) fast_sort_gather<4>(kA, lane, NA, sidx, sp, pe);
        else fast_sort_gather<8>(kA, lane, NA, sidx, sp, pe);
        // p of a B element (all equal), if any: the first one
        uint32_t bmask = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (lane * 8 + j < V && !(am & (1u << j))) bmask |= 1u << j;
        const uint64_t bm = __ballot(bmask != 0u);
        double pB = 0.;
        if (bm) {
          const int bl = __builtin_ctzll(bm);
          const int bj = __builtin_ctz((uint32_t)__shfl((int)bmask, bl, 64));
          pB = pe[bl * 8 + bj];
        }
        __syncthreads();
        if (lane == 0) bc[0] = seq_cumsum(sp, sp, NA);
        __syncthreads();
        SSTAMP(7);
        total = bc[0];
        if (pB * 18014398509481984.0 > total) {  // 2^54: the B terms would not vanish
          fast = false;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int s = lane * E + e;
            if (e < E && s < NA) cd[e] = sp[s] / total;
          }
        }
      }
    }
    if (!fast) {
      // the full path: bitonic sort of all 512 keys in registers
      sort_desc<8>(kv, lane);
      __syncthreads();
      SSTAMP(5);
      // p in sort order (slot s = lane * 8 + j holds sort position s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int s = lane * 8 + j;
        sidx[j] = (int)(uint32_t)kv[j];
        sp[s] = s < V ? pe[sidx[j]] : 0.;
      }
      __syncthreads();
      SSTAMP(6);
      if (lane == 0) bc[0] = seq_cumsum(sp, sp, V);
      __syncthreads();
      SSTAMP(7);
      total = bc[0];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int s = lane * 8 + j;
        cd[j] = s < V ? sp[s] / total : 2.0;
      }
    }
    const bool bad = !(fabs(total - 1.0) <= 1e-9);  // the host path hands such rows to np.random.choice
    // draws (the reference's redraw loop: up to 11 redraws, the last kept):
    // the first sort position whose cdf exceeds u
    auto draw = [&]() -> int {
      const double u = mt_uniform(key, pos, lane);
      int first = 8;
#pragma unroll
      for (int j = 7; j >= 0; --j)
        if (cd[j] > u) first = j;
      const uint64_t m = __ballot(first < 8);
      const int ln = m ? __builtin_ctzll(m) : 63;
      const int fj = __shfl(first, ln, 64);
      int idx = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j == (fj < 8 ? fj : 7)) idx = sidx[j];
      return __shfl(idx, ln, 64);
    };
    int idx = draw();
    SSTAMP(8);
    int n = 0;
    bool fail = false;
    while (rj[idx]) {
      idx = draw();
      if (++n > 10) { fail = true; break; }
    }
    if (lane == 0) {
      const bool l = grammar_commit(r, idx, fail, flags, len, midx, nmask, cnt, pos_t, st, tcls, eos, m0,
                                    trash_pos, max_span, src_len, ids, meta, M, out_tok, cap);
      if (bad) st[ST_ERR] |= 2;
      live += l ? 1 : 0;
    }
    __syncthreads();
  }
  SSTAMP(9);
  for (int i = lane; i < 624; i += 64) mt[i] = key[i];
  if (lane == 0) {
    mt[624] = (uint32_t)pos;
    if (RING) {
      const int s = alive[2];
      __hip_atomic_store(&ring[s % ring_n], live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      alive[2] = s + 1;
    } else {
      alive[0] = live;
    }
  }
}

extern "C" int smer_grammar_sample_step(int R, int V, const float* logits, long ldl, int32_t* state,
                                        int nst, const int8_t* targets, int max_masks, const uint8_t* keep,
                                        const uint8_t* reject, const uint8_t* cls, int eos, int m0,
                                        int trash_pos, int max_span, const int32_t* src_len, int64_t* ids,
                                        int32_t* meta, int32_t* out_tok, int cap, uint32_t* mt,
                                        int32_t* ctl, int32_t* ring, int ring_n, smer_stream_t stream) {
  SMER_REQUIRE(R > 0 && V > 0 && V <= SMX && nst >= 9 && max_masks > 0 && cap > 0,
               "smer_grammar_sample_step: sizes (V <= 512)");
  SMER_REQUIRE(ldl >= V, "smer_grammar_sample_step: logits row stride");
  SMER_REQUIRE(logits && state && targets && keep && reject && cls && src_len && ids && meta && out_tok && mt && ctl,
               "smer_grammar_sample_step: null pointer");
  SMER_REQUIRE(eos >= 0 && eos < V && m0 >= 0 && m0 < V && trash_pos > 0 && max_span > 1,
               "smer_grammar_sample_step: token ids");
  hipStream_t s = (hipStream_t)stream;
  if (ring) {
    void* dring = nullptr;
    if (hipHostGetDevicePointer(&dring, ring, 0) != hipSuccess || dring == nullptr) {
      (void)hipGetLastError();
      dring = ring;
    }
    hipLaunchKernelGGL(grammar_sample_kernel<true>, dim3(1), dim3(64), 0, s, R, V, logits, ldl, state, nst,
                       targets, max_masks, keep, reject, cls, eos, m0, trash_pos, max_span, src_len, ids, meta,
                       2 * R, out_tok, cap, ctl, (int32_t*)dring, ring_n, mt);
  } else {
    hipLaunchKernelGGL(grammar_sample_kernel<false>, dim3(1), dim3(64), 0, s, R, V, logits, ldl, state, nst,
                       targets, max_masks, keep, reject, cls, eos, m0, trash_pos, max_span, src_len, ids, meta,
                       2 * R, out_tok, cap, ctl, nullptr, 0, mt);
  }
  SMER_CHECK_LAUNCH("smer_grammar_sample_step");
  return SMER_OK;
}
