// Attention kernels: the MHA math path of the reference
// (torch/nn/functional.py:6578-6600 via transformer.py:389,459,463).
//
// bf16 flash forward / backward (gfx950 MFMA 16x16x32):
//  * "key on the row" orientation: S^T = K Q^T, so each lane holds one query
//    column and its softmax row lives in 16 registers + 2 cross-group
//    shuffles; P feeds the P.V MFMA as the B operand straight from registers
//    (the k order of the 32-key step is permuted identically on both
//    operands), V is consumed through ds_read_b64_tr_b16.
//  * backward = dK/dV pass (one workgroup per 64 keys, loops over queries)
//    + dQ pass (one workgroup per 64 queries, loops over keys): no atomics,
//    deterministic.
// f32 kernels (parity mode) are plain row-per-wave VALU kernels.
#include "common.h"

#define LOG2E_F 1.4426950408889634f
#define LN2_F 0.6931471805599453f

namespace {
constexpr int KVB = 64;  // keys (or queries) per LDS tile

template <int D>
struct AttnCfg {
  // D = 64: unpadded 128-B rows with the 16-B chunk index XORed by (row & 7):
  // conflict-free for both the ds_read_b128 row fragments and the
  // ds_read_b64_tr_b16 transposed fragments (lane groups per the LDS table
  // of the gfx950 guide).  Other D: rows padded by 16 B.
  static constexpr bool SWZ = (D == 64);
  static constexpr int ROWB = SWZ ? 128 : D * 2 + 16;  // LDS row bytes
  __device__ static __forceinline__ uint32_t off(int row, int byte) {
    if constexpr (SWZ)
      return row * 128 + ((((byte >> 4) ^ (row & 7)) << 4) | (byte & 15));
    else
      return row * ROWB + byte;
  }
  static constexpr int NS = D / 32;                  // 32-deep k-steps over the head dim
  static constexpr int NDT = D / 16;                 // 16-wide head-dim tiles
  static constexpr int CPR = D / 8;                  // 16-B chunks per row
  static constexpr int CPT = (KVB * CPR) / 256;      // chunks per thread per tile
  static constexpr int TILE = KVB * ROWB;
};

template <int D>
__device__ __forceinline__ void tile_load(uint4 (&r)[AttnCfg<D>::CPT], const bf16* base, long ld,
                                          int row0, int nrows, int tid) {
#pragma unroll
  for (int c = 0; c < AttnCfg<D>::CPT; ++c) {
    int i = tid + 256 * c;
    int row = i / AttnCfg<D>::CPR, ch = i % AttnCfg<D>::CPR;
    int gr = row0 + row;
    r[c] = gr < nrows ? *reinterpret_cast<const uint4*>(base + (long)gr * ld + ch * 8)
                      : make_uint4(0, 0, 0, 0);
  }
}
template <int D>
__device__ __forceinline__ void tile_store(const uint4 (&r)[AttnCfg<D>::CPT], char* buf, int tid) {
#pragma unroll
  for (int c = 0; c < AttnCfg<D>::CPT; ++c) {
    int i = tid + 256 * c;
    int row = i / AttnCfg<D>::CPR, ch = i % AttnCfg<D>::CPR;
    *reinterpret_cast<uint4*>(buf + AttnCfg<D>::off(row, ch * 16)) = r[c];
  }
}
// Row fragment: rows rbase+c16, head-dim k-step s (8 contiguous elements).
template <int D>
__device__ __forceinline__ bf16x8 row_frag(const char* buf, int rbase, int s, int lane) {
  return lds_read_b128(buf, AttnCfg<D>::off(rbase + (lane & 15), (s * 32 + 8 * (lane >> 4)) * 2));
}
// Transposed fragment for the 32-row step ks over head-dim tile dt: element
// j of lane-group g = row ks*32 + (j<4 ? 4g+j : 16+4g+j-4), column dt*16+c16.
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const char* buf, int ks, int dt, int lane) {
  int g = lane >> 4, c16 = lane & 15, qq = c16 >> 2, pp = c16 & 3;
  int col = (dt * 16 + 4 * pp) * 2;
  bf16x4 lo = lds_read_tr16(buf, AttnCfg<D>::off(ks * 32 + 4 * g + qq, col));
  bf16x4 hi = lds_read_tr16(buf, AttnCfg<D>::off(ks * 32 + 16 + 4 * g + qq, col));
  return cat4(lo, hi);
}
__device__ __forceinline__ bf16x8 pack_p(const float (&p)[4][4], int ks) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (bf16)p[2 * ks][j];
    r[4 + j] = (bf16)p[2 * ks + 1][j];
  }
  return r;
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  bf16x2 v;
  v[0] = (bf16)a;
  v[1] = (bf16)b;
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ bf16x8 words_bf16x8(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(bf16x8, u32x4{a, b, c, d});
}
// the lane index as an opaque value (v_mbcnt): hipcc cannot fold it into a
// thread-index register it would keep live across a loop
__device__ __forceinline__ int lane_id_fresh() {
  int r;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
  return r;
}
// each 16-bit half -> 0xFFFF if its top bit is set, else 0 (v_pk_ashrrev_i16)
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t half_masks(uint32_t x) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, x) >> (short)15);
}
// 0 / ~0 from bit `bit` of w (v_bfe_i32): AND-mask for an f32 lane
__device__ __forceinline__ uint32_t bitmask32(uint32_t w, uint32_t bit) {
  return (uint32_t)__builtin_amdgcn_sbfe((int)w, bit, 1u);
}
__device__ __forceinline__ float and_f32(float x, uint32_t m) {
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & m);
}
// max over the four 16-lane groups holding one query's keys (lanes c,
// c+16, c+32, c+48): two half / row swaps (v_permlane32/16_swap) instead of
// LDS-routed shuffles; raw v_max (the operands are never NaN)
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float max_4groups(float x) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = vmax_raw(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax_raw(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
// SMER_ATTN_PRIO (compile time, A/B): raise the issuing wave's priority
// over its MFMA sections (s_setprio), so that on a SIMD shared by three
// workgroups' waves the arbiter keeps the matrix pipe fed from whichever
// wave is in its MFMA section while the others run softmax VALU
#ifndef SMER_ATTN_PRIO
#define SMER_ATTN_PRIO 0
#endif
__device__ __forceinline__ void attn_prio_hi() {
  if constexpr (SMER_ATTN_PRIO > 0) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(SMER_ATTN_PRIO);
    __builtin_amdgcn_sched_barrier(0);
  }
}
__device__ __forceinline__ void attn_prio_lo() {
  if constexpr (SMER_ATTN_PRIO > 0) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
}
}  // namespace

// Attention-dropout keep words, generated once per attention call by
// attn_drop_mask_gen_kernel (full occupancy, pure integer VALU) and read by
// the forward and both backward kernels: one u32 per (bh, query 32-block
// q32, key 64-tile t, forward lane (G, c)); bit 8R + 4gq + mt = keep of
// (query 32*q32 + 16*gq + c, key 64t + 16mt + 4G + R), i.e. byte R of the
// SWAR compare of smer_attn_bits(rowkey(query), quad 16t + 4mt + G).  The
// byte-major order lets the forward turn a word into the 16-bit AND masks of
// its packed bf16 P pairs with one v_perm per key pair (r, r+1) and a shift
// + arithmetic shift per (gq, mt) (attn_pair_mask).
__device__ __forceinline__ uint32_t attn_mask_word(uint32_t rk0, uint32_t rk1, uint32_t t, uint32_t G,
                                                   uint32_t lo4) {
  uint32_t w = 0u;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const uint32_t quad = t * (KVB / 4) + 4 * mt + G;
    w |= ((smer_attn_ge(smer_attn_bits(rk0, quad), lo4) >> 7) & 0x01010101u) << mt;
    w |= ((smer_attn_ge(smer_attn_bits(rk1, quad), lo4) >> 7) & 0x01010101u) << (4 + mt);
  }
  return w;
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// pw = perm(word) holding key r's byte in the low 16-bit half and key r+1's
// in the high half (both bytes of each half): AND masks (0xFFFF / 0) of the
// pair's two bf16 halves from bit k of each byte
__device__ __forceinline__ uint32_t attn_pair_mask(uint32_t pw, uint32_t k) {
  const u16x2 x = __builtin_bit_cast(u16x2, pw) << (unsigned short)(15u - k);
  return half_masks(__builtin_bit_cast(uint32_t, x));
}
__device__ __forceinline__ size_t attn_mask_index(int bh, int nq32, int nkt, int q32, int t) {
  return (((size_t)bh * nq32 + q32) * nkt + t) * 64;
}

// ---------------------------------------------------------------------------
// bf16 forward
// ---------------------------------------------------------------------------
// e4m3 copies e4m3(g * qs) of bf16 attention outputs, max|g| folded into
// amax (C4 fp8: the next GEMM's input); a null pointer: no copy.  Backward:
// dQ / dK / dV; forward: O in the dq slot
struct AttnQ8 {
  uint8_t* dq;
  long lddq;
  uint8_t* dk;
  long lddk;
  uint8_t* dv;
  long lddv;
  const float* qs;
  unsigned* amax;
};

// QG query groups of 16 per wave (block = 64*QG queries): K / V fragments
// read from LDS once per wave feed QG groups, halving LDS traffic per MFMA
// at QG = 2 (the forward is otherwise LDS-bandwidth co-limited).
// MIN: the keep words come precomputed (attn_drop_mask_gen_kernel, the
// product path whenever the caller keeps the mask for the backward): one
// word per lane and key tile, prefetched a tile ahead, 3 VALU per packed P
// pair.  Hashing in the loop instead (DROP && !MIN, only when the caller
// passes no mask buffer) costs 4 hashes per lane and key tile plus SWAR
// compares: it made the C2 encoder forward 42 % slower (99.6 -> 141.6 us).
// Q8: also the e4m3 copy of O (q8.dq; C4 fp8), a separate instance so that
// the plain forward's code is untouched by it
template <int D, int QG, bool DROP, bool MIN = false, bool Q8 = false>
__global__ __launch_bounds__(256, QG == 2 && D > 64 ? 2 : 3) void attn_fwd_bf16(int B, int H, int Lq, int Lk,
                                                     const bf16* __restrict__ q, long ldq,
                                                     const bf16* __restrict__ k, long ldk,
                                                     const bf16* __restrict__ v, long ldv,
                                                     bf16* __restrict__ o, long ldo,
                                                     float* __restrict__ lse,
                                                     const uint8_t* __restrict__ kpm, int causal,
                                                     float scale, uint32_t drop_thr, uint32_t seed,
                                                     float drop_scale,
                                                     uint64_t* __restrict__ drop_mask, AttnQ8 q8) {
  // drop_mask: see smer_attn_drop_mask_bytes (16-bit words, one per lane)
  using C = AttnCfg<D>;
  constexpr int QB = 64 * QG;  // queries per block
  __shared__ __attribute__((aligned(16))) char sm[2][2][C::TILE];
  // per-key additive score bias of the staged tile: 0, or -inf for padded /
  // out-of-range keys; it seeds the S accumulators, so masking costs no VALU
  __shared__ __attribute__((aligned(16))) float kbias[2][KVB];
  __shared__ int kpad[2];  // the staged tile has a padded / out-of-range key
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  int BX, BY;
  xcd_block2d(BX, BY);
  const int bh = BY, b = bh / H, h = bh % H;
  const int q0w = BX * QB + wave * 16 * QG;  // first query of this wave
  const float c = scale * LOG2E_F;
  const int nq16 = (Lq + 15) >> 4, nkt = (Lk + KVB - 1) / KVB;
  // SWAR threshold word for smer_attn_ge (drop_thr = thr7)
  const uint32_t lo4 = drop_thr * 0x01010101u;

  // Q pre-scaled by c = scale * log2(e) (once, in registers): the scores
  // leave the MFMA in log2 units, so p = 2^(s - m) needs no multiply
  bf16x8 qf[QG][C::NS];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int qi = q0w + gq * 16 + c16;
    const bf16* qrow = q + (long)(b * Lq + min(qi, Lq - 1)) * ldq + h * D;
#pragma unroll
    for (int s = 0; s < C::NS; ++s) {
      qf[gq][s] = *reinterpret_cast<const bf16x8*>(qrow + s * 32 + 8 * g);
      if (qi >= Lq) qf[gq][s] = bf16x8{};
    }
  }
  const bf16* kb = k + (long)b * Lk * ldk + h * D;
  const bf16* vb = v + (long)b * Lk * ldv + h * D;
  const uint8_t* kp = kpm ? kpm + (long)b * Lk : nullptr;

  int n_tiles = (Lk + KVB - 1) / KVB;
  if (causal) {
    int qmax = min(Lq, BX * QB + QB);
    n_tiles = min(n_tiles, (qmax + KVB - 1) / KVB);
  }
  // Online softmax against a per-query reference m_ref (log2 units, always
  // finite): acc and l hold sums of 2^(s - m_ref).  The QK^T chain starts
  // from -m_ref, so a tile whose scores all stay within 2^THR of the
  // reference is exponentiated as it leaves the MFMA; only a tile that
  // raises some query's max past that (or brings a query its first
  // unmasked key) moves the reference and rescales (deferred max).
  constexpr float THR = 8.f;
  float m_run[QG], m_ref[QG], l_run[QG];
  f32x4 negm[QG];
  uint32_t rowkey[QG];
  f32x4 acc[QG][C::NDT];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    rowkey[gq] = (DROP && !MIN) ? smer_rowkey(seed, (uint32_t)(bh * Lq + q0w + gq * 16 + c16)) : 0u;
    m_run[gq] = -INFINITY;
    m_ref[gq] = 0.f;
    negm[gq] = f32x4{0.f, 0.f, 0.f, 0.f};
    l_run[gq] = 0.f;
#pragma unroll
    for (int i = 0; i < C::NDT; ++i) acc[gq][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  uint4 rk[C::CPT], rv[C::CPT];
  auto key_bias = [&](int key) -> float {
    return (key >= Lk || (kp && kp[key])) ? -INFINITY : 0.f;
  };
  // MIN: this wave's keep words (its 16 * QG queries lie in one 32-query
  // block; gq_k = the 16-query half of a QG = 1 wave), one per key tile
  const int nq32 = (Lq + 31) >> 5;
  const uint32_t* mwp = (DROP && MIN)
      ? reinterpret_cast<const uint32_t*>(drop_mask) + attn_mask_index(bh, nq32, nkt, min(q0w >> 5, nq32 - 1), 0) + lane
      : nullptr;
  const uint32_t gq_k = QG == 2 ? 0u : (uint32_t)((q0w >> 4) & 1);
  uint32_t mw_next = 0u;
  // hashing (QG = 2) with a buffer: the keep words it publishes
  uint32_t* mwo = (DROP && !MIN && QG == 2 && drop_mask && (q0w >> 5) < nq32)
      ? reinterpret_cast<uint32_t*>(drop_mask) + attn_mask_index(bh, nq32, nkt, q0w >> 5, 0) + lane
      : nullptr;
  if (n_tiles > 0) {
    if constexpr (DROP && MIN) mw_next = mwp[0];
    // the first tile's padding byte requested with its K / V (from K's own
    // bytes without a mask, ignored through pmask): tested only after the
    // tile has landed -- testing it at once cost every workgroup a round trip
    const uint8_t* kpb = kp ? kp : reinterpret_cast<const uint8_t*>(kb);
    const uint32_t pmask = kp ? 0xFFu : 0u;
    const uint32_t pad0 = kpb[min(lane, Lk - 1)];
    tile_load<D>(rk, kb, ldk, 0, Lk, tid);
    tile_load<D>(rv, vb, ldv, 0, Lk, tid);
    tile_store<D>(rk, sm[0][0], tid);
    tile_store<D>(rv, sm[0][1], tid);
    if (tid < KVB) {  // wave 0
      const float kbz = (tid >= Lk || (pad0 & pmask)) ? -INFINITY : 0.f;
      kbias[0][tid] = kbz;
      const uint64_t any = __ballot(kbz != 0.f);
      if (tid == 0) kpad[0] = any != 0ull;
    }
  }
  __syncthreads();
  smer_vm_drain();  // prologue loads retired before the loop (common.h)
#pragma unroll
  for (int gq = 0; gq < QG; ++gq)
#pragma unroll
    for (int s = 0; s < C::NS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[gq][s][e] = (bf16)((float)qf[gq][s][e] * c);
  for (int t = 0; t < n_tiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < n_tiles;
    // the next tile's padding byte is only loaded here and compared when it
    // is staged below: comparing it at once made hipcc wait vmcnt(0) right
    // behind the K / V prefetch, every tile
    int npad = 0;
    if (more) {
      tile_load<D>(rk, kb, ldk, (t + 1) * KVB, Lk, tid);
      tile_load<D>(rv, vb, ldv, (t + 1) * KVB, Lk, tid);
      if (kp) npad = kp[min((t + 1) * KVB + (Q8 ? lane_id_fresh() : lane), Lk - 1)];  // every lane: no exec-masked join
    }
    const char* Ks = sm[cur][0];
    const char* Vs = sm[cur][1];
    uint32_t mw = mw_next;
    if constexpr (DROP && MIN) {
      if (more) mw_next = mwp[(size_t)(t + 1) * 64];
    }
    f32x4 st[QG][4];
    attn_prio_hi();
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int gq = 0; gq < QG; ++gq) st[gq][mt] = negm[gq];
#pragma unroll
      for (int s = 0; s < C::NS; ++s) {
        const bf16x8 kf = row_frag<D>(Ks, mt * 16, s, lane);
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) st[gq][mt] = mfma16(kf, qf[gq][s], st[gq][mt]);
      }
    }
    attn_prio_lo();
    if (__builtin_amdgcn_readfirstlane(kpad[cur])) {
      // -inf on padded / out-of-range keys (tiles without any skip this)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 kbv = *reinterpret_cast<const f32x4*>(&kbias[cur][mt * 16 + 4 * g]);
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) st[gq][mt] += kbv;
      }
    }
    bf16x8 pf[QG][2];
    uint32_t kword = 0u;
#pragma unroll
    for (int gq = 0; gq < QG; ++gq) {
      const int qi = q0w + gq * 16 + c16;
      if (causal && t * KVB + KVB - 1 > q0w + gq * 16) {
        // key - query = kq0 + 16mt + r: one difference, immediate offsets
        const int kq0 = t * KVB + 4 * g - qi;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kq0 > -(mt * 16 + r)) st[gq][mt][r] = -INFINITY;
      }
      // this lane's tile max, relative to m_ref
      float tmax = -INFINITY;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) tmax = fmaxf(tmax, st[gq][mt][r]);
      const bool moved = tmax > THR || (m_run[gq] == -INFINITY && tmax != -INFINITY);
      if (__ballot(moved) != 0ull) {
        // the query's tile max over its 4 lane groups; m_ref follows the
        // running max once the query has seen a key (a no-op for lanes
        // whose max did not move: d = 0)
        const float gmax = max_4groups(tmax) + m_ref[gq];
        const float m_new = fmaxf(m_run[gq], gmax);
        const float ref = m_new == -INFINITY ? m_ref[gq] : m_new;
        const float d = ref - m_ref[gq];
        // nothing accumulated yet (l = acc = 0): a first max far below the
        // initial reference would overflow 2^-d, and 0 * inf is NaN
        const float alpha = m_run[gq] == -INFINITY ? 0.f : fast_exp2(-d);
        l_run[gq] *= alpha;
#pragma unroll
        for (int i = 0; i < C::NDT; ++i) acc[gq][i] *= alpha;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) st[gq][mt] -= d;
        m_run[gq] = m_new;
        m_ref[gq] = ref;
        negm[gq] = f32x4{-ref, -ref, -ref, -ref};
      }
      float p[4][4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[mt][r] = fast_exp2(st[gq][mt][r]);
          l_run[gq] += p[mt][r];
        }
      // P as bf16 pairs: word [mt][0] = keys (r0, r1), [mt][1] = (r2, r3).
      // Dropout zeroes dropped pairs' halves with AND masks; the survivors'
      // 1 / (1 - p) is folded into the final 1 / l.
      uint32_t pw[4][2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        pw[mt][0] = pack2(p[mt][0], p[mt][1]);
        pw[mt][1] = pack2(p[mt][2], p[mt][3]);
      }
      if (DROP && MIN) {
        // bytes [r0 r0 r1 r1] / [r2 r2 r3 r3] of the word; bit 4gq + mt of
        // each byte shifted to its half's sign and smeared over the half
        const uint32_t p01 = __builtin_amdgcn_perm(mw, mw, 0x01010000u);
        const uint32_t p23 = __builtin_amdgcn_perm(mw, mw, 0x03030202u);
        const uint32_t kq = 4u * (QG == 2 ? (uint32_t)gq : gq_k);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          pw[mt][0] &= attn_pair_mask(p01, kq + mt);
          pw[mt][1] &= attn_pair_mask(p23, kq + mt);
        }
      } else if (DROP) {
        // one hash per quad of keys (16mt + 4g .. +3): byte r decides key r
        const uint32_t quad0 = (uint32_t)(t * (KVB / 4) + g);
        const uint32_t kq = 4u * (QG == 2 ? (uint32_t)gq : gq_k);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const uint32_t ge = smer_attn_ge(smer_attn_bits(rowkey[gq], quad0 + 4 * mt), lo4);
          // bytes [r0 r0 r1 r1] / [r2 r2 r3 r3], then each 16-bit half's
          // sign (the keep bit) smeared over the half
          pw[mt][0] &= half_masks(__builtin_amdgcn_perm(ge, ge, 0x01010000u));
          pw[mt][1] &= half_masks(__builtin_amdgcn_perm(ge, ge, 0x03030202u));
          if (QG == 2) kword |= ((ge >> 7) & 0x01010101u) << (kq + mt);
        }
      }
      pf[gq][0] = words_bf16x8(pw[0][0], pw[0][1], pw[1][0], pw[1][1]);
      pf[gq][1] = words_bf16x8(pw[2][0], pw[2][1], pw[3][0], pw[3][1]);
    }
    // hashing forward with a mask buffer (QG = 2: the wave's 32 queries are
    // one 32-query block): publish the tile's keep word for the backward
    if constexpr (DROP && !MIN && QG == 2) {
      if (mwo) __builtin_nontemporal_store(kword, mwo + (size_t)t * 64);
    }
    attn_prio_hi();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int dt = 0; dt < C::NDT; ++dt) {
        const bf16x8 vf = tr_frag<D>(Vs, ks, dt, lane);
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) acc[gq][dt] = mfma16(vf, pf[gq][ks], acc[gq][dt]);
      }
    }
    attn_prio_lo();
    if (more) {
      tile_store<D>(rk, sm[cur ^ 1][0], tid);
      tile_store<D>(rv, sm[cur ^ 1][1], tid);
      asm volatile("" : "+v"(npad));  // keeps the compare (and its wait) here
      if (tid < KVB) {  // wave 0
        // Q8: the lane index from v_mbcnt (wave 0: lane == tid), not a
        // register kept across the loop (the e4m3-copy instance spilled it)
        const int kl = Q8 ? lane_id_fresh() : tid;
        const bool pk = (t + 1) * KVB + kl >= Lk || npad;
        kbias[cur ^ 1][kl] = pk ? -INFINITY : 0.f;
        const uint64_t any = __ballot(pk);
        if (kl == 0) kpad[cur ^ 1] = any != 0ull;
      }
    }
    __syncthreads();
  }
  constexpr bool w8 = Q8;
  const float q8s = w8 ? *q8.qs : 1.f;
  float am = 0.f;
  // Q8: lane indices re-formed here, so hipcc does not share the row
  // products with the prologue's and keep them live across the key loop
  // (the copy's extra row address then spilled, with a reload per tile)
  int le = lane;
  if constexpr (Q8) asm volatile("" : "+v"(le));
  const int ge = le >> 4, ce = le & 15;
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int qi = q0w + gq * 16 + ce;
    float l = l_run[gq] + __shfl_xor(l_run[gq], 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qi >= Lq) continue;
    const float inv = l > 0.f ? (DROP ? drop_scale : 1.f) / l : 0.f;
    bf16* orow = o + (long)(b * Lq + qi) * ldo + h * D;
#pragma unroll
    for (int dt = 0; dt < C::NDT; ++dt) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(acc[gq][dt][r] * inv);
      *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * ge) = w;
      if constexpr (Q8) {  // e4m3 copy of the stored (bf16-rounded) values
        float f[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) f[r] = (float)w[r];
        *reinterpret_cast<uint32_t*>(q8.dq + (long)(b * Lq + qi) * q8.lddq + h * D + dt * 16 + 4 * ge) =
            smer_q8x4(f, q8s);
        am = fmaxf(am, smer_absmax4(f));
      }
    }
    if (ge == 0) lse[(long)bh * Lq + qi] = l > 0.f ? (m_ref[gq] + log2f(l)) * LN2_F : INFINITY;
  }
  if constexpr (Q8) smer_amax_commit(q8.amax, am);
}

// ---------------------------------------------------------------------------
// bf16 backward: dK / dV
// ---------------------------------------------------------------------------
// KG key groups of 16 per wave (block = 64*KG keys): the Q / dO fragments
// read from LDS per query tile feed KG groups.
// CAUSAL: the causal instances carry the per-element key > query test on
// diagonal tiles; the non-causal ones (encoder, cross-attention) none.
template <int D, bool DROP, int KG, bool MSK, bool CAUSAL>
__global__ __launch_bounds__(256, KG == 2 ? 2 : 3) void attn_bwd_dkdv_bf16(
    int B, int H, int Lq, int Lk, const bf16* __restrict__ q, long ldq,
    const bf16* __restrict__ k, long ldk, const bf16* __restrict__ v, long ldv,
    const bf16* __restrict__ dout, long lddo, const float* __restrict__ lse,
    const float* __restrict__ delta, const uint8_t* __restrict__ kpm, int causal, float scale,
    uint32_t drop_thr, uint32_t seed, float drop_scale, bf16* __restrict__ dk, long lddk,
    bf16* __restrict__ dv, long lddv, const uint64_t* __restrict__ drop_mask, AttnQ8 q8) {
  using C = AttnCfg<D>;
  constexpr int KB = 64 * KG;  // keys per block
  const int nq16 = (Lq + 15) >> 4, nkt = (Lk + KVB - 1) / KVB;
  __shared__ __attribute__((aligned(16))) char sm[2][2][C::TILE];
  // per query of the staged tile: lse (log2 units; +inf past Lq so P = 0),
  // delta, and the dropout row key
  __shared__ __attribute__((aligned(16))) float s_lse[2][KVB];
  __shared__ __attribute__((aligned(16))) float s_del[2][KVB];
  __shared__ __attribute__((aligned(16))) uint32_t s_rk[2][KVB];
  // keep words of the staged query tile x this block's key tiles:
  // [query 32-block][key tile][64 forward lanes] (attn_mask_word)
  __shared__ __attribute__((aligned(16))) uint32_t s_msk[2][2][KG][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  int BX, BY;
  xcd_block2d(BX, BY);
  const int bh = BY, b = bh / H, h = bh % H;
  const int k0w = BX * KB + wave * 16 * KG;  // first key of this wave
  const float c = scale * LOG2E_F;

  bf16x8 kf[KG][C::NS], vf[KG][C::NS];
  // padded keys get no gradient: their dK / dV rows are written as zeros.
  // The padding bytes are kept raw until the epilogue (a test right behind
  // the load made every workgroup wait for it before its K / V loads)
  // (loaded unconditionally -- from K's own bytes without a mask, ignored
  // through kmask -- as a load under a branch left a phi copy that waited)
  uint32_t kpad[KG];
  const uint8_t* kpb = kpm ? kpm + (long)b * Lk : reinterpret_cast<const uint8_t*>(k);
  const uint32_t kmask = kpm ? 0xFFu : 0u;
#pragma unroll
  for (int gk = 0; gk < KG; ++gk) {
    const int kj = k0w + gk * 16 + c16;
    kpad[gk] = kpb[min(kj, Lk - 1)];
    long row = (long)(b * Lk + min(kj, Lk - 1));
#pragma unroll
    for (int s = 0; s < C::NS; ++s) {
      kf[gk][s] = *reinterpret_cast<const bf16x8*>(k + row * ldk + h * D + s * 32 + 8 * g);
      vf[gk][s] = *reinterpret_cast<const bf16x8*>(v + row * ldv + h * D + s * 32 + 8 * g);
    }
  }
  const bf16* qb = q + (long)b * Lq * ldq + h * D;
  const bf16* ob = dout + (long)b * Lq * lddo + h * D;
  const float* lb = lse + (long)bh * Lq;
  const float* db = delta + (long)bh * Lq;

  const int n_qt = (Lq + KVB - 1) / KVB;
  const int t0 = causal ? min(n_qt, (BX * KB) / KVB) : 0;
  f32x4 adk[KG][C::NDT], adv[KG][C::NDT];
#pragma unroll
  for (int gk = 0; gk < KG; ++gk)
#pragma unroll
    for (int i = 0; i < C::NDT; ++i) {
      adk[gk][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      adv[gk][i] = adk[gk][i];
    }

  uint4 rq[C::CPT], ro[C::CPT];
  float rl = 0.f, rd = 0.f;
  uint32_t rr = 0u;
  uint4 rm = make_uint4(0, 0, 0, 0);
  constexpr bool use_mask = DROP && MSK;
  // this thread's 16-B chunk m_ch of the words of (query 32-block 2t + m_qr,
  // key tile m_kt): 2 x KG x 16 chunks per query tile
  const int nq32 = (Lq + 31) >> 5;
  const int m_qr = tid / (16 * KG), m_kt = BX * KG + (tid / 16) % KG, m_ch = tid & 15;
  const uint4* m_base = use_mask ? reinterpret_cast<const uint4*>(drop_mask) +
                                       (attn_mask_index(bh, nq32, nkt, 0, min(m_kt, nkt - 1)) >> 2) + m_ch
                                 : nullptr;
  auto load = [&](int t) {
    tile_load<D>(rq, qb, ldq, t * KVB, Lq, tid);
    tile_load<D>(ro, ob, lddo, t * KVB, Lq, tid);
    if (tid < KVB) {
      // raw values, scaled / masked when staged: arithmetic on them here made
      // hipcc wait for this tile's Q / dO prefetch right away
      const int qq = t * KVB + tid;
      rl = lb[min(qq, Lq - 1)];
      rd = db[min(qq, Lq - 1)];
      if (DROP && !MSK) rr = smer_rowkey(seed, (uint32_t)(bh * Lq + qq));
    }
    if (use_mask && tid < 32 * KG) {
      const int q32 = t * 2 + m_qr;
      rm = (q32 < nq32 && m_kt < nkt) ? m_base[(size_t)q32 * nkt * 16] : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf, int t) {
    tile_store<D>(rq, sm[buf][0], tid);
    tile_store<D>(ro, sm[buf][1], tid);
    asm volatile("" : "+v"(rl), "+v"(rd));  // keeps the arithmetic below here
    if (tid < KVB) {
      const bool qv = t * KVB + tid < Lq;
      s_lse[buf][tid] = qv ? rl * LOG2E_F : INFINITY;
      s_del[buf][tid] = qv ? rd : 0.f;
      if (DROP && !MSK) s_rk[buf][tid] = rr;
    }
    if (use_mask && tid < 32 * KG)
      reinterpret_cast<uint4*>(&s_msk[buf][0][0][0])[tid] = rm;
  };
  if (t0 < n_qt) { load(t0); store(0, t0); }
  __syncthreads();
  smer_vm_drain();  // prologue loads retired before the loop (common.h)
  // K pre-scaled by c = scale * log2(e) and the S chain seeded with -lse
  // (log2 units): p = 2^acc leaves the MFMA with no per-score arithmetic.
  // K is this kernel's register-resident operand, so the bf16 rounding of
  // the product lands on K here and on Q in the forward / dQ kernels: the
  // recomputed scores differ from the forward's by |s| * 2^-9 at most (one
  // bf16 rounding each, the size of the bf16 rounding of Q and K
  // themselves), so P matches the forward's lse to ~|s| * 2^-8 relative.
  // Held by the dK / dV checks against fp32 torch in tests/test_kernels_gpu.py
  // (bf16 tolerance), DESIGN.md §8.
#pragma unroll
  for (int gk = 0; gk < KG; ++gk)
#pragma unroll
    for (int s = 0; s < C::NS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) kf[gk][s][e] = (bf16)((float)kf[gk][s][e] * c);
  for (int t = t0; t < n_qt; ++t) {
    const int cur = (t - t0) & 1;
    const bool more = t + 1 < n_qt;
    if (more) load(t + 1);
    const char* Qs = sm[cur][0];
    const char* Os = sm[cur][1];
    // some key of this wave is later than some query of the tile
    const bool diag = CAUSAL && t * KVB < k0w + 16 * KG;
    bf16x8 pf[KG][2], sf[KG][2];
#pragma unroll
    for (int gk = 0; gk < KG; ++gk) {
      const int kj = k0w + gk * 16 + c16;
      float pd[4][4], ds[4][4];
      const int k16 = (k0w + gk * 16) >> 4;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(&s_lse[cur][mt * 16 + 4 * g]);
        f32x4 sacc = -l4, dpacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < C::NS; ++s) {
          sacc = mfma16(row_frag<D>(Qs, mt * 16, s, lane), kf[gk][s], sacc);
          dpacc = mfma16(row_frag<D>(Os, mt * 16, s, lane), vf[gk][s], dpacc);
        }
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&s_del[cur][mt * 16 + 4 * g]);
        // forward lane (G, c) of word [q32][key tile] holds (query 16gq + c,
        // key 16*mk + 4G + R) at bit 8R + 4gq + mk: this lane (key c16 of
        // 16-block k16, queries 4g..4g+3 of 16-block mt) reads the words of
        // lanes 16*(c16>>2) + 4g .. +3 (one 16-B read), bit
        // 8*(c16&3) + 4*(mt&1) + (k16&3)
        uint4 mw4 = make_uint4(0, 0, 0, 0);
        if constexpr (use_mask) {
          const int j = (k16 >> 2) - BX * KG;
          mw4 = *reinterpret_cast<const uint4*>(&s_msk[cur][mt >> 1][j][(c16 >> 2) * 16 + 4 * g]);
        }
        const uint32_t mbit = 8 * (c16 & 3) + 4 * (mt & 1) + (k16 & 3);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = fast_exp2(sacc[r]);
          if (CAUSAL && diag && kj > t * KVB + mt * 16 + 4 * g + r) pv = 0.f;
          float dpv = dpacc[r];
          float pdv = pv;
          if (DROP) {
            uint32_t m;
            if constexpr (use_mask) {
              m = bitmask32(r == 0 ? mw4.x : r == 1 ? mw4.y : r == 2 ? mw4.z : mw4.w, mbit);
            } else {
              m = smer_attn_keep(s_rk[cur][mt * 16 + 4 * g + r], drop_thr, (uint32_t)kj) ? ~0u : 0u;
            }
            // dropped P and dP; the survivors' 1 / (1 - p) goes into the dS
            // fma here and into dV's final write
            pdv = and_f32(pv, m);
            dpv = and_f32(dpv, m);
          }
          pd[mt][r] = pdv;
          ds[mt][r] = pv * fmaf(dpv, DROP ? drop_scale : 1.f, -d4[r]);
        }
      }
      pf[gk][0] = pack_p(pd, 0);
      pf[gk][1] = pack_p(pd, 1);
      sf[gk][0] = pack_p(ds, 0);
      sf[gk][1] = pack_p(ds, 1);
    }
    attn_prio_hi();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int dt = 0; dt < C::NDT; ++dt) {
        const bf16x8 of = tr_frag<D>(Os, ks, dt, lane);
        const bf16x8 qf = tr_frag<D>(Qs, ks, dt, lane);
#pragma unroll
        for (int gk = 0; gk < KG; ++gk) {
          adv[gk][dt] = mfma16(of, pf[gk][ks], adv[gk][dt]);
          adk[gk][dt] = mfma16(qf, sf[gk][ks], adk[gk][dt]);
        }
      }
    }
    attn_prio_lo();
    if (more) store(cur ^ 1, t + 1);
    __syncthreads();
  }
  const bool w8 = q8.dk != nullptr;  // (then dv too)
  const float q8s = w8 ? *q8.qs : 1.f;
  float am = 0.f;
#pragma unroll
  for (int gk = 0; gk < KG; ++gk) {
    const int kj = k0w + gk * 16 + c16;
    if (kj >= Lk) continue;
    bf16* dkr = dk + (long)(b * Lk + kj) * lddk + h * D;
    bf16* dvr = dv + (long)(b * Lk + kj) * lddv + h * D;
    const bool kvalid = (kpad[gk] & kmask) == 0u;
    // select, not multiply: a padded key's unmasked P may have overflowed
#pragma unroll
    for (int dt = 0; dt < C::NDT; ++dt) {
      bf16x4 wk, wv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        wk[r] = (bf16)(kvalid ? adk[gk][dt][r] * scale : 0.f);
        wv[r] = (bf16)(kvalid ? adv[gk][dt][r] * (DROP ? drop_scale : 1.f) : 0.f);
      }
      if (dk) {  // (null: the e4m3 copies alone)
        *reinterpret_cast<bf16x4*>(dkr + dt * 16 + 4 * g) = wk;
        *reinterpret_cast<bf16x4*>(dvr + dt * 16 + 4 * g) = wv;
      }
      if (w8) {  // e4m3 copies of the stored (bf16-rounded) values
        float fk[4], fv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          fk[r] = (float)wk[r];
          fv[r] = (float)wv[r];
        }
        const long col = h * D + dt * 16 + 4 * g;
        *reinterpret_cast<uint32_t*>(q8.dk + (long)(b * Lk + kj) * q8.lddk + col) = smer_q8x4(fk, q8s);
        *reinterpret_cast<uint32_t*>(q8.dv + (long)(b * Lk + kj) * q8.lddv + col) = smer_q8x4(fv, q8s);
        am = fmaxf(am, fmaxf(smer_absmax4(fk), smer_absmax4(fv)));
      }
    }
  }
  if (w8) smer_amax_commit(q8.amax, am);
}

// ---------------------------------------------------------------------------
// bf16 backward: dQ
// ---------------------------------------------------------------------------
template <int D, bool DROP, int QG, bool MSK, bool CAUSAL>
__global__ __launch_bounds__(256, QG == 2 ? 2 : 3) void attn_bwd_dq_bf16(
    int B, int H, int Lq, int Lk, const bf16* __restrict__ q, long ldq,
    const bf16* __restrict__ k, long ldk, const bf16* __restrict__ v, long ldv,
    const bf16* __restrict__ dout, long lddo, const float* __restrict__ lse,
    float* __restrict__ delta, const uint8_t* __restrict__ kpm, int causal, float scale,
    uint32_t drop_thr, uint32_t seed, float drop_scale, bf16* __restrict__ dq, long lddq,
    const uint64_t* __restrict__ drop_mask, const bf16* __restrict__ o, long ldo, AttnQ8 q8) {
  using C = AttnCfg<D>;
  constexpr int QB = 64 * QG;  // queries per block
  const int nq16 = (Lq + 15) >> 4, nkt = (Lk + KVB - 1) / KVB;
  __shared__ __attribute__((aligned(16))) char sm[2][2][C::TILE];
  __shared__ __attribute__((aligned(16))) float kbias[2][KVB];
  __shared__ int kpad[2];  // the staged tile has a padded / out-of-range key
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  int BX, BY;
  xcd_block2d(BX, BY);
  const int bh = BY, b = bh / H, h = bh % H;
  const int q0w = BX * QB + wave * 16 * QG;  // first query of this wave
  const float c = scale * LOG2E_F;
  constexpr bool use_mask = DROP && MSK;
  // this wave's keep words (the forward's lane mapping: one word per lane
  // and key tile, its 16 * QG queries inside one 32-query block), prefetched
  // a tile ahead in a register
  const int nq32 = (Lq + 31) >> 5;
  const uint32_t* mwp = use_mask
      ? reinterpret_cast<const uint32_t*>(drop_mask) + attn_mask_index(bh, nq32, nkt, min(q0w >> 5, nq32 - 1), 0) + lane
      : nullptr;
  const uint32_t gq_k = QG == 2 ? 0u : (uint32_t)((q0w >> 4) & 1);
  uint32_t mw_next = 0u;
  bf16x8 qf[QG][C::NS], of[QG][C::NS], ovr[QG][C::NS];
  float lse2[QG], dlt[QG];
  uint32_t rowkey[QG];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int qi = q0w + gq * 16 + c16;
    const bool qvalid = qi < Lq;
    long row = (long)(b * Lq + min(qi, Lq - 1));
#pragma unroll
    for (int s = 0; s < C::NS; ++s) {
      qf[gq][s] = *reinterpret_cast<const bf16x8*>(q + row * ldq + h * D + s * 32 + 8 * g);
      of[gq][s] = *reinterpret_cast<const bf16x8*>(dout + row * lddo + h * D + s * 32 + 8 * g);
      if (o) ovr[gq][s] = *reinterpret_cast<const bf16x8*>(o + row * ldo + h * D + s * 32 + 8 * g);
    }
    // raw lse, scaled once the first K / V tile's loads are in flight (a
    // use right after the load would wait for it there)
    lse2[gq] = lse[(long)bh * Lq + min(qi, Lq - 1)];
    if (!o) dlt[gq] = qvalid ? delta[(long)bh * Lq + qi] : 0.f;
    rowkey[gq] = (DROP && !MSK) ? smer_rowkey(seed, (uint32_t)(bh * Lq + qi)) : 0u;
  }
  const bf16* kb = k + (long)b * Lk * ldk + h * D;
  const bf16* vb = v + (long)b * Lk * ldv + h * D;
  const uint8_t* kp = kpm ? kpm + (long)b * Lk : nullptr;
  auto key_bias = [&](int key) -> float {
    return (key >= Lk || (kp && kp[key])) ? -INFINITY : 0.f;
  };
  int n_tiles = (Lk + KVB - 1) / KVB;
  if (causal) {
    int qmax = min(Lq, BX * QB + QB);
    n_tiles = min(n_tiles, (qmax + KVB - 1) / KVB);
  }
  f32x4 adq[QG][C::NDT];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq)
#pragma unroll
    for (int i = 0; i < C::NDT; ++i) adq[gq][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 rk[C::CPT], rv[C::CPT];
  if (n_tiles > 0) {
    // first tile's padding byte requested with its K / V, tested after they
    // land (see attn_fwd_bf16)
    const uint8_t* kpb = kp ? kp : reinterpret_cast<const uint8_t*>(kb);
    const uint32_t pmask = kp ? 0xFFu : 0u;
    const uint32_t pad0 = kpb[min(lane, Lk - 1)];
    if constexpr (use_mask) mw_next = mwp[0];
    tile_load<D>(rk, kb, ldk, 0, Lk, tid);
    tile_load<D>(rv, vb, ldv, 0, Lk, tid);
    tile_store<D>(rk, sm[0][0], tid);
    tile_store<D>(rv, sm[0][1], tid);
    if (tid < KVB) {  // wave 0
      const float kbz = (tid >= Lk || (pad0 & pmask)) ? -INFINITY : 0.f;
      kbias[0][tid] = kbz;
      const uint64_t any = __ballot(kbz != 0.f);
      if (tid == 0) kpad[0] = any != 0ull;
    }
  }
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    // +inf lse past Lq: P = 0 there (that lane's dQ row is never written)
    asm volatile("" : "+v"(lse2[gq]));
    lse2[gq] = q0w + gq * 16 + c16 < Lq ? lse2[gq] * LOG2E_F : INFINITY;
  }
  if (o) {
    // delta = rowsum(dO * O), formed once the first K / V tile's loads are
    // in flight: the row's 4 lane groups hold D / 4 columns each; published
    // for the dK / dV kernel, which runs after this one
#pragma unroll
    for (int gq = 0; gq < QG; ++gq) {
      const int qi = q0w + gq * 16 + c16;
      float dd = 0.f;
#pragma unroll
      for (int s = 0; s < C::NS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) dd += (float)of[gq][s][e] * (float)ovr[gq][s][e];
      dd += __shfl_xor(dd, 16);
      dd += __shfl_xor(dd, 32);
      dlt[gq] = qi < Lq ? dd : 0.f;
      if (qi < Lq && g == 0) delta[(long)bh * Lq + qi] = dd;
    }
  }
  __syncthreads();
  smer_vm_drain();  // prologue loads retired before the loop (common.h)
  // Q pre-scaled by c = scale * log2(e) (the forward's rounding, bit for
  // bit) and the S chain seeded with -lse: p = 2^acc
  f32x4 negl[QG];
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    negl[gq] = f32x4{-lse2[gq], -lse2[gq], -lse2[gq], -lse2[gq]};
#pragma unroll
    for (int s = 0; s < C::NS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[gq][s][e] = (bf16)((float)qf[gq][s][e] * c);
  }
  for (int t = 0; t < n_tiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < n_tiles;
    int npad = 0;  // compared when staged (see attn_fwd_bf16)
    const uint32_t mw = mw_next;
    if (more) {
      tile_load<D>(rk, kb, ldk, (t + 1) * KVB, Lk, tid);
      tile_load<D>(rv, vb, ldv, (t + 1) * KVB, Lk, tid);
      if (kp) npad = kp[min((t + 1) * KVB + lane, Lk - 1)];  // every lane: no exec-masked join
      if constexpr (use_mask) mw_next = mwp[(size_t)(t + 1) * 64];
    }
    const char* Ks = sm[cur][0];
    const char* Vs = sm[cur][1];
    f32x4 sacc[QG][4], dpacc[QG][4];
    attn_prio_hi();
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int gq = 0; gq < QG; ++gq) {
        sacc[gq][mt] = negl[gq];
        dpacc[gq][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int s = 0; s < C::NS; ++s) {
        const bf16x8 kf = row_frag<D>(Ks, mt * 16, s, lane);
        const bf16x8 vfr = row_frag<D>(Vs, mt * 16, s, lane);
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) {
          sacc[gq][mt] = mfma16(kf, qf[gq][s], sacc[gq][mt]);
          dpacc[gq][mt] = mfma16(vfr, of[gq][s], dpacc[gq][mt]);
        }
      }
    }
    attn_prio_lo();
    if (__builtin_amdgcn_readfirstlane(kpad[cur])) {
      // -inf on padded / out-of-range keys (tiles without any skip this)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 kbv = *reinterpret_cast<const f32x4*>(&kbias[cur][mt * 16 + 4 * g]);
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) sacc[gq][mt] += kbv;
      }
    }
    bf16x8 sf[QG][2];
#pragma unroll
    for (int gq = 0; gq < QG; ++gq) {
      const int qi = q0w + gq * 16 + c16;
      const bool diag = CAUSAL && t * KVB + KVB - 1 > q0w + gq * 16;
      float ds[4][4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        float dpv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) dpv[r] = dpacc[gq][mt][r];
        if constexpr (use_mask) {
          // same lane mapping as the forward: bit 8r + 4gq + mt of the word
          const uint32_t kq = 4u * (QG == 2 ? (uint32_t)gq : gq_k) + mt;
#pragma unroll
          for (int r = 0; r < 4; ++r) dpv[r] = and_f32(dpv[r], bitmask32(mw, 8 * r + kq));
        } else if (DROP) {
          const uint32_t hb = smer_attn_bits(rowkey[gq], (uint32_t)(t * (KVB / 4) + mt * 4 + g));
#pragma unroll
          for (int r = 0; r < 4; ++r) dpv[r] = ((hb >> (8 * r)) & 0x7Fu) >= drop_thr ? dpv[r] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = fast_exp2(sacc[gq][mt][r]);
          if (CAUSAL && diag && t * KVB + mt * 16 + 4 * g + r > qi) pv = 0.f;
          // dS = P (keep * dP / (1 - p) - delta)
          ds[mt][r] = pv * fmaf(dpv[r], DROP ? drop_scale : 1.f, -dlt[gq]);
        }
      }
      sf[gq][0] = pack_p(ds, 0);
      sf[gq][1] = pack_p(ds, 1);
    }
    attn_prio_hi();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int dt = 0; dt < C::NDT; ++dt) {
        const bf16x8 kt = tr_frag<D>(Ks, ks, dt, lane);
#pragma unroll
        for (int gq = 0; gq < QG; ++gq) adq[gq][dt] = mfma16(kt, sf[gq][ks], adq[gq][dt]);
      }
    }
    attn_prio_lo();
    if (more) {
      tile_store<D>(rk, sm[cur ^ 1][0], tid);
      tile_store<D>(rv, sm[cur ^ 1][1], tid);
      asm volatile("" : "+v"(npad));  // keeps the compare (and its wait) here
      if (tid < KVB) {  // wave 0
        const bool pk = (t + 1) * KVB + tid >= Lk || npad;
        kbias[cur ^ 1][tid] = pk ? -INFINITY : 0.f;
        const uint64_t any = __ballot(pk);
        if (tid == 0) kpad[cur ^ 1] = any != 0ull;
      }
    }
    __syncthreads();
  }
  const bool w8 = q8.dq != nullptr;
  const float q8s = w8 ? *q8.qs : 1.f;
  float am = 0.f;
#pragma unroll
  for (int gq = 0; gq < QG; ++gq) {
    const int qi = q0w + gq * 16 + c16;
    if (qi >= Lq) continue;
    bf16* dqr = dq + (long)(b * Lq + qi) * lddq + h * D;
#pragma unroll
    for (int dt = 0; dt < C::NDT; ++dt) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16)(adq[gq][dt][r] * scale);
      if (dq) *reinterpret_cast<bf16x4*>(dqr + dt * 16 + 4 * g) = w;  // (null: the e4m3 copy alone)
      if (w8) {  // e4m3 copy of the stored (bf16-rounded) values
        float f[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) f[r] = (float)w[r];
        *reinterpret_cast<uint32_t*>(q8.dq + (long)(b * Lq + qi) * q8.lddq + h * D + dt * 16 + 4 * g) =
            smer_q8x4(f, q8s);
        am = fmaxf(am, smer_absmax4(f));
      }
    }
  }
  if (w8) smer_amax_commit(q8.amax, am);
}

template <typename T>
__global__ void attn_delta_scalar(int B, int H, int Lq, int D, const T* __restrict__ o, long ldo,
                                  const T* __restrict__ dout, long lddo, float* __restrict__ delta) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * Lq;
  if (idx >= total) return;
  int i = idx % Lq;
  int bh = idx / Lq;
  int b = bh / H, h = bh % H;
  const T* orow = o + (long)(b * Lq + i) * ldo + h * D;
  const T* drow = dout + (long)(b * Lq + i) * lddo + h * D;
  float s = 0.f;
  for (int d = 0; d < D; ++d) s += to_f32(orow[d]) * to_f32(drow[d]);
  delta[idx] = s;
}

// delta[bh, i] = sum_d dO[i, h*D + d] * O[i, h*D + d]
// LPR = D/8 lanes per (row, head), 8 elements (one 16-B bf16 load) per lane.
template <typename T, int LPR>
__global__ __launch_bounds__(256) void attn_delta(int B, int H, int Lq, int D,
                                                  const T* __restrict__ o, long ldo,
                                                  const T* __restrict__ dout, long lddo,
                                                  float* __restrict__ delta) {
  const long item = ((long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int part = threadIdx.x % LPR;
  const long total = (long)B * H * Lq;
  const bool ok = item < total;
  float s = 0.f;
  if (ok) {
    int i = item % Lq;
    int bh = item / Lq;
    int b = bh / H, h = bh % H;
    float a[8], c[8];
    load8<T>(o + (long)(b * Lq + i) * ldo + h * D + part * 8, 8, a);
    load8<T>(dout + (long)(b * Lq + i) * lddo + h * D + part * 8, 8, c);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k] * c[k];
  }
#pragma unroll
  for (int off = 1; off < LPR; off <<= 1) s += __shfl_xor(s, off, 64);
  if (ok && part == 0) {
    int i = item % Lq;
    int bh = item / Lq;
    delta[(long)bh * Lq + i] = s;
  }
}

template <typename T>
static void launch_delta(int B, int H, int Lq, int D, const void* o, long ldo, const void* dout,
                         long lddo, float* delta, hipStream_t s) {
  long threads = (long)B * H * Lq * (D / 8);
  dim3 g((threads + 255) / 256);
  if (D == 32)
    hipLaunchKernelGGL((attn_delta<T, 4>), g, dim3(256), 0, s, B, H, Lq, D, (const T*)o, ldo, (const T*)dout, lddo, delta);
  else if (D == 64)
    hipLaunchKernelGGL((attn_delta<T, 8>), g, dim3(256), 0, s, B, H, Lq, D, (const T*)o, ldo, (const T*)dout, lddo, delta);
  else if (D == 128)
    hipLaunchKernelGGL((attn_delta<T, 16>), g, dim3(256), 0, s, B, H, Lq, D, (const T*)o, ldo, (const T*)dout, lddo, delta);
  else
    hipLaunchKernelGGL((attn_delta_scalar<T>), dim3(((long)B * H * Lq + 255) / 256), dim3(256), 0, s, B, H, Lq, D, (const T*)o, ldo, (const T*)dout, lddo, delta);
}

// ---------------------------------------------------------------------------
// f32 kernels (parity mode): one wave per query row
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool attn_visible(const uint8_t* kp, int key, int qi, int causal) {
  return (!kp || !kp[key]) && (!causal || key <= qi);
}

__global__ __launch_bounds__(256) void attn_fwd_f32(int B, int H, int Lq, int Lk, int D,
                                                    const float* __restrict__ q, long ldq,
                                                    const float* __restrict__ k, long ldk,
                                                    const float* __restrict__ v, long ldv,
                                                    float* __restrict__ o, long ldo,
                                                    float* __restrict__ lse,
                                                    const uint8_t* __restrict__ kpm, int causal,
                                                    float scale, uint32_t drop_thr, uint32_t seed,
                                                    float drop_scale) {
  extern __shared__ float sc_all[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int qi = blockIdx.x * 4 + wave;
  if (qi >= Lq) return;
  float* sc = sc_all + wave * Lk;
  const float* qrow = q + (long)(b * Lq + qi) * ldq + h * D;
  const uint8_t* kp = kpm ? kpm + (long)b * Lk : nullptr;
  float mx = -INFINITY;
  for (int j = lane; j < Lk; j += 64) {
    float s = -INFINITY;
    if (attn_visible(kp, j, qi, causal)) {
      const float* krow = k + (long)(b * Lk + j) * ldk + h * D;
      float a = 0.f;
      for (int d = 0; d < D; ++d) a = fmaf(qrow[d] * scale, krow[d], a);
      s = a;
    }
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  const float mu = mx == -INFINITY ? 0.f : mx;
  float sum = 0.f;
  for (int j = lane; j < Lk; j += 64) {
    float e = expf(sc[j] - mu);
    sum += e;
    if (drop_thr) e = smer_attn_keep(smer_rowkey(seed, (uint32_t)(bh * Lq + qi)), drop_thr, (uint32_t)j) ? e * drop_scale : 0.f;
    sc[j] = e;
  }
  sum = wave_sum(sum);
  __builtin_amdgcn_wave_barrier();
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  for (int d = lane; d < D; d += 64) {
    float a = 0.f;
    for (int j = 0; j < Lk; ++j) a = fmaf(sc[j], v[(long)(b * Lk + j) * ldv + h * D + d], a);
    o[(long)(b * Lq + qi) * ldo + h * D + d] = a * inv;
  }
  if (lane == 0) lse[(long)bh * Lq + qi] = sum > 0.f ? mu + logf(sum) : INFINITY;
}

// fp32 flash forward on the fp32 MFMA (v_mfma_f32_16x16x4_f32: full fp32
// products and sums, no reduced-precision inputs), D = 64, no dropout: the
// parity-mode prefill of the plugin call (encoder self-attention over ~1k
// source tokens: 1.26 ms per layer on attn_fwd_f32's wave-per-query loop)
// and fp32 training forwards.  A wave owns 16 queries; per 64-key tile it
// forms S^T = K Q^T (16x16 blocks, keys as rows) so that a lane's four
// scores of a block (keys 4g + r, query c16) are exactly the A operand of
// the four P.V MFMAs (key sets {4g + r}), no transposition; the contraction
// over d runs in lane-group order (MFMA c sums d = 16 g + c over g), so each
// lane reads 16 consecutive floats of one Q row and one K row.  Online
// softmax with expf in fp32 (lse = m + log l, as attn_fwd_f32); rows with no
// visible key give O = 0, lse = +inf.
__global__ __launch_bounds__(256) void attn_fwd_f32_mfma(int B, int H, int Lq, int Lk,
                                                         const float* __restrict__ q, long ldq,
                                                         const float* __restrict__ k, long ldk,
                                                         const float* __restrict__ v, long ldv,
                                                         float* __restrict__ o, long ldo,
                                                         float* __restrict__ lse,
                                                         const uint8_t* __restrict__ kpm, int causal,
                                                         float scale) {
  constexpr int D = 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int q0 = blockIdx.x * 64 + wave * 16;
  if (q0 >= Lq) return;  // no block-level synchronisation below
  const int c16 = lane & 15, g = lane >> 4;
  const int qi = q0 + c16;  // this lane's query (S^T column)
  float qf[16];
  {
    const float4* qr = reinterpret_cast<const float4*>(q + (long)(b * Lq + min(qi, Lq - 1)) * ldq + h * D + 16 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 t = qr[i];
      qf[4 * i] = t.x * scale; qf[4 * i + 1] = t.y * scale; qf[4 * i + 2] = t.z * scale; qf[4 * i + 3] = t.w * scale;
    }
  }
  f32x4 oacc[4];
#pragma unroll
  for (int dq = 0; dq < 4; ++dq) oacc[dq] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;  // query qi's running max / sum (same in all 4 g lanes)
  const uint8_t* kp = kpm ? kpm + (long)b * Lk : nullptr;
  const int kend = causal ? min(Lk, q0 + 16) : Lk;
  const float* kb0 = k + (long)b * Lk * ldk + h * D;
  const float* vb0 = v + (long)b * Lk * ldv + h * D;
  for (int k0 = 0; k0 < kend; k0 += 64) {
    f32x4 st[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int key = min(k0 + 16 * kb + c16, Lk - 1);
      const float4* kr = reinterpret_cast<const float4*>(kb0 + (long)key * ldk + 16 * g);
      float kf[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 t = kr[i];
        kf[4 * i] = t.x; kf[4 * i + 1] = t.y; kf[4 * i + 2] = t.z; kf[4 * i + 3] = t.w;
      }
      st[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 16; ++c) st[kb] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[c], qf[c], st[kb], 0, 0, 0);
    }
    // V rows of the four P.V MFMAs per key block: key 16 kb + 4 g + r,
    // columns 16 dq + c16
    float vf[4][4][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* vr = vb0 + (long)min(k0 + 16 * kb + 4 * g + r, Lk - 1) * ldv + c16;
#pragma unroll
        for (int dq = 0; dq < 4; ++dq) vf[kb][r][dq] = vr[16 * dq];
      }
    // masks and the tile max of query qi
    float tmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * kb + 4 * g + r;
        const bool vis = key < Lk && (!kp || !kp[key]) && (!causal || key <= qi);
        st[kb][r] = vis ? st[kb][r] : -INFINITY;
        tmax = fmaxf(tmax, st[kb][r]);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float alpha = mn == -INFINITY ? 1.f : expf(m - mn);
    float ts = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = st[kb][r] == -INFINITY ? 0.f : expf(st[kb][r] - mn);
        st[kb][r] = p;
        ts += p;
      }
    ts += __shfl_xor(ts, 16, 64);
    ts += __shfl_xor(ts, 32, 64);
    l = l * alpha + ts;
    m = mn;
    // O rows are queries 4 g + r': their factors from lanes c16 = 4 g + r'
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
      for (int dq = 0; dq < 4; ++dq) oacc[dq][r] *= ar;
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int dq = 0; dq < 4; ++dq)
          oacc[dq] = __builtin_amdgcn_mfma_f32_16x16x4f32(st[kb][r], vf[kb][r][dq], oacc[dq], 0, 0, 0);
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qr = q0 + 4 * g + r;
    const float ir = __shfl(inv, 4 * g + r, 64);
    if (qr < Lq) {
      float* orow = o + (long)(b * Lq + qr) * ldo + h * D + c16;
#pragma unroll
      for (int dq = 0; dq < 4; ++dq) orow[16 * dq] = oacc[dq][r] * ir;
    }
  }
  if (g == 0 && qi < Lq) lse[(long)bh * Lq + qi] = l > 0.f ? m + logf(l) : INFINITY;
}

// P / dS materialisation: ws_p = dropped P, ws_s = dS  ([B*H, Lq, Lk])
__global__ void attn_bwd_ps_f32(int B, int H, int Lq, int Lk, int D, const float* q, long ldq,
                                const float* k, long ldk, const float* v, long ldv,
                                const float* dout, long lddo, const float* lse,
                                const float* delta, const uint8_t* kpm, int causal, float scale,
                                uint32_t drop_thr, uint32_t seed, float drop_scale, float* ws_p,
                                float* ws_s) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * Lq * Lk;
  if (idx >= total) return;
  int j = idx % Lk;
  long r = idx / Lk;
  int qi = r % Lq;
  int bh = r / Lq, b = bh / H, h = bh % H;
  const uint8_t* kp = kpm ? kpm + (long)b * Lk : nullptr;
  float p = 0.f, dp = 0.f;
  if (attn_visible(kp, j, qi, causal)) {
    const float* qrow = q + (long)(b * Lq + qi) * ldq + h * D;
    const float* krow = k + (long)(b * Lk + j) * ldk + h * D;
    const float* vrow = v + (long)(b * Lk + j) * ldv + h * D;
    const float* orow = dout + (long)(b * Lq + qi) * lddo + h * D;
    float s = 0.f;
    for (int d = 0; d < D; ++d) { s = fmaf(qrow[d] * scale, krow[d], s); dp = fmaf(orow[d], vrow[d], dp); }
    p = expf(s - lse[r]);
  }
  float pd = p;
  if (drop_thr) {
    bool keep = smer_attn_keep(smer_rowkey(seed, (uint32_t)(bh * Lq + qi)), drop_thr, (uint32_t)j);
    pd = keep ? p * drop_scale : 0.f;
    dp = keep ? dp * drop_scale : 0.f;
  }
  ws_p[idx] = pd;
  ws_s[idx] = p * (dp - delta[r]);
}

// dK, dV rows: thread per (bh, key, d)
__global__ void attn_bwd_kv_f32(int B, int H, int Lq, int Lk, int D, const float* q, long ldq,
                                const float* dout, long lddo, const float* ws_p,
                                const float* ws_s, float scale, float* dk, long lddk, float* dv,
                                long lddv) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * Lk * D;
  if (idx >= total) return;
  int d = idx % D;
  long r = idx / D;
  int j = r % Lk;
  int bh = r / Lk, b = bh / H, h = bh % H;
  float ak = 0.f, av = 0.f;
  const float* P = ws_p + (long)bh * Lq * Lk + j;
  const float* S = ws_s + (long)bh * Lq * Lk + j;
  for (int i = 0; i < Lq; ++i) {
    long row = (long)(b * Lq + i);
    ak = fmaf(S[(long)i * Lk], q[row * ldq + h * D + d], ak);
    av = fmaf(P[(long)i * Lk], dout[row * lddo + h * D + d], av);
  }
  dk[(long)(b * Lk + j) * lddk + h * D + d] = ak * scale;
  dv[(long)(b * Lk + j) * lddv + h * D + d] = av;
}

__global__ void attn_bwd_q_f32(int B, int H, int Lq, int Lk, int D, const float* k, long ldk,
                               const float* ws_s, float scale, float* dq, long lddq) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * H * Lq * D;
  if (idx >= total) return;
  int d = idx % D;
  long r = idx / D;
  int qi = r % Lq;
  int bh = r / Lq, b = bh / H, h = bh % H;
  const float* S = ws_s + ((long)bh * Lq + qi) * Lk;
  float a = 0.f;
  for (int j = 0; j < Lk; ++j) a = fmaf(S[j], k[(long)(b * Lk + j) * ldk + h * D + d], a);
  dq[(long)(b * Lq + qi) * lddq + h * D + d] = a * scale;
}

// head-averaged probabilities (the `weights` the reference returns)
template <typename T>
__global__ void attn_weights_kernel(int B, int H, int Lq, int Lk, int D, const T* q, long ldq,
                                    const T* k, long ldk, const float* lse, const uint8_t* kpm,
                                    int causal, float scale, float* out) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)B * Lq * Lk;
  if (idx >= total) return;
  int j = idx % Lk;
  long r = idx / Lk;
  int qi = r % Lq;
  int b = r / Lq;
  const uint8_t* kp = kpm ? kpm + (long)b * Lk : nullptr;
  float acc = 0.f;
  if (attn_visible(kp, j, qi, causal)) {
    for (int h = 0; h < H; ++h) {
      const T* qrow = q + (long)(b * Lq + qi) * ldq + h * D;
      const T* krow = k + (long)(b * Lk + j) * ldk + h * D;
      float s = 0.f;
      for (int d = 0; d < D; ++d) s = fmaf(to_f32(qrow[d]), to_f32(krow[d]), s);
      acc += expf(s * scale - lse[((long)b * H + h) * Lq + qi]);
    }
  }
  out[idx] = acc / H;
}

// ---------------------------------------------------------------------------
// decode attention (KV cache) — one workgroup per (row, head)
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void attn_decode_kernel(int H, int D, const T* __restrict__ q,
                                                          long ldq, const T* __restrict__ kc,
                                                          const T* __restrict__ vc,
                                                          long row_stride, long req_stride,
                                                          long head_stride,
                                                          const int32_t* __restrict__ row_req,
                                                          const int32_t* __restrict__ row_nkeys,
                                                          T* __restrict__ o, long ldo,
                                                          float scale) {
  extern __shared__ float dsm[];
  __shared__ float red[8];
  __shared__ float qs[256];
  __shared__ float part[4][256];
  const int r = blockIdx.x, h = blockIdx.y, tid = threadIdx.x;
  const int nk = row_nkeys[r];
  const long base = (long)row_req[r] * req_stride + h * head_stride;
  for (int d = tid; d < D; d += 256) qs[d] = to_f32(q[(long)r * ldq + h * D + d]) * scale;
  __syncthreads();
  float mx = -INFINITY;
  for (int j = tid; j < nk; j += 256) {
    const T* kr = kc + base + (long)j * row_stride;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(qs[d], to_f32(kr[d]), s);
    dsm[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int j = tid; j < nk; j += 256) {
    float e = expf(dsm[j] - mx);
    dsm[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = sum;
  __syncthreads();
  sum = red[4] + red[5] + red[6] + red[7];
  // 4 key groups x 64 lanes over d
  const int grp = tid >> 6, ln = tid & 63;
  for (int d0 = 0; d0 < D; d0 += 64) {
    int d = d0 + ln;
    float a = 0.f;
    if (d < D)
      for (int j = grp; j < nk; j += 4) a = fmaf(dsm[j], to_f32(vc[base + (long)j * row_stride + d]), a);
    part[grp][ln] = a;
    __syncthreads();
    if (grp == 0 && d < D) {
      float t = (part[0][ln] + part[1][ln]) + (part[2][ln] + part[3][ln]);
      o[(long)r * ldo + h * D + d] = from_f32<T>(sum > 0.f ? t / sum : 0.f);
    }
    __syncthreads();
  }
}

// Vectorised single-pass decode attention (online softmax).  One block per
// (row, head), NW waves.  LPK lanes own one key (each lane a 16-B slice of
// D = LPK*VEC), so a wave walks 64/LPK keys per step with 16-B K and V
// loads; UNR steps are issued together (raw 16-B registers, converted at
// use) so that NW * UNR * 2 KiB of K/V per block are in flight — the cross
// attention over a 1-4k-token memory is HBM-latency bound otherwise.  The
// UNR keys of a step update the running (max, sum, acc[VEC]) of a lane
// group with ONE rescale; groups are merged with shuffles, waves via LDS.
template <typename T>
__device__ __forceinline__ void cvt16b(const uint4& r, float (&v)[16 / sizeof(T)]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 t = __builtin_bit_cast(bf16x8, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)t[i];
  } else {
    v[0] = __uint_as_float(r.x); v[1] = __uint_as_float(r.y);
    v[2] = __uint_as_float(r.z); v[3] = __uint_as_float(r.w);
  }
}
template <typename T>
__device__ __forceinline__ void load16b(const T* p, float (&v)[16 / sizeof(T)]) {
  cvt16b<T>(*reinterpret_cast<const uint4*>(p), v);
}
// Sum over aligned groups of G (4, 8 or 16) lanes by DPP butterflies (no
// LDS round trip): quad xor 1 / xor 2, then half-mirror (8), mirror (16).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  v += dpp_f(v, 0xB1);
  v += dpp_f(v, 0x4E);
  if constexpr (G >= 8) v += dpp_f(v, 0x141);
  if constexpr (G >= 16) v += dpp_f(v, 0x140);
  return v;
}

// The cross-attention query projection with the LayerNorm in front of it
// (transformer.py:462 -> 459 -> 463), computed inside the decode attention
// block of (head h, row r): y is the pre-norm row, the block normalises it
// (ln_row_stats / ln_apply: the LayerNorm kernel's bits; blocks of head 0
// store it, the next sublayer's residual) and forms its head's D query
// values as a bf16-rounded x . Wq_h^T + bq_h (fp32 dot products, 512 / D
// threads per output), replacing the cross-Q Linear launch.
// The fp32 form (dec_q_prologue_f32, the plugin's fp32 step at batch 1) keeps
// every value in fp32, as the Linear it replaces.
struct DecQ {
  const void* y;  // the kernel's T (bf16 / fp32), as wq and x_out
  long ldy;
  const float* gamma;
  const float* beta;
  float eps;
  const void* wq;  // [H*D rows, dmodel] (this head: rows h*D ..)
  long ldw;
  const float* bq;
  void* x_out;
  long ldx;
  int dmodel;
};

// pf(): called once every load of the prologue has been issued (before any
// of them is used): the caller issues its first K / V key step there, so
// that step's HBM round trip runs under the prologue's (vmcnt counts in issue
// order: the prologue's loads are older, so waiting for them leaves the K / V
// loads in flight)
template <int D, int NT, int DM, typename PF>
__device__ __forceinline__ void dec_q_prologue(const DecQ& dq, int h, int r, int tid, float* qs,
                                               bf16* xs, bool need_q, bool store_x, PF pf) {
  constexpr int TPO = NT / D;    // threads per query value
  constexpr int KT = DM / TPO;   // K per thread (multiple of 8)
  const int lane = tid & 63, wave = tid >> 6;
  const int d = tid / TPO, part = tid % TPO;
  // the head's weight row slice, requested before the row statistics (not
  // at all for a row with <= 1 key: softmax over one key is 1 whatever q,
  // e.g. a decode session's dummy rows)
  const bf16* wr = static_cast<const bf16*>(dq.wq) + (long)(h * D + d) * dq.ldw + part * KT;
  // every load of the prologue issued before any of it is used, all
  // unconditional (chunk indices clamped; every wave reads the row and
  // gamma / beta, wave 0 normalises): the guarded loads and the gamma / beta
  // reads inside the normalisation made each block wait for one load after
  // another.  Same arithmetic as ln_row_stats / ln_apply.
  constexpr int NC = (DM + 511) / 512;  // 16-B chunks per lane
  constexpr int NCH = DM / 8;
  bf16x8 yv[NC];
  float4 gv[NC][2], bv[NC][2];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = min(lane + 64 * c, NCH - 1);
    yv[c] = *reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(dq.y) + (long)r * dq.ldy + ch * 8);
    gv[c][0] = *reinterpret_cast<const float4*>(dq.gamma + ch * 8);
    gv[c][1] = *reinterpret_cast<const float4*>(dq.gamma + ch * 8 + 4);
    bv[c][0] = *reinterpret_cast<const float4*>(dq.beta + ch * 8);
    bv[c][1] = *reinterpret_cast<const float4*>(dq.beta + ch * 8 + 4);
  }
  bf16x8 wv[KT / 8];
#pragma unroll
  for (int j = 0; j < KT / 8; ++j) wv[j] = *reinterpret_cast<const bf16x8*>(wr + 8 * j);
  __builtin_amdgcn_sched_barrier(0);
  pf();
  __builtin_amdgcn_sched_barrier(0);
  if (wave == 0) {
    float v[NC][8], mu, rs;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = (float)yv[c][i];
    ln_stats_loaded<NC>(v, DM, dq.eps, lane, mu, rs);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NCH) {
        const float g[8] = {gv[c][0].x, gv[c][0].y, gv[c][0].z, gv[c][0].w,
                            gv[c][1].x, gv[c][1].y, gv[c][1].z, gv[c][1].w};
        const float b[8] = {bv[c][0].x, bv[c][0].y, bv[c][0].z, bv[c][0].w,
                            bv[c][1].x, bv[c][1].y, bv[c][1].z, bv[c][1].w};
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (bf16)ln_apply(v[c][i], mu, rs, g[i], b[i]);
        *reinterpret_cast<bf16x8*>(xs + ch * 8) = o;
        if (store_x && dq.x_out) *reinterpret_cast<bf16x8*>(static_cast<bf16*>(dq.x_out) + (long)r * dq.ldx + ch * 8) = o;
      }
    }
  }
  __syncthreads();
  if (need_q) {  // block-uniform
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < KT / 8; ++j) {
      const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + part * KT + 8 * j);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc = fmaf((float)xv[i], (float)wv[j][i], acc);
    }
#pragma unroll
    for (int w = 1; w < TPO; w <<= 1) acc += __shfl_xor(acc, w, 64);
    if (part == 0) qs[d] = (float)(bf16)(acc + dq.bq[h * D + d]);
  } else if (part == 0) {
    qs[d] = 0.f;
  }
  __syncthreads();
}

// fp32 form: x = LN(y) in fp32 (ln_stats_loaded / ln_apply: the bits of
// gemm_skinny_ln_f32_kernel, whose x_out this replaces), q_h = x . Wq_h^T + bq_h
// in fp32 without rounding.  The NT / D threads of one output read its weight
// row interleaved (thread p takes the 16-B chunks p, p + TPO, ..: a row's
// threads read contiguous 64 B per load), all DM / TPO weights of a thread
// requested before the row statistics.
template <int D, int NT, int DM>
__device__ __forceinline__ void dec_q_prologue_f32(const DecQ& dq, int h, int r, int tid, float* qs, float* xs,
                                                   bool need_q, bool store_x) {
  constexpr int TPO = NT / D;            // threads per query value
  constexpr int NJ = DM / (4 * TPO);     // 16-B weight chunks per thread
  static_assert(DM % (4 * TPO) == 0 && DM % 8 == 0, "dec_q_prologue_f32: d_model");
  const int lane = tid & 63, wave = tid >> 6;
  const int d = tid / TPO, part = tid % TPO;
  const float* wr = static_cast<const float*>(dq.wq) + (long)(h * D + d) * dq.ldw + 4 * part;
  const float* yr = static_cast<const float*>(dq.y) + (long)r * dq.ldy;
  constexpr int NC = (DM + 511) / 512;  // 32-B chunks per lane
  constexpr int NCH = DM / 8;
  float v[NC][8], g[NC][8], b[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = min(lane + 64 * c, NCH - 1);
    load8<float>(yr + ch * 8, 8, v[c]);
    load8<float>(dq.gamma + ch * 8, 8, g[c]);
    load8<float>(dq.beta + ch * 8, 8, b[c]);
  }
  float4 wv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) wv[j] = *reinterpret_cast<const float4*>(wr + 4 * TPO * j);
  if (wave == 0) {
    float mu, rs;
    ln_stats_loaded<NC>(v, DM, dq.eps, lane, mu, rs);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < NCH) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = ln_apply(v[c][i], mu, rs, g[c][i], b[c][i]);
        *reinterpret_cast<float4*>(xs + ch * 8) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(xs + ch * 8 + 4) = make_float4(o[4], o[5], o[6], o[7]);
        if (store_x && dq.x_out) {
          float* xo = static_cast<float*>(dq.x_out) + (long)r * dq.ldx + ch * 8;
          *reinterpret_cast<float4*>(xo) = make_float4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<float4*>(xo + 4) = make_float4(o[4], o[5], o[6], o[7]);
        }
      }
    }
  }
  __syncthreads();
  if (need_q) {  // block-uniform
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 xv = *reinterpret_cast<const float4*>(xs + 4 * (TPO * j + part));
      acc = fmaf(xv.x, wv[j].x, acc);
      acc = fmaf(xv.y, wv[j].y, acc);
      acc = fmaf(xv.z, wv[j].z, acc);
      acc = fmaf(xv.w, wv[j].w, acc);
    }
#pragma unroll
    for (int w = 1; w < TPO; w <<= 1) acc += __shfl_xor(acc, w, 64);
    if (part == 0) qs[d] = acc + dq.bq[h * D + d];
  } else if (part == 0) {
    qs[d] = 0.f;
  }
  __syncthreads();
}

#ifndef SMER_DEC_QSKIP
#define SMER_DEC_QSKIP 1  // tools/build_variant.sh ... -DSMER_DEC_QSKIP=0: the A/B baseline
#endif
#ifndef SMER_DEC_QLN_EARLY
// bf16 query prologue: the first K / V key step issued behind the prologue's
// own loads, before its math (round 6; -DSMER_DEC_QLN_EARLY=0: after it)
#define SMER_DEC_QLN_EARLY 1
#endif
// NS > 0: the keys of a (row, head) split over NS blocks (blockIdx.z), each
// writing its unnormalised partial {m, l, pad, pad, acc[D]} (fp32, 4 + D
// floats) to part[((row * H + head) * NS + z) * (4 + D)] instead of o (the
// consumer merges them in fixed order: flash-decoding for few rows)
template <typename T, int LPK, int UNR, int NW, bool PIPE = false, int QP = 0, int NS = 0>
__global__ __launch_bounds__(64 * NW) void attn_decode_vec_kernel(
    const T* __restrict__ q, long ldq, const T* __restrict__ kc, const T* __restrict__ vc,
    long row_stride, long req_stride, long head_stride, const int32_t* __restrict__ row_req,
    const int32_t* __restrict__ row_nkeys, T* __restrict__ o, long ldo, float scale,
    DecQ dq = DecQ{}, int odd_first = 0, float* __restrict__ part = nullptr) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int GPW = 64 / LPK;  // key groups per wave
  constexpr int KPB = NW * GPW;  // keys per block step
  __shared__ float red_m[NW][LPK], red_l[NW][LPK], red_a[NW][LPK][VEC];
  // heads of a row dispatch together.  odd_first: block rows y < n/2 take
  // the odd rows (a decode session's last-token slots, the live ones), the
  // rest the even rows (mostly one-key dummies): dispatched in row order the
  // live blocks of an XCD alternated with dummies and so landed on every
  // other CU of its round-robin
  const int ny = gridDim.y, yb = blockIdx.y;
  const int r = (odd_first && !(ny & 1)) ? (yb < (ny >> 1) ? 2 * yb + 1 : 2 * (yb - (ny >> 1))) : yb;
  const int h = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int sub = lane % LPK, grp = wave * GPW + lane / LPK;
  const int nk_all = row_nkeys[r];
  // this block's keys [kb, nk): all of them, or split NS's slice
  int kb = 0, nk = nk_all;
  if constexpr (NS > 0) {
    const int chunk = ((nk_all + NS - 1) / NS + KPB - 1) / KPB * KPB;
    kb = min(nk_all, (int)blockIdx.z * chunk);
    nk = min(nk_all, kb + chunk);
  }
  const long base = (long)row_req[r] * req_stride + h * head_stride + sub * VEC;
  float qv[VEC];
  float m = -INFINITY, l = 0.f, acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  // the K / V rows of key step j0 (UNR keys per lane group)
  auto load_step = [&](int j0, uint4 (&kr)[UNR], uint4 (&vr)[UNR]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int j = j0 + u * KPB + grp;
      const long off = base + (long)(j < nk ? j : 0) * row_stride;
      if constexpr (NW == 8) {  // long memories: once-read per step, stream non-temporally
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(kc + off));
        const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vc + off));
        kr[u] = make_uint4(a.x, a.y, a.z, a.w);
        vr[u] = make_uint4(b.x, b.y, b.z, b.w);
      } else {
        kr[u] = *reinterpret_cast<const uint4*>(kc + off);
        vr[u] = *reinterpret_cast<const uint4*>(vc + off);
      }
    }
  };
  // PIPE (memories of >= 2048 keys): the next step's loads are issued
  // before this step's math (two steps of K / V in flight per lane group;
  // measured 5.2 -> 5.7 TB/s at 4096 keys, slower at 1000)
  uint4 kr[UNR], vr[UNR];
  constexpr bool early = QP > 0 && sizeof(T) == 2 && SMER_DEC_QLN_EARLY;
  if constexpr (QP > 0) {  // QP = d_model of the query prologue
    __shared__ float qs[LPK * VEC];
    const bool need_q = SMER_DEC_QSKIP ? nk_all > 1 : true;
    const bool store_x = h == 0 && (NS == 0 || blockIdx.z == 0);  // one block per row stores LN(y)
    if constexpr (sizeof(T) == 2) {
      __shared__ __attribute__((aligned(16))) bf16 xs[QP];
      dec_q_prologue<LPK * VEC, 64 * NW, QP>(dq, h, r, tid, qs, xs, need_q, store_x, [&] {
        if constexpr (early) {
          if (nk > kb) load_step(kb, kr, vr);
        }
      });
    } else {
      __shared__ __attribute__((aligned(16))) float xs[QP];
      dec_q_prologue_f32<LPK * VEC, 64 * NW, QP>(dq, h, r, tid, qs, xs, need_q, store_x);
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) qv[i] = qs[sub * VEC + i];
  } else {
    load16b<T>(q + (long)r * ldq + h * (LPK * VEC) + sub * VEC, qv);
  }
  // (QP: requesting the first key step's K / V before the query prologue
  // measured slower, 368 vs 336 us per decode step, and at C5's 4096-key
  // memories 46.4k vs 47.5k tokens/s: issued after it.  Without the
  // prologue the first step is requested before q is scaled, in both forms:
  // scaling q first made every block wait for q before its K / V loads.)
  if ((PIPE || QP == 0) && !early && nk > kb) load_step(kb, kr, vr);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < VEC; ++i) qv[i] *= scale;
  for (int j0 = kb; j0 < nk; j0 += KPB * UNR) {
    uint4 kn[UNR], vn[UNR];
    if constexpr (PIPE) {
      if (j0 + KPB * UNR < nk) load_step(j0 + KPB * UNR, kn, vn);
    } else {
      if ((QP != 0 && !early) || j0 != kb) load_step(j0, kr, vr);
    }
    float sc[UNR];
    float mx = m;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      float kv[VEC];
      cvt16b<T>(kr[u], kv);
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < VEC; ++i) s = fmaf(qv[i], kv[i], s);
      s = group_sum<LPK>(s);
      sc[u] = (j0 + u * KPB + grp) < nk ? s : -INFINITY;
      mx = fmaxf(mx, sc[u]);
    }
    if (mx != -INFINITY) {  // group-uniform: some key of this step is valid
      const float c = __expf(m - mx);
      l *= c;
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] *= c;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const float p = __expf(sc[u] - mx);
        float vv[VEC];
        cvt16b<T>(vr[u], vv);
        l += p;
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = fmaf(p, vv[i], acc[i]);
      }
      m = mx;
    }
    if constexpr (PIPE) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        kr[u] = kn[u];
        vr[u] = vn[u];
      }
    }
  }
  // merge the groups of a wave (lanes with equal `sub`)
#pragma unroll
  for (int w = LPK; w < 64; w <<= 1) {
    const float mo = __shfl_xor(m, w, 64), lo = __shfl_xor(l, w, 64);
    const float mn = fmaxf(m, mo);
    const float c0 = m == -INFINITY ? 0.f : __expf(m - mn);
    const float c1 = mo == -INFINITY ? 0.f : __expf(mo - mn);
    l = l * c0 + lo * c1;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = acc[i] * c0 + __shfl_xor(acc[i], w, 64) * c1;
    m = mn;
  }
  if (lane < LPK) {
    red_m[wave][lane] = m;
    red_l[wave][lane] = l;
#pragma unroll
    for (int i = 0; i < VEC; ++i) red_a[wave][lane][i] = acc[i];
  }
  __syncthreads();
  if (tid < LPK) {
    float mm = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) mm = fmaxf(mm, red_m[w][tid]);
    float ll = 0.f, out[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) out[i] = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float c = red_m[w][tid] == -INFINITY ? 0.f : __expf(red_m[w][tid] - mm);
      ll += red_l[w][tid] * c;
#pragma unroll
      for (int i = 0; i < VEC; ++i) out[i] += red_a[w][tid][i] * c;
    }
    if constexpr (NS > 0) {
      float* pr = part + (((long)r * gridDim.x + h) * NS + blockIdx.z) * (4 + LPK * VEC);
      if (tid == 0) { pr[0] = mm; pr[1] = ll; }
#pragma unroll
      for (int i = 0; i < VEC; ++i) pr[4 + tid * VEC + i] = out[i];
      return;
    }
    const float inv = ll > 0.f ? 1.f / ll : 0.f;
    T* op = o + (long)r * ldo + h * (LPK * VEC) + tid * VEC;
    if constexpr (sizeof(T) == 2) {
      bf16x8 t;
#pragma unroll
      for (int i = 0; i < VEC; ++i) t[i] = (bf16)(out[i] * inv);
      *reinterpret_cast<bf16x8*>(op) = t;
    } else {
      *reinterpret_cast<float4*>(op) = make_float4(out[0] * inv, out[1] * inv, out[2] * inv, out[3] * inv);
    }
  }
}

template <typename T>
__global__ void kv_scatter_kernel(int n_rows, int width, const T* __restrict__ src, long lds,
                                  T* __restrict__ cache, long row_stride, long req_stride,
                                  const int32_t* __restrict__ row_req,
                                  const int32_t* __restrict__ row_pos) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)n_rows * width) return;
  int r = idx / width, c = idx % width;
  cache[(long)row_req[r] * req_stride + (long)row_pos[r] * row_stride + c] = src[(long)r * lds + c];
}

// Head-major K/V cache fill (decode cross-attention memory): src row m holds
// [K heads | V heads] (2*H*D columns); element (kv, h, dd) of row m goes to
// cache[req[m]*req_stride + kv*kv_stride + h*head_stride + pos[m]*D + dd],
// so each (request, head) reads one contiguous key run per step.
template <typename T>
__global__ void kv_scatter_heads_kernel(int n_rows, int H, int D, const T* __restrict__ src,
                                        long lds, T* __restrict__ cache, long req_stride,
                                        long kv_stride, long head_stride,
                                        const int32_t* __restrict__ row_req,
                                        const int32_t* __restrict__ row_pos) {
  constexpr int VEC = 16 / sizeof(T);
  const int cpr = 2 * H * D / VEC;  // 16-B chunks per row
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)n_rows * cpr) return;
  const int m = idx / cpr, col = (idx % cpr) * VEC;
  const int kv = col / (H * D), h = (col % (H * D)) / D, dd = col % D;
  *reinterpret_cast<uint4*>(cache + (long)row_req[m] * req_stride + kv * kv_stride +
                            h * head_stride + (long)row_pos[m] * D + dd) =
      *reinterpret_cast<const uint4*>(src + (long)m * lds + col);
}

// The attention-dropout keep words of a whole [B*H, Lq, Lk] score matrix
// (layout: attn_mask_word).  One wave per (bh, query 32-block): each lane
// hashes its two row keys once and walks every key tile, 8 hashes and one
// 4-B store per tile (long-lived waves: a wave per (block, tile) spent as
// long in dispatch as in its 100 VALU instructions).  Pure integer VALU at
// full occupancy; no division anywhere.
__global__ __launch_bounds__(256) void attn_drop_mask_gen_kernel(int Lq, int nq32, int nkt, uint32_t thr,
                                                                uint32_t seed, uint32_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int q32 = blockIdx.x * 4 + (threadIdx.x >> 6), bh = blockIdx.y;
  if (q32 >= nq32) return;
  const uint32_t row0 = (uint32_t)bh * (uint32_t)Lq + (uint32_t)(q32 * 32 + (lane & 15));
  const uint32_t rk0 = smer_rowkey(seed, row0), rk1 = smer_rowkey(seed, row0 + 16u);
  const uint32_t lo4 = thr * 0x01010101u;
  uint32_t* o = out + attn_mask_index(bh, nq32, nkt, q32, 0) + lane;
  for (int t = 0; t < nkt; ++t)
    __builtin_nontemporal_store(attn_mask_word(rk0, rk1, (uint32_t)t, (uint32_t)(lane >> 4), lo4), o + (size_t)t * 64);
}

static void mask_gen_launch(int B, int H, int Lq, int Lk, uint32_t thr, uint32_t seed, void* mask,
                            hipStream_t s) {
  const int nq32 = (Lq + 31) / 32, nkt = (Lk + 63) / 64;
  hipLaunchKernelGGL(attn_drop_mask_gen_kernel, dim3((nq32 + 3) / 4, B * H), dim3(256), 0, s, Lq, nq32, nkt,
                     thr, seed, (uint32_t*)mask);
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int D>
static void fwd_bf16_launch(int B, int H, int Lq, int Lk, const void* q, long ldq, const void* k,
                            long ldk, const void* v, long ldv, void* o, long ldo, float* lse,
                            const uint8_t* kpm, int causal, float scale, uint32_t thr,
                            uint32_t seed, float ds, uint64_t* mask, int mask_in, const AttnQ8& q8,
                            hipStream_t s) {
  // two query groups per wave once there are enough blocks to fill the chip
  const bool qg2 = (long)((Lq + 127) / 128) * B * H >= 512 && D <= 64;
  dim3 grid(qg2 ? (Lq + 127) / 128 : (Lq + 63) / 64, B * H);
  // a mask buffer: the keep words come from the generator (launched here
  // first unless the caller already filled them) and the backward reads the
  // same words; no buffer: the forward hashes them itself
  // with a mask buffer the QG = 2 forward hashes the keep bits in its loop
  // and publishes them (cheaper than the separate generator: C2 encoder
  // forward + generator 125 + 29 us vs ~14x us hashing + publishing); a
  // QG = 1 wave holds half a 32-query block, so there the generator fills
  // the buffer and the forward reads it
  const bool min_ = thr && mask && (mask_in || !qg2);
  if (min_ && !mask_in) mask_gen_launch(B, H, Lq, Lk, thr, seed, mask, s);
  auto kern = qg2 ? (min_ ? attn_fwd_bf16<D, 2, true, true>
                          : (thr ? attn_fwd_bf16<D, 2, true> : attn_fwd_bf16<D, 2, false>))
                  : (min_ ? attn_fwd_bf16<D, 1, true, true>
                          : (thr ? attn_fwd_bf16<D, 1, true> : attn_fwd_bf16<D, 1, false>));
  if constexpr (D == 64) {
    if (q8.dq)
      kern = qg2 ? (min_ ? attn_fwd_bf16<D, 2, true, true, true>
                         : (thr ? attn_fwd_bf16<D, 2, true, false, true> : attn_fwd_bf16<D, 2, false, false, true>))
                 : (min_ ? attn_fwd_bf16<D, 1, true, true, true>
                         : (thr ? attn_fwd_bf16<D, 1, true, false, true> : attn_fwd_bf16<D, 1, false, false, true>));
  }
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, B, H, Lq, Lk, (const bf16*)q, ldq,
                     (const bf16*)k, ldk, (const bf16*)v, ldv, (bf16*)o, ldo, lse, kpm, causal,
                     scale, thr, seed, ds, thr ? (uint64_t*)mask : nullptr, q8);
}

// [bh][query 32-block][key 64-tile][64 lanes] u32 words (attn_mask_word):
// lane (G, c) holds (query 32*q32 + 16*gq + c, key 64*t + 16*mt + 4G + R) at
// bit 8R + 4gq + mt.  1 bit per (query, key).
extern "C" size_t smer_attn_drop_mask_bytes(int B, int H, int Lq, int Lk) {
  return (size_t)B * H * ((Lq + 31) / 32) * ((Lk + 63) / 64) * 256;
}

extern "C" int smer_attn_drop_mask_gen(int B, int H, int Lq, int Lk, float drop_p, uint32_t seed,
                                       void* mask, smer_stream_t stream) {
  SMER_REQUIRE(B > 0 && H > 0 && Lq > 0 && Lk > 0 && mask, "smer_attn_drop_mask_gen: bad arguments");
  SMER_REQUIRE((((uintptr_t)mask) & 15) == 0, "smer_attn_drop_mask_gen: mask alignment");
  SMER_REQUIRE(drop_p > 0.f && drop_p < 1.f, "smer_attn_drop_mask_gen: drop_p");
  mask_gen_launch(B, H, Lq, Lk, smer_attn_thr7(drop_p), seed, mask, (hipStream_t)stream);
  SMER_CHECK_LAUNCH("smer_attn_drop_mask_gen");
  return SMER_OK;
}

// SMER_ATTN_F32_MFMA=0 keeps the fp32 forward on attn_fwd_f32 (A/B, tests)
static bool smer_attn_f32_mfma() {
  const char* e = getenv("SMER_ATTN_F32_MFMA");
  return !(e && e[0] == '0');
}

static int attn_fwd_impl(int dtype, int B, int H, int Lq, int Lk, int D, const void* q, long ldq,
                         const void* k, long ldk, const void* v, long ldv, void* o, long ldo,
                         float* lse, const uint8_t* kpm, int causal, float scale, float drop_p,
                         uint32_t seed, void* drop_mask, int drop_mask_in, const AttnQ8& q8,
                         smer_stream_t stream) {
  SMER_REQUIRE(B > 0 && H > 0 && Lq >= 0 && Lk > 0 && D > 0, "smer_attn_fwd: bad sizes");
  SMER_REQUIRE(!drop_mask_in || drop_mask, "smer_attn_fwd: drop_mask_in without a mask");
  SMER_REQUIRE(!drop_mask || (((uintptr_t)drop_mask) & 15) == 0, "smer_attn_fwd: mask alignment");
  SMER_REQUIRE(q && k && v && o && lse, "smer_attn_fwd: null pointer");
  SMER_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "smer_attn_fwd: drop_p");
  if (Lq == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  uint32_t thr = smer_attn_thr7(drop_p);
  float ds = smer_attn_scale7(thr);
  if (dtype == SMER_BF16) {
    SMER_REQUIRE(al16(q) && al16(k) && al16(v), "smer_attn_fwd: 16-B alignment");
    SMER_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0,
                 "smer_attn_fwd: row strides must be multiples of 8");
    if (D == 32) fwd_bf16_launch<32>(B, H, Lq, Lk, q, ldq, k, ldk, v, ldv, o, ldo, lse, kpm, causal, scale, thr, seed, ds, (uint64_t*)drop_mask, drop_mask_in, q8, s);
    else if (D == 64) fwd_bf16_launch<64>(B, H, Lq, Lk, q, ldq, k, ldk, v, ldv, o, ldo, lse, kpm, causal, scale, thr, seed, ds, (uint64_t*)drop_mask, drop_mask_in, q8, s);
    else if (D == 128) fwd_bf16_launch<128>(B, H, Lq, Lk, q, ldq, k, ldk, v, ldv, o, ldo, lse, kpm, causal, scale, thr, seed, ds, (uint64_t*)drop_mask, drop_mask_in, q8, s);
    else return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_attn_fwd(bf16): head dim must be 32, 64 or 128");
  } else if (dtype == SMER_F32) {
    if (D == 64 && thr == 0 && al16(q) && al16(k) && ldq % 4 == 0 && ldk % 4 == 0 && smer_attn_f32_mfma()) {
      dim3 grid((Lq + 63) / 64, B * H);
      hipLaunchKernelGGL(attn_fwd_f32_mfma, grid, dim3(256), 0, s, B, H, Lq, Lk, (const float*)q, ldq,
                         (const float*)k, ldk, (const float*)v, ldv, (float*)o, ldo, lse, kpm, causal, scale);
      SMER_CHECK_LAUNCH("smer_attn_fwd");
      return SMER_OK;
    }
    SMER_REQUIRE((size_t)Lk * 16 <= 160 * 1024, "smer_attn_fwd(f32): Lk too large");
    dim3 grid((Lq + 3) / 4, B * H);
    hipLaunchKernelGGL(attn_fwd_f32, grid, dim3(256), (size_t)Lk * 16, s, B, H, Lq, Lk, D,
                       (const float*)q, ldq, (const float*)k, ldk, (const float*)v, ldv,
                       (float*)o, ldo, lse, kpm, causal, scale, thr, seed, ds);
  } else {
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_attn_fwd: dtype");
  }
  SMER_CHECK_LAUNCH("smer_attn_fwd");
  return SMER_OK;
}

extern "C" int smer_attn_fwd(int dtype, int B, int H, int Lq, int Lk, int D, const void* q,
                             long ldq, const void* k, long ldk, const void* v, long ldv, void* o,
                             long ldo, float* lse, const uint8_t* kpm, int causal, float scale,
                             float drop_p, uint32_t seed, void* drop_mask, int drop_mask_in,
                             smer_stream_t stream) {
  const AttnQ8 none{};
  return attn_fwd_impl(dtype, B, H, Lq, Lk, D, q, ldq, k, ldk, v, ldv, o, ldo, lse, kpm, causal, scale,
                       drop_p, seed, drop_mask, drop_mask_in, none, stream);
}

extern "C" int smer_attn_fwd_fp8(int B, int H, int Lq, int Lk, int D, const void* q, long ldq,
                                 const void* k, long ldk, const void* v, long ldv, void* o, long ldo,
                                 float* lse, const uint8_t* kpm, int causal, float scale, float drop_p,
                                 uint32_t seed, void* drop_mask, int drop_mask_in, void* o8, long ldo8,
                                 const float* qs, unsigned* amax, smer_stream_t stream) {
  SMER_REQUIRE(o8 && qs && amax && (((uintptr_t)o8) & 3) == 0 && ldo8 % 4 == 0,
               "smer_attn_fwd_fp8: 4-B aligned copy, scale and amax");
  SMER_REQUIRE(D == 64, "smer_attn_fwd_fp8: head dim 64");
  const AttnQ8 q8{(uint8_t*)o8, ldo8, nullptr, 0, nullptr, 0, qs, amax};
  return attn_fwd_impl(SMER_BF16, B, H, Lq, Lk, D, q, ldq, k, ldk, v, ldv, o, ldo, lse, kpm, causal,
                       scale, drop_p, seed, drop_mask, drop_mask_in, q8, stream);
}

extern "C" size_t smer_attn_bwd_workspace(int dtype, int B, int H, int Lq, int Lk) {
  size_t delta = ((size_t)B * H * Lq * sizeof(float) + 255) & ~(size_t)255;
  if (dtype == SMER_F32) return delta + 2 * (size_t)B * H * Lq * Lk * sizeof(float);
  return delta;
}

#ifndef SMER_DQ_DELTA
#define SMER_DQ_DELTA 1
#endif
template <int D>
static void bwd_bf16_launch(int B, int H, int Lq, int Lk, const void* q, long ldq, const void* k,
                            long ldk, const void* v, long ldv, const void* dout, long lddo,
                            const float* lse, float* delta, const uint8_t* kpm, int causal,
                            float scale, uint32_t thr, uint32_t seed, float ds, void* dq,
                            long lddq, void* dk, long lddk, void* dv, long lddv,
                            const uint64_t* mask, const void* o, long ldo, const AttnQ8& q8,
                            hipStream_t s) {
  if (!thr) mask = nullptr;
  // two key groups per wave once there are enough blocks to fill the chip
  const bool kg2 = (long)((Lk + 127) / 128) * B * H >= 512 && D <= 64;
  // dropout variants: recompute the keep bits by hashing, or read the
  // forward's stored bits (MSK); causal and non-causal instances
#define SMER_BWD_PICK(K, G, C)                                                        \
  (!thr ? K<D, false, G, false, C> : mask ? K<D, true, G, true, C> : K<D, true, G, false, C>)
  const bool cz = causal != 0;
  auto kdkdv = kg2 ? (cz ? SMER_BWD_PICK(attn_bwd_dkdv_bf16, 2, true) : SMER_BWD_PICK(attn_bwd_dkdv_bf16, 2, false))
                   : (cz ? SMER_BWD_PICK(attn_bwd_dkdv_bf16, 1, true) : SMER_BWD_PICK(attn_bwd_dkdv_bf16, 1, false));
  const bool qg2 = (long)((Lq + 127) / 128) * B * H >= 512 && D <= 64;
  auto kdq = qg2 ? (cz ? SMER_BWD_PICK(attn_bwd_dq_bf16, 2, true) : SMER_BWD_PICK(attn_bwd_dq_bf16, 2, false))
                 : (cz ? SMER_BWD_PICK(attn_bwd_dq_bf16, 1, true) : SMER_BWD_PICK(attn_bwd_dq_bf16, 1, false));
#undef SMER_BWD_PICK
  // o != null: the dQ kernel forms delta = rowsum(dO * O) itself and runs
  // first (no separate delta pass); else delta was written beforehand
  auto launch_dq = [&] {
    hipLaunchKernelGGL(kdq, dim3(qg2 ? (Lq + 127) / 128 : (Lq + 63) / 64, B * H), dim3(256), 0, s, B, H,
                       Lq, Lk, (const bf16*)q, ldq, (const bf16*)k, ldk, (const bf16*)v, ldv,
                       (const bf16*)dout, lddo, lse, delta, kpm, causal, scale, thr, seed, ds,
                       (bf16*)dq, lddq, mask, (const bf16*)o, ldo, q8);
  };
  if (o) launch_dq();
  hipLaunchKernelGGL(kdkdv, dim3(kg2 ? (Lk + 127) / 128 : (Lk + 63) / 64, B * H), dim3(256), 0, s, B, H, Lq,
                     Lk, (const bf16*)q, ldq, (const bf16*)k, ldk, (const bf16*)v, ldv,
                     (const bf16*)dout, lddo, lse, delta, kpm, causal, scale, thr, seed, ds,
                     (bf16*)dk, lddk, (bf16*)dv, lddv, mask, q8);
  if (!o) launch_dq();
}

static int attn_bwd_impl(int dtype, int B, int H, int Lq, int Lk, int D, const void* q,
                         long ldq, const void* k, long ldk, const void* v, long ldv,
                         const void* o, long ldo, const void* dout, long lddo,
                         const float* lse, const uint8_t* kpm, int causal, float scale,
                         float drop_p, uint32_t seed, void* dq, long lddq, void* dk, long lddk,
                         void* dv, long lddv, void* workspace, size_t ws_bytes,
                         const void* drop_mask, const AttnQ8& q8, smer_stream_t stream) {
  SMER_REQUIRE(B > 0 && H > 0 && Lq > 0 && Lk > 0 && D > 0, "smer_attn_bwd: bad sizes");
  // (bf16 with e4m3 copies: dq, or dk with dv, may be null beside their copies)
  SMER_REQUIRE(q && k && v && o && dout && lse && (dq || q8.dq) && (dk || q8.dk) && !dk == !dv,
               "smer_attn_bwd: null pointer");
  SMER_REQUIRE(workspace && ws_bytes >= smer_attn_bwd_workspace(dtype, B, H, Lq, Lk),
               "smer_attn_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  uint32_t thr = smer_attn_thr7(drop_p);
  float ds = smer_attn_scale7(thr);
  float* delta = (float*)workspace;
  long nrow = (long)B * H * Lq;
  if (dtype == SMER_BF16) {
    SMER_REQUIRE(al16(q) && al16(k) && al16(v) && al16(dout), "smer_attn_bwd: 16-B alignment");
    SMER_REQUIRE(al16(o) && ldo % 8 == 0 && lddo % 8 == 0, "smer_attn_bwd: O/dO alignment");
    // SMER_DQ_DELTA=0 (A/B builds): separate delta pass, dK / dV kernel first
    const void* of = SMER_DQ_DELTA ? o : nullptr;
    if (!of) launch_delta<bf16>(B, H, Lq, D, o, ldo, dout, lddo, delta, s);
    if (D == 32) bwd_bf16_launch<32>(B, H, Lq, Lk, q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, kpm, causal, scale, thr, seed, ds, dq, lddq, dk, lddk, dv, lddv, (const uint64_t*)drop_mask, of, ldo, q8, s);
    else if (D == 64) bwd_bf16_launch<64>(B, H, Lq, Lk, q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, kpm, causal, scale, thr, seed, ds, dq, lddq, dk, lddk, dv, lddv, (const uint64_t*)drop_mask, of, ldo, q8, s);
    else if (D == 128) bwd_bf16_launch<128>(B, H, Lq, Lk, q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, kpm, causal, scale, thr, seed, ds, dq, lddq, dk, lddk, dv, lddv, (const uint64_t*)drop_mask, of, ldo, q8, s);
    else return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_attn_bwd(bf16): head dim must be 32, 64 or 128");
  } else if (dtype == SMER_F32) {
    hipLaunchKernelGGL(attn_delta_scalar<float>, dim3((nrow + 255) / 256), dim3(256), 0, s, B, H,
                       Lq, D, (const float*)o, ldo, (const float*)dout, lddo, delta);
    size_t doff = ((size_t)nrow * sizeof(float) + 255) & ~(size_t)255;
    float* ws_p = (float*)((char*)workspace + doff);
    float* ws_s = ws_p + (size_t)B * H * Lq * Lk;
    long tot = (long)B * H * Lq * Lk;
    hipLaunchKernelGGL(attn_bwd_ps_f32, dim3((tot + 255) / 256), dim3(256), 0, s, B, H, Lq, Lk, D,
                       (const float*)q, ldq, (const float*)k, ldk, (const float*)v, ldv,
                       (const float*)dout, lddo, lse, delta, kpm, causal, scale, thr, seed, ds,
                       ws_p, ws_s);
    long tk = (long)B * H * Lk * D;
    hipLaunchKernelGGL(attn_bwd_kv_f32, dim3((tk + 255) / 256), dim3(256), 0, s, B, H, Lq, Lk, D,
                       (const float*)q, ldq, (const float*)dout, lddo, ws_p, ws_s, scale,
                       (float*)dk, lddk, (float*)dv, lddv);
    long tq = (long)B * H * Lq * D;
    hipLaunchKernelGGL(attn_bwd_q_f32, dim3((tq + 255) / 256), dim3(256), 0, s, B, H, Lq, Lk, D,
                       (const float*)k, ldk, ws_s, scale, (float*)dq, lddq);
  } else {
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_attn_bwd: dtype");
  }
  SMER_CHECK_LAUNCH("smer_attn_bwd");
  return SMER_OK;
}

extern "C" int smer_attn_bwd(int dtype, int B, int H, int Lq, int Lk, int D, const void* q,
                             long ldq, const void* k, long ldk, const void* v, long ldv,
                             const void* o, long ldo, const void* dout, long lddo,
                             const float* lse, const uint8_t* kpm, int causal, float scale,
                             float drop_p, uint32_t seed, void* dq, long lddq, void* dk, long lddk,
                             void* dv, long lddv, void* workspace, size_t ws_bytes,
                             const void* drop_mask, smer_stream_t stream) {
  const AttnQ8 none{};
  return attn_bwd_impl(dtype, B, H, Lq, Lk, D, q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, kpm,
                       causal, scale, drop_p, seed, dq, lddq, dk, lddk, dv, lddv, workspace, ws_bytes,
                       drop_mask, none, stream);
}

extern "C" int smer_attn_bwd_fp8(int B, int H, int Lq, int Lk, int D, const void* q, long ldq,
                                 const void* k, long ldk, const void* v, long ldv, const void* o,
                                 long ldo, const void* dout, long lddo, const float* lse,
                                 const uint8_t* kpm, int causal, float scale, float drop_p,
                                 uint32_t seed, void* dq, long lddq, void* dk, long lddk, void* dv,
                                 long lddv, void* workspace, size_t ws_bytes, const void* drop_mask,
                                 void* dq8, long lddq8, void* dk8, long lddk8, void* dv8, long lddv8,
                                 const float* qs, unsigned* amax, smer_stream_t stream) {
  SMER_REQUIRE(!dk8 == !dv8, "smer_attn_bwd_fp8: dK and dV copies go together");
  SMER_REQUIRE((!dq8 && !dk8) || (qs && amax), "smer_attn_bwd_fp8: scale and amax");
  auto al4 = [](const void* p, long ld) { return p == nullptr || ((((uintptr_t)p) & 3) == 0 && ld % 4 == 0); };
  SMER_REQUIRE(al4(dq8, lddq8) && al4(dk8, lddk8) && al4(dv8, lddv8),
               "smer_attn_bwd_fp8: 4-B aligned copies and row strides");
  const AttnQ8 q8{(uint8_t*)dq8, lddq8, (uint8_t*)dk8, lddk8, (uint8_t*)dv8, lddv8, qs, amax};
  return attn_bwd_impl(SMER_BF16, B, H, Lq, Lk, D, q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse,
                       kpm, causal, scale, drop_p, seed, dq, lddq, dk, lddk, dv, lddv, workspace,
                       ws_bytes, drop_mask, q8, stream);
}

extern "C" int smer_attn_weights(int dtype, int B, int H, int Lq, int Lk, int D, const void* q,
                                 long ldq, const void* k, long ldk, const float* lse,
                                 const uint8_t* kpm, int causal, float scale, float* out,
                                 smer_stream_t stream) {
  SMER_REQUIRE(q && k && lse && out, "smer_attn_weights: null pointer");
  long tot = (long)B * Lq * Lk;
  if (tot == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(attn_weights_kernel<bf16>, dim3((tot + 255) / 256), dim3(256), 0, s, B, H,
                       Lq, Lk, D, (const bf16*)q, ldq, (const bf16*)k, ldk, lse, kpm, causal,
                       scale, out);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(attn_weights_kernel<float>, dim3((tot + 255) / 256), dim3(256), 0, s, B,
                       H, Lq, Lk, D, (const float*)q, ldq, (const float*)k, ldk, lse, kpm, causal,
                       scale, out);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_attn_weights: dtype");
  SMER_CHECK_LAUNCH("smer_attn_weights");
  return SMER_OK;
}

// SMER_DECODE_ODD_FIRST=0: blocks in plain row order (A/B)
// SMER_DEC_PIPE_SMALL=0: grids of <= 128 blocks take the unpipelined form
static bool smer_dec_pipe_small() {
  const char* e = getenv("SMER_DEC_PIPE_SMALL");
  return !(e && e[0] == '0');
}
static int smer_dec_odd_first() {
  const char* e = getenv("SMER_DECODE_ODD_FIRST");
  return (e && e[0] == '0') ? 0 : 1;
}

// fp32 decode attention over NS = 8 key slices per (row, head): partial
// {m, l, acc} records for smer_linear_decode_merge_f32 (the plugin's batch-1
// step: 16 blocks of the unsplit form stream a ~1k-key memory each)
extern "C" int smer_attn_decode_split_f32(int n_rows, int H, int D, const void* q, long ldq, const void* kcache,
                                          const void* vcache, long row_stride, long req_stride, long head_stride,
                                          const int32_t* row_req, const int32_t* row_nkeys, float* part,
                                          float scale, smer_stream_t stream) {
  SMER_REQUIRE(D == 64 && H > 0, "smer_attn_decode_split_f32: head dim 64");
  SMER_REQUIRE(q && kcache && vcache && row_req && row_nkeys && part, "smer_attn_decode_split_f32: null pointer");
  auto al = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  SMER_REQUIRE(al(q) && al(kcache) && al(vcache) && al(part) && ldq % 4 == 0 && row_stride % 4 == 0 &&
                   req_stride % 4 == 0 && (head_stride <= 0 || head_stride % 4 == 0),
               "smer_attn_decode_split_f32: alignment / strides");
  if (n_rows == 0) return SMER_OK;
  if (head_stride <= 0) head_stride = D;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(H, n_rows, 8);
  // pipelined key loads (the next key step requested before this step's
  // math; the same arithmetic as the unpipelined form, so the same bits):
  // batch-1 plugin call 2,621 vs 2,534 tokens/s (two rounds,
  // tools/batch1_bench.py env SMER_DEC_SPLIT_CFG; 8-wave and 4-step forms
  // 2,558-2,607)
  hipLaunchKernelGGL((attn_decode_vec_kernel<float, 16, 2, 4, true, 0, 8>), grid, dim3(256), 0, s, (const float*)q,
                     ldq, (const float*)kcache, (const float*)vcache, row_stride, req_stride, head_stride, row_req,
                     row_nkeys, (float*)nullptr, 0L, scale, DecQ{}, 0, part);
  SMER_CHECK_LAUNCH("smer_attn_decode_split_f32");
  return SMER_OK;
}

// smer_attn_decode_split_f32 with the cross-attention query projection and
// the LayerNorm in front of it computed in each block (dec_q_prologue_f32):
// the plugin's fp32 step at batch 1, where the LN + Linear launch it replaces
// was one of ~40 latency-bound launches per token.  x_out = LN(y) (the
// merge's residual), written by the z = 0 block of head 0.  d_model 512.
extern "C" int smer_attn_decode_split_qln_f32(int n_rows, int H, int D, const float* y, long ldy,
                                              const float* gamma, const float* beta, float eps,
                                              const float* wq, long ldw, const float* bq, float* x_out,
                                              long ldx, int dmodel, const void* kcache, const void* vcache,
                                              long row_stride, long req_stride, long head_stride,
                                              const int32_t* row_req, const int32_t* row_nkeys, float* part,
                                              float scale, smer_stream_t stream) {
  SMER_REQUIRE(D == 64 && H > 0, "smer_attn_decode_split_qln_f32: head dim 64");
  SMER_REQUIRE(dmodel == 512, "smer_attn_decode_split_qln_f32: d_model 512 (else: Linear + split attention)");
  SMER_REQUIRE(y && gamma && beta && wq && bq && kcache && vcache && row_req && row_nkeys && part,
               "smer_attn_decode_split_qln_f32: null pointer");
  auto al = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  SMER_REQUIRE(al(y) && al(gamma) && al(beta) && al(wq) && al(kcache) && al(vcache) && al(part) &&
                   (!x_out || al(x_out)) && ldy % 4 == 0 && ldw % 4 == 0 && ldx % 4 == 0 && row_stride % 4 == 0 &&
                   req_stride % 4 == 0 && (head_stride <= 0 || head_stride % 4 == 0),
               "smer_attn_decode_split_qln_f32: 16-B alignment / strides");
  if (n_rows == 0) return SMER_OK;
  if (head_stride <= 0) head_stride = D;
  DecQ dq{y, ldy, gamma, beta, eps, wq, ldw, bq, x_out, ldx, dmodel};
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(H, n_rows, 8);
  hipLaunchKernelGGL((attn_decode_vec_kernel<float, 16, 2, 4, true, 512, 8>), grid, dim3(256), 0, s,
                     (const float*)nullptr, 0L, (const float*)kcache, (const float*)vcache, row_stride, req_stride,
                     head_stride, row_req, row_nkeys, (float*)nullptr, 0L, scale, dq, 0, part);
  SMER_CHECK_LAUNCH("smer_attn_decode_split_qln_f32");
  return SMER_OK;
}

extern "C" int smer_attn_decode_qln(int n_rows, int H, int D, const void* y, long ldy,
                                    const float* gamma, const float* beta, float eps, const void* wq,
                                    long ldw, const float* bq, void* x_out, long ldx, int dmodel,
                                    const void* kcache, const void* vcache, long row_stride,
                                    long req_stride, long head_stride, const int32_t* row_req,
                                    const int32_t* row_nkeys, void* o, long ldo, float scale,
                                    smer_stream_t stream) {
  SMER_REQUIRE(D == 64 && H > 0, "smer_attn_decode_qln: head dim 64");
  SMER_REQUIRE(dmodel == 512 || dmodel == 768 || dmodel == 1024,
               "smer_attn_decode_qln: d_model 512 / 768 / 1024 (else: Linear + smer_attn_decode)");
  SMER_REQUIRE(y && gamma && beta && wq && bq && kcache && vcache && o && row_req && row_nkeys,
               "smer_attn_decode_qln: null pointer");
  auto al = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
  SMER_REQUIRE(al(y) && al(wq) && al(kcache) && al(vcache) && al(o) && (!x_out || al(x_out)) &&
                   ldy % 8 == 0 && ldw % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && row_stride % 8 == 0 &&
                   req_stride % 8 == 0 && head_stride % 8 == 0,
               "smer_attn_decode_qln: 16-B alignment / strides");
  if (n_rows == 0) return SMER_OK;
  if (head_stride <= 0) head_stride = D;
  DecQ dq{y, ldy, gamma, beta, eps, wq, ldw, bq, x_out, ldx, dmodel};
  const int odd = smer_dec_odd_first();
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(H, n_rows);
  // long memories (>= 2048 key rows of capacity): next key step's loads
  // issued before the current step's math, as smer_attn_decode
  const long cap_rows = head_stride != D ? head_stride / (row_stride > 0 ? row_stride : 1)
                                         : req_stride / (row_stride > 0 ? row_stride : 1);
  const bool pipe = cap_rows >= 2048;
#define SMER_DEC_QLN(P, DM)                                                                        \
  hipLaunchKernelGGL((attn_decode_vec_kernel<bf16, 8, 4, 8, P, DM>), grid, dim3(512), 0, s,        \
                     (const bf16*)nullptr, 0L, (const bf16*)kcache, (const bf16*)vcache, row_stride, \
                     req_stride, head_stride, row_req, row_nkeys, (bf16*)o, ldo, scale, dq, odd)
  if (pipe) {
    if (dmodel == 512) SMER_DEC_QLN(true, 512);
    else if (dmodel == 768) SMER_DEC_QLN(true, 768);
    else SMER_DEC_QLN(true, 1024);
  } else {
    if (dmodel == 512) SMER_DEC_QLN(false, 512);
    else if (dmodel == 768) SMER_DEC_QLN(false, 768);
    else SMER_DEC_QLN(false, 1024);
  }
#undef SMER_DEC_QLN
  SMER_CHECK_LAUNCH("smer_attn_decode_qln");
  return SMER_OK;
}

extern "C" int smer_attn_decode(int dtype, int n_rows, int H, int D, const void* q, long ldq,
                                const void* kcache, const void* vcache, long row_stride,
                                long req_stride, long head_stride, const int32_t* row_req,
                                const int32_t* row_nkeys, void* o, long ldo, float scale,
                                smer_stream_t stream) {
  SMER_REQUIRE(D <= 256, "smer_attn_decode: head dim <= 256");
  if (n_rows == 0) return SMER_OK;
  if (head_stride <= 0) head_stride = D;  // heads side by side within a key row
  {
    // vectorised path: 16-B aligned rows, LPK = D / (16 / elem) in {4, 8, 16}
    const int es = dtype == SMER_BF16 ? 2 : 4, vec = 16 / es;
    auto al = [](const void* p) { return (((uintptr_t)p) & 15) == 0; };
    const bool ok = (dtype == SMER_BF16 || dtype == SMER_F32) && D % vec == 0 && al(q) &&
                    al(kcache) && al(vcache) && al(o) && ldq % vec == 0 && ldo % vec == 0 &&
                    row_stride % vec == 0 && req_stride % vec == 0 && head_stride % vec == 0;
    const int lpk = D / vec;
    hipStream_t s = (hipStream_t)stream;
    dim3 grid(H, n_rows);  // the H blocks of a row read the same K/V rows together
    // key capacity of a request (cache rows): long memories get 8 waves x
    // 4 steps of loads in flight per block, short self-attention caches 4 x 2
    const long cap_rows = head_stride != D ? head_stride / (row_stride > 0 ? row_stride : 1)
                                           : req_stride / (row_stride > 0 ? row_stride : 1);
    // pipelined loads also for few blocks (the batch-1 plugin step: 16
    // blocks stream a ~1k-key memory each); the same arithmetic as the
    // unpipelined 8-wave form, so the logits do not depend on the batch
    const bool big = cap_rows >= 512;
    const bool pipe = cap_rows >= 2048 || (big && (long)n_rows * H <= 128 && smer_dec_pipe_small());
    const int odd = smer_dec_odd_first();
#define SMER_DEC_VEC(T, L)                                                                        \
  if (pipe)                                                                                       \
    hipLaunchKernelGGL((attn_decode_vec_kernel<T, L, 4, 8, true>), grid, dim3(512), 0, s,         \
                       (const T*)q, ldq, (const T*)kcache, (const T*)vcache, row_stride,          \
                       req_stride, head_stride, row_req, row_nkeys, (T*)o, ldo, scale, DecQ{}, odd); \
  else if (big)                                                                                   \
    hipLaunchKernelGGL((attn_decode_vec_kernel<T, L, 4, 8>), grid, dim3(512), 0, s, (const T*)q,  \
                       ldq, (const T*)kcache, (const T*)vcache, row_stride, req_stride,            \
                       head_stride, row_req, row_nkeys, (T*)o, ldo, scale, DecQ{}, odd);          \
  else                                                                                            \
    hipLaunchKernelGGL((attn_decode_vec_kernel<T, L, 2, 4>), grid, dim3(256), 0, s, (const T*)q,  \
                       ldq, (const T*)kcache, (const T*)vcache, row_stride, req_stride,            \
                       head_stride, row_req, row_nkeys, (T*)o, ldo, scale, DecQ{}, odd)
    if (ok && (lpk == 4 || lpk == 8 || lpk == 16)) {
      if (dtype == SMER_BF16) {
        if (lpk == 4) SMER_DEC_VEC(bf16, 4); else if (lpk == 8) SMER_DEC_VEC(bf16, 8); else SMER_DEC_VEC(bf16, 16);
      } else {
        if (lpk == 4) SMER_DEC_VEC(float, 4); else if (lpk == 8) SMER_DEC_VEC(float, 8); else SMER_DEC_VEC(float, 16);
      }
#undef SMER_DEC_VEC
      SMER_CHECK_LAUNCH("smer_attn_decode");
      return SMER_OK;
    }
  }
  // key capacity bounded by req_stride / row_stride rows
  long cap = (head_stride != D ? head_stride : req_stride) / (row_stride > 0 ? row_stride : 1);
  SMER_REQUIRE(cap > 0 && cap * 4 <= 150 * 1024, "smer_attn_decode: cache capacity too large");
  hipStream_t s = (hipStream_t)stream;
  size_t shm = (size_t)cap * sizeof(float);
  dim3 grid(n_rows, H);
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(attn_decode_kernel<bf16>, grid, dim3(256), shm, s, H, D, (const bf16*)q, ldq,
                       (const bf16*)kcache, (const bf16*)vcache, row_stride, req_stride,
                       head_stride, row_req, row_nkeys, (bf16*)o, ldo, scale);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(attn_decode_kernel<float>, grid, dim3(256), shm, s, H, D, (const float*)q,
                       ldq, (const float*)kcache, (const float*)vcache, row_stride, req_stride,
                       head_stride, row_req, row_nkeys, (float*)o, ldo, scale);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_attn_decode: dtype");
  SMER_CHECK_LAUNCH("smer_attn_decode");
  return SMER_OK;
}

extern "C" int smer_kv_scatter(int dtype, int n_rows, int width, const void* src, long lds,
                               void* cache, long row_stride, long req_stride,
                               const int32_t* row_req, const int32_t* row_pos,
                               smer_stream_t stream) {
  long tot = (long)n_rows * width;
  if (tot == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(kv_scatter_kernel<bf16>, dim3((tot + 255) / 256), dim3(256), 0, s, n_rows,
                       width, (const bf16*)src, lds, (bf16*)cache, row_stride, req_stride, row_req,
                       row_pos);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(kv_scatter_kernel<float>, dim3((tot + 255) / 256), dim3(256), 0, s, n_rows,
                       width, (const float*)src, lds, (float*)cache, row_stride, req_stride,
                       row_req, row_pos);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_kv_scatter: dtype");
  SMER_CHECK_LAUNCH("smer_kv_scatter");
  return SMER_OK;
}

extern "C" int smer_kv_scatter_heads(int dtype, int n_rows, int H, int D, const void* src, long lds,
                                     void* cache, long req_stride, long kv_stride,
                                     long head_stride, const int32_t* row_req,
                                     const int32_t* row_pos, smer_stream_t stream) {
  const int es = dtype == SMER_BF16 ? 2 : 4, vec = 16 / es;
  SMER_REQUIRE(dtype == SMER_BF16 || dtype == SMER_F32, "smer_kv_scatter_heads: dtype");
  SMER_REQUIRE(n_rows >= 0 && H > 0 && D % vec == 0 && lds % vec == 0 && req_stride % vec == 0 &&
                   kv_stride % vec == 0 && head_stride % vec == 0 && al16(src) && al16(cache),
               "smer_kv_scatter_heads: 16-B vector layout required");
  const long tot = (long)n_rows * (2 * H * D / vec);
  if (tot == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((tot + 255) / 256));
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(kv_scatter_heads_kernel<bf16>, grid, dim3(256), 0, s, n_rows, H, D,
                       (const bf16*)src, lds, (bf16*)cache, req_stride, kv_stride, head_stride,
                       row_req, row_pos);
  else
    hipLaunchKernelGGL(kv_scatter_heads_kernel<float>, grid, dim3(256), 0, s, n_rows, H, D,
                       (const float*)src, lds, (float*)cache, req_stride, kv_stride, head_stride,
                       row_req, row_pos);
  SMER_CHECK_LAUNCH("smer_kv_scatter_heads");
  return SMER_OK;
}
