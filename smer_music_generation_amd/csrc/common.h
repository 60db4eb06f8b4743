// Shared device helpers for the SMER gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/smer_hip.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define SMER_WAVE 64

// status reporting (defined in abi.cpp)
extern "C" int smer_set_error(int code, const char* msg);
#define SMER_CHECK_LAUNCH(what)                                          \
  do {                                                                   \
    hipError_t _e = hipGetLastError();                                   \
    if (_e != hipSuccess) return smer_set_error(SMER_ERR_HIP, hipGetErrorString(_e)); \
  } while (0)
#define SMER_REQUIRE(cond, msg) \
  do { if (!(cond)) return smer_set_error(SMER_ERR_INVALID, msg); } while (0)

template <typename T> __device__ __forceinline__ float to_f32(T x);
template <> __device__ __forceinline__ float to_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ float to_f32<bf16>(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// Raw v_exp_f32 (2^x; -inf -> 0, no denormal range fix-up): the softmax
// exponents are <= 0 so the fix-up libm's exp2f adds is dead weight.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Wave-wide all-reduce without LDS round trips: DPP butterflies inside each
// 16-lane row (quad_perm xor 1 / xor 2, half-mirror, mirror), then the row
// and half exchanges of v_permlane16/32_swap.  Every lane adds the same
// pairs (commutative), so all 64 lanes hold bit-identical totals.
__device__ __forceinline__ float dpp_f(float v, int ctrl) {
  switch (ctrl) {  // the control must be an immediate
    case 0xB1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
    case 0x4E: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
    case 0x141: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  }
}
template <typename OP>
__device__ __forceinline__ float wave_reduce(float v, OP op) {
  v = op(v, dpp_f(v, 0xB1));   // lane ^ 1
  v = op(v, dpp_f(v, 0x4E));   // lane ^ 2
  v = op(v, dpp_f(v, 0x141));  // 7 - lane within 8
  v = op(v, dpp_f(v, 0x140));  // 15 - lane within 16
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = op(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return op(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float wave_sum(float v) {
  return wave_reduce(v, [](float x, float y) { return x + y; });
}
__device__ __forceinline__ float wave_max(float v) {
  return wave_reduce(v, [](float x, float y) { return fmaxf(x, y); });
}

// Dropout (every site: activations, attention probabilities, LN / embedding
// gradients).  Counter-based: one 32-bit hash per (row, column pair) feeds
// 16 bits to each of the two columns; keep iff bits >= thr16 =
// round(p * 65536); survivors are scaled by 65536 / (65536 - thr16), exactly
// unbiased for the realised rate.  The per-row key is hashed once per row,
// so a column costs half a hash (2 multiplies per pair).  numpy mirror:
// tests/hashref.py keep_mask.
__device__ __forceinline__ uint32_t smer_mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t smer_rowkey(uint32_t seed, uint32_t row) {
  return smer_mix32(smer_mix32(row ^ 0x85EBCA6Bu) ^ seed);
}
__device__ __forceinline__ uint32_t smer_pair_bits(uint32_t rowkey, uint32_t pair) {
  return smer_mix32(rowkey + pair * 0x9E3779B9u);
}
__device__ __forceinline__ bool smer_keep16(uint32_t rowkey, uint32_t thr16, uint32_t col) {
  const uint32_t h = smer_pair_bits(rowkey, col >> 1);
  return ((col & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thr16;
}
// 8 consecutive columns starting at an even col0: v[i] = keep ? v[i] * ds : 0
__device__ __forceinline__ void smer_drop8(uint32_t rowkey, uint32_t thr16, float ds, uint32_t col0,
                                           float (&v)[8]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t h = smer_pair_bits(rowkey, (col0 >> 1) + k);
    v[2 * k] = (h & 0xFFFFu) >= thr16 ? v[2 * k] * ds : 0.f;
    v[2 * k + 1] = (h >> 16) >= thr16 ? v[2 * k + 1] * ds : 0.f;
  }
}
static inline uint32_t smer_drop_thr16(float p) {
  if (p <= 0.f) return 0u;
  long t = (long)((double)p * 65536.0 + 0.5);
  return (uint32_t)(t < 1 ? 1 : (t > 65535 ? 65535 : t));
}
static inline float smer_drop_scale16(uint32_t thr16) {
  return thr16 ? (float)(65536.0 / (65536.0 - (double)thr16)) : 1.f;
}

// Attention-probability dropout: the flash forward spends its VALU budget on
// the softmax, so this site uses 7-bit keep thresholds (FlashAttention's
// uint8 dropout quantises p the same way) and a cheaper mixer.  One 32-bit
// hash per (query row, quad of 4 consecutive keys); the low 7 bits of byte r
// decide key 4*quad + r, kept when they are >= thr7 = round(p * 128)
// (realised rate thr7 / 128, survivors scaled by 128 / (128 - thr7):
// unbiased for that rate).  The mixer multiplies with the full-rate 24-bit
// multiplier (v_mul_u32_u24; the xor-shifts fold the high bits down first).
// numpy mirror: tests/hashref.py attn_keep_mask.
__device__ __forceinline__ uint32_t smer_attn_bits(uint32_t rowkey, uint32_t quad) {
  uint32_t h = rowkey + quad * 0x9E3779B9u;
  h ^= h >> 16;
  h = __umul24(h, 0xEB352Du);
  h ^= h >> 15;
  h = __umul24(h, 0x6CA68Bu);
  h ^= h >> 16;
  return h;
}
// The four byte decisions of one hash at once (SWAR): bit 8r + 7 of the
// result is set iff (byte r & 127) >= thr7; lo4 = thr7 * 0x01010101.  Every
// minuend byte is >= 128 > thr7, so no borrow crosses a byte; the other
// bits of the result are don't-care.
__device__ __forceinline__ uint32_t smer_attn_ge(uint32_t h, uint32_t lo4) {
  return (h | 0x80808080u) - lo4;
}
__device__ __forceinline__ bool smer_attn_keep(uint32_t rowkey, uint32_t thr7, uint32_t key) {
  return ((smer_attn_bits(rowkey, key >> 2) >> (8 * (key & 3))) & 0x7Fu) >= thr7;
}
static inline uint32_t smer_attn_thr7(float p) {
  if (p <= 0.f) return 0u;
  long t = (long)((double)p * 128.0 + 0.5);
  return (uint32_t)(t < 1 ? 1 : (t > 127 ? 127 : t));
}
static inline float smer_attn_scale7(uint32_t thr7) {
  return thr7 ? (float)(128.0 / (128.0 - (double)thr7)) : 1.f;
}

// out[col] (+)= scale * sum_b part[b*stride + off + col], b in fixed order
// (deterministic; two levels when nblk > 64, `scratch` of
// smer_col_reduce_scratch(nblk, N) bytes).  Defined in train_ops.hip.
size_t smer_col_reduce_scratch(int nblk, int N);
// Columns >= nsplit of the reduced row go to out2[col - nsplit] (out2 may be
// null: everything to out).
void smer_col_reduce_launch(int nblk, int N, const float* part, long stride, long off, float* out,
                            int accumulate, float scale, float* scratch, hipStream_t s,
                            float* out2 = nullptr, int nsplit = 0);

// Load 8 consecutive elements as floats (16-B vector when aligned & in range).
template <typename T, bool VEC = true>
__device__ __forceinline__ void load8(const T* p, int valid, float (&v)[8]) {
  if (VEC && valid >= 8) {
    if constexpr (sizeof(T) == 2) {
      bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
    } else {
      float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = i < valid ? (float)p[i] : 0.f;
  }
}

// LayerNorm of one row by one wave (lane c holds the 16-B chunks c, c+64, ..
// of the row, N <= 2048): the statistics and the normalised value, shared by
// ln_fwd_kernel and the decode Linear's LayerNorm prologue so that both
// produce the same bits.
constexpr int LNR_MAXC = 4;
// the statistics of a row already in v (chunks ch >= N / 8 ignored)
template <int NC = LNR_MAXC>
__device__ __forceinline__ void ln_stats_loaded(const float (&v)[NC][8], int N, float eps, int lane, float& mu,
                                                float& rs) {
  const int nch = N >> 3;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (lane + 64 * c < nch)
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
  mu = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (lane + 64 * c < nch)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mu;
        q += d * d;
      }
  rs = rsqrtf(wave_sum(q) / N + eps);
}
template <typename T, int NC = LNR_MAXC>
__device__ __forceinline__ void ln_row_stats(const T* __restrict__ xr, int N, float eps, int lane,
                                             float (&v)[NC][8], float& mu, float& rs) {
  const int nch = N >> 3;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      load8<T>(xr + ch * 8, 8, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
  }
  mu = wave_sum(s) / N;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (lane + 64 * c < nch)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mu;
        q += d * d;
      }
  rs = rsqrtf(wave_sum(q) / N + eps);
}
__device__ __forceinline__ float ln_apply(float v, float mu, float rs, float g, float b) {
  return __builtin_fmaf((v - mu) * rs, g, b);
}

// XCD-aware 2-D block index: blocks b and b+8 share an XCD (round-robin
// dispatch), so give each XCD a contiguous run of the row-major work list;
// x-neighbours (e.g. the query blocks of one (batch, head)) then share an L2.
// Bijective for any grid size.  Speed only, never correctness.
__device__ __forceinline__ void xcd_block2d(int& bx, int& by) {
  const int nx = gridDim.x, n = gridDim.x * gridDim.y;
  const int b = blockIdx.y * nx + blockIdx.x;
  const int xcd = b & 7, q = n >> 3, r = n & 7;
  const int lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  bx = lin % nx;
  by = lin / nx;
}

__device__ __forceinline__ bf16x8 lds_read_b128(const char* base, uint32_t byte_off) {
  return *reinterpret_cast<const bf16x8*>(base + byte_off);
}
// gfx950 ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q,
// columns 4p..4p+3 of a 4x16 block; lane i receives column i (rows 0..3).
__device__ __forceinline__ bf16x4 lds_read_tr16(const char* base, uint32_t byte_off) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  i16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + byte_off));
  return __builtin_bit_cast(bf16x4, r);
}
// The same read as an asm statement, for k-loops whose next stage is in
// flight by LDS-DMA (global_load_lds): hipcc cannot tell the intrinsic's LDS
// read from the DMA's destination and waits vmcnt(0) before the first one of
// every k-step (measured in the .s of every GEMM with a column-image
// operand), so a stage's load never overlapped the MFMAs of the stage before.
// The asm form is invisible to that bookkeeping AND to the lgkmcnt waits: the
// caller retires the reads with lds_tr_retire() before using the registers.
__device__ __forceinline__ bf16x4 lds_read_tr16_async(const char* base, uint32_t byte_off) {
  typedef __attribute__((address_space(3))) const char lds_char;
  const uint32_t a = (uint32_t)(uintptr_t)((lds_char*)(base + byte_off));
  i16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return __builtin_bit_cast(bf16x4, r);
}
__device__ __forceinline__ uint4 lds_read_b128_async(const char* base, uint32_t byte_off) {
  typedef __attribute__((address_space(3))) const char lds_char;
  const uint32_t a = (uint32_t)(uintptr_t)((lds_char*)(base + byte_off));
  uint4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// s_waitcnt lgkmcnt(n) for a compile-time n (asm immediates cannot come
// from an unrolled loop variable)
template <int N>
__device__ __forceinline__ void lds_wait() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt is 4 bits");
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  else if constexpr (N == 15) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
  else static_assert(N == 0 || N == 2 || N == 4 || N == 6 || N == 8 || N == 15, "add the count");
}
// Retire only the asm reads of one fragment set, issued before CNT younger
// (compiler-visible) LDS reads whose waits hipcc places itself.
template <int CNT, int NB>
__device__ __forceinline__ void lds_tr_retire_older(bf16x8 (&b)[NB]) {
  lds_wait<CNT>();
#pragma unroll
  for (int i = 0; i < NB; ++i) asm volatile("" : "+v"(b[i]));
}
// lgkmcnt(0), then every fragment register passes through an empty asm that
// the MFMAs depend on, so none of them is scheduled above the wait.
// CNT > 0: only the reads older than the CNT youngest (LDS returns in order).
template <int CNT = 0, int NA, int NB>
__device__ __forceinline__ void lds_tr_retire(bf16x8 (&a)[NA], bf16x8 (&b)[NB]) {
  lds_wait<CNT>();
#pragma unroll
  for (int i = 0; i < NA; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int i = 0; i < NB; ++i) asm volatile("" : "+v"(b[i]));
}
__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---- fp8 (OCP e4m3) activations with delayed per-tensor scaling ----------
// A producer (LayerNorm, the FFN1 epilogue) writes q = e4m3(v * qs) next to
// its bf16 output, where qs = 448 / amax of the previous step (1 when none),
// and folds max|v| into this step's amax.  Consumers dequantise with
// inv = 1 / qs.  amax is kept as float bits (non-negative floats order like
// unsigned ints, so integer atomicMax is exact and arrival-order free).
//
// v_cvt_pk_fp8_f32 is exact nearest-even on any f32 (tools/probes/
// cvt_fp8_probe.hip: 1.08 M values around every e4m3 midpoint, 0 mismatches
// against a software nearest-even), so the cast is the whole rounding.
// Workgroup barrier that settles only LDS traffic (lgkmcnt(0), vmcnt /
// expcnt left at their maxima): GEMM epilogue passes reuse an LDS staging
// tile, so the next pass needs the LDS writes / reads of the last one done,
// not its global stores (__syncthreads waits vmcnt(0): every pass would pay
// the store round trip).  The asm memory clobbers keep the compiler from
// moving memory operations across it.
// s_waitcnt vmcnt(0) as a real instruction (hipcc's wait insertion counts
// it, unlike an asm one).  Before a k-loop whose prologue loads were issued on
// a path the compiler cannot prove the loop is entered from, its static merge
// otherwise leaves those registers "pending" at the loop head and re-waits
// them inside EVERY iteration -- where the wait also drains the prefetch of
// the next tile.
__device__ __forceinline__ void smer_vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }
__device__ __forceinline__ void smer_lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Correctly rounded f32 quotient for the scales (448 / amax and back): via
// f64 the double rounding is exact for a quotient of f32 operands, whatever
// the f32 '/' lowering; the scale enters every product before the cast.
__device__ __forceinline__ float smer_div_rn(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ uint2 smer_q8x8(const float (&v)[8], float qs) {
  uint32_t w[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // saturate finite values to +-448; NaN passes through to the cast
      // (fmaxf would turn it into -448: a diverged activation must stay NaN)
      const float x = v[4 * h + k] * qs;
      f[k] = x == x ? fminf(fmaxf(x, -448.f), 448.f) : x;
    }
    int p = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    p = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], p, true);
    w[h] = (uint32_t)p;
  }
  return make_uint2(w[0], w[1]);
}
// 4 values -> 4 e4m3 bytes (little-endian in one word), as smer_q8x8
__device__ __forceinline__ uint32_t smer_q8x4(const float (&v)[4], float qs) {
  float f[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x = v[k] * qs;
    f[k] = x == x ? fminf(fmaxf(x, -448.f), 448.f) : x;
  }
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  p = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], p, true);
  return (uint32_t)p;
}
__device__ __forceinline__ float smer_absmax4(const float (&v)[4]) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) m = fmaxf(m, v[k] == v[k] ? fabsf(v[k]) : __builtin_inff());
  return m;
}
__device__ __forceinline__ float smer_absmax8(const float (&v)[8]) {
  // NaN maps to +inf (fmaxf would drop it): the amax slot then reports the
  // non-finite activation (Fp8Forward.finite) and the next scale falls back to 1
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) m = fmaxf(m, v[k] == v[k] ? fabsf(v[k]) : __builtin_inff());
  return m;
}
// wave-wide max, then at most one atomic per wave (every lane must call).
// amax only grows, so a wave whose max does not exceed the value it reads
// skips the atomic (a stale read only costs an extra atomic): the producers
// of one tensor (tens of thousands of waves) would otherwise serialise on
// one address.
__device__ __forceinline__ void smer_amax_commit(unsigned* amax, float m) {
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) {
    const unsigned b = __float_as_uint(m);
    if (b > __hip_atomic_load(amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(amax, b);
  }
}

