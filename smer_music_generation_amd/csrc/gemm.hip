// GEMM for every projection of the SMER Transformer (QKV in-proj, out-proj,
// FFN, vocab head) and their dgrad / wgrad.
//
// bf16 path: 128x128x64 block tile, 4 waves (2x2, 64x64 each),
// mfma_f32_16x16x32_bf16, register-staged double-buffered LDS (issue the
// next tile's global loads before the MFMAs, write LDS after them).
// Either operand may be K-contiguous ("row" image, XOR-swizzled 16-B chunks,
// ds_read_b128 fragments) or M/N-contiguous ("column" image, 8-B units
// XOR-swizzled, ds_read_b64_tr_b16 transposing fragments) — so forward (NT),
// dgrad (NN) and wgrad (TN) all run without an explicit transpose pass.
// f32 path (parity mode): LDS-tiled VALU FMA, same epilogue.
#include "common.h"

#include <algorithm>
#include <cstdlib>

struct GemmEpi {
  const float* bias;
  float alpha;
  int relu;
  const void* residual;
  long ldr;
  const void* gate;
  long ldg;
  float gate_scale;
  uint32_t drop_thr;
  uint32_t seed;
  float drop_scale;
  void* C;
  long ldc;
  float* Cf;
  long ldcf;
  int accumulate;
  int vec;  // every operand 16-B aligned with row strides % 8 == 0
  int rs_accumulate;  // fused row-sum output (bias gradient) accumulates
  // decode: columns >= kv_col0 are also appended to a per-request K/V cache
  // at kv[kv_req[row] * kv_req_stride + kv_pos[row] * kv_row_stride + col - kv_col0]
  void* kv;
  long kv_row_stride, kv_req_stride;
  const int32_t* kv_req;
  const int32_t* kv_pos;
  int kv_col0;
  // fp8 copy of the bf16 output (delayed scaling, common.h): q8 = e4m3(out *
  // *q8_scale); the caller folds max|out| into *q8_amax (vector path only)
  uint8_t* q8;
  long ldq8;
  const float* q8_scale;
  unsigned* q8_amax;
  // diagnostics (smer_gemm_debug_stamps): per-wave s_memtime phase stamps
  unsigned long long* dbg;
  // start skew of the persistent 256x256 forward / dgrad kernels (A/B probe,
  // SMER_G256_SKEW): every second workgroup of an XCD sleeps skew x ~2k
  // cycles before its first tile, so the all-CU epilogue store bursts of the
  // two halves no longer coincide
  int skew;
};
__device__ __forceinline__ void g2_start_skew(int skew) {
  if (skew > 0 && ((blockIdx.x >> 3) & 1))
    for (int i = 0; i < skew; ++i) __builtin_amdgcn_s_sleep(32);
}

template <typename T>
__device__ __forceinline__ void epi_apply(const GemmEpi& e, int M, int N, int row, int col,
                                          float acc) {
  if (row >= M || col >= N) return;
  float v = acc * e.alpha;
  if (e.bias) v += e.bias[col];
  if (e.relu) v = fmaxf(v, 0.f);
  if (e.drop_thr) v = smer_keep16(smer_rowkey(e.seed, (uint32_t)row), e.drop_thr, (uint32_t)col) ? v * e.drop_scale : 0.f;
  if (e.residual) v += to_f32(((const T*)e.residual)[(long)row * e.ldr + col]);
  if (e.gate) {
    float gv = to_f32(((const T*)e.gate)[(long)row * e.ldg + col]);
    v = gv > 0.f ? v * e.gate_scale : 0.f;
  }
  if (e.C) ((T*)e.C)[(long)row * e.ldc + col] = from_f32<T>(v);
  if (e.Cf) {
    float* p = e.Cf + (long)row * e.ldcf + col;
    *p = e.accumulate ? *p + v : v;
  }
  if (e.kv && col >= e.kv_col0)
    ((T*)e.kv)[(long)e.kv_req[row] * e.kv_req_stride + (long)e.kv_pos[row] * e.kv_row_stride +
               (col - e.kv_col0)] = from_f32<T>(v);
}

// Eight consecutive columns of one row (bf16 activations).  Vector path when
// the host verified 16-B alignment of every operand (e.vec) and the chunk is
// full; otherwise per element.  amax_acc: running max|out| of the fp8 copy.
__device__ __forceinline__ void epi_apply8(const GemmEpi& e, int M, int N, int row, int col,
                                           float (&v)[8], float* amax_acc = nullptr) {
  const int valid = min(8, N - col);
  if (!e.vec || valid < 8) {
    for (int k = 0; k < valid; ++k) epi_apply<bf16>(e, M, N, row, col + k, v[k]);
    return;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] *= e.alpha;
  if (e.bias) {
    const float4 b0 = *reinterpret_cast<const float4*>(e.bias + col);
    const float4 b1 = *reinterpret_cast<const float4*>(e.bias + col + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  }
  if (e.relu) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  if (e.drop_thr) smer_drop8(smer_rowkey(e.seed, (uint32_t)row), e.drop_thr, e.drop_scale, (uint32_t)col, v);
  if (e.residual) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>((const bf16*)e.residual + (long)row * e.ldr + col);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += (float)r[k];
  }
  if (e.gate) {
    const bf16x8 gt = *reinterpret_cast<const bf16x8*>((const bf16*)e.gate + (long)row * e.ldg + col);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (float)gt[k] > 0.f ? v[k] * e.gate_scale : 0.f;
  }
  if (e.C || e.kv) {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
    if (e.C) *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)row * e.ldc + col) = o;
    if (e.q8 && amax_acc) {  // fp8 copy of the stored bf16 values
      float r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = (float)o[k];
      *reinterpret_cast<uint2*>(e.q8 + (long)row * e.ldq8 + col) = smer_q8x8(r, *e.q8_scale);
      *amax_acc = fmaxf(*amax_acc, smer_absmax8(r));
    }
    if (e.kv && col >= e.kv_col0)  // kv_col0 % 8 == 0: a chunk is all K/V or all Q
      *reinterpret_cast<bf16x8*>((bf16*)e.kv + (long)e.kv_req[row] * e.kv_req_stride +
                                 (long)e.kv_pos[row] * e.kv_row_stride + (col - e.kv_col0)) = o;
  }
  if (e.Cf) {
    float* p = e.Cf + (long)row * e.ldcf + col;
    float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
    if (e.accumulate) {
      const float4 a0 = *reinterpret_cast<const float4*>(p);
      const float4 a1 = *reinterpret_cast<const float4*>(p + 4);
      o0.x += a0.x; o0.y += a0.y; o0.z += a0.z; o0.w += a0.w;
      o1.x += a1.x; o1.y += a1.y; o1.z += a1.z; o1.w += a1.w;
    }
    *reinterpret_cast<float4*>(p) = o0;
    *reinterpret_cast<float4*>(p + 4) = o1;
  }
}

// ---------------------------------------------------------------------------
// bf16 MFMA kernel
// ---------------------------------------------------------------------------
namespace {
constexpr int GBM = 128, GBN = 128, GBK = 64;
constexpr int TILE_BYTES = GBM * GBK * 2;  // 16 KiB per operand per buffer

__device__ __forceinline__ uint32_t col_swz(int k) {  // 3-bit row signature
  return (uint32_t)((k & 3) | (((k >> 3) & 1) << 2));
}

// Stage one operand tile (rows r0.., k0..) into registers.
// KC: operand stored [rows][K]; else stored [K][rows].
template <bool KC>
__device__ __forceinline__ void stage_load(uint4 (&r)[4], const bf16* P, long ld, int rows,
                                           int K, int r0, int k0, int tid) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int i = tid + 256 * c;
    int gr, gk;
    if (KC) { gr = r0 + (i >> 3); gk = k0 + (i & 7) * 8; }
    else    { gk = k0 + (i >> 4); gr = r0 + (i & 15) * 8; }
    bool ok = gr < rows && gk < K;
    const bf16* src = KC ? P + (long)gr * ld + gk : P + (long)gk * ld + gr;
    r[c] = ok ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
  }
}

template <bool KC>
__device__ __forceinline__ void stage_store(const uint4 (&r)[4], char* buf, int tid) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int i = tid + 256 * c;
    uint32_t off;
    if (KC) {
      int row = i >> 3, ch = i & 7;
      off = row * 128 + ((ch ^ (row & 7)) << 4);
    } else {
      int k = i >> 4, ch = i & 15;
      off = k * 256 + ((ch ^ (2 * col_swz(k))) << 4);
    }
    *reinterpret_cast<uint4*>(buf + off) = r[c];
  }
}

// LDS-DMA staging (global_load_lds_dwordx4): each wave instruction writes
// 1 KiB of the LDS image lane-linearly, so the XOR swizzle of the image is
// applied to the per-lane SOURCE address instead (lane i fills physical
// chunk i and fetches the logical chunk that belongs there).  No VGPR round
// trip and no ds_write.  Rows past `rows` are clamped (their products only
// reach discarded outputs); the caller guarantees the K range is full.
template <bool KC>
__device__ __forceinline__ void stage_glds(char* buf, const bf16* P, long ld, int rows,
                                           int r0, int k0, int tid) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int chunk = wave * 4 + c;  // 16 x 1 KiB per 16 KiB operand tile
    const bf16* src;
    if (KC) {
      const int row = chunk * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (row & 7);
      src = P + (long)min(r0 + row, rows - 1) * ld + k0 + lc * 8;
    } else {
      const int k = chunk * 4 + (lane >> 4);
      const int lc = (lane & 15) ^ (2 * (int)col_swz(k));
      const int col = min(r0 + lc * 8, ((rows + 7) & ~7) - 8);
      src = P + (long)(k0 + k) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(buf + chunk * 1024), 16, 0, 0);
  }
}

// Fragment (16 rows starting at rbase, k-step s) for lane l.
template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* buf, int rbase, int s, int lane) {
  int g = lane >> 4, c16 = lane & 15;
  if (KC) {
    int row = rbase + c16;
    int ch = s * 4 + g;
    return lds_read_b128(buf, row * 128 + ((ch ^ (row & 7)) << 4));
  } else {
    int q = c16 >> 2, p = c16 & 3;
    int u = (rbase >> 2) + p;
    int k0 = s * 32 + 8 * g + q;
    int k1 = k0 + 4;
    bf16x4 lo = lds_read_tr16_async(buf, k0 * 256 + ((u ^ (4 * col_swz(k0))) << 3));
    bf16x4 hi = lds_read_tr16_async(buf, k1 * 256 + ((u ^ (4 * col_swz(k1))) << 3));
    return cat4(lo, hi);
  }
}
}  // namespace

// Split-K hand-off for the fused (last-arriver) reduction: every slab /
// row-sum partial byte is stored write-through (`sc1`) and read back with
// `sc1` loads, each storing wave waits vmcnt(0), a workgroup barrier, then
// ONE lane adds to the tile's ticket (agent-scope atomic); the workgroup
// whose add returns ksplit - 1 sums the slices.  This is the first row of
// the hand-off table in MI355X_MICROARCH.md (Valid forms): no release /
// acquire fences needed.  The ticket is reset by the last arriver, so the
// ticket words stay zero between launches.
__device__ __forceinline__ void st_sc1_x4(float* p, float a, float b, float c, float d) {
  const f32x4 v = {a, b, c, d};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ f32x4 ld_sc1_x4(const float* p) {
  f32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void ld_sc1_retire(f32x4 (&b)[N]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(b[i]));
}

// The last arriver's reduction of one 128x128 tile: Cf (+)= alpha * sum of
// the ksplit slabs in slice order (the splitk_reduce_kernel arithmetic), and
// for tn == 0 tiles the bias row sums (+)= alpha * sum of the partials.
// Needs N % 4 == 0, ldcf % 4 == 0 and a 16-B aligned Cf (launcher checks).
__device__ __forceinline__ void splitk_tile_reduce(const GemmEpi& e, int M, int N, int m0, int n0,
                                                   int ksplit, const float* __restrict__ slabs,
                                                   const float* __restrict__ rs_part,
                                                   float* __restrict__ rs_final, bool rs_tile,
                                                   int tid) {
  const long MN = (long)M * N;
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {  // 8 float4 per thread per pass, all in flight
    f32x4 a[8], b[8];
    long off[8];
    bool ok[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int pos = tid + 256 * (half * 8 + i);
      const int row = pos >> 5, c4 = pos & 31;
      const int grow = m0 + row, gcol = n0 + c4 * 4;
      ok[i] = grow < M && gcol < N;
      off[i] = ok[i] ? (long)grow * N + gcol : 0;  // clamped: discarded below
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = ld_sc1_x4(slabs + off[i]);
    ld_sc1_retire(a);
#pragma unroll 1
    for (int sl = 1; sl < ksplit; ++sl) {
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = ld_sc1_x4(slabs + (long)sl * MN + off[i]);
      ld_sc1_retire(b);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        a[i][0] += b[i][0]; a[i][1] += b[i][1]; a[i][2] += b[i][2]; a[i][3] += b[i][3];
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (!ok[i]) continue;
      const int pos = tid + 256 * (half * 8 + i);
      const int row = pos >> 5, c4 = pos & 31;
      float* p = e.Cf + (long)(m0 + row) * e.ldcf + n0 + c4 * 4;
      float4 o = make_float4(a[i][0] * e.alpha, a[i][1] * e.alpha, a[i][2] * e.alpha, a[i][3] * e.alpha);
      if (e.accumulate) {
        const float4 c = *reinterpret_cast<const float4*>(p);
        o.x = c.x + o.x; o.y = c.y + o.y; o.z = c.z + o.z; o.w = c.w + o.w;
      }
      *reinterpret_cast<float4*>(p) = o;
    }
  }
  if (rs_tile && tid < GBM && m0 + tid < M) {
    const int m = m0 + tid;
    float t = 0.f;
    for (int sl = 0; sl < ksplit; ++sl)
      t += __hip_atomic_load(rs_part + (long)sl * M + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    rs_final[m] = (e.rs_accumulate ? rs_final[m] : 0.f) + e.alpha * t;
  }
}

// NSTG = 3 / 4 (weight gradients, LDS-DMA, one workgroup per CU): an
// NSTG-stage LDS ring, each k-step's tiles requested NSTG - 1 steps ahead and
// waited with a counted vmcnt before a raw barrier (the 2-stage form waits at the end of
// every k-step for the tiles it requested at its start: one HBM round trip
// per 64 of K against ~1 k cycles of MFMA work).  Fragment reads are asm,
// so hipcc's wait insertion does not see them.
template <bool AK, bool BKC, bool GL, int NSTG = 2>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(int M, int N, int K,
                                                           const bf16* __restrict__ A, long lda,
                                                           const bf16* __restrict__ B, long ldb,
                                                           GemmEpi e, int ksplit, int kchunk,
                                                           float* __restrict__ slabs,
                                                           float* __restrict__ rowsum,
                                                           unsigned* __restrict__ tickets = nullptr,
                                                           float* __restrict__ rs_final = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nbm = (M + GBM - 1) / GBM, nbn = (N + GBN - 1) / GBN;
  // fused split-K reduction (tickets): slabs / partials stored write-through
  const bool fused = tickets != nullptr && ksplit > 1;
  const int ntiles = nbm * nbn;
  const int nwg = ntiles * ksplit;
  // Persistent, XCD-aware work list: XCD x (blocks b with b % 8 == x) owns a
  // contiguous run of work items and its blocks stride through it; the K
  // slices of one tile are adjacent, tiles are walked in GM-row groups, so
  // blocks running together on one XCD share A / B panels in its L2.  With
  // a grid of exactly nwg blocks every block takes one item (bijective).
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 8;
  struct Item { int split, tm, tn, m0, n0, k_begin, k_end; };
  auto decode = [&](int lin) {
    Item it;
    it.split = lin / ntiles;
    const int wgid = lin % ntiles;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    it.tm = first_m + within % gsz;
    it.tn = within / gsz;
    it.m0 = it.tm * GBM;
    it.n0 = it.tn * GBN;
    it.k_begin = it.split * kchunk;
    it.k_end = min(K, it.k_begin + kchunk);
    return it;
  };
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;
  uint4 ra[4], rb[4];
  bool prefetched = false;

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const Item it = decode(xstart + jj);
    const int m0 = it.m0, n0 = it.n0, k_begin = it.k_begin, k_end = it.k_end;

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Fused bias gradient (weight-gradient GEMMs): the first column-tile's
    // blocks also form sum_k A[m][k] with one extra MFMA against a ones
    // fragment per 16 rows (the two wn waves split the 4 row fragments).
    const bool rsum = rowsum != nullptr && it.tn == 0;
    f32x4 accr[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};

    const int nk = (k_end - k_begin + GBK - 1) / GBK;
    static_assert(NSTG == 2 || ((NSTG == 3 || NSTG == 4) && GL && !AK && !BKC),
                  "3 / 4 stages: LDS-DMA weight gradients only");
    if constexpr (GL) {
      stage_glds<AK>(smem, A, lda, M, m0, k_begin, tid);
      stage_glds<BKC>(smem + TILE_BYTES, B, ldb, N, n0, k_begin, tid);
#pragma unroll
      for (int p = 1; p < NSTG - 1; ++p)
        if (NSTG > 2 && p < nk) {
          stage_glds<AK>(smem + p * 2 * TILE_BYTES, A, lda, M, m0, k_begin + p * GBK, tid);
          stage_glds<BKC>(smem + p * 2 * TILE_BYTES + TILE_BYTES, B, ldb, N, n0, k_begin + p * GBK, tid);
        }
    } else {
      if (!prefetched) {
        stage_load<AK>(ra, A, lda, M, k_end, m0, k_begin, tid);
        stage_load<BKC>(rb, B, ldb, N, k_end, n0, k_begin, tid);
      }
      stage_store<AK>(ra, smem, tid);
      stage_store<BKC>(rb, smem + TILE_BYTES, tid);
    }
    if constexpr (NSTG > 2) {  // stage 0 landed (stages 1.. may stay in flight: 8 DMAs per thread each)
      asm volatile("" ::: "memory");
      const int ahead = min(NSTG - 2, nk - 1);
      if (ahead >= 2) __builtin_amdgcn_s_waitcnt(0x4F70);       // vmcnt(16)
      else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8)
      else __builtin_amdgcn_s_waitcnt(0x0F70);                  // vmcnt(0)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }

    for (int kt = 0; kt < nk; ++kt) {
      const int cur = NSTG == 2 ? kt & 1 : kt % NSTG;
      const bool more = kt + 1 < nk;
      if constexpr (NSTG > 2) {
        if (kt + NSTG - 1 < nk) {
          char* nb = smem + ((kt + NSTG - 1) % NSTG) * 2 * TILE_BYTES;
          stage_glds<AK>(nb, A, lda, M, m0, k_begin + (kt + NSTG - 1) * GBK, tid);
          stage_glds<BKC>(nb + TILE_BYTES, B, ldb, N, n0, k_begin + (kt + NSTG - 1) * GBK, tid);
        }
      } else if constexpr (GL) {
        if (more) {
          char* nb = smem + (cur ^ 1) * 2 * TILE_BYTES;
          stage_glds<AK>(nb, A, lda, M, m0, k_begin + (kt + 1) * GBK, tid);
          stage_glds<BKC>(nb + TILE_BYTES, B, ldb, N, n0, k_begin + (kt + 1) * GBK, tid);
        }
      } else if (more) {
        stage_load<AK>(ra, A, lda, M, k_end, m0, k_begin + (kt + 1) * GBK, tid);
        stage_load<BKC>(rb, B, ldb, N, k_end, n0, k_begin + (kt + 1) * GBK, tid);
      }
      const char* a_s = smem + cur * 2 * TILE_BYTES;
      const char* b_s = a_s + TILE_BYTES;
      if constexpr (GL && !AK && !BKC) {
        // weight gradients: both k-steps' fragments requested up front (32
        // transposing reads); the second step's land under the first step's
        // MFMAs.  lgkmcnt(15) retires the first 16 (LDS returns in order).
        bf16x8 af0[4], bf0[4], af1[4], bf1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af0[i] = frag<false>(a_s, wm * 64 + i * 16, 0, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bf0[j] = frag<false>(b_s, wn * 64 + j * 16, 0, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) af1[i] = frag<false>(a_s, wm * 64 + i * 16, 1, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bf1[j] = frag<false>(b_s, wn * 64 + j * 16, 1, lane);
        auto kstep = [&](bf16x8 (&af)[4], bf16x8 (&bfr)[4]) {
          __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
          if (rsum) {
            accr[0] = mfma16(wn ? af[2] : af[0], ones, accr[0]);
            accr[1] = mfma16(wn ? af[3] : af[1], ones, accr[1]);
          }
            __builtin_amdgcn_sched_barrier(0);
        };
        lds_tr_retire<15>(af0, bf0);
        kstep(af0, bf0);
        lds_tr_retire<0>(af1, bf1);
        kstep(af1, bf1);
      } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag<AK>(a_s, wm * 64 + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag<BKC>(b_s, wn * 64 + j * 16, s, lane);
        if constexpr (!AK || !BKC) lds_tr_retire(af, bfr);  // asm transposing reads
        __builtin_amdgcn_sched_barrier(0);  // all 8 fragment reads, then the 16 MFMAs
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        if (rsum) {
          accr[0] = mfma16(wn ? af[2] : af[0], ones, accr[0]);
          accr[1] = mfma16(wn ? af[3] : af[1], ones, accr[1]);
        }
      }
      }
      if (!GL && more) {
        stage_store<AK>(ra, smem + (cur ^ 1) * 2 * TILE_BYTES, tid);
        stage_store<BKC>(rb, smem + (cur ^ 1) * 2 * TILE_BYTES + TILE_BYTES, tid);
      }
      if constexpr (NSTG > 2) {
        // this step's fragment reads done (the next step's DMA refills this
        // stage), the next step's tiles landed: the stages requested after
        // it (up to NSTG - 2 of them, 8 DMAs per thread each) may stay in flight
        asm volatile("" ::: "memory");
        const int ahead = min(NSTG - 2, nk - kt - 2);
        if (ahead >= 2) __builtin_amdgcn_s_waitcnt(0x4070);       // vmcnt(16) lgkmcnt(0)
        else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0078);  // vmcnt(8) lgkmcnt(0)
        else __builtin_amdgcn_s_waitcnt(0x0070);                  // vmcnt(0) lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      } else {
        __syncthreads();
      }
    }

    // prefetch the next item's first K stage: its load latency hides behind
    // this item's epilogue (register staging only: the LDS-DMA stage would
    // land under the epilogue's LDS tile)
    prefetched = !GL && jj + pstride < xcount;
    if (prefetched) {
      const Item nx = decode(xstart + jj + pstride);
      stage_load<AK>(ra, A, lda, M, nx.k_end, nx.m0, nx.k_begin, tid);
      stage_load<BKC>(rb, B, ldb, N, nx.k_end, nx.n0, nx.k_begin, tid);
    }

    if (rsum && (lane & 15) == 0) {
      // D[row 4g+r][any col] = row sum; partial per K slice, or the final
      // sum (accumulated in place) when K is not split
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + (2 * wn + j) * 16 + 4 * (lane >> 4) + r;
          if (row < M) {
            if (fused) st_sc1(rowsum + (long)it.split * M + row, accr[j][r]);
            else if (ksplit > 1) rowsum[(long)it.split * M + row] = accr[j][r];
            else rowsum[row] = (e.rs_accumulate ? rowsum[row] : 0.f) + accr[j][r] * e.alpha;
          }
        }
    }
    // Epilogue through LDS: each wave-half (wm) parks its 64x128 fp32 tile in
    // LDS, then all 256 threads walk it row-contiguously, 8 columns each, so
    // bias / residual / gate reads and C / Cf / slab writes are 16-B vectors
    // and 16 consecutive lanes cover one 256-B (bf16) row segment.
    const int g = lane >> 4, c16 = lane & 15;
    constexpr int EP_LD = GBN + 4;
    float* ep = reinterpret_cast<float*>(smem);
    float* slab = ksplit > 1 ? slabs + (long)it.split * M * N : nullptr;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (wm == half) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[(i * 16 + 4 * g + r) * EP_LD + wn * 64 + j * 16 + c16] = acc[i][j][r];
      }
      __syncthreads();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int item = tid + 256 * c;
        const int row = item >> 4, ch = item & 15;
        const int grow = m0 + half * 64 + row, gcol = n0 + ch * 8;
        if (grow < M && gcol < N) {
          float v[8];
          const float4 a = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8);
          const float4 b = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8 + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
          if (slab) {
            const int valid = min(8, N - gcol);
            float* dst = slab + (long)grow * N + gcol;
            if (fused) {  // N % 4 == 0 (launcher): whole float4 pieces
              st_sc1_x4(dst, v[0], v[1], v[2], v[3]);
              if (valid > 4) st_sc1_x4(dst + 4, v[4], v[5], v[6], v[7]);
            } else if (valid == 8 && (N & 3) == 0) {
              *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
              *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
            } else {
              for (int k = 0; k < valid; ++k) dst[k] = v[k];
            }
          } else {
            epi_apply8(e, M, N, grow, gcol, v);
          }
        }
      }
      __syncthreads();
    }
    if (fused) {
      // every wave's slab / partial stores done, then ONE lane takes the
      // tile's ticket; the slice that arrives last sums all of them
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const int tile = it.tm * nbn + it.tn;
        const unsigned old = __hip_atomic_fetch_add(tickets + tile, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(ksplit - 1);
        if (last) __hip_atomic_store(tickets + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *reinterpret_cast<volatile int*>(smem) = last;  // the epilogue tile is dead here
      }
      __syncthreads();
      if (*reinterpret_cast<volatile int*>(smem))
        splitk_tile_reduce(e, M, N, m0, n0, ksplit, slabs, rowsum, rs_final,
                           rowsum != nullptr && it.tn == 0, tid);
      __syncthreads();  // the flag word is overwritten by the next item's staging
    }
  }
}

// ---------------------------------------------------------------------------
// 64x128 bf16 tile for the mid-size forward / dgrad shapes (decoder: M =
// B*T = 8192, N = 512) where 128x128 tiles number ~one per CU and each CU
// then runs a single 4-wave workgroup, exposing every stage's load
// latency.  Halving the tile doubles the workgroups (3 resident per CU: 48
// KiB of LDS, few registers).  4 waves as 2 x 2 of 32 x 64, LDS-DMA staging
// of the same images as the 128 kernel (A: 64 K-contiguous rows; B: row or
// column image of 128), one barrier per 64-deep K step, epilogue through
// LDS in one 64-row pass.
// ---------------------------------------------------------------------------
namespace {
constexpr int G64_A = 64 * GBK * 2;            // 8 KiB
constexpr int G64_STAGE = G64_A + TILE_BYTES;  // + 16 KiB of B
__device__ __forceinline__ void a64_glds(char* buf, const bf16* P, long ld, int rows, int r0,
                                         int k0, int tid) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int chunk = wave * 2 + c;  // 8 x 1 KiB: rows 8*chunk .. +7
    const int row = chunk * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (row & 7);
    const bf16* src = P + (long)min(r0 + row, rows - 1) * ld + k0 + lc * 8;
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(buf + chunk * 1024), 16, 0, 0);
  }
}
}  // namespace

template <bool BKC>
__global__ __launch_bounds__(256, 3) void gemm64_bf16_kernel(int M, int N, int K,
                                                             const bf16* __restrict__ A, long lda,
                                                             const bf16* __restrict__ B, long ldb,
                                                             GemmEpi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nbm = (M + 63) / 64, nbn = (N + GBN - 1) / GBN;
  const int nwg = nbm * nbn;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 8;
  const int nk = K / GBK;

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const int wgid = xstart + jj;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int m0 = (first_m + within % gsz) * 64, n0 = (within / gsz) * GBN;

    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    a64_glds(smem, A, lda, M, m0, 0, tid);
    stage_glds<BKC>(smem + G64_A, B, ldb, N, n0, 0, tid);
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();  // stage kt landed; stage kt-1 fully read
      if (kt + 1 < nk) {
        char* nb = smem + ((kt + 1) & 1) * G64_STAGE;
        a64_glds(nb, A, lda, M, m0, (kt + 1) * GBK, tid);
        stage_glds<BKC>(nb + G64_A, B, ldb, N, n0, (kt + 1) * GBK, tid);
      }
      const char* a_s = smem + (kt & 1) * G64_STAGE;
      const char* b_s = a_s + G64_A;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[2], bfr[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = frag<true>(a_s, wm * 32 + i * 16, s, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag<BKC>(b_s, wn * 64 + j * 16, s, lane);
        if constexpr (!BKC) lds_tr_retire(af, bfr);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS

    const int g = lane >> 4, c16 = lane & 15;
    constexpr int EP_LD = GBN + 4;
    float* ep = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ep[(wm * 32 + i * 16 + 4 * g + r) * EP_LD + wn * 64 + j * 16 + c16] = acc[i][j][r];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int item = tid + 256 * c;  // 64 rows x 16 chunks of 8 columns
      const int row = item >> 4, ch = item & 15;
      const int grow = m0 + row, gcol = n0 + ch * 8;
      if (grow < M && gcol < N) {
        float v[8];
        const float4 a = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8);
        const float4 b = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        epi_apply8(e, M, N, grow, gcol, v);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// 256x256 bf16 GEMM for the large-M forward (NT) and dgrad (NN) shapes.
// 8 waves (2 along M x 4 along N), 128x64 outputs per wave: per 32-deep
// k-step a wave reads 8 A + 4 B fragments for 32 MFMAs, and per K tile the
// workgroup pulls 64 KiB for 8.4 MFLOP (half the L2->CU bytes per flop of
// the 128x128 tile).  Two 64 KiB LDS stages filled by LDS-DMA one K tile
// ahead, one barrier per K tile, one workgroup per CU (persistent).
// Epilogue: four 64-row passes through LDS, 8-column vectors.
// ---------------------------------------------------------------------------
namespace {
constexpr int G2 = 256, G2K = 64;
constexpr int G2_OP = G2 * G2K * 2;     // 32 KiB per operand per stage
constexpr int G2_STAGE = 2 * G2_OP;     // 64 KiB
// epilogue X (residual / gate) slots: A beyond the two stages, B after the
// fp32 staging rows (64 x (256 + 4) floats)
constexpr int G2_XA = 2 * G2_STAGE;                 // 128 KiB
constexpr int G2_XB = 64 * (G2 + 4) * 4;            // 65 KiB
constexpr int G2_LDS = G2_XA + 64 * G2 * 2;         // 160 KiB total

// 64 rows x 256 bf16 columns of X (row-major, ld) -> LDS [64][512 B], by
// LDS-DMA: wave w's instruction c fills 1 KiB = rows 2(4w+c), +1.
__device__ __forceinline__ void g2_xload(char* dst, const bf16* X, long ld, int r0, int c0, int tid) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int chunk = wave * 4 + c;
    const int row = chunk * 2 + (lane >> 5);
    const bf16* src = X + (long)(r0 + row) * ld + c0 + (lane & 31) * 8;
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(dst + chunk * 1024), 16, 0, 0);
  }
}
// 64 rows x 256 byte columns (an e4m3 gate) -> LDS [64][256 B]: wave w's
// instruction c fills rows 4(2w+c) .. +3.
__device__ __forceinline__ void g2_xload8(char* dst, const uint8_t* X, long ld, int r0, int c0, int tid) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int chunk = wave * 2 + c;
    const int row = chunk * 4 + (lane >> 4);
    const uint8_t* src = X + (long)(r0 + row) * ld + c0 + (lane & 15) * 16;
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(dst + chunk * 1024), 16, 0, 0);
  }
}
// X rows of one epilogue pass: bf16, or (G8) the bytes of an e4m3 gate
template <bool G8>
__device__ __forceinline__ void g2_xload_any(char* dst, const bf16* X, long ld, int r0, int c0, int tid) {
  if constexpr (G8) g2_xload8(dst, (const uint8_t*)X, ld, r0, c0, tid);
  else g2_xload(dst, X, ld, r0, c0, tid);
}

// LDS image of one operand stage: KC (row image): row r at r*128 B, 16-B
// chunks XOR (r & 7); column image: k-row at k*512 B, 8-B units XOR
// 4*col_swz(k) (same bank behaviour as the 256-B rows of the 128 kernel).
template <bool KC>
__device__ __forceinline__ void g2_glds(char* buf, const bf16* P, long ld, int rows, int r0,
                                        int k0, int tid) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int chunk = wave * 4 + c;  // 32 x 1 KiB
    const bf16* src;
    if (KC) {
      const int row = chunk * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (row & 7);
      src = P + (long)min(r0 + row, rows - 1) * ld + k0 + lc * 8;
    } else {
      const int k = chunk * 2 + (lane >> 5);
      const int lc = (lane & 31) ^ (2 * (int)col_swz(k));
      const int col = min(r0 + lc * 8, ((rows + 7) & ~7) - 8);
      src = P + (long)(k0 + k) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(buf + chunk * 1024), 16, 0, 0);
  }
}
template <bool KC>
__device__ __forceinline__ bf16x8 g2_frag(const char* buf, int rbase, int s, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
  if (KC) {
    const int row = rbase + c16;
    const int ch = s * 4 + g;
    return lds_read_b128(buf, row * 128 + ((ch ^ (row & 7)) << 4));
  } else {
    const int q = c16 >> 2, p = c16 & 3;
    const int u = (rbase >> 2) + p;
    const int k0 = s * 32 + 8 * g + q;
    const int k1 = k0 + 4;
    bf16x4 lo = lds_read_tr16_async(buf, k0 * 512 + ((u ^ (4 * col_swz(k0))) << 3));
    bf16x4 hi = lds_read_tr16_async(buf, k1 * 512 + ((u ^ (4 * col_swz(k1))) << 3));
    return cat4(lo, hi);
  }
}
}  // namespace

// Streamed epilogue of the 256 x 256 kernels (bf16 and fp8): the residual /
// gate tile of pass p is DMA'd into LDS (slot A for even passes, B for odd)
// one pass ahead, so the passes no longer pay a dependent HBM round trip
// each; the bias is in registers (a thread always owns the same 8 columns).
// The caller DMA'd the X rows of pass 0 into slot A during its K loop.
// Q8: also the e4m3 copy of the stored values (fp8 training forward).
// G8: the gate is an e4m3 copy (a template flag: a runtime read of it from
// the kernel arguments is a scalar load the compiler may place inside the
// k-loop, where it upsets the loop's counted lgkmcnt waits)
template <bool Q8, bool G8 = false>
__device__ __forceinline__ void g2_fast_epilogue(const GemmEpi& e, const f32x4 (&acc)[8][4], char* smem,
                                                 int m0, int n0, int tid, const float (&bv)[8],
                                                 const bf16* xsrc, long ldx, float& amax_acc) {
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int g = lane >> 4, c16 = lane & 15;
  constexpr int EP_LD = G2 + 4;
  float* ep = reinterpret_cast<float*>(smem);
  float q8s = 1.f;
  if constexpr (Q8) q8s = *e.q8_scale;
  if (xsrc) g2_xload_any<G8>(smem + G2_XB, xsrc, ldx, m0 + 64, n0, tid);
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    if (wm == (pass >> 1)) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = 4 * (pass & 1) + ii;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ep[(ii * 16 + 4 * g + r) * EP_LD + wn * 64 + j * 16 + c16] = acc[i][j][r];
      }
    }
    // ep rows written; X(pass) landed; X(pass-1) slot free (the residual /
    // gate DMA needs vmcnt; without one only LDS traffic must settle)
    if (xsrc) __syncthreads();
    else smer_lds_barrier();
    if (xsrc && pass >= 1 && pass < 3)
      g2_xload_any<G8>(smem + ((pass + 1) & 1 ? G2_XB : G2_XA), xsrc, ldx, m0 + 64 * (pass + 1), n0, tid);
    const char* xs = smem + ((pass & 1) ? G2_XB : G2_XA);
    const int ch = tid & 31;
    // Q8: one item at a time (unrolled, the four items' temporaries beside
    // the live accumulators spilled 42 VGPRs)
#pragma unroll (Q8 ? 1 : 4)
    for (int c = 0; c < 4; ++c) {
      const int row = (tid >> 5) + 16 * c;
      const int grow = m0 + pass * 64 + row, gcol = n0 + ch * 8;
      float v[8];
      const float4 a = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8);
      const float4 b = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = v[k] * e.alpha + bv[k];
      if (e.relu) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
      }
      if (e.drop_thr)
        smer_drop8(smer_rowkey(e.seed, (uint32_t)grow), e.drop_thr, e.drop_scale, (uint32_t)gcol, v);
      if constexpr (G8) {
        const uint2 gb = *reinterpret_cast<const uint2*>(xs + row * 256 + ch * 8);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t byte = ((k < 4 ? gb.x : gb.y) >> (8 * (k & 3))) & 0xffu;
          v[k] = byte - 1u < 0x7fu ? v[k] * e.gate_scale : 0.f;  // 1..127: positive
        }
      } else if (xsrc) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + row * 512 + ch * 16);
        if (e.residual) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += (float)xv[k];
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = (float)xv[k] > 0.f ? v[k] * e.gate_scale : 0.f;
        }
      }
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
      if constexpr (Q8) {  // (the e4m3 copy alone when C is null)
        if (e.C) *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)grow * e.ldc + gcol) = o;
      } else {
        *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)grow * e.ldc + gcol) = o;
      }
      if constexpr (Q8) {  // e4m3 copy of the stored (bf16-rounded) values
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (float)o[k];
        *reinterpret_cast<uint2*>(e.q8 + (long)grow * e.ldq8 + gcol) = smer_q8x8(v, q8s);
        amax_acc = fmaxf(amax_acc, smer_absmax8(v));
      }
    }
    if (xsrc) __syncthreads();
    else smer_lds_barrier();
  }
}

template <bool AK, bool BKC, bool FAST>
__global__ __launch_bounds__(512, 1) void gemm256_bf16_kernel(int M, int N, int K,
                                                              const bf16* __restrict__ A, long lda,
                                                              const bf16* __restrict__ B, long ldb,
                                                              GemmEpi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nbm = (M + G2 - 1) / G2, nbn = (N + G2 - 1) / G2;
  const int nwg = nbm * nbn;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;
  const int nk = K / G2K;
  // streamed-epilogue fast path: whole tiles, bf16 C only, at most one of
  // residual / gate (the X operand DMA'd through LDS)
  constexpr bool fast = FAST;  // host: gemm256_fast_ok
  const bf16* xsrc = (const bf16*)(e.residual ? e.residual : e.gate);
  const long ldx = e.residual ? e.ldr : e.ldg;
  g2_start_skew(e.skew);

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const int wgid = xstart + jj;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int m0 = (first_m + within % gsz) * G2, n0 = (within / gsz) * G2;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (fast && e.bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(e.bias + n0 + (tid & 31) * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(e.bias + n0 + (tid & 31) * 8 + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
      bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    }
    g2_glds<AK>(smem, A, lda, M, m0, 0, tid);
    g2_glds<BKC>(smem + G2_OP, B, ldb, N, n0, 0, tid);
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();  // stage kt landed (vmcnt(0) + barrier); stage kt-1 fully read
      // X rows of the first epilogue pass into slot A (beyond the stages)
      if (fast && xsrc && kt == nk / 2) g2_xload(smem + G2_XA, xsrc, ldx, m0, n0, tid);
      if (kt + 1 < nk) {
        char* nb = smem + ((kt + 1) & 1) * G2_STAGE;
        g2_glds<AK>(nb, A, lda, M, m0, (kt + 1) * G2K, tid);
        g2_glds<BKC>(nb + G2_OP, B, ldb, N, n0, (kt + 1) * G2K, tid);
      }
      const char* a_s = smem + (kt & 1) * G2_STAGE;
      const char* b_s = a_s + G2_OP;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // the k-step's 12 fragment reads first, then its 32 MFMAs (else the
        // compiler waits on each A fragment right behind 4 MFMAs)
        bf16x8 bfr[4], af[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = g2_frag<BKC>(b_s, wn * 64 + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = g2_frag<AK>(a_s, wm * 128 + i * 16, s, lane);
        // dgrad: the 8 asm B reads are older than the 8 A row reads, whose
        // waits hipcc places before each MFMA group itself
        if constexpr (AK && !BKC) lds_tr_retire_older<8>(bfr);
        else if constexpr (!AK || !BKC) lds_tr_retire(af, bfr);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS

    const int g = lane >> 4, c16 = lane & 15;
    constexpr int EP_LD = G2 + 4;
    float* ep = reinterpret_cast<float*>(smem);
    if constexpr (FAST) {
      float amax_unused = 0.f;
      g2_fast_epilogue<false>(e, acc, smem, m0, n0, tid, bv, xsrc, ldx, amax_unused);
      continue;
    }

    // generic epilogue: 4 passes of 64 rows x 256 columns (fp32 in LDS)
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      // rows [64*pass, 64*pass+64) belong to wm = pass >> 1, fragments
      // i = 4*(pass & 1) .. +3
      if (wm == (pass >> 1)) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = 4 * (pass & 1) + ii;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[(ii * 16 + 4 * g + r) * EP_LD + wn * 64 + j * 16 + c16] = acc[i][j][r];
        }
      }
      smer_lds_barrier();  // LDS settled; stores left in flight
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int item = tid + 512 * c;  // 64 rows x 32 chunks of 8 columns
        const int row = item >> 5, ch = item & 31;
        const int grow = m0 + pass * 64 + row, gcol = n0 + ch * 8;
        if (grow < M && gcol < N) {
          float v[8];
          const float4 a = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8);
          const float4 b = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8 + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
          epi_apply8(e, M, N, grow, gcol, v);
        }
      }
      smer_lds_barrier();  // LDS settled; stores left in flight
    }
  }
}

// ---------------------------------------------------------------------------
// Staggered 256x256 bf16 GEMM (round 4) for the forward (NT) and dgrad (NN)
// shapes with whole 256 tiles and a bf16 output (the streamed-epilogue
// cases).  Same tile and wave layout as gemm256_bf16_kernel (8 waves, 2 along
// M x 4 along N, 128x64 outputs per wave), a different schedule:
//
//  * LDS holds four 32-deep k-step slots (A [256][32] + B, 32 KiB each),
//    filled by LDS-DMA three k-steps ahead, so two slots are always in
//    flight across the barriers (counted vmcnt, never 0 in the loop);
//  * the two M halves of the workgroup run one barrier apart (waves 4-7 pass
//    one extra barrier at the start, waves 0-3 one at the end): on every
//    SIMD one wave issues its 12 fragment reads while its partner runs its
//    32 MFMAs, then they swap -- the LDS latency of a k-step hides under the
//    partner's matrix work instead of stalling both waves together;
//  * roles: waves 4-7 issue every LDS-DMA (operands and the epilogue's
//    residual / gate rows) and never store, waves 0-3 issue every global
//    store of the epilogue and never load.  gfx9's vmcnt retires in issue
//    order and counts stores too, so a wave that stores and then waits for
//    its next operand DMA waits for its stores to drain to HBM: at K = 512
//    (FFN1: 134 MB of output) that drain was 26 of the old kernel's 90 us.
//    Here the loaders' counters hold only loads and the storers never wait,
//    so a tile's output drains under the next tile's k-loop.
//  * every LDS-DMA is an asm statement (M0 set inside it), invisible to
//    hipcc's wait bookkeeping, which otherwise makes compiler-visible LDS
//    accesses wait vmcnt(0) for any DMA it thinks pending; fragment reads are
//    asm too (lds_read_*_async) and retired by explicit lgkmcnt waits.
// Row image per slot: row r at r*64 B, 16-B chunk c at c ^ (2 * bit2(r))
// (conflict-free for the 16x16x32 fragment reads' ds_read_b128 lane groups);
// the NN B operand keeps the column image of the 256 kernel (512-B k rows).
// ---------------------------------------------------------------------------
namespace {
constexpr int GS_KS = 32;                    // k-step per LDS slot
constexpr int GS_OP = G2 * GS_KS * 2;        // 16 KiB per operand per slot
constexpr int GS_SLOT = 2 * GS_OP;           // 32 KiB

__device__ __forceinline__ uint32_t lds_u32(const char* p) {
  typedef __attribute__((address_space(3))) const char lds_char;
  return (uint32_t)(uintptr_t)((lds_char*)p);
}

// 16 B per lane from sbase + voff into LDS [lds_base + 16 * lane): the
// global address is an SGPR base plus a 32-bit per-lane VGPR offset (one VGPR
// per DMA instead of a 64-bit pointer); M0 carries the wave-uniform LDS base,
// set and restored inside the statement.
__device__ __forceinline__ void glds16_asm(const void* sbase, uint32_t voff, uint32_t lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_base)
      : "memory");
}

// s_waitcnt vmcnt(N), expcnt / lgkmcnt untouched (gfx9 field layout)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | ((N >> 4) << 14));
}

__device__ __forceinline__ void gs_bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ uint32_t gs_swz(int r) { return (uint32_t)(2 * ((r >> 2) & 1)); }

__device__ __forceinline__ const void* sgpr_ptr(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// One k-step (32 deep) of A and B into a slot: 32 DMA instructions of 1 KiB,
// eight per loader wave (lw = 0..3): piece t < 4 is A rows 16 (4 lw + t) ..,
// piece t >= 4 the matching B piece.  At / Bt: the tile's operand bases at
// this k-step (wave-uniform).
template <bool BKC>
__device__ __forceinline__ void gs_piece(int t, uint32_t slot_lds, const bf16* At, long lda, const bf16* Bt,
                                         long ldb, int lw, int lane) {
  const int c = lw * 4 + (t & 3);
  if (t < 4) {  // 16 rows of 64 B
    const int row = c * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ (int)gs_swz(row);
    glds16_asm(sgpr_ptr(At), (uint32_t)((row * lda + lc * 8) * 2),
               (uint32_t)__builtin_amdgcn_readfirstlane(slot_lds + c * 1024));
    return;
  }
  uint32_t off;
  if (BKC) {
    const int row = c * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ (int)gs_swz(row);
    off = (uint32_t)((row * ldb + lc * 8) * 2);
  } else {  // 2 k-rows of 256 columns (512 B each)
    const int k = c * 2 + (lane >> 5);
    const int lc = (lane & 31) ^ (2 * (int)col_swz(k));
    off = (uint32_t)((k * ldb + lc * 8) * 2);
  }
  glds16_asm(sgpr_ptr(Bt), off, (uint32_t)__builtin_amdgcn_readfirstlane(slot_lds + GS_OP + c * 1024));
}
template <bool BKC>
__device__ __forceinline__ void gs_issue(uint32_t slot_lds, const bf16* At, long lda, const bf16* Bt,
                                         long ldb, int lw, int lane) {
#pragma unroll
  for (int t = 0; t < 8; ++t) gs_piece<BKC>(t, slot_lds, At, lda, Bt, ldb, lw, lane);
}

// Epilogue LDS map: eight 32-row passes through fp32 staging rows at 0; the
// residual / gate rows X of a pass DMA'd one pass ahead into XA (even passes;
// beyond the four k-step slots, so X(0) loads during the k-loop) or XB (odd,
// after the staging rows); the bias row (1 KiB) beside XA.
// The staging rows, XB and the two OUT buffers live in slots 2-3: slots 0-1
// take the NEXT tile's first two k-steps while this tile's epilogue runs.
constexpr int GS_EPR = 32;                          // rows per epilogue pass
constexpr int GS_XA = 4 * GS_SLOT;                  // 128 KiB
constexpr int GS_BIAS = GS_XA + GS_EPR * 512;       // 144 KiB
constexpr int GS_EP = 2 * GS_SLOT;                  // 64 KiB: 32 fp32 rows of 1 KiB
constexpr int GS_XB = GS_EP + GS_EPR * 1024;        // 96 KiB
constexpr int GS_OUT = GS_XB + GS_EPR * 512;        // 112 KiB: 2 x [16][512 B] bf16
static_assert(GS_OUT + 2 * 16 * 512 == 4 * GS_SLOT, "epilogue region = slots 2-3");
static_assert(GS_BIAS + 1024 <= G2_LDS, "LDS budget");
// fp32 staging element (row, col): 1-KiB rows, column bit 4 flipped on rows
// with bit 2 set (the owners' lanes l and l + 16 write rows 4 apart)
__device__ __forceinline__ int gs_ep_idx(int row, int col) { return row * 256 + (col ^ (((row >> 2) & 1) << 4)); }

// 32 rows x 256 columns of the epilogue operand X into an LDS slot
// [32][512 B]: four 1-KiB DMA instructions per loader wave.  Xt: X at the
// pass's (r0, c0), wave-uniform.
__device__ __forceinline__ void gs_xload(uint32_t dst_lds, const bf16* Xt, long ld, int lw, int lane) {
  const void* sx = sgpr_ptr(Xt);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int chunk = lw * 4 + t;  // 2 rows per KiB
    const int row = chunk * 2 + (lane >> 5);
    glds16_asm(sx, (uint32_t)((row * ld + (lane & 31) * 8) * 2),
               (uint32_t)__builtin_amdgcn_readfirstlane(dst_lds + chunk * 1024));
  }
}
// The tile's 256 bias floats (1 KiB) into LDS: one DMA instruction (every
// loader wave issues it, so their vmcnt bookkeeping stays uniform).
__device__ __forceinline__ void gs_bias_load(uint32_t dst_lds, const float* bt, int lane) {
  glds16_asm(sgpr_ptr(bt), (uint32_t)(lane * 16), dst_lds);
}

template <int OFF>
__device__ __forceinline__ bf16x8 lds_b128_off(uint32_t a) {
  uint4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x8, r);
}
template <int OFF>
__device__ __forceinline__ bf16x4 lds_tr16_off(uint32_t a) {
  i16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return __builtin_bit_cast(bf16x4, r);
}

// The 12 fragment reads of one k-step: 8 A (rows wm*128 + 16 i) and 4 B
// (columns wn*64 + 16 q), with immediate offsets off one or four base VGPRs.
template <bool BKC>
__device__ __forceinline__ void gs_frags(uint32_t slot_lds, int wm, int wn, int lane, bf16x8 (&af)[8],
                                         bf16x8 (&bfr)[4]) {
  const int g = lane >> 4, c16 = lane & 15;
  const uint32_t ab = slot_lds + wm * 8192 + c16 * 64 + ((g ^ gs_swz(c16)) << 4);
  if constexpr (BKC) {
    const uint32_t bb = slot_lds + GS_OP + wn * 4096 + c16 * 64 + ((g ^ gs_swz(c16)) << 4);
    bfr[0] = lds_b128_off<0>(bb);
    bfr[1] = lds_b128_off<1024>(bb);
    bfr[2] = lds_b128_off<2048>(bb);
    bfr[3] = lds_b128_off<3072>(bb);
  } else {
    const int qq = c16 >> 2, p = c16 & 3;
    const int k0 = 8 * g + qq;
    const uint32_t cs4 = 4 * col_swz(k0);
    const uint32_t kb = slot_lds + GS_OP + k0 * 512;
#define GS_BNN(Q)                                                                  \
    {                                                                              \
      const uint32_t a = kb + (((uint32_t)(wn * 16 + (Q) * 4 + p) ^ cs4) << 3);   \
      bfr[Q] = cat4(lds_tr16_off<0>(a), lds_tr16_off<2048>(a));                   \
    }
    GS_BNN(0) GS_BNN(1) GS_BNN(2) GS_BNN(3)
#undef GS_BNN
  }
  af[0] = lds_b128_off<0>(ab);
  af[1] = lds_b128_off<1024>(ab);
  af[2] = lds_b128_off<2048>(ab);
  af[3] = lds_b128_off<3072>(ab);
  af[4] = lds_b128_off<4096>(ab);
  af[5] = lds_b128_off<5120>(ab);
  af[6] = lds_b128_off<6144>(ab);
  af[7] = lds_b128_off<7168>(ab);
}
}  // namespace

template <bool BKC>
__global__ __launch_bounds__(512, 1) void gemm256s_bf16_kernel(int M, int N, int K,
                                                               const bf16* __restrict__ A, long lda,
                                                               const bf16* __restrict__ B, long ldb,
                                                               GemmEpi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3, lw = wave & 3;
  const bool loader = wm == 1;  // waves 4-7: every DMA; waves 0-3: every store
  const int nbm = M / G2, nbn = N / G2;
  const int nwg = nbm * nbn;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;
  const int nk = K / GS_KS;  // host: nk >= 4
  const bf16* xsrc = (const bf16*)(e.residual ? e.residual : e.gate);
  const long ldx = e.residual ? e.ldr : e.ldg;
  const uint32_t lds0 = lds_u32(smem);
  const int g = lane >> 4, c16 = lane & 15;
  constexpr int EP_LD = G2 + 4;

  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // e.dbg: tiles 0 and 1, 4 stamps each
  int tcount = 0;
  g2_start_skew(e.skew);
  for (int jj = braw >> 3; jj < xcount; jj += pstride, ++tcount) {
    const int wgid = xstart + jj;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int m0 = (first_m + within % gsz) * G2, n0 = (within / gsz) * G2;
    const bool stamp = e.dbg != nullptr && tcount < 2;
    if (stamp) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tcount == 0) st[0] = t_; else st[4] = t_; }

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // operand bases of this tile; k-step k adds k * 32 columns (A, NT B) or
    // k * 32 rows (NN B)
    const bf16* At = A + (long)m0 * lda;
    const bf16* Bt = BKC ? B + (long)n0 * ldb : B + n0;
    const long bstep = BKC ? GS_KS : (long)GS_KS * ldb;

    // prologue: k-steps 0..2 in flight, k-step 0 landed before the first
    // barrier (after the first tile, k-steps 0 and 1 were issued during the
    // previous tile's epilogue)
    if (loader) {
      if (tcount == 0) {
        gs_issue<BKC>(lds0 + 0 * GS_SLOT, At, lda, Bt, ldb, lw, lane);
        gs_issue<BKC>(lds0 + 1 * GS_SLOT, At + GS_KS, lda, Bt + bstep, ldb, lw, lane);
      }
      gs_issue<BKC>(lds0 + 2 * GS_SLOT, At + 2 * GS_KS, lda, Bt + 2 * bstep, ldb, lw, lane);
      vm_wait<16>();
    }
    gs_bar();
    if (loader) gs_bar();  // the lagging half: one barrier behind from here
    if (stamp) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tcount == 0) st[1] = t_; else st[5] = t_; }

    for (int j = 0; j < nk; ++j) {
      // R(j): fragment reads of slot j & 3; a loader issues the B half of
      // k-step j+3 (into the slot k-step j-1 left: every wave retired its
      // reads of it before its previous M phase) and waits for k-step j+1.
      // Issue order per loader: B(t) in R(t-3), A(t) in M(t-3).
      bf16x8 bfr[4], af[8];
      gs_frags<BKC>(lds0 + (j & 3) * GS_SLOT, wm, wn, lane, af, bfr);
      const bool do_k = loader && j + 3 < nk;
      const uint32_t kslot = lds0 + ((j + 3) & 3) * GS_SLOT;
      const bf16* Aj = At + (long)(j + 3) * GS_KS;
      const bf16* Bj = Bt + (j + 3) * bstep;
      if (do_k) {
#pragma unroll
        for (int t = 4; t < 8; ++t) gs_piece<BKC>(t, kslot, Aj, lda, Bj, ldb, lw, lane);
      }
      if (loader) {
        if (j + 3 < nk) {
          vm_wait<12>();  // k-step j+1 landed (B, A of j+2 and B of j+3 fly)
        } else if (j + 3 == nk) {
          vm_wait<8>();
        } else if (j + 2 == nk) {  // k-step nk-1 landed; bias / X(0) may fly on
          if (xsrc && e.bias) vm_wait<5>();
          else if (xsrc) vm_wait<4>();
          else if (e.bias) vm_wait<1>();
          else vm_wait<0>();
        }
      }
      gs_bar();
      // M(j): 32 MFMAs; a loader slips the A half of k-step j+3 in behind
      // every 8 of them (an LDS-DMA piece costs ~60-185 issue cycles: all
      // eight in one phase stretched it past the partner's 32 MFMAs)
      lds_tr_retire(af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] = mfma16(af[i], bfr[q], acc[i][q]);
        if ((i & 1) && do_k) {
          __builtin_amdgcn_sched_barrier(0);
          gs_piece<BKC>(i >> 1, kslot, Aj, lda, Bj, ldb, lw, lane);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (loader && j + 3 == nk) {
        // the epilogue's bias row and first X rows, beyond the four slots
        // (the bias through LDS: a register load would be a vmcnt wait
        // hipcc places itself, on the storers' outstanding stores)
        if (e.bias) gs_bias_load(lds0 + GS_BIAS, e.bias + n0, lane);
        if (xsrc) gs_xload(lds0 + GS_XA, xsrc + (long)m0 * ldx + n0, ldx, lw, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
      gs_bar();
    }
    if (!loader) gs_bar();  // realign the halves
    if (stamp) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tcount == 0) st[2] = t_; else st[6] = t_; }

    // ---- epilogue: eight 32-row passes through fp32 LDS staging ---------
    // The owning half (rows 128 wm .. +127) stages its accumulators; all 512
    // threads apply bias / ReLU / dropout / residual or gate to 2 items of 8
    // columns; the storers store theirs, the loaders hand theirs to the
    // storers as bf16 through OUT (stored one pass later): loaders never
    // store, so their vmcnt holds DMAs only.  The loaders first issue the
    // next tile's k-steps 0 and 1 (slots 0-1), which land under this
    // epilogue, then stream X one pass ahead.
    const int jn = jj + pstride;
    const bool has_next = jn < xcount;
    if (loader && has_next) {
      const int wn2 = xstart + jn;
      const int grp2 = wn2 / (GM * nbn);
      const int gsz2 = min(nbm - grp2 * GM, GM);
      const int win2 = wn2 % (GM * nbn);
      const int m1 = (grp2 * GM + win2 % gsz2) * G2, n1 = (win2 / gsz2) * G2;
      const bf16* At1 = A + (long)m1 * lda;
      const bf16* Bt1 = BKC ? B + (long)n1 * ldb : B + n1;
      if (xsrc)  // X(1) ahead of them: its wait then passes over them
        gs_xload(lds0 + GS_XB, xsrc + (long)(m0 + GS_EPR) * ldx + n0, ldx, lw, lane);
      gs_issue<BKC>(lds0 + 0 * GS_SLOT, At1, lda, Bt1, ldb, lw, lane);
      gs_issue<BKC>(lds0 + 1 * GS_SLOT, At1 + GS_KS, lda, Bt1 + bstep, ldb, lw, lane);
    } else if (loader && xsrc) {
      gs_xload(lds0 + GS_XB, xsrc + (long)(m0 + GS_EPR) * ldx + n0, ldx, lw, lane);
    }
    float* ep = reinterpret_cast<float*>(smem + GS_EP);
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int ch = tid & 31;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      if (loader) {  // X(pass) (and at pass 0 the bias) landed
        if (xsrc) {
          if (pass >= 1 && pass < 7)  // X(pass+1) into the slot X(pass-1) left
            gs_xload(lds0 + (((pass + 1) & 1) ? GS_XB : GS_XA),
                     xsrc + (long)(m0 + GS_EPR * (pass + 1)) * ldx + n0, ldx, lw, lane);
          if (pass <= 1) {
            if (has_next) vm_wait<20>();
            else vm_wait<4>();
          } else if (pass < 7) {
            vm_wait<4>();
          } else {
            vm_wait<0>();
          }
        } else if (pass == 0 && e.bias) {
          if (has_next) vm_wait<16>();
          else vm_wait<0>();
        }
      }
      if (wm == (pass >> 2)) {  // fragment rows i = 2 (pass & 3) + ii
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int i = 2 * (pass & 3) + ii;
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[gs_ep_idx(ii * 16 + 4 * g + r, wn * 64 + q * 16 + c16)] = acc[i][q][r];
        }
      }
      smer_lds_barrier();  // staging rows written, X(pass) and the bias landed
      if (pass == 0 && e.bias) {
        const float* bl = reinterpret_cast<const float*>(smem + GS_BIAS) + ch * 8;
        const float4 b0 = *reinterpret_cast<const float4*>(bl);
        const float4 b1 = *reinterpret_cast<const float4*>(bl + 4);
        bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
        bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
      }
      // storers: the loaders' items of the previous pass (bf16 in OUT)
      if (!loader && pass >= 1) {
        const char* ob = smem + GS_OUT + ((pass - 1) & 1) * 8192;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int lr = (tid >> 5) + 8 * c;  // 0..15 -> pass rows 8..15, 24..31
          const int row = (lr & 7) + 8 + 16 * (lr >> 3);
          const bf16x8 o = *reinterpret_cast<const bf16x8*>(ob + lr * 512 + ch * 16);
          *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)(m0 + (pass - 1) * GS_EPR + row) * e.ldc + n0 + ch * 8) = o;
        }
      }
      const char* xs = smem + ((pass & 1) ? GS_XB : GS_XA);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int row = (tid >> 5) + 16 * c;  // storers rows 0..7, 16..23; loaders 8..15, 24..31
        const int grow = m0 + pass * GS_EPR + row, gcol = n0 + ch * 8;
        float v[8];
        const float4 a = *reinterpret_cast<const float4*>(ep + gs_ep_idx(row, ch * 8));
        const float4 b = *reinterpret_cast<const float4*>(ep + gs_ep_idx(row, ch * 8) + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] * e.alpha + bv[k];
        if (e.relu) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
        }
        if (e.drop_thr)
          smer_drop8(smer_rowkey(e.seed, (uint32_t)grow), e.drop_thr, e.drop_scale, (uint32_t)gcol, v);
        if (xsrc) {
          const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + row * 512 + ch * 16);
          if (e.residual) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += (float)xv[k];
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (float)xv[k] > 0.f ? v[k] * e.gate_scale : 0.f;
          }
        }
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
        if (!loader) {
          *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)grow * e.ldc + gcol) = o;
        } else {
          const int lr = (row & 7) + 8 * (row >> 4);
          *reinterpret_cast<bf16x8*>(smem + GS_OUT + (pass & 1) * 8192 + lr * 512 + ch * 16) = o;
        }
      }
      smer_lds_barrier();  // staging, X(pass) and OUT(pass - 1) read before they are rewritten
    }
    if (!loader) {  // the loaders' items of the last pass
      const char* ob = smem + GS_OUT + 8192;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int lr = (tid >> 5) + 8 * c;
        const int row = (lr & 7) + 8 + 16 * (lr >> 3);
        const bf16x8 o = *reinterpret_cast<const bf16x8*>(ob + lr * 512 + ch * 16);
        *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)(m0 + 7 * GS_EPR + row) * e.ldc + n0 + ch * 8) = o;
      }
    }
    if (stamp) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); if (tcount == 0) st[3] = t_; else st[7] = t_; }
  }
  if (e.dbg && lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) e.dbg[((long)blockIdx.x * 8 + wave) * 8 + k] = st[k];
  }
}

static int smer_num_cus();
// phase stamps of the staggered kernel (diagnostics; tools/gemm256s_phases.py)
static unsigned long long* g_gemm_dbg = nullptr;
static size_t g_gemm_dbg_bytes = 0;
extern "C" int smer_gemm_debug_stamps(void* buf, size_t bytes) {
  SMER_REQUIRE(!buf || bytes >= (size_t)64 * smer_num_cus() * sizeof(unsigned long long),
               "smer_gemm_debug_stamps: the buffer holds 64 stamps per CU");
  g_gemm_dbg = (unsigned long long*)buf;
  g_gemm_dbg_bytes = buf ? bytes : 0;
  return SMER_OK;
}
// the stamp buffer for a launch of `grid` workgroups on stream s: none while
// the stream is capturing (a graph would keep the pointer past the tool's
// buffer) or when the buffer is too small for the grid
static unsigned long long* gemm_dbg_for(int grid, hipStream_t s) {
  if (!g_gemm_dbg) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  if ((size_t)grid * 64 * sizeof(unsigned long long) > g_gemm_dbg_bytes) return nullptr;
  return g_gemm_dbg;
}

// ---------------------------------------------------------------------------
// Weight gradients on the 256x256 tile: dW (+)= dY^T X with K = tokens, both
// operands M/N-contiguous (column images, transposing fragment reads).  Half
// the L2->CU bytes per flop of the 128x128 kernel and twice the MFMA work per
// stage to hide each stage's load behind (2 waves per SIMD x 2 k-steps x 32
// MFMAs).  Deterministic split-K over K slices: work item = (slice, tile),
// tiles of one slice adjacent so the blocks an XCD runs together read the
// same dY / X rows through its L2; each slice writes an fp32 slab, reduced in
// fixed order by splitk_reduce_kernel (or, unsplit, the epilogue adds into
// dW).  Fused bias gradient on the first column tile: every wave sums two of
// its eight A fragments per k-step with v_dot2c_f32_bf16 against ones (two
// VGPRs; the row-sum MFMA variant spilled), lanes of a row reduced at the end.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float rowsum_frag(bf16x8 v, float s) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
  s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(v, v, 0, 1), one, s, false);
  s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(v, v, 2, 3), one, s, false);
  s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(v, v, 4, 5), one, s, false);
  s = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(v, v, 6, 7), one, s, false);
  return s;
}

__global__ __launch_bounds__(512, 1) void gemm256_wgrad_kernel(int M, int N, int K,
                                                               const bf16* __restrict__ A, long lda,
                                                               const bf16* __restrict__ B, long ldb,
                                                               GemmEpi e, int ksplit, int kchunk,
                                                               float* __restrict__ slabs,
                                                               float* __restrict__ rowsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int wn_s = __builtin_amdgcn_readfirstlane(wn);  // wave-uniform branch below
  const int nbm = (M + G2 - 1) / G2, nbn = (N + G2 - 1) / G2;
  const int ntiles = nbm * nbn;
  const int nwg = ntiles * ksplit;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const int lin = xstart + jj;
    const int split = lin / ntiles, wgid = lin % ntiles;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int tn = within / gsz;
    const int m0 = (first_m + within % gsz) * G2, n0 = tn * G2;
    const int k_begin = split * kchunk, k_end = min(K, k_begin + kchunk);
    const int nk = (k_end - k_begin) / G2K;
    const bool rsum = rowsum != nullptr && tn == 0;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float rs0 = 0.f, rs1 = 0.f;

    g2_glds<false>(smem, A, lda, M, m0, k_begin, tid);
    g2_glds<false>(smem + G2_OP, B, ldb, N, n0, k_begin, tid);
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();  // stage kt landed; stage kt-1 fully read
      if (kt + 1 < nk) {
        char* nb = smem + ((kt + 1) & 1) * G2_STAGE;
        g2_glds<false>(nb, A, lda, M, m0, k_begin + (kt + 1) * G2K, tid);
        g2_glds<false>(nb + G2_OP, B, ldb, N, n0, k_begin + (kt + 1) * G2K, tid);
      }
      const char* a_s = smem + (kt & 1) * G2_STAGE;
      const char* b_s = a_s + G2_OP;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 bfr[4], af[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = g2_frag<false>(b_s, wn * 64 + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = g2_frag<false>(a_s, wm * 128 + i * 16, s, lane);
        lds_tr_retire(af, bfr);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        if (rsum) {  // wave wn sums A fragments 2wn, 2wn+1 (rows of its 32)
          if (wn_s == 0)      { rs0 = rowsum_frag(af[0], rs0); rs1 = rowsum_frag(af[1], rs1); }
          else if (wn_s == 1) { rs0 = rowsum_frag(af[2], rs0); rs1 = rowsum_frag(af[3], rs1); }
          else if (wn_s == 2) { rs0 = rowsum_frag(af[4], rs0); rs1 = rowsum_frag(af[5], rs1); }
          else                { rs0 = rowsum_frag(af[6], rs0); rs1 = rowsum_frag(af[7], rs1); }
        }
      }
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS

    if (rsum) {
      // lane (g, c16) holds row c16's sum over its k subset: reduce over g
      rs0 += __shfl_xor(rs0, 16); rs0 += __shfl_xor(rs0, 32);
      rs1 += __shfl_xor(rs1, 16); rs1 += __shfl_xor(rs1, 32);
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = m0 + wm * 128 + (2 * wn + j) * 16 + lane;
          const float v = j ? rs1 : rs0;
          if (row < M) {
            if (ksplit > 1) rowsum[(long)split * M + row] = v;
            else rowsum[row] = (e.rs_accumulate ? rowsum[row] : 0.f) + v * e.alpha;
          }
        }
      }
    }

    const int g = lane >> 4, c16 = lane & 15;
    constexpr int EP_LD = G2 + 4;
    float* ep = reinterpret_cast<float*>(smem);
    float* slab = ksplit > 1 ? slabs + (long)split * M * N : nullptr;
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      if (wm == (pass >> 1)) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = 4 * (pass & 1) + ii;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[(ii * 16 + 4 * g + r) * EP_LD + wn * 64 + j * 16 + c16] = acc[i][j][r];
        }
      }
      smer_lds_barrier();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int item = tid + 512 * c;  // 64 rows x 32 chunks of 8 columns
        const int row = item >> 5, ch = item & 31;
        const int grow = m0 + pass * 64 + row, gcol = n0 + ch * 8;
        if (grow < M && gcol < N) {
          float v[8];
          const float4 a = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8);
          const float4 b = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8 + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
          if (slab) {
            const int valid = min(8, N - gcol);
            float* dst = slab + (long)grow * N + gcol;
            if (valid == 8 && (N & 3) == 0) {
              *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
              *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
            } else {
              for (int k = 0; k < valid; ++k) dst[k] = v[k];
            }
          } else {
            epi_apply8(e, M, N, grow, gcol, v);
          }
        }
      }
      smer_lds_barrier();
    }
  }
}

// ---------------------------------------------------------------------------
// Staggered 256x256 weight-gradient kernel: dW (+)= dY^T X with both operands
// column images (K = tokens), the k-loop schedule of gemm256s_bf16_kernel
// (four 32-deep slots, three k-steps ahead, halves one barrier apart, waves
// 4-7 issue every DMA, waves 0-3 every store) on the split-K work items of
// gemm256_wgrad_kernel (slice, tile).  Fragments of both operands are
// transposing reads (ds_read_b64_tr_b16) of 512-B k rows; the fused bias
// gradient sums two A fragments per wave per k-step (v_dot2c, as there).
// Output fp32: a split-K slab, or dW (+)= alpha * acc unsplit.
// ---------------------------------------------------------------------------
namespace {
// piece t < 4: A k-rows 2c, 2c+1 (c = 4 lw + t), t >= 4: the B ones
__device__ __forceinline__ void gsw_piece(int t, uint32_t slot_lds, const bf16* At, long lda, const bf16* Bt,
                                          long ldb, int lw, int lane) {
  const int c = lw * 4 + (t & 3);
  const int k = c * 2 + (lane >> 5);
  const int lc = (lane & 31) ^ (2 * (int)col_swz(k));
  if (t < 4)
    glds16_asm(sgpr_ptr(At), (uint32_t)((k * lda + lc * 8) * 2),
               (uint32_t)__builtin_amdgcn_readfirstlane(slot_lds + c * 1024));
  else
    glds16_asm(sgpr_ptr(Bt), (uint32_t)((k * ldb + lc * 8) * 2),
               (uint32_t)__builtin_amdgcn_readfirstlane(slot_lds + GS_OP + c * 1024));
}
__device__ __forceinline__ void gsw_issue(uint32_t slot_lds, const bf16* At, long lda, const bf16* Bt, long ldb,
                                          int lw, int lane) {
#pragma unroll
  for (int t = 0; t < 8; ++t) gsw_piece(t, slot_lds, At, lda, Bt, ldb, lw, lane);
}
// 8 A fragments (rows wm*128 + 16 i) and 4 B (columns wn*64 + 16 q) of one
// k-step, 24 transposing reads; aoff / boff: the lane's byte offsets in a slot
__device__ __forceinline__ void gsw_frags(uint32_t slot_lds, const uint32_t (&aoff)[8], const uint32_t (&boff)[4],
                                          bf16x8 (&af)[8], bf16x8 (&bfr)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t a = slot_lds + boff[q];
    bfr[q] = cat4(lds_tr16_off<0>(a), lds_tr16_off<2048>(a));
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t a = slot_lds + aoff[i];
    af[i] = cat4(lds_tr16_off<0>(a), lds_tr16_off<2048>(a));
  }
}
}  // namespace

__global__ __launch_bounds__(512, 1) void gemm256s_wgrad_kernel(int M, int N, int K, const bf16* __restrict__ A,
                                                                long lda, const bf16* __restrict__ B, long ldb,
                                                                GemmEpi e, int ksplit, int kchunk,
                                                                float* __restrict__ slabs,
                                                                float* __restrict__ rowsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3, lw = wave & 3;
  const bool loader = wm == 1;
  const int nbm = M / G2, nbn = N / G2;
  const int ntiles = nbm * nbn;
  const int nwg = ntiles * ksplit;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;
  const uint32_t lds0 = lds_u32(smem);
  const int g = lane >> 4, c16 = lane & 15;
  uint32_t aoff[8], boff[4];
  {
    const int qq = c16 >> 2, p = c16 & 3;
    const int k0 = 8 * g + qq;
    const uint32_t cs4 = 4 * col_swz(k0);
#pragma unroll
    for (int i = 0; i < 8; ++i) aoff[i] = k0 * 512 + ((((uint32_t)(wm * 32 + i * 4 + p)) ^ cs4) << 3);
#pragma unroll
    for (int q = 0; q < 4; ++q) boff[q] = GS_OP + k0 * 512 + ((((uint32_t)(wn * 16 + q * 4 + p)) ^ cs4) << 3);
  }

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const int lin = xstart + jj;
    const int split = lin / ntiles, wgid = lin % ntiles;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int tn = within / gsz;
    const int m0 = (first_m + within % gsz) * G2, n0 = tn * G2;
    const int k_begin = split * kchunk, k_end = min(K, k_begin + kchunk);
    const int nk = (k_end - k_begin) / GS_KS;  // host: >= 1
    const bool rsum = rowsum != nullptr && tn == 0;
    const int wn_s = __builtin_amdgcn_readfirstlane(wn);

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float rs0 = 0.f, rs1 = 0.f;
    // column images: k-step k adds 32 k-rows
    const bf16* At = A + (long)k_begin * lda + m0;
    const bf16* Bt = B + (long)k_begin * ldb + n0;
    const long astep = (long)GS_KS * lda, bstep = (long)GS_KS * ldb;

    if (loader) {
      gsw_issue(lds0, At, lda, Bt, ldb, lw, lane);
      if (nk > 1) gsw_issue(lds0 + GS_SLOT, At + astep, lda, Bt + bstep, ldb, lw, lane);
      if (nk > 2) gsw_issue(lds0 + 2 * GS_SLOT, At + 2 * astep, lda, Bt + 2 * bstep, ldb, lw, lane);
      if (nk > 2) vm_wait<16>();
      else if (nk == 2) vm_wait<8>();
      else vm_wait<0>();
    }
    gs_bar();
    if (loader) gs_bar();

    for (int j = 0; j < nk; ++j) {
      bf16x8 bfr[4], af[8];
      gsw_frags(lds0 + (j & 3) * GS_SLOT, aoff, boff, af, bfr);
      const bool do_k = loader && j + 3 < nk;
      const uint32_t kslot = lds0 + ((j + 3) & 3) * GS_SLOT;
      const bf16* Aj = At + (long)(j + 3) * astep;
      const bf16* Bj = Bt + (long)(j + 3) * bstep;
      if (do_k) {
#pragma unroll
        for (int t = 4; t < 8; ++t) gsw_piece(t, kslot, Aj, lda, Bj, ldb, lw, lane);
      }
      if (loader) {
        if (j + 3 < nk) vm_wait<12>();
        else if (j + 3 == nk) vm_wait<8>();
        else if (j + 2 == nk) vm_wait<0>();
      }
      gs_bar();
      lds_tr_retire(af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] = mfma16(af[i], bfr[q], acc[i][q]);
        if ((i & 1) && do_k) {
          __builtin_amdgcn_sched_barrier(0);
          gsw_piece(i >> 1, kslot, Aj, lda, Bj, ldb, lw, lane);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (rsum) {  // wave wn sums A fragments 2wn, 2wn+1 (rows of its 32)
        if (wn_s == 0)      { rs0 = rowsum_frag(af[0], rs0); rs1 = rowsum_frag(af[1], rs1); }
        else if (wn_s == 1) { rs0 = rowsum_frag(af[2], rs0); rs1 = rowsum_frag(af[3], rs1); }
        else if (wn_s == 2) { rs0 = rowsum_frag(af[4], rs0); rs1 = rowsum_frag(af[5], rs1); }
        else                { rs0 = rowsum_frag(af[6], rs0); rs1 = rowsum_frag(af[7], rs1); }
      }
      __builtin_amdgcn_sched_barrier(0);
      gs_bar();
    }
    if (!loader) gs_bar();  // realign the halves (every wave past its last reads)

    if (rsum) {
      rs0 += __shfl_xor(rs0, 16); rs0 += __shfl_xor(rs0, 32);
      rs1 += __shfl_xor(rs1, 16); rs1 += __shfl_xor(rs1, 32);
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = m0 + wm * 128 + (2 * wn + j) * 16 + lane;
          const float v = j ? rs1 : rs0;
          if (ksplit > 1) rowsum[(long)split * M + row] = v;
          else rowsum[row] = (e.rs_accumulate ? rowsum[row] : 0.f) + v * e.alpha;
        }
      }
    }
    // ---- epilogue: eight 32-row passes through fp32 staging (slots 2-3);
    // the storers store every item (the loaders' rows 128..255 included)
    float* ep = reinterpret_cast<float*>(smem + GS_EP);
    float* slab = ksplit > 1 ? slabs + (long)split * M * N : nullptr;
    const int ch = tid & 31;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      if (wm == (pass >> 2)) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int i = 2 * (pass & 3) + ii;
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[gs_ep_idx(ii * 16 + 4 * g + r, wn * 64 + q * 16 + c16)] = acc[i][q][r];
        }
      }
      smer_lds_barrier();
      if (!loader) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int row = (tid >> 5) + 8 * c;  // 0..31
          const long grow = m0 + pass * GS_EPR + row;
          const int gcol = n0 + ch * 8;
          float4 a = *reinterpret_cast<const float4*>(ep + gs_ep_idx(row, ch * 8));
          float4 b = *reinterpret_cast<const float4*>(ep + gs_ep_idx(row, ch * 8) + 4);
          if (slab) {
            float* dst = slab + grow * N + gcol;
            *reinterpret_cast<float4*>(dst) = a;
            *reinterpret_cast<float4*>(dst + 4) = b;
          } else {
            float* dst = e.Cf + grow * e.ldcf + gcol;
            const float al = e.alpha;
            a.x *= al; a.y *= al; a.z *= al; a.w *= al;
            b.x *= al; b.y *= al; b.z *= al; b.w *= al;
            if (e.accumulate) {
              const float4 o0 = *reinterpret_cast<const float4*>(dst);
              const float4 o1 = *reinterpret_cast<const float4*>(dst + 4);
              a.x += o0.x; a.y += o0.y; a.z += o0.z; a.w += o0.w;
              b.x += o1.x; b.y += o1.y; b.z += o1.z; b.w += o1.w;
            }
            *reinterpret_cast<float4*>(dst) = a;
            *reinterpret_cast<float4*>(dst + 4) = b;
          }
        }
      }
      smer_lds_barrier();
    }
  }
}

// ---------------------------------------------------------------------------
// Skinny bf16 NT GEMM (M <= 256: decode steps, tiny batches).  The 128x128
// tile kernel would run 4-16 workgroups there; this one gives each
// workgroup a 64-row x 16-column output strip and splits K over its 8 waves.
// MFMA fragments are loaded straight from global memory (both operands are
// K-contiguous: every fragment is one 16-B load per lane), the 8 per-wave
// partial tiles are summed through LDS in fixed order (deterministic), then
// the shared epilogue runs on 8-column vectors.
// ---------------------------------------------------------------------------
namespace {
constexpr int SK_BM = 64, SK_BN = 16;
}
// The epilogue's bias / residual for one 8-column chunk, loaded BEFORE the K
// loop so that their HBM latency overlaps the operand loads (a decode-step
// GEMM is a handful of dependent memory round trips; this removes one).
// raw prefetched epilogue operands (converted at use: a conversion right
// behind the load makes hipcc wait for it there)
struct EpiPre {
  float4 b0, b1;
  bf16x8 r;
};
__device__ __forceinline__ bool epi_pre_ok(const GemmEpi& e, int M, int N, int row, int col) {
  return e.vec && row < M && col + 8 <= N;
}
// unconditional per thread (row / column clamped into the matrix; the
// caller uses the values only where epi_pre_ok holds): requested after the
// kernel's operand loads, a guarded form made every thread wait for it
// before issuing them
__device__ __forceinline__ void epi_prefetch_clamped(const GemmEpi& e, int M, int N, int row, int col, EpiPre& p) {
  if (!e.vec || N < 8) return;  // uniform
  const int c = min(col, N - 8), r = min(row, M - 1);
  if (e.bias) {
    p.b0 = *reinterpret_cast<const float4*>(e.bias + c);
    p.b1 = *reinterpret_cast<const float4*>(e.bias + c + 4);
  }
  if (e.residual) p.r = *reinterpret_cast<const bf16x8*>((const bf16*)e.residual + (long)r * e.ldr + c);
}
__device__ __forceinline__ void epi_prefetch(const GemmEpi& e, int row, int col, EpiPre& p) {
  if (e.bias) {
    p.b0 = *reinterpret_cast<const float4*>(e.bias + col);
    p.b1 = *reinterpret_cast<const float4*>(e.bias + col + 4);
  }
  if (e.residual) p.r = *reinterpret_cast<const bf16x8*>((const bf16*)e.residual + (long)row * e.ldr + col);
}
// epi_apply8 with the prefetched bias / residual (vector path only)
__device__ __forceinline__ void epi_apply8_pre(const GemmEpi& e, int row, int col, float (&v)[8],
                                               const EpiPre& p) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] *= e.alpha;
  if (e.bias) {
    const float pb[8] = {p.b0.x, p.b0.y, p.b0.z, p.b0.w, p.b1.x, p.b1.y, p.b1.z, p.b1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += pb[k];
  }
  if (e.relu) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  if (e.drop_thr) smer_drop8(smer_rowkey(e.seed, (uint32_t)row), e.drop_thr, e.drop_scale, (uint32_t)col, v);
  if (e.residual) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += (float)p.r[k];
  }
  GemmEpi e2 = e;  // the rest (gate, stores) through the shared path
  e2.alpha = 1.f; e2.bias = nullptr; e2.relu = 0; e2.drop_thr = 0; e2.residual = nullptr;
  epi_apply8(e2, row + 1, col + 8, row, col, v);
}

// Skinny bf16 NT GEMM (M <= 256: decode steps, tiny batches).  The 128x128
// tile kernel would run 4-16 workgroups there; this one gives each
// workgroup a 64-row x 16-column output strip and splits K over its NW
// waves, UNR 32-deep K steps per wave issued together (NW * UNR * 32 >= K
// in the decode shapes: one round of loads).  MFMA fragments are loaded
// straight from global memory (both operands K-contiguous: one 16-B load
// per lane per fragment); the NW partial tiles are summed through LDS in
// fixed order (deterministic), then the epilogue runs on 8-column vectors
// with its bias / residual already in registers.
// MI: 16-row fragments per workgroup (BM = 16 * MI rows).  A workgroup
// streams its BM rows of A and 16 rows of W over all of K, so its load time
// grows with (BM + 16) * K: MI = 1 quarters the A bytes per workgroup of
// the 64-row strip (4x the workgroups, each re-reading its W strip).
// KF (K % 32 == 0): every lane's 8-chunk of a valid K step is in range, so
// the operand loads are unconditional (rows / columns clamped into the
// matrices -- their outputs are dropped -- and steps past K reread the last
// step and skip their MFMAs): a guarded load (select behind it) made hipcc
// wait for each one.  The epilogue's bias / residual are requested after the
// operands (before: first, guarded, and waited for before any operand load).
template <int NW, int UNR, int MI = 4, bool KF = false>
__global__ __launch_bounds__(64 * NW) void gemm_skinny_bf16_kernel(int M, int N, int K,
                                                                   const bf16* __restrict__ A, long lda,
                                                                   const bf16* __restrict__ B, long ldb,
                                                                   GemmEpi e) {
  constexpr int BM = 16 * MI;
  __shared__ float red[NW][BM][SK_BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * SK_BN, m0 = blockIdx.y * BM;
  const int r16 = lane & 15, kq = (lane >> 4) * 8;
  const int ncol = n0 + r16;
  const bool colok = ncol < N;
  // epilogue chunk of this thread (tid < 128: row tid/2, 8 columns)
  const int erow = m0 + (tid >> 1), ecol = n0 + (tid & 1) * 8;
  const bool eth = tid < BM * 2;
  const bool pre = eth && epi_pre_ok(e, M, N, erow, ecol);
  EpiPre ep;
  if (!KF && pre) epi_prefetch(e, erow, ecol, ep);
  const bf16* bp = B + (long)(KF ? min(ncol, N - 1) : (colok ? ncol : 0)) * ldb + kq;
  const bf16* ap[MI];
  bool rowok[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = m0 + i * 16 + r16;
    rowok[i] = row < M;
    ap[i] = A + (long)(KF ? min(row, M - 1) : (rowok[i] ? row : 0)) * lda + kq;
  }
  f32x4 acc[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (K + 31) / 32;
  for (int s0 = wave; s0 < nsteps; s0 += NW * UNR) {
    bf16x8 a[UNR][MI], b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if constexpr (KF) {
        const int k = min(s0 + u * NW, nsteps - 1) * 32;
        b[u] = *reinterpret_cast<const bf16x8*>(bp + k);
#pragma unroll
        for (int i = 0; i < MI; ++i) a[u][i] = *reinterpret_cast<const bf16x8*>(ap[i] + k);
      } else {
        const int k = (s0 + u * NW) * 32;
        const bool kok = k + kq < K;  // K % 8 == 0: a lane's 8-chunk is all in or all out
        b[u] = (colok && kok) ? *reinterpret_cast<const bf16x8*>(bp + k) : bf16x8{};
#pragma unroll
        for (int i = 0; i < MI; ++i)
          a[u][i] = (rowok[i] && kok) ? *reinterpret_cast<const bf16x8*>(ap[i] + k) : bf16x8{};
      }
    }
    if (KF && s0 == wave) epi_prefetch_clamped(e, M, N, erow, ecol, ep);
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (!KF || s0 + u * NW < nsteps)  // wave-uniform
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[i] = mfma16(a[u][i], b[u], acc[i]);
  }
  if (KF && wave >= nsteps) epi_prefetch_clamped(e, M, N, erow, ecol, ep);  // waves with no K step
  // D[row 4g+r][col c16] of each 16x16 tile
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][i * 16 + 4 * g + r][r16] = acc[i][r];
  __syncthreads();
  if (eth) {
    const int row = tid >> 1, ch = tid & 1;
    if (erow < M && ecol < N) {
      float v[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[w][row][ch * 8 + c];
        v[c] = t;
      }
      if (pre) epi_apply8_pre(e, erow, ecol, v, ep);
      else epi_apply8(e, M, N, erow, ecol, v);
    }
  }
}

// Cf[m, n] (+)= alpha * sum_s slab[s][m][n]   (fixed order: deterministic);
// threads past M*N/4 reduce the fused bias-gradient partials the same way.
__global__ void splitk_reduce_kernel(int M, int N, int ksplit, const float* __restrict__ slabs,
                                     float alpha, float* __restrict__ Cf, long ldcf,
                                     int accumulate, const float* __restrict__ rs_part,
                                     float* __restrict__ rs_out, int rs_accumulate) {
  long idx = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  long MN = (long)M * N;
  if (idx >= MN) {
    const long m = ((long)blockIdx.x * blockDim.x + threadIdx.x) - MN / 4;
    if (rs_out == nullptr || m >= M) return;
    float t = 0.f;
    for (int s = 0; s < ksplit; ++s) t += rs_part[(long)s * M + m];
    rs_out[m] = (rs_accumulate ? rs_out[m] : 0.f) + alpha * t;
    return;
  }
  float4 a = *reinterpret_cast<const float4*>(slabs + idx);
  int s = 1;
  for (; s + 4 <= ksplit; s += 4) {  // four slices' loads in flight, summed in slice order
    float4 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(slabs + (long)(s + u) * MN + idx);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w;
    }
  }
  for (; s < ksplit; ++s) {
    float4 b = *reinterpret_cast<const float4*>(slabs + (long)s * MN + idx);
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  float v[4] = {a.x * alpha, a.y * alpha, a.z * alpha, a.w * alpha};
  if ((N & 3) == 0 && (ldcf & 3) == 0 && (((uintptr_t)Cf) & 15) == 0) {  // the 4 items share a row
    const long row = idx / N;
    float* p = Cf + row * ldcf + (idx - row * N);
    float4 o = make_float4(v[0], v[1], v[2], v[3]);
    if (accumulate) {
      const float4 c = *reinterpret_cast<const float4*>(p);
      o.x = c.x + o.x; o.y = c.y + o.y; o.z = c.z + o.z; o.w = c.w + o.w;
    }
    *reinterpret_cast<float4*>(p) = o;
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    long e = idx + t;
    int row = e / N, col = e % N;
    float* p = Cf + (long)row * ldcf + col;
    *p = accumulate ? *p + v[t] : v[t];
  }
}

// ---------------------------------------------------------------------------
// f32 VALU kernel (parity mode)
// ---------------------------------------------------------------------------
template <bool AK, bool BKC>
__global__ __launch_bounds__(256) void gemm_f32_kernel(int M, int N, int K,
                                                       const float* __restrict__ A, long lda,
                                                       const float* __restrict__ B, long ldb,
                                                       GemmEpi e) {
  __shared__ float As[16][68];
  __shared__ float Bs[16][68];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      int i = tid + 256 * c;
      int m, kk;
      if (AK) { m = i >> 4; kk = i & 15; } else { kk = i >> 6; m = i & 63; }
      int gm = m0 + m, gk = k0 + kk;
      float a = 0.f;
      if (gm < M && gk < K) a = AK ? A[(long)gm * lda + gk] : A[(long)gk * lda + gm];
      As[kk][m] = a;
      int n;
      if (BKC) { n = i >> 4; kk = i & 15; } else { kk = i >> 6; n = i & 63; }
      int gn = n0 + n;
      gk = k0 + kk;
      float b = 0.f;
      if (gn < N && gk < K) b = BKC ? B[(long)gn * ldb + gk] : B[(long)gk * ldb + gn];
      Bs[kk][n] = b;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      epi_apply<float>(e, M, N, m0 + ty * 4 + i, n0 + tx * 4 + j, acc[i][j]);
}

// ---------------------------------------------------------------------------
// Split-K (deterministic slabs) for a pure Cf (+)= A.B^T epilogue with few
// output tiles and a long K, i.e. the weight gradients (K = tokens): without
// it a [512 x 1536] wgrad occupies 48 of 256 CUs.
// SMER_GEMM_GLDS=0 forces register staging (A/B comparisons, tests).
static bool smer_gemm_glds_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_GEMM_GLDS");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// SMER_WGRAD_GLDS=0: register staging for the 128x128 weight gradients
// (round 5's workaround, see launch_bf16; A/B runs).  Default LDS-DMA since
// round 6: the non-repeatable overlapped step was the packed-FP32 fault
// (DESIGN.md section 8), not this kernel, and the library no longer
// contains packed-FP32 instructions
static bool smer_wgrad_glds() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD_GLDS");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// SMER_GEMM256=0 keeps every shape on the 128x128 kernel (A/B, tests).
static bool smer_gemm256_enabled() {
  const char* e = getenv("SMER_GEMM256");  // read per call: A/B scripts flip it in-process
  return !(e && e[0] == '0');
}

// Whole-tile bf16-output shapes: the staggered kernel where it measured
// faster than the two-stage one (tools/gemm256s_ab.py, round 4): K >= 1024
// (C2 FFN2 forward 69.7 vs 73.3 us, FFN1 / QKV dgrads 66.0 / 52.6 vs 71.1 /
// 56.6, C4 FFN1 dgrad 202 vs 224) and the NN dgrads with N >= 1024 (gated
// FFN2 dgrad 104.8 vs 116.9); the K = 512 forwards keep the two-stage kernel
// (FFN1 106.9 vs 101.8, QKV 68.8 vs 68.0: their epilogue, not the k-loop,
// sets the time).  SMER_GEMM256S=1 / 0 forces it on / off (read per call:
// A/B in-process).
static bool smer_gemm256s_enabled(bool bkc, int N, int K) {
  const char* e = getenv("SMER_GEMM256S");
  if (e && e[0] == '1') return true;
  if (e && e[0] == '0') return false;
  return K >= 1024 || (!bkc && N >= 1024);
}

// SMER_G256_NONPERSIST (read per call): 1 = the NN dgrad shapes of the
// 256x256 kernels run one workgroup per tile (grid = tiles) instead of a
// persistent grid of one per CU, so the hardware dispatcher balances tiles
// onto the CUs the side-stream weight gradients leave free; 2 = every
// 256x256 forward / dgrad; 0 = persistent everywhere
static int smer_g256_nonpersist() {
  const char* e = getenv("SMER_G256_NONPERSIST");
  return e ? atoi(e) : 0;
}

// SMER_G256_SKEW (A/B probe, read per call): start skew of the persistent
// 256x256 forward / dgrad kernels, in units of ~2k cycles (GemmEpi.skew)
static int smer_g256_skew() {
  const char* e = getenv("SMER_G256_SKEW");
  return e ? std::max(0, std::min(64, atoi(e))) : 0;
}

// SMER_GEMM64=0 keeps mid-size shapes on the 128x128 kernel (A/B, tests;
// read per call)
static bool smer_gemm64_enabled() {
  const char* e = getenv("SMER_GEMM64");
  return !(e && e[0] == '0');
}

static int smer_num_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// minimum K depth of a split-K slice (SMER_SPLITK_DEPTH overrides; A/B runs)
static int smer_splitk_depth() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_SPLITK_DEPTH");
    v = e ? std::max(64, atoi(e)) : 1024;
  }
  return v;
}

// Weight gradients on the 256x256 kernel for outputs of at least 1536 x 768
// (tools/bench_wgrad.py c4: 3072x768x65536 350 vs 426 us, 768x3072 316 vs
// 387, 2304x768 271 vs 315; 768x768 equal at K = 65536 and 54 vs 43 us at
// 16384; C4 step 90.1 vs 91.1 ms with every wgrad on it).  At C2's
// 512-wide outputs the 128x128 kernel with its smaller split-K slabs is as
// fast or faster.
// Round 5 sent every shape whose split-K fills the chip to it (the 128x128
// kernel then staged through registers: C2 13.66 vs 14.05 ms).  Round 6,
// with the 128x128 kernel on LDS-DMA again: outputs with both sides >= 768
// (or >= 1536 x 768) take it -- every C4 weight gradient (C4 fp8 84.5-85.0
// vs 85.6-86.3 ms with only the round-4 rule), no C2 one (C2 13.08-13.16 vs
// 13.19-13.22 ms with all of them; tools/ab_step.py, interleaved rounds).
// SMER_WGRAD256=2 (default) / 1 / 0: that rule / every shape / never (A/B);
// SMER_WGRAD256_DEPTH: minimum K depth of its split-K slices
static bool smer_wgrad256_enabled(int M, int N) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD256");
    v = (e && e[0] == '0') ? 0 : (e && e[0] == '1') ? 1 : 2;
  }
  return v == 1 || (v == 2 && ((long)M * N >= 1536L * 768 || (M >= 768 && N >= 768)));
}
// The 256x256 weight gradients on the staggered schedule
// (gemm256s_wgrad_kernel; tools/bench_wgrad.py c4: 2304x768x65536 249 vs
// 284 us, 3072x768 326 vs 356, 768x3072 302 vs 334, 768x768 equal);
// SMER_WGRAD256S=0: the two-stage gemm256_wgrad_kernel (read per call)
static bool smer_wgrad256s_enabled() {
  const char* e = getenv("SMER_WGRAD256S");
  return !(e && e[0] == '0');
}
// work items of the 256x256 weight-gradient grid (SMER_WGRAD256_SLOTS;
// default one per CU): fewer split-K slices write fewer fp32 slab bytes and
// leave CUs to the main stream's kernels (A/B runs)
// Cap on the persistent weight-gradient grids for the current call
// (smer_gemm_wgrad_bias_ex max_workgroups; 0 = none): a weight gradient
// running on a second stream beside the dgrad chain leaves the other CUs to
// that chain.  Set and cleared around one launch_bf16 call (host thread).
static thread_local long g_wgrad_cap = 0;
static long wgrad_cap(long v) { return g_wgrad_cap > 0 ? std::max(8L, std::min(v, g_wgrad_cap)) : v; }

static long smer_wgrad256_slots() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD256_SLOTS");
    v = e ? std::max(8, atoi(e)) : smer_num_cus();
  }
  return wgrad_cap(v);
}
static int smer_wgrad256_depth() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD256_DEPTH");
    v = e ? std::max(64, atoi(e)) : 512;
  }
  return v;
}

// 16-row decode Linear workgroups (SMER_SKINNY16=0: 64-row strips; A/B runs)
static bool smer_skinny16_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_SKINNY16");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

static long smer_skinny16_cap() {  // workgroups per CU (SMER_SKINNY16_CAP; A/B runs)
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_SKINNY16_CAP");
    v = e ? std::max(1, atoi(e)) : 2;
  }
  return v;
}

// Resident split-K workgroups per 2 CUs (SMER_WGRAD_WGP2: 4 = two per CU,
// the default since round 6 -- with the LDS-DMA 128x128 weight gradient back
// the overlapped C2 step is the same (13.09-13.13 vs 13.08-13.10 ms) and the
// serialised weight gradients run faster (GEMM family 0.244 vs 0.226 of
// peak, bench.py's live roofline); 2 = one per CU (round 5: C2 13.49 vs
// 13.56 ms with register staging); 1 = one per two CUs).  The weight gradients run on a second stream beside
// the main chain: a smaller persistent grid leaves CUs (and LDS) to the main
// stream's kernels and cuts the split-K slab bytes in proportion.
// SMER_WGRAD_STAGES = 2 / 3 / 4: LDS stages of the 128x128 split-K weight
// gradients at one resident workgroup per CU (A/B runs).  Default 2: the
// deeper rings hold 96 / 128 KiB of LDS per CU, which the concurrent main-
// stream kernels then cannot share (C2 step 13.28-13.33 ms at 2 stages,
// 13.52-13.56 at 3, 13.61-13.62 at 4; two interleaved rounds, one box)
static int smer_wgrad_stages() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD_STAGES");
    v = e ? std::max(2, std::min(4, atoi(e))) : 2;
  }
  return v;
}
// SMER_WGRAD_LDS_PAD (bytes, repeatability probes only): extra dynamic LDS
// requested by the LDS-DMA 128x128 weight gradient, so fewer other
// workgroups share its CU (160 KiB in all: the CU to itself as far as LDS goes)
static size_t smer_wgrad_lds_pad() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD_LDS_PAD");
    v = e ? std::max(0, std::min(96 * 1024, atoi(e))) : 0;
  }
  return (size_t)v;
}
static long smer_wgrad_resident() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_WGRAD_WGP2");
    v = e ? std::max(1, std::min(4, atoi(e))) : 4;
  }
  return wgrad_cap(std::max(8L, (v * (long)smer_num_cus()) / 2));
}

// fewest 256x256 tiles for which a forward / dgrad shape takes the 256x256
// kernel (SMER_G256_MIN, A/B runs; default: one per CU)
static long smer_g256_min_tiles() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_G256_MIN");
    v = e ? std::max(1, atoi(e)) : smer_num_cus();
  }
  return v;
}

// Split-K tickets (fused last-arriver reduction): the LAST SPLITK_TICKET_BYTES
// of a split-K workspace hold one u32 per output tile.  They must be zero
// when the workspace is first used (callers allocate it zeroed); every
// launch leaves them zero (the last arriver resets its tile's ticket).
constexpr size_t SPLITK_TICKET_BYTES = 64 * 1024;
// SMER_SPLITK_FUSED=1: the fused last-arriver reduction instead of the
// separate splitk_reduce_kernel (read per call).  Off by default: C2 step
// 13.64-16.62 ms fused vs 13.04-13.09 separate (three interleaved rounds,
// tools/ab_step.py, round 6) -- every slice waits for its 64 KiB of
// write-through slab stores before taking the ticket, and the last arriver
// sums the tile alone, both stalls of the persistent weight-gradient
// workgroups; bit-identical either way
static bool smer_splitk_fused() {
  const char* e = getenv("SMER_SPLITK_FUSED");
  return e && e[0] == '1';
}
static size_t splitk_slab_bytes(size_t ws_bytes) {
  return ws_bytes > SPLITK_TICKET_BYTES ? ws_bytes - SPLITK_TICKET_BYTES : 0;
}

static int choose_split(int M, int N, int K, const GemmEpi& e, size_t ws_bytes) {
  bool cf_only = e.Cf && !e.C && !e.bias && !e.residual && !e.gate && !e.relu && !e.drop_thr;
  if (!cf_only) return 1;
  long tiles = (long)((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  if (tiles >= 512 || K < 1024 || ((long)M * N) % 4 != 0) return 1;
  // ~2 resident workgroups per CU, K slices >= 1024 deep: more slices only
  // add slab traffic (split * M * N * 8 bytes through HBM)
  // (floor: a partial second wave of workgroups costs a whole slice time)
  long s = smer_wgrad_resident() / tiles;
  s = std::min<long>(s, K / smer_splitk_depth());
  // slabs of M*N floats plus M floats of row-sum partials per K slice
  s = std::min<long>(s, (long)(splitk_slab_bytes(ws_bytes) / (((size_t)M * N + M) * sizeof(float))));
  s = std::max<long>(1, std::min<long>(s, 64));
  return (int)s;
}

// SMER_SKINNY_KF=0: the skinny bf16 kernel's guarded-load form at every K (A/B runs)
static bool smer_skinny_kf() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_SKINNY_KF");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

template <bool AK, bool BKC>
static void launch_bf16(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                        const GemmEpi& e, void* ws, size_t ws_bytes, hipStream_t s,
                        float* rowsum = nullptr) {
  if (AK && BKC && M <= 4 * SK_BM && !rowsum) {
    const int nsteps = (K + 31) / 32;
    const int ntn = (N + SK_BN - 1) / SK_BN;
    // 16-row workgroups while that keeps the grid within two per CU
    // (per-workgroup load time, not the grid, bounds a decode Linear)
    const bool m16 = smer_skinny16_enabled() && (long)ntn * ((M + 15) / 16) <= smer_skinny16_cap() * smer_num_cus();
    const bool kf = K % 32 == 0 && smer_skinny_kf();
#define SKB(U, MI)                                                                                     \
  do {                                                                                                 \
    if (kf)                                                                                            \
      hipLaunchKernelGGL((gemm_skinny_bf16_kernel<8, U, MI, true>), grid, dim3(512), 0, s, M, N, K,    \
                         (const bf16*)A, lda, (const bf16*)B, ldb, e);                                 \
    else                                                                                               \
      hipLaunchKernelGGL((gemm_skinny_bf16_kernel<8, U, MI, false>), grid, dim3(512), 0, s, M, N, K,   \
                         (const bf16*)A, lda, (const bf16*)B, ldb, e);                                 \
  } while (0)
    if (m16) {
      const dim3 grid(ntn, (M + 15) / 16);
      if (nsteps > 16) SKB(4, 1);
      else SKB(2, 1);
      return;
    }
    const dim3 grid(ntn, (M + SK_BM - 1) / SK_BM);
    if (nsteps > 16) SKB(4, 4);  // 8 waves x 4 steps (16 waves would spill at 128 VGPRs)
    else SKB(2, 4);
#undef SKB
    return;
  }
  // large-M forward / dgrad: 256x256 tiles when they fill the chip
  if (AK && !rowsum && K % G2K == 0 && smer_gemm256_enabled()) {
    const long t2 = (long)((M + G2 - 1) / G2) * ((N + G2 - 1) / G2);
    // whole tiles with a bf16 output: the staggered kernel
    if (t2 >= smer_g256_min_tiles() && smer_gemm256s_enabled(BKC, N, K) && M % G2 == 0 && N % G2 == 0 &&
        K % GS_KS == 0 && K / GS_KS >= 4 && e.vec && e.C && !e.Cf && !e.kv && !e.q8 &&
        !(e.residual && e.gate)) {
      static bool attr_s = false;
      if (!attr_s) {
        hipFuncSetAttribute((const void*)gemm256s_bf16_kernel<true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
        hipFuncSetAttribute((const void*)gemm256s_bf16_kernel<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
        attr_s = true;
      }
      const int np = smer_g256_nonpersist();
      const bool whole = np == 2 || (np == 1 && !BKC);
      const int grid = (t2 > smer_num_cus() && !whole) ? (smer_num_cus() & ~7) : (int)t2;
      GemmEpi ed = e;
      ed.dbg = gemm_dbg_for(grid, s);
      ed.skew = smer_g256_skew();
      hipLaunchKernelGGL(gemm256s_bf16_kernel<BKC>, dim3(grid), dim3(512), G2_LDS, s,
                         M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, ed);
      return;
    }
    if (t2 >= smer_g256_min_tiles()) {
      const int np = smer_g256_nonpersist();
      const bool whole = np == 2 || (np == 1 && !BKC);
      const int grid = (t2 > smer_num_cus() && !whole) ? (smer_num_cus() & ~7) : (int)t2;
      static bool attr_set = false;  // > 64 KiB dynamic LDS must be opted into
      if (!attr_set) {
        hipFuncSetAttribute((const void*)gemm256_bf16_kernel<AK, BKC, false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
        hipFuncSetAttribute((const void*)gemm256_bf16_kernel<AK, BKC, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
        attr_set = true;
      }
      // streamed-epilogue variant: whole tiles, bf16 C only, at most one of
      // residual / gate
      const bool fast = e.vec && e.C && !e.Cf && !e.kv && M % G2 == 0 && N % G2 == 0 &&
                        !(e.residual && e.gate);
      auto kern = fast ? gemm256_bf16_kernel<AK, BKC, true> : gemm256_bf16_kernel<AK, BKC, false>;
      GemmEpi ek = e;
      ek.skew = smer_g256_skew();
      hipLaunchKernelGGL(kern, dim3(grid), dim3(512), G2_LDS, s,
                         M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, ek);
      return;
    }
  }
  // weight gradients (both operands column images, pure fp32 output): the
  // 256x256 tile when its split-K fills the chip with >= 512-deep slices
  if (!AK && !BKC && K % G2K == 0 && ws && smer_wgrad256_enabled(M, N)) {
    const bool cf_only = e.Cf && !e.C && !e.bias && !e.residual && !e.gate && !e.relu && !e.drop_thr &&
                         ((long)M * N) % 4 == 0;
    const long t2 = (long)((M + G2 - 1) / G2) * ((N + G2 - 1) / G2);
    const long cus = smer_num_cus();
    long ns = std::min<long>(smer_wgrad256_slots() / std::max<long>(1, t2), K / smer_wgrad256_depth());
    ns = std::min<long>(ns, (long)(splitk_slab_bytes(ws_bytes) / (((size_t)M * N + M) * sizeof(float))));
    ns = std::max<long>(1, std::min<long>(ns, 64));
    if (cf_only && t2 * ns * 4 >= 3 * cus) {
      int kchunk = (int)(((K + ns - 1) / ns + G2K - 1) / G2K * G2K);
      const int split = (K + kchunk - 1) / kchunk;
      static bool attr_set = false;
      if (!attr_set) {
        hipFuncSetAttribute((const void*)gemm256_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * G2_STAGE);
        attr_set = true;
      }
      float* rs_part = (split > 1 && rowsum) ? (float*)ws + (size_t)split * M * N : nullptr;
      const long nwg = t2 * split;
      const long gcap = wgrad_cap(cus);
      const int grid = nwg > gcap ? (int)(gcap & ~7L) : (int)nwg;
      if (smer_wgrad256s_enabled() && M % G2 == 0 && N % G2 == 0 && e.vec) {
        static bool attr_s = false;
        if (!attr_s) {
          hipFuncSetAttribute((const void*)gemm256s_wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              4 * GS_SLOT);
          attr_s = true;
        }
        hipLaunchKernelGGL(gemm256s_wgrad_kernel, dim3(grid), dim3(512), 4 * GS_SLOT, s, M, N, K,
                           (const bf16*)A, lda, (const bf16*)B, ldb, e, split, kchunk, (float*)ws,
                           split > 1 ? rs_part : rowsum);
      } else
      hipLaunchKernelGGL(gemm256_wgrad_kernel, dim3(grid), dim3(512), 2 * G2_STAGE, s, M, N, K,
                         (const bf16*)A, lda, (const bf16*)B, ldb, e, split, kchunk, (float*)ws,
                         split > 1 ? rs_part : rowsum);
      if (split > 1) {
        long n4 = ((long)M * N) / 4 + (rowsum ? M : 0);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((n4 + 255) / 256), dim3(256), 0, s, M, N, split,
                           (const float*)ws, e.alpha, e.Cf, e.ldcf, e.accumulate,
                           (const float*)rs_part, rowsum, e.rs_accumulate);
      }
      return;
    }
  }
  int tiles = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  int split = choose_split(M, N, K, e, ws ? ws_bytes : 0);
  // mid-size forward / dgrad: fewer 128x128 tiles than two per CU -> 64x128
  if (AK && !rowsum && split == 1 && K % GBK == 0 && tiles <= 4 * smer_num_cus() &&
      M > 4 * SK_BM && smer_gemm_glds_enabled() && smer_gemm64_enabled()) {
    const long t64 = (long)((M + 63) / 64) * ((N + GBN - 1) / GBN);
    const long res = 3L * smer_num_cus();
    const int grid = t64 > res ? (int)(res & ~7L) : (int)t64;
    hipLaunchKernelGGL((gemm64_bf16_kernel<BKC>), dim3(grid), dim3(256), 2 * G64_STAGE, s, M, N, K,
                       (const bf16*)A, lda, (const bf16*)B, ldb, e);
    return;
  }
  int kchunk = K;
  if (split > 1) {
    kchunk = ((K + split - 1) / split + GBK - 1) / GBK * GBK;
    split = (K + kchunk - 1) / kchunk;
  }
  float* rs_part = (split > 1 && rowsum) ? (float*)ws + (size_t)split * M * N : nullptr;
  // fused split-K reduction by the tile's last-arriving slice (no separate
  // reduce launch): whole float4 rows of dW
  unsigned* tickets = nullptr;
  if (split > 1 && smer_splitk_fused() && (N & 3) == 0 && (e.ldcf & 3) == 0 &&
      ((uintptr_t)e.Cf & 15) == 0 && (size_t)tiles * 4 <= SPLITK_TICKET_BYTES &&
      ws_bytes >= SPLITK_TICKET_BYTES)
    tickets = (unsigned*)((char*)ws + ws_bytes - SPLITK_TICKET_BYTES);
  // persistent grid: two resident workgroups per CU (LDS 64 KiB, <= 256 VGPRs);
  // split-K weight gradients: smer_wgrad_resident()
  const long nwg = (long)tiles * split;
  const long resident = split > 1 ? smer_wgrad_resident() : 2L * smer_num_cus();
  const int grid = nwg > resident ? (int)(resident & ~7L) : (int)nwg;
  // LDS-DMA staging needs whole 64-deep K steps in every slice.  (Round 5
  // staged the weight gradients through registers because with LDS-DMA the
  // overlapped step was not repeatable; round 6 traced that to packed-FP32
  // VALU results corrupted beside LDS-DMA on the same CU, DESIGN.md section
  // 8, and builds the library without them: SMER_WGRAD_GLDS=0 keeps the
  // register form for A/B runs)
  const bool gl = (K % GBK) == 0 && (kchunk % GBK) == 0 && smer_gemm_glds_enabled() &&
                  ((AK || BKC) || smer_wgrad_glds());
  if constexpr (!AK && !BKC) {
    // weight gradients at one resident workgroup per CU: the 3-stage ring
    const int ns = smer_wgrad_stages();
    if (gl && split > 1 && smer_wgrad_resident() <= smer_num_cus() && ns > 2) {
      static bool attr = false;
      if (!attr) {
        hipFuncSetAttribute((const void*)gemm_bf16_kernel<false, false, true, 3>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 6 * TILE_BYTES);
        hipFuncSetAttribute((const void*)gemm_bf16_kernel<false, false, true, 4>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 8 * TILE_BYTES);
        attr = true;
      }
      if (ns == 4)
        hipLaunchKernelGGL((gemm_bf16_kernel<false, false, true, 4>), dim3(grid), dim3(256), 8 * TILE_BYTES, s,
                           M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, e, split, kchunk, (float*)ws,
                           rs_part, tickets, rowsum);
      else
        hipLaunchKernelGGL((gemm_bf16_kernel<false, false, true, 3>), dim3(grid), dim3(256), 6 * TILE_BYTES, s,
                           M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, e, split, kchunk, (float*)ws,
                           rs_part, tickets, rowsum);
      goto reduce;
    }
  }
  {
    auto kern = gl ? gemm_bf16_kernel<AK, BKC, true> : gemm_bf16_kernel<AK, BKC, false>;
    size_t lds = 4 * TILE_BYTES;
    if (!AK && !BKC && gl && smer_wgrad_lds_pad()) {
      lds += smer_wgrad_lds_pad();
      static bool attr_pad = false;
      if (!attr_pad) {
        hipFuncSetAttribute((const void*)gemm_bf16_kernel<false, false, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_pad = true;
      }
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds,
                       s, M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, e, split, kchunk,
                       (float*)ws, split > 1 ? rs_part : rowsum, tickets, rowsum);
  }
reduce:
  if (split > 1 && !tickets) {
    long n4 = ((long)M * N) / 4 + (rowsum ? M : 0);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((n4 + 255) / 256), dim3(256), 0, s, M, N, split,
                       (const float*)ws, e.alpha, e.Cf, e.ldcf, e.accumulate,
                       (const float*)rs_part, rowsum, e.rs_accumulate);
  }
}
// Skinny f32 NT GEMM (parity-mode decode steps: M = 2 rows per request).
// Latency-bound: at M = 2 the step streams the fp32 weights (14.7 MB per C2
// decoder layer) with nothing else to do, so what counts is how many bytes
// are in flight at once.  A workgroup owns 4 output columns x up to 16 rows;
// lane (column lane >> 4, k-chunk lane & 15) of a wave step reads
// W[col][k + 4 (lane & 15) .. + 3] (4 columns x 64 k = 1 KiB per wave step),
// the 4 waves take the steps round-robin, 8 steps per wave in flight: a
// K = 2048 Linear issues all of its 32 KiB per workgroup up front, and the
// grid has N / 4 workgroups (128-512 at C2; round 3's 16-column strips ran
// N / 16 with 16 KiB in flight each).  Partial sums reduced over the 16
// lanes of a column by xor shuffles and over the waves through LDS, in fixed
// order (deterministic; a row's sum never depends on the other rows).
constexpr int SKF_BN = 4, SKF_BM = 16, SKF_NW = 4, SKF_UNR = 8;
__global__ __launch_bounds__(64 * SKF_NW) void gemm_skinny_f32_kernel(int M, int N, int K,
                                                                      const float* __restrict__ A, long lda,
                                                                      const float* __restrict__ B, long ldb,
                                                                      GemmEpi e) {
  __shared__ float red[SKF_NW][SKF_BM][SKF_BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = lane >> 4, kq = lane & 15;
  const int n0 = blockIdx.x * SKF_BN, m0 = blockIdx.y * SKF_BM;
  const int col = n0 + cq;
  const bool colok = col < N;
  const int mrows = min(SKF_BM, M - m0);
  const float* bp = B + (long)(colok ? col : 0) * ldb + 4 * kq;
  const float* a0 = A + (long)m0 * lda + 4 * kq;
  float acc[SKF_BM];
#pragma unroll
  for (int r = 0; r < SKF_BM; ++r) acc[r] = 0.f;
  const int nsteps = (K + 63) / 64;  // 64 k per wave step (16 lanes x 4)
  for (int s0 = wave; s0 < nsteps; s0 += SKF_NW * SKF_UNR) {
    float4 b[SKF_UNR];
#pragma unroll
    for (int u = 0; u < SKF_UNR; ++u) {
      const int k = (s0 + u * SKF_NW) * 64;
      b[u] = (colok && k + 4 * kq < K) ? *reinterpret_cast<const float4*>(bp + k) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < SKF_UNR; ++u) {
      const int k = (s0 + u * SKF_NW) * 64;
      if (k + 4 * kq >= K) continue;
#pragma unroll
      for (int r = 0; r < SKF_BM; ++r) {
        if (r < mrows) {
          const float4 a = *reinterpret_cast<const float4*>(a0 + (long)r * lda + k);
          acc[r] = fmaf(a.x, b[u].x, acc[r]);
          acc[r] = fmaf(a.y, b[u].y, acc[r]);
          acc[r] = fmaf(a.z, b[u].z, acc[r]);
          acc[r] = fmaf(a.w, b[u].w, acc[r]);
        }
      }
    }
  }
  // sum the 16 k-chunk lanes of each column, then the waves
#pragma unroll
  for (int r = 0; r < SKF_BM; ++r) {
    if (r < mrows) {
      acc[r] += __shfl_xor(acc[r], 1, 64);
      acc[r] += __shfl_xor(acc[r], 2, 64);
      acc[r] += __shfl_xor(acc[r], 4, 64);
      acc[r] += __shfl_xor(acc[r], 8, 64);
    }
  }
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < SKF_BM; ++r) red[wave][r][cq] = acc[r];
  }
  __syncthreads();
  if (tid < SKF_BM * SKF_BN) {
    const int r = tid / SKF_BN, c = tid % SKF_BN;
    if (r < mrows && n0 + c < N) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < SKF_NW; ++w) t += red[w][r][c];
      epi_apply<float>(e, M, N, m0 + r, n0 + c, t);
    }
  }
}

// fp32 NT GEMM on the fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 products and
// sums): the parity-mode prefill (encoder Linears and the cross K/V of a
// ~1k-token source) and fp32 training forwards.  64x64 tiles, 4 waves of
// 32x32 (2x2 MFMA blocks); the contraction of a 64-deep chunk runs in
// lane-group order (MFMA c sums k = 16 g + c over the lane groups g), so a
// lane streams 16 consecutive floats of one A row and one B row per block
// straight from global memory (the 4 waves share rows through L1).  Whole
// chunks are loaded unconditionally (rows outside M / N read row 0 and are
// dropped by the epilogue's bounds) into a ring of PD + 1 register buffers,
// PD chunks ahead of the MFMAs: the guarded loads of round 4 (a select
// behind each load) made hipcc wait for every outstanding load before each
// chunk's MFMAs (vmcnt(0)).  A partial last chunk (K % 64) is loaded
// guarded.  Measured (tools/gemm_f32_shapes.py, M = 1050 prefill shapes):
// the four encoder Linears 204.5 us per layer at PD = 2 vs 222.5 guarded;
// staging the chunks through a double-buffered LDS tile with coalesced
// 256-B row loads (same operands, 69.6 KB of LDS: two workgroups per CU)
// ran 248 us; a load pattern with whole rows per instruction (a timing
// probe with the wrong operands) 147-153 us, which needs the operands
// transposed across lanes.
template <int PD>
__global__ __launch_bounds__(256) void gemm_f32_mfma_kernel(int M, int N, int K, const float* __restrict__ A,
                                                            long lda, const float* __restrict__ B, long ldb,
                                                            GemmEpi e) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.y * 64 + (wave >> 1) * 32, n0 = blockIdx.x * 64 + (wave & 1) * 32;
  const float* ap[2];
  const float* bp[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = m0 + 16 * i + c16, c = n0 + 16 * i + c16;
    ap[i] = A + (long)(r < M ? r : 0) * lda + 16 * g;
    bp[i] = B + (long)(c < N ? c : 0) * ldb + 16 * g;
  }
  auto load = [&](int k0, float4 (&fa)[2][4], float4 (&fb)[2][4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        fa[i][t] = *reinterpret_cast<const float4*>(ap[i] + k0 + 4 * t);
        fb[i][t] = *reinterpret_cast<const float4*>(bp[i] + k0 + 4 * t);
      }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const float4 (&fa)[2][4], const float4 (&fb)[2][4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const float a = q == 0 ? fa[i][t].x : q == 1 ? fa[i][t].y : q == 2 ? fa[i][t].z : fa[i][t].w;
            const float b = q == 0 ? fb[j][t].x : q == 1 ? fb[j][t].y : q == 2 ? fb[j][t].z : fb[j][t].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
          }
  };
  const int nfull = K / 64;
  if (nfull > 0) {  // block-uniform
    float4 ra[PD + 1][2][4], rb[PD + 1][2][4];
#pragma unroll
    for (int p = 0; p < PD; ++p) load(64 * min(p, nfull - 1), ra[p], rb[p]);
    for (int c = 0; c < nfull; c += PD + 1) {
#pragma unroll
      for (int s = 0; s <= PD; ++s) {
        // chunk c + s sits in slot s; slot s - 1 (just consumed) takes chunk
        // c + s + PD (clamped: a redundant reload near the end)
        load(64 * min(c + s + PD, nfull - 1), ra[(s + PD) % (PD + 1)], rb[(s + PD) % (PD + 1)]);
        if (c + s < nfull) mma(ra[s], rb[s]);
      }
    }
  }
  if (K % 64) {  // partial last chunk: K % 4 == 0, a float4 is all in or all out
    float4 fa[2][4], fb[2][4];
    const int k0 = nfull * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bool kok = k0 + 16 * g + 4 * t < K;
        fa[i][t] = kok ? *reinterpret_cast<const float4*>(ap[i] + k0 + 4 * t) : make_float4(0, 0, 0, 0);
        fb[i][t] = kok ? *reinterpret_cast<const float4*>(bp[i] + k0 + 4 * t) : make_float4(0, 0, 0, 0);
      }
    mma(fa, fb);
  }
  // D[row 4g + r][col c16] of each block
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi_apply<float>(e, M, N, m0 + 16 * i + 4 * g + r, n0 + 16 * j + c16, acc[i][j][r]);
}

// SMER_GEMM_F32_MFMA=0 keeps fp32 NT shapes on the VALU tile kernel (A/B, tests)
static bool smer_gemm_f32_mfma() {
  const char* e = getenv("SMER_GEMM_F32_MFMA");
  return !(e && e[0] == '0');
}

static void launch_skinny_rows_f32(int M, int N, int K, const float* A, long lda, const float* W, long ldw,
                                   const GemmEpi& e, hipStream_t s);
// SMER_SKINNY_ROWS_F32=0: fp32 Linears of <= 64 rows on gemm_skinny_f32_kernel (A/B runs)
static bool smer_skinny_rows_f32() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SMER_SKINNY_ROWS_F32");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}
template <bool AK, bool BKC>
static void launch_f32(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                       const GemmEpi& e, hipStream_t s) {
  if (AK && BKC && M <= 64 && K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 &&
      (((uintptr_t)A | (uintptr_t)B) & 15) == 0) {
    if (K <= SKF_NW * SKF_UNR * 64 && smer_skinny_rows_f32()) {
      launch_skinny_rows_f32(M, N, K, (const float*)A, lda, (const float*)B, ldb, e, s);
      return;
    }
    const dim3 grid((N + SKF_BN - 1) / SKF_BN, (M + SKF_BM - 1) / SKF_BM);
    hipLaunchKernelGGL(gemm_skinny_f32_kernel, grid, dim3(64 * SKF_NW), 0, s, M, N, K, (const float*)A,
                       lda, (const float*)B, ldb, e);
    return;
  }
  dim3 grid((N + 63) / 64, (M + 63) / 64);
  if (AK && BKC && K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 &&
      (((uintptr_t)A | (uintptr_t)B) & 15) == 0 && smer_gemm_f32_mfma()) {
    hipLaunchKernelGGL(gemm_f32_mfma_kernel<2>, grid, dim3(256), 0, s, M, N, K, (const float*)A, lda,
                       (const float*)B, ldb, e);
    return;
  }
  hipLaunchKernelGGL((gemm_f32_kernel<AK, BKC>), grid, dim3(256), 0, s, M, N, K,
                     (const float*)A, lda, (const float*)B, ldb, e);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int smer_gemm(int dtype, int a_kcontig, int b_kcontig, int M, int N, int K,
                         const void* A, long lda, const void* B, long ldb, const float* bias,
                         float alpha, int relu, const void* residual, long ldr, const void* gate,
                         long ldg, float gate_scale, float drop_p, uint32_t drop_seed, void* C,
                         long ldc, float* Cf, long ldcf, int accumulate, void* workspace,
                         size_t ws_bytes, smer_stream_t stream) {
  SMER_REQUIRE(M >= 0 && N >= 0 && K >= 0, "smer_gemm: negative size");
  SMER_REQUIRE(A && B, "smer_gemm: null operand");
  SMER_REQUIRE(C || Cf, "smer_gemm: no output");
  SMER_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "smer_gemm: drop_p out of range");
  if (M == 0 || N == 0) return SMER_OK;
  GemmEpi e{};
  e.bias = bias; e.alpha = alpha; e.relu = relu; e.residual = residual; e.ldr = ldr;
  e.gate = gate; e.ldg = ldg; e.gate_scale = gate_scale;
  e.drop_thr = smer_drop_thr16(drop_p); e.seed = drop_seed;
  e.drop_scale = smer_drop_scale16(e.drop_thr);
  e.C = C; e.ldc = ldc; e.Cf = Cf; e.ldcf = ldcf; e.accumulate = accumulate;
  e.rs_accumulate = 0;
  auto a16 = [](const void* p, long ld) { return p == nullptr || ((((uintptr_t)p) & 15) == 0 && ld % 8 == 0); };
  e.vec = a16(bias, 8) && a16(residual, ldr) && a16(gate, ldg) && a16(C, ldc) && a16(Cf, ldcf);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SMER_BF16) {
    SMER_REQUIRE(K % 8 == 0, "smer_gemm(bf16): K must be a multiple of 8");
    SMER_REQUIRE(lda % 8 == 0 && ldb % 8 == 0, "smer_gemm(bf16): lda/ldb must be multiples of 8");
    SMER_REQUIRE(aligned16(A) && aligned16(B), "smer_gemm(bf16): operands must be 16-B aligned");
    SMER_REQUIRE(a_kcontig || lda >= (long)((M + 7) / 8) * 8,
                 "smer_gemm(bf16): column-image A needs lda >= round_up(M, 8)");
    SMER_REQUIRE(b_kcontig || ldb >= (long)((N + 7) / 8) * 8,
                 "smer_gemm(bf16): column-image B needs ldb >= round_up(N, 8)");
    SMER_REQUIRE(!workspace || aligned16(workspace), "smer_gemm: workspace alignment");
    if (K == 0) return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_gemm: K == 0");
    if (a_kcontig && b_kcontig) launch_bf16<true, true>(M, N, K, A, lda, B, ldb, e, workspace, ws_bytes, s);
    else if (a_kcontig) launch_bf16<true, false>(M, N, K, A, lda, B, ldb, e, workspace, ws_bytes, s);
    else if (b_kcontig) launch_bf16<false, true>(M, N, K, A, lda, B, ldb, e, workspace, ws_bytes, s);
    else launch_bf16<false, false>(M, N, K, A, lda, B, ldb, e, workspace, ws_bytes, s);
  } else if (dtype == SMER_F32) {
    if (a_kcontig && b_kcontig) launch_f32<true, true>(M, N, K, A, lda, B, ldb, e, s);
    else if (a_kcontig) launch_f32<true, false>(M, N, K, A, lda, B, ldb, e, s);
    else if (b_kcontig) launch_f32<false, true>(M, N, K, A, lda, B, ldb, e, s);
    else launch_f32<false, false>(M, N, K, A, lda, B, ldb, e, s);
  } else {
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_gemm: dtype");
  }
  SMER_CHECK_LAUNCH("smer_gemm");
  return SMER_OK;
}

extern "C" int smer_gemm_wgrad_bias(int dtype, int M, int N, int K, const void* dy, long lddy,
                                    const void* x, long ldx, float* dW, long lddw, int accumulate,
                                    float* db, int db_accumulate, void* workspace,
                                    size_t ws_bytes, smer_stream_t stream) {
  return smer_gemm_wgrad_bias_ex(dtype, M, N, K, dy, lddy, x, ldx, dW, lddw, accumulate, db,
                                 db_accumulate, workspace, ws_bytes, 0, stream);
}

extern "C" int smer_gemm_wgrad_bias_ex(int dtype, int M, int N, int K, const void* dy, long lddy,
                                       const void* x, long ldx, float* dW, long lddw, int accumulate,
                                       float* db, int db_accumulate, void* workspace,
                                       size_t ws_bytes, int max_workgroups, smer_stream_t stream) {
  SMER_REQUIRE(dtype == SMER_BF16, "smer_gemm_wgrad_bias: bf16 only (fp32: smer_gemm + smer_colsum)");
  SMER_REQUIRE(M > 0 && N > 0 && K > 0, "smer_gemm_wgrad_bias: bad sizes");
  SMER_REQUIRE(dy && x && dW && db, "smer_gemm_wgrad_bias: null pointer");
  SMER_REQUIRE(lddy % 8 == 0 && ldx % 8 == 0 && lddy >= (long)((M + 7) / 8) * 8 &&
                   ldx >= (long)((N + 7) / 8) * 8,
               "smer_gemm_wgrad_bias: dy / x row strides");
  SMER_REQUIRE(aligned16(dy) && aligned16(x) && (!workspace || aligned16(workspace)),
               "smer_gemm_wgrad_bias: 16-B alignment");
  GemmEpi e{};
  e.alpha = 1.f; e.drop_scale = 1.f;
  e.Cf = dW; e.ldcf = lddw; e.accumulate = accumulate; e.rs_accumulate = db_accumulate;
  auto a16 = [](const void* p, long ld) { return p == nullptr || ((((uintptr_t)p) & 15) == 0 && ld % 8 == 0); };
  e.vec = a16(dW, lddw);
  g_wgrad_cap = max_workgroups > 0 ? max_workgroups : 0;
  launch_bf16<false, false>(M, N, K, dy, lddy, x, ldx, e, workspace, ws_bytes, (hipStream_t)stream, db);
  g_wgrad_cap = 0;
  SMER_CHECK_LAUNCH("smer_gemm_wgrad_bias");
  return SMER_OK;
}

// ---------------------------------------------------------------------------
// Decode Linear with the post-norm LayerNorm in its prologue (decode steps:
// every LayerNorm of the decoder layer feeds a Linear, transformer.py:462,
// 466,469 -> 459/463/389 of the next sublayer).  A workgroup owns 16 rows x
// 16 output columns like the skinny kernel; it first normalises its 16 rows
// (one wave per row: ln_row_stats / ln_apply, the very arithmetic of
// ln_fwd_kernel, so the bits are the standalone LayerNorm's) into LDS —
// the workgroups of column strip 0 also store them (the residual the next
// sublayer adds) — then runs the K loop from LDS.  Saves the LayerNorm
// launch and its HBM round trip per norm (3 of the ~11 launches per layer).
// ---------------------------------------------------------------------------
// KF (K % 32 == 0, the decode shapes): the weight fragments, this wave's
// rows and gamma / beta are loaded unconditionally (column / row / chunk
// indices clamped: clamped rows are normalised too and dropped by the
// epilogue's bounds; nothing is stored for them), and the epilogue's bias /
// residual requested last -- the guarded loads (selects behind them) and the
// epilogue prefetch first made every workgroup wait for a load before
// issuing the next.  NC: 16-B row chunks per lane (K <= 512 NC).
template <int NW, int UNR, int NC = LNR_MAXC, bool KF = false>
__global__ __launch_bounds__(64 * NW) void gemm_skinny_ln_kernel(int M, int N, int K,
                                                                 const bf16* __restrict__ Y, long ldy,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float eps,
                                                                 bf16* __restrict__ X, long ldx,
                                                                 const bf16* __restrict__ B, long ldb,
                                                                 GemmEpi e) {
  constexpr int BM = 16;
  extern __shared__ __attribute__((aligned(16))) char xs[];  // BM rows x (2K + 32) bytes
  __shared__ float red[NW][BM][SK_BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * SK_BN, m0 = blockIdx.y * BM;
  const long xs_ld = 2L * K + 32;  // +32 B: fragment reads of 16 rows hit 16 distinct bank quads
  const int erow = m0 + (tid >> 1), ecol = n0 + (tid & 1) * 8;
  const bool eth = tid < BM * 2;
  const bool pre = eth && epi_pre_ok(e, M, N, erow, ecol);
  EpiPre ep;
  if (!KF && pre) epi_prefetch(e, erow, ecol, ep);
  // the weight fragments of the first K round are requested before the
  // LayerNorm prologue, so their HBM latency overlaps it (else two
  // dependent round trips: rows, then weights)
  const int r16 = lane & 15, kq = (lane >> 4) * 8;
  const int ncol = n0 + r16;
  const bool colok = ncol < N;
  const bf16* bp = B + (long)(KF ? min(ncol, N - 1) : (colok ? ncol : 0)) * ldb + kq;
  const int nsteps = (K + 31) / 32;
  bf16x8 b0[UNR];
#pragma unroll
  for (int u = 0; u < UNR; ++u) {
    const int k = (wave + u * NW) * 32;
    if constexpr (KF) b0[u] = *reinterpret_cast<const bf16x8*>(bp + min(k, (nsteps - 1) * 32));
    else b0[u] = (colok && k + kq < K) ? *reinterpret_cast<const bf16x8*>(bp + k) : bf16x8{};
  }
  const int nch = K >> 3;
  if constexpr (KF) {
    constexpr int RPW = BM / NW;  // rows per wave
    bf16x8 yv[RPW][NC];
    float4 gv[NC][2], bv[NC][2];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const bf16* yr = Y + (long)min(m0 + wave + NW * j, M - 1) * ldy;
#pragma unroll
      for (int c = 0; c < NC; ++c) yv[j][c] = *reinterpret_cast<const bf16x8*>(yr + 8 * min(lane + 64 * c, nch - 1));
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = min(lane + 64 * c, nch - 1);
      gv[c][0] = *reinterpret_cast<const float4*>(gamma + ch * 8);
      gv[c][1] = *reinterpret_cast<const float4*>(gamma + ch * 8 + 4);
      bv[c][0] = *reinterpret_cast<const float4*>(beta + ch * 8);
      bv[c][1] = *reinterpret_cast<const float4*>(beta + ch * 8 + 4);
    }
    epi_prefetch_clamped(e, M, N, erow, ecol, ep);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int rr = wave + NW * j, row = m0 + rr;
      char* dst = xs + rr * xs_ld;
      float v[NC][8], mu, rs;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = (float)yv[j][c][i];
      ln_stats_loaded<NC>(v, K, eps, lane, mu, rs);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + 64 * c;
        if (ch < nch) {
          const float g[8] = {gv[c][0].x, gv[c][0].y, gv[c][0].z, gv[c][0].w,
                              gv[c][1].x, gv[c][1].y, gv[c][1].z, gv[c][1].w};
          const float b[8] = {bv[c][0].x, bv[c][0].y, bv[c][0].z, bv[c][0].w,
                              bv[c][1].x, bv[c][1].y, bv[c][1].z, bv[c][1].w};
          bf16x8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (bf16)ln_apply(v[c][i], mu, rs, g[i], b[i]);
          *reinterpret_cast<bf16x8*>(dst + ch * 16) = o;
          if (X && blockIdx.x == 0 && row < M) *reinterpret_cast<bf16x8*>(X + (long)row * ldx + ch * 8) = o;
        }
      }
    }
  } else {
  for (int rr = wave; rr < BM; rr += NW) {  // wave-uniform
    const int row = m0 + rr;
    char* dst = xs + rr * xs_ld;
    if (row < M) {
      float v[LNR_MAXC][8], mu, rs;
      ln_row_stats<bf16>(Y + (long)row * ldy, K, eps, lane, v, mu, rs);
#pragma unroll
      for (int c = 0; c < LNR_MAXC; ++c) {
        const int ch = lane + 64 * c;
        if (ch < nch) {
          const float4 g0 = *reinterpret_cast<const float4*>(gamma + ch * 8);
          const float4 g1 = *reinterpret_cast<const float4*>(gamma + ch * 8 + 4);
          const float4 b0 = *reinterpret_cast<const float4*>(beta + ch * 8);
          const float4 b1 = *reinterpret_cast<const float4*>(beta + ch * 8 + 4);
          const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
          const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
          bf16x8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (bf16)ln_apply(v[c][i], mu, rs, g[i], b[i]);
          *reinterpret_cast<bf16x8*>(dst + ch * 16) = o;
          if (X && blockIdx.x == 0) *reinterpret_cast<bf16x8*>(X + (long)row * ldx + ch * 8) = o;
        }
      }
    } else {
      for (int ch = lane; ch < nch; ch += 64) *reinterpret_cast<bf16x8*>(dst + ch * 16) = bf16x8{};
    }
  }
  }
  __syncthreads();
  const char* ap = xs + r16 * xs_ld + kq * 2;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s0 = wave; s0 < nsteps; s0 += NW * UNR) {
    bf16x8 a[UNR], b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int k = (s0 + u * NW) * 32;
      const bool kok = k + kq < K;
      if (s0 == wave) b[u] = b0[u];
      else if (KF) b[u] = *reinterpret_cast<const bf16x8*>(bp + min(k, (nsteps - 1) * 32));
      else b[u] = (colok && kok) ? *reinterpret_cast<const bf16x8*>(bp + k) : bf16x8{};
      if (KF) a[u] = *reinterpret_cast<const bf16x8*>(ap + 2 * min(k, (nsteps - 1) * 32));
      else a[u] = kok ? *reinterpret_cast<const bf16x8*>(ap + 2 * k) : bf16x8{};
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (!KF || s0 + u * NW < nsteps)  // wave-uniform
        acc = mfma16(a[u], b[u], acc);
  }
  const int g = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][4 * g + r][r16] = acc[r];
  __syncthreads();
  if (eth) {
    const int row = tid >> 1, ch = tid & 1;
    if (erow < M && ecol < N) {
      float v[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[w][row][ch * 8 + c];
        v[c] = t;
      }
      if (pre) epi_apply8_pre(e, erow, ecol, v, ep);
      else epi_apply8(e, M, N, erow, ecol, v);
    }
  }
}

extern "C" int smer_linear_decode_ln(int M, int N, int K, const void* Y, long ldy, const float* gamma,
                                     const float* beta, float eps, void* X, long ldx, const void* W,
                                     long ldw, const float* bias, int relu, const void* residual,
                                     long ldr, void* C, long ldc, float* Cf, long ldcf, void* kv,
                                     long kv_row_stride, long kv_req_stride, const int32_t* kv_req,
                                     const int32_t* kv_pos, int kv_col0, smer_stream_t stream) {
  SMER_REQUIRE(M > 0 && M <= 4 * SK_BM && N > 0 && K > 0, "smer_linear_decode_ln: sizes (M <= 256)");
  SMER_REQUIRE(K % 8 == 0 && K <= 64 * 8 * LNR_MAXC, "smer_linear_decode_ln: K % 8 == 0 and K <= 2048");
  SMER_REQUIRE(Y && W && gamma && beta && (C || Cf), "smer_linear_decode_ln: null operand");
  SMER_REQUIRE(ldy % 8 == 0 && ldw % 8 == 0 && aligned16(Y) && aligned16(W) && aligned16(gamma) &&
                   aligned16(beta) && (!X || (aligned16(X) && ldx % 8 == 0)),
               "smer_linear_decode_ln: strides / alignment");
  SMER_REQUIRE(!kv || (kv_req && kv_pos && kv_col0 % 8 == 0 && kv_col0 >= 0 && kv_col0 < N &&
                       aligned16(kv) && kv_row_stride % 8 == 0 && kv_req_stride % 8 == 0),
               "smer_linear_decode_ln: kv scatter arguments");
  GemmEpi e{};
  e.bias = bias; e.alpha = 1.f; e.relu = relu; e.residual = residual; e.ldr = ldr;
  e.drop_scale = 1.f; e.C = C; e.ldc = ldc; e.Cf = Cf; e.ldcf = ldcf;
  e.kv = kv; e.kv_row_stride = kv_row_stride; e.kv_req_stride = kv_req_stride;
  e.kv_req = kv_req; e.kv_pos = kv_pos; e.kv_col0 = kv_col0;
  auto a16 = [](const void* p, long ld) { return p == nullptr || ((((uintptr_t)p) & 15) == 0 && ld % 8 == 0); };
  e.vec = a16(bias, 8) && a16(residual, ldr) && a16(C, ldc) && a16(Cf, ldcf);
  const dim3 grid((N + SK_BN - 1) / SK_BN, (M + 15) / 16);
  const size_t lds = 16 * (2 * (size_t)K + 32);
  hipStream_t s = (hipStream_t)stream;
#define SKLN(U, NC, KF)                                                                                  \
  hipLaunchKernelGGL((gemm_skinny_ln_kernel<8, U, NC, KF>), grid, dim3(512), lds, s, M, N, K, (const bf16*)Y, \
                     ldy, gamma, beta, eps, (bf16*)X, ldx, (const bf16*)W, ldw, e)
  if (K % 32 == 0 && smer_skinny_kf()) {
    if (K <= 512) SKLN(2, 1, true);
    else if (K <= 1024) SKLN(4, 2, true);
    else SKLN(4, 4, true);
  } else if ((K + 31) / 32 > 16) {
    SKLN(4, LNR_MAXC, false);
  } else {
    SKLN(2, LNR_MAXC, false);
  }
#undef SKLN
  SMER_CHECK_LAUNCH("smer_linear_decode_ln");
  return SMER_OK;
}

extern "C" int smer_linear_decode(int M, int N, int K, const void* A, long lda, const void* W,
                                  long ldw, const float* bias, int relu, const void* residual,
                                  long ldr, void* C, long ldc, float* Cf, long ldcf, void* kv,
                                  long kv_row_stride, long kv_req_stride, const int32_t* kv_req,
                                  const int32_t* kv_pos, int kv_col0, smer_stream_t stream) {
  SMER_REQUIRE(M > 0 && M <= 4 * SK_BM && N > 0 && K > 0, "smer_linear_decode: sizes (M <= 256)");
  SMER_REQUIRE(A && W && (C || Cf), "smer_linear_decode: null operand");
  SMER_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldw % 8 == 0 && aligned16(A) && aligned16(W),
               "smer_linear_decode: K / strides / alignment");
  SMER_REQUIRE(!kv || (kv_req && kv_pos && kv_col0 % 8 == 0 && kv_col0 >= 0 && kv_col0 < N &&
                       aligned16(kv) && kv_row_stride % 8 == 0 && kv_req_stride % 8 == 0),
               "smer_linear_decode: kv scatter arguments");
  GemmEpi e{};
  e.bias = bias; e.alpha = 1.f; e.relu = relu; e.residual = residual; e.ldr = ldr;
  e.drop_scale = 1.f; e.C = C; e.ldc = ldc; e.Cf = Cf; e.ldcf = ldcf;
  e.kv = kv; e.kv_row_stride = kv_row_stride; e.kv_req_stride = kv_req_stride;
  e.kv_req = kv_req; e.kv_pos = kv_pos; e.kv_col0 = kv_col0;
  auto a16 = [](const void* p, long ld) { return p == nullptr || ((((uintptr_t)p) & 15) == 0 && ld % 8 == 0); };
  e.vec = a16(bias, 8) && a16(residual, ldr) && a16(C, ldc) && a16(Cf, ldcf);
  launch_bf16<true, true>(M, N, K, A, lda, W, ldw, e, nullptr, 0, (hipStream_t)stream);
  SMER_CHECK_LAUNCH("smer_linear_decode");
  return SMER_OK;
}

// fp32 decode Linear with the post-norm LayerNorm in its prologue (the
// parity-mode decode step: LN3 -> next QKV, LN1 -> cross Q, LN2 -> FFN1,
// final norm -> vocab head), gemm_skinny_f32_kernel's 4-column workgroups.
// The weights of the (single, K <= 2048) load round are requested first, so
// their HBM latency overlaps the row statistics; each workgroup normalises
// its rows into LDS with ln_row_stats / ln_apply (the fp32 LayerNorm
// kernel's arithmetic: same bits), workgroup 0 also stores them to X.
// LN = false (smer_linear_decode_f32 and fp32 Linears of <= 64 rows with
// K <= 2048): the rows are copied into LDS unchanged -- the same products in
// the same order as gemm_skinny_f32_kernel, whose row loads sat behind the
// weight loads in one dependent chain per k step.  The weight loads are
// unconditional (column clamped to N - 1, k to K - 4; the FMAs skip k >= K):
// the guarded loads of round 4 left a phi copy behind the second load, so
// every workgroup waited for it (vmcnt(0)) before requesting the rest.
template <bool LN>
__global__ __launch_bounds__(64 * SKF_NW) void gemm_skinny_ln_f32_kernel(int M, int N, int K,
                                                                         const float* __restrict__ Y, long ldy,
                                                                         const float* __restrict__ gamma,
                                                                         const float* __restrict__ beta, float eps,
                                                                         float* __restrict__ X, long ldx,
                                                                         const float* __restrict__ B, long ldb,
                                                                         GemmEpi e) {
  extern __shared__ __attribute__((aligned(16))) char xs_raw[];
  float* xs = reinterpret_cast<float*>(xs_raw);  // mrows x K
  __shared__ float red[SKF_NW][SKF_BM][SKF_BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = lane >> 4, kq = lane & 15;
  const int n0 = blockIdx.x * SKF_BN, m0 = blockIdx.y * SKF_BM;
  const int col = n0 + cq;
  const int mrows = min(SKF_BM, M - m0);
  const float* bp = B + (long)min(col, N - 1) * ldb;
  // this wave's first row (and the LayerNorm's gamma / beta) requested up
  // front with the weights (hipcc issues the weight loads first whatever the
  // source order -- a memory clobber or sched_barrier between them does not
  // keep the rows ahead -- so the row work still waits for both: vmcnt
  // counts in order).  Chunk indices are clamped, not guarded: a clamped
  // chunk rereads (and rewrites) the row's last one.
  const int nch = K >> 3, n4 = K >> 2;
  const float* y0 = Y + (long)(m0 + min(wave, mrows - 1)) * ldy;
  float4 t[SKF_UNR];  // !LN: the first row, 16 B per lane per chunk
  float v0[LNR_MAXC][8], gv[LNR_MAXC][8], bv[LNR_MAXC][8];  // LN: 32 B per lane per chunk
  if constexpr (LN) {
#pragma unroll
    for (int c = 0; c < LNR_MAXC; ++c) {
      const int ch = min(lane + 64 * c, nch - 1);
      load8<float>(y0 + ch * 8, 8, v0[c]);
      load8<float>(gamma + ch * 8, 8, gv[c]);
      load8<float>(beta + ch * 8, 8, bv[c]);
    }
  } else {
#pragma unroll
    for (int c = 0; c < SKF_UNR; ++c) t[c] = *reinterpret_cast<const float4*>(y0 + 4 * min(lane + 64 * c, n4 - 1));
  }
  float4 b[SKF_UNR];
#pragma unroll
  for (int u = 0; u < SKF_UNR; ++u) {
    const int k = (wave + u * SKF_NW) * 64 + 4 * kq;
    b[u] = *reinterpret_cast<const float4*>(bp + min(k, K - 4));
  }
  if constexpr (!LN) {
    for (int rr = wave; rr < mrows; rr += SKF_NW) {  // wave-uniform
      if (rr != wave) {
        const float* yr = Y + (long)(m0 + rr) * ldy;
#pragma unroll
        for (int c = 0; c < SKF_UNR; ++c) t[c] = *reinterpret_cast<const float4*>(yr + 4 * min(lane + 64 * c, n4 - 1));
      }
#pragma unroll
      for (int c = 0; c < SKF_UNR; ++c) *reinterpret_cast<float4*>(xs + rr * K + 4 * min(lane + 64 * c, n4 - 1)) = t[c];
    }
  }
  for (int rr = wave; LN && rr < mrows; rr += SKF_NW) {  // wave-uniform
    const int row = m0 + rr;
    float v[LNR_MAXC][8], mu, rs;
    if (rr == wave) {
#pragma unroll
      for (int c = 0; c < LNR_MAXC; ++c)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = v0[c][i];
      ln_stats_loaded(v, K, eps, lane, mu, rs);
    } else {
      ln_row_stats<float>(Y + (long)row * ldy, K, eps, lane, v, mu, rs);
    }
#pragma unroll
    for (int c = 0; c < LNR_MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = ln_apply(v[c][i], mu, rs, gv[c][i], bv[c][i]);
        float* dst = xs + rr * K + ch * 8;
        *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(o[4], o[5], o[6], o[7]);
        if (X && blockIdx.x == 0) {
          float* xo = X + (long)row * ldx + ch * 8;
          *reinterpret_cast<float4*>(xo) = make_float4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<float4*>(xo + 4) = make_float4(o[4], o[5], o[6], o[7]);
        }
      }
    }
  }
  __syncthreads();
  float acc[SKF_BM];
#pragma unroll
  for (int r = 0; r < SKF_BM; ++r) acc[r] = 0.f;
#pragma unroll
  for (int u = 0; u < SKF_UNR; ++u) {
    const int k = (wave + u * SKF_NW) * 64 + 4 * kq;
    if (k >= K) continue;
#pragma unroll
    for (int r = 0; r < SKF_BM; ++r) {
      if (r < mrows) {
        const float4 a = *reinterpret_cast<const float4*>(xs + r * K + k);
        acc[r] = fmaf(a.x, b[u].x, acc[r]);
        acc[r] = fmaf(a.y, b[u].y, acc[r]);
        acc[r] = fmaf(a.z, b[u].z, acc[r]);
        acc[r] = fmaf(a.w, b[u].w, acc[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < SKF_BM; ++r) {
    if (r < mrows) {
      acc[r] += __shfl_xor(acc[r], 1, 64);
      acc[r] += __shfl_xor(acc[r], 2, 64);
      acc[r] += __shfl_xor(acc[r], 4, 64);
      acc[r] += __shfl_xor(acc[r], 8, 64);
    }
  }
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < SKF_BM; ++r) red[wave][r][cq] = acc[r];
  }
  __syncthreads();
  if (tid < SKF_BM * SKF_BN) {
    const int r = tid / SKF_BN, c = tid % SKF_BN;
    if (r < mrows && n0 + c < N) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < SKF_NW; ++w) t += red[w][r][c];
      epi_apply<float>(e, M, N, m0 + r, n0 + c, t);
    }
  }
}

// up to 128 KiB of dynamic LDS (16 rows x 2048) for the LDS-row skinny kernels
static void skinny_f32_lds_attr() {
  static bool set = false;
  if (!set) {
    hipFuncSetAttribute((const void*)gemm_skinny_ln_f32_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        SKF_BM * 2048 * (int)sizeof(float));
    hipFuncSetAttribute((const void*)gemm_skinny_ln_f32_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        SKF_BM * 2048 * (int)sizeof(float));
    set = true;
  }
}
// fp32 Linear of <= 64 rows, K <= 2048 (K % 4 == 0, 16-B aligned rows):
// rows through LDS, all weight loads of the single round issued first
static void launch_skinny_rows_f32(int M, int N, int K, const float* A, long lda, const float* W, long ldw,
                                   const GemmEpi& e, hipStream_t s) {
  skinny_f32_lds_attr();
  const dim3 grid((N + SKF_BN - 1) / SKF_BN, (M + SKF_BM - 1) / SKF_BM);
  const size_t lds = (size_t)std::min(M, SKF_BM) * K * sizeof(float);
  hipLaunchKernelGGL(gemm_skinny_ln_f32_kernel<false>, grid, dim3(64 * SKF_NW), lds, s, M, N, K, A, lda,
                     (const float*)nullptr, (const float*)nullptr, 0.f, (float*)nullptr, 0L, W, ldw, e);
}

// fp32 decode Linear whose input rows are the attention output merged from
// smer_attn_decode_split_f32's per-slice partials (the cross-attention
// out-projection of the plugin's fp32 step): the prologue merges the NS = 8
// {m, l, acc} records of each (row, head) in fixed order into LDS rows
// (o = sum_s e^(m_s - m) acc_s / sum_s e^(m_s - m) l_s), then the GEMM of
// gemm_skinny_ln_f32_kernel.  The weights of the single load round are
// requested first.
constexpr int DEC_NS = 8;
__global__ __launch_bounds__(64 * SKF_NW) void gemm_skinny_merge_f32_kernel(int M, int N, int K,
                                                                            const float* __restrict__ part,
                                                                            const float* __restrict__ B, long ldb,
                                                                            GemmEpi e) {
  extern __shared__ __attribute__((aligned(16))) char xs_raw[];
  float* xs = reinterpret_cast<float*>(xs_raw);  // mrows x K
  __shared__ float red[SKF_NW][SKF_BM][SKF_BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = lane >> 4, kq = lane & 15;
  const int n0 = blockIdx.x * SKF_BN, m0 = blockIdx.y * SKF_BM;
  const int col = n0 + cq;
  const int mrows = min(SKF_BM, M - m0);
  const float* bp = B + (long)min(col, N - 1) * ldb;
  float4 b[SKF_UNR];
#pragma unroll
  for (int u = 0; u < SKF_UNR; ++u) {  // unconditional (see gemm_skinny_ln_f32_kernel)
    const int k = (wave + u * SKF_NW) * 64 + 4 * kq;
    b[u] = *reinterpret_cast<const float4*>(bp + min(k, K - 4));
  }
  const int H = K / 64;
  for (int t = wave; t < mrows * H; t += SKF_NW) {  // wave-uniform: (row, head) records
    const int rr = t / H, hh = t % H;
    const float* pr = part + ((long)(m0 + rr) * H + hh) * DEC_NS * 68;
    float ms = -INFINITY;
#pragma unroll
    for (int z = 0; z < DEC_NS; ++z) ms = fmaxf(ms, pr[z * 68]);
    float L = 0.f, o = 0.f;
#pragma unroll
    for (int z = 0; z < DEC_NS; ++z) {
      const float mz = pr[z * 68];
      const float w = mz == -INFINITY ? 0.f : __expf(mz - ms);
      L += pr[z * 68 + 1] * w;
      o += pr[z * 68 + 4 + lane] * w;
    }
    xs[rr * K + hh * 64 + lane] = o * (L > 0.f ? 1.f / L : 0.f);
  }
  __syncthreads();
  float acc[SKF_BM];
#pragma unroll
  for (int r = 0; r < SKF_BM; ++r) acc[r] = 0.f;
#pragma unroll
  for (int u = 0; u < SKF_UNR; ++u) {
    const int k = (wave + u * SKF_NW) * 64 + 4 * kq;
    if (k >= K) continue;
#pragma unroll
    for (int r = 0; r < SKF_BM; ++r) {
      if (r < mrows) {
        const float4 a = *reinterpret_cast<const float4*>(xs + r * K + k);
        acc[r] = fmaf(a.x, b[u].x, acc[r]);
        acc[r] = fmaf(a.y, b[u].y, acc[r]);
        acc[r] = fmaf(a.z, b[u].z, acc[r]);
        acc[r] = fmaf(a.w, b[u].w, acc[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < SKF_BM; ++r) {
    if (r < mrows) {
      acc[r] += __shfl_xor(acc[r], 1, 64);
      acc[r] += __shfl_xor(acc[r], 2, 64);
      acc[r] += __shfl_xor(acc[r], 4, 64);
      acc[r] += __shfl_xor(acc[r], 8, 64);
    }
  }
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < SKF_BM; ++r) red[wave][r][cq] = acc[r];
  }
  __syncthreads();
  if (tid < SKF_BM * SKF_BN) {
    const int r = tid / SKF_BN, c = tid % SKF_BN;
    if (r < mrows && n0 + c < N) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < SKF_NW; ++w) t += red[w][r][c];
      epi_apply<float>(e, M, N, m0 + r, n0 + c, t);
    }
  }
}

static GemmEpi decode_epi(const float* bias, int relu, const void* residual, long ldr, void* C, long ldc,
                          float* Cf, long ldcf, void* kv, long kv_row_stride, long kv_req_stride,
                          const int32_t* kv_req, const int32_t* kv_pos, int kv_col0) {
  GemmEpi e{};
  e.bias = bias; e.alpha = 1.f; e.relu = relu; e.residual = residual; e.ldr = ldr;
  e.drop_scale = 1.f; e.C = C; e.ldc = ldc; e.Cf = Cf; e.ldcf = ldcf;
  e.kv = kv; e.kv_row_stride = kv_row_stride; e.kv_req_stride = kv_req_stride;
  e.kv_req = kv_req; e.kv_pos = kv_pos; e.kv_col0 = kv_col0;
  return e;
}

// fp32 smer_linear_decode (parity-mode decode step): every operand fp32
extern "C" int smer_linear_decode_f32(int M, int N, int K, const void* A, long lda, const void* W,
                                      long ldw, const float* bias, int relu, const void* residual,
                                      long ldr, void* C, long ldc, float* Cf, long ldcf, void* kv,
                                      long kv_row_stride, long kv_req_stride, const int32_t* kv_req,
                                      const int32_t* kv_pos, int kv_col0, smer_stream_t stream) {
  SMER_REQUIRE(M > 0 && M <= 64 && N > 0 && K > 0, "smer_linear_decode_f32: sizes (M <= 64)");
  SMER_REQUIRE(A && W && (C || Cf), "smer_linear_decode_f32: null operand");
  SMER_REQUIRE(K % 4 == 0 && lda % 4 == 0 && ldw % 4 == 0 && aligned16(A) && aligned16(W),
               "smer_linear_decode_f32: K / strides / alignment");
  SMER_REQUIRE(!kv || (kv_req && kv_pos && kv_col0 >= 0 && kv_col0 < N), "smer_linear_decode_f32: kv scatter arguments");
  const GemmEpi e = decode_epi(bias, relu, residual, ldr, C, ldc, Cf, ldcf, kv, kv_row_stride, kv_req_stride,
                               kv_req, kv_pos, kv_col0);
  if (K <= SKF_NW * SKF_UNR * 64 && smer_skinny_rows_f32()) {
    launch_skinny_rows_f32(M, N, K, (const float*)A, lda, (const float*)W, ldw, e, (hipStream_t)stream);
  } else {
    const dim3 grid((N + SKF_BN - 1) / SKF_BN, (M + SKF_BM - 1) / SKF_BM);
    hipLaunchKernelGGL(gemm_skinny_f32_kernel, grid, dim3(64 * SKF_NW), 0, (hipStream_t)stream, M, N, K,
                       (const float*)A, lda, (const float*)W, ldw, e);
  }
  SMER_CHECK_LAUNCH("smer_linear_decode_f32");
  return SMER_OK;
}

// fp32 smer_linear_decode_ln
extern "C" int smer_linear_decode_ln_f32(int M, int N, int K, const void* Y, long ldy, const float* gamma,
                                         const float* beta, float eps, void* X, long ldx, const void* W,
                                         long ldw, const float* bias, int relu, const void* residual,
                                         long ldr, void* C, long ldc, float* Cf, long ldcf, void* kv,
                                         long kv_row_stride, long kv_req_stride, const int32_t* kv_req,
                                         const int32_t* kv_pos, int kv_col0, smer_stream_t stream) {
  SMER_REQUIRE(M > 0 && M <= 64 && N > 0 && K > 0, "smer_linear_decode_ln_f32: sizes (M <= 64)");
  SMER_REQUIRE(K % 8 == 0 && K <= SKF_NW * SKF_UNR * 64 && K <= 64 * 8 * LNR_MAXC,
               "smer_linear_decode_ln_f32: K % 8 == 0 and K <= 2048");
  SMER_REQUIRE(Y && W && gamma && beta && (C || Cf), "smer_linear_decode_ln_f32: null operand");
  SMER_REQUIRE(ldy % 4 == 0 && ldw % 4 == 0 && aligned16(Y) && aligned16(W) &&
                   (!X || (aligned16(X) && ldx % 4 == 0)),
               "smer_linear_decode_ln_f32: strides / alignment");
  SMER_REQUIRE(!kv || (kv_req && kv_pos && kv_col0 >= 0 && kv_col0 < N), "smer_linear_decode_ln_f32: kv scatter arguments");
  const GemmEpi e = decode_epi(bias, relu, residual, ldr, C, ldc, Cf, ldcf, kv, kv_row_stride, kv_req_stride,
                               kv_req, kv_pos, kv_col0);
  const dim3 grid((N + SKF_BN - 1) / SKF_BN, (M + SKF_BM - 1) / SKF_BM);
  const size_t lds = (size_t)std::min(M, SKF_BM) * K * sizeof(float);
  skinny_f32_lds_attr();
  hipLaunchKernelGGL(gemm_skinny_ln_f32_kernel<true>, grid, dim3(64 * SKF_NW), lds, (hipStream_t)stream, M, N, K,
                     (const float*)Y, ldy, gamma, beta, eps, (float*)X, ldx, (const float*)W, ldw, e);
  SMER_CHECK_LAUNCH("smer_linear_decode_ln_f32");
  return SMER_OK;
}

// fp32 decode Linear on the merged split-attention partials (see above)
extern "C" int smer_linear_decode_merge_f32(int M, int N, int K, const float* part, const void* W, long ldw,
                                            const float* bias, int relu, const void* residual, long ldr, void* C,
                                            long ldc, float* Cf, long ldcf, smer_stream_t stream) {
  SMER_REQUIRE(M > 0 && M <= 64 && N > 0 && K > 0 && K % 64 == 0 && K <= SKF_NW * SKF_UNR * 64,
               "smer_linear_decode_merge_f32: sizes (M <= 64, K = 64 * heads <= 2048)");
  SMER_REQUIRE(part && W && (C || Cf) && ldw % 4 == 0 && aligned16(W),
               "smer_linear_decode_merge_f32: operands / alignment");
  const GemmEpi e = decode_epi(bias, relu, residual, ldr, C, ldc, Cf, ldcf, nullptr, 0, 0, nullptr, nullptr, 0);
  const dim3 grid((N + SKF_BN - 1) / SKF_BN, (M + SKF_BM - 1) / SKF_BM);
  const size_t lds = (size_t)std::min(M, SKF_BM) * K * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_skinny_merge_f32_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        SKF_BM * 2048 * (int)sizeof(float));
    attr_set = true;
  }
  hipLaunchKernelGGL(gemm_skinny_merge_f32_kernel, grid, dim3(64 * SKF_NW), lds, (hipStream_t)stream, M, N, K, part,
                     (const float*)W, ldw, e);
  SMER_CHECK_LAUNCH("smer_linear_decode_merge_f32");
  return SMER_OK;
}

// ---------------------------------------------------------------------------
// fp8 (OCP e4m3) forward GEMM, per-tensor scaled (BASELINE C4: "fp8 MFMA
// GEMMs on CDNA4").  C = (a_inv * b_inv) * A8 . B8^T + epilogue, where
// A8 = e4m3(A * 448 / amax(A)) and a_inv = amax(A) / 448 (likewise B).
// MFMA: the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0
// scales (127) — the K = 128 form runs at the fp8 rate, 2x bf16 (the plain
// 16x16x32 fp8 MFMA runs at the bf16 rate).  Tile / staging as the bf16
// 256x256 kernel: a K stage is 128 fp8 = 128 B per row, so the LDS image
// (128-B rows, 16-B chunks XOR (row & 7)) and its LDS-DMA fill are the same
// bytes; a 16x16x128 fragment is 32 B per lane (two chunks).
// ---------------------------------------------------------------------------
typedef int i32x8 __attribute__((ext_vector_type(8)));
namespace {
constexpr int F8K = 128;  // K per stage (bytes per row)

// Row swizzle of the 16-B chunks: physical chunk = logical ^ f8_swz(row).
// A fragment read (ds_read_b128 x 2) is serviced in lane groups of 16 that
// mix two logical chunks (g and g + 1 of the 16x16x128 layout) over 16 rows;
// h(r) = bit1(r) | bit2(r) << 2 sends every group's 16 x 16 B to distinct
// bank quads (the bf16 kernel's (row & 7) swizzle gives 2-way conflicts
// here: SQ_LDS_BANK_CONFLICT / IDX_ACTIVE measured 0.475).
__device__ __forceinline__ int f8_swz(int row) { return ((row >> 1) & 1) | (row & 4); }

__device__ __forceinline__ void f8_glds(char* buf, const uint8_t* P, long ld, int rows, int r0,
                                        int k0, int tid) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int chunk = wave * 4 + c;  // 32 x 1 KiB = 256 rows x 128 B
    const int row = chunk * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ f8_swz(row);
    const uint8_t* src = P + (long)min(r0 + row, rows - 1) * ld + k0 + lc * 16;
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(buf + chunk * 1024), 16, 0, 0);
  }
}
__device__ __forceinline__ f32x4 mfma_f8(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
// lane (c16, g): row rbase + c16, k bytes [32g, 32g + 32) = chunks 2g, 2g + 1;
// asm reads (lds_read_b128_async: hipcc otherwise waits vmcnt(0) for the next
// stage's LDS-DMA before the first read of a k-step)
__device__ __forceinline__ i32x8 f8_frag_async(const char* buf, int rbase, int lane) {
  const int g = lane >> 4, row = rbase + (lane & 15);
  const int h = f8_swz(row);
  const uint4 lo = lds_read_b128_async(buf, row * 128 + (((2 * g) ^ h) << 4));
  const uint4 hi = lds_read_b128_async(buf, row * 128 + (((2 * g + 1) ^ h) << 4));
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}
// row fragment I of the k-step: read A fragment I + AHEAD, retire fragment I
// (counted lgkmcnt: the 2 reads of each younger fragment stay in flight),
// then its 4 MFMAs
template <int I, int AHEAD>
__device__ __forceinline__ void f8_kstep(f32x4 (&acc)[8][4], i32x8 (&af)[8], i32x8 (&bfr)[4],
                                         const char* a_s, int wm, int lane) {
  if constexpr (I + AHEAD < 8) af[I + AHEAD] = f8_frag_async(a_s, wm * 128 + (I + AHEAD) * 16, lane);
  lds_wait<2 * ((7 - I) < AHEAD ? (7 - I) : AHEAD)>();
  asm volatile("" : "+v"(af[I]));
  if constexpr (I == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(bfr[j]));
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[I][j] = mfma_f8(af[I], bfr[j], acc[I][j]);
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace

// FAST: the streamed epilogue (e.vec: 16-B aligned vectors; LDS G2_LDS);
// Q8: also write the e4m3 copy of the output (launched with the generic
// epilogue: the streamed one spills 37 VGPRs with it and measured slower).
template <bool FAST, bool Q8, bool G8 = false>
__global__ __launch_bounds__(512, 1) void gemm256_fp8_kernel(int M, int N, int K,
                                                             const uint8_t* __restrict__ A, long lda,
                                                             const uint8_t* __restrict__ B, long ldb,
                                                             const float* __restrict__ a_inv,
                                                             const float* __restrict__ b_inv,
                                                             GemmEpi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nbm = M / G2, nbn = N / G2;
  const int nwg = nbm * nbn;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;
  const int nk = K / F8K;
  GemmEpi ee = e;
  ee.alpha = e.alpha * (*a_inv) * (*b_inv);  // dequantisation of both operands
  float amax_acc = 0.f;
  const bf16* xsrc = (const bf16*)(e.residual ? e.residual : e.gate);  // streamed epilogue operand (G8: bytes)
  const long ldx = e.residual ? e.ldr : e.ldg;
  g2_start_skew(e.skew);

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const int wgid = xstart + jj;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int m0 = (first_m + within % gsz) * G2, n0 = (within / gsz) * G2;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // FAST: bias columns
    // (Q8: loaded after the K loop, so its 8 registers are not live across it)
    if (FAST && !Q8 && e.bias) {
      const float4 b0 = *reinterpret_cast<const float4*>(e.bias + n0 + (tid & 31) * 8);
      const float4 b1 = *reinterpret_cast<const float4*>(e.bias + n0 + (tid & 31) * 8 + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
      bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    }
    f8_glds(smem, A, lda, M, m0, 0, tid);
    f8_glds(smem + G2_OP, B, ldb, N, n0, 0, tid);
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();  // stage kt landed; stage kt-1 fully read
      // X rows of the first epilogue pass into slot A (beyond the stages)
      if (FAST && xsrc && kt == nk / 2) g2_xload_any<G8>(smem + G2_XA, xsrc, ldx, m0, n0, tid);
      if (kt + 1 < nk) {
        char* nb = smem + ((kt + 1) & 1) * G2_STAGE;
        f8_glds(nb, A, lda, M, m0, (kt + 1) * F8K, tid);
        f8_glds(nb + G2_OP, B, ldb, N, n0, (kt + 1) * F8K, tid);
      }
      const char* a_s = smem + (kt & 1) * G2_STAGE;
      const char* b_s = a_s + G2_OP;
      // A fragments run 4 ahead of the MFMAs that use them (a read issued
      // right before its 4 MFMAs exposes one LDS latency per fragment; all 12
      // up front does not fit beside the 128 accumulators)
      constexpr int AHEAD = FAST ? 1 : 3;  // FAST: bias registers leave no room for more
      i32x8 bfr[4], af[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = f8_frag_async(b_s, wn * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < AHEAD; ++i) af[i] = f8_frag_async(a_s, wm * 128 + i * 16, lane);
      f8_kstep<0, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<1, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<2, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<3, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<4, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<5, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<6, AHEAD>(acc, af, bfr, a_s, wm, lane);
      f8_kstep<7, AHEAD>(acc, af, bfr, a_s, wm, lane);
    }
    __syncthreads();  // all fragment reads done before the epilogue reuses LDS

    if constexpr (FAST) {
      if (Q8 && e.bias) {
        const float4 b0 = *reinterpret_cast<const float4*>(e.bias + n0 + (tid & 31) * 8);
        const float4 b1 = *reinterpret_cast<const float4*>(e.bias + n0 + (tid & 31) * 8 + 4);
        bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
        bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
      }
      g2_fast_epilogue<Q8, G8>(ee, acc, smem, m0, n0, tid, bv, xsrc, ldx, amax_acc);
      continue;
    }
    const int g = lane >> 4, c16 = lane & 15;
    constexpr int EP_LD = G2 + 4;
    float* ep = reinterpret_cast<float*>(smem);
    // the tile's 256 bias values staged in LDS behind the fp32 rows (no
    // dependent global load per epilogue pass, no extra registers)
    GemmEpi eb = ee;
    if (ee.bias) {
      float* bl = reinterpret_cast<float*>(smem + G2_XB);
      if (tid < 64) reinterpret_cast<float4*>(bl)[tid] = reinterpret_cast<const float4*>(ee.bias + n0)[tid];
      eb.bias = bl - n0;
    }
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      if (wm == (pass >> 1)) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          const int i = 4 * (pass & 1) + ii;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ep[(ii * 16 + 4 * g + r) * EP_LD + wn * 64 + j * 16 + c16] = acc[i][j][r];
        }
      }
      smer_lds_barrier();  // (pass 0: also the bias slice); stores left in flight
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int item = tid + 512 * c;  // 64 rows x 32 chunks of 8 columns
        const int row = item >> 5, ch = item & 31;
        const int grow = m0 + pass * 64 + row, gcol = n0 + ch * 8;
        float v[8];
        const float4 a = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8);
        const float4 b = *reinterpret_cast<const float4*>(ep + row * EP_LD + ch * 8 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        epi_apply8(eb, M, N, grow, gcol, v, &amax_acc);
      }
      smer_lds_barrier();
    }
  }
  if (Q8) smer_amax_commit(e.q8_amax, amax_acc);
}

// amax(|x|) over a [rows, cols] bf16 view: float bits of non-negative values
// order like unsigned ints, so an integer atomicMax is exact and the result
// does not depend on the order of arrival.
__global__ __launch_bounds__(256) void amax_bf16_kernel(int rows, int cols, const bf16* __restrict__ x,
                                                       long ldx, unsigned int* __restrict__ out) {
  const int cpr = cols >> 3;
  const long n = (long)rows * cpr;
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cpr, c = (i % cpr) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + r * ldx + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf((float)v[k]));
  }
  m = wave_max(m);
  __shared__ float wm_[4];
  if ((threadIdx.x & 63) == 0) wm_[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm_[0], wm_[1]), fmaxf(wm_[2], wm_[3]));
    atomicMax(out, __float_as_uint(m));
  }
}

// q = e4m3(x * 448 / amax) (round to nearest even, saturating), inv = amax / 448
__global__ __launch_bounds__(256) void quant_fp8_kernel(int rows, int cols, const bf16* __restrict__ x,
                                                       long ldx, uint8_t* __restrict__ q, long ldq,
                                                       const unsigned int* __restrict__ amax,
                                                       float* __restrict__ inv) {
  const float am = __uint_as_float(*amax);
  const float sc = am > 0.f ? smer_div_rn(448.f, am) : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) *inv = smer_div_rn(1.f, sc);
  const int cpr = cols >> 3;
  const long n = (long)rows * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cpr, c = (i % cpr) * 8;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + r * ldx + c);
    uint32_t w[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float f[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) f[k] = fminf(fmaxf((float)v[4 * h + k] * sc, -448.f), 448.f);
      int p = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
      p = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], p, true);
      w[h] = (uint32_t)p;
    }
    *reinterpret_cast<uint2*>(q + r * ldq + c) = make_uint2(w[0], w[1]);
  }
}

// Batched per-tensor quantisation of many contiguous bf16 tensors (every fp8
// weight of a model after an optimizer step: 2 launches + 1 memset instead
// of 3 per tensor).  seg[3 * s] = (src bf16*, dst uint8*, n elements).
__global__ __launch_bounds__(256) void amax_seg_kernel(const int64_t* __restrict__ seg,
                                                      unsigned int* __restrict__ amax) {
  const int s = blockIdx.y;
  const bf16* x = reinterpret_cast<const bf16*>(seg[3 * s]);
  const long n8 = seg[3 * s + 2] >> 3;
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf((float)v[k]));
  }
  m = wave_max(m);
  __shared__ float wm_[4];
  if ((threadIdx.x & 63) == 0) wm_[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm_[0], wm_[1]), fmaxf(wm_[2], wm_[3]));
    atomicMax(amax + s, __float_as_uint(m));
  }
}

__global__ __launch_bounds__(256) void quant_seg_kernel(const int64_t* __restrict__ seg,
                                                       const unsigned int* __restrict__ amax,
                                                       float* __restrict__ inv) {
  const int s = blockIdx.y;
  const bf16* x = reinterpret_cast<const bf16*>(seg[3 * s]);
  uint8_t* q = reinterpret_cast<uint8_t*>(seg[3 * s + 1]);
  const long n8 = seg[3 * s + 2] >> 3;
  const float am = __uint_as_float(amax[s]);
  const float sc = am > 0.f ? smer_div_rn(448.f, am) : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) inv[s] = smer_div_rn(1.f, sc);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = (float)v[k];
    *reinterpret_cast<uint2*>(q + 8 * i) = smer_q8x8(f, sc);
  }
}

extern "C" int smer_fp8_quantize_segments(int nseg, const int64_t* seg, unsigned* amax_ws, float* inv_scale,
                                          int blocks_per_seg, smer_stream_t stream) {
  SMER_REQUIRE(nseg >= 0 && nseg <= 65535 && blocks_per_seg > 0, "smer_fp8_quantize_segments: sizes");
  if (nseg == 0) return SMER_OK;
  SMER_REQUIRE(seg && amax_ws && inv_scale, "smer_fp8_quantize_segments: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(amax_ws, 0, sizeof(unsigned) * nseg, s) != hipSuccess)
    return smer_set_error(SMER_ERR_HIP, "smer_fp8_quantize_segments: memset");
  const dim3 grid(blocks_per_seg, nseg);
  hipLaunchKernelGGL(amax_seg_kernel, grid, dim3(256), 0, s, seg, amax_ws);
  hipLaunchKernelGGL(quant_seg_kernel, grid, dim3(256), 0, s, seg, (const unsigned*)amax_ws, inv_scale);
  SMER_CHECK_LAUNCH("smer_fp8_quantize_segments");
  return SMER_OK;
}

// Batched transposing e4m3 quantisation (the dgrad operands W^T of the fp8
// backward): seg[4 s] = (src bf16 [rows, cols], dst uint8 [cols, rows], rows,
// cols), rows and cols multiples of 64.  Per-tensor scale from the amax of
// the whole tensor (transpose-invariant: the same scale as the forward copy).
// A 256-thread block moves one 64 x 64 tile through LDS: rows read and
// columns written 128 B at a time.
__global__ __launch_bounds__(256) void amax_seg4_kernel(const int64_t* __restrict__ seg,
                                                       unsigned int* __restrict__ amax) {
  const int s = blockIdx.y;
  const bf16* x = reinterpret_cast<const bf16*>(seg[4 * s]);
  const long n8 = (seg[4 * s + 2] * seg[4 * s + 3]) >> 3;
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + 8 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf((float)v[k]));
  }
  m = wave_max(m);
  __shared__ float wm_[4];
  if ((threadIdx.x & 63) == 0) wm_[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm_[0], wm_[1]), fmaxf(wm_[2], wm_[3]));
    atomicMax(amax + s, __float_as_uint(m));
  }
}

__global__ __launch_bounds__(256) void quant_seg_t_kernel(const int64_t* __restrict__ seg,
                                                         const unsigned int* __restrict__ amax,
                                                         float* __restrict__ inv) {
  __shared__ uint8_t t[64][72];
  const int s = blockIdx.y;
  const bf16* x = reinterpret_cast<const bf16*>(seg[4 * s]);
  uint8_t* q = reinterpret_cast<uint8_t*>(seg[4 * s + 1]);
  const int rows = (int)seg[4 * s + 2], cols = (int)seg[4 * s + 3];
  const int tr = rows >> 6, tc = cols >> 6;
  const float am = __uint_as_float(amax[s]);
  const float sc = am > 0.f ? smer_div_rn(448.f, am) : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) inv[s] = smer_div_rn(1.f, sc);
  const int tid = threadIdx.x;
  for (int tile = blockIdx.x; tile < tr * tc; tile += gridDim.x) {
    const int r0 = (tile / tc) * 64, c0 = (tile % tc) * 64;
    // 64 rows x 8 chunks of 8 columns: 2 chunks per thread
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int item = tid + 256 * h, r = item >> 3, ch = item & 7;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (long)(r0 + r) * cols + c0 + ch * 8);
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = (float)v[k];
      const uint2 w = smer_q8x8(f, sc);
      const uint8_t* b = reinterpret_cast<const uint8_t*>(&w);
#pragma unroll
      for (int k = 0; k < 8; ++k) t[ch * 8 + k][r] = b[k];
    }
    __syncthreads();
    // dst rows c0 .. c0+63 (a source column each), 64 bytes: 8 x 8 B per row
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int item = tid + 256 * h, c = item >> 3, ch = item & 7;
      uint2 w;
      uint8_t* b = reinterpret_cast<uint8_t*>(&w);
#pragma unroll
      for (int k = 0; k < 8; ++k) b[k] = t[c][ch * 8 + k];
      *reinterpret_cast<uint2*>(q + (long)(c0 + c) * rows + r0 + ch * 8) = w;
    }
    __syncthreads();
  }
}

extern "C" int smer_fp8_quantize_segments_t(int nseg, const int64_t* seg, unsigned* amax_ws, float* inv_scale,
                                            int blocks_per_seg, smer_stream_t stream) {
  SMER_REQUIRE(nseg >= 0 && nseg <= 65535 && blocks_per_seg > 0, "smer_fp8_quantize_segments_t: sizes");
  if (nseg == 0) return SMER_OK;
  SMER_REQUIRE(seg && amax_ws && inv_scale, "smer_fp8_quantize_segments_t: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(amax_ws, 0, sizeof(unsigned) * nseg, s) != hipSuccess)
    return smer_set_error(SMER_ERR_HIP, "smer_fp8_quantize_segments_t: memset");
  const dim3 grid(blocks_per_seg, nseg);
  hipLaunchKernelGGL(amax_seg4_kernel, grid, dim3(256), 0, s, seg, amax_ws);
  hipLaunchKernelGGL(quant_seg_t_kernel, grid, dim3(256), 0, s, seg, (const unsigned*)amax_ws, inv_scale);
  SMER_CHECK_LAUNCH("smer_fp8_quantize_segments_t");
  return SMER_OK;
}

extern "C" size_t smer_fp8_quantize_workspace(void) { return 16; }

extern "C" int smer_fp8_quantize(int rows, int cols, const void* x, long ldx, void* q, long ldq,
                                 void* workspace, float* inv_scale, smer_stream_t stream) {
  SMER_REQUIRE(rows >= 0 && cols > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldq % 8 == 0,
               "smer_fp8_quantize: cols / strides must be multiples of 8");
  SMER_REQUIRE(x && q && workspace && inv_scale && aligned16(x) && ((uintptr_t)q & 7) == 0,
               "smer_fp8_quantize: pointers / alignment");
  hipStream_t s = (hipStream_t)stream;
  unsigned int* am = (unsigned int*)workspace;
  if (hipMemsetAsync(am, 0, sizeof(unsigned int), s) != hipSuccess)
    return smer_set_error(SMER_ERR_HIP, "smer_fp8_quantize: memset");
  const long n = (long)rows * (cols / 8);
  const int grid = (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8L * smer_num_cus()));
  hipLaunchKernelGGL(amax_bf16_kernel, dim3(grid), dim3(256), 0, s, rows, cols, (const bf16*)x, ldx, am);
  hipLaunchKernelGGL(quant_fp8_kernel, dim3(grid), dim3(256), 0, s, rows, cols, (const bf16*)x, ldx,
                     (uint8_t*)q, ldq, (const unsigned int*)am, inv_scale);
  SMER_CHECK_LAUNCH("smer_fp8_quantize");
  return SMER_OK;
}

// ---------------------------------------------------------------------------
// fp8 (e4m3) staggered 256x256 GEMM for long-K NT products (the C4 fp8
// dgrads, K >= 1024): gemm256s_bf16_kernel's schedule, slots and epilogue
// with the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (unit E8M0 scales,
// 2x the bf16 rate): a 32-deep bf16 k-step of the LDS image is 64 e4m3 per
// row, exactly one K = 64 MFMA step; a wave's 128x64 outputs are 4 x 2
// blocks of 32 x 32 (8 MFMAs of 64 cycles per k-step, as the bf16 kernel's
// 32 of 16).  Lane l holds A[row l & 31][k 32 (l >> 5) .. + 31] (32 B: two
// 16-B chunks, contiguous under the chunk ^ 2 bit2(row) swizzle).
// ---------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma_f8_32(i32x8 a, i32x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
__device__ __forceinline__ i32x8 f8_cat(uint4 lo, uint4 hi) {
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}
template <int OFF>
__device__ __forceinline__ uint4 lds_u4_off(uint32_t a) {
  uint4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
// the 6 fragments of one k-step (12 reads): A blocks i (rows wm*128 + 32 i),
// B blocks q (columns wn*64 + 32 q)
__device__ __forceinline__ void gs_frags_f8(uint32_t slot_lds, int wm, int wn, int lane, i32x8 (&af)[4],
                                            i32x8 (&bfr)[2]) {
  const int r32 = lane & 31, h = lane >> 5;
  const uint32_t off = r32 * 64 + (((2 * h) ^ gs_swz(r32)) << 4);
  const uint32_t ab = slot_lds + wm * 8192 + off;
  const uint32_t bb = slot_lds + GS_OP + wn * 4096 + off;
  bfr[0] = f8_cat(lds_u4_off<0>(bb), lds_u4_off<16>(bb));
  bfr[1] = f8_cat(lds_u4_off<2048>(bb), lds_u4_off<2064>(bb));
  af[0] = f8_cat(lds_u4_off<0>(ab), lds_u4_off<16>(ab));
  af[1] = f8_cat(lds_u4_off<2048>(ab), lds_u4_off<2064>(ab));
  af[2] = f8_cat(lds_u4_off<4096>(ab), lds_u4_off<4112>(ab));
  af[3] = f8_cat(lds_u4_off<6144>(ab), lds_u4_off<6160>(ab));
}
// fp32 staging index for the 32x32 C layout (lanes l and l + 32 write rows 4
// apart: column bit 5 flipped on rows with bit 2 set)
__device__ __forceinline__ int gs_ep_idx32(int row, int col) { return row * 256 + (col ^ (((row >> 2) & 1) << 5)); }
__device__ __forceinline__ void f8_retire(i32x8 (&a)[4], i32x8 (&b)[2]) {
  lds_wait<0>();
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(a[i]));
#pragma unroll
  for (int i = 0; i < 2; ++i) asm volatile("" : "+v"(b[i]));
}

__global__ __launch_bounds__(512, 1) void gemm256s_fp8_kernel(int M, int N, int K,
                                                              const uint8_t* __restrict__ A8, long lda8,
                                                              const uint8_t* __restrict__ B8, long ldb8,
                                                              const float* __restrict__ a_inv,
                                                              const float* __restrict__ b_inv, GemmEpi e) {
  constexpr bool BKC = true;
  // the LDS-DMA moves bytes: address the e4m3 rows as bf16 pairs, so a
  // 32-"element" k-step is 64 fp8 and every slot / piece is the bf16 kernel's
  const bf16* A = reinterpret_cast<const bf16*>(A8);
  const bf16* B = reinterpret_cast<const bf16*>(B8);
  const long lda = lda8 / 2, ldb = ldb8 / 2;
  e.alpha = e.alpha * (*a_inv) * (*b_inv);  // dequantisation of both operands
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3, lw = wave & 3;
  const bool loader = wm == 1;  // waves 4-7: every DMA; waves 0-3: every store
  const int nbm = M / G2, nbn = N / G2;
  const int nwg = nbm * nbn;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;
  const int nk = K / (2 * GS_KS);  // 64 fp8 per k-step; host: nk >= 4
  const bf16* xsrc = (const bf16*)(e.residual ? e.residual : e.gate);
  const long ldx = e.residual ? e.ldr : e.ldg;
  const uint32_t lds0 = lds_u32(smem);
  const int g = lane >> 4, c16 = lane & 15;
  constexpr int EP_LD = G2 + 4;

  int tcount = 0;
  for (int jj = braw >> 3; jj < xcount; jj += pstride, ++tcount) {
    const int wgid = xstart + jj;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int m0 = (first_m + within % gsz) * G2, n0 = (within / gsz) * G2;

    f32x16 acc[4][2];  // 32x32 blocks: rows wm*128 + 32 i, columns wn*64 + 32 q
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // operand bases of this tile (bf16-pair units); k-step k adds k * 32
    // pairs = 64 e4m3 columns
    const bf16* At = A + (long)m0 * lda;
    const bf16* Bt = BKC ? B + (long)n0 * ldb : B + n0;
    const long bstep = BKC ? GS_KS : (long)GS_KS * ldb;

    // prologue: k-steps 0..2 in flight, k-step 0 landed before the first
    // barrier (after the first tile, k-steps 0 and 1 were issued during the
    // previous tile's epilogue)
    if (loader) {
      if (tcount == 0) {
        gs_issue<BKC>(lds0 + 0 * GS_SLOT, At, lda, Bt, ldb, lw, lane);
        gs_issue<BKC>(lds0 + 1 * GS_SLOT, At + GS_KS, lda, Bt + bstep, ldb, lw, lane);
      }
      gs_issue<BKC>(lds0 + 2 * GS_SLOT, At + 2 * GS_KS, lda, Bt + 2 * bstep, ldb, lw, lane);
      vm_wait<16>();
    }
    gs_bar();
    if (loader) gs_bar();  // the lagging half: one barrier behind from here

    for (int j = 0; j < nk; ++j) {
      // R(j): fragment reads of slot j & 3; a loader issues the B half of
      // k-step j+3 (into the slot k-step j-1 left: every wave retired its
      // reads of it before its previous M phase) and waits for k-step j+1.
      // Issue order per loader: B(t) in R(t-3), A(t) in M(t-3).
      i32x8 bfr[2], af[4];
      gs_frags_f8(lds0 + (j & 3) * GS_SLOT, wm, wn, lane, af, bfr);
      const bool do_k = loader && j + 3 < nk;
      const uint32_t kslot = lds0 + ((j + 3) & 3) * GS_SLOT;
      const bf16* Aj = At + (long)(j + 3) * GS_KS;
      const bf16* Bj = Bt + (j + 3) * bstep;
      if (do_k) {
#pragma unroll
        for (int t = 4; t < 8; ++t) gs_piece<BKC>(t, kslot, Aj, lda, Bj, ldb, lw, lane);
      }
      if (loader) {
        if (j + 3 < nk) {
          vm_wait<12>();  // k-step j+1 landed (B, A of j+2 and B of j+3 fly)
        } else if (j + 3 == nk) {
          vm_wait<8>();
        } else if (j + 2 == nk) {  // k-step nk-1 landed; bias / X(0) may fly on
          if (xsrc && e.bias) vm_wait<5>();
          else if (xsrc) vm_wait<4>();
          else if (e.bias) vm_wait<1>();
          else vm_wait<0>();
        }
      }
      gs_bar();
      // M(j): 8 MFMAs of 64 cycles; a loader slips one A piece of k-step
      // j+3 in behind every 2 of them
      f8_retire(af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[i][q] = mfma_f8_32(af[i], bfr[q], acc[i][q]);
        if (do_k) {  // one A piece of k-step j+3 behind every 2 MFMAs (64 cycles each)
          __builtin_amdgcn_sched_barrier(0);
          gs_piece<BKC>(i, kslot, Aj, lda, Bj, ldb, lw, lane);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (loader && j + 3 == nk) {
        // the epilogue's bias row and first X rows, beyond the four slots
        // (the bias through LDS: a register load would be a vmcnt wait
        // hipcc places itself, on the storers' outstanding stores)
        if (e.bias) gs_bias_load(lds0 + GS_BIAS, e.bias + n0, lane);
        if (xsrc) gs_xload(lds0 + GS_XA, xsrc + (long)m0 * ldx + n0, ldx, lw, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
      gs_bar();
    }
    if (!loader) gs_bar();  // realign the halves

    // ---- epilogue: eight 32-row passes through fp32 LDS staging ---------
    // The owning half (rows 128 wm .. +127) stages its accumulators; all 512
    // threads apply bias / ReLU / dropout / residual or gate to 2 items of 8
    // columns; the storers store theirs, the loaders hand theirs to the
    // storers as bf16 through OUT (stored one pass later): loaders never
    // store, so their vmcnt holds DMAs only.  The loaders first issue the
    // next tile's k-steps 0 and 1 (slots 0-1), which land under this
    // epilogue, then stream X one pass ahead.
    const int jn = jj + pstride;
    const bool has_next = jn < xcount;
    if (loader && has_next) {
      const int wn2 = xstart + jn;
      const int grp2 = wn2 / (GM * nbn);
      const int gsz2 = min(nbm - grp2 * GM, GM);
      const int win2 = wn2 % (GM * nbn);
      const int m1 = (grp2 * GM + win2 % gsz2) * G2, n1 = (win2 / gsz2) * G2;
      const bf16* At1 = A + (long)m1 * lda;
      const bf16* Bt1 = BKC ? B + (long)n1 * ldb : B + n1;
      if (xsrc)  // X(1) ahead of them: its wait then passes over them
        gs_xload(lds0 + GS_XB, xsrc + (long)(m0 + GS_EPR) * ldx + n0, ldx, lw, lane);
      gs_issue<BKC>(lds0 + 0 * GS_SLOT, At1, lda, Bt1, ldb, lw, lane);
      gs_issue<BKC>(lds0 + 1 * GS_SLOT, At1 + GS_KS, lda, Bt1 + bstep, ldb, lw, lane);
    } else if (loader && xsrc) {
      gs_xload(lds0 + GS_XB, xsrc + (long)(m0 + GS_EPR) * ldx + n0, ldx, lw, lane);
    }
    float* ep = reinterpret_cast<float*>(smem + GS_EP);
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int ch = tid & 31;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      if (loader) {  // X(pass) (and at pass 0 the bias) landed
        if (xsrc) {
          if (pass >= 1 && pass < 7)  // X(pass+1) into the slot X(pass-1) left
            gs_xload(lds0 + (((pass + 1) & 1) ? GS_XB : GS_XA),
                     xsrc + (long)(m0 + GS_EPR * (pass + 1)) * ldx + n0, ldx, lw, lane);
          if (pass <= 1) {
            if (has_next) vm_wait<20>();
            else vm_wait<4>();
          } else if (pass < 7) {
            vm_wait<4>();
          } else {
            vm_wait<0>();
          }
        } else if (pass == 0 && e.bias) {
          if (has_next) vm_wait<16>();
          else vm_wait<0>();
        }
      }
      if (wm == (pass >> 2)) {  // 32x32 row block i = pass & 3: row (r&3) + 8 (r>>2) + 4 (lane>>5)
        const int i = pass & 3;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            ep[gs_ep_idx32((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), wn * 64 + q * 32 + (lane & 31))] = acc[i][q][r];
      }
      smer_lds_barrier();  // staging rows written, X(pass) and the bias landed
      if (pass == 0 && e.bias) {
        const float* bl = reinterpret_cast<const float*>(smem + GS_BIAS) + ch * 8;
        const float4 b0 = *reinterpret_cast<const float4*>(bl);
        const float4 b1 = *reinterpret_cast<const float4*>(bl + 4);
        bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
        bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
      }
      // storers: the loaders' items of the previous pass (bf16 in OUT)
      if (!loader && pass >= 1) {
        const char* ob = smem + GS_OUT + ((pass - 1) & 1) * 8192;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int lr = (tid >> 5) + 8 * c;  // 0..15 -> pass rows 8..15, 24..31
          const int row = (lr & 7) + 8 + 16 * (lr >> 3);
          const bf16x8 o = *reinterpret_cast<const bf16x8*>(ob + lr * 512 + ch * 16);
          *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)(m0 + (pass - 1) * GS_EPR + row) * e.ldc + n0 + ch * 8) = o;
        }
      }
      const char* xs = smem + ((pass & 1) ? GS_XB : GS_XA);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int row = (tid >> 5) + 16 * c;  // storers rows 0..7, 16..23; loaders 8..15, 24..31
        const int grow = m0 + pass * GS_EPR + row, gcol = n0 + ch * 8;
        float v[8];
        const float4 a = *reinterpret_cast<const float4*>(ep + gs_ep_idx32(row, ch * 8));
        const float4 b = *reinterpret_cast<const float4*>(ep + gs_ep_idx32(row, ch * 8) + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] * e.alpha + bv[k];
        if (e.relu) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
        }
        if (e.drop_thr)
          smer_drop8(smer_rowkey(e.seed, (uint32_t)grow), e.drop_thr, e.drop_scale, (uint32_t)gcol, v);
        if (xsrc) {
          const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + row * 512 + ch * 16);
          if (e.residual) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += (float)xv[k];
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (float)xv[k] > 0.f ? v[k] * e.gate_scale : 0.f;
          }
        }
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
        if (!loader) {
          *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)grow * e.ldc + gcol) = o;
        } else {
          const int lr = (row & 7) + 8 * (row >> 4);
          *reinterpret_cast<bf16x8*>(smem + GS_OUT + (pass & 1) * 8192 + lr * 512 + ch * 16) = o;
        }
      }
      smer_lds_barrier();  // staging, X(pass) and OUT(pass - 1) read before they are rewritten
    }
    if (!loader) {  // the loaders' items of the last pass
      const char* ob = smem + GS_OUT + 8192;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int lr = (tid >> 5) + 8 * c;
        const int row = (lr & 7) + 8 + 16 * (lr >> 3);
        const bf16x8 o = *reinterpret_cast<const bf16x8*>(ob + lr * 512 + ch * 16);
        *reinterpret_cast<bf16x8*>((bf16*)e.C + (long)(m0 + 7 * GS_EPR + row) * e.ldc + n0 + ch * 8) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fp8 (e4m3) weight gradient dW (+)= a_inv b_inv dY^T X from tokens-major
// e4m3 copies of both operands (K = tokens): gemm256s_wgrad_kernel's
// staggered schedule (four slots, three k-steps ahead, halves one barrier
// apart, waves 4-7 issue every DMA, waves 0-3 every store) with 64-deep
// k-steps -- the same 16 KiB per operand per slot, 64 k-rows of 256 B -- on
// the block-scaled 32x32x64 MFMA (2x the bf16 rate).  The MFMA wants 32
// consecutive k per lane and the k-rows land tokens-major, so every fragment
// is four ds_read_b64_tr_b8: in a group of 16 lanes, source lane 2k' + h
// addresses k-row k' (of 8) at bytes 8h .. 8h+7 of a 16-column block, and
// lane j receives column j's 8 k-rows (tools/probes/tr8_probe.hip).  The
// 16-B chunks of k-row k sit at chunk ^ 2 (k & 7): the eight k-rows of one
// read fall on eight different 32-B bank groups.  Output: alpha * acc into
// a split-K slab, or dW (+)= alpha * acc unsplit.  The bias gradient rides
// along from the same e4m3 dY: wave wn sums A fragment wn (32 e4m3 per lane,
// converted to fp32) on the k-steps j with j % (column tiles) == its column
// tile, so the extra VALU work is spread evenly over a row of tiles (summed
// by the first column tile alone it cost the whole grid +20 %: everyone
// waits for the slowest tile); partials [slice][column tile][M], reduced in
// fixed order by wgrad_rowsum_reduce_kernel.
// ---------------------------------------------------------------------------
namespace {
typedef int i32x2 __attribute__((ext_vector_type(2)));
template <int OFF>
__device__ __forceinline__ i32x2 lds_tr8_off(uint32_t a) {
  i32x2 r;
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
// 32 k of one 32-feature block: k-rows 8r + k' (r = 0..3) of the lane's half
__device__ __forceinline__ i32x8 tr8_frag(uint32_t a) {
  const i32x2 r0 = lds_tr8_off<0>(a), r1 = lds_tr8_off<2048>(a);
  const i32x2 r2 = lds_tr8_off<4096>(a), r3 = lds_tr8_off<6144>(a);
  return i32x8{r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y};
}
// piece t < 4: A k-rows 4c .. 4c+3 (c = 4 lw + t), t >= 4: the B ones
__device__ __forceinline__ void gw8_piece(int t, uint32_t slot_lds, const uint8_t* At, long lda,
                                          const uint8_t* Bt, long ldb, int lw, int lane) {
  const int c = lw * 4 + (t & 3);
  const int k = c * 4 + (lane >> 4);
  const int lc = (lane & 15) ^ (2 * (k & 7));
  if (t < 4)
    glds16_asm(sgpr_ptr(At), (uint32_t)(k * lda + lc * 16),
               (uint32_t)__builtin_amdgcn_readfirstlane(slot_lds + c * 1024));
  else
    glds16_asm(sgpr_ptr(Bt), (uint32_t)(k * ldb + lc * 16),
               (uint32_t)__builtin_amdgcn_readfirstlane(slot_lds + GS_OP + c * 1024));
}
// running fp32 sum of the 32 e4m3 values of a fragment (fixed order)
__device__ __forceinline__ float rowsum_f8(const i32x8& f, float acc) {
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(f[d], false);
    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(f[d], true);
    p0 += lo[0]; p1 += lo[1]; p0 += hi[0]; p1 += hi[1];
  }
  return acc + (p0 + p1);
}
__device__ __forceinline__ void gw8_issue(uint32_t slot_lds, const uint8_t* At, long lda, const uint8_t* Bt,
                                          long ldb, int lw, int lane) {
#pragma unroll
  for (int t = 0; t < 8; ++t) gw8_piece(t, slot_lds, At, lda, Bt, ldb, lw, lane);
}
}  // namespace

__global__ __launch_bounds__(512, 1) void gemm256s_wgrad_fp8_kernel(int M, int N, int K,
                                                                    const uint8_t* __restrict__ A, long lda,
                                                                    const uint8_t* __restrict__ B, long ldb,
                                                                    const float* __restrict__ a_inv,
                                                                    const float* __restrict__ b_inv,
                                                                    GemmEpi e, int ksplit, int kchunk,
                                                                    float* __restrict__ slabs,
                                                                    float* __restrict__ rowsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3, lw = wave & 3;
  const bool loader = wm == 1;
  const int nbm = M / G2, nbn = N / G2;
  const int ntiles = nbm * nbn;
  const int nwg = ntiles * ksplit;
  const int braw = blockIdx.x, xcd = braw & 7;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int xstart = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcount = q8 + (xcd < r8 ? 1 : 0);
  const int pstride = (int)gridDim.x >= nwg ? xcount : ((int)gridDim.x >> 3);
  constexpr int GM = 4;
  constexpr int KS = 2 * GS_KS;  // 64 tokens per k-step
  const float alpha = e.alpha * (*a_inv) * (*b_inv);
  const float rs_scale = e.alpha * (*a_inv);  // the bias gradient dequantises dY only
  const uint32_t lds0 = lds_u32(smem);
  uint32_t aoff[4], boff[2];
  {
    const int g = lane >> 4, j = lane & 15, kq = j >> 1, hh = j & 1;
    const uint32_t krow = (uint32_t)(32 * (g >> 1) + kq) * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] = krow + ((((uint32_t)(8 * wm + 2 * i + (g & 1))) ^ (2 * kq)) << 4) + 8 * hh;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      boff[q] = GS_OP + krow + ((((uint32_t)(4 * wn + 2 * q + (g & 1))) ^ (2 * kq)) << 4) + 8 * hh;
  }

  for (int jj = braw >> 3; jj < xcount; jj += pstride) {
    const int lin = xstart + jj;
    const int split = lin / ntiles, wgid = lin % ntiles;
    const int grp = wgid / (GM * nbn);
    const int first_m = grp * GM;
    const int gsz = min(nbm - first_m, GM);
    const int within = wgid % (GM * nbn);
    const int tn = within / gsz;
    const int m0 = (first_m + within % gsz) * G2, n0 = tn * G2;
    const int k_begin = split * kchunk, k_end = min(K, k_begin + kchunk);
    const int nk = (k_end - k_begin) / KS;  // host: >= 1
    const bool rsum = rowsum != nullptr;
    const int wn_s = __builtin_amdgcn_readfirstlane(wn);
    float rs = 0.f;

    f32x16 acc[4][2];  // 32x32 blocks: rows wm*128 + 32 i, columns wn*64 + 32 q
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][q][r] = 0.f;
    const uint8_t* At = A + (long)k_begin * lda + m0;
    const uint8_t* Bt = B + (long)k_begin * ldb + n0;
    const long astep = (long)KS * lda, bstep = (long)KS * ldb;

    if (loader) {
      gw8_issue(lds0, At, lda, Bt, ldb, lw, lane);
      if (nk > 1) gw8_issue(lds0 + GS_SLOT, At + astep, lda, Bt + bstep, ldb, lw, lane);
      if (nk > 2) gw8_issue(lds0 + 2 * GS_SLOT, At + 2 * astep, lda, Bt + 2 * bstep, ldb, lw, lane);
      if (nk > 2) vm_wait<16>();
      else if (nk == 2) vm_wait<8>();
      else vm_wait<0>();
    }
    gs_bar();
    if (loader) gs_bar();

    for (int j = 0; j < nk; ++j) {
      const uint32_t slot = lds0 + (j & 3) * GS_SLOT;
      i32x8 af[4], bfr[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) bfr[q] = tr8_frag(slot + boff[q]);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = tr8_frag(slot + aoff[i]);
      const bool do_k = loader && j + 3 < nk;
      const uint32_t kslot = lds0 + ((j + 3) & 3) * GS_SLOT;
      const uint8_t* Aj = At + (long)(j + 3) * astep;
      const uint8_t* Bj = Bt + (long)(j + 3) * bstep;
      if (do_k) {
#pragma unroll
        for (int t = 4; t < 8; ++t) gw8_piece(t, kslot, Aj, lda, Bj, ldb, lw, lane);
      }
      if (loader) {
        if (j + 3 < nk) vm_wait<12>();
        else if (j + 3 == nk) vm_wait<8>();
        else if (j + 2 == nk) vm_wait<0>();
      }
      gs_bar();
      f8_retire(af, bfr);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[i][q] = mfma_f8_32(af[i], bfr[q], acc[i][q]);
        if (do_k) {  // one A piece of k-step j+3 behind every 2 MFMAs (64 cycles each)
          __builtin_amdgcn_sched_barrier(0);
          gw8_piece(i, kslot, Aj, lda, Bj, ldb, lw, lane);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (rsum && j % nbn == tn) {  // wave wn: A fragment wn (rows wm*128 + 32 wn + (lane & 31))
        if (wn_s == 0) rs = rowsum_f8(af[0], rs);
        else if (wn_s == 1) rs = rowsum_f8(af[1], rs);
        else if (wn_s == 2) rs = rowsum_f8(af[2], rs);
        else rs = rowsum_f8(af[3], rs);
      }
      __builtin_amdgcn_sched_barrier(0);
      gs_bar();
    }
    if (!loader) gs_bar();  // realign the halves (every wave past its last reads)
    if (rsum) {
      rs += __shfl_xor(rs, 32);  // the two k-halves of a row
      if (lane < 32) {
        const int row = m0 + wm * 128 + 32 * wn + lane;
        rowsum[((long)split * nbn + tn) * M + row] = rs * rs_scale;
      }
    }

    // ---- epilogue: eight 32-row passes through fp32 staging (slot 2)
    float* ep = reinterpret_cast<float*>(smem + GS_EP);
    float* slab = ksplit > 1 ? slabs + (long)split * M * N : nullptr;
    const int ch = tid & 31;
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      if (wm == (pass >> 2)) {  // 32x32 row block i = pass & 3: row (r&3) + 8 (r>>2) + 4 (lane>>5)
        const int i = pass & 3;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            ep[gs_ep_idx32((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), wn * 64 + q * 32 + (lane & 31))] =
                acc[i][q][r];
      }
      smer_lds_barrier();
      if (!loader) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int row = (tid >> 5) + 8 * c;  // 0..31
          const long grow = m0 + pass * GS_EPR + row;
          const int gcol = n0 + ch * 8;
          float4 a = *reinterpret_cast<const float4*>(ep + gs_ep_idx32(row, ch * 8));
          float4 b = *reinterpret_cast<const float4*>(ep + gs_ep_idx32(row, ch * 8) + 4);
          a.x *= alpha; a.y *= alpha; a.z *= alpha; a.w *= alpha;
          b.x *= alpha; b.y *= alpha; b.z *= alpha; b.w *= alpha;
          float* dst = slab ? slab + grow * N + gcol : e.Cf + grow * e.ldcf + gcol;
          if (!slab && e.accumulate) {
            const float4 o0 = *reinterpret_cast<const float4*>(dst);
            const float4 o1 = *reinterpret_cast<const float4*>(dst + 4);
            a.x += o0.x; a.y += o0.y; a.z += o0.z; a.w += o0.w;
            b.x += o1.x; b.y += o1.y; b.z += o1.z; b.w += o1.w;
          }
          *reinterpret_cast<float4*>(dst) = a;
          *reinterpret_cast<float4*>(dst + 4) = b;
        }
      }
      smer_lds_barrier();
    }
  }
}

// db[m] (+)= sum_p part[p][m], p in order (deterministic).  64-thread
// blocks (M / 64 of them) with 8 partial loads in flight per thread: a
// serial chain of dependent-latency loads ran ~50 us per call beside the
// main stream's kernels.
__global__ __launch_bounds__(64) void wgrad_rowsum_reduce_kernel(int M, int nparts, const float* __restrict__ part,
                                                                 float* __restrict__ db, int accumulate) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float t = 0.f;
  int p = 0;
  for (; p + 8 <= nparts; p += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(long)(p + u) * M + m];
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  for (; p < nparts; ++p) t += part[(long)p * M + m];
  db[m] = (accumulate ? db[m] : 0.f) + t;
}

// dW[M, N] (+)= dy_inv x_inv sum_t dy8[t, m] x8[t, n],
// db[M] (+)= dy_inv sum_t dy8[t, m]  (K = tokens)
extern "C" int smer_gemm_wgrad_fp8(int M, int N, int K, const void* dy8, long lddy, const void* x8, long ldx,
                                   const float* dy_inv, const float* x_inv, float* dW, long lddw, int accumulate,
                                   float* db, int db_accumulate, void* workspace, size_t ws_bytes,
                                   int max_workgroups, smer_stream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % G2 || N % G2 || K % (2 * GS_KS))
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_gemm_wgrad_fp8: needs M, N % 256 == 0 and K % 64 == 0");
  SMER_REQUIRE(dy8 && x8 && dy_inv && x_inv && dW && (!db || workspace), "smer_gemm_wgrad_fp8: null pointer");
  SMER_REQUIRE(aligned16(dy8) && aligned16(x8) && lddy % 16 == 0 && ldx % 16 == 0 && lddy >= M && ldx >= N &&
                   aligned16(dW) && lddw % 4 == 0 && lddw >= N && (!workspace || aligned16(workspace)),
               "smer_gemm_wgrad_fp8: operand strides / alignment");
  hipStream_t s = (hipStream_t)stream;
  GemmEpi e{};
  e.alpha = 1.f; e.drop_scale = 1.f;
  e.Cf = dW; e.ldcf = lddw; e.accumulate = accumulate; e.vec = 1; e.rs_accumulate = db_accumulate;
  g_wgrad_cap = max_workgroups > 0 ? max_workgroups : 0;
  const long t2 = (long)(M / G2) * (N / G2);
  const int nbn = N / G2;
  const long cus = smer_num_cus();
  long ns = std::min<long>(smer_wgrad256_slots() / t2, K / smer_wgrad256_depth());
  // per slice: an M x N slab and nbn x M bias partials
  ns = std::min<long>(ns, (long)(splitk_slab_bytes(workspace ? ws_bytes : 0) /
                                 (((size_t)M * N + (size_t)nbn * M) * sizeof(float))));
  ns = std::max<long>(1, std::min<long>(ns, 64));
  const int KS = 2 * GS_KS;
  const int kchunk = (int)(((K + ns - 1) / ns + KS - 1) / KS * KS);
  const int split = (K + kchunk - 1) / kchunk;
  const long nwg = t2 * split;
  const long gcap = wgrad_cap(cus);
  g_wgrad_cap = 0;
  const int grid = nwg > gcap ? (int)(gcap & ~7L) : (int)nwg;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)gemm256s_wgrad_fp8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        4 * GS_SLOT);
    attr = true;
  }
  // split-K: alpha-scaled slabs, then the bias partials
  const size_t slab_floats = split > 1 ? (size_t)split * M * N : 0;
  float* rs_part = db ? (float*)workspace + slab_floats : nullptr;
  if (db && (slab_floats + (size_t)split * nbn * M) * sizeof(float) > splitk_slab_bytes(ws_bytes))
    return smer_set_error(SMER_ERR_INVALID, "smer_gemm_wgrad_fp8: workspace too small for the bias partials");
  hipLaunchKernelGGL(gemm256s_wgrad_fp8_kernel, dim3(grid), dim3(512), 4 * GS_SLOT, s, M, N, K,
                     (const uint8_t*)dy8, lddy, (const uint8_t*)x8, ldx, dy_inv, x_inv, e, split, kchunk,
                     (float*)workspace, rs_part);
  if (split > 1) {
    const long n4 = ((long)M * N) / 4;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((n4 + 255) / 256), dim3(256), 0, s, M, N, split,
                       (const float*)workspace, 1.f, dW, lddw, accumulate, (const float*)nullptr, (float*)nullptr,
                       0);
  }
  if (db)
    hipLaunchKernelGGL(wgrad_rowsum_reduce_kernel, dim3((M + 63) / 64), dim3(64), 0, s, M, split * nbn,
                       (const float*)rs_part, db, db_accumulate);
  SMER_CHECK_LAUNCH("smer_gemm_wgrad_fp8");
  return SMER_OK;
}


extern "C" int smer_gemm_fp8_q(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                               const float* a_inv, const float* b_inv, const float* bias, int relu,
                               const void* residual, long ldr, float drop_p, uint32_t drop_seed,
                               void* C, long ldc, void* q8, long ldq8, const float* q8_scale,
                               unsigned* q8_amax, smer_stream_t stream);

// The staggered fp8 kernel for whole-tile bf16-output products: opt-in
// (SMER_GEMM256S_FP8=1 / 0 forces it on / off, read per call).  Isolated
// and warm (tools/gemm256s_fp8_ab.py, C4 rows 65536, operands re-used across
// iterations) it wins at K >= 1024 (FFN2 forward 122.3 vs 133.1 us, FFN1 /
// QKV dgrads 113.8 / 125.1 vs 123.0 / 131.7) and loses at K = 768 (QKV
// forward 160.7 vs 151.7); inside the C4 fp8 train step, whose operands
// arrive cold from HBM, the same K >= 1024 calls ran slower (paired
// kernel trace: 133.5 vs 129.3 us at the 130-us shapes, 794 vs 698 at the
// vocabulary-long K) and the step did not move (86.3 vs 85.9 ms), so the
// two-stage kernel stays the default.
// The e4m3-copy products (the gated FFN2 dgrad, FFN1 with SMER_FP8_FFN2)
// on the streamed epilogue, whose residual / gate rows arrive by LDS-DMA a
// pass ahead, one item at a time (round 6: C4 gated dgrad 65536 x 2048 x
// 768 301 -> 245 us, step 78.96-78.99 -> 78.48-78.57 ms); SMER_FP8_Q8_FAST=0
// (read per call) keeps the generic epilogue, whose gate loads are a
// dependent HBM round trip per pass
static bool smer_fp8_q8_fast() {
  const char* e = getenv("SMER_FP8_Q8_FAST");
  return !(e && e[0] == '0');
}
static bool smer_gemm256s_fp8_enabled(int K) {
  (void)K;
  const char* e = getenv("SMER_GEMM256S_FP8");
  return e && e[0] == '1';
}

extern "C" int smer_gemm_fp8(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                             const float* a_inv, const float* b_inv, const float* bias, int relu,
                             const void* residual, long ldr, float drop_p, uint32_t drop_seed,
                             void* C, long ldc, smer_stream_t stream) {
  return smer_gemm_fp8_q(M, N, K, A, lda, B, ldb, a_inv, b_inv, bias, relu, residual, ldr, drop_p,
                         drop_seed, C, ldc, nullptr, 0, nullptr, nullptr, stream);
}

extern "C" int smer_gemm_fp8_q(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                               const float* a_inv, const float* b_inv, const float* bias, int relu,
                               const void* residual, long ldr, float drop_p, uint32_t drop_seed,
                               void* C, long ldc, void* q8, long ldq8, const float* q8_scale,
                               unsigned* q8_amax, smer_stream_t stream) {
  return smer_gemm_fp8_ex(M, N, K, A, lda, B, ldb, a_inv, b_inv, bias, relu, residual, ldr, nullptr, 0, 1.f,
                          drop_p, drop_seed, C, ldc, q8, ldq8, q8_scale, q8_amax, stream);
}

static int gemm_fp8_impl(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                         const float* a_inv, const float* b_inv, const float* bias, int relu,
                         const void* residual, long ldr, const void* gate, long ldg, int gate_u8,
                         float gate_scale, float drop_p, uint32_t drop_seed, void* C, long ldc,
                         void* q8, long ldq8, const float* q8_scale, unsigned* q8_amax,
                         smer_stream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % G2 || N % G2 || K % F8K)
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_gemm_fp8: needs M, N % 256 == 0 and K % 128 == 0");
  // (C may be null only beside an e4m3 copy on the streamed epilogue: the
  // copy alone is written)
  const bool c_less = !C && q8 && smer_fp8_q8_fast();
  SMER_REQUIRE(A && B && (C || c_less) && a_inv && b_inv, "smer_gemm_fp8: null pointer");
  SMER_REQUIRE(!gate_u8 || (gate && q8 && smer_fp8_q8_fast() && ((uintptr_t)gate & 15) == 0 && ldg % 16 == 0),
               "smer_gemm_fp8_gate8: e4m3 gate needs the streamed e4m3-copy epilogue and 16-B aligned rows");
  SMER_REQUIRE(lda % 16 == 0 && ldb % 16 == 0 && aligned16(A) && aligned16(B),
               "smer_gemm_fp8: operand strides / alignment");
  SMER_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "smer_gemm_fp8: drop_p out of range");
  GemmEpi e{};
  e.bias = bias; e.alpha = 1.f; e.relu = relu; e.residual = residual; e.ldr = ldr;
  e.drop_thr = smer_drop_thr16(drop_p); e.seed = drop_seed;
  e.drop_scale = smer_drop_scale16(e.drop_thr);
  e.C = C; e.ldc = ldc;
  e.gate = gate; e.ldg = ldg; e.gate_scale = gate_scale;
  SMER_REQUIRE(!(gate && residual), "smer_gemm_fp8_ex: residual and gate are exclusive");
  auto a16 = [](const void* p, long ld) { return p == nullptr || ((((uintptr_t)p) & 15) == 0 && ld % 8 == 0); };
  e.vec = a16(bias, 8) && a16(residual, ldr) && a16(gate, ldg) && a16(C, ldc);
  SMER_REQUIRE((C && !gate_u8) || e.vec, "smer_gemm_fp8: the e4m3-only output and the e4m3 gate need aligned vectors");
  if (q8) {
    SMER_REQUIRE(e.vec && q8_scale && q8_amax && (((uintptr_t)q8) & 7) == 0 && ldq8 % 8 == 0,
                 "smer_gemm_fp8_q: fp8 output needs aligned vectors, scale and amax");
    e.q8 = (uint8_t*)q8; e.ldq8 = ldq8; e.q8_scale = q8_scale; e.q8_amax = q8_amax;
  }
  hipStream_t s = (hipStream_t)stream;
  const long tiles = (long)(M / G2) * (N / G2);
  const int grid = tiles > smer_num_cus() ? (smer_num_cus() & ~7) : (int)tiles;
  if (e.vec && !q8 && K % (2 * GS_KS) == 0 && K / (2 * GS_KS) >= 4 && smer_gemm256s_fp8_enabled(K)) {
    static bool attr_s = false;
    if (!attr_s) {
      hipFuncSetAttribute((const void*)gemm256s_fp8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
      attr_s = true;
    }
    hipLaunchKernelGGL(gemm256s_fp8_kernel, dim3(grid), dim3(512), G2_LDS, s, M, N, K, (const uint8_t*)A, lda,
                       (const uint8_t*)B, ldb, a_inv, b_inv, e);
    SMER_CHECK_LAUNCH("smer_gemm_fp8");
    return SMER_OK;
  }
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm256_fp8_kernel<false, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * G2_STAGE);
    hipFuncSetAttribute((const void*)gemm256_fp8_kernel<true, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
    hipFuncSetAttribute((const void*)gemm256_fp8_kernel<false, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * G2_STAGE);
    attr_set = true;
  }
  if (!e.vec)  // (q8 requires e.vec)
    hipLaunchKernelGGL((gemm256_fp8_kernel<false, false>), dim3(grid), dim3(512), 2 * G2_STAGE, s, M, N,
                       K, (const uint8_t*)A, lda, (const uint8_t*)B, ldb, a_inv, b_inv, e);
  else if (gate_u8) {
    static bool attr_g8 = false;
    if (!attr_g8) {
      hipFuncSetAttribute((const void*)gemm256_fp8_kernel<true, true, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, G2_LDS);
      attr_g8 = true;
    }
    hipLaunchKernelGGL((gemm256_fp8_kernel<true, true, true>), dim3(grid), dim3(512), G2_LDS, s, M, N, K,
                       (const uint8_t*)A, lda, (const uint8_t*)B, ldb, a_inv, b_inv, e);
  } else if (q8 && smer_fp8_q8_fast()) {
    static bool attr_q = false;
    if (!attr_q) {
      hipFuncSetAttribute((const void*)gemm256_fp8_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          G2_LDS);
      attr_q = true;
    }
    hipLaunchKernelGGL((gemm256_fp8_kernel<true, true>), dim3(grid), dim3(512), G2_LDS, s, M, N, K,
                       (const uint8_t*)A, lda, (const uint8_t*)B, ldb, a_inv, b_inv, e);
  } else if (q8)
    hipLaunchKernelGGL((gemm256_fp8_kernel<false, true>), dim3(grid), dim3(512), 2 * G2_STAGE, s, M, N, K,
                       (const uint8_t*)A, lda, (const uint8_t*)B, ldb, a_inv, b_inv, e);
  else
    hipLaunchKernelGGL((gemm256_fp8_kernel<true, false>), dim3(grid), dim3(512), G2_LDS, s, M, N, K,
                       (const uint8_t*)A, lda, (const uint8_t*)B, ldb, a_inv, b_inv, e);
  SMER_CHECK_LAUNCH("smer_gemm_fp8");
  return SMER_OK;
}

extern "C" int smer_gemm_fp8_ex(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                                const float* a_inv, const float* b_inv, const float* bias, int relu,
                                const void* residual, long ldr, const void* gate, long ldg,
                                float gate_scale, float drop_p, uint32_t drop_seed, void* C, long ldc,
                                void* q8, long ldq8, const float* q8_scale, unsigned* q8_amax,
                                smer_stream_t stream) {
  return gemm_fp8_impl(M, N, K, A, lda, B, ldb, a_inv, b_inv, bias, relu, residual, ldr, gate, ldg, 0,
                       gate_scale, drop_p, drop_seed, C, ldc, q8, ldq8, q8_scale, q8_amax, stream);
}

// The gated FFN2 dgrad of the fp8 step with FFN1's e4m3 copy as the ReLU /
// dropout gate (open where the byte is a positive nonzero e4m3), so FFN1
// need not keep its bf16 output (transformer.py:467-469 under train.py:783).
extern "C" int smer_gemm_fp8_gate8(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                                   const float* a_inv, const float* b_inv, const void* gate8, long ldg,
                                   float gate_scale, void* C, long ldc, void* q8, long ldq8,
                                   const float* q8_scale, unsigned* q8_amax, smer_stream_t stream) {
  return gemm_fp8_impl(M, N, K, A, lda, B, ldb, a_inv, b_inv, nullptr, 0, nullptr, 0, gate8, ldg, 1,
                       gate_scale, 0.f, 0u, C, ldc, q8, ldq8, q8_scale, q8_amax, stream);
}
