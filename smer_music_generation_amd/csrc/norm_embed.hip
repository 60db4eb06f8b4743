// LayerNorm (post-LN residual blocks, eps 1e-5; transformer.py:392,395,462,
// 466,469 and the final norms 274-275, 329-330) and the embedding + PE
// front end (model.py:91-92, 124-125).  All HBM-bound: one wave per row,
// 16-B vector loads, fp32 math, deterministic two-stage column reductions
// for dgamma / dbeta / dtable.
#include "common.h"

namespace {
constexpr int LN_MAXC = 4;  // 16-B chunks per lane: N <= 64*8*4 = 2048

template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&v)[8]) {
    bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
  }
  static __device__ __forceinline__ void store(bf16* p, const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = r;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
};
}  // namespace

// Q8: also the e4m3 copy of y (delayed scaling, common.h) for an fp8 GEMM;
// NC: 16-B chunks per lane the register arrays are sized for (N <= 512 * NC)
template <typename T, bool Q8 = false, int NC = LN_MAXC>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int M, int N, const T* __restrict__ x, long ldx,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     T* __restrict__ y, long ldy,
                                                     float* __restrict__ mean,
                                                     float* __restrict__ rstd,
                                                     uint8_t* __restrict__ q8 = nullptr, long ldq = 0,
                                                     const float* __restrict__ qs_p = nullptr,
                                                     unsigned* __restrict__ amax = nullptr) {
  const int lane = threadIdx.x & 63;
  const int nch = N >> 3;
  float gb[NC][16];  // gamma | beta of the lane's chunks, issued before x
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      Vec8<float>::load(gamma + ch * 8, *reinterpret_cast<float(*)[8]>(&gb[c][0]));
      Vec8<float>::load(beta + ch * 8, *reinterpret_cast<float(*)[8]>(&gb[c][8]));
    }
  }
  float am = 0.f;
  // a wave is one row (wave-uniform loop; the grid covers M once except in
  // the Q8 form, whose capped grid loops so that the amax of the whole
  // tensor is committed by <= 2048 workgroups instead of one atomic per row)
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += gridDim.x * 4) {
  float v[NC][8], mu, rs;
  ln_row_stats<T, NC>(x + (long)row * ldx, N, eps, lane, v, mu, rs);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int ch = lane + 64 * c;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = ln_apply(v[c][i], mu, rs, gb[c][i], gb[c][8 + i]);
      Vec8<T>::store(y + (long)row * ldy + ch * 8, o);
      if constexpr (Q8) {
        // quantise the value the bf16 output holds (what the bf16 path reads)
        float r[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = (float)(T)o[i];
        *reinterpret_cast<uint2*>(q8 + (long)row * ldq + ch * 8) = smer_q8x8(r, *qs_p);
        am = fmaxf(am, smer_absmax8(r));
      }
    }
  }
  if (lane == 0) {
    if (mean) mean[row] = mu;
    if (rstd) rstd[row] = rs;
  }
  }
  if constexpr (Q8) {
    __shared__ float wam[4];
    am = wave_max(am);
    if (lane == 0) wam[threadIdx.x >> 6] = am;
    __syncthreads();
    if (threadIdx.x < 64) smer_amax_commit(amax, lane < 4 ? wam[lane] : 0.f);
  }
}

// bf16 forward, RPW rows per wave: all RPW rows' loads are issued before
// the first row's statistics (raw registers: a conversion right after a
// load would make hipcc wait for it there), so a wave keeps RPW KiB of x in
// flight instead of one row's; gamma / beta are read once per RPW rows.
// NC = 16-B chunks per lane (N <= 512 * NC) sizes the register arrays, so a
// d = 512 row costs a few dozen VGPRs.  Per-row arithmetic is ln_row_stats'
// (bit-identical outputs).
template <int RPW, int NC>
__global__ __launch_bounds__(256) void ln_fwd_rows_kernel(int M, int N, const bf16* __restrict__ x,
                                                          long ldx, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          bf16* __restrict__ y, long ldy,
                                                          float* __restrict__ mean,
                                                          float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int nch = N >> 3;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= M) return;  // wave-uniform
  bf16x8 raw[RPW][NC];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const long row = min(row0 + r, M - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c)  // chunk clamped, not guarded (a guarded load waited behind it)
      raw[r][c] = *reinterpret_cast<const bf16x8*>(x + row * ldx + min(lane + 64 * c, nch - 1) * 8);
  }
  float gb[NC][16];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = min(lane + 64 * c, nch - 1);
    Vec8<float>::load(gamma + ch * 8, *reinterpret_cast<float(*)[8]>(&gb[c][0]));
    Vec8<float>::load(beta + ch * 8, *reinterpret_cast<float(*)[8]>(&gb[c][8]));
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int row = row0 + r;
    if (row >= M) break;  // wave-uniform
    float v[NC][8], s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (lane + 64 * c < nch)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          v[c][i] = (float)raw[r][c][i];
          s += v[c][i];
        }
    const float mu = wave_sum(s) / N;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (lane + 64 * c < nch)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = v[c][i] - mu;
          q += d * d;
        }
    const float rs = rsqrtf(wave_sum(q) / N + eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = ln_apply(v[c][i], mu, rs, gb[c][i], gb[c][8 + i]);
        Vec8<bf16>::store(y + (long)row * ldy + ch * 8, o);
      }
    }
    if (lane == 0) {
      if (mean) mean[row] = mu;
      if (rstd) rstd[row] = rs;
    }
  }
}

// rows per wave of the bf16 forward: 1 from 16384 rows, else 4 (measured,
// tools/ln_bench.py: 32768 x 512 13.3 us at 1, 14.0 at 2, 16.5 at 4, 18.8
// for ln_fwd_kernel, whose arrays sized for N = 2048 cost 130 VGPRs; 8192
// rows 9.2-9.8 us for all); SMER_LN_RPW = 1 / 2 / 4 forces it, 0 = the
// one-row ln_fwd_kernel (A/B)
static int ln_fwd_rpw(int M) {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("SMER_LN_RPW");
    v = e ? atoi(e) : -1;
    if (v != 0 && v != 1 && v != 2 && v != 4) v = -1;
  }
  return v >= 0 ? v : (M >= 16384 ? 1 : 4);
}

// rows per workgroup: 64 (16 per wave) for large M; 16 (one RB batch of 4
// per wave) when 64 would leave the grid under ~2 workgroups per CU (the
// decoder's 8192 rows: 19.6 vs 23.9 us; 64 stays better at 32768 rows,
// where 4x the column partials cost more than the extra parallelism gives)
constexpr int LN_BWD_ROWS = 64;
constexpr int LN_BWD_ROWS_SMALL = 16;
static inline int ln_bwd_rows_fixed(int M) { return M <= 16384 ? LN_BWD_ROWS_SMALL : LN_BWD_ROWS; }
static int ln_bwd_rows(int M, int N);  // below the kernel (needs its occupancy)

// One wave per row, NC 16-B chunks per lane (N <= 512 * NC); a wave takes
// its 16 rows of the block RB at a time with all RB rows' loads issued
// together (the rows are otherwise a chain of dependent HBM round trips at
// 2 waves per SIMD).  Column partials for dgamma / dbeta accumulate in a
// fixed row order (deterministic).
// Q8 (fp8 backward): also the e4m3 copy of the stored gradient that feeds the
// next dgrad (dxd when given, else dx) and its amax (delayed scaling, common.h)
template <typename T, bool DYF, int NC, int RB, bool PFB, bool Q8 = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int M, int N, const void* __restrict__ dyv,
                                                     long lddy, const T* __restrict__ x, long ldx,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma,
                                                     T* __restrict__ dx, long lddx,
                                                     T* __restrict__ dxd, long ldxd,
                                                     uint32_t thr, uint32_t seed, float dscale,
                                                     float* __restrict__ part, int rows_per_blk,
                                                     uint8_t* __restrict__ q8 = nullptr, long ldq = 0,
                                                     const float* __restrict__ qs_p = nullptr,
                                                     unsigned* __restrict__ amax = nullptr) {
  constexpr int LN_MAXC = NC;
  __shared__ float red[4][2][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = N >> 3;
  float pg[NC][8], pb[NC][8], gm[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) Vec8<float>::load(gamma + ch * 8, gm[c]);
#pragma unroll
    for (int i = 0; i < 8; ++i) { pg[c][i] = 0.f; pb[c][i] = 0.f; }
  }
  const int r0 = blockIdx.x * rows_per_blk;
  float q8s = 1.f, am = 0.f;
  if constexpr (Q8) q8s = *qs_p;
  // bf16: the next batch's rows are fetched raw (16-B words, unclamped
  // statistics) before this batch's math, so a wave keeps two batches in
  // flight; every conversion / validity select happens at unpack time (a
  // select right behind a load makes hipcc wait for it there)
  // (bf16 without PFB -- one batch per wave -- fetches its batch raw the
  // same way, just not a batch ahead: the guarded, converted loads of the
  // plain path made hipcc wait behind each load)
  constexpr bool RAW = sizeof(T) == 2;
  constexpr bool PF = PFB && RAW;  // PFB: several batches per wave (64-row blocks)
  constexpr int DW = DYF ? 2 : 1;  // 16-B words of dy per 8 columns
  uint4 px[RAW ? RB : 1][NC], pd[RAW ? RB : 1][NC][DW];
  float pmu[RAW ? RB : 1], prs[RAW ? RB : 1];
  auto fetch = [&](int rb) {
    if constexpr (RAW) {
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int row = min(r0 + wave + 4 * (rb + u), M - 1);
        pmu[u] = mean[row];
        prs[u] = rstd[row];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int ch = lane + 64 * c;
          if (ch < nch) {
            px[u][c] = *reinterpret_cast<const uint4*>(x + (long)row * ldx + ch * 8);
            if constexpr (DYF) {
              const uint4* d = reinterpret_cast<const uint4*>((const float*)dyv + (long)row * lddy + ch * 8);
              pd[u][c][0] = d[0];
              pd[u][c][DW - 1] = d[1];
            } else {
              pd[u][c][0] = *reinterpret_cast<const uint4*>((const T*)dyv + (long)row * lddy + ch * 8);
            }
          }
        }
      }
    }
  };
  if constexpr (PF) fetch(0);
  for (int rb = 0; rb < rows_per_blk / 4; rb += RB) {
    float xh[RB][NC][8], gd[RB][NC][8], mu[RB], rs[RB];
    bool ok[RB];
    if constexpr (RAW && !PF) fetch(rb);
    if constexpr (RAW) {
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int row = r0 + wave + 4 * (rb + u);
        ok[u] = row < M;
        mu[u] = ok[u] ? pmu[u] : 0.f;
        rs[u] = ok[u] ? prs[u] : 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const bf16x8 xv = __builtin_bit_cast(bf16x8, px[u][c]);
#pragma unroll
          for (int i = 0; i < 8; ++i) xh[u][c][i] = (float)xv[i];
          if constexpr (DYF) {
            const float* f0 = reinterpret_cast<const float*>(&pd[u][c][0]);
            const float* f1 = reinterpret_cast<const float*>(&pd[u][c][DW - 1]);
#pragma unroll
            for (int i = 0; i < 4; ++i) { gd[u][c][i] = f0[i]; gd[u][c][4 + i] = f1[i]; }
          } else {
            const bf16x8 dv = __builtin_bit_cast(bf16x8, pd[u][c][0]);
#pragma unroll
            for (int i = 0; i < 8; ++i) gd[u][c][i] = (float)dv[i];
          }
        }
      }
      if (PF && rb + RB < rows_per_blk / 4) fetch(rb + RB);
    } else {
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const int row = r0 + wave + 4 * (rb + u);
        ok[u] = row < M;
        mu[u] = ok[u] ? mean[row] : 0.f;
        rs[u] = ok[u] ? rstd[row] : 0.f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int ch = lane + 64 * c;
          if (ok[u] && ch < nch) {
            Vec8<T>::load(x + (long)row * ldx + ch * 8, xh[u][c]);
            if (DYF) Vec8<float>::load((const float*)dyv + (long)row * lddy + ch * 8, gd[u][c]);
            else Vec8<T>::load((const T*)dyv + (long)row * lddy + ch * 8, gd[u][c]);
          }
        }
      }
    }
    float s1[RB], s2[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = 0.f;
      s2[u] = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + 64 * c;
        if (ok[u] && ch < nch)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float dv = gd[u][c][i];
            const float h = (xh[u][c][i] - mu[u]) * rs[u];
            const float gg = dv * gm[c][i];
            xh[u][c][i] = h;
            gd[u][c][i] = gg;
            s1[u] += gg;
            s2[u] += gg * h;
            pg[c][i] += dv * h;
            pb[c][i] += dv;
          }
      }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = wave_sum(s1[u]) / N;
      s2[u] = wave_sum(s2[u]) / N;
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = r0 + wave + 4 * (rb + u);
      const uint32_t rowkey = thr ? smer_rowkey(seed, (uint32_t)row) : 0u;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + 64 * c;
        if (ok[u] && ch < nch) {
          float o[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = rs[u] * (gd[u][c][i] - s1[u] - xh[u][c][i] * s2[u]);
          Vec8<T>::store(dx + (long)row * lddx + ch * 8, o);
          if (dxd || (Q8 && thr)) {  // (Q8 without dxd: the dropped values' e4m3 copy alone)
            if (thr) smer_drop8(rowkey, thr, dscale, (uint32_t)(ch * 8), o);
            if (dxd) Vec8<T>::store(dxd + (long)row * ldxd + ch * 8, o);
          }
          if constexpr (Q8) {  // e4m3 copy of the stored (T-rounded) values
            float r[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = (float)(T)o[i];
            *reinterpret_cast<uint2*>(q8 + (long)row * ldq + ch * 8) = smer_q8x8(r, q8s);
            am = fmaxf(am, smer_absmax8(r));
          }
        }
      }
    }
  }
  if constexpr (Q8) {  // one atomic per workgroup (per wave: 16k waves contend on one address)
    __shared__ float wam[4];
    am = wave_max(am);
    if (lane == 0) wam[wave] = am;
    __syncthreads();
    if (threadIdx.x < 64) smer_amax_commit(amax, lane < 4 ? wam[lane] : 0.f);
  }
  if (!part) return;
  // combine the 4 waves' column partials in fixed order, in <=512-col slabs
  for (int base = 0; base < N; base += 512) {
#pragma unroll
    for (int c = 0; c < LN_MAXC; ++c) {
      int ch = lane + 64 * c;
      if (ch < nch && ch * 8 >= base && ch * 8 < base + 512)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          red[wave][0][ch * 8 + i - base] = pg[c][i];
          red[wave][1][ch * 8 + i - base] = pb[c][i];
        }
    }
    __syncthreads();
    for (int col = threadIdx.x; col < 512 && base + col < N; col += 256) {
      float a = (red[0][0][col] + red[1][0][col]) + (red[2][0][col] + red[3][0][col]);
      float b = (red[0][1][col] + red[1][1][col]) + (red[2][1][col] + red[3][1][col]);
      part[(long)blockIdx.x * 2 * N + base + col] = a;
      part[(long)blockIdx.x * 2 * N + N + base + col] = b;
    }
    __syncthreads();
  }
}


// ---------------------------------------------------------------------------
// embedding + sinusoidal PE
// ---------------------------------------------------------------------------
// Q8 (fp8 training, the first layers' QKV input): also the e4m3 copy
// e4m3(out * *qs) of the stored bf16 values, max |out| folded into *amax
// (delayed scaling, common.h)
template <typename T, bool Q8 = false>
__global__ void embed_fwd_kernel(int n_tok, int d, const int64_t* __restrict__ ids,
                                 const int32_t* __restrict__ positions, int L,
                                 const float* __restrict__ table, const float* __restrict__ pe,
                                 float scale, uint32_t thr, uint32_t seed, float dscale,
                                 T* __restrict__ out, long ldo, uint8_t* __restrict__ q8 = nullptr,
                                 long ldq = 0, const float* __restrict__ qs_p = nullptr,
                                 unsigned* __restrict__ amax = nullptr) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = d >> 2;
  const bool ok = idx < (long)n_tok * per;
  if (!Q8 && !ok) return;  // (Q8: every lane reaches the wave-wide amax)
  float am = 0.f;
  if (ok) {
    int t = idx / per, c = (idx % per) * 4;
    long id = ids[t];
    int pos = positions ? positions[t] : t % L;
    float4 e = *reinterpret_cast<const float4*>(table + id * d + c);
    float4 p = *reinterpret_cast<const float4*>(pe + (long)pos * d + c);
    float v[4] = {e.x * scale + p.x, e.y * scale + p.y, e.z * scale + p.z, e.w * scale + p.w};
    T* o = out + (long)t * ldo + c;
    float f[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float w = v[i];
      if (thr) w = smer_keep16(smer_rowkey(seed, (uint32_t)t), thr, (uint32_t)(c + i)) ? w * dscale : 0.f;
      const T ov = from_f32<T>(w);
      o[i] = ov;
      f[i] = to_f32(ov);
    }
    if constexpr (Q8) {
      *reinterpret_cast<uint32_t*>(q8 + (long)t * ldq + c) = smer_q8x4(f, *qs_p);
      am = smer_absmax4(f);
    }
  }
  if constexpr (Q8) smer_amax_commit(amax, am);
}

constexpr int EMB_CHUNK = 512;  // tokens per workgroup in the per-vocab gather

// part[chunk][v][:] = sum over tokens t of this chunk with id v of dx[t] * keep
// A lane owns 8 consecutive columns (chunks lane, lane + 64: d <= 1024) and
// reads them with one 16-B load per row; the matching rows of a 64-token
// group are fetched up to 4 at a time (independent loads in flight) and
// added in ascending token order, so the sums are those of a serial scan.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_gather(
    int V, int d, const int64_t* __restrict__ ids0, const T* __restrict__ dx0, long ld0, int n0,
    uint32_t thr0, uint32_t seed0, float ds0, const int64_t* __restrict__ ids1,
    const T* __restrict__ dx1, long ld1, int n1, uint32_t thr1, uint32_t seed1, float ds1,
    float* __restrict__ part) {
  __shared__ float red[4][1024];
  const int v = blockIdx.x, chunk = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nch = d >> 3;  // 8-column chunks (d % 8 == 0 for bf16 / fp32 vectors)
  float acc[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[c][i] = 0.f;
  const int n = n0 + n1;
  const int t_begin = chunk * EMB_CHUNK + wave * (EMB_CHUNK / 4);
  for (int g0 = t_begin; g0 < t_begin + EMB_CHUNK / 4 && g0 < n; g0 += 64) {
    int t = g0 + lane;
    bool hit = false;
    if (t < n) hit = (t < n0 ? ids0[t] : ids1[t - n0]) == v;
    unsigned long long mask = __ballot(hit);
    while (mask) {
      int tt[4], cnt = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        tt[k] = -1;
        if (mask) {
          tt[k] = g0 + __ffsll((long long)mask) - 1;
          mask &= mask - 1;
          cnt = k + 1;
        }
      }
      float g[4][2][8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < cnt) {
          const bool s0 = tt[k] < n0;
          const int tl = s0 ? tt[k] : tt[k] - n0;
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int ch = lane + 64 * c;
            if (ch < nch) {
              if (s0) Vec8<T>::load(dx0 + (long)tl * ld0 + ch * 8, g[k][c]);
              else Vec8<T>::load(dx1 + (long)tl * ld1 + ch * 8, g[k][c]);
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < cnt) {
          const bool s0 = tt[k] < n0;
          const int tl = s0 ? tt[k] : tt[k] - n0;
          const uint32_t thr = s0 ? thr0 : thr1;
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int ch = lane + 64 * c;
            if (ch < nch) {
              if (thr) smer_drop8(smer_rowkey(s0 ? seed0 : seed1, (uint32_t)tl), thr, s0 ? ds0 : ds1,
                                  (uint32_t)(ch * 8), g[k][c]);
#pragma unroll
              for (int i = 0; i < 8; ++i) acc[c][i] += g[k][c][i];
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[wave][ch * 8 + i] = acc[c][i];
  }
  __syncthreads();
  float* dst = part + ((long)chunk * V + v) * d;
  for (int col = threadIdx.x; col < d; col += 256)
    dst[col] = (red[0][col] + red[1][col]) + (red[2][col] + red[3][col]);
}

__global__ void embed_bwd_reduce(int V, int d, int nchunk, const float* __restrict__ part,
                                 float scale, float* __restrict__ dtable) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)V * d) return;
  float a = 0.f;
  for (int c = 0; c < nchunk; ++c) a += part[(long)c * V * d + idx];
  dtable[idx] += a * scale;
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" int smer_layernorm_fwd(int dtype, int M, int N, const void* x, long ldx,
                                  const float* gamma, const float* beta, float eps, void* y,
                                  long ldy, float* mean, float* rstd, smer_stream_t stream) {
  SMER_REQUIRE(N % 8 == 0 && N <= 64 * 8 * LN_MAXC, "smer_layernorm_fwd: N % 8 == 0 and N <= 2048");
  SMER_REQUIRE(ldx % 8 == 0 && ldy % 8 == 0, "smer_layernorm_fwd: strides % 8");
  SMER_REQUIRE((((uintptr_t)gamma | (uintptr_t)beta) & 15) == 0,
               "smer_layernorm_fwd: gamma / beta must be 16-B aligned");
  if (M == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((M + 3) / 4);
  const int rpw = dtype == SMER_BF16 ? ln_fwd_rpw(M) : 0;
  if (rpw > 0) {
    const int nc = N <= 512 ? 1 : N <= 1024 ? 2 : 4;
#define LNF(R) (nc == 1 ? ln_fwd_rows_kernel<R, 1> : nc == 2 ? ln_fwd_rows_kernel<R, 2> : ln_fwd_rows_kernel<R, 4>)
    auto kern = rpw == 1 ? LNF(1) : rpw == 2 ? LNF(2) : LNF(4);
#undef LNF
    hipLaunchKernelGGL(kern, dim3((M + 4 * rpw - 1) / (4 * rpw)), dim3(256), 0, s, M, N,
                       (const bf16*)x, ldx, gamma, beta, eps, (bf16*)y, ldy, mean, rstd);
  } else if (dtype == SMER_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16>, grid, dim3(256), 0, s, M, N, (const bf16*)x, ldx, gamma,
                       beta, eps, (bf16*)y, ldy, mean, rstd);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, s, M, N, (const float*)x, ldx,
                       gamma, beta, eps, (float*)y, ldy, mean, rstd);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_layernorm_fwd: dtype");
  SMER_CHECK_LAUNCH("smer_layernorm_fwd");
  return SMER_OK;
}

extern "C" int smer_layernorm_fwd_fp8(int M, int N, const void* x, long ldx, const float* gamma,
                                      const float* beta, float eps, void* y, long ldy, float* mean,
                                      float* rstd, void* q8, long ldq, const float* qs,
                                      unsigned* amax, smer_stream_t stream) {
  SMER_REQUIRE(N % 8 == 0 && N <= 64 * 8 * LN_MAXC, "smer_layernorm_fwd_fp8: N % 8 == 0 and N <= 2048");
  SMER_REQUIRE(ldx % 8 == 0 && ldy % 8 == 0 && ldq % 8 == 0, "smer_layernorm_fwd_fp8: strides % 8");
  SMER_REQUIRE(q8 && qs && amax && (((uintptr_t)q8) & 7) == 0, "smer_layernorm_fwd_fp8: fp8 output");
  SMER_REQUIRE((((uintptr_t)gamma | (uintptr_t)beta) & 15) == 0,
               "smer_layernorm_fwd_fp8: gamma / beta must be 16-B aligned");
  if (M == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(std::min((M + 3) / 4, 2048));
  auto kern = N <= 512 ? ln_fwd_kernel<bf16, true, 1> : N <= 1024 ? ln_fwd_kernel<bf16, true, 2>
                                                                   : ln_fwd_kernel<bf16, true, 4>;
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, M, N, (const bf16*)x, ldx, gamma, beta, eps,
                     (bf16*)y, ldy, mean, rstd, (uint8_t*)q8, ldq, qs, amax);
  SMER_CHECK_LAUNCH("smer_layernorm_fwd_fp8");
  return SMER_OK;
}

// Delayed scaling: per site, the scale of this step from the amax the
// producers recorded in the previous one (amax_prev), and the next step's
// amax slot cleared.  qs = 448 / amax, inv = amax / 448 (1 / 1 when zero).
__global__ void fp8_scales_kernel(int n, const unsigned* __restrict__ amax_prev,
                                  float* __restrict__ qs, float* __restrict__ inv,
                                  unsigned* __restrict__ amax_next) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = __uint_as_float(amax_prev[i]);
  const bool ok = a > 0.f && a < 3.0e38f;
  qs[i] = ok ? smer_div_rn(448.f, a) : 1.f;
  inv[i] = ok ? smer_div_rn(a, 448.f) : 1.f;
  amax_next[i] = 0u;
}

extern "C" int smer_fp8_scales(int n, const unsigned* amax_prev, float* qs, float* inv,
                               unsigned* amax_next, smer_stream_t stream) {
  SMER_REQUIRE(n >= 0 && (n == 0 || (amax_prev && qs && inv && amax_next)), "smer_fp8_scales: pointers");
  if (n == 0) return SMER_OK;
  hipLaunchKernelGGL(fp8_scales_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n,
                     amax_prev, qs, inv, amax_next);
  SMER_CHECK_LAUNCH("smer_fp8_scales");
  return SMER_OK;
}

// bf16 backward for 512 < N <= 768 (C4: d = 768): lane l owns columns
// 8l .. 8l+7 (16-B chunk) and 512 + 4l .. +3 (8-B chunk), so every lane
// carries 12 columns instead of ln_bwd_kernel's two 16-B chunks with half
// the lanes idle on the second; RB rows per batch, the next batch fetched
// raw before this batch's math.  Same per-element arithmetic, dropout
// decisions (pair hashes of (row, col)) and partial layout as ln_bwd_kernel;
// the row sums s1 / s2 add the lane's 12 columns in another order.
template <int RB, bool Q8 = false>
__global__ __launch_bounds__(256) void ln_bwd_t4_kernel(int M, int N, const bf16* __restrict__ dy,
                                                        long lddy, const bf16* __restrict__ x, long ldx,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma,
                                                        bf16* __restrict__ dx, long lddx,
                                                        bf16* __restrict__ dxd, long ldxd,
                                                        uint32_t thr, uint32_t seed, float dscale,
                                                        float* __restrict__ part, int rows_per_blk,
                                                        uint8_t* __restrict__ q8 = nullptr, long ldq = 0,
                                                        const float* __restrict__ qs_p = nullptr,
                                                        unsigned* __restrict__ amax = nullptr) {
  __shared__ float red[4][2][256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = 8 * lane, ct = 512 + 4 * lane;
  const bool tok = ct < N;
  float gm[12], pg[12], pb[12];
  {
    const float4 a = *reinterpret_cast<const float4*>(gamma + c0);
    const float4 b2 = *reinterpret_cast<const float4*>(gamma + c0 + 4);
    const float4 t = tok ? *reinterpret_cast<const float4*>(gamma + ct) : make_float4(0.f, 0.f, 0.f, 0.f);
    gm[0] = a.x; gm[1] = a.y; gm[2] = a.z; gm[3] = a.w; gm[4] = b2.x; gm[5] = b2.y; gm[6] = b2.z;
    gm[7] = b2.w; gm[8] = t.x; gm[9] = t.y; gm[10] = t.z; gm[11] = t.w;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  const int r0 = blockIdx.x * rows_per_blk;
  float q8s = 1.f, am = 0.f;
  if constexpr (Q8) q8s = *qs_p;
  uint4 px[RB], pd[RB];
  uint2 pxt[RB], pdt[RB];
  float pmu[RB], prs[RB];
  auto fetch = [&](int rb) {
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = min(r0 + wave + 4 * (rb + u), M - 1);
      pmu[u] = mean[row];
      prs[u] = rstd[row];
      px[u] = *reinterpret_cast<const uint4*>(x + (long)row * ldx + c0);
      pd[u] = *reinterpret_cast<const uint4*>(dy + (long)row * lddy + c0);
      if (tok) {
        pxt[u] = *reinterpret_cast<const uint2*>(x + (long)row * ldx + ct);
        pdt[u] = *reinterpret_cast<const uint2*>(dy + (long)row * lddy + ct);
      } else {
        pxt[u] = make_uint2(0u, 0u);
        pdt[u] = make_uint2(0u, 0u);
      }
    }
  };
  fetch(0);
  for (int rb = 0; rb < rows_per_blk / 4; rb += RB) {
    float xh[RB][12], gd[RB][12], mu[RB], rs[RB];
    bool ok[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int row = r0 + wave + 4 * (rb + u);
      ok[u] = row < M;
      mu[u] = ok[u] ? pmu[u] : 0.f;
      rs[u] = ok[u] ? prs[u] : 0.f;
      const bf16x8 xv = __builtin_bit_cast(bf16x8, px[u]);
      const bf16x8 dv = __builtin_bit_cast(bf16x8, pd[u]);
      const bf16x4 xt = __builtin_bit_cast(bf16x4, pxt[u]);
      const bf16x4 dt = __builtin_bit_cast(bf16x4, pdt[u]);
#pragma unroll
      for (int i = 0; i < 8; ++i) { xh[u][i] = (float)xv[i]; gd[u][i] = (float)dv[i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i) { xh[u][8 + i] = (float)xt[i]; gd[u][8 + i] = (float)dt[i]; }
    }
    if (rb + RB < rows_per_blk / 4) fetch(rb + RB);
    float s1[RB], s2[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = 0.f;
      s2[u] = 0.f;
      if (ok[u])
#pragma unroll
        for (int i = 0; i < 12; ++i) {
          if (i >= 8 && !tok) continue;
          const float dv = gd[u][i];
          const float h = (xh[u][i] - mu[u]) * rs[u];
          const float gg = dv * gm[i];
          xh[u][i] = h;
          gd[u][i] = gg;
          s1[u] += gg;
          s2[u] += gg * h;
          pg[i] += dv * h;
          pb[i] += dv;
        }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      s1[u] = wave_sum(s1[u]) / N;
      s2[u] = wave_sum(s2[u]) / N;
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      if (!ok[u]) continue;
      const int row = r0 + wave + 4 * (rb + u);
      float o[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) o[i] = rs[u] * (gd[u][i] - s1[u] - xh[u][i] * s2[u]);
      bf16x8 w;
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = (bf16)o[i];
      *reinterpret_cast<bf16x8*>(dx + (long)row * lddx + c0) = w;
      bf16x4 wt;
#pragma unroll
      for (int i = 0; i < 4; ++i) wt[i] = (bf16)o[8 + i];
      if (tok) *reinterpret_cast<bf16x4*>(dx + (long)row * lddx + ct) = wt;
      if (dxd || (Q8 && thr)) {  // (Q8 without dxd: the dropped values' e4m3 copy alone)
        float od[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) od[i] = o[i];
        const uint32_t rowkey = thr ? smer_rowkey(seed, (uint32_t)row) : 0u;
        if (thr) smer_drop8(rowkey, thr, dscale, (uint32_t)c0, od);
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = (bf16)od[i];
        if (dxd) *reinterpret_cast<bf16x8*>(dxd + (long)row * ldxd + c0) = w;
        if (tok) {
          float ot[4] = {o[8], o[9], o[10], o[11]};
          if (thr) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const uint32_t hh = smer_pair_bits(rowkey, ((uint32_t)ct >> 1) + k);
              ot[2 * k] = (hh & 0xFFFFu) >= thr ? ot[2 * k] * dscale : 0.f;
              ot[2 * k + 1] = (hh >> 16) >= thr ? ot[2 * k + 1] * dscale : 0.f;
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) wt[i] = (bf16)ot[i];
          if (dxd) *reinterpret_cast<bf16x4*>(dxd + (long)row * ldxd + ct) = wt;
        }
      }
      if constexpr (Q8) {  // e4m3 copy of the last stored (bf16) values: w / wt
        float r[8], rt[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = (float)w[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) { rt[i] = tok ? (float)wt[i] : 0.f; rt[4 + i] = 0.f; }
        *reinterpret_cast<uint2*>(q8 + (long)row * ldq + c0) = smer_q8x8(r, q8s);
        am = fmaxf(am, fmaxf(smer_absmax8(r), smer_absmax8(rt)));
        if (tok) *reinterpret_cast<uint32_t*>(q8 + (long)row * ldq + ct) = smer_q8x8(rt, q8s).x;
      }
    }
  }
  if constexpr (Q8) {  // one atomic per workgroup (per wave: 16k waves contend on one address)
    __shared__ float wam[4];
    am = wave_max(am);
    if (lane == 0) wam[wave] = am;
    __syncthreads();
    if (threadIdx.x < 64) smer_amax_commit(amax, lane < 4 ? wam[lane] : 0.f);
  }
  if (!part) return;
  // the 4 waves' column partials in fixed order: columns 0..511 in two
  // 256-column halves, then the tail
  for (int base = 0; base < N; base += 256) {
    if (base < 512) {
      if (c0 >= base && c0 < base + 256)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          red[wave][0][c0 + i - base] = pg[i];
          red[wave][1][c0 + i - base] = pb[i];
        }
    } else if (tok) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[wave][0][4 * lane + i] = pg[8 + i];
        red[wave][1][4 * lane + i] = pb[8 + i];
      }
    }
    __syncthreads();
    const int col = threadIdx.x;
    if (base + col < N) {
      const float a = (red[0][0][col] + red[1][0][col]) + (red[2][0][col] + red[3][0][col]);
      const float b = (red[0][1][col] + red[1][1][col]) + (red[2][1][col] + red[3][1][col]);
      part[(long)blockIdx.x * 2 * N + base + col] = a;
      part[(long)blockIdx.x * 2 * N + N + base + col] = b;
    }
    __syncthreads();
  }
}

// SMER_LN_BWD_T4=0 keeps 512 < N <= 768 on ln_bwd_kernel (A/B, tests)
static bool ln_bwd_t4_enabled() {
  const char* e = getenv("SMER_LN_BWD_T4");  // per call: tests flip it in-process
  return !(e && e[0] == '0');
}
static inline bool ln_bwd_t4_shape(int N) { return N > 512 && N <= 768 && N % 4 == 0; }
// rows per batch of ln_bwd_t4_kernel: 4, or 2 with the e4m3 copy (65536 x
// 768: 94.5 vs 95.7 us without it, 105.0 vs 109.7 with it, tools/ln_bench.py);
// SMER_LN_BWD_T4_RB = 2 / 4 forces it (A/B runs)
static int ln_bwd_t4_rb(bool q8) {
  const char* e = getenv("SMER_LN_BWD_T4_RB");  // per call: A/B scripts flip it in-process
  return e ? (e[0] == '2' ? 2 : 4) : (q8 ? 2 : 4);
}

// Rows per workgroup.  N > 512 at large M (C4: 65536 x 768): 64-row blocks
// made 1024 workgroups for ~768 resident slots (3 per CU at that register
// footprint), so a second, one-third-full round of workgroups ran alone
// (134.7 us, 3.0 TB/s).  There the rows are spread over exactly the resident
// slots (a multiple of 16 rows per workgroup: every wave's batches whole),
// one round.  N <= 512 keeps the measured 64 (C2: 4.8 TB/s).
static int ln_bwd_rows(int M, int N) {
  const int fixed = ln_bwd_rows_fixed(M);
  const char* e = getenv("SMER_LN_BWD_BALANCE");
  if (M <= 16384 || N <= 512 || (e && e[0] == '0')) return fixed;
  static int occ[3] = {0, 0, 0};  // NC = 2, NC = 4, t4
  const int which = ln_bwd_t4_shape(N) && ln_bwd_t4_enabled() ? 2 : N <= 1024 ? 0 : 1;
  if (!occ[which]) {
    int nb = 0;
    const void* kern = which == 2   ? (const void*)ln_bwd_t4_kernel<4>
                       : which == 0 ? (const void*)ln_bwd_kernel<bf16, false, 2, 2, true>
                                    : (const void*)ln_bwd_kernel<bf16, false, 4, 1, true>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 256, 0) != hipSuccess || nb <= 0) nb = 1;
    occ[which] = nb;
  }
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const long resident = (long)cus * occ[which];
  const long per = (M + resident - 1) / resident;
  const int rows = (int)((per + 15) / 16 * 16);
  return rows > fixed ? fixed : rows;  // never more rows (fewer blocks) than the fixed split
}

extern "C" size_t smer_layernorm_bwd_workspace(int M, int N) {
  size_t nblk = (size_t)(M + ln_bwd_rows(M, N) - 1) / ln_bwd_rows(M, N);
  return nblk * 2 * N * sizeof(float) + smer_col_reduce_scratch((int)nblk, 2 * N);
}

// reduce: 0 = write the per-block dgamma / dbeta partials only (reduced
// later by smer_layernorm_param_reduce, e.g. on another stream)
static int ln_bwd_impl(int dtype, int M, int N, const void* dy, long lddy, int dy_f32,
                       const void* x, long ldx, const float* mean, const float* rstd,
                       const float* gamma, void* dx, long lddx, void* dx_drop, long ldxd,
                       float drop_p, uint32_t seed, float* dgamma, float* dbeta, int accumulate,
                       void* workspace, size_t ws_bytes, smer_stream_t stream, bool params,
                       bool reduce, uint8_t* q8 = nullptr, long ldq = 0, const float* qs = nullptr,
                       unsigned* amax = nullptr) {
  SMER_REQUIRE(N % 8 == 0 && N <= 64 * 8 * LN_MAXC, "smer_layernorm_bwd: N % 8 == 0 and N <= 2048");
  SMER_REQUIRE(dx && dy && x && mean && rstd && gamma, "smer_layernorm_bwd: null pointer");
  SMER_REQUIRE(!params || (workspace && ws_bytes >= smer_layernorm_bwd_workspace(M, N)),
               "smer_layernorm_bwd: workspace too small");
  if (M == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  const int rpb = ln_bwd_rows(M, N);
  int nblk = (M + rpb - 1) / rpb;
  uint32_t thr = smer_drop_thr16(drop_p);
  float ds = smer_drop_scale16(thr);
  float* part = params ? (float*)workspace : nullptr;
  SMER_REQUIRE(((uintptr_t)gamma & 15) == 0, "smer_layernorm_bwd: gamma must be 16-B aligned");
#define LNB2(T, F, NC, RB, PF)                                                                 \
  hipLaunchKernelGGL((ln_bwd_kernel<T, F, NC, RB, PF>), dim3(nblk), dim3(256), 0, s, M, N, dy, \
                     lddy, (const T*)x, ldx, mean, rstd, gamma, (T*)dx, lddx, (T*)dx_drop, ldxd, \
                     thr, seed, ds, part, rpb)
  // next-batch prefetch only where a wave has more than one batch (32768
  // rows: 32.6 -> 31.2 us; single-batch 16-row blocks measured slower with it)
#define LNB1(T, F, NC, RB)                                          \
  do {                                                              \
    if (rpb / 4 > (RB)) LNB2(T, F, NC, RB, true);                   \
    else LNB2(T, F, NC, RB, false);                                 \
  } while (0)
#define LNB(T, F)                                  \
  do {                                             \
    if (N <= 512) LNB1(T, F, 1, 4);                \
    else if (N <= 1024) LNB1(T, F, 2, 2);          \
    else LNB1(T, F, 4, 1);                         \
  } while (0)
  if (q8) {
    SMER_REQUIRE(dtype == SMER_BF16 && !dy_f32 && qs && amax && ((uintptr_t)q8 & 7) == 0 && ldq % 8 == 0,
                 "smer_layernorm_bwd_fp8: bf16 dy, aligned q8, scale and amax");
    SMER_REQUIRE(((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dx & 15) == 0 &&
                     ((uintptr_t)dx_drop & 15) == 0 && lddy % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0 &&
                     ldxd % 8 == 0,
                 "smer_layernorm_bwd_fp8: 16-B aligned rows");
  }
  const bool t4 = dtype == SMER_BF16 && !dy_f32 && ln_bwd_t4_shape(N) && ln_bwd_t4_enabled() &&
                  ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dx & 15) == 0 &&
                  ((uintptr_t)dx_drop & 15) == 0 && lddy % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0 &&
                  ldxd % 8 == 0;
#define LNBT4R(R, Q)                                                                                       \
  hipLaunchKernelGGL((ln_bwd_t4_kernel<R, Q>), dim3(nblk), dim3(256), 0, s, M, N, (const bf16*)dy, lddy,    \
                     (const bf16*)x, ldx, mean, rstd, gamma, (bf16*)dx, lddx, (bf16*)dx_drop, ldxd, thr,    \
                     seed, ds, part, rpb, q8, ldq, qs, amax)
#define LNBT4(Q)                                         \
  do {                                                   \
    if (ln_bwd_t4_rb(Q) == 2) LNBT4R(2, Q);              \
    else LNBT4R(4, Q);                                   \
  } while (0)
#define LNBQ(NC, RB, PF)                                                                                   \
  hipLaunchKernelGGL((ln_bwd_kernel<bf16, false, NC, RB, PF, true>), dim3(nblk), dim3(256), 0, s, M, N,    \
                     dy, lddy, (const bf16*)x, ldx, mean, rstd, gamma, (bf16*)dx, lddx, (bf16*)dx_drop,    \
                     ldxd, thr, seed, ds, part, rpb, q8, ldq, qs, amax)
#define LNBQ1(NC, RB)                                  \
  do {                                                 \
    if (rpb / 4 > (RB)) LNBQ(NC, RB, true);            \
    else LNBQ(NC, RB, false);                          \
  } while (0)
  if (q8) {
    if (t4) LNBT4(true);
    else if (N <= 512) LNBQ1(1, 4);
    else if (N <= 1024) LNBQ1(2, 2);
    else LNBQ1(4, 1);
  } else if (t4) {
    LNBT4(false);
  } else if (dtype == SMER_BF16) { if (dy_f32) LNB(bf16, true); else LNB(bf16, false); }
  else if (dtype == SMER_F32) { LNB(float, false); }
  else return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_layernorm_bwd: dtype");
#undef LNB
#undef LNB1
#undef LNB2
#undef LNBT4
#undef LNBT4R
#undef LNBQ
#undef LNBQ1
  if (reduce) {
    if (dgamma && dbeta)  // both vectors in one reduction over the [nblk][2N] partials
      smer_col_reduce_launch(nblk, 2 * N, part, (long)2 * N, 0L, dgamma, accumulate, 1.f,
                             part + (size_t)nblk * 2 * N, s, dbeta, N);
    else if (dgamma)
      smer_col_reduce_launch(nblk, N, part, (long)2 * N, 0L, dgamma, accumulate, 1.f,
                             part + (size_t)nblk * 2 * N, s);
    else if (dbeta)
      smer_col_reduce_launch(nblk, N, part, (long)2 * N, (long)N, dbeta, accumulate, 1.f,
                             part + (size_t)nblk * 2 * N, s);
  }
  SMER_CHECK_LAUNCH("smer_layernorm_bwd");
  return SMER_OK;
}

extern "C" int smer_layernorm_bwd(int dtype, int M, int N, const void* dy, long lddy, int dy_f32,
                                  const void* x, long ldx, const float* mean, const float* rstd,
                                  const float* gamma, void* dx, long lddx, void* dx_drop,
                                  long ldxd, float drop_p, uint32_t seed, float* dgamma,
                                  float* dbeta, int accumulate, void* workspace, size_t ws_bytes,
                                  smer_stream_t stream) {
  return ln_bwd_impl(dtype, M, N, dy, lddy, dy_f32, x, ldx, mean, rstd, gamma, dx, lddx, dx_drop,
                     ldxd, drop_p, seed, dgamma, dbeta, accumulate, workspace, ws_bytes, stream,
                     dgamma || dbeta, true);
}

extern "C" int smer_layernorm_bwd_partials(int dtype, int M, int N, const void* dy, long lddy,
                                           int dy_f32, const void* x, long ldx, const float* mean,
                                           const float* rstd, const float* gamma, void* dx,
                                           long lddx, void* dx_drop, long ldxd, float drop_p,
                                           uint32_t seed, void* workspace, size_t ws_bytes,
                                           smer_stream_t stream) {
  SMER_REQUIRE(workspace, "smer_layernorm_bwd_partials: workspace required");
  return ln_bwd_impl(dtype, M, N, dy, lddy, dy_f32, x, ldx, mean, rstd, gamma, dx, lddx, dx_drop,
                     ldxd, drop_p, seed, nullptr, nullptr, 0, workspace, ws_bytes, stream, true,
                     false);
}

extern "C" int smer_layernorm_bwd_fp8(int M, int N, const void* dy, long lddy, const void* x, long ldx,
                                      const float* mean, const float* rstd, const float* gamma, void* dx,
                                      long lddx, void* dx_drop, long ldxd, float drop_p, uint32_t seed,
                                      void* q8, long ldq, const float* qs, unsigned* amax, float* dgamma,
                                      float* dbeta, int accumulate, void* workspace, size_t ws_bytes,
                                      int partials_only, smer_stream_t stream) {
  SMER_REQUIRE(q8, "smer_layernorm_bwd_fp8: q8 required");
  SMER_REQUIRE(!partials_only || workspace, "smer_layernorm_bwd_fp8: partials need a workspace");
  const bool params = partials_only || dgamma || dbeta;
  return ln_bwd_impl(SMER_BF16, M, N, dy, lddy, 0, x, ldx, mean, rstd, gamma, dx, lddx, dx_drop, ldxd,
                     drop_p, seed, dgamma, dbeta, accumulate, workspace, ws_bytes, stream, params,
                     !partials_only, (uint8_t*)q8, ldq, qs, amax);
}

extern "C" int smer_layernorm_param_reduce(int M, int N, void* workspace, size_t ws_bytes,
                                           float* dgamma, float* dbeta, int accumulate,
                                           smer_stream_t stream) {
  SMER_REQUIRE(workspace && ws_bytes >= smer_layernorm_bwd_workspace(M, N),
               "smer_layernorm_param_reduce: workspace too small");
  if (M == 0 || (!dgamma && !dbeta)) return SMER_OK;
  const int nblk = (M + ln_bwd_rows(M, N) - 1) / ln_bwd_rows(M, N);
  float* part = (float*)workspace;
  hipStream_t s = (hipStream_t)stream;
  if (dgamma && dbeta)
    smer_col_reduce_launch(nblk, 2 * N, part, (long)2 * N, 0L, dgamma, accumulate, 1.f,
                           part + (size_t)nblk * 2 * N, s, dbeta, N);
  else if (dgamma)
    smer_col_reduce_launch(nblk, N, part, (long)2 * N, 0L, dgamma, accumulate, 1.f,
                           part + (size_t)nblk * 2 * N, s);
  else
    smer_col_reduce_launch(nblk, N, part, (long)2 * N, (long)N, dbeta, accumulate, 1.f,
                           part + (size_t)nblk * 2 * N, s);
  SMER_CHECK_LAUNCH("smer_layernorm_param_reduce");
  return SMER_OK;
}

extern "C" int smer_embed_fwd(int dtype, int n_tok, int d, const int64_t* ids,
                              const int32_t* positions, int L, const float* table,
                              const float* pe, float scale, float drop_p, uint32_t seed,
                              void* out, long ldo, smer_stream_t stream) {
  SMER_REQUIRE(d % 4 == 0, "smer_embed_fwd: d % 4 == 0");
  SMER_REQUIRE(positions || L > 0, "smer_embed_fwd: L");
  if (n_tok == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  long tot = (long)n_tok * (d / 4);
  uint32_t thr = smer_drop_thr16(drop_p);
  float ds = smer_drop_scale16(thr);
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(embed_fwd_kernel<bf16>, dim3((tot + 255) / 256), dim3(256), 0, s, n_tok, d,
                       ids, positions, L, table, pe, scale, thr, seed, ds, (bf16*)out, ldo);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(embed_fwd_kernel<float>, dim3((tot + 255) / 256), dim3(256), 0, s, n_tok, d,
                       ids, positions, L, table, pe, scale, thr, seed, ds, (float*)out, ldo);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_embed_fwd: dtype");
  SMER_CHECK_LAUNCH("smer_embed_fwd");
  return SMER_OK;
}

extern "C" int smer_embed_fwd_fp8(int n_tok, int d, const int64_t* ids, const int32_t* positions, int L,
                                  const float* table, const float* pe, float scale, float drop_p,
                                  uint32_t seed, void* out, long ldo, void* q8, long ldq, const float* qs,
                                  unsigned* amax, smer_stream_t stream) {
  SMER_REQUIRE(d % 4 == 0 && ldq % 4 == 0 && ((uintptr_t)q8 & 3) == 0, "smer_embed_fwd_fp8: d, ldq % 4 == 0");
  SMER_REQUIRE(positions || L > 0, "smer_embed_fwd_fp8: L");
  SMER_REQUIRE(ids && table && pe && out && q8 && qs && amax, "smer_embed_fwd_fp8: null pointer");
  if (n_tok == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  long tot = (long)n_tok * (d / 4);
  uint32_t thr = smer_drop_thr16(drop_p);
  float ds = smer_drop_scale16(thr);
  hipLaunchKernelGGL((embed_fwd_kernel<bf16, true>), dim3((tot + 255) / 256), dim3(256), 0, s, n_tok, d, ids,
                     positions, L, table, pe, scale, thr, seed, ds, (bf16*)out, ldo, (uint8_t*)q8, ldq, qs, amax);
  SMER_CHECK_LAUNCH("smer_embed_fwd_fp8");
  return SMER_OK;
}

extern "C" size_t smer_embed_bwd_workspace(int V, int d, int n_tok_total) {
  size_t nchunk = (size_t)(n_tok_total + EMB_CHUNK - 1) / EMB_CHUNK;
  if (nchunk == 0) nchunk = 1;
  return nchunk * V * d * sizeof(float);
}

extern "C" int smer_embed_bwd(int dtype, int V, int d, float scale, const int64_t* ids0,
                              const void* dx0, long ld0, int n0, float p0, uint32_t seed0,
                              const int64_t* ids1, const void* dx1, long ld1, int n1, float p1,
                              uint32_t seed1, float* dtable, void* workspace, size_t ws_bytes,
                              smer_stream_t stream) {
  SMER_REQUIRE(d % 64 == 0 && d <= 1024, "smer_embed_bwd: d % 64 == 0 and d <= 1024");
  SMER_REQUIRE((!dx0 || (ld0 % 8 == 0 && ((uintptr_t)dx0 & 15) == 0)) &&
                   (!dx1 || (ld1 % 8 == 0 && ((uintptr_t)dx1 & 15) == 0)),
               "smer_embed_bwd: dx rows must be 16-B aligned (ld % 8 == 0)");
  SMER_REQUIRE(workspace && ws_bytes >= smer_embed_bwd_workspace(V, d, n0 + n1),
               "smer_embed_bwd: workspace too small");
  int n = n0 + n1;
  if (n == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  int nchunk = (n + EMB_CHUNK - 1) / EMB_CHUNK;
  uint32_t t0 = smer_drop_thr16(p0), t1 = smer_drop_thr16(p1);
  float ds0 = smer_drop_scale16(t0), ds1 = smer_drop_scale16(t1);
  dim3 grid(V, nchunk);
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(embed_bwd_gather<bf16>, grid, dim3(256), 0, s, V, d, ids0, (const bf16*)dx0,
                       ld0, n0, t0, seed0, ds0, ids1, (const bf16*)dx1, ld1, n1, t1, seed1, ds1,
                       (float*)workspace);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(embed_bwd_gather<float>, grid, dim3(256), 0, s, V, d, ids0,
                       (const float*)dx0, ld0, n0, t0, seed0, ds0, ids1, (const float*)dx1, ld1,
                       n1, t1, seed1, ds1, (float*)workspace);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_embed_bwd: dtype");
  long tot = (long)V * d;
  hipLaunchKernelGGL(embed_bwd_reduce, dim3((tot + 255) / 256), dim3(256), 0, s, V, d, nchunk,
                     (const float*)workspace, scale, dtable);
  SMER_CHECK_LAUNCH("smer_embed_bwd");
  return SMER_OK;
}
