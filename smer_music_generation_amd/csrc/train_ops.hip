// Training-step tail: the fused multi-criterion weighted cross entropy
// (train.py:555-642, 726-780), torch.optim.Adam (train.py:264, 786), bias
// gradient column sums and dtype casts.  All HBM-bound elementwise / row
// kernels; reductions are fixed-order (bitwise reproducible).
#include "common.h"

// denom = sum_i ce_all[y_i]   (single workgroup, fixed order)
__global__ __launch_bounds__(256) void wce_denom_kernel(int n, const int64_t* __restrict__ y,
                                                        const float* __restrict__ ce_all,
                                                        float* __restrict__ denom) {
  __shared__ float red[256];
  float a = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) a += ce_all[y[i]];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *denom = red[0];
}

template <typename T>
__global__ __launch_bounds__(256) void wce_kernel(int R, int V, const float* __restrict__ logits,
                                                  long ldl, const int64_t* __restrict__ y,
                                                  const float* __restrict__ w,
                                                  const float* __restrict__ denom,
                                                  float* __restrict__ row_loss,
                                                  T* __restrict__ dlog, long ldd,
                                                  float grad_scale) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* x = logits + (long)r * ldl;
  const long yt = y[r];
  float mx = -INFINITY;
  for (int v = lane; v < V; v += 64) mx = fmaxf(mx, x[v]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int v = lane; v < V; v += 64) se += expf(x[v] - mx);
  se = wave_sum(se);
  const float lse = mx + logf(se);
  const float wy = yt == 0 ? 0.f : w[yt];
  if (lane == 0) row_loss[r] = wy * (lse - x[yt]);
  if (dlog) {
    const float coef = grad_scale * wy / *denom;
    const float inv = 1.f / se;
    for (int v = lane; v < V; v += 64) {
      float g = coef * (expf(x[v] - mx) * inv - (v == yt ? 1.f : 0.f));
      dlog[(long)r * ldd + v] = from_f32<T>(g);
    }
  }
}

__global__ __launch_bounds__(256) void sum_div_kernel(int n, const float* __restrict__ x,
                                                      const float* __restrict__ denom,
                                                      float* __restrict__ out) {
  __shared__ float red[256];
  float a = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) a += x[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = denom ? red[0] / *denom : red[0];
}

// torch.optim.Adam (_single_tensor_adam): m.lerp_(g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adam_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                            float* __restrict__ m, float* __restrict__ v, bf16* __restrict__ pb,
                            float lr, float b1, float b2, float eps, float bc1, float bc2s) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const float step = lr / bc1;
  for (; i < n; i += stride) {
    float gi = g[i];
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    float den = sqrtf(vi) / bc2s + eps;
    float pi = p[i] - step * (mi / den);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (pb) pb[i] = (bf16)pi;
  }
}

template <typename S, typename D>
__global__ void cast_kernel(long n, const S* __restrict__ s, D* __restrict__ d) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n; i += stride) d[i] = from_f32<D>(to_f32(s[i]));
}

// Stage 1: workgroup = 512 columns (64 lanes x 8 via 16-B loads) x CS_ROWS
// rows (4 row groups, 4 independent loads in flight each); fixed-order
// combine of the 4 groups -> part[rowblock][N].
constexpr int CS_ROWS = 64;
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void colsum_part_kernel(int M, int N, const T* __restrict__ x,
                                                          long ldx, float* __restrict__ part) {
  __shared__ float red[4][512];
  const int cg = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + cg * 8;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(M, r0 + CS_ROWS);
  const int valid = min(8, N - c0);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (valid > 0) {
    int r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
      float v0[8], v1[8], v2[8], v3[8];
      load8<T, VEC>(x + (long)r * ldx + c0, valid, v0);
      load8<T, VEC>(x + (long)(r + 4) * ldx + c0, valid, v1);
      load8<T, VEC>(x + (long)(r + 8) * ldx + c0, valid, v2);
      load8<T, VEC>(x + (long)(r + 12) * ldx + c0, valid, v3);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += (v0[i] + v1[i]) + (v2[i] + v3[i]);
    }
    for (; r < r1; r += 4) {
      float v0[8];
      load8<T, VEC>(x + (long)r * ldx + c0, valid, v0);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v0[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[rg][cg * 8 + i] = acc[i];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    int col = blockIdx.x * 512 + c;
    if (col < N) part[(long)blockIdx.y * N + col] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
  }
}

// Workgroup (x = 64-column tile, y = chunk of `chunk` partial rows) writes
// out[y * ostride + col] (columns >= nsplit go to out2[col - nsplit]); rows
// summed in a fixed order (deterministic).
__global__ void __launch_bounds__(256) smer_col_reduce(int nblk, int N, const float* __restrict__ part,
                                                       long stride, long off, float* __restrict__ out,
                                                       long ostride, int chunk, int accumulate,
                                                       float scale, float* __restrict__ out2,
                                                       int nsplit) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  const int b0 = blockIdx.y * chunk, b1 = min(nblk, b0 + chunk);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (col < N) {
    const float* p = part + off + col;
    int b = b0 + g;
    for (; b + 12 < b1; b += 16) {
      a0 += p[(long)b * stride];
      a1 += p[(long)(b + 4) * stride];
      a2 += p[(long)(b + 8) * stride];
      a3 += p[(long)(b + 12) * stride];
    }
    for (; b < b1; b += 4) a0 += p[(long)b * stride];
  }
  red[g][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (g == 0 && col < N) {
    float a = ((red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl])) * scale;
    float* o = col < nsplit ? out + (long)blockIdx.y * ostride + col
                            : out2 + (long)blockIdx.y * ostride + (col - nsplit);
    *o = accumulate ? *o + a : a;
  }
}

size_t smer_col_reduce_scratch(int nblk, int N) {
  return nblk > 64 ? (size_t)((nblk + 63) / 64) * N * sizeof(float) : 0;
}

void smer_col_reduce_launch(int nblk, int N, const float* part, long stride, long off, float* out,
                            int accumulate, float scale, float* scratch, hipStream_t s,
                            float* out2, int nsplit) {
  dim3 gx((N + 63) / 64);
  if (!out2) nsplit = N;
  if (nblk > 64) {
    int g = (nblk + 63) / 64;
    hipLaunchKernelGGL(smer_col_reduce, dim3(gx.x, g), dim3(256), 0, s, nblk, N, part, stride,
                       off, scratch, (long)N, 64, 0, 1.f, (float*)nullptr, N);
    hipLaunchKernelGGL(smer_col_reduce, dim3(gx.x, 1), dim3(256), 0, s, g, N,
                       (const float*)scratch, (long)N, 0L, out, 0L, g, accumulate, scale, out2,
                       nsplit);
  } else {
    hipLaunchKernelGGL(smer_col_reduce, dim3(gx.x, 1), dim3(256), 0, s, nblk, N, part, stride,
                       off, out, 0L, nblk, accumulate, scale, out2, nsplit);
  }
}

// ---------------------------------------------------------------------------
extern "C" int smer_wce_denom(int n, const int64_t* y, const float* ce_all, float* denom,
                              smer_stream_t stream) {
  SMER_REQUIRE(y && ce_all && denom, "smer_wce_denom: null pointer");
  hipLaunchKernelGGL(wce_denom_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, n, y, ce_all,
                     denom);
  SMER_CHECK_LAUNCH("smer_wce_denom");
  return SMER_OK;
}

extern "C" int smer_wce_fwd_bwd(int dtype, int R, int V, const float* logits, long ldl,
                                const int64_t* y, const float* w, const float* denom,
                                float* row_loss, float* loss_out, void* dlogits, long ldd,
                                float grad_scale, smer_stream_t stream) {
  SMER_REQUIRE(logits && y && w && denom && row_loss, "smer_wce_fwd_bwd: null pointer");
  if (R == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((R + 3) / 4);
  if (dtype == SMER_BF16)
    hipLaunchKernelGGL(wce_kernel<bf16>, grid, dim3(256), 0, s, R, V, logits, ldl, y, w, denom,
                       row_loss, (bf16*)dlogits, ldd, grad_scale);
  else if (dtype == SMER_F32)
    hipLaunchKernelGGL(wce_kernel<float>, grid, dim3(256), 0, s, R, V, logits, ldl, y, w, denom,
                       row_loss, (float*)dlogits, ldd, grad_scale);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_wce_fwd_bwd: dtype");
  if (loss_out)
    hipLaunchKernelGGL(sum_div_kernel, dim3(1), dim3(256), 0, s, R, row_loss, denom, loss_out);
  SMER_CHECK_LAUNCH("smer_wce_fwd_bwd");
  return SMER_OK;
}

extern "C" int smer_adam(long n, float* p, const float* g, float* m, float* v, void* p_bf16,
                         float lr, float b1, float b2, float eps, float bc1, float bc2_sqrt,
                         smer_stream_t stream) {
  SMER_REQUIRE(p && g && m && v, "smer_adam: null pointer");
  if (n == 0) return SMER_OK;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, p, g, m, v,
                     (bf16*)p_bf16, lr, b1, b2, eps, bc1, bc2_sqrt);
  SMER_CHECK_LAUNCH("smer_adam");
  return SMER_OK;
}

extern "C" int smer_cast(int src_dtype, int dst_dtype, long n, const void* src, void* dst,
                         smer_stream_t stream) {
  if (n == 0) return SMER_OK;
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipStream_t s = (hipStream_t)stream;
  if (src_dtype == SMER_F32 && dst_dtype == SMER_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(blocks), dim3(256), 0, s, n,
                       (const float*)src, (bf16*)dst);
  else if (src_dtype == SMER_BF16 && dst_dtype == SMER_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(blocks), dim3(256), 0, s, n,
                       (const bf16*)src, (float*)dst);
  else if (src_dtype == SMER_F32 && dst_dtype == SMER_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(blocks), dim3(256), 0, s, n,
                       (const float*)src, (float*)dst);
  else if (src_dtype == SMER_BF16 && dst_dtype == SMER_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(blocks), dim3(256), 0, s, n,
                       (const bf16*)src, (bf16*)dst);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_cast: dtype");
  SMER_CHECK_LAUNCH("smer_cast");
  return SMER_OK;
}

template <typename S, typename D>
__global__ void cast2d_kernel(int rows, int cols, const S* __restrict__ s, long lds,
                              D* __restrict__ d, long ldd) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)rows * cols) return;
  int r = idx / cols, c = idx % cols;
  d[(long)r * ldd + c] = from_f32<D>(to_f32(s[(long)r * lds + c]));
}

extern "C" int smer_cast2d(int src_dtype, int dst_dtype, int rows, int cols, const void* src,
                           long lds, void* dst, long ldd, smer_stream_t stream) {
  long n = (long)rows * cols;
  if (n == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  dim3 g((n + 255) / 256);
  if (src_dtype == SMER_F32 && dst_dtype == SMER_BF16)
    hipLaunchKernelGGL((cast2d_kernel<float, bf16>), g, dim3(256), 0, s, rows, cols, (const float*)src, lds, (bf16*)dst, ldd);
  else if (src_dtype == SMER_F32 && dst_dtype == SMER_F32)
    hipLaunchKernelGGL((cast2d_kernel<float, float>), g, dim3(256), 0, s, rows, cols, (const float*)src, lds, (float*)dst, ldd);
  else if (src_dtype == SMER_BF16 && dst_dtype == SMER_F32)
    hipLaunchKernelGGL((cast2d_kernel<bf16, float>), g, dim3(256), 0, s, rows, cols, (const bf16*)src, lds, (float*)dst, ldd);
  else if (src_dtype == SMER_BF16 && dst_dtype == SMER_BF16)
    hipLaunchKernelGGL((cast2d_kernel<bf16, bf16>), g, dim3(256), 0, s, rows, cols, (const bf16*)src, lds, (bf16*)dst, ldd);
  else
    return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_cast2d: dtype");
  SMER_CHECK_LAUNCH("smer_cast2d");
  return SMER_OK;
}

extern "C" size_t smer_colsum_workspace(int M, int N) {
  size_t nblk = (size_t)(M + CS_ROWS - 1) / CS_ROWS;
  return nblk * N * sizeof(float) + smer_col_reduce_scratch((int)nblk, N);
}

extern "C" int smer_colsum(int dtype, int M, int N, const void* x, long ldx, float* out,
                           int accumulate, void* workspace, size_t ws_bytes,
                           smer_stream_t stream) {
  SMER_REQUIRE(x && out, "smer_colsum: null pointer");
  SMER_REQUIRE(workspace && ws_bytes >= smer_colsum_workspace(M, N), "smer_colsum: workspace");
  if (N == 0) return SMER_OK;
  hipStream_t s = (hipStream_t)stream;
  int nblk = (M + CS_ROWS - 1) / CS_ROWS;
  dim3 grid((N + 511) / 512, nblk > 0 ? nblk : 1);
  bool vec = ((uintptr_t)x & 15) == 0 && ldx % 8 == 0;
  if (M > 0) {
    if (dtype == SMER_BF16) {
      if (vec) hipLaunchKernelGGL((colsum_part_kernel<bf16, true>), grid, dim3(256), 0, s, M, N, (const bf16*)x, ldx, (float*)workspace);
      else hipLaunchKernelGGL((colsum_part_kernel<bf16, false>), grid, dim3(256), 0, s, M, N, (const bf16*)x, ldx, (float*)workspace);
    } else if (dtype == SMER_F32) {
      if (vec) hipLaunchKernelGGL((colsum_part_kernel<float, true>), grid, dim3(256), 0, s, M, N, (const float*)x, ldx, (float*)workspace);
      else hipLaunchKernelGGL((colsum_part_kernel<float, false>), grid, dim3(256), 0, s, M, N, (const float*)x, ldx, (float*)workspace);
    } else {
      return smer_set_error(SMER_ERR_UNSUPPORTED, "smer_colsum: dtype");
    }
  }
  smer_col_reduce_launch(nblk, N, (const float*)workspace, (long)N, 0L, out, accumulate, 1.f,
                         (float*)workspace + (size_t)nblk * N, s);
  SMER_CHECK_LAUNCH("smer_colsum");
  return SMER_OK;
}

// ---------------------------------------------------------------------------
// Debug checksum (repeatability probes, tools/ck_log.py): partial[b] =
// sum over the 4-byte words w_i of a strided 2-D region of w_i * (2 i + 1)
// (mod 2^64), word i = r * (row_bytes / 4) + c, block b taking every
// nparts-th row.  The host adds the partials; the sum is order-independent,
// so two runs over the same bits give the same value.  One launch on the
// caller's stream, no allocation, no sync.
__global__ __launch_bounds__(256) void checksum_kernel(const uint32_t* __restrict__ p, long rows,
                                                       long row_words, long ld_words,
                                                       unsigned long long* __restrict__ out) {
  __shared__ unsigned long long red[256];
  unsigned long long a = 0;
  for (long r = blockIdx.x; r < rows; r += gridDim.x) {
    const uint32_t* row = p + r * ld_words;
    const unsigned long long base = (unsigned long long)r * (unsigned long long)row_words;
    for (long c = threadIdx.x; c < row_words; c += 256)
      a += (unsigned long long)row[c] * (2ull * (base + (unsigned long long)c) + 1ull);
  }
  red[threadIdx.x] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

extern "C" int smer_debug_checksum(const void* p, long rows, long row_bytes, long ld_bytes,
                                   unsigned long long* out, int nparts, smer_stream_t stream) {
  SMER_REQUIRE(p && out, "smer_debug_checksum: null pointer");
  SMER_REQUIRE(row_bytes % 4 == 0 && ld_bytes % 4 == 0 && ((uintptr_t)p & 3) == 0 && nparts > 0,
               "smer_debug_checksum: 4-byte words only");
  hipLaunchKernelGGL(checksum_kernel, dim3(nparts), dim3(256), 0, (hipStream_t)stream,
                     (const uint32_t*)p, rows, row_bytes / 4, ld_bytes / 4, out);
  SMER_CHECK_LAUNCH("smer_debug_checksum");
  return SMER_OK;
}

// ---------------------------------------------------------------------------
// Validation accuracy (train.py:988-1034 `accuracy`, as validate() calls it):
// one wave per row; pred = the first index of the row's max logit
// (torch.argmax), target y; rows whose target is the pad index are skipped;
// counts[2 c] += 1 and counts[2 c + 1] += (pred == y) for the target's token
// class c = cls[y], and the same for the total in the last pair (c = ncls).
// Integer atomics: the counts are exact and order-independent.
__global__ __launch_bounds__(256) void argmax_acc_kernel(int R, int V, const float* __restrict__ logits,
                                                         long ldl, const int64_t* __restrict__ y,
                                                         const int32_t* __restrict__ cls, int ncls,
                                                         int pad, unsigned* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const long yt = y[r];
  if (yt == pad) return;
  const float* x = logits + (long)r * ldl;
  float best = -INFINITY;
  int bi = V;  // V: no finite value seen yet (all -inf: index 0, as torch)
  for (int v = lane; v < V; v += 64) {
    const float xv = x[v];
    if (xv > best || bi == V) { best = xv; bi = v; }  // per lane: ascending v, first max kept
  }
#pragma unroll
  for (int w = 1; w < 64; w <<= 1) {
    const float ob = __shfl_xor(best, w, 64);
    const int oi = __shfl_xor(bi, w, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) {
    const int c = (yt >= 0 && yt < V) ? cls[yt] : ncls;
    const unsigned hit = (long)bi == yt ? 1u : 0u;
    if (c >= 0 && c < ncls) {
      atomicAdd(counts + 2 * c, 1u);
      atomicAdd(counts + 2 * c + 1, hit);
    }
    atomicAdd(counts + 2 * ncls, 1u);
    atomicAdd(counts + 2 * ncls + 1, hit);
  }
}

extern "C" int smer_argmax_accuracy(int R, int V, const float* logits, long ldl, const int64_t* y,
                                    const int32_t* cls, int ncls, int pad, unsigned* counts,
                                    smer_stream_t stream) {
  SMER_REQUIRE(R >= 0 && V > 0 && ncls >= 0, "smer_argmax_accuracy: bad sizes");
  SMER_REQUIRE(logits && y && cls && counts, "smer_argmax_accuracy: null pointer");
  if (R == 0) return SMER_OK;
  hipLaunchKernelGGL(argmax_acc_kernel, dim3((R + 3) / 4), dim3(256), 0, (hipStream_t)stream, R, V, logits,
                     ldl, y, cls, ncls, pad, counts);
  SMER_CHECK_LAUNCH("smer_argmax_accuracy");
  return SMER_OK;
}
