/*
 * smer_hip.h — C-ABI of the MI355X (gfx950) SMER engine, libsmer_hip.so.
 *
 * Plain pointers (device memory owned by the caller), explicit sizes and row
 * strides (in ELEMENTS), a dtype code, and a hipStream_t.  Every entry
 * returns 0 on success or a negative status; smer_last_error() holds the
 * message.  No entry allocates device memory or synchronises the stream, so
 * every call can be captured into a hipGraph.
 *
 * Each entry names the reference operation it replaces (the reference is
 * pure Python on PyTorch ATen; file:line of the call site):
 *
 *   smer_gemm            nn.Linear / MHA in- and out-projections, FFN, head
 *                        (transformer.py:389,393,459,463,467; model.py:106;
 *                        torch/nn/functional.py:6435) and their autograd
 *                        dgrad / wgrad (train.py:783)
 *   smer_attn_fwd/bwd    MHA scaled-dot-product path with key-padding and
 *                        causal masks (functional.py:6578-6600 via
 *                        transformer.py:389,459,463) and its backward
 *   smer_attn_weights    head-averaged cross-attention weights
 *                        (functional.py:6606, transformer.py:332, model.py:101)
 *   smer_attn_decode     KV-cached single-step attention for the infill loop
 *                        (replaces the full recompute of generation.py:217)
 *   smer_kv_scatter      append new K/V rows to a per-request cache
 *   smer_kv_scatter_heads  the cross-attention memory K/V (transformer.py:463)
 *                        into a head-major per-request cache at prefill
 *   smer_linear_decode_ln  the same with the LayerNorm of its input fused in
 *   smer_attn_decode_qln  decode cross attention with LN + query projection fused in
 *   smer_linear_decode   decode-step Linear (M <= 256 rows) whose epilogue
 *                        also appends the new K/V columns to the cache
 *                        (transformer.py:459 per generated token)
 *   smer_grammar_greedy_step  the greedy infill grammar loop on device:
 *                        state -> mask -> argmax -> commit -> next feed
 *                        (generation.py:528-687 with weighted_sampling as
 *                        argmax; replaces the per-token host round trip)
 *   smer_grammar_sample_step  the sampled (default, weighted_sampling)
 *                        grammar loop on device: float64 softmax, sort, cdf
 *                        search and redraws on the numpy MT19937 stream
 *                        (generation.py:33-95, 528-687)
 *   smer_layernorm_*     residual LayerNorm, eps 1e-5 (transformer.py:392,395,
 *                        462,466,469; final norms 274-275, 329-330)
 *   smer_embed_*         embedding gather x sqrt(d) + sinusoidal PE + dropout
 *                        (model.py:91-92,124-125) and its scatter backward
 *   smer_wce_*           the 7-12 weighted cross-entropy criteria fused into
 *                        one pass (train.py:555-642,726-780)
 *   smer_adam            torch.optim.Adam step (train.py:264,786)
 *   smer_gemm_wgrad_bias nn.Linear weight AND bias gradients in one pass
 *                        (autograd of transformer.py:389-469 / model.py:106
 *                        linears, train.py:783)
 *   smer_colsum          bias gradients (autograd of nn.Linear bias)
 *   smer_cast            fp32 master -> bf16 working copies
 *   smer_fp8_quantize    per-tensor e4m3 quantisation (amax + scaled cast) of
 *                        a bf16 activation / weight for the fp8 GEMM
 *   smer_gemm_fp8(_q), smer_layernorm_fwd_fp8, smer_fp8_scales: the fp8
 *                        training forward (delayed per-tensor scaling)
 *   smer_gemm_fp8        fp8 (e4m3 x e4m3, fp32 accumulate) forward Linear of
 *                        the QKV / FFN contractions (BASELINE C4)
 */
#ifndef SMER_HIP_H
#define SMER_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* smer_stream_t; /* == hipStream_t */

#define SMER_OK 0
#define SMER_ERR_INVALID (-1)
#define SMER_ERR_HIP (-2)
#define SMER_ERR_UNSUPPORTED (-3)

#define SMER_F32 0
#define SMER_BF16 1

int smer_abi_version(void);
const char* smer_last_error(void);

/* C = epilogue(alpha * op(A) op(B)^T).
 *   a_kcontig=1: A is [M,K] row-major (lda >= K); 0: A is [K,M] (lda >= M).
 *   b_kcontig=1: B is [N,K] row-major (ldb >= K); 0: B is [K,N] (ldb >= N).
 * epilogue(v) = residual + dropout(relu?(v + bias))  then  *gate-mask,
 *   gate (nullable, [M,N] ld ldg): v *= (gate > 0 ? gate_scale : 0)
 * outputs: C (activation dtype, nullable) and/or Cf (fp32, nullable;
 *   accumulate=1 adds into Cf).  bf16 path: MFMA 16x16x32; f32 path: VALU.
 * workspace (nullable, 16-B aligned): lets a Cf-only GEMM with few output
 *   tiles and a long K (weight gradients) split K into deterministic fp32
 *   slabs of M*N floats each, summed in fixed slice order by the tile's
 *   last-arriving slice (or a second kernel).  Its last 64 KiB hold per-tile
 *   tickets: they must be ZERO when the workspace is first used (allocate
 *   it zeroed); every call leaves them zero.  One workspace per stream. */
int smer_gemm(int dtype, int a_kcontig, int b_kcontig, int M, int N, int K,
              const void* A, long lda, const void* B, long ldb,
              const float* bias, float alpha, int relu,
              const void* residual, long ldr,
              const void* gate, long ldg, float gate_scale,
              float drop_p, uint32_t drop_seed,
              void* C, long ldc, float* Cf, long ldcf, int accumulate,
              void* workspace, size_t ws_bytes, smer_stream_t stream);

/* Weight + bias gradient of y = x W^T + b (bf16):
 *   dW[M,N] (+)= dy^T x,  db[M] (+)= sum_k dy[k, :]
 * dy: [K, M] row-major (K = tokens, ld lddy), x: [K, N] (ld ldx); dW fp32.
 * The bias sum rides the GEMM as one extra MFMA against a ones fragment in
 * the first column-tile's workgroups; with split-K both are reduced by the
 * same deterministic pass.  workspace as smer_gemm (slabs + M floats per
 * K slice).  fp32 returns SMER_ERR_UNSUPPORTED (use smer_gemm + smer_colsum). */
int smer_gemm_wgrad_bias(int dtype, int M, int N, int K, const void* dy, long lddy,
                         const void* x, long ldx, float* dW, long lddw, int accumulate,
                         float* db, int db_accumulate, void* workspace, size_t ws_bytes,
                         smer_stream_t stream);
/* The same with max_workgroups > 0 capping the persistent weight-gradient
 * grid (0: the whole chip): a weight gradient issued on a second stream
 * beside the dgrad chain (the overlapped train step) leaves the remaining
 * CUs to that chain.  The split-K slice count follows the grid, so results
 * are deterministic for a given cap (not bitwise equal across caps). */
int smer_gemm_wgrad_bias_ex(int dtype, int M, int N, int K, const void* dy, long lddy,
                            const void* x, long ldx, float* dW, long lddw, int accumulate,
                            float* db, int db_accumulate, void* workspace, size_t ws_bytes,
                            int max_workgroups, smer_stream_t stream);
/* fp8 weight gradient of y = x W^T (transformer.py:389,393,459,463,467 under
 * train.py:783, precision "fp8"): dW[M,N] (+)= dy_inv * x_inv * dy8^T x8 from
 * the e4m3 copies dy8 [K, M] (ld lddy bytes) and x8 [K, N] (ld ldx bytes),
 * K = tokens, with *dy_inv / *x_inv (device) their dequantisation scales.
 * With db non-NULL also db[M] (+)= dy_inv * sum_t dy8[t, :] (the bias
 * gradient from the same e4m3 dy).  M, N % 256 == 0, K % 64 == 0 (else
 * SMER_ERR_UNSUPPORTED, nothing launched); 16-B aligned operands, strides
 * % 16.  workspace, max_workgroups: as smer_gemm_wgrad_bias_ex (split-K
 * slabs + M floats per slice, deterministic fixed-order reduce). */
int smer_gemm_wgrad_fp8(int M, int N, int K, const void* dy8, long lddy, const void* x8, long ldx,
                        const float* dy_inv, const float* x_inv, float* dW, long lddw, int accumulate,
                        float* db, int db_accumulate, void* workspace, size_t ws_bytes,
                        int max_workgroups, smer_stream_t stream);

/* Diagnostics: when buf (device, bytes >= 64 * num_CUs uint64) is non-NULL, the
 * staggered 256x256 GEMM (the forward / dgrad shapes of transformer.py:389-395,
 * 459-469) writes per wave s_memtime stamps of its first two tiles (tile
 * start, k-loop start, k-loop end, epilogue end) at buf[(block * 8 + wave) * 8
 * + k].  NULL (the default) turns them off; launches on a capturing stream
 * never stamp.  Used by tools/gemm256s_phases.py. */
int smer_gemm_debug_stamps(void* buf, size_t bytes);

/* Flash attention over [B*L, *] token-row layouts (row = b*L + i), head h
 * at column h*D.  kpm: uint8 [B, Lk] (1 = padded key) or NULL.  causal:
 * key j visible to query i iff j <= i.  lse: fp32 [B, H, Lq] (natural log).
 * Attention-probability dropout with (drop_p, seed). */
/* Attention-dropout keep bits of a [B*H, Lq, Lk] score matrix (layout: see
 * smer_attn_drop_mask_bytes), the same keep decisions the forward hashes in
 * its loop when it gets no mask buffer; smer_attn_fwd(..., drop_mask,
 * drop_mask_in = 1) reads them (the forward is VALU-bound), and so does
 * smer_attn_bwd. */
int smer_attn_drop_mask_gen(int B, int H, int Lq, int Lk, float drop_p, uint32_t seed, void* mask,
                            smer_stream_t stream);
int smer_attn_fwd(int dtype, int B, int H, int Lq, int Lk, int D,
                  const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                  void* o, long ldo, float* lse, const uint8_t* kpm, int causal, float scale,
                  float drop_p, uint32_t seed, void* drop_mask, int drop_mask_in,
                  smer_stream_t stream);
/* drop_mask (nullable, 16-B aligned, smer_attn_drop_mask_bytes bytes: one
 * u32 per (b*H+h, 32-query block, 64-key tile, lane), 1 bit per (query,
 * key)): with drop_p > 0 and drop_mask_in = 0 the bf16 forward first fills
 * it (smer_attn_drop_mask_gen on the same stream), then reads it, and so does
 * smer_attn_bwd given the same buffer; NULL: the forward and the backward
 * hash the keep bits in their loops.  The mask is the same either way. */
size_t smer_attn_drop_mask_bytes(int B, int H, int Lq, int Lk);
size_t smer_attn_bwd_workspace(int dtype, int B, int H, int Lq, int Lk);
int smer_attn_bwd(int dtype, int B, int H, int Lq, int Lk, int D,
                  const void* q, long ldq, const void* k, long ldk, const void* v, long ldv,
                  const void* o, long ldo, const void* dout, long lddo, const float* lse,
                  const uint8_t* kpm, int causal, float scale, float drop_p, uint32_t seed,
                  void* dq, long lddq, void* dk, long lddk, void* dv, long lddv,
                  void* workspace, size_t ws_bytes, const void* drop_mask,
                  smer_stream_t stream);
/* smer_attn_bwd (bf16) that also writes e4m3 copies e4m3(g * qs[0]) of dQ
 * (dq8, nullable) and of dK / dV (dk8 and dv8 together, nullable) beside the
 * bf16 gradients, folding max|g| into *amax (float bits, atomicMax): the fp8
 * input of the QKV / cross-Q dgrads in the C4 fp8 step (transformer.py:389,
 * 459 differentiated by train.py:783).  Copies 4-B aligned, strides % 4.
 * A gradient with a copy may be null itself (dk with dv): the copy alone. */
int smer_attn_bwd_fp8(int B, int H, int Lq, int Lk, int D, const void* q, long ldq,
                      const void* k, long ldk, const void* v, long ldv, const void* o, long ldo,
                      const void* dout, long lddo, const float* lse, const uint8_t* kpm,
                      int causal, float scale, float drop_p, uint32_t seed, void* dq, long lddq,
                      void* dk, long lddk, void* dv, long lddv, void* workspace, size_t ws_bytes,
                      const void* drop_mask, void* dq8, long lddq8, void* dk8, long lddk8,
                      void* dv8, long lddv8, const float* qs, unsigned* amax, smer_stream_t stream);
/* smer_attn_fwd (bf16) that also writes the output's e4m3 copy
 * e4m3(o * qs[0]) (4-B aligned, ldo8 % 4 == 0), max|o| folded into *amax:
 * the fp8 input of the attention out-projection in the C4 fp8 forward
 * (transformer.py:389 -> 390/463 -> 464 out_proj).  Head dim 64, drop_mask_in 0. */
int smer_attn_fwd_fp8(int B, int H, int Lq, int Lk, int D, const void* q, long ldq, const void* k,
                      long ldk, const void* v, long ldv, void* o, long ldo, float* lse,
                      const uint8_t* kpm, int causal, float scale, float drop_p, uint32_t seed,
                      void* drop_mask, int drop_mask_in, void* o8, long ldo8, const float* qs,
                      unsigned* amax, smer_stream_t stream);
/* out fp32 [B, Lq, Lk] = mean over heads of the attention probabilities. */
int smer_attn_weights(int dtype, int B, int H, int Lq, int Lk, int D,
                      const void* q, long ldq, const void* k, long ldk, const float* lse,
                      const uint8_t* kpm, int causal, float scale, float* out,
                      smer_stream_t stream);
/* Decode attention: row r (query q[r], head h at column h*D) attends keys
 * 0..row_nkeys[r]-1 of request row_req[r] in caches laid out
 * cache[req * req_stride + h * head_stride + j * row_stride + d]
 * (head_stride <= 0 means D: heads side by side within a key row). */
int smer_attn_decode(int dtype, int n_rows, int H, int D, const void* q, long ldq,
                     const void* kcache, const void* vcache, long row_stride, long req_stride,
                     long head_stride, const int32_t* row_req, const int32_t* row_nkeys,
                     void* o, long ldo, float scale, smer_stream_t stream);
/* Head-major K/V fill: row m of src = [K heads | V heads] (2*H*D columns);
 * (kv, h, dd) -> cache[row_req[m]*req_stride + kv*kv_stride + h*head_stride
 * + row_pos[m]*D + dd] (the decode cross-attention memory, written once per
 * request at prefill). */
int smer_kv_scatter_heads(int dtype, int n_rows, int H, int D, const void* src, long lds,
                          void* cache, long req_stride, long kv_stride, long head_stride,
                          const int32_t* row_req, const int32_t* row_pos, smer_stream_t stream);
int smer_kv_scatter(int dtype, int n_rows, int width, const void* src, long lds,
                    void* cache, long row_stride, long req_stride,
                    const int32_t* row_req, const int32_t* row_pos, smer_stream_t stream);
/* Decode Linear (M <= 256 rows, bf16): C[M,N] (or fp32 Cf) = A W^T + bias
 * (+ReLU) (+residual); kv (optional): output columns >= kv_col0 are also
 * written to kv[kv_req[m]*kv_req_stride + kv_pos[m]*kv_row_stride + col -
 * kv_col0] (the new token's self-attention K/V appended to the cache). */
int smer_linear_decode(int M, int N, int K, const void* A, long lda, const void* W, long ldw,
                       const float* bias, int relu, const void* residual, long ldr, void* C,
                       long ldc, float* Cf, long ldcf, void* kv, long kv_row_stride,
                       long kv_req_stride, const int32_t* kv_req, const int32_t* kv_pos,
                       int kv_col0, smer_stream_t stream);
/* Decode cross attention with its query projection and the LayerNorm in
 * front of it fused in (transformer.py:462 -> 459 -> 463): the (head, row)
 * block normalises the pre-norm row y (bits of smer_layernorm_fwd; stored
 * to x_out by the head-0 blocks when given), forms q_h = bf16(LN(y) .
 * wq[h*D..h*D+D-1]^T + bq[h*D..]) and attends like smer_attn_decode over
 * the cache.  bf16, D == 64, dmodel in {512, 768, 1024}. */
int smer_attn_decode_qln(int n_rows, int H, int D, const void* y, long ldy, const float* gamma,
                         const float* beta, float eps, const void* wq, long ldw, const float* bq,
                         void* x_out, long ldx, int dmodel, const void* kcache, const void* vcache,
                         long row_stride, long req_stride, long head_stride, const int32_t* row_req,
                         const int32_t* row_nkeys, void* o, long ldo, float scale,
                         smer_stream_t stream);
/* smer_linear_decode with the post-norm LayerNorm in its prologue: the
 * Linear's input is LN(Y) (row statistics and normalisation bit-identical
 * to smer_layernorm_fwd with the same eps), also stored to X when X is
 * given (the residual of the next sublayer).  K % 8 == 0, K <= 2048. */
int smer_linear_decode_ln(int M, int N, int K, const void* Y, long ldy, const float* gamma,
                          const float* beta, float eps, void* X, long ldx, const void* W, long ldw,
                          const float* bias, int relu, const void* residual, long ldr, void* C,
                          long ldc, float* Cf, long ldcf, void* kv, long kv_row_stride,
                          long kv_req_stride, const int32_t* kv_req, const int32_t* kv_pos,
                          int kv_col0, smer_stream_t stream);
/* fp32 forms of smer_linear_decode / smer_linear_decode_ln (every operand
 * fp32; M <= 64): the parity-mode decode step of the plugin call, which
 * replaces the reference's per-token full fp32 recompute
 * (generation.py:542-545 -> model_generate, generation.py:209-225). */
int smer_linear_decode_f32(int M, int N, int K, const void* A, long lda, const void* W, long ldw,
                           const float* bias, int relu, const void* residual, long ldr, void* C,
                           long ldc, float* Cf, long ldcf, void* kv, long kv_row_stride,
                           long kv_req_stride, const int32_t* kv_req, const int32_t* kv_pos,
                           int kv_col0, smer_stream_t stream);
int smer_linear_decode_ln_f32(int M, int N, int K, const void* Y, long ldy, const float* gamma,
                              const float* beta, float eps, void* X, long ldx, const void* W,
                              long ldw, const float* bias, int relu, const void* residual,
                              long ldr, void* C, long ldc, float* Cf, long ldcf, void* kv,
                              long kv_row_stride, long kv_req_stride, const int32_t* kv_req,
                              const int32_t* kv_pos, int kv_col0, smer_stream_t stream);
/* Flash-decoding for the fp32 plugin step (transformer.py:463 per token):
 * smer_attn_decode_split_f32 attends each (row, head) over 8 key slices in
 * separate blocks, writing unnormalised partials {m, l, 0, 0, acc[64]}
 * (68 floats) at part[((row * H + head) * 8 + slice) * 68];
 * smer_linear_decode_merge_f32 merges them in fixed order into its input
 * rows (K = 64 * H) and applies the Linear + bias (+ReLU) (+residual)
 * (the cross-attention out-projection, transformer.py:463-464).  fp32, D 64. */
int smer_attn_decode_split_f32(int n_rows, int H, int D, const void* q, long ldq, const void* kcache,
                               const void* vcache, long row_stride, long req_stride, long head_stride,
                               const int32_t* row_req, const int32_t* row_nkeys, float* part, float scale,
                               smer_stream_t stream);
/* smer_attn_decode_split_f32 whose query is LN(y) . wq^T + bq (fp32,
 * bits of smer_linear_decode_ln_f32's normalisation), both computed in the
 * attention blocks: replaces smer_linear_decode_ln_f32 (cross-Q) + split
 * attention for the fp32 plugin step at batch 1 (transformer.py:462 -> 459
 * -> 463).  x_out <- LN(y) when given.  D == 64, dmodel == 512. */
int smer_attn_decode_split_qln_f32(int n_rows, int H, int D, const float* y, long ldy, const float* gamma,
                                   const float* beta, float eps, const float* wq, long ldw, const float* bq,
                                   float* x_out, long ldx, int dmodel, const void* kcache, const void* vcache,
                                   long row_stride, long req_stride, long head_stride, const int32_t* row_req,
                                   const int32_t* row_nkeys, float* part, float scale, smer_stream_t stream);
int smer_linear_decode_merge_f32(int M, int N, int K, const float* part, const void* W, long ldw,
                                 const float* bias, int relu, const void* residual, long ldr, void* C,
                                 long ldc, float* Cf, long ldcf, smer_stream_t stream);
/* One greedy grammar step for R requests (generation.py:528-687).
 * logits: fp32 [2R, >=V] rows (request r's last fed token at row 2r+1).
 * state: int32 [R, nst>=9] = pos, flags(sep|cont<<1|pitch<<2|rest<<3), span
 * length, mask index, n_masks, done, no_whole, emitted count, error.
 * targets: int8 [R, max_masks] control target per mask (0 r,1 d,2 o,3 p,4 t).
 * keep: uint8 [13, V] sampling masks per grammar state; cls: uint8 [V] token
 * class bits (1 continue, 2 pitch, 4 duration-only, 8 'sep', 16 'rest',
 * 32 control).  Writes the next step's ids int64 [2R] and meta int32
 * [4, 2R] (position, request, self keys, cross keys; unused rows go to
 * trash_pos), appends the id to out_tok [R, cap], stores #live in *alive. */
int smer_grammar_greedy_step(int R, int V, const float* logits, long ldl, int32_t* state,
                             int nst, const int8_t* targets, int max_masks, const uint8_t* keep,
                             const uint8_t* cls, int eos, int m0, int trash_pos, int max_span,
                             const int32_t* src_len, int64_t* ids, int32_t* meta,
                             int32_t* out_tok, int cap, int32_t* alive, smer_stream_t stream);
/* The same step with no per-step memset or host copy (the decode loop's
 * replays then run back to back): ctl int32 [3] device words {live count,
 * tickets, step} zeroed once by the caller; after the step its live count is
 * written to ring[step % ring_n], pinned host memory the host reads once the
 * step's event has completed.  Replaces the same generation.py:528-687 loop. */
int smer_grammar_greedy_step_ring(int R, int V, const float* logits, long ldl, int32_t* state,
                                  int nst, const int8_t* targets, int max_masks,
                                  const uint8_t* keep, const uint8_t* cls, int eos, int m0,
                                  int trash_pos, int max_span, const int32_t* src_len,
                                  int64_t* ids, int32_t* meta, int32_t* out_tok, int cap,
                                  int32_t* ctl, int32_t* ring, int ring_n, smer_stream_t stream);
/* One sampled grammar step for R requests, drawn in request order as the
 * host loop does (generation.py:33-95 weighted_sampling + sampling, 528-687
 * the span loop with its redraws): e = exp(where(keep, f64(logit), -100)),
 * p = e / np.sum(e) (numpy's pairwise order), p /= sequential sum, sort
 * descending (ties: descending index), cdf = sequential cumsum / cdf[-1],
 * u = numpy legacy random_sample from mt (uint32 [625]: the 624 MT19937 key
 * words and the position, np.random.get_state() layout; updated in place),
 * id = first cdf > u; while reject[state][id] redraw, at most 11 times.
 * Arguments as smer_grammar_greedy_step; reject: uint8 [13, V] (the
 * redraw checks of generation.py:556-615); out_tok ids carry bit 16 when
 * the redraw loop gave up (the reference logs it).  state[r][8] bit 1: the
 * row's probabilities did not sum to 1 within 1e-9 (np.random.choice's
 * territory: the caller redoes the call on the host).  ring != NULL: ctl
 * int32 [3] (ctl[2] = step) and the live count goes to ring[step % ring_n]
 * (pinned host memory); else it is written to ctl[0].  V <= 512. */
int smer_grammar_sample_step(int R, int V, const float* logits, long ldl, int32_t* state, int nst,
                             const int8_t* targets, int max_masks, const uint8_t* keep,
                             const uint8_t* reject, const uint8_t* cls, int eos, int m0,
                             int trash_pos, int max_span, const int32_t* src_len, int64_t* ids,
                             int32_t* meta, int32_t* out_tok, int cap, uint32_t* mt, int32_t* ctl,
                             int32_t* ring, int ring_n, smer_stream_t stream);

int smer_layernorm_fwd(int dtype, int M, int N, const void* x, long ldx,
                       const float* gamma, const float* beta, float eps,
                       void* y, long ldy, float* mean, float* rstd, smer_stream_t stream);
size_t smer_layernorm_bwd_workspace(int M, int N);
/* dx = dLN/d(input); optional dx_drop = dx * keep(seed,row,col)/(1-p).
 * dy_f32=1: dy is fp32 (else activation dtype).  dgamma/dbeta (fp32,
 * nullable) receive (accumulate=1: +=) the column sums. */
int smer_layernorm_bwd(int dtype, int M, int N, const void* dy, long lddy, int dy_f32,
                       const void* x, long ldx, const float* mean, const float* rstd,
                       const float* gamma, void* dx, long lddx,
                       void* dx_drop, long ldxd, float drop_p, uint32_t seed,
                       float* dgamma, float* dbeta, int accumulate,
                       void* workspace, size_t ws_bytes, smer_stream_t stream);
/* The same backward split in two, so the dgamma / dbeta column reduction
 * (which only feeds the optimizer) can run on the weight-gradient stream:
 * _partials writes dx (+ dx_drop) and the per-block column partials into
 * `workspace`; _param_reduce sums them into dgamma / dbeta (nullable). */
int smer_layernorm_bwd_partials(int dtype, int M, int N, const void* dy, long lddy, int dy_f32,
                                const void* x, long ldx, const float* mean, const float* rstd,
                                const float* gamma, void* dx, long lddx, void* dx_drop,
                                long ldxd, float drop_p, uint32_t seed, void* workspace,
                                size_t ws_bytes, smer_stream_t stream);
int smer_layernorm_param_reduce(int M, int N, void* workspace, size_t ws_bytes, float* dgamma,
                                float* dbeta, int accumulate, smer_stream_t stream);

/* out[t] = dropout(table[ids[t]] * scale + pe[pos(t)]), pos(t) = positions
 * ? positions[t] : t % L.  table/pe fp32; out activation dtype. */
int smer_embed_fwd(int dtype, int n_tok, int d, const int64_t* ids, const int32_t* positions,
                   int L, const float* table, const float* pe, float scale,
                   float drop_p, uint32_t seed, void* out, long ldo, smer_stream_t stream);
/* smer_embed_fwd (bf16) plus the e4m3 copy q8 = e4m3(out * *qs) of the stored
 * values, max |out| folded into *amax: the fp8 step's first-layer QKV input
 * (transformer.py:389 after model.py:76, precision "fp8"; delayed scaling). */
int smer_embed_fwd_fp8(int n_tok, int d, const int64_t* ids, const int32_t* positions, int L,
                       const float* table, const float* pe, float scale, float drop_p, uint32_t seed,
                       void* out, long ldo, void* q8, long ldq, const float* qs, unsigned* amax,
                       smer_stream_t stream);
size_t smer_embed_bwd_workspace(int V, int d, int n_tok_total);
/* dtable[v] += scale * sum over both segments of dx[t] * keep/(1-p). */
int smer_embed_bwd(int dtype, int V, int d, float scale,
                   const int64_t* ids0, const void* dx0, long ld0, int n0, float p0, uint32_t seed0,
                   const int64_t* ids1, const void* dx1, long ld1, int n1, float p1, uint32_t seed1,
                   float* dtable, void* workspace, size_t ws_bytes, smer_stream_t stream);

/* denom = sum_i ce_all[y_i] (train.py:736-742). */
int smer_wce_denom(int n, const int64_t* y, const float* ce_all, float* denom,
                   smer_stream_t stream);
/* Per row r: l_r = w[y_r] * (logsumexp(x_r) - x_r[y_r]) (0 for y_r == 0);
 * dlogits_r = grad_scale * w[y_r]/denom * (softmax(x_r) - onehot(y_r)).
 * loss = sum_r l_r / denom written to loss_out (fp32 scalar).  dlog dtype. */
int smer_wce_fwd_bwd(int dtype, int R, int V, const float* logits, long ldl, const int64_t* y,
                     const float* w, const float* denom, float* row_loss, float* loss_out,
                     void* dlogits, long ldd, float grad_scale, smer_stream_t stream);

/* torch.optim.Adam step on flat fp32 buffers; p_bf16 (nullable) receives
 * the bf16 working copy.  bc1 = 1-b1^t, bc2_sqrt = sqrt(1-b2^t). */
int smer_adam(long n, float* p, const float* g, float* m, float* v, void* p_bf16,
              float lr, float b1, float b2, float eps, float bc1, float bc2_sqrt,
              smer_stream_t stream);

int smer_cast(int src_dtype, int dst_dtype, long n, const void* src, void* dst,
              smer_stream_t stream);
/* strided 2-D copy with dtype conversion (dst[r*ldd+c] = src[r*lds+c]). */
int smer_cast2d(int src_dtype, int dst_dtype, int rows, int cols, const void* src, long lds,
                void* dst, long ldd, smer_stream_t stream);
/* Debug: order-independent checksum of a strided region (rows x row_bytes,
 * row stride ld_bytes, 4-byte words): out[0..nparts) receive partial sums
 * of w_i * (2 i + 1) mod 2^64 that the caller adds (repeatability probes,
 * tools/ck_log.py; not on the product path). */
int smer_debug_checksum(const void* p, long rows, long row_bytes, long ld_bytes,
                        unsigned long long* out, int nparts, smer_stream_t stream);
/* Validation accuracy counts (train.py:988-1034 `accuracy` inside
 * validate(), train.py:1037-1195): logits fp32 [R, V] (ld ldl), targets y
 * int64 [R]; rows with y == pad are skipped; for the others pred = the first
 * index of the row maximum (torch.argmax) and, with c = cls[y] (int32 [V],
 * token class ids 0..ncls-1), counts[2c] += 1, counts[2c+1] += (pred == y),
 * and the same in counts[2 ncls], counts[2 ncls + 1] for the total.
 * counts: (2 ncls + 2) uint32, accumulated (zero it for one batch). */
int smer_argmax_accuracy(int R, int V, const float* logits, long ldl, const int64_t* y,
                         const int32_t* cls, int ncls, int pad, unsigned* counts,
                         smer_stream_t stream);
size_t smer_colsum_workspace(int M, int N);
/* out[n] (+)= sum_m x[m, n] (deterministic two-stage). */
int smer_colsum(int dtype, int M, int N, const void* x, long ldx, float* out, int accumulate,
                void* workspace, size_t ws_bytes, smer_stream_t stream);

/* fp8 (OCP e4m3), per-tensor scaled.  smer_fp8_quantize: q[rows, cols] =
 * e4m3(x * 448 / amax|x|), *inv_scale = amax / 448 (device float, no host
 * sync); workspace = smer_fp8_quantize_workspace() bytes (16-B aligned).
 * smer_gemm_fp8: C[M,N] bf16 = (a_inv * b_inv) * A8[M,K] . B8[N,K]^T + bias
 * (+ReLU) (+dropout) (+residual); M, N % 256 == 0, K % 128 == 0, else
 * SMER_ERR_UNSUPPORTED (callers fall back to bf16). */
size_t smer_fp8_quantize_workspace(void);
int smer_fp8_quantize(int rows, int cols, const void* x, long ldx, void* q, long ldq,
                      void* workspace, float* inv_scale, smer_stream_t stream);
/* Batched smer_fp8_quantize over nseg contiguous bf16 tensors: seg is a
 * DEVICE array of nseg x 3 int64 (src bf16*, dst uint8*, n elements; n % 8
 * == 0, src 16-B / dst 8-B aligned); amax_ws: nseg uints of workspace;
 * inv_scale[s] = amax_s / 448.  Same numerics as one smer_fp8_quantize per
 * tensor (per-tensor current scaling); blocks_per_seg: grid.x per tensor. */
int smer_fp8_quantize_segments(int nseg, const int64_t* seg, unsigned* amax_ws, float* inv_scale,
                               int blocks_per_seg, smer_stream_t stream);
int smer_gemm_fp8(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                  const float* a_inv, const float* b_inv, const float* bias, int relu,
                  const void* residual, long ldr, float drop_p, uint32_t drop_seed, void* C,
                  long ldc, smer_stream_t stream);

/* fp8 training forward with delayed per-tensor scaling (BASELINE C4, the
 * QKV / FFN contractions transformer.py:389,393,459,467).  Producers write
 * an e4m3 copy q8 = e4m3(out * *qs) beside their bf16 output and fold
 * max|out| into *amax (float bits, atomicMax); qs / inv come from the
 * previous step's amax via smer_fp8_scales.  smer_gemm_fp8_q is
 * smer_gemm_fp8 plus such a copy of C (the FFN1 output feeding FFN2; C may
 * be null on the streamed epilogue, SMER_FP8_Q8_FAST, to write the copy alone);
 * smer_layernorm_fwd_fp8 is smer_layernorm_fwd (bf16) plus such a copy of y.
 * smer_fp8_scales: for i < n, qs[i] = 448 / amax_prev[i], inv[i] =
 * amax_prev[i] / 448 (both 1 when amax_prev is 0), amax_next[i] = 0. */
int smer_gemm_fp8_q(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                    const float* a_inv, const float* b_inv, const float* bias, int relu,
                    const void* residual, long ldr, float drop_p, uint32_t drop_seed, void* C,
                    long ldc, void* q8, long ldq8, const float* qs, unsigned* amax,
                    smer_stream_t stream);
int smer_layernorm_fwd_fp8(int M, int N, const void* x, long ldx, const float* gamma,
                           const float* beta, float eps, void* y, long ldy, float* mean,
                           float* rstd, void* q8, long ldq, const float* qs, unsigned* amax,
                           smer_stream_t stream);
int smer_fp8_scales(int n, const unsigned* amax_prev, float* qs, float* inv, unsigned* amax_next,
                    smer_stream_t stream);

/* fp8 backward dgrads (C4, `train.py:783` differentiating the Linears of
 * transformer.py:389,393,459,463,467): dX = dY . W runs as the NT product
 * e4m3(dY) . e4m3(W^T)^T.
 * smer_fp8_quantize_segments_t: seg is a DEVICE array of nseg x 4 int64
 * (src bf16 [rows, cols] row-major, dst uint8 [cols, rows], rows, cols; rows
 * and cols multiples of 64): dst = e4m3(src^T * 448 / amax|src|),
 * inv_scale[s] = amax / 448 (current scaling, once per optimizer step).
 * smer_gemm_fp8_ex: smer_gemm_fp8_q plus a ReLU gate (C = gv > 0 ? v *
 * gate_scale : 0, exclusive with residual) for the FFN2 dgrad.
 * smer_layernorm_bwd_fp8: smer_layernorm_bwd (bf16) plus the e4m3 copy
 * q8 = e4m3(g * *qs) of the gradient that feeds the next dgrad (the dropped
 * gradient when drop_p > 0, else dx; with drop_p > 0 and dx_drop null that
 * gradient is written only as its copy), max|g| folded into *amax;
 * partials_only != 0 writes the
 * dgamma / dbeta partials only (smer_layernorm_param_reduce later). */
int smer_fp8_quantize_segments_t(int nseg, const int64_t* seg, unsigned* amax_ws, float* inv_scale,
                                 int blocks_per_seg, smer_stream_t stream);
int smer_gemm_fp8_ex(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                     const float* a_inv, const float* b_inv, const float* bias, int relu,
                     const void* residual, long ldr, const void* gate, long ldg, float gate_scale,
                     float drop_p, uint32_t drop_seed, void* C, long ldc, void* q8, long ldq8,
                     const float* qs, unsigned* amax, smer_stream_t stream);
/* smer_gemm_fp8_ex's gated product (the FFN2 dgrad, transformer.py:467-469
 * under train.py:783) with the gate read from FFN1's e4m3 copy: out = gate
 * byte a positive nonzero e4m3 ? v * gate_scale : 0, plus the e4m3 copy of
 * out (q8 required; 16-B aligned gate rows, ldg % 16 == 0).  With it FFN1
 * may write its e4m3 copy alone (smer_gemm_fp8_q with C null). */
int smer_gemm_fp8_gate8(int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                        const float* a_inv, const float* b_inv, const void* gate8, long ldg,
                        float gate_scale, void* C, long ldc, void* q8, long ldq8, const float* q8_scale,
                        unsigned* q8_amax, smer_stream_t stream);
int smer_layernorm_bwd_fp8(int M, int N, const void* dy, long lddy, const void* x, long ldx,
                           const float* mean, const float* rstd, const float* gamma, void* dx,
                           long lddx, void* dx_drop, long ldxd, float drop_p, uint32_t seed,
                           void* q8, long ldq, const float* qs, unsigned* amax, float* dgamma,
                           float* dbeta, int accumulate, void* workspace, size_t ws_bytes,
                           int partials_only, smer_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMER_HIP_H */
