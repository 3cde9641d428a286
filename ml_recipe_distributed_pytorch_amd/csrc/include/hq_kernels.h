// Host-side launch interface of the gfx950 kernels (raw pointers + hipStream_t; no torch headers,
// so each .hip translation unit compiles in seconds).  bindings.cpp wraps these for PyTorch.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <algorithm>
#include <type_traits>

// --precision fp8: 8-bit linear code of gelu'(pre) between the FFN1 forward and the FFN2 dgrad (hq_common.h,
// hq_gd_encode8 / hq_gd_decode8): g = kHqGdLo + q·kHqGdStep over gelu''s exact range [−0.12890, 1.12890]
constexpr float kHqGdLo = -0.12890625f;
constexpr float kHqGdStep = 1.2578125f / 255.f;
constexpr float kHqGdInv = 255.f / 1.2578125f;       // encode: q = rne(fma(g, kHqGdInv, kHqGdOff)), clamp 0…255
constexpr float kHqGdOff = -kHqGdLo * kHqGdInv;
void hq_gelud_encode8(const uint16_t* g, uint8_t* q, size_t n, hipStream_t s);   // bf16 gelu' -> code (n % 8 == 0)

struct HqOuts {  // up to 4 fp32 column-sum destinations (null = skip), passed by value
  float* p[4];
};

// ---- dropout streams ---------------------------------------------------------------------------
// Register (or clear with nullptr) a device uint32 seed that every dropout kernel launched afterwards reads
// instead of its host seed argument (norm.hip).
void hq_set_dropout_seed_ptr(const uint32_t* p);
struct HqDropKey;
HqDropKey hq_drop_key(uint32_t seed, uint32_t opid);

// ---- norm.hip --------------------------------------------------------------------------------
int hq_ln_bwd_partials(int T);
int hq_rowblock_partials(int T);
// y8 != null (fp8 path): y also as e4m3 under the delayed-scaling state q8 [4] at `phase` (see hq_common.h);
// resid == null (bf16 only): `a` already is z (an EPI_BDR GEMM wrote it) — only y, mean, rstd are written
void hq_ln_fwd(const uint16_t* a, const uint16_t* resid, const float* gamma, const float* beta, uint16_t* y, uint16_t* z,
               float* mean, float* rstd, int T, int H, float eps, float p, uint32_t seed, uint32_t opid, hipStream_t s,
               uint8_t* y8 = nullptr, float* q8 = nullptr, int phase = 0);
// da8 != null (--precision fp8 backward): da also as e5m2 under the delayed-scaling state q8 at `phase`
void hq_ln_bwd(const uint16_t* dy, const uint16_t* dy2, const uint16_t* z, const float* gamma, const float* mean,
               const float* rstd, uint16_t* dz, uint16_t* da, float* part, HqOuts outs, int T, int H, float p,
               uint32_t seed, uint32_t opid, bool accumulate, hipStream_t s, uint8_t* da8 = nullptr,
               float* q8 = nullptr, int phase = 0, const float* beta = nullptr);   // beta: z is the output y
void hq_embed_fwd(const int64_t* ids, const int64_t* pids, const int64_t* tids, const uint16_t* ww, const uint16_t* wp,
                  const uint16_t* wt, const float* gamma, const float* beta, uint16_t* y, float* mean, float* rstd, int T,
                  int H, float eps, float p, uint32_t seed, uint32_t opid, int V, int P, int NTY, hipStream_t s);
// deterministic embedding backward scratch (norm.hip: id sort, word-run carries, position partials)
struct HqEmbScratch {
  int32_t *keys, *rows, *skeys, *srows;   // [T] each: (id, row) pairs and their id-sorted copies
  void* sort_tmp;                          // radix-sort digit histograms (sort_bytes)
  size_t sort_bytes;
  float* carry;                            // [chunks][2][H]
  float* ppart;                            // [pos_rows][H] (unused when pos_rows == 0)
};
struct HqEmbScratchSizes {
  size_t sort_bytes;
  int chunks, pos_rows;
};
HqEmbScratchSizes hq_embed_bwd_scratch(int T, int V, int L, int P);
size_t hq_sort_ids_bytes(int T, int V);
void hq_sort_ids(const int64_t* ids, int T, int V, int32_t* keys, int32_t* rows, int32_t* skeys, int32_t* srows,
                 void* hist, size_t hist_bytes, hipStream_t s);
void hq_embed_bwd(const uint16_t* dy, const int64_t* ids, const int64_t* pids, const int64_t* tids, const uint16_t* ww,
                  const uint16_t* wp, const uint16_t* wt, const float* gamma, const float* mean, const float* rstd,
                  float* g_word, float* g_pos, float* g_type, float* part, HqOuts outs, int T, int H, int n_types,
                  int pad_word, int pad_pos, float p, uint32_t seed, uint32_t opid, bool accumulate, int V, int P,
                  int L, const HqEmbScratch& sc, hipStream_t s);
// partial-sum rows embed_bwd needs for T tokens laid out as [T / L][L] (L <= 0: one sequence)
int hq_embed_bwd_partials(int T, int L);
void hq_gelu_fwd(const uint16_t* pre, uint16_t* out, size_t n, hipStream_t s);
void hq_key_bias(const uint8_t* mask, float* kb, int n, hipStream_t s);

// ---- f32_ops.hip: --precision fp32 row-wise ops and flash attention ----------------------------------------------
int hq_f32_row_partials(int T);   // partial rows of the column-partial kernels for T rows
int hq_f32_part_rows(int T);      // rows to allocate for their `part` scratch (partials + the fold's level 1)
void hq_f32_embed_fwd(const int64_t* ids, const int64_t* pids, const int64_t* tids, const float* ww, const float* wp,
                      const float* wt, const float* gamma, const float* beta, float* y, float* mean, float* rstd, int T, int H,
                      float eps, float p, uint32_t seed, uint32_t opid, int V, int P, int NTY, hipStream_t s);
void hq_f32_embed_bwd(const float* dy, const int64_t* ids, const int64_t* pids, const int64_t* tids, const float* ww,
                      const float* wp, const float* wt, const float* gamma, const float* mean, const float* rstd,
                      float* g_word, float* g_pos, float* g_type, float* part, HqOuts outs, int T, int H, int pad_word,
                      int pad_pos, float p, uint32_t seed, uint32_t opid, bool accumulate, int V, int P, int NTY,
                      hipStream_t s);
void hq_f32_ln_fwd(const float* a, const float* resid, const float* gamma, const float* beta, float* y, float* z, float* mean,
                   float* rstd, int T, int H, float eps, float p, uint32_t seed, uint32_t opid, hipStream_t s);
void hq_f32_ln_bwd(const float* dy, const float* dy2, const float* z, const float* gamma, const float* beta, const float* mean,
                   const float* rstd, float* dz, float* da, float* part, HqOuts outs, int T, int H, float p, uint32_t seed,
                   uint32_t opid, bool accumulate, hipStream_t s);
void hq_f32_gelu_fwd(const float* x, float* y, size_t n, hipStream_t s);
void hq_f32_gelu_bwd(const float* dout, const float* x, float* d, float* part, float* g_bias, int T, int N, bool accumulate,
                     hipStream_t s);
void hq_f32_colsum(const float* x, float* part, float* out, int T, int N, bool accumulate, hipStream_t s);
void hq_f32_attn_fwd(const float* qkv, const float* key_bias, float* ctx, float* lse, int B, int L, int nh, float p,
                     uint32_t seed, uint32_t opid, float scale, hipStream_t s);
void hq_f32_attn_bwd(const float* dctx, const float* qkv, const float* ctx, const float* lse, const float* key_bias,
                     float* dqkv, float* delta, int B, int L, int nh, float p, uint32_t seed, uint32_t opid, float scale,
                     hipStream_t s);
void hq_ln_guard(const float* master, const int64_t* goff, const int64_t* boff, int n, int H, float ratio, uint8_t* flags,
                 hipStream_t s);
void hq_gelu_bwd(const uint16_t* dout, const uint16_t* pre, uint16_t* dpre, float* part, HqOuts outs, int T, int N,
                 bool accumulate, hipStream_t s);
void hq_bias_grad(const uint16_t* dy, float* part, HqOuts outs, int T, int N, bool accumulate, hipStream_t s);

// ---- attention.hip ----------------------------------------------------------------------------
void hq_attn_set_force_slow(int v);          // tests: every ring-forward workgroup takes the slow path
size_t hq_attn_mask_bytes(int B, int L, int nh);   // dropout keep-bits written by fwd, read by bwd
// ctx8 / q8 / phase (optional, --precision fp8): ctx also written as e4m3 under the delayed-scaling state q8;
// in the backward dqkv8 / q8 / phase: dQKV also as e5m2 (the QKV dgrad's fp8 input)
void hq_attn_fwd(const uint16_t* qkv, const float* key_bias, uint16_t* ctx, float* lse, uint16_t* mbits, int B, int L,
                 int nh, int dh, float p, uint32_t seed, uint32_t opid, float scale, hipStream_t s,
                 uint8_t* ctx8 = nullptr, float* q8 = nullptr, int phase = 0);
void hq_attn_bwd(const uint16_t* dctx, const uint16_t* qkv, const uint16_t* ctx, const float* lse, const float* key_bias,
                 const uint16_t* mbits, uint16_t* dqkv, float* delta, int B, int L, int nh, int dh, float p, float scale,
                 bool deterministic, hipStream_t s, uint8_t* dqkv8 = nullptr, float* q8 = nullptr, int phase = 0,
                 float* bpart = nullptr);
// bpart != null (with dqkv8): dqkv (bf16) is NOT written; instead the QKV bias-gradient column partials
// bpart[B·ceil(L/32)][3H] (sum over rows = Σ_t dQKV[t, :]) for the fp8 weight gradient.

// ---- optim.hip --------------------------------------------------------------------------------
struct HqOptChunk {      // one work item of the fused optimizer: <= kOptChunk elements of one segment
  int64_t start;
  int32_t numel;
  int32_t group;         // param group index (weight decay / lr factor table)
};
constexpr int kOptChunk = 8192;
constexpr int kOptMaxGroups = 8;
struct HqOptGroups {
  float lr[kOptMaxGroups];
  float wd[kOptMaxGroups];
};
void hq_sq_norm_partials(const float* g, int64_t n, float* partials, int nparts, hipStream_t s);
void hq_fingerprint(const float* x, int64_t n, int nparts, uint64_t* out, hipStream_t s);
// Σg² of chunks c0 … c1-1 of the grad arena (chunks: int64 [C][2] = start, numel; numel <= kNormChunk, % 4 == 0)
constexpr int64_t kNormChunk = 1 << 18;
void hq_sq_norm_chunks(const float* g, const int64_t* chunks, int c0, int c1, float* partials, hipStream_t s);
void hq_clip_coef(const float* partials, int nparts, float max_norm, float* norm_out, float* coef_out, hipStream_t s);
void hq_adamw(float* master, uint16_t* compute, const float* grad, float* m, float* v, const HqOptChunk* chunks,
              int nchunks, HqOptGroups groups, float beta1, float beta2, float eps, float step_size_mult,
              const float* clip_coef, hipStream_t s);
void hq_adamod(float* master, uint16_t* compute, const float* grad, float* m, float* v, float* n, const HqOptChunk* chunks,
               int nchunks, HqOptGroups groups, float beta1, float beta2, float beta3, float eps, float bias_corr,
               const float* clip_coef, hipStream_t s);
void hq_cast_f32_bf16(const float* src, uint16_t* dst, int64_t n, float scale, hipStream_t s);
void hq_cast_bf16_f32(const uint16_t* src, float* dst, int64_t n, float scale, hipStream_t s);

// ------------------------------------------------------------------ MFMA GEMM (gemm.hip)
enum { HQ_EPI_NONE = 0, HQ_EPI_BIAS = 1, HQ_EPI_GELU = 2, HQ_EPI_DGELU = 3, HQ_EPI_RESID = 4, HQ_EPI_GELUD = 5, HQ_EPI_DMUL = 6,
       HQ_EPI_BDR = 7 };
// kernel family for this shape: 256 / 128 = the 256-row kernels with that block width, 1 = the 128²-tile
// kernel (M tails, low-fill grids), 0 = unsupported (need N % 128 == 0, K % 64 == 0)
int hq_gemm_nt_supported(int M, int N, int K);
// rows of the DGELU / DMUL column-partial buffer for this shape ([rows][N])
int hq_gemm_nt_part_rows(int M, int N, int K);
// 0 = auto (128² tiles for M % 256 != 0 or < 80 % CU fill; else the persistent v3 kernel for K <= 2304,
// v2 above), 1 = v1, 2 = v2, 3 = v3 (the 256-row kernels wherever M % 256 == 0), 4 = 128² tiles always
void hq_gemm_set_variant(int v);
void hq_zero_f32(float* p, size_t n, hipStream_t s);   // own zero-fill kernel (no runtime memset node in graphs)
void hq_gemm_set_store_policy(int v);   // persistent-kernel epilogue stores: 0 default, 1 nt|sc1 at K <= 768, 2 always
void hq_gemm_set_stagger(int v);   // v3 start offset of half the workgroups (units of s_sleep(127))
// v3 tile scheduling: 1 = dynamic (a workgroup's third and later tiles come from per-XCD atomic ticket
// counters, so CUs held by another stream's kernels — RCCL all-reduce under the backward — cost the GEMM
// only their share), 0 = static round-robin (tile = id + k·grid); HQ_GEMM_SCHED sets it, default 0 (the
// DP reducer selects 1 when world > 1)
void hq_gemm_set_sched(int v);
int hq_gemm_get_sched();   // the setting in effect (HQ_GEMM_SCHED at load, or the last set)
// Diagnostic: `blocks` workgroups (one per CU: 96 KiB LDS each) that spin for `usec` µs on stream s —
// stands in for a collective kernel holding CUs while a GEMM runs (tools/gemm_contention_bench.py)
// C[M,N] = A[M,K]·B[N,K]^T (+epilogue); P = GELU pre-activation (out for EPI_GELU, in for EPI_DGELU)
// or its derivative gelu'(pre) (out for EPI_GELUD, in for EPI_DMUL);
// R = residual (EPI_RESID, EPI_BDR); part = [M/256][N] column partial sums (EPI_DGELU)
// EPI_BDR: C = z = dropout_p(bf16(acc + bias)) + R with the counter-hash stream (seed, opid) at element
// index m·ldc + n — exactly what ln_fwd computes as z, so the following LayerNorm reads z alone
// ws: fp32 split-K workspace of hq_gemm_nt_ws_floats(M, N, K, epi) floats (caller-allocated on stream s, e.g.
// from the stream-aware caching allocator; may be null when that size is 0)
size_t hq_gemm_nt_ws_floats(int M, int N, int K, int epi);
void hq_gemm_nt(const uint16_t* A, const uint16_t* B, uint16_t* C, const float* bias, uint16_t* P, const uint16_t* R,
                float* part, int M, int N, int K, int lda, int ldb, int ldc, int epi, int bn, hipStream_t s,
                float drop_p = 0.f, uint32_t drop_seed = 0, uint32_t drop_opid = 0, float* ws = nullptr);

// Exact-fp32 strided GEMM on the f32 MFMA (gemm_f32.hip, --precision fp32): C = alpha·A·Bᵀ (+bias[j]) (+R),
// A(i,k) = A[i·sa_i + k·sa_k], B(j,k) = B[j·sb_j + k·sb_k] (sa_k == 1 or sa_i == 1; likewise B), batch z =
// outer·nb_in + inner with per-operand strides (C and R share C's); ksplit > 1 (batch 1): ws holds ksplit M·N slabs.
int hq_gemm_f32_splits(int M, int N, int K, int batch);
void hq_gemm_f32(const float* A, const float* B, float* C, const float* bias, const float* R, float* ws, int M, int N,
                 int K, long long sa_i, long long sa_k, long long sb_j, long long sb_k, int ldc, int ldr, int batch,
                 int nb_in, long long ba_out, long long ba_in, long long bb_out, long long bb_in, long long bc_out,
                 long long bc_in, float alpha, int ksplit, hipStream_t s);

// Weight-gradient GEMM (gemm_tn.hip): out[N,K] (+)= Aᵀ·B, A = dy [T,N] bf16, B = x [T,K] bf16 (token-major),
// split-K over T into S fp32 slabs part[S][N][K] (caller-provided) reduced into out; with bout != null
// also the fused bias gradient bout[N] (+)= Σ_t A[t, n] through slabs bpart[S][N].
// hq_gemm_tn_splits: the split count for this shape, 0 = unsupported (need N%256, K%256 == 0, T >= 128;
// a token tail T % 64 != 0 stages zero rows through the buffer descriptors' bounds).
void hq_gemm_tn_set_variant(int v);   // bias-free wgrad kernel: 0 auto, 1 lockstep, 5 alternating rows (A/B, tests)
int hq_gemm_tn_splits(int T, int N, int K);
void hq_gemm_tn(const uint16_t* A, const uint16_t* B, float* part, float* out, float* bpart, float* bout, int T, int N, int K,
                int S, bool accumulate, hipStream_t s);
// fp8 form (--precision fp8): A = dy e5m2, B = x e4m3 (token-major bytes), dequantised by sa[0]·sb[0]; same
// slabs / reduce, no fused bias.  hq_gemm_tn8_splits: split count, 0 = unsupported.
int hq_gemm_tn8_splits(int T, int N, int K);
void hq_gemm_tn8(const uint8_t* A, const uint8_t* B, const float* sa, const float* sb, float* part, float* out, int T,
                 int N, int K, int S, bool accumulate, hipStream_t s);

// fp8 NT GEMM (gemm_fp8.hip): C = A8·B8ᵀ·sa·sb (+ epilogue), B8 e4m3.  Forward epi ∈ {HQ_EPI_BIAS,
// HQ_EPI_GELUD} with A8 e4m3; backward epi ∈ {HQ_EPI_NONE, HQ_EPI_RESID (C + P), HQ_EPI_DMUL (C ⊙ P,
// column sums into part[M/256][N])} with A8 e5m2.  C8 != null (GELUD / DMUL): the output also as e4m3 / e5m2 under
// delayed scaling driven by the 4-float state q8 / phase.
int hq_gemm_fp8_supported(int M, int N, int K);
void hq_gemm_fp8_set_variant(int v);   // 0 auto (persistent but the Q8 DMUL), 2 = per-tile v2, 3 = persistent
void hq_gemm_fp8(const uint8_t* A, const uint8_t* B, uint16_t* C, const float* bias, uint16_t* P, const float* sa,
                 const float* sb, uint8_t* C8, float* q8, int phase, int M, int N, int K, int epi, hipStream_t s,
                 float* part = nullptr, int gd8 = 1);
// delayed-scaling e4m3 quantiser (one pass): y = x / s(prev amax), amax tracked in q8 (see gemm_fp8.hip)
void hq_fp8_quant_delayed(const uint16_t* x, uint8_t* y, size_t n, float* q8, int phase, hipStream_t s);
long long hq_fp8_quant_multi_blocks(long long n8);   // blocks of one segment of n8 8-element groups
// fp8 producers write per-wave amax partials into this device scratch (>= n floats, current device) and
// hq_fp8_amax_fold folds them into the delayed-scaling state q8 (slot `phase`, clears (phase+1)%3, q8[3]).
// A producer also publishes q8[3] itself (hq_fp8_publish_scale), so under hq_fp8_fold_defer(1) a site's fold may
// wait: the partials come from a per-device arena (pass the site's state q8 and stream s) and the folds of many
// sites run as one batched launch at hq_fp8_fold_flush() — or earlier, automatically, when a site with a pending
// fold produces again, a producer runs on another stream, or the arena is full.
float* hq_fp8_amax_parts(size_t n, const float* q8 = nullptr, hipStream_t s = nullptr);
void hq_fp8_amax_fold(const float* part, int n, float* q8, int phase, hipStream_t s, float fmax = 448.f);
int hq_fp8_fold_defer(int on);   // on = 0 flushes the pending folds and returns to immediate folds
void hq_fp8_fold_flush();
int hq_fp8_fold_pending();
void hq_fp8_quant_delayed_multi(const uint16_t* x, uint8_t* y, const long long* seg, int nseg, long long blocks,
                                float* states, int phase, hipStream_t s);

// tiles: int32 [ntiles][6] = (src_off, dst_off, rows, cols, r0, c0); src [rows][cols] -> dst [cols][rows]
void hq_transpose_tiles(const uint16_t* src, uint16_t* dst, const int* tiles, int ntiles, hipStream_t s);
void hq_transpose_tiles8(const uint8_t* src, uint8_t* dst, const int* tiles, int ntiles, hipStream_t s);
// out[c] (+)= sum_p part[p][c], part f32 [P][N]
void hq_colsum(const float* part, int P, int N, float* out, bool accumulate, hipStream_t s);

// ------------------------------------------------------------------ fp8 (fp8.hip); n % 8 == 0
void hq_amax_bf16(const uint16_t* x, size_t n, unsigned* amax, hipStream_t s);
void hq_fp8_quant(const uint16_t* x, uint8_t* y, size_t n, const unsigned* amax, float* scale, hipStream_t s);

// ------------------------------------------------------------------ QA span head (norm.hip)
void hq_span_fwd(const uint16_t* seq, const float* w, const float* b, float* logits, int T, int H, hipStream_t s);
// part: [hq_ln_bwd_partials(T)][2][H] scratch; dw: [2][H] (+)=
void hq_span_bwd(const uint16_t* seq, const float* w, const float* g, uint16_t* dseq, float* part, float* dw, int T,
                 int H, bool accumulate, hipStream_t s);
// out_q[c] (+)= Σ_p part[p][q·Hq + c] for the (≤ 4) destinations of outs, part f32 [P][N]
void hq_colsum_outs(const float* part, int P, int N, HqOuts outs, int Hq, bool accumulate, hipStream_t s);

// ------------------------------------------------------------------ fused QA heads + losses (heads.hip)
struct HqHeadWeights {  // fp32 master weights: pooler, classifier [NL,H], reg start/end [1,H], span [2,H]
  const float *wp, *bp, *wc, *bc, *wrs, *brs, *wre, *bre, *wsp, *bsp;
};
struct HqHeadGrads {    // fp32 arena gradients (null = not trainable)
  float *gwp, *gbp, *gwc, *gbc, *gwrs, *gbrs, *gwre, *gbre, *gwsp, *gbsp;
};
struct HqLossCfg {
  int kind;             // 0 = CE (optional class weights, ignore_cls), 1 = focal (ignore -1), 2 = label smoothing
  int ignore_cls;
  float w[5];           // start, end, start_reg, end_reg, cls
  float alpha, gamma;   // focal
  float conf, fill;     // label smoothing target distribution
};
size_t hq_qa_heads_fwd_scratch(int B, int H);   // floats of the fwd head-partial scratch
// logits [B·L, 2], pooled [B, H], cls [B, NL], reg [B, 2] (sigmoid); cnt: a zeroed device word, one per stream
// seq / dseq: bf16 (seq_f32 = false) or fp32 [B·L, H]
void hq_qa_heads_fwd(const void* seq, const HqHeadWeights& w, float* logits, float* pooled, float* cls, float* reg,
                     float* hpart, unsigned* cnt, int B, int L, int H, int NL, float p, uint32_t seed, uint32_t opid,
                     hipStream_t s, bool seq_f32 = false);
int hq_qa_loss_partials(int B);                 // rows of the [rows][4] loss scratch
// losses[6] = start, end, start_reg, end_reg, cls, total; dlog [B·L, 2] and dheads [B, 16] = d total / d preds
void hq_qa_loss(const float* logits, const float* cls, const float* reg, const int64_t* t_start, const int64_t* t_end,
                const int64_t* t_cls, const float* t_rs, const float* t_re, const float* lw, float* dlog, float* dheads,
                float* losses, float* part, unsigned* cnt, int B, int L, int NL, const HqLossCfg& cfg, const int* seg_len,
                int nseg, hipStream_t s);   // nseg equal segments (seg_len [nseg] span lengths, or null = L)
int hq_qa_heads_bwd_span_blocks(int T);         // rows of the [rows][2H + 2] span partial scratch
void hq_qa_heads_bwd(const void* seq, const float* dlog, const float* dheads, const float* gscale, const float* pooled,
                     const float* reg, const HqHeadWeights& w, const HqHeadGrads& g, void* dseq, float* span_part,
                     int B, int L, int H, int NL, bool accumulate, float p, uint32_t seed, uint32_t opid, hipStream_t s,
                     bool seq_f32 = false, float* dpre = nullptr);   // dpre: [B][H] scratch (dL/d pooler pre-activation)
