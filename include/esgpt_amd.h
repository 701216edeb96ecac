/*
 * esgpt_amd.h — C ABI of the MI355X (gfx950) kernels behind eventstreamgpt_amd.
 *
 * The reference (Jwoo5/EventStreamGPT) is pure Python/PyTorch: its swap points are module classes, not an FFI.
 * Each entry point below replaces the ATen ops inside one reference module method (cited per function); the
 * Python side (eventstreamgpt_amd/_lib.py, ctypes) binds these symbols exactly as a maintainer would bind them
 * from the reference (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - All data pointers are DEVICE pointers; sizes are int64; bool tensors are 1-byte (uint8) arrays.
 *   - `stream` is a hipStream_t passed as void*. Every call is asynchronous and stream-ordered; no call
 *     synchronises with the host, allocates, or frees. Callers own all outputs and workspaces.
 *   - Return value: ESGPT_OK or an ESGPT_ERR_* code for invalid arguments / launch failures. Data-dependent
 *     errors (out-of-range embedding index, NaN TTE log-likelihood, subject without observed TTE) are OR-ed
 *     into the caller-provided device error block `err` (16 bytes, 8-B aligned, zeroed by the caller: int32
 *     ESGPT_FLAG_* bits at byte 0, an int32 sticky word at byte 4 (esgpt_step_begin), and at bytes 8..15 the
 *     int64 maximum of every out-of-range embedding index).
 *     esgpt_adamw skips its update while the flags or the sticky word are non-zero (the reference raises before
 *     its optimizer step);
 *     the Python wrapper reads the block once per step and raises the reference's exception type and message.
 *   - dtype codes: ESGPT_F32 (float) or ESGPT_BF16 (bfloat16) for activation tensors; masters are f32.
 */
#ifndef ESGPT_AMD_H_
#define ESGPT_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ESGPT_OK 0
#define ESGPT_ERR_INVALID_ARG 1
#define ESGPT_ERR_LAUNCH 2
#define ESGPT_ERR_UNSUPPORTED 3

#define ESGPT_F32 0
#define ESGPT_BF16 1

#define ESGPT_FLAG_BAD_INDEX 1    /* "Invalid embedding! {max} >= {V}"  (data_embedding_layer.py:485-488) */
#define ESGPT_FLAG_TTE_NAN 2      /* "NaNs in TTE_LL"                    (model_output.py:1362-1363)     */
#define ESGPT_FLAG_TTE_NO_OBS 4   /* "No observed time-to-event ..."     (model_output.py:1366-1367)     */
#define ESGPT_FLAG_BAD_LABEL 8    /* classification / regression target outside its vocabulary slice      */
#define ESGPT_FLAG_PEER_RANK 16   /* set by the host DDP exchange: another rank's step raised a flag         */

/* embedding flags */
#define ESGPT_EMB_NORMALIZE 1     /* do_normalize_by_measurement_index                                     */
#define ESGPT_EMB_STATIC 2        /* StaticEmbeddingMode.SUM_ALL                                           */
#define ESGPT_EMB_TIME 4          /* add TemporalPositionEncoding (at dependency-graph level 0)            */
#define ESGPT_EMB_CUMSUM 8        /* NA input layer: cumulative sum over dependency-graph levels           */
#define ESGPT_EMB_TIME_ABS 16     /* use batch.time instead of the exclusive cumsum of time_delta          */

/* bag-backward selectors */
#define ESGPT_BAG_JOINT 0         /* weight = (values_mask & num-bucket) ? value : 1                       */
#define ESGPT_BAG_CAT 1           /* weight = cat-bucket ? 1 : 0                                           */
#define ESGPT_BAG_NUM 2           /* weight = (values_mask & num-bucket) ? value : 0                       */

/* Common batch view (PytorchBatch fields, data/types.py:86-163). */
typedef struct {
  const int64_t* dyn_idx;       /* [B,L,M] dynamic_indices                       */
  const int64_t* dyn_meas;      /* [B,L,M] dynamic_measurement_indices           */
  const float* dyn_vals;        /* [B,L,M] dynamic_values                        */
  const uint8_t* dyn_vmask;     /* [B,L,M] dynamic_values_mask                   */
  const uint8_t* event_mask;    /* [B,L]   event_mask                            */
  const float* time_delta;      /* [B,L]   time_delta                            */
  const float* time_abs;        /* [B,L]   time (optional, NULL)                 */
  const int64_t* st_idx;        /* [B,S]   static_indices (optional)             */
  const int64_t* st_meas;       /* [B,S]   static_measurement_indices (optional) */
  int64_t B, L, M, S;
} esgpt_batch;

/* Dependency-graph buckets (split_by_measurement_indices, data_embedding_layer.py:505-561): bit k of
 * cat_bits[g] / num_bits[g] is set when measurement index k belongs to bucket g categorically / numerically.
 * G = 1 with all bits set reproduces the un-bucketed (CI) layer. Measurement indices must be < 64. */
typedef struct {
  int64_t G;
  uint64_t cat_bits[8];
  uint64_t num_bits[8];
} esgpt_buckets;

/* ---- Input layer ------------------------------------------------------------------------------------------
 * JOINT mode, fully fused: DataEmbeddingLayer.forward (data_embedding_layer.py:609-708) with _joint_embed
 * (:351-388), static SUM_ALL merge (:693-708), + TemporalPositionEncoding (transformer.py:594-619), event mask
 * and (NA) the level-0 time add + cumsum over levels (transformer.py:926-936).
 * out: f32 [B, L, G, D]. weights: static_w, dynamic_w already normalised as in data_embedding_layer.py:277-280. */
int esgpt_embed_joint_fwd(const esgpt_batch* batch, const esgpt_buckets* buckets, const float* table,
                          int64_t V, int64_t D, const float* sin_div, const float* cos_div, int flags,
                          float static_w, float dynamic_w, float* out, int32_t* err, void* stream);
/* The same over a table stored as table_dtype (ESGPT_F32 or ESGPT_BF16; rows are widened to f32 and accumulated in
 * f32): the SURVEY §8(d) bf16-table gather microbench, and a bf16 embedding table kept by the caller. */
int esgpt_embed_joint_fwd_ex(const esgpt_batch* batch, const esgpt_buckets* buckets, const void* table,
                             int table_dtype, int64_t V, int64_t D, const float* sin_div, const float* cos_div,
                             int flags, float static_w, float dynamic_w, float* out, int32_t* err, void* stream);

/* Event times t[b][l] = sum_{j<l} event_mask[b][j] * time_delta[b][j] (f32 deltas summed in double; the reference's
 * time_from_deltas, transformer.py:305-313 / TemporalPositionEncoding's input), f32 [B, L]: computed once per subject
 * and handed to the input-layer kernels as batch->time_abs with ESGPT_EMB_TIME_ABS (replaces their per-event
 * O(L) prefix). */
int esgpt_event_times(const esgpt_batch* batch, float* times, void* stream);

/* SPLIT_CATEGORICAL_NUMERICAL mode, the gather part of _split_embed (:390-450) for every (event, bucket):
 * x[e,g] = [cat_scale * bag_cat + static_scale * static_bag_cat , num_scale * bag_num]  (f32, [B*L*G, Dc+Dn]).
 * The caller applies one GEMM with [cat_proj | num_proj] and then esgpt_embed_epilogue_fwd. */
int esgpt_embed_split_bags_fwd(const esgpt_batch* batch, const esgpt_buckets* buckets, const float* cat_table,
                               int64_t Dc, const float* num_table, int64_t Dn, int64_t V, int flags,
                               float cat_scale, float num_scale, float static_scale, float* x, int32_t* err,
                               void* stream);

/* out[e,g] = mask_e * cumsum_g'<=g ( y[e,g'] + [g'==0] * time_enc(e) )  (CUMSUM flag; else no cumsum). */
int esgpt_embed_epilogue_fwd(const esgpt_batch* batch, int64_t G, int64_t D, const float* y, const float* sin_div,
                             const float* cos_div, int flags, float* out, void* stream);
/* dy[e,g] = mask_e * sum_{g'>=g} dout[e,g'] (CUMSUM) or mask_e * dout[e,g]. */
int esgpt_embed_epilogue_bwd(const esgpt_batch* batch, int64_t G, int64_t D, const float* dout, int flags,
                             float* dy, void* stream);
/* The same with dy in dy_dtype (ESGPT_F32 or ESGPT_BF16: the SPLIT projection's bf16 backward GEMM operand). */
int esgpt_embed_epilogue_bwd_ex(const esgpt_batch* batch, int64_t G, int64_t D, const float* dout, int flags, void* dy,
                                int dy_dtype, void* stream);
/* SPLIT projection (data_embedding_layer.py:390-450, cat_proj(cat bags) + num_proj(num bags)) as one GEMM over the
 * concatenated bag columns x [N, Dc+Dn] (esgpt_embed_split_bags_fwd's output):
 *   esgpt_split_proj_prep: w_lp [D, Dc+Dn] = [cat_w | num_w] in `dtype` (ESGPT_BF16 / ESGPT_F32), bias [D] =
 *     a_c·cat_b + a_n·num_b (f32, unfused multiply then add), and for ESGPT_BF16 x_lp = bf16(x) (x f32, 16-B
 *     aligned, (Dc+Dn) % 4 == 0); the f32 form leaves x as the GEMM operand (x / x_lp unused). One launch.
 *   esgpt_split_proj_post: from the grouped backward's dw [D, Dc+Dn] and db [D]: cat_dw [D, Dc], num_dw [D, Dn]
 *     (the column blocks), cat_db = a_c·db and num_db = a_n·db (either may be NULL), and for ESGPT_BF16 with dx_lp
 *     given dx = f32(dx_lp) [N, Dc+Dn] (the bag backward's operand). One launch. */
int esgpt_split_proj_prep(const float* x, int64_t N, void* x_lp, const float* cat_w, const float* num_w, int64_t D,
                          int64_t Dc, int64_t Dn, const float* cat_b, const float* num_b, float a_c, float a_n,
                          void* w_lp, float* bias, int dtype, void* stream);
int esgpt_split_proj_post(const void* dx_lp, int64_t N, float* dx, const float* dw, const float* db, int64_t D,
                          int64_t Dc, int64_t Dn, float a_c, float a_n, float* cat_dw, float* num_dw, float* cat_db,
                          float* num_db, int dtype, void* stream);

/* Table gradient of the bag sums (EmbeddingBag backward, atomic-free CSR form):
 * dtable[v,:] = sum over entries (e,g,m) with index v of w(e,g,m) * dsrc[e*G+g, :]
 *             + sum over static entries (b,s) of static_scale * w_s * sum_{e in b valid, g} dsrc[e*G+g, :].
 * dsrc rows have leading dimension ld (elements); D columns are used. dtable: f32 [V, D], fully written. */
size_t esgpt_embed_bag_bwd_workspace(const esgpt_batch* batch, int64_t G, int64_t V, int64_t D);
int esgpt_embed_bag_bwd(const esgpt_batch* batch, const esgpt_buckets* buckets, int selector, int flags,
                        float dyn_scale, float static_scale, const float* dsrc, int64_t ld, int64_t D,
                        int64_t V, float* dtable, void* workspace, size_t workspace_bytes, void* stream);

/* ---- Attention ---------------------------------------------------------------------------------------------
 * InnerSelfAttention._attn (transformer.py:171-217): s = q.k (NO 1/sqrt(d) scaling), causal band (global, or
 * local: 0 <= i-j < window; transformer.py:109-119), additive key-padding mask, softmax in f32, p.v.
 * Element (b,t,h,d) of k/v lives at base + (b*Lk + t)*ld_in + h*hd + d, of q (and dq) at base + (b*tq + t)*ld_in
 * + h*hd + d, of o/dout at base + (b*Lq + t)*ld_o + h*hd + d (q/k/v may alias one packed [.,3D] buffer).
 * Query i sits at key position i + (Lk - Lq): static_kv_first (transformer.py:256-259) drops query 0, i.e. pass
 * q = packed + ld_in, tq = Lk, Lq = Lk - 1 (esgpt_attn_bwd_lead with dq_lead = 1 also writes token 0's zero dq).
 * Rows whose query is padded (query_mask == 0) are written as zeros (the reference zeroes them downstream,
 * transformer.py:818-823). lse: f32 [B,H,Lq] (natural-log softmax normaliser, for the backward).
 * Attention-probability dropout (transformer.py:208): dropout_p in [0,1); keep(b,h,i,j) is a counter hash of
 * (*seed, (bh*Lq + i)*Lk + j) (device uint64, read at kernel start; the backward must see the same value). */
int esgpt_attn_fwd(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                   float* lse,
                   const uint8_t* key_mask, const uint8_t* query_mask, int64_t B, int64_t H, int64_t Lq,
                   int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed, int dtype,
                   void* stream);
/* The same, also writing the dropout keep bits the MFMA forward drew, for esgpt_attn_bwd_ex to read instead of
 * re-hashing them: keep (uint32, esgpt_attn_keep_words(...) words, caller-owned) holds bit (key % 32) of word
 * (bh*Lq + i)*ceil(Lk/32) + key/32 = keep(b, h, i, key) for every (query, key) pair the forward computed (pairs it
 * skips — masked, outside the causal / local band — are left unwritten and never read as kept). keep may be NULL,
 * and is ignored when esgpt_attn_keep_words returns 0 (no dropout, not the MFMA path, or the bits would exceed the
 * cap: Lk > 2048 or more than 256 MiB per launch — the keep bits cost Lq·ceil(Lk/32)·4 bytes per (batch, head), so
 * above the cap the backward re-hashes the same mask and attention memory stays O(L)). */
int64_t esgpt_attn_keep_words(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int64_t tq, int64_t ld_in,
                              int64_t ld_o, int dtype, float dropout_p);
int esgpt_attn_fwd_ex(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                      float* lse, const uint8_t* key_mask, const uint8_t* query_mask, int64_t B, int64_t H, int64_t Lq,
                      int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed, int dtype,
                      uint32_t* keep, void* stream);
size_t esgpt_attn_bwd_workspace(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd);
/* The kernel family esgpt_attn_fwd / esgpt_attn_bwd launch for these arguments (labels for measurements): MFMA
 * (attn_fwd_mfma_kernel / attn_bwd_kernel: bf16, hd in {16, 32, 64, 128}, Lk >= 16), SMALL (one wave per (sequence,
 * head), Lk <= 16: the dependency graph), MFMA_F32 (f32 operands, exact-f32 MFMA) or GENERIC (lane-per-query VALU
 * kernels: other head dims, unaligned operands). */
#define ESGPT_ATTN_PATH_GENERIC 0
#define ESGPT_ATTN_PATH_MFMA 1
#define ESGPT_ATTN_PATH_SMALL 2
#define ESGPT_ATTN_PATH_MFMA_F32 3 /* attn_*_f32_kernel: f32, hd in {16, 32, 64, 128}, Lk > 16, v_mfma_f32_32x32x2_f32 */
int esgpt_attn_path(int64_t hd, int64_t Lq, int64_t Lk, int64_t tq, int64_t ld_in, int64_t ld_o, int dtype);
/* Backward exchange tickets: the MFMA backward runs two workgroups per key block (even / odd query tiles) that add
 * their partial dK / dV through the workspace; `counters` (esgpt_attn_bwd_counters(B, H, Lk) int32, zeroed once
 * by the caller, left zeroed; stream-ordered use) pairs them. NULL counters: one workgroup per key block. */
int64_t esgpt_attn_bwd_counters(int64_t B, int64_t H, int64_t Lk);
int esgpt_attn_bwd(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                   int64_t ld_o,
                   const void* dout, int64_t ld_do, const float* lse, const uint8_t* key_mask,
                   const uint8_t* query_mask, void* dq, void* dk, void* dv, int64_t ld_dqkv, int64_t B, int64_t H,
                   int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed,
                   int dtype, void* workspace, size_t workspace_bytes, int32_t* counters, void* stream);
/* The same reading the forward's keep bits (esgpt_attn_fwd_ex; NULL: regenerate them from the seed). */
int esgpt_attn_bwd_ex(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                      int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* key_mask,
                      const uint8_t* query_mask, void* dq, void* dk, void* dv, int64_t ld_dqkv, int64_t B, int64_t H,
                      int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed,
                      const uint32_t* keep, int dtype, void* workspace, size_t workspace_bytes, int32_t* counters,
                      void* stream);
/* The same, also zero-filling the dq rows t in [-dq_lead, 0) of every sequence (0 <= dq_lead <= 4, Lq + dq_lead <=
 * tq): static_kv_first's token 0, which is no query (transformer.py:256-259), in the same launch on the small
 * (dependency-graph) path, one small extra kernel on the others. Replaces a strided framework fill. */
int esgpt_attn_bwd_lead(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                        int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* key_mask,
                        const uint8_t* query_mask, void* dq, void* dk, void* dv, int64_t ld_dqkv, int64_t B, int64_t H,
                        int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed,
                        const uint32_t* keep, int dtype, void* workspace, size_t workspace_bytes, int32_t* counters,
                        int64_t dq_lead, void* stream);

/* ---- Generation: KV-cache decode -------------------------------------------------------------------------
 * InnerSelfAttention.forward with layer_past / use_cache (transformer.py:261-268 + _attn :171-217), driven by
 * CIPPTForGenerativeSequenceModeling.prepare_inputs_for_generation (conditionally_independent_model.py:198-248).
 * The cache of one layer is a preallocated token-major pair k_cache / v_cache [B, cap, D] (D = H*hd), replacing the
 * reference's per-step torch.cat of [B, H, L, hd] tensors.
 * esgpt_kv_append: rows [past, past+Lq) of both caches <- the k / v thirds of the packed qkv rows [B, Lq, ld_qkv].
 * esgpt_attn_decode: o[b, i] = softmax_j(q_i . k_j) v_j over cache rows j < Lk = past + Lq with query i at key
 *   position Lk - Lq + i (causal; local: position - j < window; key_mask [B, Lk] the full event mask). Rows of
 *   padded queries (query_mask [B, Lq]) and rows without a visible key are zeros. hd <= 128, hd % 4 == 0 (f32) or
 *   hd % 8 == 0 (bf16); q / o row strides ld_q / ld_o elements (q may point into a packed qkv buffer). */
int esgpt_kv_append(const void* qkv, int64_t ld_qkv, void* k_cache, void* v_cache, int64_t B, int64_t Lq,
                    int64_t past, int64_t cap, int64_t D, int dtype, void* stream);
int esgpt_attn_decode(const void* q, int64_t ld_q, const void* k_cache, const void* v_cache, const uint8_t* key_mask,
                      const uint8_t* query_mask, void* o, int64_t ld_o, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                      int64_t cap, int64_t hd, int64_t window, int dtype, void* stream);

/* ---- Output layer losses -----------------------------------------------------------------------------------
 * GenerativeOutputLayerBase.get_{classification,regression,TTE}_outputs (model_output.py:1311-1721) with
 * weighted_loss / safe_weighted_avg (utils.py:134-234), fused: one pass computes every per-event loss, the
 * per-subject/per-term normalisers, the scalar losses and d(total loss)/d(logits). */
#define ESGPT_TERM_SINGLE 1   /* CE(scores, label) + BCE(is_obs, has_label), masked by event & has_label     */
#define ESGPT_TERM_MULTI 2    /* mean_j BCE(scores_j, multi_hot_j), masked by event                           */
#define ESGPT_TERM_MVREG 3    /* safe_weighted_avg_m NLL(Normal(gathered)), masked by event & any(selected)    */
#define ESGPT_TERM_UVREG 4    /* NLL(Normal) + BCE(is_obs, measured), masked by event & has_value             */
#define ESGPT_TTE_EXP 1
#define ESGPT_TTE_LNM 2

typedef struct {
  int32_t kind, meas_idx, vocab_start, vocab_end;
  int32_t col;      /* first logit column of the term (scores / (mean,std) pairs)        */
  int32_t obs_col;  /* is-observed logit column (SINGLE, UVREG), -1 otherwise             */
  int32_t level;    /* content level (NA: dependency-graph level - 1); 0 for CI          */
  int32_t pad;
} esgpt_loss_term;

typedef struct {
  int32_t kind, K, col, pad;
  float mean_log, std_log;
} esgpt_tte_spec;

#define ESGPT_MAX_TERMS 16

/* zc: content logits, rows (b*L + l)*n_levels + level, leading dim ldc; `shift` = 1 (CI): position l reads
 * row l-1 and position 0 reads `zc_bias` (the head bias: Linear(0) = bias). zt: TTE params, rows b*L+l.
 * dzc/dzt: same layout/dtype as zc/zt, must be zero-filled by the caller; dbias: f32 [B, ldc] (position-0
 * content grads, shift mode). losses: f32 [n_terms + 2] = per-term losses, -TTE_LL, total loss. */
size_t esgpt_output_loss_workspace(int64_t B, int64_t L, int n_terms);
int esgpt_output_loss(const esgpt_batch* batch, const void* zc, int64_t ldc, int64_t n_levels, int shift,
                      const void* zc_bias, const void* zt, int64_t ldt, int dtype, const esgpt_loss_term* terms,
                      int n_terms, const esgpt_tte_spec* tte, void* dzc, void* dzt, float* dbias, float* losses,
                      void* workspace, size_t workspace_bytes, int32_t* err, void* stream);
/* The same with an explicit event-kernel path (esgpt_output_loss = ESGPT_LOSS_PATH_AUTO): STREAM (one wave per logit
 * row, the row streamed once in 16-B chunks: dense per-range rules + sparse patches; needs disjoint term columns,
 * <= 4 SINGLE/MULTI terms per level, <= 128 sparse gradient columns per row), ROW_STAGED (the whole row in LDS:
 * ldc·(s + 4) B per wave <= 64 KiB), GENERIC (column by column over zero-filled gradients; any layout). AUTO takes
 * the first that applies. A forced path that does not apply returns ESGPT_ERR_UNSUPPORTED. Every path yields the
 * same gradients bit for bit; the MULTI per-term losses are summed in a path-dependent order. */
#define ESGPT_LOSS_PATH_AUTO 0
#define ESGPT_LOSS_PATH_STREAM 1
#define ESGPT_LOSS_PATH_ROW_STAGED 2
#define ESGPT_LOSS_PATH_GENERIC 3
int esgpt_output_loss_ex(const esgpt_batch* batch, const void* zc, int64_t ldc, int64_t n_levels, int shift,
                         const void* zc_bias, const void* zt, int64_t ldt, int dtype, const esgpt_loss_term* terms,
                         int n_terms, const esgpt_tte_spec* tte, void* dzc, void* dzt, float* dbias, float* losses,
                         void* workspace, size_t workspace_bytes, int32_t* err, int path, void* stream);

/* ---- Fused block elementwise stages ---------------------------------------------------------------------
 * InnerBlock residual adds + resid_dropout + the CI encoder's per-block event mask + the following LayerNorm
 * (transformer.py:350-461, 810-831) in one pass:
 *   h = row_mask ? x + dropout(y + bias) : 0   (f32, x/y/bias/row_mask/h optional)
 *   out = LayerNorm(h; ln_w, ln_b, eps)          (y_dtype / out_dtype: ESGPT_F32 or ESGPT_BF16); mean/rstd f32 [N].
 * Backward: dh = row_mask ? dh_in + LN'(dout) : 0; dx = dh; dy = dropout'(dh); part: f32 workspace
 * [esgpt_residual_ln_partials(N), 3, D]; sums: f32 [3, D] = (d ln_w, d ln_b, d bias). Dropout keep-mask as in
 * attention, counter = row*D + col. Requires D % 4 == 0, D <= 1024, 16-B aligned rows. */
int64_t esgpt_residual_ln_partials(int64_t N);
int esgpt_residual_ln_fwd(const float* x, const void* y, int y_dtype, const float* bias, const uint8_t* row_mask,
                          float dropout_p, const uint64_t* seed, const float* ln_w, const float* ln_b, float eps,
                          int64_t N, int64_t D, float* h, void* out, int out_dtype, float* mean, float* rstd,
                          void* stream);
/* Backward: sums f32 [3, D] = (dgamma, dbeta, dbias) column sums (per-block partials in part, then a second
 * small launch sums them in a fixed order: deterministic). part: f32 workspace [esgpt_residual_ln_partials(N), 3,
 * D]. sums == NULL: the partials only — the caller sums them later, e.g. every LayerNorm of a backward pass in
 * ONE esgpt_colsum_jobs launch ({part, esgpt_residual_ln_partials(N) (1 when N == 0), 3·D, sums}), bit for bit the
 * same sums. counters: reserved (esgpt_residual_ln_counters returns 0; may be NULL). */
int64_t esgpt_residual_ln_counters(int64_t N);
int esgpt_residual_ln_bwd(const float* dh_in, const void* dout, int out_dtype, const float* h, const float* mean,
                          const float* rstd, const float* ln_w, const uint8_t* row_mask, float dropout_p,
                          const uint64_t* seed, int64_t N, int64_t D, float* dx, void* dy, int y_dtype, float* part,
                          float* sums, int32_t* counters, void* stream);
/* The same with skip_T = T > 1: x = [N / (T-1), T, D] and output row r reads x's rows after each sequence's first
 * one (the static_kv_first residual, transformer.py:437); the backward's dx covers all of x's rows (zeros for the
 * first rows). skip_T = 0: the plain forms above. */
int esgpt_residual_ln_fwd_ex(const float* x, const void* y, int y_dtype, const float* bias, const uint8_t* row_mask,
                             float dropout_p, const uint64_t* seed, const float* ln_w, const float* ln_b, float eps,
                             int64_t N, int64_t D, int64_t skip_T, float* h, void* out, int out_dtype, float* mean,
                             float* rstd, void* stream);
int esgpt_residual_ln_bwd_ex(const float* dh_in, const void* dout, int out_dtype, const float* h, const float* mean,
                             const float* rstd, const float* ln_w, const uint8_t* row_mask, float dropout_p,
                             const uint64_t* seed, int64_t N, int64_t D, int64_t skip_T, float* dx, void* dy,
                             int y_dtype, float* part, float* sums, void* stream);
/* Column sums of many partial tables in one launch: sums[c] = Σ_b part[b·width + c] (b ascending in 16 fixed-order
 * row groups, as the residual_ln backward's own sum launch). width % 4 == 0, 16-B aligned part / sums. */
typedef struct esgpt_colsum_job {
  const float* part;
  int64_t n_parts;
  int64_t width;
  float* sums;
} esgpt_colsum_job;
int esgpt_colsum_jobs(const esgpt_colsum_job* jobs, int64_t n_jobs, void* stream);
/* g = act(f + bias) (InnerMLP c_fc bias + activation, transformer.py:378-391); act: 0 exact-erf GELU ("gelu"),
 * 1 tanh GELU ("gelu_new"), 2 ReLU. Backward: dz = dg * act'(f + bias), dbias = column sums (part workspace
 * f32 [esgpt_bias_act_partials(N), F]). Requires F % 4 == 0. */
int esgpt_bias_act_fwd(const void* f, const float* bias, int act, int64_t N, int64_t F, void* g, int dtype,
                       void* stream);
int64_t esgpt_bias_act_partials(int64_t N);
int esgpt_bias_act_bwd(const void* dg, const void* f, const float* bias, int act, int64_t N, int64_t F, void* dz,
                       float* part, float* dbias, int dtype, void* stream);
/* out[c] = sum_r x[r, c] for x [N, F] (ESGPT_F32 / ESGPT_BF16): the bias gradient of a Linear whose output
 * gradient is x (torch's dim-0 reduction of a bf16 matrix is ~20x off the HBM roofline). Fixed summation order
 * (deterministic). part: f32 workspace [esgpt_column_sum_partials(N), F]. */
int64_t esgpt_column_sum_partials(int64_t N);
int esgpt_column_sum(const void* x, int dtype, int64_t N, int64_t F, float* part, float* out, void* stream);

/* ---- Nested-attention glue (structured.hip) -----------------------------------------------------------------
 * StructuredAttention.forward's tensor shuffles (structured_attention.py:28-219: the sequence module on each event's
 * last graph element, the dependency-graph sequence [h_{i-1}, e_{i,1} .. e_{i,G-1}, ctx_i], the event-mask wheres) and
 * the InnerBlock residual (transformer.py:409-461), f32 [rows, D] with D % 4 == 0, 16-B aligned.
 * esgpt_residual_fwd: h[r] = mask(r) ? x[xr(r)] + dropout(y[r]) : 0, mask(r) = row_mask[r / mask_div] (NULL: all);
 *   xr(r) = r, or with skip_T = T > 1 the rows of x = [N / (T-1), T, D] after each first one (static_kv_first
 *   residual, transformer.py:437); y f32 or bf16; dropout as the other kernels (counter hash of r·D + c).
 * esgpt_residual_bwd: dy = mask ? dropout'(dh) : 0 (y's dtype); dx (may be NULL) over all rows of x, zeros where no
 *   output reads them.
 * esgpt_na_split_fwd: per[e] = event_mask[e] ? x[e, G-1] : 0 (x [B·L, G, D]); _bwd writes level G-1 of dx only.
 * esgpt_na_assemble_fwd: seq[e] = [l > 0 ? ctx[e-1] : 0, x[e, 0 .. G-2], ctx[e]] (seq [B·L, G+1, D], e = b·L + l;
 *   ctx is the masked sequence-module output); _bwd: dctx[e] = dseq[e, G] + dseq[e+1, 0] (same subject), and levels
 *   0 .. G-2 of dx = dseq[e, 1 .. G-1]. */
int esgpt_residual_fwd(const float* x, const void* y, int y_dtype, const uint8_t* row_mask, int64_t mask_div,
                       int64_t skip_T, float dropout_p, const uint64_t* seed, int64_t N, int64_t D, float* h,
                       void* stream);
int esgpt_residual_bwd(const float* dh, const uint8_t* row_mask, int64_t mask_div, int64_t skip_T, float dropout_p,
                       const uint64_t* seed, int64_t N, int64_t D, float* dx, void* dy, int y_dtype, void* stream);
int esgpt_na_split_fwd(const float* x, const uint8_t* event_mask, int64_t BL, int64_t G, int64_t D, float* per,
                       void* stream);
int esgpt_na_split_bwd(const float* dper, const uint8_t* event_mask, int64_t BL, int64_t G, int64_t D, float* dx,
                       void* stream);
int esgpt_na_assemble_fwd(const float* ctx, const float* x, int64_t B, int64_t L, int64_t G, int64_t D, float* seq,
                          void* stream);
int esgpt_na_assemble_bwd(const float* dseq, int64_t B, int64_t L, int64_t G, int64_t D, float* dctx, float* dx,
                          void* stream);
/* NA output layer operands (model_output.py NA heads): x f32 [B·L, G, D] -> head [B·L, G-1, D] and last [B·L, D] in
 * out_dtype (ESGPT_F32 / ESGPT_BF16, the head GEMM's), one pass; backward dx = [dhead | dlast] in f32 (a NULL
 * gradient reads as zeros). */
int esgpt_na_head_split_fwd(const float* x, int64_t BL, int64_t G, int64_t D, void* head, void* last, int out_dtype,
                            void* stream);
int esgpt_na_head_split_bwd(const void* dhead, const void* dlast, int in_dtype, int64_t BL, int64_t G, int64_t D,
                            float* dx, void* stream);

/* ---- Projection GEMM -------------------------------------------------------------------------------------
 * C[M, N] = alpha · (A · B) (+ bias[n]) with bf16 operands and f32 accumulation (the q/k/v/out, c_fc/c_proj and head
 * projections and their input / weight gradients, transformer.py:133-163, 378-391). Operand layouts:
 *   A: ESGPT_GEMM_K_CONTIG  A[m][k] = a[m*lda + k]     ESGPT_GEMM_MN_CONTIG  A[m][k] = a[k*lda + m]
 *   B: ESGPT_GEMM_K_CONTIG  B[k][n] = b[n*ldb + k]     ESGPT_GEMM_MN_CONTIG  B[k][n] = b[k*ldb + n]
 * so y = x·Wᵀ is (K, K), dx = dy·W is (K, MN) and dW = dyᵀ·x is (MN, MN). c_dtype ESGPT_BF16 or ESGPT_F32;
 * accumulate (f32 only): C += alpha·A·B (+ bias). alpha: optional DEVICE pointer to one f32 (NULL = 1), read at
 * run time (e.g. the incoming gradient of a loss, without a host sync or a separate scaling kernel). Requires K > 0,
 * K (when either operand is K-contig; a dW product (MN, MN) takes any token count), lda, ldb multiples of 8, the
 * MN-contig extents multiples of 8, 16-B aligned A, B, C (and bias), and N, ldc
 * multiples of 8 (bf16 C) / 4 (f32 C). Split-K: f32 slabs in `workspace` (esgpt_gemm_workspace(M, N, K) bytes, 0 =
 * none needed) and one int32 ticket per output tile in `counters` (esgpt_gemm_counters(M, N) entries, zeroed once
 * by the caller; every launch leaves them zeroed; launches sharing a counter array must be stream-ordered). The
 * last workgroup of each tile sums the slabs in a fixed order inside the same launch: results are deterministic. */
/* Row-tile mask for the token-row GEMMs of the NA dependency-graph module, whose token matrix holds every padded
 * event's G+1 rows (the reference compacts padded events away first, structured_attention.py:162-165,186-193):
 *   esgpt_row_tiles: tiles[t] = 1 iff some event overlapping rows [64t, 64t+64) of a matrix with rows_per_event rows
 *     per event is not padded (event_mask [n_events]); ceil(n_events·rows_per_event / 64) bytes.
 *   esgpt_gemm_row_tiles: the mask (or NULL) of the next esgpt_linear_fwd / _f32 launches and of the dX half of
 *     esgpt_linear_bwd_* issued from this host thread. A tile whose rows all fall in 0-blocks skips its k loop: its
 *     output rows hold act(bias) (forward) or zeros (dX); every other row is bitwise unchanged. Valid when those
 *     rows' values reach no unmasked output and their incoming gradients are zero (the padded events': masked at
 *     the module output). The dW half is never masked (padded rows contribute exact zeros). */
int esgpt_row_tiles(const uint8_t* event_mask, int64_t n_events, int64_t rows_per_event, uint8_t* tiles, void* stream);
int esgpt_gemm_row_tiles(const uint8_t* tiles);
#define ESGPT_GEMM_K_CONTIG 0
#define ESGPT_GEMM_MN_CONTIG 1
size_t esgpt_gemm_workspace(int64_t M, int64_t N, int64_t K);
int64_t esgpt_gemm_counters(int64_t M, int64_t N);
int esgpt_gemm_bf16(int a_layout, const void* A, int64_t lda, int b_layout, const void* B, int64_t ldb, int64_t M,
                    int64_t N, int64_t K, const float* bias, const float* alpha, void* C, int64_t ldc, int c_dtype,
                    int accumulate, void* workspace, size_t workspace_bytes, int32_t* counters, void* stream);
/* Linear layer y = x·wᵀ (nn.Linear: w [out, in] bf16 row-major, x [T, in] bf16 with row stride ldx) in the layouts
 * above:
 *   esgpt_linear_fwd: y = x·wᵀ + bias (f32 [out], optional). With act >= 0 (0 exact-erf GELU, 1 tanh GELU, 2 ReLU)
 *     the bf16 pre-activation goes to `pre` and y = act(pre): InnerMLP's c_fc + activation (transformer.py:
 *     378-391) in one launch. y and pre: [T, out], row stride ldy.
 *   esgpt_linear_bwd: ONE launch for dx = alpha·dy·w (bf16 [T, in]; times act'(pre) when act >= 0, i.e. the
 *     gradient w.r.t. the pre-activation of an input x = act(pre)), dw = alpha·dyᵀ·x (f32 [out, in]) and
 *     db = alpha·Σ_rows dy (f32 [out], optional). dx = NULL skips the input gradient. Split-K workspace:
 *     esgpt_linear_bwd_workspace(T, in, out, dx != NULL) bytes; counters as for esgpt_gemm_bf16 with
 *     esgpt_gemm_counters(out, in) entries. T == 0 zero-fills dw and db.
 *   esgpt_linear_bwd_ex: the same plus n_extra f32 rows db_extra [n_extra, out] added into db before the alpha
 *     scaling, db = alpha·(Σ_rows dy + Σ_b db_extra[b]) — the generative head's bias gradient, whose position-0
 *     rows the loss kernel accumulates per subject (model_output.py:1253-1721; replaces a sum + scale + add).
 *   act | ESGPT_ACT_DERIV (forward and backward together): `pre` carries the activation's DERIVATIVE at the
 *     pre-activation, act'(pre) (computed in the forward's epilogue from the same bf16 / f32 pre-activation, beside
 *     act(pre)), instead of pre itself; the backward multiplies by it. The transcendental work of act' moves into
 *     the forward epilogue, which evaluates the same normal density for act anyway (InnerMLP: esgpt::mlp).
 *   esgpt_linear_bwd_split: esgpt_linear_bwd_ex as two launches on two streams: dx on `stream`; dw, db (and the
 *     split-K workspace / counters, which must not be shared with work on `stream`) on `stream_dw` after it waits
 *     for everything queued on `stream` before the call. The caller joins `stream_dw` back (an event wait) before
 *     reading dw / db. Same tiles and split plan as the grouped launch: bitwise equal results. The weight gradient
 *     then leaves backward's critical path (transformer.py:133-163, 378-391 Linear backward). */
#define ESGPT_ACT_DERIV 8
int esgpt_linear_fwd(const void* x, int64_t ldx, const void* w, int64_t T, int64_t in, int64_t out,
                     const float* bias, int act, void* pre, void* y, int64_t ldy, void* stream);
size_t esgpt_linear_bwd_workspace(int64_t T, int64_t in, int64_t out, int has_dx);
int esgpt_linear_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T, int64_t in,
                     int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre, void* dx,
                     int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes, int32_t* counters,
                     void* stream);
int esgpt_linear_bwd_ex(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T, int64_t in,
                        int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre, void* dx,
                        int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes,
                        int32_t* counters, const float* db_extra, int64_t n_extra, void* stream);
int esgpt_linear_bwd_split(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, int64_t T,
                           int64_t in, int64_t out, const float* alpha, int act, const void* pre, int64_t ldpre,
                           void* dx, int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes,
                           int32_t* counters, const float* db_extra, int64_t n_extra, void* stream, void* stream_dw);
/* f32 forms (the reference's precision: scripts/pretrain.py:24 trains in f32; gfx950 has no TF32 / xf32): every
 * operand, pre-activation and output f32, products on v_mfma_f32_32x32x2_f32 — exact f32, one fmaf per product in
 * k order, at the f32 vector rate. Same semantics, workspace / counter rules and deterministic split-K as the bf16
 * entry points above; K, lda, ldb, ldc multiples of 4, the MN-contig extents and N multiples of 4, 16-B aligned.
 *   esgpt_gemm_f32: C (f32) [+]= alpha·A·B (+ bias); workspace esgpt_gemm_workspace(M, N, K).
 *   esgpt_linear_fwd_f32: y = x·wᵀ + bias, or with act >= 0 pre = x·wᵀ + bias (f32) and y = act(pre).
 *   esgpt_linear_bwd_f32: the grouped backward (dx f32 [· act'(pre)], dw, db [+ db_extra]) in one launch;
 *     workspace esgpt_linear_bwd_f32_workspace(T, in, out, dx != NULL). */
int esgpt_gemm_f32(int a_layout, const float* A, int64_t lda, int b_layout, const float* B, int64_t ldb, int64_t M,
                   int64_t N, int64_t K, const float* bias, const float* alpha, float* C, int64_t ldc, int accumulate,
                   void* workspace, size_t workspace_bytes, int32_t* counters, void* stream);
int esgpt_linear_fwd_f32(const float* x, int64_t ldx, const float* w, int64_t T, int64_t in, int64_t out,
                         const float* bias, int act, float* pre, float* y, int64_t ldy, void* stream);
size_t esgpt_linear_bwd_f32_workspace(int64_t T, int64_t in, int64_t out, int has_dx);
int esgpt_linear_bwd_f32(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* w, int64_t T,
                         int64_t in, int64_t out, const float* alpha, int act, const float* pre, int64_t ldpre,
                         float* dx, int64_t lddx, float* dw, float* db, void* workspace, size_t workspace_bytes,
                         int32_t* counters, const float* db_extra, int64_t n_extra, void* stream);
/* `waiter` waits (device-side, an event) for every piece of work queued on `signaller` before the call: the join of
 * esgpt_linear_bwd_split's weight-gradient stream (and its fork). Both may be captured into one HIP graph. */
int esgpt_stream_wait(void* waiter, void* signaller);
/* Dropout seed bank of one training step (the per-site keep-mask seeds, generative_modeling.py's torch RNG
 * stream replaced by a device counter): bank[i] = *counter + i for i < slots, then *counter += slots — one launch,
 * capturable into a HIP graph (every replay draws fresh seeds). */
int esgpt_seed_bank(int64_t* counter, int64_t* bank, int64_t slots, void* stream);
/* The first launch of a training step: esgpt_seed_bank plus, when err != NULL, the step's own flags started: the
 * previous step's flags (int32 word 0) are OR-ed into the sticky word (int32 word 1), then word 0 is zeroed (and the
 * max bad index, int64 at byte 8, when no error is pending). The flags a step's kernels raise belong to that step alone; the sticky word
 * keeps every later AdamW a no-op until the host has read the block and cleared it (a step queued behind a failed
 * one is discarded, as the reference never runs it). */
int esgpt_step_begin(int64_t* counter, int64_t* bank, int64_t slots, int32_t* err, void* stream);

/* ---- Parameter packing -------------------------------------------------------------------------------------
 * The compute-dtype copies of the f32 parameters a step reads, in ONE launch: the blocks' flat bf16 weight shadow
 * and the generative head's row-concatenated weights / biases (zero rows up to a multiple of 8; model_output.py
 * concatenates nothing — its heads are separate nn.Linear modules). Segment s writes dst[0 .. n) = src[0 .. n)
 * converted to dst_dtype (ESGPT_F32 or ESGPT_BF16, round-to-nearest-even) and dst[n .. n_pad) = 0; src = NULL
 * writes zeros only. Replaces torch.cat + .to(bfloat16) pairs (one launch each). */
typedef struct esgpt_pack_seg {
  const float* src;
  void* dst;
  int64_t n, n_pad;
  int32_t dst_dtype;
  int32_t reserved;
} esgpt_pack_seg;
int esgpt_pack(const esgpt_pack_seg* segs, int64_t n_segs, void* stream);

/* ---- Optimizer ------------------------------------------------------------------------------------------
 * Fused AdamW step (torch.optim.AdamW semantics: decoupled weight decay, bias-corrected moments;
 * generative_modeling.py:460-485 configure_optimizers) over many parameter tensors in ONE launch.
 * table: device array of esgpt_adam_tensor; blocks: device array of (tensor index << 40 | first element), one
 * entry per esgpt_adamw_chunk() elements of each tensor. step = the 1-based optimizer step (bias corrections) shared
 * by every tensor, or per_tensor (device f32 [n_tensors][2] = (lr / (1 - beta1^step_t), sqrt(1 - beta2^step_t)) with
 * tensor t's own step count, as torch keeps one `step` per parameter; NULL = use `step`). err: the error block of
 * the step's forward (NULL = none); a non-zero flag word or sticky word makes the launch a no-op. */
typedef struct esgpt_adam_tensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
} esgpt_adam_tensor;
int64_t esgpt_adamw_chunk(void);
int esgpt_adamw(const esgpt_adam_tensor* table, const int64_t* blocks, int64_t n_blocks, float lr, float beta1,
                float beta2, float eps, float weight_decay, int64_t step, const float* per_tensor,
                const int32_t* err, void* stream);
/* The optimizer step with no host arguments (HIP-graph replayable): esgpt_adamw_prepare advances the device step
 * counters — counters[active[t]] (each parameter's 1-based step) and counters[n_params] (the schedule's step) —
 * and writes the step's learning rate (*lr_out) and per-tensor table per_tensor[t] = (lr / (1 - beta1^step),
 * sqrt(1 - beta2^step)) (betas as doubles, like torch's); esgpt_adamw_dev then updates with the device lr and that
 * table. Both are no-ops while err holds a flag or a sticky word, so a failed or discarded step advances nothing.
 * Schedule kind 0: constant init_lr; kind 1: transformers' polynomial decay with warmup
 * (generative_modeling.py:467-485): lr = init_lr · lambda(step), LambdaLR's step counting. */
typedef struct esgpt_lr_schedule {
  int64_t kind, warmup, total;
  double power, init_lr, end_lr;
} esgpt_lr_schedule;
int esgpt_adamw_prepare(int64_t* counters, const int32_t* active, int n_active, int n_params,
                        const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor, float* lr_out,
                        const int32_t* err, void* stream);
/* The same, also writing the step's hand-off entry, whatever the error state: with ring (16-B aligned, ring_len
 * entries of round_up(n_copy, 4) + 4 floats) entry ring_ctr % ring_len (entry 0 without a counter) receives n_copy
 * (<= 1024) floats of copy_src (a replayed step's loss, which the next replay overwrites) followed, at float offset
 * round_up(n_copy, 4), by the error block's four 32-bit words; *ring_ctr then advances by one. The caller reads its
 * step's loss and error words from the ring without a copy launch of their own (the error words by a D2H copy off
 * the compute stream). */
int esgpt_adamw_prepare_ex(int64_t* counters, const int32_t* active, int n_active, int n_params,
                           const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor,
                           float* lr_out, const int32_t* err, const float* copy_src, int64_t n_copy, float* ring,
                           int64_t* ring_ctr, int64_t ring_len, void* stream);
/* The same with the hand-off entries as separate allocations: ring_tab is a device array of ring_len pointers (8-B
 * aligned), entry k = ring_tab[k] (16-B aligned, round_up(n_copy, 4) + 4 floats), read at launch time — the caller
 * may re-point an entry between launches (TrainStep does so when it still holds a loss returned from that entry).
 * host_words (optional; requires ring_ctr): the device address of ring_len x 4 int32 words of coherent mapped host
 * memory (esgpt_host_words_alloc); the error words of entry k are also written to host_words[4k .. 4k+3], which the
 * host reads once an event recorded after the launch has completed — no D2H copy launch per step. */
int esgpt_adamw_prepare_tab(int64_t* counters, const int32_t* active, int n_active, int n_params,
                            const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor,
                            float* lr_out, const int32_t* err, const float* copy_src, int64_t n_copy,
                            float* const* ring_tab, int64_t* ring_ctr, int64_t ring_len, int32_t* host_words,
                            void* stream);
/* Coherent, device-mapped, zeroed host memory (hipHostMalloc mapped + coherent): *host = the host address, *dev =
 * the address kernels write through. Freed with esgpt_host_words_free(host). */
int esgpt_host_words_alloc(int64_t bytes, void** host, void** dev);
int esgpt_host_words_free(void* host);
int esgpt_adamw_dev(const esgpt_adam_tensor* table, const int64_t* blocks, int64_t n_blocks, const float* lr_dev,
                    float beta1, float beta2, float eps, float weight_decay, const float* per_tensor,
                    const int32_t* err, void* stream);

/* ---- Batch producer (host) ----------------------------------------------------------------------------------
 * PytorchDataset.collate (pytorch_dataset.py:527-701) over flat ragged arrays (the DL_reps parquet columns):
 * subject b = events ev_start[b] .. +ev_count[b]-1 of time_delta (f64; NaN = padded event), event e = elements
 * el_off[e] .. el_off[e+1]-1 of idx / meas (int64, null = 0) and vals (f64, NaN = missing), static elements
 * st_start[b] .. +st_count[b]-1 of st_idx / st_meas (st_count NULL: no static data). HOST pointers; outputs are
 * caller-allocated host buffers (pinned for an async H2D copy) of the shape esgpt_collate_shape returns:
 * event_mask u8 [B,L], time_delta f32 [B,L], dyn_idx / dyn_meas int64 [B,L,M], dyn_vals f32 [B,L,M], dyn_vmask u8
 * [B,L,M], st_idx / st_meas int64 [B,S]. padding_left: sequence padding on the left (generation) instead of the
 * right. esgpt_collate_shape returns ESGPT_ERR_INVALID_ARG when the batch has no dynamic element (the reference's
 * ValueError). n_threads host threads split the subjects. */
int esgpt_collate_shape(int64_t B, const int64_t* ev_start, const int64_t* ev_count, const int64_t* el_off,
                        const int64_t* st_count, int64_t* L, int64_t* M, int64_t* S);
int esgpt_collate(int64_t B, const int64_t* ev_start, const int64_t* ev_count, const double* time_delta,
                  const int64_t* el_off, const int64_t* idx, const int64_t* meas, const double* vals,
                  const int64_t* st_start, const int64_t* st_count, const int64_t* st_idx, const int64_t* st_meas,
                  int64_t L, int64_t M, int64_t S, int padding_left, uint8_t* event_mask, float* time_delta_out,
                  int64_t* dyn_idx, int64_t* dyn_meas, float* dyn_vals, uint8_t* dyn_vmask, int64_t* st_idx_out,
                  int64_t* st_meas_out, int n_threads);

/* ---- Misc ----------------------------------------------------------------------------------------------- */
const char* esgpt_version(void);
int esgpt_device_arch_ok(void); /* 1 if device 0 is gfx950 */

#ifdef __cplusplus
}
#endif

#endif /* ESGPT_AMD_H_ */
