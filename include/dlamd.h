/*
 * dlamd.h — C ABI of the MI355X-native CTR training hot path (libdlamd.so).
 *
 * The reference (RodJohn/deep_learning) is TensorFlow-1.x graph code: its hot
 * path is TF's own C++ kernels behind `sess.run(op)` ("Third-party
 * native arithmetic").  Each entry point below replaces one group of those TF
 * ops at a reference call site (cited per function).  Host code (Python,
 * deep_learning_amd/_lib.py) binds this header through ctypes.
 *
 * Conventions:
 *   - extern "C" only; device pointers (row-major, contiguous); explicit dims.
 *   - every call is asynchronous on the given HIP stream (`stream` is a
 *     hipStream_t passed as void*; NULL = default stream); no allocation and no
 *     host synchronisation inside any call, so a caller may capture a whole
 *     training step into a hipGraph.
 *   - return 0 on success, otherwise a nonzero code; the message is available
 *     from dl_last_error() (thread-local).  No C++ exception crosses the ABI.
 *   - out-of-range ids never fault: they read as zero rows and raise the
 *     caller-provided device error word (`err`, may be NULL) which the host
 *     turns into an exception (TF's InvalidArgumentError "indices[...] = k is
 *     not in [0, N)").
 */
#ifndef DLAMD_H
#define DLAMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DL_ABI_VERSION 1

int dl_abi_version(void);
const char* dl_last_error(void);
/* hipDeviceSynchronize + error check (host utility, never inside a step). */
int dl_device_sync(void);

/* ------------------------------------------------------------------------
 * Embedding layout shared by the forward and backward embedding kernels.
 * One instance describes how a model maps a batch onto the table rows:
 *   FM fields  = [C cont fields (row fm_cont_offset+j, value cont[b][j]) if fm_cont]
 *              + [S single cate fields (row id+fm_cate_offset, value 1)]
 *              + [fm_extra pooled fields (vectors already in x0 at x0_pool_col,
 *                 first-order values already in fm_out at column fm_single)]
 *   deep input = x0[b][x0_cont_col..+C] = cont, x0[b][x0_vec_col..+V] = vector,
 *                x0[b][x0_cat_col + f*E ..] = table[id_f + deep_cate_offset]
 *   fm_out[b]  = [first (F = fm_single + fm_extra) | second (E)]
 * -------------------------------------------------------------------- */
typedef struct dl_emb_layout {
  int64_t n_rows;           /* rows of table [n_rows, E] and first-order [n_rows]   */
  int64_t fm_cont_offset;   /* deepfm_pipeline.py:58-61,89 (0); deepfm_multi.py:139 */
  int64_t fm_cate_offset;   /* deepfm_pipeline.py:89 (+C)                            */
  int64_t deep_cate_offset; /* deepfm_pipeline.py:120 (0: raw ids — ledger item 1)   */
  int32_t batch;            /* B                                                     */
  int32_t emb_dim;          /* E in {4, 8, 16, 32, 64}                               */
  int32_t cont_fields;      /* C                                                     */
  int32_t vector_size;      /* V                                                     */
  int32_t cate_fields;      /* S single-valued ids per sample                        */
  int32_t cate_ld;          /* int64 elements between samples in the id matrix       */
  int32_t fm_cont;          /* 1: the C cont fields are FM fields                    */
  int32_t use_fm;           /* 0: no FM outputs (dnn / wdl)                           */
  int32_t fm_extra;         /* M pooled multi-hot fields appended to the FM           */
  int32_t zero_row0;        /* 1: row 0 reads as zeros and gets no gradient (:83-86) */
  int32_t x0_ld;            /* floats between samples in x0                          */
  int32_t x0_cont_col;      /* -1: cont not copied into x0                           */
  int32_t x0_vec_col;       /* -1: vector not copied into x0                         */
  int32_t x0_cat_col;       /* column of the first single-cate embedding in x0 (-1:
                               not written — dl_embed_fwd / _slots / _indexed only, the
                               embeddings then read by dl_gemm_s3_nt_gather)          */
  int32_t x0_pool_col;      /* column of the first pooled vector in x0 (fm_extra>0)  */
  int32_t fm_ld;            /* floats between samples in fm_out                      */
  int32_t dx0_ld;           /* floats between samples in dx0 (backward)              */
  int32_t dx0_cat_col;      /* column of the first single-cate gradient in dx0       */
  int32_t multi_width;      /* multi-hot id columns after the S singles that the batch
                               index also covers (record path of deepfm_multi_cate; 0 = none):
                               index refs per sample = (use_fm ? S : 0) + S + multi_width */
  int32_t cont_rows_compact;/* 1: the FM cont-field rows are addressed as rows 0..C-1 of the
                               row buffer handed over (the gathered rows of the record and
                               sharded paths; their gradients in a [C] buffer), while which
                               of them is the zero row is still decided on the table row
                               fm_cont_offset + f (deepfm_multi.py:139 puts them after the
                               cate ids; deepfm_pipeline.py:58-61 at the top)           */
  int32_t x0_bf16;          /* 1: the forward's x0 is a bf16 matrix (uint16, x0_ld elements per
                               sample; the bf16 tower's first operand, config C5): cate, cont
                               and vector columns are written rounded to nearest-even.
                               Requires fm_extra == 0 (pooled vectors are read back as f32) */
} dl_emb_layout;

/* Embedding gather + FM first/second order + deep-input assembly (forward).
 * Replaces GatherV2 x3, ConcatV2 (row-0 zero), Mul/Sum/Square/Sub at
 * models/deepfm_pipeline.py:83-123 (also dnn_pipeline.py:72-83, wdl.py:132-179,
 * deepfm_multi_cate.py:127-171 for the single fields).
 * fm_sum [B, E] keeps sum_f e_f for the backward (may be NULL when !use_fm). */
int dl_embed_fwd(const dl_emb_layout* L, const float* table, const float* first_order,
                 const int64_t* cate, const float* cont, const float* vector,
                 float* x0, float* fm_out, float* fm_sum, int32_t* err, void* stream);
/* dl_embed_fwd over a slot plane [n_rows][2E] (dl_rec_flush with DL_REC_PLANE_SLOTS): row r's
 * embedding in columns 0..E-1, its first-order weight in column E — an FM reference's row and
 * weight in one 128-B slot (E = 16), one random request instead of two (predict on a flushed
 * lazy table; same outputs as dl_embed_fwd on separate planes, bit for bit). */
int dl_embed_fwd_slots(const dl_emb_layout* L, const float* slots, const int64_t* cate, const float* cont,
                       const float* vector, float* x0, float* fm_out, float* fm_sum, int32_t* err, void* stream);
/* The FM side of predict's fused front (with dl_gemm_s3_nt_gather_tab): dl_embed_fwd_slots
 * (slot_plane = 1) or dl_embed_fwd on the p plane (slot_plane = 0, models without FM) with
 * x0_cat_col = -1, which instead of the deep rows writes their byte offsets in the plane into
 * gtab ([ceil(B / 256)][fields][272] u32, 0xFFFFFF00 for a masked or invalid id — the first
 * tower layer's LDS table as it stands: 16 samples of a field one 64-B write).  x0 may be NULL
 * when x0_cont_col and x0_vec_col are -1 too (nothing of x0 written), fm_sum may be NULL
 * (predict: no backward reads it).  Same fm_out and x0 cont / vector columns as
 * dl_embed_fwd_slots bit for bit. */
int dl_embed_fwd_gtab_ok(const dl_emb_layout* L);   /* 1: the layout qualifies (E = 8 / 16, FM slots in <= 4 passes) */
int dl_embed_fwd_gtab(const dl_emb_layout* L, const float* plane, int32_t slot_plane, const int64_t* cate,
                      const float* cont, const float* vector, float* x0, float* fm_out, float* fm_sum, uint32_t* gtab,
                      int32_t* err, void* stream);

/* Backward of dl_embed_fwd for the FM (single fields) and deep lookups.
 * dz [B] = dL/dlogit, w_head = head weights whose first F+E entries weight
 * [first | second]; dx0 = dL/dx0.  Scatter-adds row gradients into the dense
 * gradient tables g_table [n_rows, E], g_first [n_rows] (f32 atomics), marks
 * touched rows in `touched` [n_rows] (uint8), and writes the hot cont-field
 * rows as per-block partials into cont_slab [grid][C*(E+1)] which
 * dl_embed_cont_reduce folds in.  Replaces the Gather gradients
 * (UnsortedSegmentSum) + StridedSliceGrad of deepfm_pipeline.py:188. */
int dl_embed_bwd(const dl_emb_layout* L, const float* table, const int64_t* cate,
                 const float* cont, const float* dz, const float* w_head,
                 const float* fm_sum, const float* dx0, float* g_table, float* g_first,
                 uint8_t* touched, float* cont_slab, int32_t cont_slab_blocks, void* stream);
int dl_embed_bwd_grid(const dl_emb_layout* L);   /* grid size = cont_slab blocks */
int dl_embed_cont_reduce(const dl_emb_layout* L, const float* cont_slab, int32_t blocks,
                         float* g_table, float* g_first, uint8_t* touched, void* stream);

/* Indexed forward (row-sharded tables): the row of reference ref = b*n_slot + slot
 * (index order of dl_index_build) is inv_base + inv[ref] in `rows` / `rows_first`
 * (the rows exchanged for this batch; rows below inv_base hold the replicated
 * cont-field rows read by the FM cont fields). */
int dl_embed_fwd_indexed(const dl_emb_layout* L, const float* rows, const float* rows_first,
                         const int32_t* inv, int32_t inv_base, const float* cont,
                         const float* vector, float* x0, float* fm_out, float* fm_sum,
                         void* stream);
/* Staged forward, after dl_rec_gather_scatter: the FM sums per sample over the staging rows
 * fmst (cont fields: compact rows [0, C) x their values; cate field f of sample b: row
 * n_rep + b*S + f), the cont fields' first-order outputs from rows_first[0, C), x0's cont /
 * vector columns, and zeros for every reference without a row (inv < 0: the zero row) —
 * its FM row, first-order output or x0 columns; everything the gather scattered is left. */
int dl_pool_fwd_staged(const dl_emb_layout* L, const float* mst, const float* mst1, const int32_t* inv,
                       const int32_t* slot_start, const int32_t* slot_end, int32_t n_slots, int32_t fm_col,
                       float* x0, float* fm_out, float* cnt_emb, float* cnt_first, void* stream);
/* dl_pool_fwd_indexed with multi position l of sample b read from the gather's multi-hot
 * staging rows mst[b * multi_width + l] (mst1 the first-order weights); positions without a
 * row (inv < 0: padding) count as none.  Same sums, same order. */
int dl_embed_fwd_staged(const dl_emb_layout* L, const float* fmst, const float* rows_first, const int32_t* inv,
                        int32_t n_rep, const float* cont, const float* vector, float* x0, float* fm_out,
                        float* fm_sum, void* stream);

/* Record forward (single GPU, lazy-exact Adam): dl_embed_fwd with the cate rows read
 * straight from the row records (rec.hip layout) and caught up to step opt[7] - lag in
 * registers (lag 1 in training, 0 for predict), instead of dl_rec_gather writing the
 * batch's unique rows and dl_embed_fwd_indexed reading them back.  The C FM cont-field
 * rows (every sample's) come compact and caught up in rows_rep / rows_rep1 (dl_rec_gather
 * with no unique rows); needs L->cont_rows_compact when there are any.  Outputs are
 * bit-identical to the gather + indexed pair.  Single-valued fields only (multi_width 0). */
int dl_embed_fwd_rec(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                     const float* rows_rep, const float* rows_rep1, const int64_t* cate,
                     const float* cont, const float* vector, const float* hist, int32_t hist_len,
                     const float* opt, int32_t lag, float* x0, float* fm_out, float* fm_sum,
                     int32_t* err, void* stream);
/* The record forward on a flushed table (every row caught up to step opt[7]: after
 * dl_rec_flush, before any further update): the plain lookup — each reference reads only its
 * record's first 128-B line (p, and the first-order weight beside it); a row whose stamp is not
 * opt[7] sets DL_STATUS_LAG (the host raises) instead of being read stale.  Same outputs as
 * dl_embed_fwd_rec at lag 0.  rows_rep / rows_rep1: the C FM cont-field rows, compact. */
int dl_embed_fwd_rec_flat(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                          const float* rows_rep, const float* rows_rep1, const int64_t* cate,
                          const float* cont, const float* vector, const float* opt, float* x0,
                          float* fm_out, float* fm_sum, int32_t* err, void* stream);

/* Hot cont-field rows only (the FM cont part of dl_embed_bwd): per-block
 * partials into cont_slab[0 .. min(cont_slab_blocks, dl_embed_bwd_grid)), folded in by
 * dl_embed_cont_reduce (blocks beyond the samples' share hold zeros, so passing only the
 * blocks that hold samples gives the same partials). */
int dl_embed_cont_bwd(const dl_emb_layout* L, const float* table, const float* cont,
                      const float* dz, const float* w_head, const float* fm_sum, float* cont_slab,
                      int32_t cont_slab_blocks, void* stream);

/* Batch reference index (index.hip): every (sample, slot) reference — slots are
 * the S FM cate fields (if use_fm) then the S deep fields — keyed by
 * (owner << 27 | local) with owner = row % world, local = row / world (rows below
 * replicated_below: owner = world, local = row); sorted (radix), deduplicated:
 * uniq_keys[0..n_uniq), segment offsets seg_off[0..n_uniq] into sorted_refs
 * (ref = b * n_slot + slot), inverse map inv[ref] -> unique id (-1 invalid; may be
 * NULL), owner_counts[world+1] unique rows per owner (may be NULL).
 * Invalid refs (row 0 under zero_row0, out-of-range -> err) are excluded. */
int64_t dl_index_workspace_bytes(int64_t n_refs);
int dl_index_build(const dl_emb_layout* L, const int64_t* cate, int32_t world,
                   int32_t replicated_below, void* ws, int64_t ws_bytes, uint32_t* sorted_keys,
                   int32_t* sorted_refs, uint32_t* uniq_keys, int32_t* seg_off, int32_t* n_uniq,
                   int32_t* inv, int32_t* owner_counts, int32_t* err, void* stream);
/* Two id sets indexed by ONE sort (single GPU, world 1): the table references of (L, cate) and
 * a second set (L2, cate2: the wdl wide ids, wdl.py:44-47 / :132 read wdl_weights through
 * embedding_lookup) keyed into owner groups 0 and 1 of one radix sort + segmented unique —
 * one launch sequence over n1 + n2 references in place of two builds over n1 and n2.
 * Outputs are exactly dl_index_build(L, cate, 1, 0, ...)'s for the first set (uniq_keys,
 * seg_off, n_uniq, inv; sorted_refs within its segments) and dl_index_build(L2, cate2, ...)'s
 * for the second (uniq2, seg_off2, n_uniq2, inv2, sorted_refs2), references numbered per set.
 * sorted_keys / sorted_refs / inv / uniq_keys / seg_off hold n1 + n2 (+1) entries; the second
 * set's arrays n2 (+1).  Workspace: dl_index_workspace_bytes(n1 + n2). */
int dl_index_build_pair(const dl_emb_layout* L, const int64_t* cate, const dl_emb_layout* L2,
                        const int64_t* cate2, void* ws, int64_t ws_bytes, uint32_t* sorted_keys,
                        int32_t* sorted_refs, uint32_t* uniq_keys, int32_t* seg_off, int32_t* n_uniq,
                        int32_t* inv, uint32_t* uniq2, int32_t* sorted_refs2, int32_t* seg_off2,
                        int32_t* n_uniq2, int32_t* inv2, int32_t* err, void* stream);
/* Generic form for the sharded owners: sort n int32 keys (< 2^key_bits; a key of -1 — an empty
 * slot of a fixed-capacity exchange block — is dropped) with their positions, dedup:
 * uniq_keys [n_uniq], seg_off [n_uniq+1] into sorted_pos, and inv[i] = unique id of keys[i]
 * (may be NULL).  Workspace: dl_index_workspace_bytes(n). */
int dl_sort_unique(const int32_t* keys, int64_t n_keys, int32_t key_bits, void* ws, int64_t ws_bytes,
                   int32_t* sorted_keys, int32_t* sorted_pos, int32_t* uniq_keys, int32_t* seg_off,
                   int32_t* n_uniq, int32_t* inv, void* stream);
/* Deterministic (atomic-free) embedding backward over the index: each unique
 * row's gradient is the ordered sum of its references.  compact=0: plain stores
 * into the dense gradient tables g_out [n_rows, E] / g1_out [n_rows] + touched
 * flags (single GPU); compact=1: g_out [u][E], g1_out [u] per unique id (the
 * sharded path sends these to the owners).  rows_u: gathered rows per unique id
 * (sharded) or NULL to read `table`.  upos (compact only, may be NULL): unique row u's slot in
 * rows_u / g_out / g1_out (the fixed-capacity exchange blocks of dl_shard_route; a slot of -1
 * is skipped) in place of u. */
int dl_embed_bwd_sorted(const dl_emb_layout* L, const float* table, const float* rows_u,
                        const uint32_t* uniq_keys, const int32_t* seg_off, const int32_t* n_uniq,
                        const int32_t* sorted_refs, int32_t world, int64_t max_uniq,
                        const float* dz, const float* w_head, const float* fm_sum,
                        const float* dx0, float* g_out, float* g1_out, uint8_t* touched,
                        int32_t compact, const int32_t* upos, void* stream);

/* Multi-hot nonzero-mean pooling (deepfm_multi_cate.py:71-111).
 * ids [B, ids_ld] int64 (padding id 0); slot m covers columns
 * [slot_start[m], slot_end[m]) of the multi-hot block that starts at column
 * ids_col.  Writes pooled vectors to x0[b][x0_pool_col + m*E ..], pooled
 * first-order to fm_out[b][fm_col + m] (if first_order != NULL) and the
 * integer counts cnt_emb / cnt_first [B, M] (float-valued, bit-exact). */
int dl_pool_fwd(const dl_emb_layout* L, const float* table, const float* first_order,
                const int64_t* ids, int32_t ids_col, const int32_t* slot_start,
                const int32_t* slot_end, int32_t n_slots, int32_t fm_col, float* x0,
                float* fm_out, float* cnt_emb, float* cnt_first, int32_t* err, void* stream);
/* Pooling over record rows (lazy Adam, L->multi_width > 0): the row of multi position l
 * of sample b is inv_base + inv[b*ns + (use_fm ? S : 0) + S + l] of rows/rows_first
 * (dl_rec_gather output, dl_index_build inv; -1 = padding id). */
int dl_pool_fwd_indexed(const dl_emb_layout* L, const float* rows, const float* rows_first,
                        const int32_t* inv, int32_t inv_base, const int32_t* slot_start,
                        const int32_t* slot_end, int32_t n_slots, int32_t fm_col, float* x0,
                        float* fm_out, float* cnt_emb, float* cnt_first, void* stream);
/* Backward of pooling: d pooled = dsecond*(fm_sum - pooled) + dx0[pool cols];
 * each slot id gets d/cnt (div_no_nan gradient), first-order likewise. */
int dl_pool_bwd(const dl_emb_layout* L, const int64_t* ids, int32_t ids_col,
                const int32_t* slot_start, const int32_t* slot_end, int32_t n_slots,
                int32_t fm_col, const float* x0, const float* fm_sum, const float* dz,
                const float* w_head, const float* dx0, int32_t dx0_pool_col,
                const float* cnt_emb, const float* cnt_first, float* g_table,
                float* g_first, uint8_t* touched, void* stream);
/* Weighted nonzero-mean pooling (models/dnn_multi_textline.py:94-103, the deep-only
 * multi-hot lookup of the textline DNN): pooled = div_no_nan(sum_l value_l * V[id_l], cnt)
 * with cnt = count_nonzero(sum_E V[id_l]) of the UNweighted rows (:94-95).  values [B,
 * values_ld] f32, the value of multi position l (same column numbering as the slot ranges,
 * relative to ids_col).  The frozen word2vec table of slot 'tag' (:45-47,85-88) is a
 * separate dl_pool_fwd_weighted call with that table and no backward.  The backward
 * scatter-adds value_l * d pooled / cnt into g_table (f32 atomics) and marks touched. */
int dl_pool_fwd_weighted(const dl_emb_layout* L, const float* table, const int64_t* ids,
                         int32_t ids_col, const float* values, int32_t values_ld,
                         const int32_t* slot_start, const int32_t* slot_end, int32_t n_slots,
                         float* x0, float* cnt_emb, int32_t* err, void* stream);
int dl_pool_bwd_weighted(const dl_emb_layout* L, const int64_t* ids, int32_t ids_col,
                         const float* values, int32_t values_ld, const int32_t* slot_start,
                         const int32_t* slot_end, int32_t n_slots, const float* dx0,
                         int32_t dx0_pool_col, const float* cnt_emb, float* g_table,
                         uint8_t* touched, void* stream);

/* ------------------------------------------------------------------------
 * Dense tower: fp32 GEMM on v_mfma_f32_16x16x4_f32 (exact fp32, k-ordered fma).
 * C[i][j] (op) sum_r A(i,r) B(r,j); A(i,r) = ta ? A[r*lda+i] : A[i*lda+r];
 * B(r,j) = tb ? B[j*ldb+r] : B[r*ldb+j].
 * epi: 0 store, 1 ReLU (bias folded as a ones column), 2 multiply by
 * (mask[i*ldm+j] > 0) (ReluGrad), 3 split-K partial slabs:
 * C + z*c_split_stride for split z of `splits` (K chunks of a multiple of 16).
 * Requirements: lda, ldb, ldc multiples of 4; the contiguous extent of each
 * operand a multiple of 4 (zero padded). Replaces MatMul+Add+Relu
 * (deepfm_pipeline.py:150-152) and their gradients. */
int dl_gemm_f32(int32_t ta, int32_t tb, int32_t M, int32_t N, int32_t K, const float* A,
                int32_t lda, const float* B, int32_t ldb, float* C, int32_t ldc, int32_t epi,
                const float* mask, int32_t ldm, int32_t splits, int64_t c_split_stride,
                void* stream);
/* dst[c*ldd + r] = src[r*lds + c] (r < rows, c < cols): W^T for the dX product, so
 * both dX operands are read from LDS images in their HBM layout. */
int dl_transpose_f32(const float* src, int32_t rows, int32_t cols, int32_t lds, float* dst, int32_t ldd,
                     void* stream);
/* dst[r*ldd + c] = bf16(src[r*lds + c]), round to nearest even (bf16 tower operands). */
int dl_cast_bf16(const float* src, int32_t rows, int32_t cols, int32_t lds, uint16_t* dst, int32_t ldd,
                 void* stream);
/* dst[c*ldd + r] = bf16(src[r*lds + c]) (src f32 when src_f32, else bf16): the k-contiguous
 * operand copies of the bf16 tower (W^T, X^T, dY^T). */
int dl_transpose_bf16(const void* src, int32_t src_f32, int32_t rows, int32_t cols, int32_t lds,
                      uint16_t* dst, int32_t ldd, void* stream);
/* bf16 variant for the Wide&Deep tower (config C5): A, B bf16 (uint16 bits),
 * fp32 accumulate, C fp32 or bf16 (c_bf16 = 1). Same semantics otherwise.  ta = 0, tb = 1
 * with lda, ldb multiples of 8 and 16-B aligned operands takes the fast k-contiguous
 * kernel (b128 LDS images, BK = 64); other forms a general element-staged kernel. */
int dl_gemm_bf16(int32_t ta, int32_t tb, int32_t M, int32_t N, int32_t K, const uint16_t* A,
                 int32_t lda, const uint16_t* B, int32_t ldb, void* C, int32_t ldc,
                 int32_t c_bf16, int32_t epi, const void* mask, int32_t ldm, int32_t splits,
                 int64_t c_split_stride, void* stream);

/* fp32 tower products on the bf16 matrix cores, three-plane split (gemm_s3.hip):
 * every f32 operand splits exactly into bf16 planes hi + mid + lo and a product takes the
 * six significant plane products (hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi) in f32
 * accumulation: f32 accuracy (dropped terms <= 2^-25 |a.b|) at up to 2.7x the f32 MFMA rate.
 * Replaces dl_gemm_f32 for deepfm_pipeline.py:150-152 and its gradients.
 *
 * dl_split3: planes of src [rows][cols] (ld lds) at dst + q * plane_stride (q = 0 hi,
 *   1 mid, 2 lo), [r][c] with ld ldd, or [c][r] when `transpose`.  In a library built with
 *   DL_S3_KPERM (dl_s3_kperm() == 1) the k index (the row position: c, or r when transposed;
 *   K = cols, or rows) of every whole 32-deep chunk is stored permuted — position
 *   8q + j (j < 4) holds k = 4q + j, position 8q + 4 + j holds k = 16 + 4q + j — the order
 *   dl_gemm_s3_nt reads; a trailing partial chunk keeps natural order.
 * dl_gemm_s3_nt: C[M][N] = A[M][K] . B[N][K]^T (+ epilogue: 0 store, 1 ReLU, 2 mask
 *   (C = mask[i][j] > 0 ? C : 0, mask f32 with ld ldm)); A f32 (lda % 4 == 0, 16-B
 *   aligned), B as planes from dl_split3 (ldb % 8 == 0, plane stride b_plane); K % 8 == 0.
 * dl_gemm_s3_tn: split-K weight gradient, slab z of C (at C + z * c_split_stride, ld ldc)
 *   = sum over k in split z of X[k][m] Y[k][n]; X [K][lda], Y [K][ldb] f32, N <= 416;
 *   splits of ceil(K / splits) rounded up to 64 rows (ceil(K / that) slabs). */
int dl_split3(const float* src, int32_t rows, int32_t cols, int32_t lds, int32_t transpose, uint16_t* dst,
              int32_t ldd, int64_t plane_stride, void* stream);
int dl_s3_kperm(void);
int dl_gemm_s3_nt(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const uint16_t* B,
                  int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi, const float* mask,
                  int32_t ldm, void* stream);
int dl_gemm_s3_tn(int32_t M, int32_t N, int32_t K, const float* X, int32_t lda, const float* Y, int32_t ldb,
                  float* C, int32_t ldc, int32_t splits, int64_t c_split_stride, void* stream);
/* dl_gemm_s3_nt_bits: dl_gemm_s3_nt with the ReLU sign bitmask — bits [M][ldbits] uint16,
 * bit (c & 15) of halfword [i][c >> 4] = (C[i][c] > 0), ldbits >= ceil(N / 16).  epi 1 (ReLU)
 * also writes the bitmask when bits != NULL; epi 3 applies the ReluGrad mask from it
 * (C = bit ? C : 0) in place of epi 2's f32 mask rows: 2 bytes per 16 columns read instead of
 * 64 (the tower's dX, deepfm_pipeline.py:150-152 gradients). */
int dl_gemm_s3_nt_bits(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const uint16_t* B,
                       int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi, const float* mask,
                       int32_t ldm, uint16_t* bits, int32_t ldbits, void* stream);
/* dl_gemm_s3_nt_gather: dl_gemm_s3_nt_bits (epi 0 / 1) for the first tower layer of the
 * flushed-table forward with the embedding lookup fused into its A stream (the north star's
 * "gather into tiles feeding MFMA"; replaces the GatherV2 -> ConcatV2 -> MatMul chain of
 * deepfm_pipeline.py:117-153 / dnn_pipeline.py:72-96 at predict): columns [0, fields * emb_dim)
 * of A's row m are not read from A but from table row (ids[m * ids_ld + f] + id_offset) —
 * f = k / emb_dim, column k % emb_dim, table rows table_ld floats apart (the slot or p plane
 * of dl_rec_flush) — a row outside [0, n_rows), or row 0 with zero_row0, reads as zeros (the
 * lookup's zero row; the lookup itself reports invalid ids).  The remaining columns come from A
 * (the cont / vector / bias columns the lookup writes with x0_cat_col = -1).  Bit-identical
 * to dl_embed_fwd(_slots) writing those columns followed by dl_gemm_s3_nt_bits.  Requires
 * emb_dim in {8, 16, 32, 64}, fields * emb_dim a multiple of 32 and <= K, fields <= 40,
 * n_rows * table_ld * 4 < 0xFFFFFF00 bytes (one buffer range). */
int dl_gemm_s3_nt_gather(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const float* table,
                         int64_t n_rows, int32_t table_ld, const int64_t* ids, int32_t ids_ld, int64_t id_offset,
                         int32_t zero_row0, int32_t fields, int32_t emb_dim, const uint16_t* B, int32_t ldb,
                         int64_t b_plane, float* C, int32_t ldc, int32_t epi, uint16_t* bits, int32_t ldbits,
                         void* stream);
/* dl_gemm_s3_nt_gather_rows: the training form — the deep rows of the batch's compact caught-up
 * rows (dl_rec_gather's rows_u) through the batch index's inverse map: row idx_base + idx[m *
 * idx_ld + f] (idx < 0: the zero row), and the gathered columns also written into A (x0) by the
 * first column tile's blocks, for the weight gradient that streams x0 (the lookup then runs with
 * x0_cat_col = -1).  Bit-identical to dl_embed_fwd_indexed writing those columns followed by
 * dl_gemm_s3_nt_bits. */
int dl_gemm_s3_nt_gather_rows(int32_t M, int32_t N, int32_t K, float* A, int32_t lda, const float* rows,
                              int64_t n_rows, int32_t rows_ld, const int32_t* idx, int32_t idx_ld, int32_t idx_base,
                              int32_t fields, int32_t emb_dim, const uint16_t* B, int32_t ldb, int64_t b_plane,
                              float* C, int32_t ldc, int32_t epi, uint16_t* bits, int32_t ldbits, void* stream);
/* dl_gemm_s3_nt_gather_tab: dl_gemm_s3_nt_gather with the rows resolved beforehand — the deep
 * rows' byte offsets come in gtab (dl_embed_fwd_gtab's table, staged into the block's LDS as it
 * stands, one contiguous copy instead of the ids' loads and range checks: entry
 * [m / 256][f * 272 + m % 256], 0xFFFFFF00 = a zero row); A's other columns from A (x0 with its
 * cont / ones columns written).  Bit-identical to dl_embed_fwd(_slots) + dl_gemm_s3_nt_bits
 * and to dl_gemm_s3_nt_gather.  gtab holds ceil(M / 256) * fields * 272 u32, 16-B aligned. */
int dl_gemm_s3_nt_gather_tab(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const float* table,
                             int64_t n_rows, int32_t table_ld, const uint32_t* gtab, int32_t fields, int32_t emb_dim,
                             const uint16_t* B, int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi,
                             uint16_t* bits, int32_t ldbits, void* stream);

/* ------------------------------------------------------------------------
 * Output layer + sigmoid + eps-log-loss, forward and backward fused
 * (deepfm_pipeline.py:157-183, dnn_pipeline.py:119-131):
 * z = [fm_out(F+E) | h(H)] . w + w[F+E+H];  p = sigmoid(z);
 * loss_b = -y ln(p+eps) - (1-y) ln(1-p+eps);  dz = (dL/dp) p (1-p) / B;
 * dh = dz * w_h * (h > 0) written into dh [B, ldh] (cols < H);
 * per-block partials: slab[block][0..F+E+H) = sum dz*feat, [F+E+H] = sum dz,
 * [F+E+H+1] = sum loss_b.  `fm_cols` = F+E (0 for dnn). inv_batch = 1/B_global. */
int dl_head_fwd_bwd(int32_t B, int32_t fm_cols, int32_t H, const float* fm_out, int32_t fm_ld,
                    const float* h, int32_t ldh, const float* w, const float* label,
                    float eps, float inv_batch, float* score, float* z_out, float* dz,
                    float* dh, float* slab, int32_t slab_blocks, void* stream);
int dl_head_grid(int32_t B);
/* Blocks (= slab rows) of dl_wdl_head_fwd_bwd[_bf16] for batch B. */
int dl_wdl_head_grid(int32_t B);

/* Wide&Deep cross logit, forward and backward fused (models/wdl.py:225-275):
 * z = sum_f w[wide_f] + sum_j w[Fw+j] h_j + bias[0] (w = wdl_weights [w_rows]; the
 * deep-output rows Fw..Fw+H alias wide ids); sigmoid + eps-log-loss as dl_head_fwd_bwd.
 * Wide-row gradients dz are added to g_w (int64 fixed point, units 1/DL_WIDE_GRAD_SCALE:
 * integer atomics, so the segment sum is deterministic) (+ touched); the dense part leaves
 * slab[block][0..H) = sum dz*h, [H] = sum dz, [H+1] = sum loss (fold with
 * dl_slab_fold_rows into g_w rows Fw..Fw+H).  g_w = NULL: forward only (predict). */
int dl_wdl_head_fwd_bwd(int32_t B, int32_t Fw, int32_t H, const int64_t* wide, int32_t wide_ld,
                        const float* h, int32_t ldh, const float* w, const float* bias, int64_t w_rows,
                        const float* label, float eps, float inv_batch, float* score, float* z_out,
                        float* dz, float* dh, int64_t* g_w, uint8_t* touched, float* slab,
                        int32_t slab_blocks, int32_t* err, void* stream);
/* As dl_wdl_head_fwd_bwd with dh written as bf16 (round-to-nearest-even): the bf16
 * tower's dY operand (config C5), 8-B aligned, same leading dimension ldh as h. */
int dl_wdl_head_fwd_bwd_bf16(int32_t B, int32_t Fw, int32_t H, const int64_t* wide, int32_t wide_ld,
                             const float* h, int32_t ldh, const float* w, const float* bias, int64_t w_rows,
                             const float* label, float eps, float inv_batch, float* score, float* z_out,
                             float* dz, uint16_t* dh, int64_t* g_w, uint8_t* touched, float* slab,
                             int32_t slab_blocks, int32_t* err, void* stream);
/* g[row0+j] += sum over `blocks` slab rows of slab[blk*width + col0 + j], j < n, as int64
 * fixed point (units 1/DL_WIDE_GRAD_SCALE, the wide gradient's form). */
int dl_slab_fold_rows(const float* slab, int32_t blocks, int32_t width, int32_t col0, int32_t n,
                      int64_t* g, int64_t row0, uint8_t* touched, void* stream);

/* ------------------------------------------------------------------------
 * TF1 Adam (training_ops.cc ApplyAdam, dense semantics: every element's m, v
 * decay each step — SURVEY.md ledger item 6).  `opt` is a device float[16]:
 * [0] beta1_power [1] beta2_power [2] lr [3] alpha [4] beta1 [5] beta2
 * [6] epsilon [7] step (as float, exact < 2^24), [8..15] per-step accumulators
 * (zeroed by dl_adam_begin_step; [8..9] = opt + DL_OPT_REG is the step's regulariser sum as
 * int64 fixed point, the sq_out / acc_out target), [16] the status word (int32
 * bits, sticky until the host clears it: what the host reports), [17] the skip
 * word (int32 bits of the CURRENT step only, rewritten by dl_step_guard /
 * dl_step_begin), [18] the global step at which the last bad batch was skipped,
 * [19] how many batches were skipped since the host last cleared the status;
 * DL_OPT_LEN floats in all.
 * dl_adam_begin_step computes alpha = lr_t*sqrt(1-b2p)/(1-b1p) with
 * lr_t = lr*rate^floor(step/decay_steps) and then advances b1p*=b1, b2p*=b2,
 * step+=1 (TF's _finish + global_step).
 *
 * A nonzero SKIP word poisons the step: dl_adam_begin_step and every call that
 * writes parameters or Adam state (dl_adam_*, dl_rec_bwd_adam, dl_rec_apply_*)
 * return without writing them; gradient buffers they would consume are still
 * reset.  A batch whose ids fail validation therefore changes nothing, as TF's
 * failing sess.run applies nothing before raising InvalidArgumentError
 * (deepfm_pipeline.py:219-221), and the next batch applies normally (the skip word
 * belongs to one step); the host reads the sticky status word back and raises.
 * Internal faults (DL_STATUS_LAG / DL_STATUS_INDEX) set both words and keep every
 * later step skipped until the host clears the status. */
#define DL_OPT_LEN 32
#define DL_OPT_REG 8        /* int64 fixed point (units 1/DL_REG_SUM_SCALE) in opt[8..9]: the step's regulariser sum */
/* Regulariser sums (every sq_out / acc_out / sq_untouched below) are signed 64-bit fixed point
 * in units of 1/DL_REG_SUM_SCALE, 8-byte aligned: each block adds its fixed-order partial as an
 * integer, so the sum is the same bits whatever order the blocks land in (|sum| < 2^31). */
#define DL_REG_SUM_SCALE 4294967296.0 /* 2^32 */
#define DL_OPT_STATUS 16
#define DL_OPT_SKIP 17
#define DL_OPT_BAD_STEP 18
#define DL_OPT_BAD_COUNT 19
#define DL_OPT_SEQ 20       /* int32 bits: steps reported through dl_loss_accumulate's status ring */
#define DL_OPT_BAD_RANKS 21 /* int32 bits: sharded step — bit p set when rank p's batch held a bad id */
#define DL_STATUS_BAD_ID 1   /* a categorical / wide id outside [0, N) */
#define DL_STATUS_LAG 2      /* a row record lagged past the alpha ring (flush schedule broken) */
#define DL_STATUS_INDEX 4    /* a batch-index entry out of range (index consumers report, never skip silently) */
#define DL_STATUS_OVERFLOW 8 /* sharded step: a rank had more unique rows for an owner than a block holds */
#define DL_STATUS_DESYNC 16  /* sharded step: the ranks' headers named different global steps */
int dl_adam_begin_step(float* opt, float decay_rate, float decay_steps, void* stream);
/* The step's skip word := the batch's validation bits (batch_err[0], written by
 * dl_index_build / dl_validate_batch) | the sticky internal-fault bits; a bad batch
 * also sets opt[DL_OPT_STATUS], records the global step it was skipped at and counts
 * itself.  Issued before dl_adam_begin_step so the step of a bad batch is poisoned
 * from its start. */
int dl_step_guard(const int32_t* batch_err, float* opt, void* stream);
/* The batch's id-validation word, before its step begins: reset != 0 zeroes err[0] first
 * (one word per batch, not sticky); then every cate id (cate non-NULL, [L->batch][L->cate_ld]:
 * single columns against their deep row id + deep_cate_offset and, with FM, their FM row
 * id + fm_cate_offset; multi-hot columns against id + deep_cate_offset, all in [0, n_rows))
 * and every wide id (wide non-NULL, [batch][wide_ld], first wide_cols: [0, wide_rows)) sets
 * DL_STATUS_BAD_ID in err[0] if out of range.  For the batches no dl_index_build validates
 * (dense-layout gathers) and wdl's wide ids (models/wdl.py:225-228). */
int dl_validate_batch(const dl_emb_layout* L, const int64_t* cate, const int64_t* wide, int32_t wide_cols,
                      int32_t wide_ld, int64_t wide_rows, int32_t reset, int32_t* err, void* stream);
/* dl_step_guard, dl_adam_begin_step and (hist non-NULL) dl_adam_hist_record in one
 * launch, same operations in the same order: the step's opening graph node. */
int dl_step_begin(const int32_t* batch_err, float* opt, float decay_rate, float decay_steps, float* hist,
                  int32_t hist_len, void* stream);
/* The running loss of a training loop (the load-style fit's per-epoch mean, wdl.py:305-313):
 * acc[0] += sum_r slab[r * pitch + col] * inv_b (the step's data term; double, fixed order),
 * acc[1] += reg_coef * the step's regulariser sum (opt + DL_OPT_REG), acc[2] += 1; nothing for a skipped
 * step.  acc: double[3] on the device, read by the host once per epoch.  (Wide&Deep with lazy
 * wide records adds the wide L2 term per record step through dl_wide_rec_update / _flush acc.)
 * status_ring (may be NULL): int32[8] of pinned host memory; every call (skipped steps too)
 * advances the step sequence opt[DL_OPT_SEQ] to k and writes k to ring[2(k & 3)] and the status
 * word to ring[2(k & 3) + 1] in one 8-byte store: the host's per-step status report without a
 * device-to-host copy. */
int dl_loss_accumulate(const float* slab, int32_t rows, int32_t pitch, int32_t col, double inv_b, float* opt,
                       float reg_coef, double* acc, int32_t* status_ring, void* stream);
/* Dense parameter whose gradient is the sum of `nslab` partial slabs
 * (g = sum_s slab[s*slab_stride + i]); l2 * p is added for i < l2_count;
 * p_prev (may be NULL) receives the pre-update values; sq_out (may be NULL, int64 fixed
 * point, DL_REG_SUM_SCALE) gets sum p_pre^2 over the L2-regularised elements added — the
 * loss's l2_regularizer term of the step, read back without copying the parameters. */
/* dl_adam_dense_split3: dl_adam_dense_reg on a tower weight W [rows][cols] (n = rows * cols,
 * no p_prev) that also writes the updated W's three bf16 planes in dl_split3's two layouts —
 * wp[q][r][c] and wtp[q][c][r], plane stride rows * cols — in place of two dl_split3 launches
 * after the update (the s3 GEMMs' operands; deepfm_pipeline.py:184-188 ApplyAdam on W). */
int dl_adam_dense_split3(float* p, float* m, float* v, const float* slab, int32_t nslab, int64_t slab_stride,
                         int32_t rows, int32_t cols, float reg, int64_t reg_count, int32_t reg_kind, const float* opt,
                         int64_t* acc_out, uint16_t* wp, uint16_t* wtp, void* stream);
/* dl_adam_dense_bf16: the same for the bf16 tower (C5): the updated W's bf16 copy wb [rows][cols]
 * and its transpose wbt [cols][rows] (dl_cast_bf16 / dl_transpose_bf16's rounding). */
int dl_adam_dense_bf16(float* p, float* m, float* v, const float* slab, int32_t nslab, int64_t slab_stride,
                       int32_t rows, int32_t cols, float reg, int64_t reg_count, int32_t reg_kind, const float* opt,
                       int64_t* acc_out, uint16_t* wb, uint16_t* wbt, void* stream);
int dl_adam_dense(float* p, float* m, float* v, const float* slab, int32_t nslab,
                  int64_t slab_stride, int64_t n, float l2, int64_t l2_count, const float* opt,
                  float* p_prev, int64_t* sq_out, void* stream);
/* One tower weight's update for dl_adam_dense_layers: W [rows][cols] (p, m, v), its gradient as
 * `nslab` partial slabs `slab_stride` floats apart, the regulariser (reg_kind 0 = L2, 1 = L1) on
 * the first reg_count elements with its loss term added to *acc_out (may be NULL), and the
 * operand copies wp / wtp the update writes (dl_adam_dense_split3 / dl_adam_dense_bf16). */
typedef struct dl_adam_layer {
  float* p;
  float* m;
  float* v;
  const float* slab;
  int64_t slab_stride;
  int64_t reg_count;
  int64_t* acc_out;
  uint16_t* wp;
  uint16_t* wtp;
  int32_t nslab;
  int32_t rows, cols;
  int32_t reg_kind;
  float reg;
  int32_t pad_;
} dl_adam_layer;
/* dl_adam_dense_layers: dl_adam_dense_split3 (copies = 3) or dl_adam_dense_bf16 (copies = 1) on
 * up to DL_ADAM_MAX_LAYERS tower weights in one launch — the same per-element operations, so the
 * same results as one launch per layer (the regulariser sum: the same total, other block
 * partials).  One launch instead of one per hidden layer at the end of the backward. */
#define DL_ADAM_MAX_LAYERS 4
int dl_adam_dense_layers(int32_t n_layers, const dl_adam_layer* layers, int32_t copies, const float* opt,
                         void* stream);
/* dl_adam_dense with the regulariser kind explicit: reg_kind 0 = L2 as above, 1 = L1
 * (tf.contrib.layers.l1_regularizer at models/dnn.py:88-90: g += reg * sign(p) for
 * i < reg_count, acc_out += |p_pre|). */
int dl_adam_dense_reg(float* p, float* m, float* v, const float* slab, int32_t nslab,
                      int64_t slab_stride, int64_t n, float reg, int64_t reg_count, int32_t reg_kind,
                      const float* opt, float* p_prev, int64_t* acc_out, void* stream);
/* Embedding tables, every row updated: g = g_table row if touched else 0;
 * consumed gradients are reset to 0.  rows_flags: DL_ROWS_CLEAR_TOUCHED resets the
 * flags (on the last table that shares them); DL_ROWS_SPARSE_ADAM selects the update
 * TF applies to a Variable read by embedding_lookup directly (Adam._apply_sparse_shared:
 * m = m*b1 + g*(1-b1), v = v*b2 + (g*g)*(1-b2), p -= lr*m/(sqrt(v)+eps); wdl.py:44-47,132,
 * deepfm.py:57-60, dnn.py:49-54), else ApplyAdam's (the pipeline models' tables, whose
 * gradient is densified by the row-0 concat, deepfm_pipeline.py:83-86).
 * width = E (table) or 1 (first-order).  DL_ROWS_GRAD_FIXED (width 1): g is int64 fixed
 * point in units of 1/DL_WIDE_GRAD_SCALE (the wdl wide-weight gradient of
 * dl_wdl_head_fwd_bwd / dl_slab_fold_rows).
 * State form: `v` holds the ROOT state s = sqrt(v) for the embedding tables (every call
 * without DL_ROWS_GRAD_FIXED) — the form the row records keep, so the g = 0 step is
 * s' = s*sqrt(b2) (one reciprocal, no square root); a g != 0 step forms v = s*s, applies
 * the update above and stores sqrt(v').  With DL_ROWS_GRAD_FIXED (the wdl wide weights)
 * `v` is TF's v.  Callers convert at the boundary (engine.py adam_state / set_adam_state). */
#define DL_ROWS_CLEAR_TOUCHED 1
#define DL_ROWS_SPARSE_ADAM 2
#define DL_ROWS_GRAD_FIXED 4
#define DL_WIDE_GRAD_SCALE 281474976710656.0 /* 2^48 */
int dl_adam_rows(float* p, float* m, float* v, void* g, uint8_t* touched, int64_t n_rows,
                 int32_t width, float l2, int32_t rows_flags, const float* opt, int64_t* sq_out,
                 void* stream);

/* ------------------------------------------------------------------------
 * Lazy-exact Adam on interleaved row records (rec.hip).  Same result as the
 * dense sweep of dl_adam_rows (bit-identical: the skipped zero-gradient steps
 * are replayed with the same float operations when a row is next read), but a
 * step only touches the rows its batch references.  Record of rec_ld floats
 * (rec_ld >= 3E+4, multiple of 32): [p(E) | w1 m1 s1 stamp | m(E) | s(E) | pad],
 * s = sqrt(v) (the root state of dl_adam_rows); stamp = int32 bits of the last step applied.  hist = ring of hist_len (power
 * of two) per-step alphas; the caller keeps every row's lag < hist_len by
 * calling dl_rec_flush at least once per hist_len steps.
 * Replaces, for the table and first-order Variables, the dense ApplyAdam of
 * deepfm_pipeline.py:184-188 / dnn_pipeline.py:132-136 and the sparse-apply Adam
 * of wdl.py:277-285 / deepfm.py:157-162 / dnn.py:92-93.
 * rec_flags: DL_REC_FIRST = the record carries a first-order weight (FM models);
 * DL_REC_SPARSE_ADAM = the table is updated in TF's sparse-apply form (see
 * dl_adam_rows), else ApplyAdam's.  The catch-up replays the same form. */
#define DL_REC_FIRST 1
#define DL_REC_SPARSE_ADAM 2
/* dl_rec_flush only: p_plane is a slot plane [n_rows][2E] — row r's p in columns 0..E-1 and its
 * first-order weight in column E (128-B slots for E = 16; columns E+1.. unwritten), w1_plane unused */
#define DL_REC_PLANE_SLOTS 4
/* hist[step & (hist_len-1)] = alpha of the step dl_adam_begin_step just began. */
int dl_adam_hist_record(const float* opt, float* hist, int32_t hist_len, void* stream);
/* rows_u[i] = p(row_i) caught up to step opt[7]-lag (rows_u1[i] = w1), row_i =
 * L->fm_cont_offset + i for i < n_rep (the replicated FM cont-field rows) else the row of uniq_keys[i-n_rep] (batch index,
 * dl_index_build keys; n_uniq = NULL: max_uniq keys, e.g. an owner's received local
 * rows with world = 1).  Records are only read.  mv_u (may be NULL) receives the
 * moment stash for dl_rec_bwd_adam / dl_rec_apply_segments, dl_rec_stash_floats(E) floats a row:
 * m(E) | m1 s1 lag 0 (the backward takes s from the record it rewrites, decayed over `lag`
 * zero-gradient steps: the same bits), or, in builds with DL_STASH_M=0, m(E) | s(E) | m1 s1 0 0.
 * lag = 1 inside a training step, 0 for predict. */
int32_t dl_rec_stash_floats(int32_t emb_dim);
int dl_rec_gather(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                  int32_t n_rep, const uint32_t* uniq_keys, const int32_t* n_uniq, int64_t max_uniq,
                  int32_t world, const float* hist, int32_t hist_len, const float* opt, int32_t lag,
                  float* rows_u, float* rows_u1, float* mv_u, void* stream);
/* dl_rec_gather (world 1, every output the same) that ALSO writes each caught-up row to the
 * references reading it, through the batch index's sorted segments (seg_off, sorted_refs of
 * dl_index_build): FM reference (b, f) -> fmst[n_rep + b*S + f][E] and fm_out[b][Cf + f] =
 * w1; deep reference (b, f) -> x0[b][x0_cat_col + f*E] (bf16 when L->x0_bf16); the
 * replicated rows -> fmst[0, n_rep).  Multi-hot reference (b, l) -> mst[b * multi_width + l][E]
 * and mst1[...] = w1 when mst is given (then dl_pool_fwd_staged pools them), else left to
 * the pooling kernels.
 * Random 64-B writes in place of dl_embed_fwd_indexed's random 64-B reads through the
 * inverse map (the forward of models/deepfm_pipeline.py:89-123 reorganised around the
 * batch's unique rows); follow with dl_embed_fwd_staged.  fmst: [n_rep + B*S][E]. */
int dl_rec_gather_scatter(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                          int32_t n_rep, const uint32_t* uniq_keys, const int32_t* n_uniq, int64_t max_uniq,
                          const int32_t* seg_off, const int32_t* sorted_refs, const float* hist, int32_t hist_len,
                          const float* opt, int32_t lag, float* rows_u, float* rows_u1, float* mv_u, float* fmst,
                          void* x0, float* fm_out, float* mst, float* mst1, void* stream);
/* Fused backward + Adam: per unique row the ordered segment sum of its references
 * (as dl_embed_bwd_sorted) is applied with step opt[7]'s alpha to the caught-up
 * state of dl_rec_gather (rows_u, rows_u1, mv_u — full arrays, replicated rows
 * first; mv_u = NULL: the record is re-read and its catch-up replayed, using
 * hist), and the record is written with stamp = step.  The replicated rows
 * (L->fm_cont_offset + j, j < n_rep) instead add their gradient into g_rep[j][E] /
 * g1_rep[j] (finished by dl_rec_apply_rows with row0 = L->fm_cont_offset). */
/* Multi-hot pooling state for dl_rec_bwd_adam (deepfm_multi_cate.py:71-111): slot ranges
 * within the multi block, the head column of the pooled first-order outputs, dx0's pooled
 * columns, the pooled x0 (L->x0_pool_col), the nonzero counts of dl_pool_fwd_indexed and
 * scratch g_pool [B][n_slots][E], g1_pool [B][n_slots] for the per-slot gradients.
 * g_pitch > 0 (>= E + 1, a multiple of 4): row (b, m) of g_pool at g_pool + (b*n_slots + m)*g_pitch
 * and its first-order gradient at g1_pool[(b*n_slots + m)*g_pitch] — with g1_pool = g_pool + E
 * and g_pitch = 32 (E = 16) both sit in one 128-B line, so a multi-hot reference's gradient
 * costs one line fetch instead of two; g_pitch = 0: the packed layouts above. */
typedef struct dl_pool_desc {
  const int32_t* slot_start;
  const int32_t* slot_end;
  int32_t n_slots;
  int32_t fm_col;
  int32_t dx0_pool_col;
  int32_t g_pitch;
  const float* x0;
  const float* cnt_emb;
  const float* cnt_first;
  float* g_pool;
  float* g1_pool;
} dl_pool_desc;
/* pool: required when L->multi_width > 0 (multi refs add (dp/cnt) to the row gradient
 * and dz*w_head[fm_col+m]/cnt_first to the first-order one), else may be NULL.
 * hot_ws (may be NULL; dl_rec_bwd_workspace_bytes(batch * index slots, E) bytes, 16-B aligned):
 * the rows with more than 32 references (Zipf-hot ids) are summed in chunks of 1,024
 * references spread over the whole grid, the chunk sums added in chunk order — the same
 * canonical sum as the single-block pass used without it (and by dl_embed_bwd_sorted). */
int dl_rec_bwd_adam(const dl_emb_layout* L, float* rec, int32_t rec_ld, int32_t rec_flags, int32_t n_rep,
                    const float* rows_u, const float* rows_u1, const float* mv_u,
                    const uint32_t* uniq_keys, const int32_t* seg_off, const int32_t* n_uniq,
                    const int32_t* sorted_refs, int32_t world, int64_t max_uniq, const float* dz,
                    const float* w_head, const float* fm_sum, const float* dx0, float* g_rep,
                    float* g1_rep, const float* hist, int32_t hist_len, const float* opt,
                    const dl_pool_desc* pool, void* hot_ws, int64_t hot_ws_bytes, void* stream);
int64_t dl_rec_bwd_workspace_bytes(int64_t nrefs, int32_t emb_dim);
/* Sharded owners without a sort: link every received position into its row's arrival
 * chain (head[local_rows] starts at -1; next[n]).  Then apply: one leader per row sums its
 * arrivals g[pos][E], g1[pos] in ascending position order (as dl_rec_apply_segments over a
 * stable sort), catches the record up and steps it; head is reset to -1 afterwards. */
int dl_rec_chain_link(const int32_t* ids, int64_t n, int32_t* head, int32_t* next, void* stream);
int dl_rec_apply_chain(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, const int32_t* ids,
                       int64_t n, int32_t* head, const int32_t* next, const float* g, const float* g1,
                       const float* hist, int32_t hist_len, const float* opt, void* stream);
/* Rows [row0, row0+n): step-t update with dense gradients g[n][E], g1[n] (zeroed after). */
int dl_rec_apply_rows(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, int64_t row0,
                      int64_t n, float* g, float* g1, const float* hist, int32_t hist_len,
                      const float* opt, void* stream);
/* Sharded owners, deterministic: per unique received row (dl_sort_unique over the received
 * ids) the ordered sum of its arrivals g[pos][E], g1[pos] is applied (step opt[7]).  With
 * mv (the owner gather's moment stash, [n][dl_rec_stash_floats(E)]) the row's caught-up state is taken from
 * rows[pos][E] / rows1[pos] / mv[pos] at its first arrival — the owner gather's outputs —
 * and the record is only written; without it the record is read and caught up again. */
int dl_rec_apply_segments(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, const int32_t* uniq,
                          const int32_t* seg_off, const int32_t* n_uniq, int64_t max_uniq, int64_t n,
                          const int32_t* sorted_pos, const float* g, const float* g1, const float* rows,
                          const float* rows1, const float* mv, const float* hist, int32_t hist_len,
                          const float* opt, void* stream);
/* Every row caught up to step opt[7] (before export/checkpoint, and every hist_len steps).
 * p_plane [n_rows][E] / w1_plane [n_rows] (may be NULL): every row's caught-up p and first-order
 * weight written out densely — the table predict's plain lookup then reads (dl_embed_fwd on the
 * planes: 64-B rows instead of the records' 128-B first lines); with DL_REC_PLANE_SLOTS in
 * rec_flags, one slot plane [n_rows][2E] holding both (dl_embed_fwd_slots). */
int dl_rec_flush(float* rec, int32_t rec_ld, int32_t emb_dim, int32_t rec_flags, int64_t n_rows,
                 const float* hist, int32_t hist_len, const float* opt, float* p_plane, float* w1_plane,
                 void* stream);

/* ------------------------------------------------------------------------
 * Row-sharded tables (shard.hip).  Owner side of the all-to-all lookup:
 * out[i] = table[ids[i]], out_first[i] = first[ids[i]] (first may be NULL);
 * and of the gradient return: G[ids[i]] += g[i] (f32 atomics: a row may come
 * from several peers), touched[ids[i]] = 1. */
int dl_shard_gather(const float* table, const float* first, const int32_t* ids, int64_t n,
                    int32_t emb_dim, float* out, float* out_first, void* stream);
int dl_shard_scatter_add(const float* g, const float* g_first, const int32_t* ids, int64_t n,
                         int32_t emb_dim, float* G, float* G_first, uint8_t* touched, void* stream);
/* Fixed-capacity exchange blocks of the sharded step (one hipGraph per step).
 * Arrays of 2W - 1 blocks of `cap` slots: block p < W = what peer p sends this rank (block
 * `rank`: this rank's own requests, in place), block W + p - (p > rank) = this rank's requests
 * to / answers from peer p.  dl_shard_route, from the batch index (unique keys grouped by owner,
 * owner_counts [W + 1] with the replicated group last): ids[block(p) cap + j] = the j-th unique
 * row owned by p (local row), -1 past its count; hdr[block(p) * 4] = {count, flags, rank, 0}
 * with flags = DL_STATUS_BAD_ID if err[0] and DL_STATUS_OVERFLOW if any owner's count exceeds
 * cap (or the replicated group rep_cap); rep_ids[j] = the replicated rows (-1 past the count);
 * upos[u] (may be NULL; u < n_max) = unique row u's slot block(p) cap + j, or
 * (2W - 1) cap + j for the replicated group, -1 past a capacity; inv (may be NULL, n_refs
 * entries) remapped in place from unique ids to slots.  The forward then reads rows_u[slot],
 * the backward writes its gradients at slots (dl_embed_bwd_sorted upos), and the exchanges
 * (dl_shard_exchange) move whole blocks.
 * dl_shard_stamp: before the request exchange, every outgoing header gets this rank's sticky
 * fault bits and its global step.
 * dl_shard_step_begin (after it): the step's guard from every rank's header — a bad id on any
 * rank skips the step everywhere (status DL_STATUS_BAD_ID, opt[DL_OPT_BAD_RANKS] |= the ranks),
 * an overflow / sticky fault on any rank or different steps (DL_STATUS_DESYNC) poison this and
 * every later step everywhere until the host clears the status — then dl_adam_begin_step and
 * (hist non-NULL) dl_adam_hist_record, as dl_step_begin.  hdr2 (may be NULL; blocks of cap2
 * slots): a second id set's headers (wdl's wide ids), counted and flagged alike. */
int dl_shard_route(const uint32_t* uniq_keys, const int32_t* n_uniq, const int32_t* owner_counts, int32_t world,
                   int32_t rank, int64_t cap, int32_t rep_cap, const int32_t* err, int32_t* ids, int32_t* hdr,
                   int32_t* rep_ids, int32_t* upos, int32_t* inv, int64_t n_refs, int64_t n_max, void* stream);
int dl_shard_stamp(int32_t* hdr, int32_t world, int32_t rank, const float* opt, void* stream);
int dl_shard_step_begin(const int32_t* hdr, const int32_t* hdr2, int32_t world, int64_t cap, int64_t cap2, float* opt,
                        float decay_rate, float decay_steps, float* hist, int32_t hist_len, void* stream);
/* out[i] = sum_s slab[s*stride + i] (dense gradients before the all-reduce). */
int dl_slab_sum(const float* slab, int32_t nslab, int64_t stride, int64_t n, float* out, void* stream);
/* out[i] = local row of uniq key i (i < min(n_uniq, cap)): the id send list. */
int dl_keys_to_local(const uint32_t* keys, const int32_t* n_uniq, int64_t cap, int32_t* out,
                     void* stream);

/* Row-sharded wdl_weights (wdl.py:241-285): row r on rank r % world, local r / world.
 * dl_shard_gather_scalar: out[i] = w[ids[i]] (owner side of the wide lookup);
 * dl_shard_add_fixed: G[ids[i]] += g[i] (int64 fixed point, integer atomics: order-free);
 * dl_wide_fold_owned: the deep-output rows row0 + j (j < H) this rank owns get
 *   G[(row0+j)/world] += fixed(gdeep[j]) (gdeep: the all-reduced sums of dz*h);
 * dl_wide_owned_values: out[j] = w[(row0+j)/world] if owned here, else 0 (sum over ranks =
 *   the replicated deep-output rows);
 * dl_wide_local_ids: out[k] = offset + inv[k] (-1 where inv < 0): wide ids into the
 *   rank's local wide table (exchanged rows). */
int dl_shard_gather_scalar(const float* w, const int32_t* ids, int64_t n, float* out, void* stream);
int dl_shard_add_fixed(const int64_t* g, const int32_t* ids, int64_t n, int64_t* G, uint8_t* touched,
                       void* stream);
int dl_wide_fold_owned(const float* gdeep, int32_t H, int64_t row0, int32_t world, int32_t rank, int64_t* G,
                       uint8_t* touched, void* stream);
int dl_wide_owned_values(const float* w, int32_t H, int64_t row0, int32_t world, int32_t rank, float* out,
                         void* stream);
int dl_wide_local_ids(const int32_t* inv, int64_t n, int64_t offset, int64_t* out, void* stream);
/* Lazy-exact TF1 Adam for Wide&Deep's wide weights (wide.hip; models/wdl.py:241-285, L2 on
 * every row: TF's dense gradient l2 * w reaches every row each step).  rec [w_rows][4] =
 * {w, m, v, stamp}; a row's skipped steps are replayed on read (g = l2 * w, adam_elem),
 * bit-identical to the dense dl_adam_rows sweep.
 * dl_wide_rec_gather: the deep-output rows Fw..Fw+H and the unique wide rows uniq_rows[u]
 * (dl_index_build keys, world 1) caught up to step opt[7] - lag into the head's local table
 * wloc = [— (Fw) | deep rows (H) | unique rows]; stash[u] (may be NULL) = {w, m, v, row bits};
 * rep_sq[u] (may be NULL) = the sum of w^2 over the steps replayed for unique row u (each
 * step's pre-update state: that step's L2 loss term for the row), counted by the update.
 * dl_wide_seg_grad: the batch's wide-weight gradient per unique wide row from the wide index
 *   (dl_index_build over the wide ids: sorted references `refs`, segment offsets `seg_off`, count
 *   n_uniq on the device): q[u] = sum over the row's references e of wide_fixed(dz[e / Fw]), int64
 *   fixed point (DL_WIDE_GRAD_SCALE) — the same bits as the head's per-reference atomics, without
 *   them (the head then runs with g_w = NULL).  long_ws: int32 [max_uniq + 1] scratch (hot rows).
 * dl_wide_rec_update: step opt[7] on the unique rows (gradient gloc[Fw + H + u] + the deep
 * term gloc[row] of a row in Fw..Fw+H, exact int64, + l2 w) from the stash, then on the deep
 * rows not covered; gloc reset; the pre-update w^2 of those rows as per-block partial sums
 * written to sq_out[0 .. dl_wide_update_blocks(max_uniq, H)) (may be NULL; the caller sums).
 * acc (may be NULL; double[65536], one slot per block index): the running loss's wide L2
 * term — every pre-update w^2 of the rows this step applies, and of the steps replayed for
 * them (rep_sq, or the deep rows' own replay) — added per block.
 * dl_wide_rec_flush: every row caught up to step opt[7]; the pre-update w^2 of the rows the
 * last step left untouched (the loss's L2 term for them) added to sq_untouched (int64 fixed
 * point, DL_REG_SUM_SCALE); every replayed
 * step's pre-update w^2 added to acc's slots (may be NULL).  Summed over acc after a flush, the
 * slots hold sum_t sum_r w_r(t-1)^2 over the steps since acc was zeroed on a flushed table. */
int dl_wide_rec_gather(const float* rec, int64_t w_rows, const uint32_t* uniq_rows, const int32_t* n_uniq,
                       int64_t max_uniq, int32_t Fw, int32_t H, const float* hist, int32_t hist_len,
                       const float* opt, float l2, int32_t lag, float* wloc, float* stash, float* rep_sq,
                       void* stream);
int64_t dl_wide_update_blocks(int64_t max_uniq, int32_t H);
int dl_wide_seg_grad(const float* dz, int32_t Fw, const int32_t* refs, const int32_t* seg_off, const int32_t* n_uniq,
                     int64_t max_uniq, int64_t nrefs, int64_t* q, int32_t* long_ws, const float* opt, void* stream);
int dl_wide_rec_update(float* rec, const int32_t* n_uniq, int64_t max_uniq, const float* stash, int64_t* gloc,
                       int32_t Fw, int32_t H, float l2, const float* hist, int32_t hist_len,
                       const float* opt, uint8_t* dmark, float* sq_out, const float* rep_sq, double* acc,
                       void* stream);
int dl_wide_rec_flush(float* rec, int64_t w_rows, float l2, const float* hist, int32_t hist_len,
                      const float* opt, int64_t* sq_untouched, double* acc, void* stream);
#define DL_LOSS_ACC_SLOTS 65536   /* slots of the wide running-loss accumulator (>= any grid above) */

/* ------------------------------------------------------------------------
 * RCCL collectives of the row-sharded step (comm.cpp; SURVEY.md §8(b)3
 * comm_init / all_to_allv / all_reduce), for a host that binds this library
 * directly.  One communicator per rank (one GPU each); calls are stream-ordered.
 * RCCL errors return 2000 + ncclResult_t.  The Python engine (shard.py) reaches the
 * same RCCL through torch.distributed (backend "nccl").
 *   dl_comm_get_unique_id: rank 0 creates the id (dl_comm_unique_id_bytes() bytes)
 *     and ships it to the other ranks out of band (the reference-side launcher's job);
 *   dl_all_to_allv: rows of row_bytes each, grouped by peer in rank order; counts are
 *     host arrays of nranks row counts (the step's owner-count all-gather gives them);
 *   dl_all_reduce_f32: sum, in place when send == recv;
 *   dl_all_gather: `bytes` per rank into recv[nranks][bytes]. */
int dl_comm_unique_id_bytes(void);
int dl_comm_get_unique_id(void* id_out);
int dl_comm_init(const void* unique_id, int32_t nranks, int32_t rank, void** comm_out);
int dl_comm_destroy(void* comm);
int dl_all_to_allv(void* comm, const void* send, const int64_t* send_counts, void* recv,
                   const int64_t* recv_counts, int64_t row_bytes, void* stream);
int dl_all_reduce_f32(void* comm, const float* send, float* recv, int64_t n, void* stream);
int dl_all_gather(void* comm, const void* send, void* recv, int64_t bytes, void* stream);
/* The sharded step's exchanges (dl_shard_route's block layout; replaces the id / row / gradient
 * all-to-alls of SURVEY §8(e) with fixed sizes, so the whole step is one hipGraph): for each of
 * n_arrays device arrays of 2W - 1 blocks of block_bytes[a] bytes (host arrays), every block
 * this rank sends to / receives from every other peer, in one RCCL group.  dir 0 (to the
 * owners): send block W + p - (p > rank), receive peer p's into block p; dir 1 (back to the
 * senders): send block p, receive into block W + p - (p > rank).  world 1: no-op. */
int dl_shard_exchange(void* comm, int32_t n_arrays, void* const* bases, const int64_t* block_bytes, int32_t dir,
                      void* stream);

/* ------------------------------------------------------------------------
 * Utilities. */
/* Counter-based (Philox-4x32-10) init: dist 0 normal(mean, scale), 1 uniform[mean, mean+scale). */
int dl_init_random(float* p, int64_t n, int32_t dist, float mean, float scale, uint64_t seed,
                   uint64_t offset, void* stream);

/* ------------------------------------------------------------------------
 * Evaluation metric (metrics.hip): exact tie-aware ROC-AUC, the semantics of
 * sklearn.metrics.roc_auc_score that the reference calls on the collected scores
 * (models/deepfm_pipeline.py:311,344; wdl.py:343-358; deepfm.py:229).
 * scores[i * s_stride], labels[i * l_stride] (label > 0.5 = positive), n <= 2^31-1.
 * Writes the AUC to out[0] (device double; NaN when only one class is present, where
 * sklearn raises).  The numerator is an exact integer count (ties: 1/2), so the result
 * is deterministic.  Workspace: dl_auc_workspace_bytes(n). */
int64_t dl_auc_workspace_bytes(int64_t n);
int dl_auc(const float* scores, int64_t s_stride, const float* labels, int64_t l_stride, int64_t n,
           void* ws, int64_t ws_bytes, double* out, void* stream);
/* Streaming copy of `bytes` (a multiple of 16, both pointers 16-B aligned) from src to dst: the
 * measured HBM yardstick bench.py reports beside the 8 TB/s specification (roofline.peak_measured). */
int dl_hbm_copy(const void* src, void* dst, int64_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DLAMD_H */
