/*
 * ebert.h -- C ABI of the MI355X-native embedding-similarity retrieval engine (libebert.so).
 *
 * This is the drop-in boundary for the reference's recommend/top-K hot path:
 *   /root/reference/src/backend/app/lib.py:51-55   cosine_similarity -> mean -> exclude rated
 *                                                   -> sort_values(desc)[:k]
 *   /root/reference/src/backend/app/lib.py:105-106  the same mean-cosine for search re-weighting
 *   /root/reference/src/backend/app/constants.py:55-56  catalog residency (load-time)
 * The reference has no plugin/operator API for this path; the seam is that inline block, so the
 * entry points below are what its Python binding (ctypes) calls in place of
 * scikit-learn `cosine_similarity` (metrics/pairwise.py:1683-1738) and the pandas sort.
 *
 * Conventions
 *   - Every pointer argument is DEVICE memory owned by the caller (torch tensors), except where
 *     a comment says "host". The library never allocates or frees caller memory; scratch space
 *     is a caller-provided workspace sized by ebt_cosine_topk_workspace().
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream). Every entry point only
 *     enqueues work on that stream and returns; nothing synchronises except ebt_timer_query().
 *   - Return value: EBT_OK (0) or a negative EBT_E* code; the message of the last failure on the
 *     calling thread is available from ebt_last_error(). All entry points are reentrant: no
 *     mutable global state apart from the thread-local error string and a per-device cache of
 *     the compute-unit count (atomic; every writer stores the same value).
 *   - Row ids: catalog rows are addressed by their row number inside the (shard-local) matrix;
 *     results carry GLOBAL row ids = local row + row_offset (a catalog row-sharded over ranks).
 *   - Ordering of every top-k result: score descending, then row ascending. The reference's
 *     pandas sort is an unstable introsort (pandas core/sorting.py:436-441), so its tie order is
 *     unspecified; this is the deterministic order the build defines.
 *   - Non-finite catalog rows: a row holding a NaN or an infinity has a NaN cosine against every
 *     query; such a row is never a candidate on any path (the selects, merges, the filter
 *     epilogue and the large-k sort all drop NaN scores), so it only shows as an empty NaN / -1
 *     slot when k exceeds the remaining candidates. pandas would list it last with score NaN
 *     (sort_values(na_position="last")); the reference's catalogs are finite ALS / embedding
 *     factors, and no reference fixture holds a non-finite row (parity unpinned on this edge).
 */
#ifndef EBERT_H_
#define EBERT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------- */
#define EBT_OK 0
#define EBT_EINVAL (-1)      /* bad argument (shape, dtype, null pointer, k/kprime range)   */
#define EBT_EHIP (-2)        /* a HIP runtime call or kernel launch failed                    */
#define EBT_ENOMEM (-3)      /* workspace too small                                           */
#define EBT_EUNSUPPORTED (-4)

/* ---- element types --------------------------------------------------------------------- */
#define EBT_F32 0
#define EBT_BF16 1
#define EBT_F16 2
#define EBT_F64 3

/* Library version (major*10000 + minor*100 + patch).
 * 0.2.0: ebt_rescore gained `timer`; ebt_comm gained the trailing `all_reduce_f64` pointer (the
 *        library calls it whenever it is non-NULL: zero-initialise every ebt_comm).
 * 0.3.0: ebt_timer_count_rows / ebt_timer_rows (additive).
 * 0.3.1: eps from the measured image errors (ebt_query_image); ebt_catalog_init measures u_cat
 *        and its state holds 256 bytes more for a non-native catalog (ebt_catalog_state_bytes);
 *        ebt_cosine_sample_lead / ebt_cosine_screen_at_lead (additive).
 * 0.3.2: ebt_sort_exclusions and the full-sort path hand-written (workspace sizes shrink; host
 *        arithmetic only); the exclusion-order check of ebt_cosine_topk* runs inside the rescore
 *        (certified = -3 from ebt_cosine_topk_prepared / ebt_rescore's callers for a query whose
 *        segment is not ascending); ebt_shard_sample_tiles (additive); the row counter of
 *        ebt_timer_count_rows is device-aware.
 * 0.3.3: a pinned certificate buffer of ebt_cosine_topk_submit / ebt_cosine_topk_sharded_submit
 *        is written by the kernels themselves (no copy launch; EBT_EHIP from _finish if one was
 *        not delivered); the speculative screen's segment thresholds come from its wave merges;
 *        ebt_merge_packed also flags a query with more than min(R k, 2 k + 256) entries. */
int ebt_version(void);

/* Message for the last non-zero return on this thread ("" if none). */
const char* ebt_last_error(void);

/* ---- catalog load: constants.py:55-56 (+ sklearn row_norms, preprocessing/_data.py:2011) ---
 * Guarded L2 norm of every row in float64: gnorm[i] = ||x_i|| unless ||x_i|| < 10*DBL_EPSILON,
 * in which case 1.0 (sklearn _handle_zeros_in_scale, preprocessing/_data.py:118-123), and the
 * float32 reciprocal inv32[i] = 1/gnorm[i] used by the screening epilogue. inv32 may be NULL.
 * x: n rows of d elements of `dtype`, row stride `ld` ELEMENTS. */
int ebt_row_norms(const void* x, int dtype, int64_t n, int32_t d, int64_t ld,
                  double* gnorm64, float* inv32, void* stream);

/* Screening image of a matrix: img[i][j] = round_to(img_dtype, x[i][j] * s_i) for j < d and 0 for
 * d <= j < ld_img, where s_i = 1/gnorm64[i] if `normalize` else 1. img_dtype is EBT_F16 or
 * EBT_BF16; ld_img (row stride in elements) must be a multiple of 64 and >= d. Rows of the
 * image past n are not touched. */
int ebt_screen_image(const void* x, int dtype, int64_t n, int32_t d, int64_t ld,
                     const double* gnorm64, int normalize, int img_dtype, void* img,
                     int32_t ld_img, void* stream);

/* ---- queries: lib.py:51-52 folded into one query vector per user -------------------------
 * Dense queries (one vector per query, the L = 1 case of lib.py:51):
 *   q64[b] = q[b] / gnorm(q[b])  (float64, sklearn normalize semantics).
 * Liked-rows queries (the collaborative path): for CSR lists liked_off[B+1] / liked_rows[] of
 * LOCAL catalog rows, q64[b] = sum_l cat[l] / gnorm64_cat[l]  (a SUM; the caller divides by the
 * user's liked count L_b after an optional cross-shard all-reduce). liked_off/liked_rows NULL
 * selects the dense form. q64 is B x d float64, row stride d. */
int ebt_query_dense(const void* q, int dtype, int64_t B, int32_t d, int64_t ldq, double* q64,
                    void* stream);
int ebt_query_liked_sum(const void* cat, int dtype, int32_t d, int64_t ld,
                        const double* gnorm64_cat, int64_t B, const int64_t* liked_off,
                        const int64_t* liked_rows, double* q64, void* stream);
/* ebt_query_dense + ebt_query_image in one launch for dense queries (d <= 4096; same q64,
 * qimg, qscale and eps; with native_q the query dtype must equal img_dtype). */
int ebt_query_prep(const void* q, int dtype, int64_t B, int64_t B_pad, int32_t d, int64_t ldq,
                   int img_dtype, int native_q, float u_cat, double* q64, void* qimg,
                   int32_t ld_img, float* qscale, float* eps, void* stream);
/* q64[b] *= scale[b] (scale is device float64[B]); used for the 1/L of lib.py:52. */
int ebt_scale_rows_f64(double* q64, int64_t B, int32_t d, const double* scale, void* stream);

/* Screening image + certification bound of a query batch.
 *   qimg[b][j] = round_to(img_dtype, q64[b][j]) (rows B..B_pad-1 and columns d..ld_img-1 = 0),
 *   qscale[b]  = 1,
 *   eps[b]     = a rigorous bound on |approx score - exact float64 score| for every catalog
 *                row, given `u_cat` >= ||image row - row/gnorm||_2 for every row (0 for a
 *                native image whose values are exact; ebt_catalog_init measures it for a
 *                float16-rounded normalised image, and the unit round-off 2^-11 always holds):
 *                eps = 1.05*(dq + |q|*u_cat + dq*u_cat + (d+8)*2^-24*(|q|+1)) + 1e-9,
 *                with dq = ||qimg[b] - q64[b]||_2 measured by the kernel (ABI 0.3.1; before it
 *                dq was bounded by |q| times the unit round-off of img_dtype).
 * With `native_q` != 0 the image is instead the raw query `q` (same dtype as img_dtype, the
 * native-catalog screening mode): qimg = q, qscale[b] = 1/gnorm(q[b]) and dq = 0. */
int ebt_query_image(const double* q64, int64_t B, int64_t B_pad, int32_t d, int img_dtype,
                    const void* q_native, int64_t ldq, int native_q, float u_cat, void* qimg,
                    int32_t ld_img, float* qscale, float* eps, void* stream);

/* ---- kernels of the search pipeline (exposed for tests and the bench) --------------------
 * Screening GEMM on MFMA: scores[b][i] = qscale[b]*cscale[i]*sum_j qimg[b][j]*cimg[i][j] for
 * b < B_pad (multiple of 128) and i < n_rows; f16 or bf16 inputs, float32 accumulate.
 * cscale may be NULL (= 1). ld_scores must be a multiple of 4 and >= n_rows. */
int ebt_screen_scores(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                      int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                      const float* cscale, float* scores, int64_t ld_scores, void* stream);

/* The fused screen's GEMM: the same product, but only scores >= thr[b] leave the kernel.
 * Catalog rows are grouped by G = ebt_filter_group_rows(B_pad) (the kernel's tile: 256 rows
 * when B_pad % 256 == 0, else 128); the first `slots` hits of query b in group g go to
 * cand[b*ld_cand + g*slots + p] as u64 composites (order-preserving key of the f32 score << 32 |
 * ~(uint32)(idx_base + local row)), and counts[b*ld_counts + g] = the group's hit count
 * (saturated at 255). A count above `slots` drops hits and sets ovf[b] = 1. Buffers have B_pad
 * rows, 1 <= slots <= EBT_FILTER_SLOTS_MAX, ld_cand >= groups*slots, ld_counts >= groups; thr
 * has B_pad entries (+inf for padding). */
#define EBT_FILTER_SLOTS_MAX 128
int64_t ebt_filter_group_rows(int64_t B_pad);
/* Long filter launches (0.3.0): a fused segment of the pipeline (ebt_cosine_topk*, ebt_cosine_screen*)
 * over more than ~1.5 x T x (CUs / query tiles) tiles of 256 rows is run as consecutive
 * ebt_screen_filter launches of whole rounds, each at most T tiles per workgroup
 * (default T = 32 since 0.3.1, 512 in 0.3.0; EBT_FILTER_TPW in the environment), so that the persistent walk's
 * workgroups start in step again (screening GEMM). Same tiles, hits and counts.
 * ebt_filter_split(T) sets T for the process (0: never split; T < 0: query) and returns the
 * previous value. */
int64_t ebt_filter_split(int64_t tiles_per_workgroup);
int ebt_screen_filter(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                      int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                      const float* cscale, const float* thr, uint64_t* cand, int64_t ld_cand,
                      int32_t slots, uint8_t* counts, int64_t ld_counts, int32_t* ovf,
                      int64_t idx_base, void* stream);

/* Excluded rows (lib.py:48,55: rated movies are not candidates): for every b < B and every
 * GLOBAL row g in excl_rows[excl_off[b] .. excl_off[b+1]) with col_begin <= g < col_end,
 * scores[b][g - col_begin] = -inf. */
int ebt_mask_excluded(float* scores, int64_t ld_scores, int64_t B, int64_t col_begin,
                      int64_t col_end, const int64_t* excl_off, const int64_t* excl_rows,
                      void* stream);

/* Streaming top-k' select (one HBM pass over the scores): for each row b < B and each of `segs`
 * equal segments of its n entries, write the kprime largest (value desc, index asc) entries,
 * sorted, to out_vals/out_idx[b*ld_out + seg*kprime + j]. Entries that are NaN or -inf are
 * never selected; missing slots get -inf / -1. Dense form (idx == NULL): the index of entry j
 * is idx_base + j. Candidate-list form: idx[b*ld + j] gives it (values < 2^31, -1 = empty).
 * 1 <= kprime <= 4096. */
int ebt_select_topk(const float* vals, const int64_t* idx, int64_t ld, int64_t B, int64_t n,
                    int64_t idx_base, int32_t kprime, int32_t segs, float* out_vals,
                    int64_t* out_idx, int64_t ld_out, void* stream);

/* Exact float64 rescore of the screened candidates + final top-k + certification.
 * For each b: candidates cand_rows[b*kprime + j] (LOCAL rows, -1 = empty), sorted by their
 * approx scores cand_vals (desc). score = (q64[b] . cat[row]) / gnorm64[row] in float64; the k
 * best by (score desc, row asc) go to out_scores/out_rows[b*k + j] (rows + row_offset; empty
 * slots NaN / -1). certified[b] = 1 iff the candidate set provably contains the exact top-k:
 * kprime >= n_rows (every row is a candidate),
 * fewer than kprime valid candidates, or approx[kprime-1] < cut[b] (below, after its rise).
 * n_rows is the catalog's row count; a candidate row >= n_rows is never read and gives
 * certified[b] = -2 (corrupt candidate list).
 * Candidates with approx < cut[b] = max(approx[k-1] - 2*eps[b], t_floor[b] - eps[b]) cannot
 * be in the top k and are not gathered (equal cand_vals and eps = 0 rescore every candidate).
 * With eps[b] > 0 the cut then rises to s_min - eps[b], s_min = the smallest exact score of the
 * list's first k entries (k rows score >= s_min, so a row with exact < s_min is not in the top
 * k): those k are scored first and later candidates below the raised cut are skipped. t_floor
 * (float64 [B], NULL = none) is a lower bound of the k-th best EXACT score over the whole
 * (sharded) catalog, e.g. the all-reduced max over shards of approx[k-1] - eps: a shard then
 * rescores only rows that can enter the GLOBAL top k, and the slots of its top k that such a
 * cut leaves empty read NaN / -1: the certificate is then about the GLOBAL top k (a row
 * dropped below approx[kprime-1] < t_floor - eps has exact < t_floor). */
int ebt_rescore(const double* q64, int64_t B, int32_t d, const void* cat, int dtype, int64_t ld,
                const double* gnorm64, int64_t row_offset, const float* cand_vals,
                const int64_t* cand_rows, int32_t kprime, int32_t k, int64_t n_rows, const float* eps,
                const double* t_floor, double* out_scores, int64_t* out_rows, int32_t* certified,
                void* timer, void* stream);

/* Diagnostics of the rescore's arithmetic (tests, A/B tools; not needed by a caller).
 * ebt_rescore_form(form): which form of the exact dot products ebt_rescore (and every entry
 * point that rescores) launches from now on, process-wide: 1 = the lane's query values held in
 * registers (the default where d fits 512 16-byte chunks), 0 = the query staged in LDS; -1
 * leaves it. Returns the form in effect before the call. Both forms give bitwise equal scores.
 * ebt_wave_sum_check: for each of n_waves waves of 64 doubles in[64 w + l], out_a[64 w + l] =
 * the library's wave sum (cross-lane VALU moves), out_b[...] = the same xor butterfly through
 * shuffles; the two are expected bitwise equal in every lane. */
int ebt_rescore_form(int form);
int ebt_wave_sum_check(const double* in, int64_t n_waves, double* out_a, double* out_b,
                       void* stream);

/* The fused screen's merge step: query b's candidate list (fv/fi[b*kprime + j], a PARTITIONED
 * list: see below; a sorted list, as ebt_select_topk leaves it, is one) and the hits
 * ebt_screen_filter left in `n_groups` groups of cand/counts (same slots/ld as that call) -> the
 * kprime best of both, back into fv/fi, partitioned at k (1 <= k <= kprime):
 *   [0, k-1) the k-1 best in any order, [k-1] the k-th best, [k, n-1) the rest in any order,
 *   [n-1] the smallest kept, [n, kprime) empty (-inf / -1), n = min(kprime, entries).
 * (Lists of k' > 512, merged by the block kernel, come back fully sorted: also partitioned.)
 * Exclusions (GLOBAL rows, CSR sorted per query, or NULL) are dropped from the hits; a group
 * count above `slots`, or more hits than the merge holds, sets ovf[b] = 1. */
int ebt_merge_hits(float* fv, int64_t* fi, int64_t B, int32_t kprime, int32_t k,
                   const uint64_t* cand, int64_t ld_cand, int32_t slots, const uint8_t* counts,
                   int64_t ld_counts, int64_t n_groups, int64_t row_offset,
                   const int64_t* excl_off, const int64_t* excl_rows, int32_t* ovf, void* stream);
/* Groups one block merge (k' > 512) indexes at once: its LDS holds the list + hit entries and a
 * u16 position per group; ebt_merge_hits merges more groups in consecutive parts of this many
 * (rounded down to 16). Host call, no device work after the first (reads the kernel's static
 * LDS size). */
int64_t ebt_merge_block_max_groups(int32_t kprime);

/* Exclusion CSR order: the search entry points binary-search each exclusion segment and take
 * it sorted ascending. ebt_sort_exclusions sorts every segment of a caller's CSR on the device:
 * segment b = rows_in[off[b] .. off[b+1]) (ABSOLUTE positions, off[0] may be > 0), sorted into
 * the same positions of rows_out; positions outside every segment are copied unchanged; rows_out
 * may equal rows_in. nnz = the length of the rows array. Offsets are clamped into [0, nnz] before
 * use (a malformed CSR is then rejected by the search entry's own check). Workspace: device,
 * ebt_sort_exclusions_bytes(B, nnz) bytes (0 = invalid sizes: B < 1 or > 2^24, nnz >= 2^31;
 * 0.3.2: one hand-written launch, 8 * nnz bytes of workspace). */
size_t ebt_sort_exclusions_bytes(int64_t B, int64_t nnz);
int ebt_sort_exclusions(const int64_t* off, const int64_t* rows_in, int64_t* rows_out, int64_t B,
                        int64_t nnz, void* workspace, size_t ws_bytes, void* stream);

/* Merge R partial top-k lists (scores/rows [R][B][k], each sorted) into the global top-k per
 * query -- the post-all-gather step of a row-sharded catalog. k <= 4096, any R. */
int ebt_merge_topk(const double* scores, const int64_t* rows, int32_t R, int64_t B, int32_t k,
                   double* out_scores, int64_t* out_rows, void* stream);

/* The compact form of that exchange (what the row-sharded step sends). After the catalog-wide
 * floor (ebt_union_floor), a shard's entries below t_floor[b] -- a lower bound of query b's k-th
 * best exact score over the WHOLE catalog -- cannot enter the global top k. ebt_shard_pack keeps
 * of each sorted list (scores/rows [B][k], row < 0 = padding; t_floor NULL = keep every real
 * entry) the prefix with score >= t_floor[b] and packs it into `send`
 * (ebt_shard_pack_bytes(B, cap) bytes, device): u32 start[B], u32 len[B] (query b's entries are
 * [start[b], start[b] + len[b]); 0.3.2 -- ebt_shard_pack writes the starts in query order, the
 * sharded C entry's rescore reserves each query's range by an atomic, so any order is valid)
 * and block totals, then f64 scores[cap], then i32 GLOBAL rows[cap]. Entries at positions
 * >= cap are counted but not sent. After an all-gather of the R buffers
 * (recv, R * ebt_shard_pack_bytes bytes, rank order), ebt_merge_packed writes the same global
 * top-k as ebt_merge_topk over the full lists, and sets *incomplete (device int32; set to 1,
 * never cleared) when some rank's entries did not all fit its cap, or (0.3.3) when one query
 * received more than min(R k, 2 k + 256) entries (a floor band wider than k + 256): the caller
 * must then merge the full lists instead (the rows of an incomplete batch are not final).
 * ebt_shard_pack_cap: the cap the library uses, B * ebt_shard_list_width(k, world), or 0 when
 * the compact form does not apply (world < 2, world * k > 8192, n_global >= 2^31).
 * ebt_shard_list_width(k, world) = min(k, ceil(1.5 k / world) + 8): also the per-shard width of
 * the floor all-gather (a shard's widest share of the global top k, with margin; a narrower
 * floor is still a valid lower bound). */
int64_t ebt_shard_list_width(int32_t k, int32_t world);
/* The shared screening threshold's sample of the row-sharded step (0.3.2, host arithmetic): the
 * 256-row tiles each shard samples for this catalog size, world and padded batch (0 = every
 * shard screens at its own threshold; -1 bad arguments). The same rule as distributed.py
 * shared_sample_tiles; world * 4 * tiles <= 2048 (ebt_pool_kth's limit). */
int64_t ebt_shard_sample_tiles(int64_t n_global, int32_t world, int64_t B_pad);
int64_t ebt_shard_pack_cap(int64_t B, int32_t k, int32_t world, int64_t n_global);
size_t ebt_shard_pack_bytes(int64_t B, int64_t cap);
int ebt_shard_pack(const double* scores, const int64_t* rows, int64_t B, int32_t k,
                   const double* t_floor, int64_t cap, void* send, void* stream);
int ebt_merge_packed(const void* recv, int32_t R, int64_t B, int32_t k, int64_t cap,
                     double* out_scores, int64_t* out_rows, int32_t* incomplete, void* stream);

/* Exact screen: scores[b*ld_scores + j] = (float)((q64_b . c_j) / gnorm64_j) in float64
 * arithmetic for every row j < n_rows (no replacement in the reference: the fallback screen of
 * EBT_FLAG_EXACT, whose only error is the final f32 rounding). */
int ebt_screen_exact(const double* q64, int64_t B, int32_t d, const void* cat, int dtype,
                     int64_t ld, const double* gnorm64, int64_t n_rows, float* scores,
                     int64_t ld_scores, void* stream);

/* ---- the whole pipeline -------------------------------------------------------------------
 * flags: EBT_FLAG_NO_FUSE disables the fused screen (every score row is materialised).
 * EBT_FLAG_EXACT screens with ebt_screen_exact instead of the MFMA image (unfused; qimg,
 * qscale, eps and cimg may be NULL): the last resort for a query that cannot be certified at
 * kprime = 4096, certified with eps = EBT_EXACT_EPS (|q64| <= 1 as the ebt_query_* make it). */
#define EBT_FLAG_NO_FUSE 1
#define EBT_FLAG_EXACT 2
#define EBT_FLAG_THETA 4 /* internal: set by ebt_cosine_screen_at (workspace sizing only) */
#define EBT_EXACT_EPS 1.1920928955078125e-07f /* 2^-23 >= f32 rounding of |s| <= 1 + f64 error */
/* How ebt_cosine_topk_prepared will run these sizes (host pointers out): head rows screened unfused,
 * the largest fused tail segment in rows (cap; 0 = not fused), score chunk rows, fused flag. */
int ebt_cosine_topk_plan(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                         int64_t chunk_rows, int flags, int64_t* head_rows, int64_t* cap,
                         int64_t* chunk, int32_t* fused);
/* The speculative fused screen ebt_cosine_topk_prepared uses for these sizes (all 0: not used).
 * sample_tiles full 256-row tiles, tile_stride tiles apart (tiles 0, s, 2s, ...), go through the
 * screening GEMM keeping only each query's max per 64-row subgroup; the rank-th largest of those
 * maxima is the query's speculative threshold theta for one filter pass over the whole catalog;
 * hits = the expected hits per query. theta is checked afterwards (theta <= the k-th best approx
 * - 2 eps, else certified = -1: rerun unfused), so it never costs exactness. */
int ebt_cosine_topk_spec_plan(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                              int flags, int64_t* sample_tiles, int64_t* tile_stride,
                              int32_t* rank, double* hits);
/* The speculative screen's lead (0.3.0): its sample's first `lead` tiles are the catalog's first
 * tiles (the rest of the sample strided after them: tiles 0 .. lead-1, lead, lead + s, ...), their
 * scores are kept and their hits taken at theta, and the filter GEMM covers rows [256 lead, n)
 * only -- lead is chosen so that those are whole rounds of the persistent grid (one 256 x 256
 * output tile per CU and round); every segment but the last is whole rounds too. Returns the
 * lead in tiles (0: none; -1: bad arguments). ebt_spec_lead(on) switches it on (1, default) or
 * off (0) for the process (on < 0: query); returns the previous setting. Results are the same
 * either way: the lead's hits are the filter's own, value for value. */
int64_t ebt_cosine_topk_spec_lead(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                                  int flags);
int ebt_spec_lead(int on);
/* Workspace bytes needed by ebt_cosine_topk_prepared for these sizes. */
size_t ebt_cosine_topk_workspace(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                                 int64_t chunk_rows, int flags);

/* The prepared-query pipeline under ebt_cosine_topk (one pass, no retries): query x catalog
 * cosine top-k over one (shard of a) catalog:
 *   unfused: for every catalog chunk of chunk_rows rows: screening GEMM -> mask excluded ->
 *   streaming select of kprime candidates; then a select across chunks; then the exact float64
 *   rescore.
 *   speculative fused (default for B_pad % 256 == 0, kprime <= 512 and >= 8 sample tiles, see
 *   ebt_cosine_topk_spec_plan): a pooled sample gives each query a threshold, the whole catalog
 *   is filtered in a few large segments (later ones at max(theta, the list's k-th - 2 eps)),
 *   then theta is verified (failure: certified = -1).
 *   fused (otherwise, when n_rows >= 2*H, H = max(65536, 256*kprime)): the head rows [0, H) go
 *   through the unfused path; the k'-th best head score of each query is a lower bound of its
 *   global k'-th best. The tail rows [H, n) are screened in doubling segments (each as large as
 *   all rows before it): the GEMM appends only scores >= the query's current bound to its
 *   candidate list (epilogue filter: no score matrix in HBM), exclusions are removed from the
 *   list (excl_rows must be sorted ascending per query), the k' best are kept and the bound is
 *   raised to their k'-th score before the next segment -- about k' appends per query per
 *   segment. The final k' are rescored. certified[b] = -1 reports a segment whose appends
 *   exceeded the capacity (rerun the query with EBT_FLAG_NO_FUSE).
 * Inputs: the query batch prepared by ebt_query_* (q64, qimg, qscale, eps; B real rows, B_pad
 * image rows), the catalog (cat/dtype/ld with gnorm64; its screening image cimg with cscale or
 * NULL, ld_img, d_pad), exclusions as CSR of GLOBAL rows (NULL = none), k <= kprime.
 * Outputs: out_scores (float64 [B][k]), out_rows (int64 [B][k], global), certified (int32 [B]);
 * certified[b] = -3 when query b's exclusion segment is not ascending (checked by the rescore,
 * 0.3.2: its results are then not valid). timer (NULL or an ebt_timer) collects per-stage GPU
 * time. */
int ebt_cosine_topk_prepared(const double* q64, const void* qimg, const float* qscale, const float* eps,
                    int64_t B, int64_t B_pad, const void* cat, int dtype, int64_t ld,
                    const double* gnorm64, const void* cimg, const float* cscale, int img_dtype,
                    int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad, int64_t row_offset,
                    const int64_t* excl_off, const int64_t* excl_rows, int32_t k, int32_t kprime,
                    int64_t chunk_rows, int flags, void* workspace, size_t ws_bytes,
                    double* out_scores, int64_t* out_rows, int32_t* certified, void* timer,
                    void* stream);

/* ---- the self-contained path: one call per batch ------------------
 * What a non-Python caller binds (cgo / JNI / N-API / ctypes): raw queries
 * in, certified float64 top-k out; query prep, the screen, the certificate check and every
 * retry (fused-list overflow -> unfused rerun, uncertified -> k' x 4 -> float64 screen) run
 * inside the library. Replaces /root/reference/src/backend/app/lib.py:51-55 (cosine_similarity
 * of the liked rows against the catalog, mean over them, exclusion of rated rows, descending
 * sort, [:k]) for a batch of users, and constants.py:55-56 (the resident catalog).
 *
 * ebt_catalog: the resident (shard of a) catalog, filled by ebt_catalog_init from the caller's
 * device matrix and a caller-provided device STATE buffer of ebt_catalog_state_bytes() bytes
 * (float64 guarded row norms, float32 inverse norms, and the f16 screening image unless the
 * matrix itself is the MFMA operand: f16 / bf16 with d, ld % 64 == 0). Immutable afterwards;
 * the struct and the state buffer must outlive every call that uses them. For a non-native
 * catalog (f32 / f64) ebt_catalog_init waits for `stream` once, to read back u_cat, the largest
 * row error of the image its kernel measured (0.3.1); a native catalog's init stays asynchronous. */
typedef struct ebt_catalog {
  const void* data;       /* [n][ld] of dtype (device, caller-owned)                        */
  int32_t dtype, d;
  int64_t n, ld, row_offset; /* row_offset: global id of local row 0 (row-sharded catalogs)  */
  double* gnorm64;        /* [n]                   (state)                                  */
  float* inv32;           /* [round_up(n, 128)]    (state)                                  */
  const void* image;      /* [n][ld_img] f16/bf16  (state, or `data` itself)                */
  const float* cscale;    /* epilogue row scales: inv32 for native images, NULL otherwise   */
  int32_t img_dtype, ld_img, d_pad, native;
  float u_cat;            /* bound on ||image row - row/gnorm||_2 (0: exact native values;
                             measured by ebt_catalog_init; 2^-11 is always a valid value)    */
} ebt_catalog;

size_t ebt_catalog_state_bytes(const void* data, int dtype, int64_t n, int32_t d, int64_t ld);
int ebt_catalog_init(ebt_catalog* cat, const void* data, int dtype, int64_t n, int32_t d,
                     int64_t ld, int64_t row_offset, void* state, size_t state_bytes,
                     void* stream);

/* Optional knobs (NULL = defaults; a zero field = its default): kprime = the screen's candidate
 * count k' (default: k + slack for the image's error band), chunk_rows = catalog rows per
 * materialised score chunk of the unfused path (default: 4 GiB of f32 scores),
 * flags = EBT_FLAG_NO_FUSE to disable the fused screen. Results do not depend on them.
 * flags |= EBT_FLAG_LIKED_CHECKED (0.3.2, ebt_cosine_topk / _submit only): the caller has
 * checked its liked CSR on the host -- every user has >= 1 liked row and every row lies in the
 * catalog's [row_offset, row_offset + n) -- so _submit does not read the CSR back (no stream
 * synchronisation: the liked path enqueues asynchronously, as the dense one; the 1/L scales
 * are taken from the offsets on the device, the same float64 values). An unchecked CSR with
 * this flag is undefined behaviour (rows out of range are read). */
#define EBT_FLAG_LIKED_CHECKED 8
typedef struct ebt_options {
  int32_t kprime;
  int32_t flags;
  int64_t chunk_rows;
} ebt_options;

/* Device workspace bytes ebt_cosine_topk needs for a batch of B queries and top-k
 * (0 = invalid arguments). */
size_t ebt_workspace_bytes(const ebt_catalog* cat, int64_t B, int32_t k, const ebt_options* opt);

/* Top-k by cosine for B queries, ordered (score desc, row asc), rows GLOBAL ids.
 * Queries: EITHER dense q [B][ldq] of q_dtype (EBT_F32 / F64 / BF16 / F16; a zero row scores
 * 0 against everything, sklearn's zero-norm guard), OR liked rows (q = NULL): CSR liked_off
 * [B+1] / liked_rows (GLOBAL rows of this catalog) and the query of user b is the mean of its
 * liked rows' normalised vectors (lib.py:51-52). A user with no liked row fails with
 * EBT_EINVAL and sklearn's message ("Found array with 0 sample(s) ..."), as the reference
 * raises ValueError; a liked row outside the catalog fails with EBT_EINVAL.
 * Exclusions (the rated movies, lib.py:48,55): CSR excl_off [B+1] / excl_rows of GLOBAL rows,
 * each segment sorted ascending (checked: EBT_EINVAL otherwise), or both NULL.
 * Output: out_scores float64 [B][k] (within 1e-12 of the float64 reference), out_rows int64
 * [B][k]; slots past the catalog's candidates (k > n minus exclusions) are NaN / -1.
 * ebt_cosine_topk synchronises the stream once (the certificates) and returns when the results
 * are final. The two halves let a caller overlap batches: _submit enqueues the first pass
 * (no synchronisation for dense queries; the liked path reads its CSR offsets on the host) and
 * fills the caller's ebt_pending; _finish waits for THAT batch only (an event), reads its
 * certificates from cert_host (host memory, B + 1 int32) and runs the retries. Pinned
 * cert_host (hipHostMalloc / hipHostRegister, e.g. torch pin_memory) is written by the rescore
 * kernel itself, one store per query across the host link (0.3.3: no copy launch; _submit
 * marks the entries unset first and _finish fails with EBT_EHIP on one that was not
 * delivered); pageable memory gets a copy from the workspace (EBT_HOST_DIRECT=0 forces the
 * copy). Workspace, outputs and cert_host stay in use until _finish returns. timer: NULL or
 * an ebt_timer. */
typedef struct ebt_pending {
  const ebt_catalog* cat;
  ebt_options opt;
  int64_t B, B_pad, chunk;
  int32_t k, k_eff, kprime, flags;
  const int64_t* excl_off;
  const int64_t* excl_rows;
  char* ws;
  size_t ws_bytes;
  double* out_scores;
  int64_t* out_rows;
  int32_t* cert_host;
  void* event;
  void* timer;
  void* stream;
} ebt_pending;
int ebt_cosine_topk(const ebt_catalog* cat, const void* q, int q_dtype, int64_t B, int64_t ldq,
                    const int64_t* liked_off, const int64_t* liked_rows, int32_t k,
                    const int64_t* excl_off, const int64_t* excl_rows, const ebt_options* opt,
                    void* workspace, size_t ws_bytes, double* out_scores, int64_t* out_rows,
                    void* timer, void* stream);
int ebt_cosine_topk_submit(const ebt_catalog* cat, const void* q, int q_dtype, int64_t B,
                           int64_t ldq, const int64_t* liked_off, const int64_t* liked_rows,
                           int32_t k, const int64_t* excl_off, const int64_t* excl_rows,
                           const ebt_options* opt, void* workspace, size_t ws_bytes,
                           double* out_scores,
                           int64_t* out_rows, int32_t* cert_host, ebt_pending* pending,
                           void* timer, void* stream);
int ebt_cosine_topk_finish(ebt_pending* pending);

/* ---- row-sharded catalog, self-contained: one call per batch on every rank ---------------
 * The per-shard protocol of robot_ebert_amd/distributed.py (score_topk_sharded_local_stages)
 * inside the library, for a host without Python: every rank holds one shard (an ebt_catalog
 * whose row_offset is the shard's first GLOBAL row) and calls ebt_cosine_topk_sharded with the
 * same queries, k and exclusions; every rank returns the same GLOBAL top-k, equal to
 * ebt_cosine_topk over the whole catalog (rows bit-exact, float64 scores). For liked queries
 * the query is the same up to float64 round-off of its sum: each shard sums its own liked rows
 * and the partial sums are added in rank order, so the additions are grouped by shard (equal to
 * the single-GPU sum when no shard after the first holds two of a user's liked rows); rows
 * within round-off of a tie may then swap -- as they may against the reference itself, which
 * averages the per-row cosine scores instead of the rows (lib.py:51-52). Per batch:
 *   query prep (liked rows: each shard sums its own, one all-gather of the [B][d] float64
 *   partial sums completes the means); when the shards are small (<= 200K rows, >= 2 ranks, the
 *   fused screen) a catalog-wide screening threshold from every shard's sample maxima (one
 *   all-gather); the shard's screen; the catalog-wide floor of the k-th exact score (one
 *   all-gather of [B][k+1] float32) so each shard rescores only rows that can enter the global
 *   top k (each shard sends its ebt_shard_list_width best approx, [B][w+1] float32); the
 *   float64 rescore + certificate; the local retries (no collective: every rank issues the same
 *   all-gathers in the same order whatever its retries); one all-gather of the shards' entries
 *   above that floor (ebt_shard_pack: int32 rows behind per-query starts) and the merge
 *   (ebt_merge_packed) -- or, when the compact form does not apply or a rank's entries exceed
 *   its capacity, two all-gathers of the full [B][k] lists and ebt_merge_topk.
 * The caller supplies the collective, an all-gather over its communicator:
 *   all_gather(ctx, send, recv, bytes, stream): recv (device, world * bytes) receives every
 *   rank's `bytes` from send (device) in rank order. It is called after the work producing
 *   `send` has been enqueued on `stream`, and the library enqueues work reading `recv` on
 *   `stream` right after it returns: a stream-ordered collective (RCCL: ncclAllGather(send,
 *   recv, bytes, ncclInt8, comm, stream)) or a blocking one both work.
 *   It returns 0 on success; anything else fails the call with EBT_EHIP (the other ranks are
 *   then left in their next all_gather: the caller's collective timeout must end them).
 * Limits: k <= 4096 (the merge); B, k, the queries and the exclusions equal on every rank
 * (argument errors are then detected alike everywhere before the first collective). The call
 * returns when the results are final. Workspace: ebt_sharded_workspace_bytes (device). */
typedef int (*ebt_allgather_fn)(void* ctx, const void* send, void* recv, size_t bytes,
                                void* stream);
/* Optional: buf[0 .. count) (device float64) <- the sum over ranks of every rank's buf, in place
 * (RCCL: ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, comm, stream)). The liked path's
 * partial sums use it when it is set -- about 2 / R of the all-gather's volume; the sum's order
 * of additions is then the collective's, a float64 round-off-level difference -- else an
 * all-gather of every rank's partial sums added in rank order. NULL = not provided. */
typedef int (*ebt_allreduce_f64_fn)(void* ctx, double* buf, size_t count, void* stream);
/* Zero-initialise (`ebt_comm c = {0};`, or memset) before filling it in: a field a caller built
 * against an older layout does not set must read NULL (see ebt_version). */
typedef struct ebt_comm {
  int32_t rank, world;
  int64_t n_global;           /* rows of the whole catalog: every shard's row_offset + n <= it */
  ebt_allgather_fn all_gather;
  void* ctx;
  ebt_allreduce_f64_fn all_reduce_f64;  /* optional (NULL), same ctx */
} ebt_comm;
/* An RCCL communicator for an ebt_comm: the library opens librccl.so.1 at first use (it does not
 * link it). Rank 0 calls ebt_rccl_unique_id (128 bytes) and hands the id to every rank out of
 * band (e.g. a torch.distributed broadcast); each rank calls ebt_rccl_comm_init with its HIP
 * device current; then comm.all_gather = ebt_rccl_all_gather, comm.all_reduce_f64 =
 * ebt_rccl_all_reduce_f64, comm.ctx = the handle (ncclAllGather of `bytes` int8, ncclAllReduce
 * of float64 sums, on `stream`). EBT_EUNSUPPORTED when RCCL cannot be loaded. */
int ebt_rccl_unique_id(void* id_out, size_t bytes);
int ebt_rccl_comm_init(const void* id, int32_t rank, int32_t world, void** comm_out);
int ebt_rccl_comm_destroy(void* comm);
int ebt_rccl_all_gather(void* comm, const void* send, void* recv, size_t bytes, void* stream);
int ebt_rccl_all_reduce_f64(void* comm, double* buf, size_t count, void* stream);
size_t ebt_sharded_workspace_bytes(const ebt_catalog* cat, const ebt_comm* comm, int64_t B,
                                   int32_t k, const ebt_options* opt);
/* The same in three calls, so that a caller can keep batches in flight (the collectives and
 * the host's waits of one batch behind the GPU work of the next):
 *   _submit enqueues query prep, the threshold and floor all-gathers, the screen, the rescore
 *     and the certificates into host[0 .. B] (caller's host memory, B + 2 int32; pinned: the
 *     rescore's own stores, else a copy -- as ebt_cosine_topk_submit) and fills *pending;
 *   _finish waits for THAT batch's certificates, runs the shard's local retries, packs the
 *     shard's entries above the catalog-wide floor (ebt_shard_pack), all-gathers them, merges
 *     (ebt_merge_packed) into out_scores / out_rows on the stream and brings the merge's
 *     "incomplete" flag to host[B + 1] (pinned: written by the merge itself);
 *   _wait waits for that flag (an event) and, when a rank's entries did not fit its packed
 *     capacity, re-merges from the full lists (two more all-gathers: every rank sees the same
 *     flag). The results are final when _wait returns.
 * Every rank must make the same sequence of calls (each issues collectives). Workspace, host
 * buffer and outputs belong to the batch until its _wait returns, so a pipelined caller cycles
 * through (at least) three workspaces, e.g. per step: submit(i), finish(i-1), wait(i-2).
 * ebt_cosine_topk_sharded = submit + finish + wait. */
typedef struct ebt_sharded_pending {
  ebt_pending local;  /* the shard's own first pass and retries */
  ebt_comm comm;
  double* out_scores;
  int64_t* out_rows;
  int32_t* host;
  void* event;
  int32_t stage;      /* 1 submitted, 2 finished, 0 done */
} ebt_sharded_pending;
int ebt_cosine_topk_sharded_submit(const ebt_catalog* cat, const ebt_comm* comm, const void* q,
                                   int q_dtype, int64_t B, int64_t ldq,
                                   const int64_t* liked_off, const int64_t* liked_rows,
                                   int32_t k, const int64_t* excl_off, const int64_t* excl_rows,
                                   const ebt_options* opt, void* workspace, size_t ws_bytes,
                                   double* out_scores, int64_t* out_rows, int32_t* host,
                                   ebt_sharded_pending* pending, void* timer, void* stream);
int ebt_cosine_topk_sharded_finish(ebt_sharded_pending* pending);
int ebt_cosine_topk_sharded_wait(ebt_sharded_pending* pending);
int ebt_cosine_topk_sharded(const ebt_catalog* cat, const ebt_comm* comm, const void* q,
                            int q_dtype, int64_t B, int64_t ldq, const int64_t* liked_off,
                            const int64_t* liked_rows, int32_t k, const int64_t* excl_off,
                            const int64_t* excl_rows, const ebt_options* opt, void* workspace,
                            size_t ws_bytes, double* out_scores, int64_t* out_rows, void* timer,
                            void* stream);

/* ---- two-phase top-k over a row-sharded catalog (robot_ebert_amd/distributed.py) ---------
 * Phase 1, every rank: ebt_cosine_screen = ebt_cosine_topk_prepared without the rescore: the shard's k'
 * best approx candidates, list_vals (f32) / list_rows (GLOBAL, -1 empty) [B][kprime]
 * partitioned at k as ebt_merge_hits describes (sorted when the unfused path ran),
 * ovf_out[b] = 1 when the fused screen overflowed for b, eps_out = the eps the certificate
 * must use. The ranks all-gather the lists and keep the k' best of all shards
 * (ebt_select_topk over [B][R*kprime] with the rows as indices).
 * Phase 2: ebt_rescore_owned writes the exact float64 score of every merged candidate whose
 * row is in [row_offset, row_offset + n_rows) and whose approx is >= approx[k-1] - 2 eps, 0.0
 * for the rest; an all-reduce (SUM) of `exact` completes it; ebt_finalize_topk sorts the
 * candidates above the cut by (exact desc, row asc) into out_scores/out_rows [B][k] and
 * certifies like ebt_rescore (ovf = the all-reduced (MAX) overflow flags -> certified -1). */
int ebt_cosine_screen(const double* q64, const void* qimg, const float* qscale, const float* eps,
                      int64_t B, int64_t B_pad, const void* cat, int dtype, int64_t ld,
                      const double* gnorm64, const void* cimg, const float* cscale, int img_dtype,
                      int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad, int64_t row_offset,
                      const int64_t* excl_off, const int64_t* excl_rows, int32_t k, int32_t kprime,
                      int64_t chunk_rows, int flags, void* workspace, size_t ws_bytes,
                      float* list_vals, int64_t* list_rows, int32_t* ovf_out, float* eps_out,
                      void* timer, void* stream);
/* ---- shared screening threshold over a row-sharded catalog (distributed.py) -------------
 * The per-shard path (every rank: its exact top-k, then one all-gather + ebt_merge_topk)
 * screens every shard at ONE catalog-wide threshold instead of each shard's own:
 *   1. ebt_cosine_sample: `tiles` full 256-row tiles of this shard, `tile_stride` tiles apart
 *      from tile 0, through the screening GEMM keeping only the max of every 64-row subgroup:
 *      pooled[b * ld_pooled + 4 t + s] (B_pad rows, 4 * tiles maxima each; B_pad % 256 == 0).
 *   2. the ranks all-gather the maxima; ebt_pool_kth: theta[b] = the j-th largest of the G
 *      values pooled[b * ld + 0 .. G) (G <= 2048), -inf when fewer than j are >= -inf;
 *      theta[b] = +inf for B <= b < B_pad.
 *   3. ebt_cosine_screen_at = ebt_cosine_screen with the filter threshold theta[b] (device,
 *      [B]) instead of the shard's own sample estimate, `hits` = the expected hits per query on
 *      this shard (segment sizing). The list then holds this shard's rows with approx >= theta
 *      (and >= the list's own k-th - 2 eps once it has k rows): often fewer than k. Rows below
 *      theta are not screened out silently: theta is NOT checked here -- the caller must
 *      verify theta[b] <= t_floor[b] - eps[b] with the catalog-wide floor it passes to
 *      ebt_rescore, and rerun a query that fails (unfused, locally). kprime <= 512.
 * Replaces nothing in the reference (no sharding there). */
int ebt_cosine_sample(const void* qimg, const float* qscale, int64_t B_pad, const void* cimg,
                      const float* cscale, int img_dtype, int32_t ld_img, int64_t n_rows,
                      int32_t d_pad, int64_t tiles, int64_t tile_stride, float* pooled,
                      int64_t ld_pooled, void* timer, void* stream);
int ebt_pool_kth(const float* pooled, int64_t ld, int64_t B, int64_t B_pad, int32_t G, int32_t j,
                 float* theta, void* stream);
int ebt_cosine_screen_at(const double* q64, const void* qimg, const float* qscale,
                         const float* eps, int64_t B, int64_t B_pad, const void* cat, int dtype,
                         int64_t ld, const double* gnorm64, const void* cimg, const float* cscale,
                         int img_dtype, int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad,
                         int64_t row_offset, const int64_t* excl_off, const int64_t* excl_rows,
                         int32_t k, int32_t kprime, int64_t chunk_rows, int flags,
                         void* workspace, size_t ws_bytes, float* list_vals, int64_t* list_rows,
                         int32_t* ovf_out, float* eps_out, const float* theta, double hits,
                         void* timer, void* stream);
/* The same two calls with a LEAD (0.3.1; lead = 0 is the calls above): the sample's first `lead`
 * tiles are the shard's first `lead` tiles (rows 0 .. 256 lead), the other tiles - lead follow
 * from tile `lead` on, `tile_stride` apart, and the lead tiles' scores are kept in
 * lead_scores[b * ld_lead + r] (ld_lead >= 256 lead). ebt_cosine_screen_at_lead takes the lead's
 * hits at theta from those scores and filters rows 256 lead .. n_rows only, so that the shard's
 * filter launches cover whole rounds of the persistent grid (driver.hip: the C ABI's sharded
 * step picks lead = ceil(n/256) mod (catalog tiles per round); 0 turns it off). */
int ebt_cosine_sample_lead(const void* qimg, const float* qscale, int64_t B_pad,
                           const void* cimg, const float* cscale, int img_dtype, int32_t ld_img,
                           int64_t n_rows, int32_t d_pad, int64_t tiles, int64_t tile_stride,
                           float* pooled, int64_t ld_pooled, int64_t lead, float* lead_scores,
                           int64_t ld_lead, void* timer, void* stream);
int ebt_cosine_screen_at_lead(const double* q64, const void* qimg, const float* qscale,
                              const float* eps, int64_t B, int64_t B_pad, const void* cat,
                              int dtype, int64_t ld, const double* gnorm64, const void* cimg,
                              const float* cscale, int img_dtype, int32_t ld_img, int64_t n_rows,
                              int32_t d, int32_t d_pad, int64_t row_offset,
                              const int64_t* excl_off, const int64_t* excl_rows, int32_t k,
                              int32_t kprime, int64_t chunk_rows, int flags, void* workspace,
                              size_t ws_bytes, float* list_vals, int64_t* list_rows,
                              int32_t* ovf_out, float* eps_out, const float* theta, double hits,
                              int64_t lead, const float* lead_scores, int64_t ld_lead,
                              void* timer, void* stream);
/* After the floor all-gather of the per-shard path: g = [R][B][ld] float32 (each shard's k best
 * approx in columns [0, ld-1), its eps in column ld-1) ->
 * t_floor[b] = the k-th largest of g[r][b][j] - g[r][b][ld-1] over all r and j < ld-1, in float64
 * (NaN counts as -inf): a lower bound of query b's k-th best exact score over the catalog. */
int ebt_union_floor(const float* gathered, int32_t R, int64_t B, int32_t ld, int32_t k,
                    double* t_floor, void* stream);
/* What a shard sends for that floor: out[b] = (the w largest of list_vals[b*ld + 0 .. n),
 * n = min(k_eff, ld), -inf padded to w; then eps[b], or -inf when eps is NULL) as [B][w + 1]
 * float32. The list may be
 * partitioned (any order): the w largest are selected. w = ebt_shard_list_width(k, world)
 * narrows the gather: the k-th largest over a subset of the shards' values is still a lower
 * bound, and with w >= a shard's share of the global top k it is the same bound. */
int ebt_floor_pack(const float* list_vals, int64_t ld, int64_t B, int32_t k_eff, int32_t w,
                   const float* eps, float* out, void* stream);
/* cert[b] = -1 (rerun unfused) where ovf[b] != 0, or where theta (if not NULL) may have dropped
 * a global top-k row: !(theta[b] <= t_floor[b] - eps[b]); a -2 (corrupt list) stays. */
int ebt_certify_cut(int32_t* cert, const int32_t* ovf, const float* theta,
                    const double* t_floor, const float* eps, int64_t B, void* stream);
int ebt_rescore_owned(const double* q64, int64_t B, int32_t d, const void* cat, int dtype,
                      int64_t ld, const double* gnorm64, int64_t row_offset, int64_t n_rows,
                      const float* cand_vals, const int64_t* cand_rows, int32_t kprime, int32_t k,
                      const float* eps, double* exact, void* stream);
int ebt_finalize_topk(const float* cand_vals, const int64_t* cand_rows, const double* exact,
                      int64_t B, int32_t kprime, int32_t k, int64_t n_rows_global,
                      const float* eps, const int32_t* ovf, double* out_scores, int64_t* out_rows,
                      int32_t* certified, void* stream);

/* ---- implicit-feedback ALS (offline factor training) ---------
 * Replaces pyspark.ml ALS(rank=32, maxIter=15, regParam=0.1, implicitPrefs=True) of
 * notebooks/create-embeddings.ipynb:1055 (Spark ALS.scala computeFactors, implicit branch).
 * ebt_als_gram: out[i*rank + j] = sum_r Y[r*rank + i] * Y[r*rank + j] (float64), Y n x rank f32.
 * ebt_als_solve: for every destination u (users from item factors Y, or items from user
 *   factors), with its ratings src[off[u] .. off[u+1]) / rating[...] (CSR):
 *     A = YtY + sum alpha|r| y y^T + reg * n_pos I,  b = sum_{r > 0} (1 + alpha|r|) y,
 *     X[u*rank ..] = (float) A^-1 b  (Cholesky in float64; n_pos = #ratings > 0).
 *   rank <= 64. */
int ebt_als_gram(const float* Y, int64_t n, int32_t rank, double* out, void* stream);
int ebt_als_solve(const double* YtY, const float* Y, int32_t rank, int64_t n_dst,
                  const int64_t* off, const int32_t* src, const float* rating, float alpha,
                  float reg, float* X, void* stream);

/* ---- per-stage GPU timing (hipEvents recorded on the launch stream) -----------------------
 * Stages: 0 screening GEMM (score-writing), 1 exclusion mask, 2 chunk select, 3 candidate
 * select (across chunks / head + fused tail), 4 rescore, 5 fused screening GEMM (filtering),
 * and the caller-bracketed stages of a row-sharded step: 6 query prep, 7 merge of the gathered
 * shard results, 8 stream stalls on collectives, 9 small per-batch kernels (thresholds, floors,
 * certificate checks).
 * ebt_timer_query synchronises the recorded events and returns the total milliseconds and the
 * number of launches of `stage` since the last reset. Host pointers.
 * ebt_timer_begin / ebt_timer_end bracket a caller's region of `stream` as one record of
 * `stage` (at most one open region per stage; nothing is recorded for a masked stage). */
#define EBT_STAGE_GEMM 0
#define EBT_STAGE_MASK 1
#define EBT_STAGE_SELECT 2
#define EBT_STAGE_MERGE_SELECT 3
#define EBT_STAGE_RESCORE 4
#define EBT_STAGE_GEMM_FILTER 5
#define EBT_STAGE_PREP 6
#define EBT_STAGE_SHARD_MERGE 7
#define EBT_STAGE_COLLECTIVE 8
#define EBT_STAGE_SMALL 9
#define EBT_NUM_STAGES 10
void* ebt_timer_create(void);
void ebt_timer_destroy(void* timer);
int ebt_timer_reset(void* timer);
/* Record only the stages whose bit (1 << EBT_STAGE_*) is set (default: all). */
int ebt_timer_set_mask(void* timer, uint32_t stage_mask);
int ebt_timer_query(void* timer, int stage, double* total_ms, int64_t* launches);
int ebt_timer_begin(void* timer, int stage, void* stream);
int ebt_timer_end(void* timer, int stage, void* stream);
/* Row accounting for the top-K roofline (bench.py `roofline_topk`): with on != 0 the timer owns
 * one device counter (allocated on the current device) to which every rescore kernel recorded
 * under EBT_STAGE_RESCORE on a stream of that device adds the candidate rows it gathered (one
 * atomic per query; launches on another device's streams are not counted, 0.3.2);
 * ebt_timer_reset zeroes it, ebt_timer_rows reads it (on the counter's device whatever device
 * is current; synchronise the launch streams first).
 * on = 0 frees it. Costs nothing when off. */
int ebt_timer_count_rows(void* timer, int on);
int ebt_timer_rows(void* timer, int64_t* rows);

#ifdef __cplusplus
}
#endif
#endif /* EBERT_H_ */
