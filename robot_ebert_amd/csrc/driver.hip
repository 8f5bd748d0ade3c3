// The self-contained C-ABI path (include/ebert.h: ebt_catalog_init, ebt_workspace_bytes,
// ebt_cosine_topk{,_submit,_finish}): what a caller without Python binds in place of
// /root/reference/src/backend/app/lib.py:51-55 (and the resident catalog of constants.py:55-56).
//
// One batch = query prep (ebt_query_prep / ebt_query_liked_sum + ebt_query_image) -> the
// prepared-query pipeline (ebt_cosine_topk_prepared: screen + exact float64 rescore +
// certificate) -> on the host, after ONE wait for this batch's certificates, the retries:
//   certified -1 (a fused candidate list overflowed, or the speculative threshold was wrong)
//                -> the query again with EBT_FLAG_NO_FUSE at the same k';
//   certified  0 (more than k' rows inside the screen's error band) -> k' x 4 up to 4096, then
//                the float64 screen (EBT_FLAG_EXACT); still 0 there is an error (more than
//                4096 rows tied at f32 resolution), never a silent approximation;
//   certified -2 (a corrupt candidate row) -> error.
// Retried queries are gathered into groups of at most RETRY_GROUP (their prepared rows, their
// exclusion segments), run through the same pipeline and scattered back. Everything lives in
// the caller's workspace; the library allocates no device memory.
#include <cmath>
#include <cstring>
#include <vector>

#include "common.h"

namespace ebt {

int query_liked_sum(const void*, int, int32_t, int64_t, const double*, int64_t, const int64_t*,
                    const int64_t*, double*, hipStream_t, int64_t row_offset, int64_t n_local);
size_t large_topk_bytes(int64_t B, int64_t n, int64_t* Bg_out);
int large_topk(const double*, int64_t, int32_t, const void*, int, int64_t, const double*, int64_t,
               int64_t, const int64_t*, const int64_t*, int32_t, double*, int64_t*, void*, size_t,
               hipStream_t);
int rescore_sharded(const double*, int64_t, int32_t, const void*, int, int64_t, const double*,
                    int64_t, const float*, const int64_t*, int32_t, int32_t, int64_t, const float*,
                    const double*, double*, int64_t*, int32_t*, const int*, const float*, void*,
                    hipStream_t, int64_t list_base, const int64_t* excl_off,
                    const int64_t* excl_rows, const ShardPackOut* pack);
int union_floor(const float* gathered, int32_t R, int64_t B, int32_t ld, int32_t k,
                double* t_floor, hipStream_t stream, uint32_t* zero2);
int shard_pack_lens(const double* scores, const int64_t* rows, int64_t B, int32_t k,
                    int64_t cap, void* send, hipStream_t st);
int screen_at_local(const double*, const void*, const float*, const float*, int64_t, int64_t,
                    const void*, int, int64_t, const double*, const void*, const float*, int,
                    int32_t, int64_t, int32_t, int32_t, int64_t, const int64_t*, const int64_t*,
                    int32_t, int32_t, int64_t, void*, size_t, float*, int64_t*, const float*,
                    int64_t, int, int, int, double, int64_t, const float*, int64_t, const float**,
                    const int**, const float**, void*, hipStream_t, float* floor_out,
                    int floor_w);
int pool_kth(const float*, int64_t, int64_t, int64_t, int, int, float*, hipStream_t, float*,
             int64_t*, int, int*, const float*, int64_t, int, uint64_t*, int64_t, int, uint8_t*,
             int64_t, int, int64_t);

namespace {

constexpr int64_t KPRIME_MAX = 4096;
constexpr int64_t QUERY_PREP_MAX_D = 4096;
constexpr int64_t SCORE_BUDGET = 4LL << 30;   // f32 score bytes of the unfused path per pass
constexpr int64_t RETRY_GROUP = 256;          // queries per retry pass
constexpr int64_t RETRY_BUDGET = 256LL << 20; // f32 score bytes of a retry pass
constexpr int64_t RETRY_EXCL_MAX = 1LL << 20; // gathered exclusion rows per retry pass

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

// The caller's certificate buffer, seen from the device when it is pinned host memory
// (hipHostMalloc / hipHostRegister, e.g. a torch pin_memory tensor): the rescore then stores each
// query's certificate straight into it -- one 4-byte store per query across the host link, no
// copy launch behind the kernels (a D2H copy is a blit kernel here: ~4 us plus its boundary, 2 %
// of a C2 batch). Anything else (pageable memory) -> nullptr: the workspace's certificates and
// one hipMemcpyAsync, as before. EBT_HOST_DIRECT=0 keeps the copy (A/B).
int32_t* host_mapped(int32_t* host) {
  static const bool on = [] {
    const char* v = getenv("EBT_HOST_DIRECT");
    return !(v && v[0] == '0');
  }();
  void* dp = nullptr;
  if (!on || !host) return nullptr;
  if (hipHostGetDevicePointer(&dp, host, 0) != hipSuccess || !dp) {
    (void)hipGetLastError();  // (pageable memory: clear the query's error for later checks)
    return nullptr;
  }
  return (int32_t*)dp;
}
// written by the host into a directly delivered certificate buffer before the kernels run: a
// value that is still there when the batch's event has passed was never delivered (the finish
// fails loudly instead of reading a previous batch's leftovers as certificates)
constexpr int32_t CERT_UNSET = 0x7fffffff;

int64_t pad_batch(int64_t B) {
  B = B < 1 ? 1 : B;
  return B <= 128 ? round_up(B, 128) : round_up(B, 256);
}

// search.py default_kprime: the rows inside the 2 eps band around the k-th score grow with k;
// native images have the smaller band
int32_t default_kprime(const ebt_catalog& c, int64_t k_eff) {
  int64_t kp = c.native ? k_eff + (k_eff / 4 > 16 ? k_eff / 4 : 16)
                        : (2 * k_eff > k_eff + 32 ? 2 * k_eff : k_eff + 32);
  kp = round_up(kp, 8);
  kp = kp < KPRIME_MAX ? kp : KPRIME_MAX;
  int64_t lo = round_up(k_eff, 4), hi = round_up(c.n, 4);
  kp = round_up(kp, 4);
  kp = kp < hi ? kp : hi;
  kp = kp < KPRIME_MAX ? kp : KPRIME_MAX;
  return (int32_t)(kp > lo ? kp : lo);
}

int64_t chunk_rows(const ebt_catalog& c, int64_t B_pad, int64_t budget) {
  int64_t rows = budget / (4 * B_pad);
  rows = rows / 128 * 128;
  rows = rows < 128 ? 128 : rows;
  const int64_t cap = round_up(c.n, 128);
  return rows < cap ? rows : cap;
}

int elem_size(int dt) { return dt == EBT_F64 ? 8 : dt == EBT_F32 ? 4 : 2; }

// Per-batch prepared queries (the ebt_query_* outputs) for `rows` queries.
struct PrepLayout {
  size_t q64, qimg, qscale, eps, bytes;
};
PrepLayout prep_layout(const ebt_catalog& c, int64_t rows) {
  const int64_t rp = pad_batch(rows);
  PrepLayout p{};
  size_t o = 0;
  p.q64 = o;
  o = al(o + (size_t)rows * c.d * 8);
  p.qimg = o;
  o = al(o + (size_t)rp * c.ld_img * 2);
  p.qscale = o;
  o = al(o + (size_t)rp * 4);
  p.eps = o;
  o = al(o + (size_t)rp * 4);
  p.bytes = o;
  return p;
}

// The whole workspace of one batch:
//   [prep B] [pass: max(first pass, every retry pass)] [results k_eff < k] [cert B + flag]
//   [retry: prep R, results R x k_eff, cert R, gather indices, exclusion CSR of the group]
// large: min(k, n) > 4096, the full-sort path (large_k.hip): [prep B] [sort buffers] [cert B + flag]
struct DriverLayout {
  int64_t B, B_pad, R, chunk, chunk_r;
  int32_t k_eff, kprime, flags;
  bool large;
  PrepLayout prep, prep_r;
  size_t off_prep, off_pass, pass_bytes, off_res_s, off_res_r, off_cert, off_rprep, off_rs,
      off_rr, off_rcert, off_idx, off_roff, off_rrows, off_big, big_bytes, bytes;
};

bool driver_layout(const ebt_catalog& c, int64_t B, int32_t k, const ebt_options& opt,
                   DriverLayout* L) {
  if (B < 1 || k < 1 || c.n < 1 || opt.kprime < 0 || opt.chunk_rows < 0 ||
      (opt.chunk_rows && opt.chunk_rows % 128) ||
      (opt.flags & ~(EBT_FLAG_NO_FUSE | EBT_FLAG_LIKED_CHECKED)))
    return false;
  DriverLayout& D = *L;
  D = DriverLayout{};
  D.B = B;
  D.B_pad = pad_batch(B);
  D.k_eff = (int32_t)(k < c.n ? k : c.n);
  if (D.k_eff > KPRIME_MAX) {  // beyond the screen's k' range: every score, a full sort
    const size_t big = large_topk_bytes(B, c.n, nullptr);
    if (big == 0) return false;
    D.large = true;
    D.flags = opt.flags & EBT_FLAG_NO_FUSE;  // (LIKED_CHECKED: the submit's, not the screen's)
    D.prep = prep_layout(c, B);
    size_t o = 0;
    D.off_prep = o;
    o = al(o + D.prep.bytes);
    D.off_big = o;
    D.big_bytes = big > (size_t)B * 8 ? big : (size_t)B * 8;  // also the liked path's scratch
    o = al(o + D.big_bytes);
    D.off_cert = o;
    o = al(o + (size_t)(B + 1) * 4);
    D.bytes = o;
    return true;
  }
  D.kprime = default_kprime(c, D.k_eff);
  if (opt.kprime) {  // search.py's clamp: [round_up(k, 4), min(round_up(n, 4), 4096)]
    int64_t kp = round_up(opt.kprime, 4), hi = round_up(c.n, 4), lo = round_up(D.k_eff, 4);
    kp = kp < hi ? kp : hi;
    kp = kp < KPRIME_MAX ? kp : KPRIME_MAX;
    D.kprime = (int32_t)(kp > lo ? kp : lo);
  }
  D.flags = opt.flags & EBT_FLAG_NO_FUSE;  // (LIKED_CHECKED: the submit's, not the screen's)
  D.chunk = opt.chunk_rows ? opt.chunk_rows : chunk_rows(c, D.B_pad, SCORE_BUDGET);
  D.R = B < RETRY_GROUP ? B : RETRY_GROUP;
  const int64_t R_pad = pad_batch(D.R);
  D.chunk_r = opt.chunk_rows ? opt.chunk_rows : chunk_rows(c, R_pad, RETRY_BUDGET);
  size_t pass = ebt_cosine_topk_workspace(B, D.B_pad, c.n, D.kprime, D.chunk, D.flags);
  if (pass == 0) return false;
  // every retry configuration: k' from the first pass up to 4096 (x 4 steps), fused or not,
  // and the float64 screen from the default k' up
  const int64_t kcap = round_up(c.n, 4) < KPRIME_MAX ? round_up(c.n, 4) : KPRIME_MAX;
  const int fl[3] = {D.flags, EBT_FLAG_NO_FUSE, EBT_FLAG_EXACT};
  for (int f = 0; f < 3; ++f) {
    for (int64_t kp = D.kprime;; kp = kp * 4 < kcap ? kp * 4 : kcap) {
      const size_t w = ebt_cosine_topk_workspace(D.R, R_pad, c.n, (int32_t)kp, D.chunk_r, fl[f]);
      if (w == 0) return false;
      pass = w > pass ? w : pass;
      if (kp >= kcap) break;
    }
  }
  D.prep = prep_layout(c, B);
  D.prep_r = prep_layout(c, D.R);
  size_t o = 0;
  D.off_prep = o;
  o = al(o + D.prep.bytes);
  D.off_pass = o;
  D.pass_bytes = pass;
  o = al(o + pass);
  D.off_res_s = o;
  if (D.k_eff < k) o = al(o + (size_t)B * D.k_eff * 8);
  D.off_res_r = o;
  if (D.k_eff < k) o = al(o + (size_t)B * D.k_eff * 8);
  D.off_cert = o;
  o = al(o + (size_t)(B + 1) * 4);
  D.off_rprep = o;
  o = al(o + D.prep_r.bytes);
  D.off_rs = o;
  o = al(o + (size_t)D.R * D.k_eff * 8);
  D.off_rr = o;
  o = al(o + (size_t)D.R * D.k_eff * 8);
  D.off_rcert = o;
  o = al(o + (size_t)D.R * 4);
  D.off_idx = o;
  o = al(o + (size_t)D.R * 8);
  D.off_roff = o;
  o = al(o + (size_t)(D.R + 1) * 8);
  D.off_rrows = o;
  o = al(o + (size_t)RETRY_EXCL_MAX * 8);
  D.bytes = o;
  return true;
}

// ------------------------------------------------------------------------------ kernels ----
// dst row i <- src row idx[i] (gather) or dst row idx[i] <- src row i (scatter), 4-byte words
__global__ void move_rows_kernel(const uint32_t* __restrict__ src, int64_t src_ld,
                                 uint32_t* __restrict__ dst, int64_t dst_ld,
                                 const int64_t* __restrict__ idx, int64_t n, int64_t words,
                                 int scatter) {
  const int64_t total = n * words;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / words, w = t - i * words;
    if (scatter) dst[idx[i] * dst_ld + w] = src[i * src_ld + w];
    else dst[i * dst_ld + w] = src[idx[i] * src_ld + w];
  }
}

int move_rows(const void* src, int64_t src_ld_bytes, void* dst, int64_t dst_ld_bytes,
              const int64_t* idx, int64_t n, int64_t row_bytes, bool scatter, hipStream_t st) {
  if (n == 0) return EBT_OK;
  const int64_t words = row_bytes / 4, total = n * words;
  int64_t blocks = (total + 255) / 256;
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(move_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const uint32_t*)src, src_ld_bytes / 4, (uint32_t*)dst, dst_ld_bytes / 4,
                     idx, n, words, scatter ? 1 : 0);
  return launch_check("move_rows_kernel");
}

// the exclusion segments of the retried queries, gathered (new offsets computed on the host)
__global__ void csr_gather_kernel(const int64_t* __restrict__ off, const int64_t* __restrict__ rows,
                                  const int64_t* __restrict__ idx,
                                  const int64_t* __restrict__ new_off, int64_t* __restrict__ out) {
  const int64_t i = blockIdx.x;
  const int64_t s = off[idx[i]], n = new_off[i + 1] - new_off[i];
  for (int64_t t = threadIdx.x; t < n; t += blockDim.x) out[new_off[i] + t] = rows[s + t];
}

// out[b][j] = j < k_eff ? res[b][j] : NaN / -1
__global__ void pad_results_kernel(const double* __restrict__ rs, const int64_t* __restrict__ rr,
                                   int64_t B, int k_eff, int k, double* __restrict__ os,
                                   int64_t* __restrict__ orow) {
  const int64_t total = B * k;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / k, j = t - b * k;
    os[t] = j < k_eff ? rs[b * k_eff + j] : __builtin_nan("");
    orow[t] = j < k_eff ? rr[b * k_eff + j] : -1;
  }
}

// flag[0] = 1 when some exclusion segment is not sorted ascending (the fused merge drops
// excluded rows by binary search); one block per query
__global__ void csr_sorted_kernel(const int64_t* __restrict__ off, const int64_t* __restrict__ rows,
                                  int32_t* __restrict__ flag) {
  const int64_t b = blockIdx.x;
  const int64_t s = off[b], e = off[b + 1];
  bool bad = e < s;
  for (int64_t t = s + threadIdx.x; t + 1 < e; t += blockDim.x) bad |= rows[t] > rows[t + 1];
  if (bad) flag[0] = 1;
}

int prep_dense(const ebt_catalog& c, const void* q, int q_dtype, int64_t B, int64_t ldq,
               const PrepLayout& P, char* base, hipStream_t st) {
  double* q64 = (double*)(base + P.q64);
  void* qimg = base + P.qimg;
  float* qscale = (float*)(base + P.qscale);
  float* eps = (float*)(base + P.eps);
  const int64_t B_pad = pad_batch(B);
  const int native_q = c.native && q_dtype == c.img_dtype;
  if (c.d <= QUERY_PREP_MAX_D)
    return ebt_query_prep(q, q_dtype, B, B_pad, c.d, ldq, c.img_dtype, native_q, c.u_cat, q64,
                          qimg, c.ld_img, qscale, eps, st);
  int rc = ebt_query_dense(q, q_dtype, B, c.d, ldq, q64, st);
  if (rc) return rc;
  return ebt_query_image(q64, B, B_pad, c.d, c.img_dtype, native_q ? q : nullptr,
                         native_q ? ldq : 0, native_q, c.u_cat, qimg, c.ld_img, qscale, eps, st);
}

// q64[b] *= 1 / (off[b+1] - off[b]): the 1/L of lib.py:52 from the liked CSR's offsets (the
// same float64 scale the host computes, then the same product as scale_rows_kernel)
__global__ void scale_by_count_kernel(double* __restrict__ q64, int64_t total, int d,
                                      const int64_t* __restrict__ off) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / d;
    const double s = 1.0 / (double)(off[b + 1] - off[b]);
    q64[t] *= s;
  }
}

// liked path: validated on the host (counts >= 1 with sklearn's message, rows in the catalog),
// unless the caller did (EBT_FLAG_LIKED_CHECKED): then nothing is read back
int prep_liked(const ebt_catalog& c, const int64_t* off, const int64_t* rows, int64_t B,
               const PrepLayout& P, char* base, char* scratch, size_t scratch_bytes,
               hipStream_t st, bool checked) {
  if (checked) {
    double* q64 = (double*)(base + P.q64);
    int rc = query_liked_sum(c.data, c.dtype, c.d, c.ld, c.gnorm64, B, off, rows, q64, st,
                             c.row_offset, 0);
    if (rc) return rc;
    int64_t blocks = ceil_div(B * c.d, 256);
    blocks = blocks > 8192 ? 8192 : blocks;
    hipLaunchKernelGGL(scale_by_count_kernel, dim3((unsigned)blocks), dim3(256), 0, st, q64,
                       B * c.d, c.d, off);
    rc = launch_check("scale_by_count_kernel");
    if (rc) return rc;
    return ebt_query_image(q64, B, pad_batch(B), c.d, c.img_dtype, nullptr, 0, 0, c.u_cat,
                           base + P.qimg, c.ld_img, (float*)(base + P.qscale),
                           (float*)(base + P.eps), st);
  }
  std::vector<int64_t> h_off(B + 1);
  int rc = hip_check(hipMemcpyAsync(h_off.data(), off, (B + 1) * 8, hipMemcpyDeviceToHost, st),
                     "hipMemcpyAsync");
  if (!rc) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (rc) return rc;
  const int64_t nnz = h_off[B] - h_off[0];
  std::vector<double> scale(B);
  for (int64_t b = 0; b < B; ++b) {
    const int64_t cnt = h_off[b + 1] - h_off[b];
    if (cnt <= 0) {
      set_error("Found array with 0 sample(s) (shape=(0, %d)) while a minimum of 1 is required "
                "by check_pairwise_arrays.", c.d);
      return EBT_EINVAL;
    }
    scale[b] = 1.0 / (double)cnt;
  }
  if (nnz > 0) {
    std::vector<int64_t> h_rows(nnz);
    rc = hip_check(hipMemcpy(h_rows.data(), rows + h_off[0], nnz * 8, hipMemcpyDeviceToHost),
                   "hipMemcpy");
    if (rc) return rc;
    for (int64_t r : h_rows)
      if (r < c.row_offset || r >= c.row_offset + c.n) {
        set_error("liked row %lld is not in the catalog rows [%lld, %lld)", (long long)r,
                  (long long)c.row_offset, (long long)(c.row_offset + c.n));
        return EBT_EINVAL;
      }
  }
  if (scratch_bytes < (size_t)B * 8) {
    set_error("ebt_cosine_topk: workspace too small for the liked-query scales");
    return EBT_ENOMEM;
  }
  double* d_scale = (double*)scratch;
  rc = hip_check(hipMemcpy(d_scale, scale.data(), B * 8, hipMemcpyHostToDevice), "hipMemcpy");
  if (rc) return rc;
  double* q64 = (double*)(base + P.q64);
  rc = query_liked_sum(c.data, c.dtype, c.d, c.ld, c.gnorm64, B, off, rows, q64, st,
                       c.row_offset, 0);
  if (!rc) rc = ebt_scale_rows_f64(q64, B, c.d, d_scale, st);
  if (rc) return rc;
  return ebt_query_image(q64, B, pad_batch(B), c.d, c.img_dtype, nullptr, 0, 0, c.u_cat,
                         base + P.qimg, c.ld_img, (float*)(base + P.qscale),
                         (float*)(base + P.eps), st);
}

int run_prepared(const ebt_catalog& c, const PrepLayout& P, char* base, int64_t B,
                 const int64_t* excl_off, const int64_t* excl_rows, int32_t k_eff, int32_t kp,
                 int64_t chunk, int flags, char* pass, size_t pass_bytes, double* out_s,
                 int64_t* out_r, int32_t* cert, void* timer, hipStream_t st) {
  const bool exact = flags & EBT_FLAG_EXACT;
  return ebt_cosine_topk_prepared(
      (const double*)(base + P.q64), exact ? nullptr : base + P.qimg,
      exact ? nullptr : (const float*)(base + P.qscale),
      exact ? nullptr : (const float*)(base + P.eps), B, pad_batch(B), c.data, c.dtype, c.ld,
      c.gnorm64, c.image, c.cscale, c.img_dtype, c.ld_img, c.n, c.d, c.d_pad, c.row_offset,
      excl_off, excl_rows, k_eff, kp, chunk, flags, pass, pass_bytes, out_s, out_r, cert, timer,
      st);
}

bool valid_catalog(const ebt_catalog* c) {
  return c && c->data && c->gnorm64 && c->image && c->n > 0 && c->d > 0 && c->ld >= c->d &&
         c->d_pad % 64 == 0 && c->d_pad >= c->d && c->ld_img >= c->d_pad;
}

}  // namespace

int screen_image(const void*, int, int64_t, int32_t, int64_t, const double*, int, int, void*,
                 int32_t, hipStream_t, unsigned int* err_max);
int64_t shard_lead_tiles(int64_t B_pad, int64_t n_rows, int64_t sample_tiles);
int64_t shard_lead_room(int64_t B_pad, int64_t n_rows, int64_t sample_tiles);

}  // namespace ebt

using namespace ebt;

extern "C" {

size_t ebt_catalog_state_bytes(const void* data, int dtype, int64_t n, int32_t d, int64_t ld) {
  if (n < 1 || d < 1 || ld < d || dtype < 0 || dtype > 3) return 0;
  const int64_t d_pad = round_up(d, 64);
  const bool native = dtype == EBT_F16 || dtype == EBT_BF16;
  const bool alias = native && d % 64 == 0 && ld % 64 == 0 && ((uintptr_t)data & 15) == 0;
  size_t o = al((size_t)n * 8) + al((size_t)round_up(n, 128) * 4);
  if (!alias) o += al((size_t)n * d_pad * 2);
  if (!native) o += al(4);  // the image's measured rounding error (ebt_catalog_init)
  return o;
}

int ebt_catalog_init(ebt_catalog* cat, const void* data, int dtype, int64_t n, int32_t d,
                     int64_t ld, int64_t row_offset, void* state, size_t state_bytes,
                     void* stream) {
  const size_t need = ebt_catalog_state_bytes(data, dtype, n, d, ld);
  if (!cat || !data || !state || need == 0 || row_offset < 0) {
    set_error("ebt_catalog_init: bad arguments (n=%lld d=%d ld=%lld dtype=%d)", (long long)n, d,
              (long long)ld, dtype);
    return EBT_EINVAL;
  }
  if (state_bytes < need) {
    set_error("ebt_catalog_init: state %zu < %zu bytes", state_bytes, need);
    return EBT_ENOMEM;
  }
  hipStream_t st = (hipStream_t)stream;
  ebt_catalog c{};
  c.data = data;
  c.dtype = dtype;
  c.d = d;
  c.n = n;
  c.ld = ld;
  c.row_offset = row_offset;
  c.d_pad = (int32_t)round_up(d, 64);
  char* s = (char*)state;
  c.gnorm64 = (double*)s;
  c.inv32 = (float*)(s + al((size_t)n * 8));
  char* img = s + al((size_t)n * 8) + al((size_t)round_up(n, 128) * 4);
  const float one = 1.0f;
  uint32_t one_bits;
  memcpy(&one_bits, &one, 4);
  int rc = EBT_OK;
  if (round_up(n, 128) > n)
    rc = hip_check(hipMemsetD32Async((hipDeviceptr_t)(c.inv32 + n), (int)one_bits,
                                     (size_t)(round_up(n, 128) - n), st), "hipMemsetD32Async");
  if (!rc) rc = ebt_row_norms(data, dtype, n, d, ld, c.gnorm64, c.inv32, st);
  if (rc) return rc;
  const bool native = dtype == EBT_F16 || dtype == EBT_BF16;
  if (native) {
    c.img_dtype = dtype;
    c.u_cat = 0.0f;
    c.cscale = c.inv32;
    c.native = 1;
    if (d % 64 == 0 && ld % 64 == 0 && ((uintptr_t)data & 15) == 0) {
      c.image = data;  // the matrix itself is the MFMA operand
      c.ld_img = (int32_t)ld;
    } else {
      c.ld_img = c.d_pad;
      c.image = img;
      rc = ebt_screen_image(data, dtype, n, d, ld, c.gnorm64, 0, c.img_dtype, img, c.ld_img, st);
    }
  } else {
    // f16 image of the normalised rows. u_cat = the largest ||image row - row / gnorm||_2 over
    // the rows, measured by the image kernel (rounded up to a float; rows with non-finite
    // values left out) -- ~0.4 x the unit round-off 2^-11 that bounds it a priori, so the
    // certificate's eps band (and the rows the rescore gathers) is about half as wide; one
    // stream sync to read it back, once per catalog
    c.img_dtype = EBT_F16;
    c.cscale = nullptr;
    c.native = 0;
    c.ld_img = c.d_pad;
    c.image = img;
    unsigned int* d_err = (unsigned int*)(img + al((size_t)n * c.d_pad * 2));
    unsigned int h_err = 0;
    rc = hip_check(hipMemsetAsync(d_err, 0, 4, st), "hipMemsetAsync");
    if (!rc)
      rc = screen_image(data, dtype, n, d, ld, c.gnorm64, 1, c.img_dtype, img, c.ld_img, st,
                        d_err);
    if (!rc)
      rc = hip_check(hipMemcpyAsync(&h_err, d_err, 4, hipMemcpyDeviceToHost, st),
                     "hipMemcpyAsync");
    if (!rc) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    if (rc) return rc;
    float u;
    memcpy(&u, &h_err, 4);
    c.u_cat = std::isfinite(u) && u >= 0.0f ? u : 1.0f / 2048.0f;
  }
  if (rc) return rc;
  *cat = c;
  return EBT_OK;
}

size_t ebt_workspace_bytes(const ebt_catalog* cat, int64_t B, int32_t k, const ebt_options* opt) {
  if (!valid_catalog(cat)) return 0;
  DriverLayout L;
  if (!driver_layout(*cat, B, k, opt ? *opt : ebt_options{}, &L)) return 0;
  return L.bytes;
}

int ebt_cosine_topk_submit(const ebt_catalog* cat, const void* q, int q_dtype, int64_t B,
                           int64_t ldq, const int64_t* liked_off, const int64_t* liked_rows,
                           int32_t k, const int64_t* excl_off, const int64_t* excl_rows,
                           const ebt_options* opt, void* workspace, size_t ws_bytes,
                           double* out_scores, int64_t* out_rows, int32_t* cert_host,
                           ebt_pending* p, void* timer, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!valid_catalog(cat) || !p || !workspace || !out_scores || !out_rows || !cert_host ||
      B < 1 || k < 1 || ((q == nullptr) == (liked_off == nullptr)) ||
      (liked_off && !liked_rows) || ((excl_off == nullptr) != (excl_rows == nullptr)) ||
      (q && (q_dtype < 0 || q_dtype > 3 || ldq < cat->d))) {
    set_error("ebt_cosine_topk: bad arguments (B=%lld k=%d; pass exactly one of q / liked)",
              (long long)B, k);
    return EBT_EINVAL;
  }
  const ebt_options o = opt ? *opt : ebt_options{};
  DriverLayout L;
  if (!driver_layout(*cat, B, k, o, &L)) {
    set_error("ebt_cosine_topk: unsupported sizes or options (B=%lld k=%d n=%lld: n < 2^31; "
              "chunk_rows % 128 == 0; flags EBT_FLAG_NO_FUSE only)",
              (long long)B, k, (long long)cat->n);
    return EBT_EINVAL;
  }
  if (ws_bytes < L.bytes) {
    set_error("ebt_cosine_topk: workspace %zu < %zu bytes (ebt_workspace_bytes)", ws_bytes,
              L.bytes);
    return EBT_ENOMEM;
  }
  char* ws = (char*)workspace;
  char* prep = ws + L.off_prep;
  int rc = q ? prep_dense(*cat, q, q_dtype, B, ldq, L.prep, prep, st)
             : prep_liked(*cat, liked_off, liked_rows, B, L.prep, prep,
                          ws + (L.large ? L.off_big : L.off_pass),
                          L.large ? L.big_bytes : L.pass_bytes, st,
                          (o.flags & EBT_FLAG_LIKED_CHECKED) != 0);
  if (rc) return rc;
  int32_t* cert = (int32_t*)(ws + L.off_cert);
  // the full-sort path fills its certificates by a memset and adds the exclusion flag: copied
  int32_t* direct = L.large ? nullptr : host_mapped(cert_host);
  if (direct) {
    for (int64_t b = 0; b < B; ++b) cert_host[b] = CERT_UNSET;
    cert = direct;
  }
  if (L.large) {  // exact: every certificate is 1, the results are final
    rc = large_topk((const double*)(prep + L.prep.q64), B, cat->d, cat->data, cat->dtype,
                    cat->ld, cat->gnorm64, cat->n, cat->row_offset, excl_off, excl_rows, k,
                    out_scores, out_rows, ws + L.off_big, L.big_bytes, st);
    if (!rc) rc = hip_check(hipMemsetD32Async((hipDeviceptr_t)cert, 1, (size_t)B, st),
                            "hipMemsetD32Async");
  } else {
    const bool padded = L.k_eff < k;
    double* rs = padded ? (double*)(ws + L.off_res_s) : out_scores;
    int64_t* rr = padded ? (int64_t*)(ws + L.off_res_r) : out_rows;
    rc = run_prepared(*cat, L.prep, prep, B, excl_off, excl_rows, L.k_eff, L.kprime, L.chunk,
                      L.flags, ws + L.off_pass, L.pass_bytes, rs, rr, cert, timer, st);
  }
  if (rc) return rc;
  // the exclusion check: the rescore's certificate -3 (ebt_cosine_topk_prepared); the full-sort
  // path has no rescore, so its flag sits right after the certificates, one copy bringing both
  // (otherwise the flag is neither set nor read)
  if (excl_off && L.large) {
    rc = hip_check(hipMemsetAsync(cert + B, 0, 4, st), "hipMemsetAsync");
    if (rc) return rc;
    hipLaunchKernelGGL(csr_sorted_kernel, dim3((unsigned)B), dim3(256), 0, st, excl_off,
                       excl_rows, cert + B);
    rc = launch_check("csr_sorted_kernel");
    if (rc) return rc;
  }
  if (!direct) {
    rc = hip_check(hipMemcpyAsync(cert_host, cert, (size_t)(B + (excl_off && L.large)) * 4,
                                 hipMemcpyDeviceToHost, st),
                   "hipMemcpyAsync");
    if (rc) return rc;
  }
  hipEvent_t ev = event_get(st);
  if (!ev) return hip_check(hipErrorOutOfMemory, "hipEventCreate");
  rc = hip_check(hipEventRecord(ev, st), "hipEventRecord");
  if (rc) {
    event_put(ev, st);
    return rc;
  }
  ebt_pending P{};
  P.cat = cat;
  P.opt = o;
  P.B = B;
  P.B_pad = L.B_pad;
  P.chunk = L.chunk;
  P.k = k;
  P.k_eff = L.k_eff;
  P.kprime = L.kprime;
  P.excl_off = excl_off;
  P.excl_rows = excl_rows;
  P.ws = ws;
  P.ws_bytes = ws_bytes;
  P.out_scores = out_scores;
  P.out_rows = out_rows;
  P.cert_host = cert_host;
  P.event = ev;
  P.timer = timer;
  P.stream = stream;
  *p = P;
  return EBT_OK;
}

int ebt_cosine_topk_finish(ebt_pending* p) {
  if (!p || !p->event || !p->cat) {
    set_error("ebt_cosine_topk_finish: not a submitted batch");
    return EBT_EINVAL;
  }
  hipStream_t st = (hipStream_t)p->stream;
  const ebt_catalog& c = *p->cat;
  hipEvent_t ev = (hipEvent_t)p->event;
  int rc = hip_check(hipEventSynchronize(ev), "hipEventSynchronize");
  event_put(ev, st);
  p->event = nullptr;
  if (rc) return rc;
  const int64_t B = p->B;
  DriverLayout L;
  if (!driver_layout(c, B, p->k, p->opt, &L)) {
    set_error("ebt_cosine_topk_finish: bad pending batch");
    return EBT_EINVAL;
  }
  const bool unsorted_excl = p->excl_off && (L.large ? p->cert_host[B] != 0 : [&] {
    for (int64_t b = 0; b < B; ++b)
      if (p->cert_host[b] == -3) return true;
    return false;
  }());
  for (int64_t b = 0; b < B; ++b)
    if (p->cert_host[b] < -3 || p->cert_host[b] > 1) {
      set_error("ebt_cosine_topk_finish: query %lld's certificate %d was not delivered",
                (long long)b, p->cert_host[b]);
      return EBT_EHIP;
    }
  if (unsorted_excl) {
    set_error("ebt_cosine_topk: exclusion rows must be sorted ascending within each query");
    return EBT_EINVAL;
  }
  if (L.large) return EBT_OK;  // the full-sort path is exact: nothing to retry or pad
  char* ws = p->ws;
  const bool padded = L.k_eff < p->k;
  double* rs = padded ? (double*)(ws + L.off_res_s) : p->out_scores;
  int64_t* rr = padded ? (int64_t*)(ws + L.off_res_r) : p->out_rows;
  const int32_t kcap = (int32_t)(round_up(c.n, 4) < KPRIME_MAX ? round_up(c.n, 4) : KPRIME_MAX);
  // per-query retry state
  std::vector<int32_t> cert(p->cert_host, p->cert_host + B);
  std::vector<int32_t> kp(B, L.kprime), fl(B, L.flags);
  std::vector<int64_t> h_off;
  char* prep = ws + L.off_prep;
  char* rprep = ws + L.off_rprep;
  int64_t* d_idx = (int64_t*)(ws + L.off_idx);
  int64_t* d_roff = (int64_t*)(ws + L.off_roff);
  int64_t* d_rrows = (int64_t*)(ws + L.off_rrows);
  double* r_s = (double*)(ws + L.off_rs);
  int64_t* r_r = (int64_t*)(ws + L.off_rr);
  int32_t* r_c = (int32_t*)(ws + L.off_rcert);
  const int64_t qrow = (int64_t)c.d * 8, irow = (int64_t)c.ld_img * 2;
  for (int round = 0;; ++round) {
    // next configuration of every query that needs one
    std::vector<int64_t> todo;
    for (int64_t b = 0; b < B; ++b) {
      if (cert[b] == 1) continue;
      if (cert[b] == -2 || cert[b] < -2 || cert[b] > 1) {
        set_error("internal error: candidate row out of range (certificate %d)", cert[b]);
        return EBT_EHIP;
      }
      if (cert[b] == -1) {
        fl[b] |= EBT_FLAG_NO_FUSE;
      } else if (kp[b] < kcap) {
        kp[b] = kp[b] * 4 < kcap ? kp[b] * 4 : kcap;
      } else if (!(fl[b] & EBT_FLAG_EXACT)) {
        fl[b] = EBT_FLAG_EXACT;
        kp[b] = L.kprime;
      } else {
        set_error("query %lld could not be certified at k'=%d (more than k' rows tie with the "
                  "k-th score at f32 precision)", (long long)b, kp[b]);
        return EBT_EUNSUPPORTED;
      }
      todo.push_back(b);
    }
    if (todo.empty()) break;
    if (round > 64) {
      set_error("ebt_cosine_topk: retries did not converge");
      return EBT_EHIP;
    }
    if (p->excl_off && h_off.empty()) {
      h_off.resize(B + 1);
      rc = hip_check(hipMemcpy(h_off.data(), p->excl_off, (B + 1) * 8, hipMemcpyDeviceToHost),
                     "hipMemcpy");
      if (rc) return rc;
    }
    // groups of equal (k', flags), at most R queries and RETRY_EXCL_MAX exclusion rows each
    std::vector<char> done(todo.size(), 0);
    for (size_t s = 0; s < todo.size(); ++s) {
      if (done[s]) continue;
      const int32_t gkp = kp[todo[s]], gfl = fl[todo[s]];
      std::vector<int64_t> grp;
      std::vector<int64_t> goff(1, 0);
      bool solo = false;  // one query whose own segment exceeds the gather buffer
      for (size_t u = s; u < todo.size() && (int64_t)grp.size() < L.R; ++u) {
        const int64_t b = todo[u];
        if (done[u] || kp[b] != gkp || fl[b] != gfl) continue;
        const int64_t len = p->excl_off ? h_off[b + 1] - h_off[b] : 0;
        if (len > RETRY_EXCL_MAX) {
          if (!grp.empty()) continue;
          solo = true;
        } else if (goff.back() + len > RETRY_EXCL_MAX) {
          continue;
        }
        grp.push_back(b);
        goff.push_back(goff.back() + len);
        done[u] = 1;
        if (solo) break;
      }
      const int64_t m = (int64_t)grp.size(), m_pad = pad_batch(m);
      rc = hip_check(hipMemcpy(d_idx, grp.data(), m * 8, hipMemcpyHostToDevice), "hipMemcpy");
      if (rc) return rc;
      // the group's prepared queries (padding rows: zero image, scale 1, eps 0)
      const PrepLayout& RP = L.prep_r;
      rc = hip_check(hipMemsetAsync(rprep + RP.qimg, 0, (size_t)m_pad * irow, st), "memset");
      if (!rc) rc = hip_check(hipMemsetAsync(rprep + RP.eps, 0, (size_t)m_pad * 4, st), "memset");
      if (!rc)  // qscale = 1.0f (bits 0x3f800000), as ebt_query_image leaves padding rows
        rc = hip_check(hipMemsetD32Async((hipDeviceptr_t)(rprep + RP.qscale), 0x3f800000,
                                         (size_t)m_pad, st),
                       "memsetD32");
      if (!rc) rc = move_rows(prep + L.prep.q64, qrow, rprep + RP.q64, qrow, d_idx, m, qrow,
                              false, st);
      if (!rc) rc = move_rows(prep + L.prep.qimg, irow, rprep + RP.qimg, irow, d_idx, m, irow,
                              false, st);
      if (!rc) rc = move_rows(prep + L.prep.qscale, 4, rprep + RP.qscale, 4, d_idx, m, 4, false,
                              st);
      if (!rc) rc = move_rows(prep + L.prep.eps, 4, rprep + RP.eps, 4, d_idx, m, 4, false, st);
      if (rc) return rc;
      const int64_t* eo = nullptr;
      const int64_t* er = nullptr;
      if (p->excl_off) {
        if (solo) {  // the segment in place: offsets {off[b], off[b+1]} into the caller's rows
          rc = hip_check(hipMemcpy(d_roff, p->excl_off + grp[0], 16, hipMemcpyDeviceToDevice),
                         "hipMemcpy");
          if (rc) return rc;
          eo = d_roff;
          er = p->excl_rows;
        } else {
          rc = hip_check(hipMemcpy(d_roff, goff.data(), (m + 1) * 8, hipMemcpyHostToDevice),
                         "hipMemcpy");
          if (rc) return rc;
          hipLaunchKernelGGL(csr_gather_kernel, dim3((unsigned)m), dim3(256), 0, st, p->excl_off,
                             p->excl_rows, d_idx, d_roff, d_rrows);
          rc = launch_check("csr_gather_kernel");
          if (rc) return rc;
          eo = d_roff;
          er = d_rrows;
        }
      }
      rc = run_prepared(c, RP, rprep, m, eo, er, L.k_eff, gkp, L.chunk_r, gfl, ws + L.off_pass,
                        L.pass_bytes, r_s, r_r, r_c, p->timer, st);
      if (!rc) rc = move_rows(r_s, (int64_t)L.k_eff * 8, rs, (int64_t)L.k_eff * 8, d_idx, m,
                              (int64_t)L.k_eff * 8, true, st);
      if (!rc) rc = move_rows(r_r, (int64_t)L.k_eff * 8, rr, (int64_t)L.k_eff * 8, d_idx, m,
                              (int64_t)L.k_eff * 8, true, st);
      if (rc) return rc;
      std::vector<int32_t> gc(m);
      rc = hip_check(hipMemcpyAsync(gc.data(), r_c, m * 4, hipMemcpyDeviceToHost, st),
                     "hipMemcpyAsync");
      if (!rc) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
      if (rc) return rc;
      for (int64_t i = 0; i < m; ++i) cert[grp[i]] = gc[i];
    }
  }
  if (padded) {
    const int64_t total = B * p->k;
    int64_t blocks = (total + 255) / 256;
    blocks = blocks > 4096 ? 4096 : blocks;
    hipLaunchKernelGGL(pad_results_kernel, dim3((unsigned)blocks), dim3(256), 0, st, rs, rr, B,
                       L.k_eff, p->k, p->out_scores, p->out_rows);
    rc = launch_check("pad_results_kernel");
    if (rc) return rc;
  }
  return EBT_OK;
}

int ebt_cosine_topk(const ebt_catalog* cat, const void* q, int q_dtype, int64_t B, int64_t ldq,
                    const int64_t* liked_off, const int64_t* liked_rows, int32_t k,
                    const int64_t* excl_off, const int64_t* excl_rows, const ebt_options* opt,
                    void* workspace, size_t ws_bytes, double* out_scores, int64_t* out_rows,
                    void* timer, void* stream) {
  std::vector<int32_t> cert((size_t)(B > 0 ? B : 0) + 1);
  ebt_pending p{};
  int rc = ebt_cosine_topk_submit(cat, q, q_dtype, B, ldq, liked_off, liked_rows, k, excl_off,
                                  excl_rows, opt, workspace, ws_bytes, out_scores, out_rows,
                                  cert.data(), &p, timer, stream);
  if (rc) return rc;
  rc = ebt_cosine_topk_finish(&p);
  if (!rc) rc = hip_check(hipStreamSynchronize((hipStream_t)stream), "hipStreamSynchronize");
  return rc;
}

}  // extern "C"

// =========================================================== the row-sharded self-contained entry
// ebt_cosine_topk_sharded (include/ebert.h): distributed.py's per-shard protocol
// (score_topk_sharded_local_stages) in C++ over a caller-supplied all-gather. Reference:
// /root/reference/src/backend/app/lib.py:51-55 restated on every shard; the merge of the shards'
// exact top-k is the only thing the reference (one CPU process) has no counterpart for.
namespace ebt {
namespace {

constexpr int SH_MERGE_WAVE_KMAX = 512;          // search.py MERGE_WAVE_KMAX
#ifndef EBT_SH_SHARED_MAX
#define EBT_SH_SHARED_MAX 300000  // (build knob for A/B; round 5: 200000 -> 300000, C3/4 -1.6 %)
#endif
constexpr int64_t SH_SHARED_MAX_SHARD_ROWS = EBT_SH_SHARED_MAX;  // distributed.py SHARED_MAX_SHARD_ROWS
constexpr int64_t SH_SAMPLE_TILES_MAX = 64;
constexpr int SH_K_MAX = 4096;                   // ebt_merge_topk

// search.py spec_rank: the smallest j with P(Poisson(lam) >= j) <= 1e-6
int sh_spec_rank(double lam) {
  double pmf = exp(-lam), cdf = 0.0;
  int j = 0;
  while (j < 100000 && 1.0 - cdf > 1e-6) {
    cdf += pmf;
    pmf *= lam / (j + 1);
    ++j;
  }
  return j > 1 ? j : 1;
}

// distributed.py shared_sample_tiles: 256-row sample tiles per shard for the catalog-wide
// screening threshold (0 = every shard screens at its own); depends only on (n_global, world,
// B_pad), so every rank decides alike
int64_t sh_tiles(int64_t n_global, int world, int64_t B_pad) {
  const int64_t shard = ceil_div(n_global, world);
  if (world < 2 || B_pad % 256 != 0 || shard > SH_SHARED_MAX_SHARD_ROWS) return 0;
  const int64_t full = shard / 256;
  int64_t cap = ceil_div(SH_SAMPLE_TILES_MAX, world);
  cap = cap > 4 ? cap : 4;
  int64_t P = SH_SAMPLE_TILES_MAX < full / 24 ? SH_SAMPLE_TILES_MAX : full / 24;
  P = P < cap ? P : cap;
  const int64_t per = 256 / (B_pad / 256) > 1 ? 256 / (B_pad / 256) : 1;
  if (P / per * per >= 8) P = P / per * per;
  // a sample GEMM of less than one round of the persistent grid takes a round's time anyway:
  // fill it (C3 on 8 ranks: 8 -> 16 tiles per shard, room for the lead)
  // (only while the fill stays within the sample's caps: at B_pad = 512 a round is 128 tiles,
  // and 8 ranks x 4 x 128 maxima would exceed ebt_pool_kth's 2048 -- distributed.py alike)
  if (P < per && per <= full / 6 && per <= SH_SAMPLE_TILES_MAX && world * 4 * per <= 2048)
    P = per;
  return (P >= 1 && world * P >= 8) ? P : 0;
}

struct ShardLayout {
  DriverLayout D;
  int64_t tiles, G, RG, J, GJ;  // sample maxima per shard (G), sent per shard (J + 1 of them)
  int64_t lead, ld_lead;        // this shard's sample lead (its first tiles' scores kept)
  size_t screen_bytes;
  int64_t fw, cap;  // floor gather width per shard and query; packed results per rank (0: full)
  size_t pack_bytes;
  size_t off_spass, off_pool, off_gsamp, off_lv, off_lr, off_ovf,
      off_eps, off_fsend, off_frecv, off_tfloor, off_ls, off_lrr, off_gs, off_gr, off_scale,
      off_qrecv, off_psend, off_precv, off_incomplete, off_lead, bytes;
};

bool shard_layout(const ebt_catalog& c, const ebt_comm& cm, int64_t B, int32_t k,
                  const ebt_options& opt, ShardLayout* S) {
  if (k < 1 || k > SH_K_MAX || cm.world < 1 || cm.rank < 0 || cm.rank >= cm.world ||
      cm.n_global < c.row_offset + c.n || !cm.all_gather)
    return false;
  ShardLayout& L = *S;
  L = ShardLayout{};
  if (!driver_layout(c, B, k, opt, &L.D) || L.D.large) return false;
  const DriverLayout& D = L.D;
  const int64_t R = cm.world, kp = D.kprime;
  // the shared threshold only serves the wave-merge screen (k' <= 512); decided from
  // rank-invariant sizes (k against the WHOLE catalog), since its all-gather is a collective
  const int64_t kg = k < cm.n_global ? k : cm.n_global;
  int64_t kpg = opt.kprime ? round_up(opt.kprime, 4)
                           : round_up(c.native ? kg + (kg / 4 > 16 ? kg / 4 : 16)
                                               : (2 * kg > kg + 32 ? 2 * kg : kg + 32), 8);
  L.tiles = (opt.flags & EBT_FLAG_NO_FUSE) || kpg > SH_MERGE_WAVE_KMAX
                ? 0
                : sh_tiles(cm.n_global, cm.world, D.B_pad);
  L.G = 4 * L.tiles;
  L.RG = R * L.G;
  if (L.RG > 2048) L.tiles = L.G = L.RG = 0;  // ebt_pool_kth's limit (sh_tiles keeps within it)
  // theta = the j-th largest of all R G maxima, j <= J (J from the catalog-wide k', rank-
  // invariant, >= every rank's own j): the j-th of the union of each shard's J largest is the
  // same value, so each shard sends its J largest (+ a -inf column: ebt_floor_pack's layout)
  L.J = L.GJ = 0;
  if (L.tiles) {
    const double m_total = 256.0 * (double)L.tiles * R;
    L.J = sh_spec_rank((double)kpg * m_total / (double)cm.n_global);
    if (L.J > L.RG / 2) L.tiles = L.G = L.RG = L.J = 0;  // the sample would decide nothing
    L.J = L.J < L.G ? L.J : L.G;
    L.GJ = L.J + 1;
  }
  size_t scr = ebt_cosine_topk_workspace(B, D.B_pad, c.n, D.kprime, D.chunk, D.flags);
  if (L.tiles) {
    const size_t t = ebt_cosine_topk_workspace(B, D.B_pad, c.n, D.kprime, D.chunk, EBT_FLAG_THETA);
    scr = t > scr ? t : scr;
  }
  if (scr == 0) return false;
  L.screen_bytes = scr;
  size_t o = al(D.bytes);
  L.off_spass = D.off_pass;
  if (scr > D.pass_bytes) {  // the first pass's screen needs more than the retries' region
    L.off_spass = o;
    o = al(o + scr);
  }
  L.off_pool = o;
  o = al(o + (size_t)D.B_pad * L.G * 4);
  // the lead: only where the shared threshold drives the screen (ebt_cosine_screen_at_lead)
  L.lead = L.ld_lead = 0;
  if (L.tiles && D.flags == 0 && D.kprime <= SH_MERGE_WAVE_KMAX) {
    const int64_t own = L.tiles < c.n / 256 ? L.tiles : c.n / 256;
    // (the room regardless of ebt_spec_lead: offsets never depend on the knob)
    L.lead = own == L.tiles ? shard_lead_tiles(D.B_pad, c.n, own) : 0;
    L.ld_lead = own == L.tiles ? 256 * shard_lead_room(D.B_pad, c.n, own) : 0;
  }
  L.off_lead = o;
  o = al(o + (size_t)D.B_pad * L.ld_lead * 4);
  L.off_gsamp = o;
  o = al(o + (size_t)B * L.GJ * 4 * (R + 1));  // this shard's J largest, then every shard's
  L.off_lv = o;
  o = al(o + (size_t)B * kp * 4);
  L.off_lr = o;
  o = al(o + (size_t)B * kp * 8);
  L.off_ovf = o;
  o = al(o + (size_t)B * 4);
  L.off_eps = o;
  o = al(o + (size_t)B * 4);
  // the compact exchange (rescore.hip): each shard's w best approx for the floor, its entries
  // above the floor for the results (int32 rows behind per-query starts)
  L.fw = ebt_shard_list_width(k, (int32_t)R);
  L.cap = ebt_shard_pack_cap(B, k, (int32_t)R, cm.n_global);
  if (!L.cap) L.fw = k;
  L.pack_bytes = L.cap ? ebt_shard_pack_bytes(B, L.cap) : 0;
  L.off_fsend = o;
  o = al(o + (size_t)B * (L.fw + 1) * 4);
  L.off_frecv = o;
  o = al(o + (size_t)R * B * (L.fw + 1) * 4);
  L.off_tfloor = o;
  o = al(o + (size_t)B * 8);
  L.off_ls = o;
  o = al(o + (size_t)B * k * 8);
  L.off_lrr = o;
  o = al(o + (size_t)B * k * 8);
  L.off_gs = o;
  o = al(o + (size_t)R * B * k * 8);
  L.off_gr = o;
  o = al(o + (size_t)R * B * k * 8);
  L.off_scale = o;
  o = al(o + (size_t)B * 8);
  L.off_qrecv = o;
  if (!cm.all_reduce_f64) o = al(o + (size_t)R * B * c.d * 8);  // the liked path's gathered sums
  L.off_psend = o;
  o = al(o + L.pack_bytes);
  L.off_precv = o;
  o = al(o + (size_t)R * L.pack_bytes);
  L.off_incomplete = o;   // int32 "incomplete" flag, then the rescore's pack counter (u32)
  o = al(o + 8);
  L.bytes = o;
  return true;
}

// out[t] = sum over ranks r (in rank order) of in[r * total + t]: the all-reduce of the liked
// queries' partial sums, identical on every rank
__global__ void sum_ranks_kernel(const double* __restrict__ in, int R, int64_t total,
                                 double* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int r = 0; r < R; ++r) s += in[(int64_t)r * total + t];
    out[t] = s;
  }
}

unsigned grid_for(int64_t total) {
  int64_t b = ceil_div(total, 256);
  return (unsigned)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

int sh_gather(const ebt_comm& cm, const void* send, void* recv, size_t bytes, void* timer,
              hipStream_t st) {
  if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_COLLECTIVE, st);
  const int rc = cm.all_gather(cm.ctx, send, recv, bytes, (void*)st);
  if (timer) (void)ebt_timer_end(timer, EBT_STAGE_COLLECTIVE, st);
  if (rc) {
    set_error("ebt_cosine_topk_sharded: the caller's all_gather returned %d", rc);
    return EBT_EHIP;
  }
  return EBT_OK;
}

// liked rows of a row-sharded catalog: GLOBAL rows, each shard sums its own, the partial sums
// are all-gathered and added in rank order, then / L_b (lib.py:51-52)
int prep_liked_sharded(const ebt_catalog& c, const ebt_comm& cm, const int64_t* off,
                       const int64_t* rows, int64_t B, const PrepLayout& P, char* base,
                       double* d_scale, double* qrecv, void* timer, hipStream_t st) {
  std::vector<int64_t> h_off(B + 1);
  int rc = hip_check(hipMemcpyAsync(h_off.data(), off, (B + 1) * 8, hipMemcpyDeviceToHost, st),
                     "hipMemcpyAsync");
  if (!rc) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (rc) return rc;
  std::vector<double> scale(B);
  for (int64_t b = 0; b < B; ++b) {
    const int64_t cnt = h_off[b + 1] - h_off[b];
    if (cnt <= 0) {
      set_error("Found array with 0 sample(s) (shape=(0, %d)) while a minimum of 1 is required "
                "by check_pairwise_arrays.", c.d);
      return EBT_EINVAL;
    }
    scale[b] = 1.0 / (double)cnt;
  }
  const int64_t nnz = h_off[B] - h_off[0];
  if (nnz > 0) {
    std::vector<int64_t> h_rows(nnz);
    rc = hip_check(hipMemcpy(h_rows.data(), rows + h_off[0], nnz * 8, hipMemcpyDeviceToHost),
                   "hipMemcpy");
    if (rc) return rc;
    for (int64_t r : h_rows)
      if (r < 0 || r >= cm.n_global) {
        set_error("liked row %lld is not in the catalog rows [0, %lld)", (long long)r,
                  (long long)cm.n_global);
        return EBT_EINVAL;
      }
  }
  rc = hip_check(hipMemcpy(d_scale, scale.data(), B * 8, hipMemcpyHostToDevice), "hipMemcpy");
  if (rc) return rc;
  double* q64 = (double*)(base + P.q64);
  rc = query_liked_sum(c.data, c.dtype, c.d, c.ld, c.gnorm64, B, off, rows, q64, st,
                       c.row_offset, c.n);
  if (rc) return rc;
  if (cm.all_reduce_f64) {  // the caller's all-reduce (RCCL: about 2 / R of the gather's bytes)
    if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_COLLECTIVE, st);
    const int e = cm.all_reduce_f64(cm.ctx, q64, (size_t)B * c.d, (void*)st);
    if (timer) (void)ebt_timer_end(timer, EBT_STAGE_COLLECTIVE, st);
    if (e) {
      set_error("ebt_cosine_topk_sharded: the caller's all_reduce_f64 returned %d", e);
      return EBT_EHIP;
    }
  } else {
    rc = sh_gather(cm, q64, qrecv, (size_t)B * c.d * 8, timer, st);
    if (rc) return rc;
    hipLaunchKernelGGL(sum_ranks_kernel, dim3(grid_for(B * c.d)), dim3(256), 0, st, qrecv,
                       (int)cm.world, B * c.d, q64);
    rc = launch_check("sum_ranks_kernel");
  }
  if (!rc) rc = ebt_scale_rows_f64(q64, B, c.d, d_scale, st);
  if (rc) return rc;
  return ebt_query_image(q64, B, pad_batch(B), c.d, c.img_dtype, nullptr, 0, 0, c.u_cat,
                         base + P.qimg, c.ld_img, (float*)(base + P.qscale),
                         (float*)(base + P.eps), st);
}

// the full exchange: every shard's [B][k] exact list (f64 scores, i64 rows), ebt_merge_topk
int sh_full_merge(const ShardLayout& S, const ebt_comm& cm, char* ws, int64_t B, int32_t k,
                  double* out_s, int64_t* out_r, void* timer, hipStream_t st) {
  double* ls = (double*)(ws + S.off_ls);
  int64_t* lrr = (int64_t*)(ws + S.off_lrr);
  double* gs = (double*)(ws + S.off_gs);
  int64_t* gr = (int64_t*)(ws + S.off_gr);
  int rc = sh_gather(cm, ls, gs, (size_t)B * k * 8, timer, st);
  if (!rc) rc = sh_gather(cm, lrr, gr, (size_t)B * k * 8, timer, st);
  if (rc) return rc;
  if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_SHARD_MERGE, st);
  rc = ebt_merge_topk(gs, gr, cm.world, B, k, out_s, out_r, st);
  if (timer) (void)ebt_timer_end(timer, EBT_STAGE_SHARD_MERGE, st);
  return rc;
}
}  // namespace
}  // namespace ebt

extern "C" {

size_t ebt_sharded_workspace_bytes(const ebt_catalog* cat, const ebt_comm* comm, int64_t B,
                                   int32_t k, const ebt_options* opt) {
  if (!valid_catalog(cat) || !comm) return 0;
  ShardLayout S;
  if (!shard_layout(*cat, *comm, B, k, opt ? *opt : ebt_options{}, &S)) return 0;
  return S.bytes;
}

int ebt_cosine_topk_sharded_submit(const ebt_catalog* cat, const ebt_comm* comm, const void* q,
                                   int q_dtype, int64_t B, int64_t ldq,
                                   const int64_t* liked_off, const int64_t* liked_rows,
                                   int32_t k, const int64_t* excl_off, const int64_t* excl_rows,
                                   const ebt_options* opt, void* workspace, size_t ws_bytes,
                                   double* out_scores, int64_t* out_rows, int32_t* host,
                                   ebt_sharded_pending* pending, void* timer, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!valid_catalog(cat) || !comm || !workspace || !out_scores || !out_rows || !host ||
      !pending || B < 1 || k < 1 || ((q == nullptr) == (liked_off == nullptr)) ||
      (liked_off && !liked_rows) || ((excl_off == nullptr) != (excl_rows == nullptr)) ||
      (q && (q_dtype < 0 || q_dtype > 3 || ldq < cat->d))) {
    set_error("ebt_cosine_topk_sharded: bad arguments (B=%lld k=%d; pass exactly one of q / "
              "liked)", (long long)B, k);
    return EBT_EINVAL;
  }
  const ebt_options o = opt ? *opt : ebt_options{};
  ShardLayout S;
  if (!shard_layout(*cat, *comm, B, k, o, &S)) {
    set_error("ebt_cosine_topk_sharded: unsupported sizes, options or communicator (B=%lld "
              "k=%d <= %d, n=%lld, row_offset=%lld, n_global=%lld, rank %d of %d)",
              (long long)B, k, SH_K_MAX, (long long)cat->n, (long long)cat->row_offset,
              (long long)comm->n_global, comm->rank, comm->world);
    return EBT_EINVAL;
  }
  if (ws_bytes < S.bytes) {
    set_error("ebt_cosine_topk_sharded: workspace %zu < %zu bytes "
              "(ebt_sharded_workspace_bytes)", ws_bytes, S.bytes);
    return EBT_ENOMEM;
  }
  const ebt_catalog& c = *cat;
  const ebt_comm& cm = *comm;
  const DriverLayout& L = S.D;
  const int R = cm.world;
  char* ws = (char*)workspace;
  char* prep = ws + L.off_prep;
  const double* q64 = (const double*)(prep + L.prep.q64);
  const void* qimg = prep + L.prep.qimg;
  const float* qscale = (const float*)(prep + L.prep.qscale);
  const float* qeps = (const float*)(prep + L.prep.eps);
  int rc = EBT_OK;
  // 1. the queries (lib.py:51-52)
  if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_PREP, st);
  rc = q ? prep_dense(c, q, q_dtype, B, ldq, L.prep, prep, st)
         : prep_liked_sharded(c, cm, liked_off, liked_rows, B, L.prep, prep,
                              (double*)(ws + S.off_scale), (double*)(ws + S.off_qrecv), timer, st);
  if (timer) (void)ebt_timer_end(timer, EBT_STAGE_PREP, st);
  if (rc) return rc;
  // 2. the catalog-wide screening threshold from every shard's sample maxima (taken by the
  // screen's first launch, step 3)
  bool accept = false;
  const float* recv_s = nullptr;
  int j_s = 0;
  double hits = 0.0;
  if (S.tiles) {
    float* pool = (float*)(ws + S.off_pool);
    float* gsamp = (float*)(ws + S.off_gsamp);
    const int64_t own = S.tiles < c.n / 256 ? S.tiles : c.n / 256;
    // -inf where this shard has no sample tile (a shard smaller than the sample); a full sample
    // writes every maximum itself (one API call less per step)
    if (own < S.tiles) {
      rc = hip_check(hipMemsetD32Async((hipDeviceptr_t)pool, (int)0xff800000u,
                                       (size_t)L.B_pad * S.G, st), "hipMemsetD32Async");
      if (rc) return rc;
    }
    if (own >= 1) {
      // the lead's tiles first, the rest evenly spaced over the shard after them
      int64_t stride = (c.n / 256 - S.lead) / (own - S.lead);
      if (stride > 1 && stride % 2 == 0) stride -= 1;
      rc = ebt_cosine_sample_lead(qimg, qscale, L.B_pad, c.image, c.cscale, c.img_dtype,
                                  c.ld_img, c.n, c.d_pad, own, stride, pool, S.G, S.lead,
                                  (float*)(ws + S.off_lead), S.ld_lead, timer, st);
      if (rc) return rc;
    }
    float* send = gsamp;                          // [B][J + 1]
    float* recv = gsamp + (size_t)B * S.GJ;       // [R][B][J + 1]
    if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_SMALL, st);
    rc = ebt_floor_pack(pool, S.G, B, (int32_t)S.G, (int32_t)S.J, nullptr, send, st);
    if (timer) (void)ebt_timer_end(timer, EBT_STAGE_SMALL, st);
    if (!rc) rc = sh_gather(cm, send, recv, (size_t)B * S.GJ * 4, timer, st);
    if (rc) return rc;
    const double m_total = 256.0 * (double)S.tiles * R;
    const int j = sh_spec_rank((double)L.kprime * m_total / (double)cm.n_global);
    // exact for j <= J; when J was clamped to G every shard sent all of its maxima, and any
    // j <= RG / 2 is (distributed.theta_from_samples decides alike)
    if (j <= S.J || (S.J == S.G && j <= S.RG / 2)) {
      accept = true;
      recv_s = recv;
      j_s = j;
      hits = ((double)j + (double)j * j / (2.0 * (double)S.RG)) * (double)c.n / m_total;
    }
  }
  const bool use_theta = accept && L.flags == 0 && L.kprime <= SH_MERGE_WAVE_KMAX;
  const float* theta = nullptr;   // the shared threshold, where the screen wrote it
  // 3. the shard's screen: its k' best approx candidates (GLOBAL rows)
  float* lv = (float*)(ws + S.off_lv);
  int64_t* lr = (int64_t*)(ws + S.off_lr);
  int32_t* ovf = (int32_t*)(ws + S.off_ovf);
  float* eps = (float*)(ws + S.off_eps);
  // at the shared threshold the list keeps LOCAL rows and the screen's overflow flags and eps
  // are read where it wrote them (no export launch); otherwise GLOBAL rows, exported
  const int* ovf_p = ovf;
  const float* eps_p = eps;
  // (the j-th of every rank's maxima, read in the gathered [R][B][J + 1] layout, is taken by
  // the launch that starts the list and takes the lead's hits: one launch for both; and at the
  // shared threshold the screen's last wave merge also writes this shard's floor entries,
  // step 4's send buffer: no ebt_floor_pack launch)
  float* fsend = (float*)(ws + S.off_fsend);
  if (use_theta)
    rc = screen_at_local(q64, qimg, qscale, qeps, B, L.B_pad, c.data, c.dtype, c.ld, c.gnorm64,
                         c.image, c.cscale, c.img_dtype, c.ld_img, c.n, c.d, c.d_pad,
                         c.row_offset, excl_off, excl_rows, L.k_eff, L.kprime, L.chunk,
                         ws + S.off_spass, S.screen_bytes, lv, lr, recv_s, B * S.GJ,
                         (int)(R * S.GJ), (int)S.GJ, j_s, hits, S.lead,
                         (const float*)(ws + S.off_lead), S.ld_lead, &theta, &ovf_p, &eps_p,
                         timer, st, fsend, (int)S.fw);
  else
    rc = ebt_cosine_screen(q64, qimg, qscale, qeps, B, L.B_pad, c.data, c.dtype, c.ld, c.gnorm64,
                           c.image, c.cscale, c.img_dtype, c.ld_img, c.n, c.d, c.d_pad,
                           c.row_offset, excl_off, excl_rows, L.k_eff, L.kprime, L.chunk,
                           L.flags, ws + S.off_spass, S.screen_bytes, lv, lr, ovf, eps, timer,
                           st);
  if (rc) return rc;
  // 4. the catalog-wide floor: the k-th largest (approx - eps) over every shard's fw best
  float* frecv = (float*)(ws + S.off_frecv);
  double* tfloor = (double*)(ws + S.off_tfloor);
  if (!use_theta) {
    if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_SMALL, st);
    rc = ebt_floor_pack(lv, L.kprime, B, L.k_eff, (int32_t)S.fw, eps_p, fsend, st);
    if (timer) (void)ebt_timer_end(timer, EBT_STAGE_SMALL, st);
  }
  if (!rc) rc = sh_gather(cm, fsend, frecv, (size_t)B * (S.fw + 1) * 4, timer, st);
  if (rc) return rc;
  // (the floor's launch also zeroes the merge's "incomplete" flag and the pack counter that
  // the rescore and the finish use: no memset launch)
  uint32_t* zero2 = (uint32_t*)(ws + S.off_incomplete);
  if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_SMALL, st);
  rc = union_floor(frecv, R, B, (int32_t)S.fw + 1, k, tfloor, st, zero2);
  if (timer) (void)ebt_timer_end(timer, EBT_STAGE_SMALL, st);
  if (rc) return rc;
  // 5. the rescore of the rows that can enter the global top k, the certificate
  double* ls = (double*)(ws + S.off_ls);
  int64_t* lrr = (int64_t*)(ws + S.off_lrr);
  const bool padded = L.k_eff < k;
  double* rs = padded ? (double*)(ws + L.off_res_s) : ls;
  int64_t* rr = padded ? (int64_t*)(ws + L.off_res_r) : lrr;
  int32_t* cert = (int32_t*)(ws + L.off_cert);
  int32_t* direct = host_mapped(host);  // (see the dense submit)
  if (direct) {
    for (int64_t b = 0; b < B; ++b) host[b] = CERT_UNSET;
    cert = direct;
  }
  // (the list's rows read as they are: local at the shared threshold, global otherwise; the
  // certificate with ebt_certify_cut's tests)
  // (the rescore also checks the exclusion segments' order -- certificate -3 -- and packs the
  // shard's entries above the floor for the results exchange: ebt_shard_pack's two launches
  // folded in; the finish packs again only for a batch whose retries changed lists)
  const ShardPackOut pack{S.cap && !padded ? (uint32_t*)(ws + S.off_psend) + B : nullptr};
  rc = rescore_sharded(q64, B, c.d, c.data, c.dtype, c.ld, c.gnorm64, c.row_offset, lv, lr,
                       L.kprime, L.k_eff, c.n, eps_p, tfloor, rs, rr, cert, ovf_p,
                       use_theta ? theta : nullptr, timer, st, use_theta ? 0 : c.row_offset,
                       excl_off, excl_rows, &pack);
  if (rc) return rc;
  // the certificates to the caller's host buffer (unless the rescore wrote them there); one
  // event for them
  if (!direct) {
    rc = hip_check(hipMemcpyAsync(host, cert, (size_t)B * 4, hipMemcpyDeviceToHost, st),
                   "hipMemcpyAsync");
    if (rc) return rc;
  }
  hipEvent_t ev = event_get(st);
  if (!ev) return hip_check(hipErrorOutOfMemory, "hipEventCreate");
  rc = hip_check(hipEventRecord(ev, st), "hipEventRecord");
  if (rc) {
    event_put(ev, st);
    return rc;
  }
  ebt_sharded_pending P{};
  ebt_pending& lp = P.local;
  lp.cat = cat;
  lp.opt = o;
  lp.B = B;
  lp.B_pad = L.B_pad;
  lp.chunk = L.chunk;
  lp.k = k;
  lp.k_eff = L.k_eff;
  lp.kprime = L.kprime;
  lp.excl_off = excl_off;
  lp.excl_rows = excl_rows;
  lp.ws = ws;
  lp.ws_bytes = ws_bytes;
  lp.out_scores = ls;
  lp.out_rows = lrr;
  lp.cert_host = host;
  lp.event = ev;
  lp.timer = timer;
  lp.stream = stream;
  P.comm = cm;
  P.out_scores = out_scores;
  P.out_rows = out_rows;
  P.host = host;
  P.event = nullptr;
  P.stage = 1;
  *pending = P;
  return EBT_OK;
}


int ebt_cosine_topk_sharded_finish(ebt_sharded_pending* p) {
  if (!p || p->stage != 1 || !p->local.cat) {
    set_error("ebt_cosine_topk_sharded_finish: not a submitted batch");
    return EBT_EINVAL;
  }
  ebt_pending& lp = p->local;
  hipStream_t st = (hipStream_t)lp.stream;
  ShardLayout S;
  if (!shard_layout(*lp.cat, p->comm, lp.B, lp.k, lp.opt, &S)) {
    set_error("ebt_cosine_topk_sharded_finish: bad pending batch");
    return EBT_EINVAL;
  }
  // the local retries (ebt_cosine_topk_finish: unfused reruns, k' x 4, the float64 screen) on
  // this shard alone: a retried query gets the shard's exact top k, which the merge accepts
  int rc = ebt_cosine_topk_finish(&lp);
  if (rc) return rc;
  p->stage = 2;
  char* ws = lp.ws;
  const int64_t B = lp.B;
  const int32_t k = lp.k;
  void* timer = lp.timer;
  p->host[B + 1] = 0;
  if (S.cap) {
    // 6. every shard's entries above the floor, packed (int32 rows), ONE all-gather, the merge.
    // The rescore counted them already (len[b] in the header; the "incomplete" flag was zeroed
    // in the submit): one launch places and copies them. Counted again (ebt_shard_pack) only when
    // retries rewrote some query's list (its first-pass certificate was not 1) or the list was
    // padded to k in the finish
    int32_t* incomplete = (int32_t*)(ws + S.off_incomplete);
    bool repack = lp.k_eff < k;
    for (int64_t b = 0; b < B && !repack; ++b) repack = lp.cert_host[b] != 1;
    if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_SMALL, st);
    rc = repack ? ebt_shard_pack((const double*)(ws + S.off_ls), (const int64_t*)(ws + S.off_lrr),
                                 B, k, (const double*)(ws + S.off_tfloor), S.cap,
                                 ws + S.off_psend, st)
                : shard_pack_lens((const double*)(ws + S.off_ls),
                                  (const int64_t*)(ws + S.off_lrr), B, k, S.cap,
                                  ws + S.off_psend, st);
    if (timer) (void)ebt_timer_end(timer, EBT_STAGE_SMALL, st);
    if (!rc) rc = sh_gather(p->comm, ws + S.off_psend, ws + S.off_precv, S.pack_bytes, timer, st);
    if (rc) return rc;
    if (timer) (void)ebt_timer_begin(timer, EBT_STAGE_SHARD_MERGE, st);
    // (the flag straight into the host buffer when it is pinned: zeroed above, only ever set
    // to 1 by the merge's stores; else the workspace's flag and one copy)
    int32_t* direct = host_mapped(p->host + B + 1);
    rc = ebt_merge_packed(ws + S.off_precv, p->comm.world, B, k, S.cap, p->out_scores,
                          p->out_rows, direct ? direct : incomplete, st);
    if (timer) (void)ebt_timer_end(timer, EBT_STAGE_SHARD_MERGE, st);
    if (!rc && !direct)
      rc = hip_check(hipMemcpyAsync(p->host + B + 1, incomplete, 4, hipMemcpyDeviceToHost, st),
                     "hipMemcpyAsync");
  } else {
    rc = sh_full_merge(S, p->comm, ws, B, k, p->out_scores, p->out_rows, timer, st);
  }
  if (rc) return rc;
  hipEvent_t ev = event_get(st);
  if (!ev) return hip_check(hipErrorOutOfMemory, "hipEventCreate");
  rc = hip_check(hipEventRecord(ev, st), "hipEventRecord");
  if (rc) {
    event_put(ev, st);
    return rc;
  }
  p->event = ev;
  return EBT_OK;
}

int ebt_cosine_topk_sharded_wait(ebt_sharded_pending* p) {
  if (!p || p->stage != 2 || !p->event) {
    set_error("ebt_cosine_topk_sharded_wait: not a finished batch");
    return EBT_EINVAL;
  }
  ebt_pending& lp = p->local;
  hipStream_t st = (hipStream_t)lp.stream;
  hipEvent_t ev = (hipEvent_t)p->event;
  int rc = hip_check(hipEventSynchronize(ev), "hipEventSynchronize");
  event_put(ev, st);
  p->event = nullptr;
  p->stage = 0;
  if (rc) return rc;
  if (p->host[lp.B + 1] == 0) return EBT_OK;
  // some rank's entries above the floor exceeded its packed capacity (every rank sees the same
  // gathered starts, so every rank takes this branch): the full exchange
  ShardLayout S;
  if (!shard_layout(*lp.cat, p->comm, lp.B, lp.k, lp.opt, &S)) {
    set_error("ebt_cosine_topk_sharded_wait: bad pending batch");
    return EBT_EINVAL;
  }
  rc = sh_full_merge(S, p->comm, lp.ws, lp.B, lp.k, p->out_scores, p->out_rows, lp.timer, st);
  if (!rc) rc = hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  return rc;
}

int64_t ebt_shard_sample_tiles(int64_t n_global, int32_t world, int64_t B_pad) {
  if (n_global < 1 || world < 1 || B_pad < 1) return -1;
  return sh_tiles(n_global, world, B_pad);
}

int ebt_cosine_topk_sharded(const ebt_catalog* cat, const ebt_comm* comm, const void* q,
                            int q_dtype, int64_t B, int64_t ldq, const int64_t* liked_off,
                            const int64_t* liked_rows, int32_t k, const int64_t* excl_off,
                            const int64_t* excl_rows, const ebt_options* opt, void* workspace,
                            size_t ws_bytes, double* out_scores, int64_t* out_rows, void* timer,
                            void* stream) {
  std::vector<int32_t> host((size_t)(B > 0 ? B : 0) + 2);
  ebt_sharded_pending p{};
  int rc = ebt_cosine_topk_sharded_submit(cat, comm, q, q_dtype, B, ldq, liked_off, liked_rows,
                                          k, excl_off, excl_rows, opt, workspace, ws_bytes,
                                          out_scores, out_rows, host.data(), &p, timer, stream);
  if (!rc) rc = ebt_cosine_topk_sharded_finish(&p);
  if (!rc) rc = ebt_cosine_topk_sharded_wait(&p);
  return rc;
}

}  // extern "C"
