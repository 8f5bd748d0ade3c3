// Top-k for large k (min(k, n) > 4096, beyond the screen's k' range): the reference's own
// algorithm restated on the GPU -- every score in float64, a full descending sort, the first k
// (lib.py:51-55: cosine_similarity(...).mean(axis=0), .loc[unrated], .sort_values(ascending=
// False)[:k]; pandas core/series.py:3706-3716). No screen, no certificate: nothing is approximate.
//
// Per group of Bg queries (float64 scores of Bg x n as 64-bit order keys, ~1 GiB at most):
//   exact_keys_kernel  key[b][i] = order key of (q64_b . c_i) / gnorm64_i (the float64 FMA
//                      tiling of the EXACT screen, rescore.hip); a NaN score (a catalog row with
//                      a NaN / inf element) gets key 0 and is dropped like an excluded row: the
//                      convention of every other path of the library, whose selects never take
//                      a NaN (include/ebert.h, "Non-finite catalog rows")
//   mask_keys_kernel   the query's excluded rows (its CSR segment) -> key 0 (dropped)
//   lk_block_sort_kernel  per query, runs of LK_RUN (key, row) pairs sorted in LDS (bitonic on
//                      (key desc, row asc) -- the rows are distinct, so that order is total and
//                      ties of the score keep row order: the (score desc, row asc) order of the
//                      rest of the library)
//   lk_merge_kernel    pairwise merges of the runs by merge path (each thread finds its first
//                      output's split by binary search and merges LK_ITEMS outputs), alternating
//                      between two buffers; a merged run is cut at k entries (only the first k
//                      can reach the answer), so once runs are k long every pass halves the data
//   large_out_kernel   the first k entries of the one remaining run -> out_scores / out_rows,
//                      NaN / -1 past the query's valid rows.
// Round 6: hand-written, replacing one radix sort per query through the CUB-compatible API.
// A rare path (no caller of the reference asks for more than k = 100): plain, not tuned.
#include "common.h"

namespace ebt {

namespace {

constexpr int LT = 64, LK = 16;
constexpr int64_t LARGE_KEY_BUDGET = 1LL << 30;  // key bytes of one group of queries
constexpr int64_t LARGE_GROUP_MAX = 64;

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

__device__ __forceinline__ uint64_t score_key(double v) {
  if (v != v) return 0ull;  // NaN: not a candidate (the key of an excluded row)
  v += 0.0;  // -0 -> +0: one value, as they compare equal
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_score(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)u);
}

template <int DT>
__global__ __launch_bounds__(256) void exact_keys_kernel(
    const double* __restrict__ q64, int64_t B, int d, const void* __restrict__ cat, int64_t ld,
    const double* __restrict__ gnorm, int64_t n, uint64_t* __restrict__ keys) {
  __shared__ double qs[LK][LT + 1], cs[LK][LT + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * LT, b0 = (int64_t)blockIdx.y * LT;
  double acc[4][4] = {};
  for (int k0 = 0; k0 < d; k0 += LK) {
    // the tile's 4 elements per thread loaded before any is stored (guarded loads would each
    // be waited for in turn): out-of-range indices read a clamped in-range element, then 0
    constexpr int NE = LT * LK / 256;
    double cv[NE], qv[NE];
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      const int rr = e / LK, kk = e % LK;
      const int64_t row = r0 + rr, qb = b0 + rr;
      const int kc = k0 + kk < d ? k0 + kk : d - 1;
      cv[u] = load_as_f64<DT>(cat, (row < n ? row : n - 1) * ld + kc);
      qv[u] = q64[(qb < B ? qb : B - 1) * d + kc];
    }
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      const int rr = e / LK, kk = e % LK;
      const int64_t row = r0 + rr, qb = b0 + rr;
      const bool kin = k0 + kk < d;
      cs[kk][rr] = (kin && row < n) ? cv[u] : 0.0;
      qs[kk][rr] = (kin && qb < B) ? qv[u] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < LK; ++kk) {
      double a[4], c[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = qs[kk][ty * 4 + i];
        c[i] = cs[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fma(a[i], c[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t qb = b0 + ty * 4 + i;
    if (qb >= B) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = r0 + tx * 4 + j;
      if (row < n) keys[qb * n + row] = score_key(acc[i][j] / gnorm[row]);
    }
  }
}

// one block per query of the group: its excluded (global) rows -> key 0
__global__ void mask_keys_kernel(uint64_t* __restrict__ keys, int64_t n,
                                 const int64_t* __restrict__ eo, const int64_t* __restrict__ er,
                                 int64_t row_offset) {
  const int64_t j = blockIdx.x;
  for (int64_t t = eo[j] + threadIdx.x; t < eo[j + 1]; t += blockDim.x) {
    const int64_t r = er[t] - row_offset;
    if (r >= 0 && r < n) keys[j * n + r] = 0ull;
  }
}

constexpr int LK_THREADS = 256;
constexpr int LK_RUN = 2048;   // pairs sorted in LDS per workgroup (24 KiB)
constexpr int LK_ITEMS = 8;    // merge outputs per thread

// (key desc, row asc): the order of the results
__device__ __forceinline__ bool lk_before(uint64_t ka, int32_t ra, uint64_t kb, int32_t rb) {
  return ka > kb || (ka == kb && ra < rb);
}

// keys[q][r0 + i] with rows r0 + i, sorted per run of LK_RUN in place (rows into ids)
__global__ __launch_bounds__(LK_THREADS) void lk_block_sort_kernel(uint64_t* __restrict__ keys,
                                                                    int32_t* __restrict__ ids,
                                                                    int64_t n) {
  __shared__ uint64_t sk[LK_RUN];
  __shared__ int32_t sr[LK_RUN];
  const int64_t q = blockIdx.y, r0 = (int64_t)blockIdx.x * LK_RUN;
  const int m = n - r0 < LK_RUN ? (int)(n - r0) : LK_RUN;
  uint64_t* k = keys + q * n + r0;
  for (int i = threadIdx.x; i < LK_RUN; i += LK_THREADS) {
    sk[i] = i < m ? k[i] : 0ull;
    sr[i] = i < m ? (int32_t)(r0 + i) : INT32_MAX;   // padding sorts last
  }
  __syncthreads();
  for (int size = 2; size <= LK_RUN; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < LK_RUN / 2; t += LK_THREADS) {
        const int lo = ((t & ~(stride - 1)) << 1) | (t & (stride - 1));
        const int hi = lo + stride;
        const uint64_t ka = sk[lo], kb = sk[hi];
        const int32_t ra = sr[lo], rb = sr[hi];
        const bool first = (lo & size) == 0;
        if (first ? lk_before(kb, rb, ka, ra) : lk_before(ka, ra, kb, rb)) {
          sk[lo] = kb;
          sk[hi] = ka;
          sr[lo] = rb;
          sr[hi] = ra;
        }
      }
      __syncthreads();
    }
  }
  int32_t* id = ids + q * n + r0;
  for (int i = threadIdx.x; i < m; i += LK_THREADS) {
    k[i] = sk[i];
    id[i] = sr[i];
  }
}

// One merge pass: run j of the input holds min(cap_in, len of its window) entries at
// [j * slot_in, ...), the window of run j being rows [j w, (j + 1) w) of the query; output run j
// merges input runs 2j and 2j + 1 and keeps its first min(k, ...) entries at j * slot_out.
// grid: (output pieces of LK_THREADS * LK_ITEMS, output runs, queries)
__global__ __launch_bounds__(LK_THREADS) void lk_merge_kernel(
    const uint64_t* __restrict__ ks, const int32_t* __restrict__ is, uint64_t* __restrict__ kd,
    int32_t* __restrict__ id, int64_t n, int64_t w, int64_t slot_in, int64_t slot_out, int64_t k) {
  const int64_t q = blockIdx.z, j = blockIdx.y;
  auto run_len = [&](int64_t r) {
    const int64_t lo = r * w;
    const int64_t m = lo >= n ? 0 : (n - lo < w ? n - lo : w);
    return m < k ? m : k;
  };
  const int64_t la = run_len(2 * j), lb = run_len(2 * j + 1);
  const int64_t tot = la + lb < k ? la + lb : k;
  const uint64_t* ak = ks + q * n + 2 * j * slot_in;
  const int32_t* ai = is + q * n + 2 * j * slot_in;
  const uint64_t* bk = ak + slot_in;
  const int32_t* bi = ai + slot_in;
  uint64_t* ok = kd + q * n + j * slot_out;
  int32_t* oi = id + q * n + j * slot_out;
  const int64_t o0 = ((int64_t)blockIdx.x * LK_THREADS + threadIdx.x) * LK_ITEMS;
  if (o0 >= tot) return;
  // merge path: how many of the first o0 outputs come from A
  int64_t lo = o0 > lb ? o0 - lb : 0, hi = o0 < la ? o0 : la;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int64_t bj = o0 - 1 - mid;
    if (lk_before(ak[mid], ai[mid], bk[bj], bi[bj])) lo = mid + 1;
    else hi = mid;
  }
  int64_t a = lo, bb = o0 - lo;
  const int64_t o1 = o0 + LK_ITEMS < tot ? o0 + LK_ITEMS : tot;
  for (int64_t o = o0; o < o1; ++o) {
    const bool fromA = bb >= lb || (a < la && lk_before(ak[a], ai[a], bk[bb], bi[bb]));
    if (fromA) {
      ok[o] = ak[a];
      oi[o] = ai[a];
      ++a;
    } else {
      ok[o] = bk[bb];
      oi[o] = bi[bb];
      ++bb;
    }
  }
}

__global__ void large_out_kernel(const uint64_t* __restrict__ keys, const int32_t* __restrict__ rows,
                                 int64_t n, int k, int64_t row_offset, double* __restrict__ os,
                                 int64_t* __restrict__ orow) {
  const int64_t q = blockIdx.y;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k;
       t += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = t < n ? keys[q * n + t] : 0ull;
    os[q * k + t] = key ? key_score(key) : __builtin_nan("");
    orow[q * k + t] = key ? (int64_t)rows[q * n + t] + row_offset : -1;
  }
}

}  // namespace

// Workspace of the large-k path (queries prepared elsewhere): two buffers of Bg x n (key, row)
// pairs (12 bytes each). 0 when n is beyond the merge grid (2.7e8 rows).
size_t large_topk_bytes(int64_t B, int64_t n, int64_t* Bg_out) {
  // (n: the merge grid's run count ceil(n / 2 LK_RUN) within 65535)
  if (B < 1 || n < 1 || n > 65535LL * 2 * LK_RUN) return 0;
  int64_t Bg = LARGE_KEY_BUDGET / (24 * n);
  Bg = Bg < 1 ? 1 : Bg;
  Bg = Bg > LARGE_GROUP_MAX ? LARGE_GROUP_MAX : Bg;
  Bg = Bg > B ? B : Bg;
  if (Bg_out) *Bg_out = Bg;
  return 2 * (al256((size_t)Bg * n * 8) + al256((size_t)Bg * n * 4));
}

int large_topk(const double* q64, int64_t B, int32_t d, const void* cat, int dtype, int64_t ld,
               const double* gnorm, int64_t n, int64_t row_offset, const int64_t* excl_off,
               const int64_t* excl_rows, int32_t k, double* out_s, int64_t* out_r, void* ws,
               size_t ws_bytes, hipStream_t st) {
  int64_t Bg = 0;
  const size_t need = large_topk_bytes(B, n, &Bg);
  if (need == 0 || ws_bytes < need || !q64 || !cat || !gnorm || !out_s || !out_r || k < 1) {
    set_error("large_topk: bad arguments (B=%lld n=%lld k=%d ws=%zu need=%zu)", (long long)B,
              (long long)n, k, ws_bytes, need);
    return EBT_EINVAL;
  }
  char* w = (char*)ws;
  uint64_t* k0 = (uint64_t*)w;
  w += al256((size_t)Bg * n * 8);
  int32_t* i0 = (int32_t*)w;
  w += al256((size_t)Bg * n * 4);
  uint64_t* k1 = (uint64_t*)w;
  w += al256((size_t)Bg * n * 8);
  int32_t* i1 = (int32_t*)w;
  int rc = EBT_OK;
  for (int64_t b0 = 0; b0 < B; b0 += Bg) {
    const int64_t m = B - b0 < Bg ? B - b0 : Bg;
    const dim3 grid((unsigned)ceil_div(n, LT), (unsigned)ceil_div(m, LT)), block(256);
    const double* q = q64 + b0 * d;
    switch (dtype) {
      case EBT_F32:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_F32>, grid, block, 0, st, q, m, d, cat, ld, gnorm,
                           n, k0);
        break;
      case EBT_BF16:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_BF16>, grid, block, 0, st, q, m, d, cat, ld,
                           gnorm, n, k0);
        break;
      case EBT_F16:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_F16>, grid, block, 0, st, q, m, d, cat, ld, gnorm,
                           n, k0);
        break;
      default:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_F64>, grid, block, 0, st, q, m, d, cat, ld, gnorm,
                           n, k0);
        break;
    }
    rc = launch_check("exact_keys_kernel");
    if (rc) return rc;
    if (excl_off) {
      hipLaunchKernelGGL(mask_keys_kernel, dim3((unsigned)m), dim3(256), 0, st, k0, n,
                         excl_off + b0, excl_rows, row_offset);
      rc = launch_check("mask_keys_kernel");
      if (rc) return rc;
    }
    hipLaunchKernelGGL(lk_block_sort_kernel, dim3((unsigned)ceil_div(n, LK_RUN), (unsigned)m),
                       dim3(LK_THREADS), 0, st, k0, i0, n);
    rc = launch_check("lk_block_sort_kernel");
    if (rc) return rc;
    uint64_t *ks = k0, *kd = k1;
    int32_t *is = i0, *id = i1;
    for (int64_t w2 = LK_RUN; w2 < n; w2 <<= 1) {
      const int64_t slot_in = w2 < k ? w2 : k, slot_out = 2 * w2 < k ? 2 * w2 : k;
      const int64_t runs_out = ceil_div(n, 2 * w2);
      const dim3 mg((unsigned)ceil_div(slot_out, (int64_t)LK_THREADS * LK_ITEMS),
                    (unsigned)runs_out, (unsigned)m);
      hipLaunchKernelGGL(lk_merge_kernel, mg, dim3(LK_THREADS), 0, st, ks, is, kd, id, n, w2,
                         slot_in, slot_out, (int64_t)k);
      rc = launch_check("lk_merge_kernel");
      if (rc) return rc;
      std::swap(ks, kd);
      std::swap(is, id);
    }
    const int64_t blocks = ceil_div(k, 256) < 1024 ? ceil_div(k, 256) : 1024;
    hipLaunchKernelGGL(large_out_kernel, dim3((unsigned)blocks, (unsigned)m), dim3(256), 0, st,
                       ks, is, n, k, row_offset, out_s + b0 * k, out_r + b0 * k);
    rc = launch_check("large_out_kernel");
    if (rc) return rc;
  }
  return EBT_OK;
}

}  // namespace ebt
