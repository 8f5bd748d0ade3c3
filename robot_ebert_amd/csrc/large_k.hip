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
//   per query: hipcub DeviceRadixSort (keys descending, row ids as values; a radix sort is
//              stable and the ids enter in ascending order, so ties keep row order: the
//              (score desc, row asc) order of the rest of the library), then the first k
//              entries -> out_scores / out_rows, NaN / -1 past the query's valid rows.
// A rare path (no caller of the reference asks for more than k = 100): plain, not tuned.
#include "common.h"  // hip_runtime first: hipcub's platform checks need it

#include <hipcub/device/device_radix_sort.hpp>

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

__global__ void iota_kernel(int32_t* __restrict__ v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    v[i] = (int32_t)i;
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

__global__ void large_out_kernel(const uint64_t* __restrict__ keys, const int32_t* __restrict__ rows,
                                 int64_t n, int k, int64_t row_offset, double* __restrict__ os,
                                 int64_t* __restrict__ orow) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k;
       t += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = t < n ? keys[t] : 0ull;
    os[t] = key ? key_score(key) : __builtin_nan("");
    orow[t] = key ? (int64_t)rows[t] + row_offset : -1;
  }
}

size_t sort_temp_bytes(int64_t n) {
  size_t b = 0;
  if (hipcub::DeviceRadixSort::SortPairsDescending(
          (void*)nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
          (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 64, (hipStream_t)0) !=
      hipSuccess)
    return 0;
  return b;
}

}  // namespace

// Workspace of the large-k path (queries prepared elsewhere): [group keys Bg x n] [row ids n]
// [sorted keys n] [sorted ids n] [radix-sort temporaries]. 0 when n does not fit an int.
size_t large_topk_bytes(int64_t B, int64_t n, int64_t* Bg_out) {
  if (B < 1 || n < 1 || n > 0x7fffffffLL) return 0;
  int64_t Bg = LARGE_KEY_BUDGET / (8 * n);
  Bg = Bg < 1 ? 1 : Bg;
  Bg = Bg > LARGE_GROUP_MAX ? LARGE_GROUP_MAX : Bg;
  Bg = Bg > B ? B : Bg;
  const size_t temp = sort_temp_bytes(n);
  if (temp == 0) return 0;
  if (Bg_out) *Bg_out = Bg;
  return al256((size_t)Bg * n * 8) + al256((size_t)n * 4) + al256((size_t)n * 8) +
         al256((size_t)n * 4) + al256(temp);
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
  uint64_t* gkeys = (uint64_t*)w;
  w += al256((size_t)Bg * n * 8);
  int32_t* ids = (int32_t*)w;
  w += al256((size_t)n * 4);
  uint64_t* skeys = (uint64_t*)w;
  w += al256((size_t)n * 8);
  int32_t* sids = (int32_t*)w;
  w += al256((size_t)n * 4);
  void* temp = w;
  size_t temp_bytes = sort_temp_bytes(n);
  hipLaunchKernelGGL(iota_kernel, dim3(1024), dim3(256), 0, st, ids, n);
  int rc = launch_check("iota_kernel");
  if (rc) return rc;
  for (int64_t b0 = 0; b0 < B; b0 += Bg) {
    const int64_t m = B - b0 < Bg ? B - b0 : Bg;
    const dim3 grid((unsigned)ceil_div(n, LT), (unsigned)ceil_div(m, LT)), block(256);
    const double* q = q64 + b0 * d;
    switch (dtype) {
      case EBT_F32:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_F32>, grid, block, 0, st, q, m, d, cat, ld, gnorm,
                           n, gkeys);
        break;
      case EBT_BF16:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_BF16>, grid, block, 0, st, q, m, d, cat, ld,
                           gnorm, n, gkeys);
        break;
      case EBT_F16:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_F16>, grid, block, 0, st, q, m, d, cat, ld, gnorm,
                           n, gkeys);
        break;
      default:
        hipLaunchKernelGGL(exact_keys_kernel<EBT_F64>, grid, block, 0, st, q, m, d, cat, ld, gnorm,
                           n, gkeys);
        break;
    }
    rc = launch_check("exact_keys_kernel");
    if (rc) return rc;
    if (excl_off) {
      hipLaunchKernelGGL(mask_keys_kernel, dim3((unsigned)m), dim3(256), 0, st, gkeys, n,
                         excl_off + b0, excl_rows, row_offset);
      rc = launch_check("mask_keys_kernel");
      if (rc) return rc;
    }
    for (int64_t j = 0; j < m; ++j) {
      rc = hip_check(hipcub::DeviceRadixSort::SortPairsDescending(
                         temp, temp_bytes, (const uint64_t*)(gkeys + j * n), skeys,
                         (const int32_t*)ids, sids, (int)n, 0, 64, st),
                     "hipcub radix sort");
      if (rc) return rc;
      const int64_t blocks = ceil_div(k, 256) < 1024 ? ceil_div(k, 256) : 1024;
      hipLaunchKernelGGL(large_out_kernel, dim3((unsigned)blocks), dim3(256), 0, st, skeys, sids,
                         n, k, row_offset, out_s + (b0 + j) * k, out_r + (b0 + j) * k);
      rc = launch_check("large_out_kernel");
      if (rc) return rc;
    }
  }
  return EBT_OK;
}

}  // namespace ebt
