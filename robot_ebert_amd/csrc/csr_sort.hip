// ebt_sort_exclusions: every segment of a caller's exclusion CSR sorted ascending on the device,
// so that the rated-movie lists of lib.py:48,55 (`catalog.index.difference(rated)` then
// `.loc[unrated]`) can be handed over in any order. The search entry points binary-search the
// segments and reject unsorted ones (include/ebert.h, ebt_cosine_topk); this is the one place
// a caller's order is fixed, for the C ABI and the Python layer alike.
//
// Offsets are ABSOLUTE positions into rows[0, nnz): segment b is rows[off[b], off[b+1]), so
// off[0] may be > 0 (a sub-batch that slices the offsets of a larger CSR) and positions outside
// every segment keep their value. The offsets are clamped into [0, nnz] on the device before the
// sort reads them (a malformed CSR sorts what lies inside its clamped segments and is rejected
// by the search entry's own check; it never makes the sort read out of bounds).
//
// One launch, one workgroup per segment (round 6: hand-written, replacing a segmented radix sort
// of the CUB-compatible API -- a key-width radix pass per 8 bits over segments that hold a few
// hundred rows). A segment is read ONCE into LDS and its order checked there: a sorted segment
// (the usual case: lists built sorted on the host) is only copied (out of place) or left alone
// (in place); an unsorted one of up to XS_LDS rows is bitonic-sorted in LDS and written back.
// Longer segments (a user with thousands of rated movies) sort XS_LDS-row runs in LDS into the
// workspace and merge them pairwise in global memory by merge path, the workgroup's threads each
// producing XS_ITEMS consecutive outputs of a pass; passes alternate between the workspace and
// rows_out. Extra workgroups past the segments copy the head [0, begin[0]) and the tail
// [end[B-1], nnz) out of place.
#include "common.h"

namespace ebt {

namespace {

constexpr int XS_THREADS = 256;
constexpr int XS_LDS = 4096;      // rows sorted in LDS at once (32 KiB)
constexpr int XS_ITEMS = 8;       // merge outputs per thread and round
constexpr int XS_COPY_BLOCKS = 64;

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

__device__ __forceinline__ int64_t clamp_off(int64_t x, int64_t nnz) {
  return x < 0 ? 0 : (x > nnz ? nnz : x);
}

// ascending bitonic sort of v[0, P) in LDS (P a power of two <= XS_LDS), whole workgroup
__device__ void bitonic_i64(int64_t* v, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += XS_THREADS) {
        const int lo = ((t & ~(stride - 1)) << 1) | (t & (stride - 1));
        const int hi = lo + stride;
        const int64_t a = v[lo], c = v[hi];
        const bool up = (lo & size) == 0;
        if (up ? a > c : a < c) {
          v[lo] = c;
          v[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

// rows [s, s + m) of src (m <= XS_LDS) into LDS, INT64_MAX past them up to P; returns whether
// the m rows were already ascending
__device__ bool load_run(int64_t* v, const int64_t* __restrict__ src, int64_t s, int m, int P) {
  for (int i = threadIdx.x; i < P; i += XS_THREADS) v[i] = i < m ? src[s + i] : INT64_MAX;
  __syncthreads();
  int bad = 0;
  for (int i = threadIdx.x; i + 1 < m; i += XS_THREADS) bad |= v[i] > v[i + 1];
  return !__syncthreads_or(bad);
}

// merge path: of the first `diag` outputs of merge(A[0, la), B[0, lb)) (ascending, A first on
// ties), how many come from A
__device__ __forceinline__ int64_t merge_split(const int64_t* __restrict__ A, int64_t la,
                                               const int64_t* __restrict__ Bv, int64_t lb,
                                               int64_t diag) {
  int64_t lo = diag > lb ? diag - lb : 0, hi = diag < la ? diag : la;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (A[mid] <= Bv[diag - 1 - mid]) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(XS_THREADS) void sort_segments_kernel(
    const int64_t* __restrict__ off, int64_t B, int64_t nnz, const int64_t* rows_in,
    int64_t* rows_out, int64_t* __restrict__ tmp) {
  __shared__ int64_t v[XS_LDS];
  const int tid = threadIdx.x;
  if ((int64_t)blockIdx.x >= B) {
    // copy blocks (out of place only): the head and the tail outside every clamped segment
    // (begin[b] = clamp(off[b]), end[b] = clamp(max(off[b+1], off[b])): consecutive clamped
    // segments leave no gap between them)
    const int64_t head = clamp_off(off[0], nnz);
    int64_t tail = clamp_off(off[B], nnz);
    const int64_t lastb = clamp_off(off[B - 1], nnz);
    tail = tail < lastb ? lastb : tail;
    const int64_t t0 = ((int64_t)blockIdx.x - B) * XS_THREADS + tid;
    const int64_t stride = (int64_t)XS_COPY_BLOCKS * XS_THREADS;
    for (int64_t i = t0; i < head; i += stride) rows_out[i] = rows_in[i];
    for (int64_t i = tail + t0; i < nnz; i += stride) rows_out[i] = rows_in[i];
    return;
  }
  const int64_t b = blockIdx.x;
  const int64_t s = clamp_off(off[b], nnz), e0 = off[b + 1];
  const int64_t e = e0 < s ? s : (e0 > nnz ? nnz : e0);
  const int64_t len = e - s;
  if (len <= 0) return;
  const bool in_place = rows_out == rows_in;
  if (len <= XS_LDS) {
    int P = 1;
    while (P < len) P <<= 1;
    if (load_run(v, rows_in, s, (int)len, P)) {
      if (!in_place)
        for (int i = tid; i < len; i += XS_THREADS) rows_out[s + i] = v[i];
      return;
    }
    bitonic_i64(v, P);
    for (int i = tid; i < len; i += XS_THREADS) rows_out[s + i] = v[i];
    return;
  }
  // a long segment: already ascending?
  int bad = 0;
  for (int64_t i = s + tid; i + 1 < e; i += XS_THREADS) bad |= rows_in[i] > rows_in[i + 1];
  if (!__syncthreads_or(bad)) {
    if (!in_place)
      for (int64_t i = s + tid; i < e; i += XS_THREADS) rows_out[i] = rows_in[i];
    return;
  }
  // runs of XS_LDS rows sorted in LDS into tmp (same absolute positions)
  for (int64_t r0 = s; r0 < e; r0 += XS_LDS) {
    const int m = e - r0 < XS_LDS ? (int)(e - r0) : XS_LDS;
    int P = 1;
    while (P < m) P <<= 1;
    (void)load_run(v, rows_in, r0, m, P);
    bitonic_i64(v, P);
    for (int i = tid; i < m; i += XS_THREADS) tmp[r0 + i] = v[i];
    __syncthreads();
  }
  // pairwise merges, tmp -> rows_out -> tmp ...; the workgroup's global writes are visible to
  // its own threads after the barrier (one CU, workgroup-scope fence)
  int64_t* src = tmp;
  int64_t* dst = rows_out;
  for (int64_t w = XS_LDS; w < len; w <<= 1) {
    for (int64_t p0 = 0; p0 < len; p0 += 2 * w) {
      const int64_t la = len - p0 < w ? len - p0 : w;
      const int64_t lb = len - p0 - la < w ? len - p0 - la : w;
      const int64_t* A = src + s + p0;
      const int64_t* Bv = A + la;
      int64_t* out = dst + s + p0;
      const int64_t tot = la + lb;
      for (int64_t o0 = (int64_t)tid * XS_ITEMS; o0 < tot; o0 += (int64_t)XS_THREADS * XS_ITEMS) {
        int64_t i = merge_split(A, la, Bv, lb, o0), j = o0 - i;
        const int64_t o1 = o0 + XS_ITEMS < tot ? o0 + XS_ITEMS : tot;
        for (int64_t o = o0; o < o1; ++o) {
          const bool fromA = j >= lb || (i < la && A[i] <= Bv[j]);
          out[o] = fromA ? A[i++] : Bv[j++];
        }
      }
    }
    __syncthreads();
    int64_t* t = src;
    src = dst;
    dst = t;
  }
  if (src != rows_out)  // an odd number of passes left the result in tmp
    for (int64_t i = s + tid; i < e; i += XS_THREADS) rows_out[i] = src[i];
}

}  // namespace

}  // namespace ebt

using namespace ebt;

extern "C" {

size_t ebt_sort_exclusions_bytes(int64_t B, int64_t nnz) {
  // (B: one workgroup per segment, the grid's threads within 32 bits)
  if (B < 1 || nnz < 0 || nnz > 0x7fffffffLL || B > (1LL << 24)) return 0;
  return al256((size_t)(nnz > 0 ? nnz : 1) * 8);
}

int ebt_sort_exclusions(const int64_t* off, const int64_t* rows_in, int64_t* rows_out, int64_t B,
                        int64_t nnz, void* workspace, size_t ws_bytes, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t need = ebt_sort_exclusions_bytes(B, nnz);
  if (need == 0 || !off || (nnz > 0 && (!rows_in || !rows_out)) || !workspace ||
      ws_bytes < need) {
    set_error("ebt_sort_exclusions: bad arguments (B=%lld nnz=%lld ws=%zu need=%zu)",
              (long long)B, (long long)nnz, ws_bytes, need);
    return EBT_EINVAL;
  }
  if (nnz <= 1) {
    if (nnz == 1 && rows_out != rows_in)
      return hip_check(hipMemcpyAsync(rows_out, rows_in, 8, hipMemcpyDeviceToDevice, st),
                       "hipMemcpyAsync");
    return EBT_OK;
  }
  const int64_t grid = B + (rows_out != rows_in ? XS_COPY_BLOCKS : 0);
  hipLaunchKernelGGL(sort_segments_kernel, dim3((unsigned)grid), dim3(XS_THREADS), 0, st, off, B,
                     nnz, rows_in, rows_out, (int64_t*)workspace);
  return launch_check("sort_segments_kernel");
}

}  // extern "C"
