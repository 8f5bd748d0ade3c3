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
#include "common.h"  // hip_runtime first: hipcub's platform checks need it

#include <hipcub/device/device_segmented_radix_sort.hpp>

namespace ebt {

namespace {

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

// begin[b] = clamp(off[b]), end[b] = clamp(max(off[b + 1], off[b])): inside [0, nnz]. Then
// end[b] >= begin[b + 1] for every b, so the clamped segments leave no gap between them: the only
// positions outside every segment are the head [0, begin[0]) and the tail [end[B - 1], nnz),
// which `keep` (rows_out when it is not rows_in) receives from rows_in here
__global__ void clamp_offsets_kernel(const int64_t* __restrict__ off, int64_t B, int64_t nnz,
                                     int64_t* __restrict__ begin, int64_t* __restrict__ end,
                                     const int64_t* __restrict__ rows_in,
                                     int64_t* __restrict__ keep) {
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto clamp = [&](int64_t x) { return x < 0 ? 0 : (x > nnz ? nnz : x); };
  for (int64_t b = t0; b < B; b += stride) {
    const int64_t s = clamp(off[b]), e0 = off[b + 1];
    const int64_t e = e0 < s ? s : (e0 > nnz ? nnz : e0);
    begin[b] = s;
    end[b] = e;
  }
  if (keep) {
    const int64_t head = clamp(off[0]);
    int64_t tail = clamp(off[B]);
    const int64_t lastb = clamp(off[B - 1]);
    tail = tail < lastb ? lastb : tail;   // end[B - 1]
    for (int64_t i = t0; i < head; i += stride) keep[i] = rows_in[i];
    for (int64_t i = tail + t0; i < nnz; i += stride) keep[i] = rows_in[i];
  }
}

size_t sort_temp_bytes(int64_t B, int64_t nnz) {
  size_t b = 0;
  if (hipcub::DeviceSegmentedRadixSort::SortKeys(
          (void*)nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr, (int)nnz, (int)B,
          (const int64_t*)nullptr, (const int64_t*)nullptr, 0, 64, (hipStream_t)0) != hipSuccess)
    return 0;
  return b;
}

}  // namespace

}  // namespace ebt

using namespace ebt;

extern "C" {

size_t ebt_sort_exclusions_bytes(int64_t B, int64_t nnz) {
  if (B < 1 || nnz < 0 || nnz > 0x7fffffffLL || B > 0x7fffffffLL) return 0;
  const size_t temp = sort_temp_bytes(B, nnz > 0 ? nnz : 1);
  if (temp == 0) return 0;
  return al256((size_t)(nnz > 0 ? nnz : 1) * 8) + 2 * al256((size_t)B * 8) + al256(temp);
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
  char* w = (char*)workspace;
  int64_t* keys = (int64_t*)w;
  w += al256((size_t)nnz * 8);
  int64_t* begin = (int64_t*)w;
  w += al256((size_t)B * 8);
  int64_t* end = (int64_t*)w;
  w += al256((size_t)B * 8);
  size_t temp_bytes = sort_temp_bytes(B, nnz);
  // the sort reads its keys from rows_in straight into rows_out when they differ (the clamp
  // kernel copies the head and tail outside every segment); in place, from a copy in `keys`.
  // Positions outside every segment keep their value either way.
  const bool in_place = rows_out == rows_in;
  int rc = EBT_OK;
  if (in_place)
    rc = hip_check(hipMemcpyAsync(keys, rows_in, (size_t)nnz * 8, hipMemcpyDeviceToDevice, st),
                   "hipMemcpyAsync");
  if (rc) return rc;
  const int64_t need_thr = B > nnz ? B : nnz;
  const int64_t blocks = ceil_div(need_thr, 256) < 1024 ? ceil_div(need_thr, 256) : 1024;
  hipLaunchKernelGGL(clamp_offsets_kernel, dim3((unsigned)blocks), dim3(256), 0, st, off, B, nnz,
                     begin, end, rows_in, in_place ? nullptr : rows_out);
  rc = launch_check("clamp_offsets_kernel");
  if (rc) return rc;
  return hip_check(hipcub::DeviceSegmentedRadixSort::SortKeys(
                       w, temp_bytes, in_place ? (const int64_t*)keys : rows_in, rows_out,
                       (int)nnz, (int)B, (const int64_t*)begin, (const int64_t*)end, 0, 64, st),
                   "hipcub segmented radix sort");
}

}  // extern "C"
