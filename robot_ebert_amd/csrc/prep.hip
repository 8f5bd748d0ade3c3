// Load-time and per-batch preparation kernels (all HBM-bound, vectorised 16 B per lane).
//
//  * row_norms      -- sklearn row_norms + _handle_zeros_in_scale (utils/extmath.py:76,
//                      preprocessing/_data.py:118-123,2011): guarded float64 L2 norm per row.
//                      The reference recomputes this for the whole catalog on EVERY call
//                      (metrics/pairwise.py:1730-1734); here it runs once at catalog load
//                      (constants.py:55-56) and is kept resident in HBM.
//  * screen_image   -- the f16/bf16 MFMA operand of a matrix (normalised or raw), zero-padded to
//                      a multiple of 64 columns.
//  * query_dense / query_liked_sum / scale_rows -- q64 = normalize(q), or the liked-row mean of
//                      lib.py:51-52 folded into ONE query vector per user (sum here, 1/L later).
//  * query_image    -- the query's MFMA operand, its epilogue scale and the certification bound.
//  * mask_excluded  -- rated movies are not candidates (lib.py:48,55).
#include "common.h"

namespace ebt {

// ---------------------------------------------------------------------------- row norms ----
template <int DT, bool VEC>
__global__ __launch_bounds__(256) void row_norms_kernel(const void* __restrict__ x, int64_t n,
                                                         int d, int64_t ld,
                                                         double* __restrict__ gnorm,
                                                         float* __restrict__ inv32) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  double s = 0.0;
  if constexpr (VEC) {
    constexpr int ES = (DT == EBT_F64) ? 8 : (DT == EBT_F32 ? 4 : 2);
    constexpr int PER = 16 / ES;  // elements per 16-byte chunk
    const char* base = (const char*)x + row * ld * ES;
    const int nchunks = d / PER;
    for (int c = lane; c < nchunks; c += 64) {
      const uint4 raw = *(const uint4*)(base + (int64_t)c * 16);
      if constexpr (DT == EBT_F32) {
        const float* f = (const float*)&raw;
#pragma unroll
        for (int e = 0; e < 4; ++e) s += (double)f[e] * (double)f[e];
      } else if constexpr (DT == EBT_F64) {
        const double* f = (const double*)&raw;
        s += f[0] * f[0] + f[1] * f[1];
      } else {
        const uint16_t* h = (const uint16_t*)&raw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const double v = DT == EBT_BF16 ? bf16_bits_to_f64(h[e]) : f16_bits_to_f64(h[e]);
          s += v * v;
        }
      }
    }
  } else {
    for (int j = lane; j < d; j += 64) {
      const double v = load_as_f64<DT>(x, row * ld + j);
      s += v * v;
    }
  }
  s = wave_sum_f64(s);
  if (lane == 0) {
    const double g = guard_norm(sqrt(s));
    gnorm[row] = g;
    if (inv32) inv32[row] = (float)(1.0 / g);
  }
}

static bool vec_ok(const void* p, int dtype, int64_t ld, int d) {
  const int es = dtype == EBT_F64 ? 8 : (dtype == EBT_F32 ? 4 : 2);
  return (((uintptr_t)p & 15) == 0) && ((ld * es) % 16 == 0) && (((int64_t)d * es) % 16 == 0);
}

int row_norms(const void* x, int dtype, int64_t n, int32_t d, int64_t ld, double* gnorm,
              float* inv32, hipStream_t st) {
  if (!x || !gnorm || n < 0 || d <= 0 || ld < d || dtype < 0 || dtype > 3) {
    set_error("ebt_row_norms: bad arguments");
    return EBT_EINVAL;
  }
  if (n == 0) return EBT_OK;
  const bool v = vec_ok(x, dtype, ld, d);
  dim3 grid((unsigned)ceil_div(n, 4)), block(256);
#define EBT_RN(DT)                                                                         \
  if (v) hipLaunchKernelGGL((row_norms_kernel<DT, true>), grid, block, 0, st, x, n, d, ld, \
                            gnorm, inv32);                                                 \
  else hipLaunchKernelGGL((row_norms_kernel<DT, false>), grid, block, 0, st, x, n, d, ld,  \
                          gnorm, inv32);
  switch (dtype) {
    case EBT_F32: EBT_RN(EBT_F32) break;
    case EBT_BF16: EBT_RN(EBT_BF16) break;
    case EBT_F16: EBT_RN(EBT_F16) break;
    default: EBT_RN(EBT_F64) break;
  }
#undef EBT_RN
  return launch_check("row_norms_kernel");
}

// ------------------------------------------------------------------------- screen image ----
// One wave per row (grid-stride over rows): the row's scale 1/gnorm is computed once per lane,
// lanes take consecutive 16-byte output chunks (coalesced loads and stores), and with VEC the 8
// source elements of a chunk come in 16-byte vector loads (one for 16-bit sources, two for f32,
// four for f64). Same arithmetic as the element form: round_to(img, x * (1/gnorm)) in float64.
template <int DT>
__device__ __forceinline__ void load8_f64(const void* __restrict__ x, int64_t off, double (&v)[8]) {
  if constexpr (DT == EBT_F32) {
    const float4 a = *(const float4*)((const float*)x + off);
    const float4 b = *(const float4*)((const float*)x + off + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else if constexpr (DT == EBT_F64) {
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const double2 a = *(const double2*)((const double*)x + off + e);
      v[e] = a.x;
      v[e + 1] = a.y;
    }
  } else {
    const u16x8_t h = *(const u16x8_t*)((const uint16_t*)x + off);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = DT == EBT_BF16 ? bf16_bits_to_f64(h[e]) : f16_bits_to_f64(h[e]);
  }
}

// (image value - x)^2 in float64, for the image's measured rounding error
template <int IMG>
__device__ __forceinline__ double sq_err(uint16_t h, double x) {
  const double r = (IMG == EBT_F16 ? f16_bits_to_f64(h) : bf16_bits_to_f64(h)) - x;
  return r * r;
}

template <int DT, int IMG, bool VEC>
__global__ __launch_bounds__(256) void screen_image_kernel(const void* __restrict__ x, int64_t n,
                                                            int d, int64_t ld,
                                                            const double* __restrict__ gnorm,
                                                            int normalize,
                                                            uint16_t* __restrict__ img,
                                                            int ld_img,
                                                            unsigned int* __restrict__ err_max) {
  constexpr int SI_CH = 4;     // chunks per lane whose loads are in flight together
  const int cpr = ld_img / 8;  // 16-byte chunks per image row
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < n;
       row += waves) {
    const double s = normalize ? 1.0 / gnorm[row] : 1.0;
    double es = 0.0;   // err_max: sum of (image - x s)^2 over the lane's elements
    for (int c0 = lane; c0 < cpr; c0 += 64 * SI_CH) {
      if (VEC) {
        // all of the lane's full chunks loaded before any is converted (a loop that converts
        // each chunk as it arrives waits for every load in turn); a chunk past d (or past the
        // row) re-reads chunk 0 and is replaced below
        double v[SI_CH][8];
#pragma unroll
        for (int u = 0; u < SI_CH; ++u) {
          const int c = c0 + 64 * u;
          load8_f64<DT>(x, row * ld + (c * 8 + 8 <= d ? c * 8 : 0), v[u]);
        }
#pragma unroll
        for (int u = 0; u < SI_CH; ++u) {
          const int c = c0 + 64 * u;
          if (c >= cpr) continue;
          u16x8_t o;
          if (c * 8 + 8 <= d) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              o[e] = f64_to_img<IMG>(v[u][e] * s);
              if (err_max) es += sq_err<IMG>(o[e], v[u][e] * s);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int jj = c * 8 + e;
              const double w = jj < d ? load_as_f64<DT>(x, row * ld + jj) * s : 0.0;
              o[e] = f64_to_img<IMG>(w);
              if (err_max) es += sq_err<IMG>(o[e], w);
            }
          }
          *(u16x8_t*)(img + row * ld_img + c * 8) = o;
        }
      } else {
        for (int c = c0; c < cpr && c < c0 + 64 * SI_CH; c += 64) {
          u16x8_t o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int jj = c * 8 + e;
            const double w = jj < d ? load_as_f64<DT>(x, row * ld + jj) * s : 0.0;
            o[e] = f64_to_img<IMG>(w);
            if (err_max) es += sq_err<IMG>(o[e], w);
          }
          *(u16x8_t*)(img + row * ld_img + c * 8) = o;
        }
      }
    }
    if (err_max) {
      // the row's ||image - x s||_2, rounded up to a float; the largest over the rows by an
      // unsigned max on the bits (non-negative floats order as their bits). A row with
      // non-finite values is left out (its scores are not certified by any rounding bound)
      es = wave_sum_f64(es);
      if (lane == 0 && es <= 1.0) {
        const double e = sqrt(es);
        float f = (float)e;
        if ((double)f < e) f = nextafterf(f, 1.0f);
        atomicMax(err_max, __float_as_uint(f));
      }
    }
  }
}

int screen_image(const void* x, int dtype, int64_t n, int32_t d, int64_t ld,
                 const double* gnorm, int normalize, int img_dtype, void* img, int32_t ld_img,
                 hipStream_t st, unsigned int* err_max) {
  if (!x || !img || n < 0 || d <= 0 || ld < d || ld_img < d || ld_img % 64 != 0 ||
      (normalize && !gnorm) || (img_dtype != EBT_F16 && img_dtype != EBT_BF16) || dtype < 0 ||
      dtype > 3 || ((uintptr_t)img & 15)) {
    set_error("ebt_screen_image: bad arguments");
    return EBT_EINVAL;
  }
  if (n == 0) return EBT_OK;
  int64_t blocks = ceil_div(n, 4);  // one wave per row, 4 waves per block
  if (blocks > (1 << 20)) blocks = 1 << 20;
  dim3 grid((unsigned)blocks), block(256);
  const int es = dtype == EBT_F64 ? 8 : (dtype == EBT_F32 ? 4 : 2);
  const bool vec = ((uintptr_t)x & 15) == 0 && (ld * es) % 16 == 0;
#define EBT_SI_V(DT, IMG)                                                                      \
  if (vec)                                                                                     \
    hipLaunchKernelGGL((screen_image_kernel<DT, IMG, true>), grid, block, 0, st, x, n, d, ld,  \
                       gnorm, normalize, (uint16_t*)img, ld_img, err_max);                     \
  else                                                                                         \
    hipLaunchKernelGGL((screen_image_kernel<DT, IMG, false>), grid, block, 0, st, x, n, d, ld, \
                       gnorm, normalize, (uint16_t*)img, ld_img, err_max);
#define EBT_SI(DT)                                                                             \
  if (img_dtype == EBT_F16) {                                                                  \
    EBT_SI_V(DT, EBT_F16)                                                                      \
  } else {                                                                                     \
    EBT_SI_V(DT, EBT_BF16)                                                                     \
  }
  switch (dtype) {
    case EBT_F32: EBT_SI(EBT_F32) break;
    case EBT_BF16: EBT_SI(EBT_BF16) break;
    case EBT_F16: EBT_SI(EBT_F16) break;
    default: EBT_SI(EBT_F64) break;
  }
#undef EBT_SI
#undef EBT_SI_V
  return launch_check("screen_image_kernel");
}

// --------------------------------------------------------------------------- block sums ----
__device__ __forceinline__ double block_sum_f64(double v, double* red) {
  v = wave_sum_f64(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// ------------------------------------------------------------------------------ queries ----
template <int DT>
__global__ __launch_bounds__(256) void query_dense_kernel(const void* __restrict__ q, int d,
                                                           int64_t ldq, double* __restrict__ q64) {
  __shared__ double red[4];
  const int64_t b = blockIdx.x;
  double s = 0.0;
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    const double v = load_as_f64<DT>(q, b * ldq + j);
    s += v * v;
  }
  const double g = guard_norm(sqrt(block_sum_f64(s, red)));
  for (int j = threadIdx.x; j < d; j += blockDim.x)
    q64[b * d + j] = load_as_f64<DT>(q, b * ldq + j) / g;
}

int query_dense(const void* q, int dtype, int64_t B, int32_t d, int64_t ldq, double* q64,
                hipStream_t st) {
  if (!q || !q64 || B < 0 || d <= 0 || ldq < d || dtype < 0 || dtype > 3) {
    set_error("ebt_query_dense: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  dim3 grid((unsigned)B), block(256);
  switch (dtype) {
    case EBT_F32: hipLaunchKernelGGL(query_dense_kernel<EBT_F32>, grid, block, 0, st, q, d, ldq, q64); break;
    case EBT_BF16: hipLaunchKernelGGL(query_dense_kernel<EBT_BF16>, grid, block, 0, st, q, d, ldq, q64); break;
    case EBT_F16: hipLaunchKernelGGL(query_dense_kernel<EBT_F16>, grid, block, 0, st, q, d, ldq, q64); break;
    default: hipLaunchKernelGGL(query_dense_kernel<EBT_F64>, grid, block, 0, st, q, d, ldq, q64); break;
  }
  return launch_check("query_dense_kernel");
}

// n_local > 0: rows outside [row_offset, row_offset + n_local) are skipped (a row-sharded
// catalog: each shard sums its own liked rows; the caller adds the shards' partial sums)
template <int DT>
__global__ __launch_bounds__(256) void query_liked_kernel(const void* __restrict__ cat, int d,
                                                           int64_t ld,
                                                           const double* __restrict__ gnorm,
                                                           const int64_t* __restrict__ off,
                                                           const int64_t* __restrict__ rows,
                                                           int64_t row_offset, int64_t n_local,
                                                           double* __restrict__ q64) {
  const int64_t b = blockIdx.x;
  const int64_t l0 = off[b], l1 = off[b + 1];
  for (int j = threadIdx.x; j < d; j += blockDim.x) {
    double acc = 0.0;
    for (int64_t l = l0; l < l1; ++l) {
      const int64_t r = rows[l] - row_offset;
      if (n_local > 0 && (r < 0 || r >= n_local)) continue;
      acc += load_as_f64<DT>(cat, r * ld + j) / gnorm[r];
    }
    q64[b * d + j] = acc;
  }
}

// The same sums for 16-byte-aligned rows (ld * size and the base 16-byte aligned, d a multiple of
// the elements per 16 bytes): the query's rows and norms staged in LDS, each thread owning whole
// 16-byte chunks of the row, UL liked rows' chunks loaded before any is added (the loop above
// waits for every element load in turn). The per-element sum runs over the liked rows in the
// same order with the same operations: bit-identical to query_liked_kernel.
constexpr int QL_STAGE = 256;   // liked rows staged per round
constexpr int QL_UL = 8;        // liked rows in flight per chunk
template <int DT>
__global__ __launch_bounds__(256) void query_liked_vec_kernel(
    const void* __restrict__ cat, int d, int64_t ld, const double* __restrict__ gnorm,
    const int64_t* __restrict__ off, const int64_t* __restrict__ rows, int64_t row_offset,
    int64_t n_local, double* __restrict__ q64) {
  constexpr int ES = DT == EBT_F64 ? 8 : (DT == EBT_F32 ? 4 : 2);
  constexpr int PER = 16 / ES;   // elements per 16-byte chunk
  __shared__ int64_t srow[QL_STAGE];
  __shared__ double sg[QL_STAGE];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t l0 = off[b], l1 = off[b + 1];
  const int nch = d / PER;
  // a thread's chunks: c = tid, tid + 256, ... (at most QL_CPT of them: d <= 256 * PER * QL_CPT)
  constexpr int QL_CPT = 2;
  double acc[QL_CPT][PER];
#pragma unroll
  for (int i = 0; i < QL_CPT; ++i)
#pragma unroll
    for (int e = 0; e < PER; ++e) acc[i][e] = 0.0;
  for (int64_t s0 = l0; s0 < l1; s0 += QL_STAGE) {
    const int ns = l1 - s0 < QL_STAGE ? (int)(l1 - s0) : QL_STAGE;
    __syncthreads();
    if (tid < ns) {
      const int64_t r = rows[s0 + tid] - row_offset;
      const bool skip = n_local > 0 && (r < 0 || r >= n_local);   // another shard's row
      srow[tid] = skip ? -1 : r;
      sg[tid] = skip ? 1.0 : gnorm[r];
    }
    __syncthreads();
    for (int u0 = 0; u0 < ns; u0 += QL_UL) {
#pragma unroll
      for (int i = 0; i < QL_CPT; ++i) {
        const int c = tid + 256 * i;
        if (c >= nch) break;
        uint4 raw[QL_UL];
#pragma unroll
        for (int u = 0; u < QL_UL; ++u) {   // loads first (a skipped / past-the-end row reads row 0)
          const int64_t r = u0 + u < ns ? srow[u0 + u] : -1;
          raw[u] = *(const uint4*)((const char*)cat + ((r >= 0 ? r : 0) * ld + (int64_t)c * PER) * ES);
        }
#pragma unroll
        for (int u = 0; u < QL_UL; ++u) {
          if (u0 + u >= ns || srow[u0 + u] < 0) continue;
          const double g = sg[u0 + u];
#pragma unroll
          for (int e = 0; e < PER; ++e) {
            double x;
            if constexpr (DT == EBT_F32) x = (double)((const float*)&raw[u])[e];
            else if constexpr (DT == EBT_F64) x = ((const double*)&raw[u])[e];
            else if constexpr (DT == EBT_BF16) x = bf16_bits_to_f64(((const uint16_t*)&raw[u])[e]);
            else x = f16_bits_to_f64(((const uint16_t*)&raw[u])[e]);
            acc[i][e] += x / g;
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < QL_CPT; ++i) {
    const int c = tid + 256 * i;
    if (c >= nch) break;
#pragma unroll
    for (int e = 0; e < PER; ++e) q64[b * d + (int64_t)c * PER + e] = acc[i][e];
  }
}

// rows are catalog rows + row_offset (the self-contained path passes GLOBAL rows; the caller
// guarantees every row lies inside the catalog)
int query_liked_sum(const void* cat, int dtype, int32_t d, int64_t ld, const double* gnorm,
                    int64_t B, const int64_t* off, const int64_t* rows, double* q64,
                    hipStream_t st, int64_t row_offset, int64_t n_local) {
  if (!cat || !gnorm || !off || !q64 || B < 0 || d <= 0 || ld < d || dtype < 0 || dtype > 3) {
    set_error("ebt_query_liked_sum: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  dim3 grid((unsigned)B), block(256);
  const int es = dtype == EBT_F64 ? 8 : (dtype == EBT_F32 ? 4 : 2);
  const int per = 16 / es;
  if (((uintptr_t)cat & 15) == 0 && (ld * es) % 16 == 0 && d % per == 0 && d <= 256 * per * 2) {
#define EBT_QLV(DT)                                                                            \
  hipLaunchKernelGGL(query_liked_vec_kernel<DT>, grid, block, 0, st, cat, d, ld, gnorm, off,   \
                     rows, row_offset, n_local, q64)
    switch (dtype) {
      case EBT_F32: EBT_QLV(EBT_F32); break;
      case EBT_BF16: EBT_QLV(EBT_BF16); break;
      case EBT_F16: EBT_QLV(EBT_F16); break;
      default: EBT_QLV(EBT_F64); break;
    }
#undef EBT_QLV
    return launch_check("query_liked_vec_kernel");
  }
  switch (dtype) {
    case EBT_F32: hipLaunchKernelGGL(query_liked_kernel<EBT_F32>, grid, block, 0, st, cat, d, ld, gnorm, off, rows, row_offset, n_local, q64); break;
    case EBT_BF16: hipLaunchKernelGGL(query_liked_kernel<EBT_BF16>, grid, block, 0, st, cat, d, ld, gnorm, off, rows, row_offset, n_local, q64); break;
    case EBT_F16: hipLaunchKernelGGL(query_liked_kernel<EBT_F16>, grid, block, 0, st, cat, d, ld, gnorm, off, rows, row_offset, n_local, q64); break;
    default: hipLaunchKernelGGL(query_liked_kernel<EBT_F64>, grid, block, 0, st, cat, d, ld, gnorm, off, rows, row_offset, n_local, q64); break;
  }
  return launch_check("query_liked_kernel");
}

__global__ void scale_rows_kernel(double* q64, int64_t total, int d, const double* scale) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x)
    q64[t] *= scale[t / d];
}

int scale_rows_f64(double* q64, int64_t B, int32_t d, const double* scale, hipStream_t st) {
  if (!q64 || !scale || B < 0 || d <= 0) {
    set_error("ebt_scale_rows_f64: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  int64_t blocks = ceil_div(B * d, 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(scale_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, q64, B * d, d,
                     scale);
  return launch_check("scale_rows_kernel");
}

// ---------------------------------------------------------------------- query image/eps ----
// The certificate's bound on |approx score - exact float64 score| for one query and every
// catalog row: with q the float64 query (norm qnrm), dq = ||image(q) - q||_2
// measured here, and u_cat a bound on ||image(c) - c/|c|||_2 for every row (measured at catalog
// init, or the unit round-off 2^-11; 0 for a native image), image(q).image(c) - q.c/|c| =
// dq_vec.c + q.dc_vec + dq_vec.dc_vec is at most dq + qnrm u_cat + dq u_cat by Cauchy-Schwarz;
// the float32 accumulation of d products (and the epilogue's scales) adds (d+8) 2^-24 (qnrm+1).
__device__ __forceinline__ float query_eps(double qnrm, double dq, float u_cat, int d) {
  const double uc = (double)u_cat;
  return (float)(1.05 * (dq + qnrm * uc + dq * uc + (d + 8) * 0x1p-24 * (qnrm + 1.0)) + 1e-9);
}

template <int IMG>
__global__ __launch_bounds__(256) void query_image_kernel(
    const double* __restrict__ q64, int64_t B, int d, const uint16_t* __restrict__ qn,
    int64_t ldq, int native_q, float u_cat, uint16_t* __restrict__ qimg, int ld_img,
    float* __restrict__ qscale, float* __restrict__ eps) {
  __shared__ double red[4];
  const int64_t b = blockIdx.x;
  uint16_t* orow = qimg + b * ld_img;
  if (b >= B) {  // padding rows
    for (int j = threadIdx.x; j < ld_img; j += blockDim.x) orow[j] = 0;
    if (threadIdx.x == 0) {
      qscale[b] = 1.f;
      if (eps) eps[b] = 0.f;
    }
    return;
  }
  double s = 0.0, sn = 0.0;
  // eight of a thread's elements loaded before any is summed (same order of additions as one at
  // a time; a plain strided loop waits for each load in turn)
  for (int j0 = threadIdx.x; j0 < d; j0 += 8 * blockDim.x) {
    double v[8];
    uint16_t h[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * blockDim.x;
      const int jc = j < d ? j : d - 1;
      v[u] = q64[b * d + jc];
      h[u] = native_q ? qn[b * ldq + jc] : (uint16_t)0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (j0 + u * (int)blockDim.x >= d) break;
      s += v[u] * v[u];
      if (native_q) {
        const double w = IMG == EBT_F16 ? f16_bits_to_f64(h[u]) : bf16_bits_to_f64(h[u]);
        sn += w * w;
      }
    }
  }
  const double qnrm = sqrt(block_sum_f64(s, red));
  const double nrm_native = native_q ? sqrt(block_sum_f64(sn, red)) : 1.0;
  double se = 0.0;
  for (int j = threadIdx.x; j < ld_img; j += blockDim.x) {
    uint16_t o = 0;
    if (j < d) {
      o = native_q ? qn[b * ldq + j] : f64_to_img<IMG>(q64[b * d + j]);
      if (!native_q) se += sq_err<IMG>(o, q64[b * d + j]);
    }
    orow[j] = o;
  }
  const double dq = native_q ? 0.0 : sqrt(block_sum_f64(se, red));
  if (threadIdx.x == 0) {
    qscale[b] = native_q ? (float)(1.0 / guard_norm(nrm_native)) : 1.f;
    if (eps) eps[b] = query_eps(qnrm, dq, u_cat, d);
  }
}

int query_image(const double* q64, int64_t B, int64_t B_pad, int32_t d, int img_dtype,
                const void* q_native, int64_t ldq, int native_q, float u_cat, void* qimg,
                int32_t ld_img, float* qscale, float* eps, hipStream_t st) {
  if (!q64 || !qimg || !qscale || B < 0 || B_pad < B || d <= 0 || ld_img < d ||
      ld_img % 64 != 0 || (native_q && (!q_native || ldq < d)) ||
      (img_dtype != EBT_F16 && img_dtype != EBT_BF16)) {
    set_error("ebt_query_image: bad arguments");
    return EBT_EINVAL;
  }
  if (B_pad == 0) return EBT_OK;
  dim3 grid((unsigned)B_pad), block(256);
  if (img_dtype == EBT_F16)
    hipLaunchKernelGGL(query_image_kernel<EBT_F16>, grid, block, 0, st, q64, B, d,
                       (const uint16_t*)q_native, ldq, native_q, u_cat, (uint16_t*)qimg, ld_img,
                       qscale, eps);
  else
    hipLaunchKernelGGL(query_image_kernel<EBT_BF16>, grid, block, 0, st, q64, B, d,
                       (const uint16_t*)q_native, ldq, native_q, u_cat, (uint16_t*)qimg, ld_img,
                       qscale, eps);
  return launch_check("query_image_kernel");
}

// ------------------------------------------------------ dense queries in one pass ----------
// query_dense + query_image for dense queries with d <= 16 * 256: each thread keeps its elements
// (j = tid, tid + 256, ...: the same order, so the same float64 sums as the two kernels) in
// registers; the row is read once and q64, the image, qscale and eps are written in one launch.
constexpr int QP_PER = 16;
template <int DT, int IMG>
__global__ __launch_bounds__(256) void query_prep_kernel(
    const void* __restrict__ q, int64_t B, int d, int64_t ldq, int native_q, float u_cat,
    double* __restrict__ q64, uint16_t* __restrict__ qimg, int ld_img,
    float* __restrict__ qscale, float* __restrict__ eps) {
  __shared__ double red[4];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  uint16_t* orow = qimg + b * ld_img;
  if (b >= B) {  // padding rows
    for (int j = tid; j < ld_img; j += blockDim.x) orow[j] = 0;
    if (tid == 0) {
      qscale[b] = 1.f;
      eps[b] = 0.f;
    }
    return;
  }
  double v[QP_PER];
  double s = 0.0;
#pragma unroll
  for (int e = 0; e < QP_PER; ++e) {
    const int j = tid + e * 256;
    v[e] = j < d ? load_as_f64<DT>(q, b * ldq + j) : 0.0;
    s += v[e] * v[e];
  }
  const double nq = sqrt(block_sum_f64(s, red));
  const double g = guard_norm(nq);
  double s2 = 0.0, se = 0.0;
#pragma unroll
  for (int e = 0; e < QP_PER; ++e) {
    const int j = tid + e * 256;
    if (j < d) {
      const double x = v[e] / g;
      q64[b * d + j] = x;
      s2 += x * x;
      const uint16_t o = native_q ? ((const uint16_t*)q)[b * ldq + j] : f64_to_img<IMG>(x);
      if (!native_q) se += sq_err<IMG>(o, x);
      orow[j] = o;
    }
  }
  for (int j = d + tid; j < ld_img; j += blockDim.x) orow[j] = 0;
  const double qnrm = sqrt(block_sum_f64(s2, red));
  const double dq = native_q ? 0.0 : sqrt(block_sum_f64(se, red));
  if (tid == 0) {
    // native: the image holds q itself, scaled by 1 / ||q|| in the epilogue (query_image)
    qscale[b] = native_q ? (float)(1.0 / g) : 1.f;
    eps[b] = query_eps(qnrm, dq, u_cat, d);
  }
}

// The same for 16-byte-aligned rows with d % 8 == 0 and d <= 2048 (every BASELINE shape): one
// wave per query, lane l holding 8-element chunks l, l + 64, ... from 16-byte vector loads, the
// sums by wave shuffles (no block barriers), q64 and the image written in 64- and 16-byte
// pieces. Arithmetic per element as above (x = v / g, img = round(x)); the sums' order differs
// (within float64 round-off of the norms).
constexpr int QPW_CH = 4;   // chunks of 8 per lane: d <= 64 * 8 * 4
template <int DT, int IMG>
__global__ __launch_bounds__(256) void query_prep_wave_kernel(
    const void* __restrict__ q, int64_t B, int64_t B_pad, int d, int64_t ldq, int native_q,
    float u_cat, double* __restrict__ q64, uint16_t* __restrict__ qimg, int ld_img,
    float* __restrict__ qscale, float* __restrict__ eps) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B_pad) return;
  uint16_t* orow = qimg + b * ld_img;
  const int nch = d >> 3, cpr = ld_img >> 3;
  if (b >= B) {  // padding rows
    for (int c = lane; c < cpr; c += 64) *(u16x8_t*)(orow + c * 8) = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    if (lane == 0) {
      qscale[b] = 1.f;
      eps[b] = 0.f;
    }
    return;
  }
  // every chunk's raw 16-byte pieces loaded before any is used (a guarded load per chunk
  // would wait for each in turn); chunks past the row re-read its first chunk, then count 0
  constexpr int ES = DT == EBT_F64 ? 8 : (DT == EBT_F32 ? 4 : 2);
  constexpr int PC = ES / 2;   // 16-byte pieces per 8-element chunk
  uint4 raw[QPW_CH][PC];
#pragma unroll
  for (int i = 0; i < QPW_CH; ++i) {
    const int c = lane + 64 * i < nch ? lane + 64 * i : 0;
    const uint4* src = (const uint4*)((const char*)q + (b * ldq + (int64_t)c * 8) * ES);
#pragma unroll
    for (int p = 0; p < PC; ++p) raw[i][p] = src[p];
  }
  double v[QPW_CH][8];
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < QPW_CH; ++i) {
    const bool in = lane + 64 * i < nch;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      double x;
      if constexpr (DT == EBT_F32) x = (double)((const float*)raw[i])[e];
      else if constexpr (DT == EBT_F64) x = ((const double*)raw[i])[e];
      else if constexpr (DT == EBT_BF16) x = bf16_bits_to_f64(((const uint16_t*)raw[i])[e]);
      else x = f16_bits_to_f64(((const uint16_t*)raw[i])[e]);
      v[i][e] = in ? x : 0.0;
      s += v[i][e] * v[i][e];
    }
  }
  const double g = guard_norm(sqrt(wave_sum_f64(s)));
  double s2 = 0.0, se = 0.0;
#pragma unroll
  for (int i = 0; i < QPW_CH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      double x[8];
      u16x8_t o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        x[e] = v[i][e] / g;
        s2 += x[e] * x[e];
        o[e] = f64_to_img<IMG>(x[e]);
        if (!native_q) se += sq_err<IMG>(o[e], x[e]);
      }
      double2* dst = (double2*)(q64 + b * d + c * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = make_double2(x[2 * e], x[2 * e + 1]);
      if (native_q) o = *(const u16x8_t*)raw[i];   // native (DT == IMG): the query's own bits
      *(u16x8_t*)(orow + c * 8) = o;
    }
  }
  for (int c = nch + lane; c < cpr; c += 64) *(u16x8_t*)(orow + c * 8) = u16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
  const double qnrm = sqrt(wave_sum_f64(s2));
  const double dq = native_q ? 0.0 : sqrt(wave_sum_f64(se));
  if (lane == 0) {
    qscale[b] = native_q ? (float)(1.0 / g) : 1.f;
    eps[b] = query_eps(qnrm, dq, u_cat, d);
  }
}

int query_prep(const void* q, int dtype, int64_t B, int64_t B_pad, int32_t d, int64_t ldq,
               int img_dtype, int native_q, float u_cat, double* q64, void* qimg, int32_t ld_img,
               float* qscale, float* eps, hipStream_t st) {
  if (!q || !q64 || !qimg || !qscale || !eps || B < 0 || B_pad < B || d <= 0 ||
      d > QP_PER * 256 || ldq < d || ld_img < d || ld_img % 64 != 0 || dtype < 0 || dtype > 3 ||
      (img_dtype != EBT_F16 && img_dtype != EBT_BF16) ||
      (native_q && dtype != img_dtype)) {
    set_error("ebt_query_prep: bad arguments");
    return EBT_EINVAL;
  }
  if (B_pad == 0) return EBT_OK;
  const int es = dtype == EBT_F64 ? 8 : (dtype == EBT_F32 ? 4 : 2);
  const bool wave = d % 8 == 0 && d <= 64 * 8 * QPW_CH && ((uintptr_t)q & 15) == 0 &&
                    (ldq * es) % 16 == 0 && ((uintptr_t)q64 & 15) == 0 &&
                    ((uintptr_t)qimg & 15) == 0;
  dim3 grid(wave ? (unsigned)ceil_div(B_pad, 4) : (unsigned)B_pad), block(256);
#define EBT_QP(DT, IMG)                                                                        \
  if (wave)                                                                                    \
    hipLaunchKernelGGL((query_prep_wave_kernel<DT, IMG>), grid, block, 0, st, q, B, B_pad, d,  \
                       ldq, native_q, u_cat, q64, (uint16_t*)qimg, ld_img, qscale, eps);       \
  else                                                                                         \
    hipLaunchKernelGGL((query_prep_kernel<DT, IMG>), grid, block, 0, st, q, B, d, ldq,         \
                       native_q, u_cat, q64, (uint16_t*)qimg, ld_img, qscale, eps)
  const bool f16 = img_dtype == EBT_F16;
  switch (dtype) {
    case EBT_F32: if (f16) { EBT_QP(EBT_F32, EBT_F16); } else { EBT_QP(EBT_F32, EBT_BF16); } break;
    case EBT_BF16: if (f16) { EBT_QP(EBT_BF16, EBT_F16); } else { EBT_QP(EBT_BF16, EBT_BF16); } break;
    case EBT_F16: if (f16) { EBT_QP(EBT_F16, EBT_F16); } else { EBT_QP(EBT_F16, EBT_BF16); } break;
    default: if (f16) { EBT_QP(EBT_F64, EBT_F16); } else { EBT_QP(EBT_F64, EBT_BF16); } break;
  }
#undef EBT_QP
  return launch_check(wave ? "query_prep_wave_kernel" : "query_prep_kernel");
}

// ------------------------------------------------------------------------- exclusions ------
__global__ __launch_bounds__(256) void mask_excluded_kernel(float* __restrict__ s, int64_t ld,
                                                             int64_t c0, int64_t c1,
                                                             const int64_t* __restrict__ off,
                                                             const int64_t* __restrict__ rows) {
  const int64_t b = blockIdx.x;
  for (int64_t i = off[b] + threadIdx.x; i < off[b + 1]; i += blockDim.x) {
    const int64_t g = rows[i];
    if (g >= c0 && g < c1) s[b * ld + (g - c0)] = -__builtin_inff();
  }
}

int mask_excluded(float* s, int64_t ld, int64_t B, int64_t c0, int64_t c1, const int64_t* off,
                  const int64_t* rows, hipStream_t st) {
  if (!s || !off || B < 0 || c1 < c0 || ld < c1 - c0) {
    set_error("ebt_mask_excluded: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  hipLaunchKernelGGL(mask_excluded_kernel, dim3((unsigned)B), dim3(256), 0, st, s, ld, c0, c1,
                     off, rows);
  return launch_check("mask_excluded_kernel");
}

}  // namespace ebt
