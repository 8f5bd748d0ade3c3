// Implicit-feedback ALS: the offline factor training that produces
// the collaborative catalog robot-ebert serves (notebooks/create-embeddings.ipynb:1055,
// pyspark.ml ALS(rank=32, maxIter=15, regParam=0.1, implicitPrefs=True), alpha = 1).
//
// One half-iteration recomputes every destination factor (users from item factors, or items
// from user factors) from the source factors Y, Spark's computeFactors for implicit prefs:
//   A_u = Y^T Y + sum_{i in R(u)} c1_ui y_i y_i^T,   c1 = alpha |r_ui|
//   b_u = sum_{i in R(u), r_ui > 0} (1 + c1_ui) y_i
//   x_u = solve(A_u + reg * n_u I, b_u),              n_u = #{i in R(u): r_ui > 0}
// in float64 (Spark's NormalEquation holds doubles), factors stored as float32 (Spark's
// Array[Float]). Y^T Y is one small gram kernel; the solve is one workgroup per destination:
// the normal equation accumulates in LDS (rank <= 64), then one wave factors it (Cholesky) and
// substitutes. Integer/float work on a few KiB per destination: latency-bound, not MFMA work.
#include "common.h"

namespace ebt {

constexpr int ALS_THREADS = 256;
constexpr int ALS_RANK_MAX = 64;

// out[i][j] += sum over rows r in this block's range of Y[r][i] * Y[r][j] (float64)
__global__ __launch_bounds__(ALS_THREADS) void als_gram_kernel(const float* __restrict__ Y,
                                                               int64_t n, int rank,
                                                               int64_t rows_per_block,
                                                               double* __restrict__ out) {
  __shared__ float ys[64][ALS_RANK_MAX];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  const int pairs = rank * rank;
  double acc[ALS_RANK_MAX * ALS_RANK_MAX / ALS_THREADS];
  for (int p = 0; p < ALS_RANK_MAX * ALS_RANK_MAX / ALS_THREADS; ++p) acc[p] = 0.0;
  for (int64_t c0 = r0; c0 < r1; c0 += 64) {
    const int nr = (int)((r1 - c0) < 64 ? (r1 - c0) : 64);
    for (int e = tid; e < 64 * rank; e += ALS_THREADS) {
      const int rr = e / rank, cc = e - rr * rank;
      ys[rr][cc] = rr < nr ? Y[(c0 + rr) * rank + cc] : 0.f;
    }
    __syncthreads();
    for (int p = 0; p * ALS_THREADS + tid < pairs; ++p) {
      const int q = p * ALS_THREADS + tid, i = q / rank, j = q - i * rank;
      double s = 0.0;
      for (int rr = 0; rr < nr; ++rr) s += (double)ys[rr][i] * (double)ys[rr][j];
      acc[p] += s;
    }
    __syncthreads();
  }
  for (int p = 0; p * ALS_THREADS + tid < pairs; ++p) {
    const int q = p * ALS_THREADS + tid;
    atomicAdd(out + q, acc[p]);
  }
}

// One destination per workgroup: A = YtY + sum c1 y y^T (+ reg n I), b = sum (1 + c1) y over
// the positive ratings, x = A^-1 b by Cholesky (one wave), stored as float32. Thread t owns the
// BS x BS block (t / 16, t % 16) of A (padded to 16 BS columns) in REGISTERS for the whole
// rating loop: per rating 2 BS factor reads from LDS for BS^2 float64 FMAs (an LDS-resident A
// needed 2 reads and a read-modify-write per entry: 64 GB/s of ratings at ml-25m).
constexpr int ALS_ROUND = 16;  // ratings staged per round
template <int BS>
__global__ __launch_bounds__(ALS_THREADS) void als_solve_kernel(
    const double* __restrict__ YtY, const float* __restrict__ Y, int rank,
    const int64_t* __restrict__ off, const int32_t* __restrict__ src,
    const float* __restrict__ rating, float alpha, float reg, float* __restrict__ X) {
  constexpr int RP = 16 * BS;  // padded rank
  __shared__ double A[ALS_RANK_MAX * ALS_RANK_MAX];
  __shared__ double b[ALS_RANK_MAX];
  __shared__ float yb[ALS_ROUND][RP];
  __shared__ float cb[ALS_ROUND], pb[ALS_ROUND];
  __shared__ int npos_s;
  const int tid = threadIdx.x;
  const int64_t u = blockIdx.x;
  const int i0 = (tid >> 4) * BS, j0 = (tid & 15) * BS;
  double a[BS][BS];
#pragma unroll
  for (int x = 0; x < BS; ++x)
#pragma unroll
    for (int y = 0; y < BS; ++y)
      a[x][y] = (i0 + x < rank && j0 + y < rank) ? YtY[(i0 + x) * rank + j0 + y] : 0.0;
  double bl = 0.0;  // b[tid] for tid < rank
  const int64_t e0 = off[u], e1 = off[u + 1];
  int npos = 0;     // thread 0's count of positive ratings
  for (int64_t c0 = e0; c0 < e1; c0 += ALS_ROUND) {
    const int nr = (int)((e1 - c0) < ALS_ROUND ? (e1 - c0) : ALS_ROUND);
    for (int e = tid; e < ALS_ROUND * RP; e += ALS_THREADS) {
      const int rr = e / RP, cc = e - rr * RP;
      yb[rr][cc] = (rr < nr && cc < rank) ? Y[(int64_t)src[c0 + rr] * rank + cc] : 0.f;
    }
    if (tid < ALS_ROUND) {
      const float r = tid < nr ? rating[c0 + tid] : 0.f;
      cb[tid] = alpha * fabsf(r);                        // c1
      pb[tid] = r > 0.f ? 1.f + alpha * fabsf(r) : 0.f;  // weight of y in b
    }
    if (tid == 0)
      for (int rr = 0; rr < nr; ++rr) npos += rating[c0 + rr] > 0.f ? 1 : 0;
    __syncthreads();
    for (int rr = 0; rr < nr; ++rr) {
      const double c = (double)cb[rr];
      double yi[BS], yj[BS];
#pragma unroll
      for (int x = 0; x < BS; ++x) {
        yi[x] = (double)yb[rr][i0 + x];
        yj[x] = (double)yb[rr][j0 + x];
      }
#pragma unroll
      for (int x = 0; x < BS; ++x)
#pragma unroll
        for (int y = 0; y < BS; ++y) a[x][y] += c * yi[x] * yj[y];
      if (tid < rank) bl += (double)pb[rr] * (double)yb[rr][tid];
    }
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < BS; ++x)
#pragma unroll
    for (int y = 0; y < BS; ++y)
      if (i0 + x < rank && j0 + y < rank) A[(i0 + x) * rank + j0 + y] = a[x][y];
  if (tid < rank) b[tid] = bl;
  if (tid == 0) npos_s = npos;
  __syncthreads();
  if (tid < rank) A[tid * rank + tid] += (double)reg * (double)npos_s;
  __syncthreads();
  // Cholesky A = L L^T (lower, in place) and two triangular solves, by the first wave
  if (tid < 64) {
    const int lane = tid;
    for (int k = 0; k < rank; ++k) {
      if (lane == 0) {
        double d = A[k * rank + k];
        A[k * rank + k] = d > 0.0 ? sqrt(d) : 0.0;
      }
      // one wave: its LDS accesses complete in program order; the fences keep the compiler
      // from reordering them (no s_barrier: the other waves are not here)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      const double lkk = A[k * rank + k];
      if (lane > k && lane < rank) A[lane * rank + k] = lkk > 0.0 ? A[lane * rank + k] / lkk : 0.0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      // trailing update of the lower triangle, column by column: lane = row i
      if (lane > k && lane < rank) {
        const double lik = A[lane * rank + k];
        for (int j = k + 1; j <= lane; ++j) A[lane * rank + j] -= lik * A[j * rank + k];
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    // forward: L z = b (lane 0 serial; rank <= 64 steps of a dot product over lanes)
    for (int i = 0; i < rank; ++i) {
      double s = lane < i ? A[i * rank + lane] * b[lane] : 0.0;
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0) b[i] = A[i * rank + i] > 0.0 ? (b[i] - s) / A[i * rank + i] : 0.0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    // backward: L^T x = z
    for (int i = rank - 1; i >= 0; --i) {
      double s = (lane > i && lane < rank) ? A[lane * rank + i] * b[lane] : 0.0;
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0) b[i] = A[i * rank + i] > 0.0 ? (b[i] - s) / A[i * rank + i] : 0.0;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
    if (lane < rank) X[u * rank + lane] = (float)b[lane];
  }
}

}  // namespace ebt

using namespace ebt;

extern "C" {

int ebt_als_gram(const float* Y, int64_t n, int32_t rank, double* out, void* stream) {
  if (!Y || !out || n < 0 || rank < 1 || rank > ALS_RANK_MAX) {
    set_error("ebt_als_gram: bad arguments (n=%lld rank=%d)", (long long)n, rank);
    return EBT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  int rc = hip_check(hipMemsetAsync(out, 0, sizeof(double) * rank * rank, st), "hipMemsetAsync");
  if (rc || n == 0) return rc;
  const int64_t per = 4096;
  const int64_t blocks = ceil_div(n, per);
  hipLaunchKernelGGL(als_gram_kernel, dim3((unsigned)blocks), dim3(ALS_THREADS), 0, st, Y, n,
                     (int)rank, per, out);
  return launch_check("als_gram_kernel");
}

int ebt_als_solve(const double* YtY, const float* Y, int32_t rank, int64_t n_dst,
                  const int64_t* off, const int32_t* src, const float* rating, float alpha,
                  float reg, float* X, void* stream) {
  if (!YtY || !Y || !off || !X || (!src != !rating) || n_dst < 0 || rank < 1 ||
      rank > ALS_RANK_MAX || n_dst > 0x7fffffffLL) {
    set_error("ebt_als_solve: bad arguments (n_dst=%lld rank=%d)", (long long)n_dst, rank);
    return EBT_EINVAL;
  }
  if (n_dst == 0) return EBT_OK;
  if (rank <= 32)
    hipLaunchKernelGGL(als_solve_kernel<2>, dim3((unsigned)n_dst), dim3(ALS_THREADS), 0,
                       (hipStream_t)stream, YtY, Y, (int)rank, off, src, rating, alpha, reg, X);
  else
    hipLaunchKernelGGL(als_solve_kernel<4>, dim3((unsigned)n_dst), dim3(ALS_THREADS), 0,
                       (hipStream_t)stream, YtY, Y, (int)rank, off, src, rating, alpha, reg, X);
  return launch_check("als_solve_kernel");
}

}  // extern "C"
