// Shared device helpers for libebert (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "../../include/ebert.h"

namespace ebt {

constexpr int kWave = 64;  // CDNA wavefront

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8_t __attribute__((ext_vector_type(8)));

// ---- error reporting (thread-local, set by the host wrappers) -------------------------------
void set_error(const char* fmt, ...);
int hip_check(hipError_t e, const char* what);
int launch_check(const char* what);
void set_max_lds(const void* fn, int bytes);
hipEvent_t event_get();
void event_put(hipEvent_t e);
std::mutex& event_pool_mutex();
std::vector<hipEvent_t>* event_pool();

// ---- element conversion --------------------------------------------------------------------
__device__ __forceinline__ double bf16_bits_to_f64(uint16_t h) {
  return (double)__uint_as_float(((uint32_t)h) << 16);
}
__device__ __forceinline__ double f16_bits_to_f64(uint16_t h) {
  _Float16 v = __builtin_bit_cast(_Float16, h);
  return (double)v;
}

template <int DT>
__device__ __forceinline__ double load_as_f64(const void* p, int64_t i) {
  if constexpr (DT == EBT_F32) return (double)((const float*)p)[i];
  else if constexpr (DT == EBT_F64) return ((const double*)p)[i];
  else if constexpr (DT == EBT_BF16) return bf16_bits_to_f64(((const uint16_t*)p)[i]);
  else return f16_bits_to_f64(((const uint16_t*)p)[i]);
}

// Round a double to the 16-bit image type (round-to-nearest-even through float; the extra
// float rounding is covered by the 1.05 factor of the eps bound).
template <int IMG>
__device__ __forceinline__ uint16_t f64_to_img(double v) {
  float f = (float)v;
  if constexpr (IMG == EBT_F16) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(uint16_t, h);
  } else {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
  }
}

// ---- order-preserving float keys (0 = invalid: NaN or -inf) ---------------------------------
__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  if (!(f == f) || f == -__builtin_inff()) return 0u;
  if (f == 0.f) return 0x80000000u;  // -0 and +0 are one value (they compare equal)
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  if (k == 0u) return -__builtin_inff();
  uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(u);
}

// Workgroup barrier for LDS traffic only. __syncthreads() also waits for the wave's outstanding
// GLOBAL loads (its release fence is s_waitcnt vmcnt(0)), which empties a register prefetch
// pipeline at every barrier; LDS ops complete in order, so lgkmcnt(0) + s_barrier suffices when
// the barrier protects LDS only.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- wave reductions -----------------------------------------------------------------------
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Guarded norm: sklearn _handle_zeros_in_scale (preprocessing/_data.py:118-123).
__device__ __forceinline__ double guard_norm(double nrm) {
  return nrm < 10.0 * 2.220446049250313e-16 ? 1.0 : nrm;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ebt_shard_pack's buffer: u32 starts[B + 1], u32 block totals[ceil(B / 256)] (scratch of the
// pack, sent along), 16-byte aligned; then f64 scores[cap]; then i32 rows[cap]
constexpr int SHARD_PACK_QPB = 256;  // queries per pack workgroup
__host__ __device__ inline int64_t shard_pack_hdr_bytes(int64_t B) {
  return ((B + 1 + (B + SHARD_PACK_QPB - 1) / SHARD_PACK_QPB) * 4 + 15) & ~(int64_t)15;
}

}  // namespace ebt
