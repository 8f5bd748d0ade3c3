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
hipEvent_t event_get(hipStream_t st);
void event_put(hipEvent_t e, hipStream_t st);
std::mutex& event_pool_mutex();
std::vector<hipEvent_t>* event_pool();
// A timed stage that is ONE kernel launch (api.hip KernelStage): the launch site takes the
// stage's event pair and passes it to hipExtLaunchKernelGGL, which binds the events to the
// dispatch itself instead of two marker packets around it (take: returns false when none).
bool take_launch_events(hipEvent_t* start, hipEvent_t* stop);

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
// The xor butterfly v += v(lane ^ o), o = 32, 16, 8, 4, 2, 1, through ds_bpermute (LDS pipe,
// two per level for a double, each waited for). Kept as the reference form of the tree.
__device__ __forceinline__ double wave_sum_f64_shfl(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ double f64_from_halves(uint32_t lo, uint32_t hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return f64_from_halves(lo, hi);
}
// v(lane ^ 32) / v(lane ^ 16) by the gfx950 half-exchanges of a register with itself
__device__ __forceinline__ double xor32_f64(double v, int lane) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const auto a = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  return lane < 32 ? f64_from_halves(a[1], b[1]) : f64_from_halves(a[0], b[0]);
}
__device__ __forceinline__ double xor16_f64(double v, int lane) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const auto a = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  return (lane & 16) ? f64_from_halves(a[0], b[0]) : f64_from_halves(a[1], b[1]);
}

// One butterfly level of two independent values at once: lanes < 32 (lanes in even 16-lane
// rows) get x + x(lane ^ 32) (^ 16), the others y + y(lane ^ 32) (^ 16) -- each lane the value
// its own row's butterfly has there, from one half-exchange per dword.
__device__ __forceinline__ double pair_sum32_f64(double x, double y) {
  const uint64_t ux = (uint64_t)__double_as_longlong(x), uy = (uint64_t)__double_as_longlong(y);
  const auto a = __builtin_amdgcn_permlane32_swap((uint32_t)ux, (uint32_t)uy, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap((uint32_t)(ux >> 32), (uint32_t)(uy >> 32), false, false);
  return f64_from_halves(a[0], b[0]) + f64_from_halves(a[1], b[1]);
}
__device__ __forceinline__ double pair_sum16_f64(double x, double y) {
  const uint64_t ux = (uint64_t)__double_as_longlong(x), uy = (uint64_t)__double_as_longlong(y);
  const auto a = __builtin_amdgcn_permlane16_swap((uint32_t)ux, (uint32_t)uy, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap((uint32_t)(ux >> 32), (uint32_t)(uy >> 32), false, false);
  return f64_from_halves(a[0], b[0]) + f64_from_halves(a[1], b[1]);
}

// The SAME butterfly (bitwise equal to wave_sum_f64_shfl: every level adds the value of lane ^ o)
// in VALU cross-lane moves, no LDS traffic: levels 32 and 16 by permlane32/16_swap, 8 by DPP
// row_ror:8 (= xor 8 inside a 16-lane row), 4 by row_ror:4 (after levels 32..8 the value
// depends on lane mod 8 only, and lane +- 4 mod 8 = lane ^ 4 mod 8), 2 and 1 by quad_perm.
// Every lane of the wave must be active (as for the shuffles it replaces).
__device__ __forceinline__ double wave_sum_f64(double v) {
  const int lane = (int)(threadIdx.x & (kWave - 1));
  v += xor32_f64(v, lane);
  v += xor16_f64(v, lane);
  v += dpp_f64<0x128>(v);  // row_ror:8
  v += dpp_f64<0x124>(v);  // row_ror:4
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  return v;
}

// The butterflies of NR (1, 2, 4 or 8) values at once, each bitwise equal to its own
// wave_sum_f64: the first log2(NR) levels pair values up (pair_sum32 / pair_sum16 / DPP), so that
// from then on each lane carries one value through the remaining levels. Returns, in every lane,
// the total of value (lane >> 5) (NR = 2), (lane >> 4) (NR = 4) or (lane >> 3) (NR = 8):
// wave_rows_owner<NR>(lane).
template <int NR>
__device__ __forceinline__ double wave_sum_f64_rows(const double (&s)[NR]) {
  static_assert(NR == 1 || NR == 2 || NR == 4 || NR == 8, "NR");
  const int lane = (int)(threadIdx.x & (kWave - 1));
  double v;
  if constexpr (NR == 1) {
    return wave_sum_f64(s[0]);
  } else if constexpr (NR == 2) {
    v = pair_sum32_f64(s[0], s[1]);  // lanes < 32: value 0, lanes >= 32: value 1
    v += xor16_f64(v, lane);
    v += dpp_f64<0x128>(v);
  } else if constexpr (NR == 4) {
    const double t0 = pair_sum32_f64(s[0], s[2]);  // lanes < 32: 0, >= 32: 2
    const double t1 = pair_sum32_f64(s[1], s[3]);  // lanes < 32: 1, >= 32: 3
    v = pair_sum16_f64(t0, t1);                    // 16-lane rows: 0, 1, 2, 3
    v += dpp_f64<0x128>(v);
  } else {
    // levels 32 and 16 pair the eight values into two per lane (u0: values 0, 2, 4, 6 by
    // 16-lane row; u1: 1, 3, 5, 7), level 8 (row_ror:8 = xor 8) keeps u0 in the lanes with
    // bit 3 clear and u1 in the others: lane l then carries value l >> 3
    const double t0 = pair_sum32_f64(s[0], s[4]);
    const double t1 = pair_sum32_f64(s[1], s[5]);
    const double t2 = pair_sum32_f64(s[2], s[6]);
    const double t3 = pair_sum32_f64(s[3], s[7]);
    const double u0 = pair_sum16_f64(t0, t2);
    const double u1 = pair_sum16_f64(t1, t3);
    const double a = dpp_f64<0x128>(u0), b = dpp_f64<0x128>(u1);
    v = (lane & 8) ? u1 + b : u0 + a;
    // level 4 inside each 8-lane group (its neighbours hold other values, so row_ror:4 would
    // cross into them): lane ^ 4 as row_shl:4 for lanes with bit 2 clear, row_shr:4 otherwise
    const double up = dpp_f64<0x104>(v), dn = dpp_f64<0x114>(v);
    v += (lane & 4) ? dn : up;
    v += dpp_f64<0x4E>(v);
    v += dpp_f64<0xB1>(v);
    return v;
  }
  v += dpp_f64<0x124>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0xB1>(v);
  return v;
}
template <int NR>
__device__ __forceinline__ int wave_rows_owner(int lane) {
  return NR == 1 ? 0 : (NR == 2 ? lane >> 5 : (NR == 4 ? lane >> 4 : lane >> 3));
}

// Inclusive wave scans of a 32-bit value in DPP moves (no LDS): Hillis-Steele steps row_shr 1, 2,
// 4, 8 inside each 16-lane row, then row_bcast:15 (rows 1, 3 take lane 15 of the row before) and
// row_bcast:31 (rows 2, 3 take lane 31). Lanes a move has no source for read 0, the identity of
// both ops. Every lane of the wave must be active.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32_or0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_scan_add_u32(uint32_t v) {
  v += dpp_u32_or0<0x111, 0xF>(v);
  v += dpp_u32_or0<0x112, 0xF>(v);
  v += dpp_u32_or0<0x114, 0xF>(v);
  v += dpp_u32_or0<0x118, 0xF>(v);
  v += dpp_u32_or0<0x142, 0xA>(v);
  v += dpp_u32_or0<0x143, 0xC>(v);
  return v;
}
__device__ __forceinline__ uint32_t wave_scan_max_u32(uint32_t v) {
  v = max(v, dpp_u32_or0<0x111, 0xF>(v));
  v = max(v, dpp_u32_or0<0x112, 0xF>(v));
  v = max(v, dpp_u32_or0<0x114, 0xF>(v));
  v = max(v, dpp_u32_or0<0x118, 0xF>(v));
  v = max(v, dpp_u32_or0<0x142, 0xA>(v));
  v = max(v, dpp_u32_or0<0x143, 0xC>(v));
  return v;
}
// wave-wide max / min (uniform): the scan's last lane
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_max_u32(v), 63);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return ~wave_max_u32(~v); }

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Guarded norm: sklearn _handle_zeros_in_scale (preprocessing/_data.py:118-123).
__device__ __forceinline__ double guard_norm(double nrm) {
  return nrm < 10.0 * 2.220446049250313e-16 ? 1.0 : nrm;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ebt_shard_pack's buffer (0.3.2): u32 start[B], u32 len[B] (query b's entries are
// [start[b], start[b] + len[b]) -- in any order of b: the sharded rescore reserves each query's
// range by an atomic), u32 block totals[ceil(B / SHARD_PACK_QPB)] (scratch of the two-launch
// pack, sent along), 16-byte aligned; then f64 scores[cap]; then i32 rows[cap]
constexpr int SHARD_PACK_QPB = 64;  // queries per pack workgroup (one wave counts them)
__host__ __device__ inline int64_t shard_pack_hdr_bytes(int64_t B) {
  return ((2 * B + (B + SHARD_PACK_QPB - 1) / SHARD_PACK_QPB) * 4 + 15) & ~(int64_t)15;
}

// The sharded rescore's share of the pack (rescore_sharded): each query's workgroup counts its
// entries >= t_floor from the exact scores it holds in LDS and writes len[b] into the send
// buffer's header; one launch (shard_pack_lens) then places and copies them -- ebt_shard_pack's
// counting launch folded into the rescore
struct ShardPackOut {
  uint32_t* len;       // NULL: no count
};

}  // namespace ebt
