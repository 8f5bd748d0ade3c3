// Screening GEMM on CDNA4 MFMA: scores[q][i] = qscale[q]*cscale[i]*sum_k Q[q][k]*C[i][k].
//
// Replaces the dgemm inside sklearn cosine_similarity (utils/extmath.py:203 via
// metrics/pairwise.py:1736, reached from lib.py:51) with an f16/bf16 MFMA GEMM whose result is
// only a SCREEN: the exact float64 scores are recomputed for the selected candidates
// (rescore.hip), and a rigorous error bound certifies the candidate set.
//
// Shape: "NT" GEMM -- both operands are row-major with k contiguous (catalog [N][d_pad],
// queries [B_pad][d_pad]), so both MFMA fragments are contiguous 16-byte LDS reads.
// Tile: 128 catalog rows x 128 queries x 64 k per stage, 256 threads = 4 waves (2 x 2), each
// wave 64 x 64 = 4 x 4 tiles of v_mfma_f32_16x16x32_{f16,bf16}. The catalog tile is the MFMA A
// operand so each lane ends up owning 4 CONSECUTIVE catalog rows of one query: the epilogue
// stores one float4 per accumulator into the query's score row.
// Staging: global_load_lds_dwordx4 (16 B/lane, 1 KiB per wave-instruction = 8 rows x 128 B)
// into a double-buffered 64 KiB LDS ring; the XOR swizzle slot = chunk ^ (row & 7) is applied to
// the per-lane SOURCE address (LDS-DMA writes lane-linearly), and the same XOR on the read side
// makes every ds_read_b128 lane group conflict-free.
// Block order: XCD-bijective remap (blocks sharing an XCD get a contiguous logical range), then
// groups of 8 catalog tiles walked query-tile-major, so a catalog tile is fetched from HBM once
// per XCD and re-read from L2 by the 32 query tiles that use it.
#include "common.h"

namespace ebt {

constexpr int GBM = 128;  // catalog rows per block
constexpr int GBN = 128;  // queries per block
constexpr int GBK = 64;   // k per LDS stage
constexpr int GTHREADS = 256;
constexpr int GTILE_BYTES = GBM * GBK * 2;       // 16 KiB per operand tile
constexpr int GSTAGE_BYTES = 2 * GTILE_BYTES;    // catalog + query
constexpr int GLDS_BYTES = 2 * GSTAGE_BYTES;     // double buffer: 64 KiB
constexpr int GGROUP_C = 8;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_cvoid;

// One wave stages 4 x 1 KiB pieces (32 rows x 128 B) of one operand tile.
__device__ __forceinline__ void stage_operand(const uint16_t* __restrict__ X, int64_t ldx,
                                              int64_t row0, int64_t last_row, int k0,
                                              char* tile_lds, int wave, int lane) {
  const int slot = lane & 7;
  const int sub = lane >> 3;  // row inside the 8-row piece (== row & 7)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int piece = wave * 4 + j;
    const int rr = piece * 8 + sub;
    int64_t grow = row0 + rr;
    grow = grow > last_row ? last_row : grow;  // clamp: rows past the end are never stored
    const int chunk = slot ^ sub;
    const uint16_t* src = X + grow * ldx + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvoid*)src, (lds_void*)(tile_lds + piece * 1024), 16,
                                     0, 0);
  }
}

template <bool BF16>
__device__ __forceinline__ f32x4_t mfma16(const u16x8_t& a, const u16x8_t& b, f32x4_t c) {
  if constexpr (BF16) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                   __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8_t, a),
                                                  __builtin_bit_cast(half8_t, b), c, 0, 0, 0);
  }
}

template <bool BF16>
__global__ __launch_bounds__(GTHREADS, 2) void screen_gemm_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ C, int64_t ld_img,
    int64_t n_rows, int n_qtiles, int64_t n_ctiles, int ksteps,
    const float* __restrict__ qscale, const float* __restrict__ cscale,
    float* __restrict__ S, int64_t ld_s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- block -> (catalog tile, query tile) ----
  const int64_t nwg = (int64_t)n_qtiles * n_ctiles;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int64_t L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int64_t per_group = (int64_t)GGROUP_C * n_qtiles;
  const int64_t g = L / per_group, w = L - g * per_group;
  const int64_t gc_rem = n_ctiles - g * GGROUP_C;
  const int64_t gc = gc_rem < GGROUP_C ? gc_rem : GGROUP_C;
  const int64_t ct = g * GGROUP_C + w % gc;
  const int64_t qt = w / gc;
  const int64_t c0 = ct * GBM;
  const int64_t q0 = qt * GBN;

  const int wi = wave >> 1;  // catalog half
  const int wj = wave & 1;   // query half

  f32x4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment offsets inside a tile (bytes), swizzled
  int a_off[4][2], b_off[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      const int ra = wi * 64 + t * 16 + (lane & 15);
      const int rb = wj * 64 + t * 16 + (lane & 15);
      a_off[t][kk] = ra * 128 + ((c ^ (ra & 7)) << 4);
      b_off[t][kk] = rb * 128 + ((c ^ (rb & 7)) << 4);
    }

  const int64_t last_c = n_rows - 1;
  const int64_t last_q = (int64_t)n_qtiles * GBN - 1;
  stage_operand(C, ld_img, c0, last_c, 0, smem, wave, lane);
  stage_operand(Q, ld_img, q0, last_q, 0, smem + GTILE_BYTES, wave, lane);

  for (int kt = 0; kt < ksteps; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < ksteps) {
      char* nb = smem + ((kt + 1) & 1) * GSTAGE_BYTES;
      stage_operand(C, ld_img, c0, last_c, (kt + 1) * GBK, nb, wave, lane);
      stage_operand(Q, ld_img, q0, last_q, (kt + 1) * GBK, nb + GTILE_BYTES, wave, lane);
    }
    const char* cb = smem + (kt & 1) * GSTAGE_BYTES;
    const char* qb = cb + GTILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u16x8_t af[4], bf[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        af[t] = *(const u16x8_t*)(cb + a_off[t][kk]);
        bf[t] = *(const u16x8_t*)(qb + b_off[t][kk]);
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma16<BF16>(af[a], bf[b], acc[a][b]);
    }
  }

  // ---- epilogue: lane owns catalog rows i0..i0+3 of query q for each (a, b) tile ----
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int64_t q = q0 + wj * 64 + b * 16 + (lane & 15);
    const float qs = qscale[q];
    float* srow = S + q * ld_s;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t i0 = c0 + wi * 64 + a * 16 + 4 * (lane >> 4);
      if (i0 + 3 < n_rows) {
        float4 cs = cscale ? *(const float4*)(cscale + i0) : make_float4(1.f, 1.f, 1.f, 1.f);
        float4 v;
        v.x = acc[a][b][0] * qs * cs.x;
        v.y = acc[a][b][1] * qs * cs.y;
        v.z = acc[a][b][2] * qs * cs.z;
        v.w = acc[a][b][3] * qs * cs.w;
        *(float4*)(srow + i0) = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (i0 + r < n_rows) {
            const float cs = cscale ? cscale[i0 + r] : 1.f;
            srow[i0 + r] = acc[a][b][r] * qs * cs;
          }
        }
      }
    }
  }
}

int screen_gemm(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows, int32_t d_pad,
                int32_t ld_img, int img_dtype, const float* qscale, const float* cscale,
                float* scores, int64_t ld_scores, hipStream_t stream) {
  if (!qimg || !cimg || !qscale || !scores) {
    set_error("ebt_screen_scores: null pointer");
    return EBT_EINVAL;
  }
  if (B_pad <= 0 || B_pad % GBN != 0 || n_rows <= 0 || d_pad <= 0 || d_pad % GBK != 0 ||
      ld_img < d_pad || ld_img % 64 != 0 || ld_scores < n_rows || ld_scores % 4 != 0 ||
      (img_dtype != EBT_F16 && img_dtype != EBT_BF16)) {
    set_error("ebt_screen_scores: bad shape (B_pad=%lld n=%lld d_pad=%d ld_img=%d ld_s=%lld)",
              (long long)B_pad, (long long)n_rows, d_pad, ld_img, (long long)ld_scores);
    return EBT_EINVAL;
  }
  if (cscale && ((uintptr_t)cscale & 15)) {
    set_error("ebt_screen_scores: cscale must be 16-byte aligned");
    return EBT_EINVAL;
  }
  const int n_qtiles = (int)(B_pad / GBN);
  const int64_t n_ctiles = ceil_div(n_rows, GBM);
  const int64_t nwg = n_ctiles * n_qtiles;
  if (nwg > 0x7fffffffLL) {
    set_error("ebt_screen_scores: grid too large");
    return EBT_EINVAL;
  }
  dim3 grid((unsigned)nwg), block(GTHREADS);
  if (img_dtype == EBT_BF16)
    hipLaunchKernelGGL(screen_gemm_kernel<true>, grid, block, GLDS_BYTES, stream,
                       (const uint16_t*)qimg, (const uint16_t*)cimg, (int64_t)ld_img, n_rows,
                       n_qtiles, n_ctiles, d_pad / GBK, qscale, cscale, scores, ld_scores);
  else
    hipLaunchKernelGGL(screen_gemm_kernel<false>, grid, block, GLDS_BYTES, stream,
                       (const uint16_t*)qimg, (const uint16_t*)cimg, (int64_t)ld_img, n_rows,
                       n_qtiles, n_ctiles, d_pad / GBK, qscale, cscale, scores, ld_scores);
  return launch_check("screen_gemm_kernel");
}

}  // namespace ebt
