// Screening GEMM on CDNA4 MFMA: scores[q][i] = qscale[q]*cscale[i]*sum_k Q[q][k]*C[i][k].
//
// Replaces the dgemm inside sklearn cosine_similarity (utils/extmath.py:203 via
// metrics/pairwise.py:1736, reached from lib.py:51) with an f16/bf16 MFMA GEMM whose result is
// only a SCREEN: the exact float64 scores are recomputed for the selected candidates
// (rescore.hip), and a rigorous error bound certifies the candidate set.
//
// Shape: "NT" GEMM -- both operands are row-major with k contiguous (catalog [N][d_pad],
// queries [B_pad][d_pad]), so both MFMA fragments are contiguous 16-byte LDS reads.
// Two kernels: the 256 x 256 "quadrant phase" kernel for batches padded to 256 (below), and a
// 128 x 128 one (128 catalog rows x 128 queries x 64 k per stage, 4 waves of 64 x 64) for
// B_pad = 128. Both use v_mfma_f32_16x16x32_{f16,bf16} with the catalog tile as the MFMA A
// operand, so each lane ends up owning 4 CONSECUTIVE catalog rows of one query: the epilogue
// stores one float4 per accumulator into the query's score row (or, in the fused screen, appends
// the values >= the query's threshold to its candidate list).
// Staging: global_load_lds_dwordx4 (16 B/lane, 1 KiB per wave-instruction = 8 rows x 128 B)
// into a double-buffered 64 KiB LDS ring; the XOR swizzle slot = chunk ^ (row & 7) is applied to
// the per-lane SOURCE address (LDS-DMA writes lane-linearly), and the same XOR on the read side
// makes every ds_read_b128 lane group conflict-free.
// Block order: XCD-bijective remap (blocks sharing an XCD get a contiguous logical range), then
// groups of 8 (128-kernel) / 4 (256-kernel) catalog tiles walked query-tile-major, so a catalog
// tile is fetched from HBM about once per XCD and re-read from L2 by the query tiles that use it.
#include <cstdlib>
#include <type_traits>

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

// Epilogue destinations. Store mode: the float32 score matrix S[q][i]. Filter mode (the fused
// screen): only scores >= thr[q] leave the kernel, appended to the query's candidate list
// (cand_v / cand_i [q*ld_cand + cand_off + slot], slot from an atomic counter cnt[q]; slots past
// `cap` are dropped and counted, so cnt[q] > cap flags an overflow). thr[q] is a lower bound of
// the query's k'-th best approx score, so no candidate of the true top-k' is ever filtered.
// Filter-mode output (the fused screen): catalog rows are grouped by the kernel's tile
// (FILTER_GROUP rows: 256 for the quadrant-phase kernel, 128 for the small-batch one); for query
// q and group g, up to `slots` hits go to cand[q*ld_cand + g*slots + p] as u64
// composites (f2key(score) << 32 | ~row, row = idx_base + local row) and the group's hit count to
// counts[q*ld_counts + g] (saturated at 255; > slots sets ovf[q]). Slots are claimed with LDS
// atomics per workgroup tile, so the epilogue does no global atomics and no dependent loads.

struct EpiArgs {
  float* S;  // store mode
  int64_t ld_s;
  const float* thr;  // filter mode
  uint64_t* cand;
  int64_t ld_cand;
  uint8_t* counts;
  int64_t ld_counts;
  int* ovf;
  int64_t idx_base;
  int slots;
};

// The row scales of catalog rows i0 .. i0+3 (1 past the end / without scales).
__device__ __forceinline__ float4 row_scales4(const float* __restrict__ cscale, int64_t i0,
                                              int64_t n_rows) {
  float4 cs = make_float4(1.f, 1.f, 1.f, 1.f);
  if (cscale) {
    if (i0 + 3 < n_rows) {
      cs = *(const float4*)(cscale + i0);
    } else {
      cs.x = i0 + 0 < n_rows ? cscale[i0 + 0] : 1.f;
      cs.y = i0 + 1 < n_rows ? cscale[i0 + 1] : 1.f;
      cs.z = i0 + 2 < n_rows ? cscale[i0 + 2] : 1.f;
      cs.w = i0 + 3 < n_rows ? cscale[i0 + 3] : 1.f;
    }
  }
  return cs;
}

// The filter's cold path: append the values >= th of rows i0 .. i0+3 (row < n_rows) to the
// (query, group) slots.
__device__ __forceinline__ void filter_hits(const EpiArgs& e, int64_t q, int64_t i0,
                                            int64_t n_rows, const float (&v)[4], float th,
                                            uint32_t* lcnt, int64_t grp) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t i = i0 + r;
    if (i < n_rows && v[r] >= th) {
      const uint32_t p = atomicAdd(lcnt, 1u);
      if (p < (uint32_t)e.slots) {
        const uint32_t row = (uint32_t)(e.idx_base + i);
        e.cand[q * e.ld_cand + grp * e.slots + p] =
            ((uint64_t)f2key(v[r]) << 32) | (uint64_t)(~row);
      }
    }
  }
}

// One accumulator (4 consecutive catalog rows i0.. of query q) with its scales in hand.
template <bool FILTER>
__device__ __forceinline__ void epilogue4v(const EpiArgs& e, int64_t q, int64_t i0,
                                           int64_t n_rows, const f32x4_t& acc, float qs,
                                           float th, float4 cs, uint32_t* lcnt, int64_t grp) {
  const float v[4] = {acc[0] * qs * cs.x, acc[1] * qs * cs.y, acc[2] * qs * cs.z,
                      acc[3] * qs * cs.w};
  if constexpr (!FILTER) {
    float* srow = e.S + q * e.ld_s;
    if (i0 + 3 < n_rows) {
      *(float4*)(srow + i0) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (i0 + r < n_rows) srow[i0 + r] = v[r];
    }
  } else {
    // a cheap all-miss test first: the append path is taken for ~k'/rows-so-far of the values;
    // keeping it cold keeps the accumulators in registers
    const bool any = (v[0] >= th && i0 < n_rows) || (v[1] >= th && i0 + 1 < n_rows) ||
                     (v[2] >= th && i0 + 2 < n_rows) || (v[3] >= th && i0 + 3 < n_rows);
    if (__builtin_expect(any, 0)) filter_hits(e, q, i0, n_rows, v, th, lcnt, grp);
  }
}

template <bool FILTER>
__device__ __forceinline__ void epilogue4(const EpiArgs& e, int64_t q, int64_t i0,
                                          int64_t n_rows, const f32x4_t& acc, float qs,
                                          float th, const float* __restrict__ cscale,
                                          uint32_t* lcnt, int64_t grp) {
  epilogue4v<FILTER>(e, q, i0, n_rows, acc, qs, th, row_scales4(cscale, i0, n_rows), lcnt, grp);
}

// End of a filter-mode tile: publish the per-query hit counts of group `grp` (LDS counters of
// queries q0 .. q0 + nq - 1), after every wave's epilogue.
__device__ __forceinline__ void filter_finish(const EpiArgs& e, const uint32_t* lcnt, int64_t q0,
                                              int nq, int64_t grp) {
  // LDS-only barrier: the counters are LDS atomics, the hits are read by a later kernel, so
  // the waves need not wait for their hit stores here (__syncthreads() adds vmcnt(0); measured
  // no difference either way on MI355X -- the hit path's cost is its instructions)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int t = threadIdx.x; t < nq; t += blockDim.x) {
    const uint32_t c = lcnt[t];
    const int64_t q = q0 + t;
    e.counts[q * e.ld_counts + grp] = (uint8_t)(c < 255u ? c : 255u);
    if (c > (uint32_t)e.slots) e.ovf[q] = 1;
  }
}

template <bool BF16, bool FILTER>
__global__ __launch_bounds__(GTHREADS, 2) void screen_gemm_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ C, int64_t ld_img,
    int64_t n_rows, int n_qtiles, int64_t n_ctiles, int ksteps,
    const float* __restrict__ qscale, const float* __restrict__ cscale, EpiArgs e) {
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
  uint32_t* lcnt = (uint32_t*)(smem + GLDS_BYTES);  // filter mode: hits per query of the tile
  if constexpr (FILTER) {
    if (tid < GBN) lcnt[tid] = 0u;
  }

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
    const float th = FILTER ? e.thr[q] : 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int64_t i0 = c0 + wi * 64 + a * 16 + 4 * (lane >> 4);
      epilogue4<FILTER>(e, q, i0, n_rows, acc[a][b], qs, th, cscale, lcnt + (q - q0), ct);
    }
  }
  if constexpr (FILTER) filter_finish(e, lcnt, q0, GBN, ct);
}

// =============================================================================================
// 256 x 256 tile, 8 waves, BK = 64, "quadrant phases" (the default large-batch kernel).
//
// The LDS holds two K-tiles (buffer = tile & 1), each as four 16 KiB half-tiles: A0/A1 = catalog
// rows 0-127 / 128-255, B0/B1 = queries 0-127 / 128-255 (128 rows x 128 B, chunk c of row r at
// slot c ^ (r & 7): conflict-free ds_read_b128 for the 16x16x32 operand map). A K-tile is
// computed in four phases, one output QUADRANT each -- Q1 (A0,B0), Q2 (A0,B1), Q3 (A1,B1),
// Q4 (A1,B0) -- with all 8 waves on the same quadrant (2 x 4 waves of 64 x 32 outputs: 16
// MFMAs per wave per phase). So every half-tile dies early (A0 after Q2, B1 after Q3, A1 and B0
// after Q4) and its region is restaged for tile t+2 one phase later: each phase issues exactly
// one half-tile (2 LDS-DMA pieces per lane), keeping 3-4 half-tiles in flight.
// Accumulators: 4 quadrants x 4 x 2 tiles (128 VGPRs).
// =============================================================================================
constexpr int QP_THREADS = 512;
constexpr int QP_HALF = 128 * 128;            // 16 KiB: 128 rows x 64 k x 2 B
constexpr int QP_BUF = 4 * QP_HALF;           // one K-tile
constexpr int QP_LDS = 2 * QP_BUF;            // 128 KiB
constexpr int QP_GROUP_C = 4;
constexpr int QP_TILE = 256;
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}
// s_waitcnt with an immediate chosen at run time (near the last tiles fewer loads follow).
__device__ __forceinline__ void wait_vm_halves(int halves_after) {
  if (halves_after >= 4) wait_vm<8>();
  else if (halves_after == 3) wait_vm<6>();
  else if (halves_after == 2) wait_vm<4>();
  else if (halves_after == 1) wait_vm<2>();
  else wait_vm<0>();
}

// s_barrier is a no-memory intrinsic to LLVM: the empty asm with a memory clobber keeps LDS
// reads from being hoisted above it at IR level; sched_barrier(0) does the same for the
// machine scheduler.
__device__ __forceinline__ void qp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}


// =============================================================================================
// Pipelined quadrant phases (qp2): ONE barrier per phase, and the fragments of the NEXT phase
// are read while the current phase's 16 MFMAs run (interleaved by sched_group_barrier), so LDS
// reads and barriers do not sit between MFMA clusters. Register sets: A0 / A1 fragments (32 VGPRs each) and two
// B sets whose roles swap every K-tile (B0(t) is read in Q4(t-1) and kept until Q4(t), B1(t) is
// read in Q1(t)), 224 VGPRs with the accumulators.
// Half-tile schedule (phase P = 4t + quadrant issues sequence index P + 7, index = 4u + type
// with type A0, B0, B1, A1): a region is restaged >= 2 phases after its last ds_read issue and
// `s_waitcnt vmcnt(8)` before the barrier of every phase that reads retires exactly the half
// that phase reads (A0/B0 of t+1 in Q4(t), B1(t) in Q1(t), A1(t) in Q2(t)).
// =============================================================================================
enum { P_A0 = 0, P_B0 = 1, P_B1 = 2, P_A1 = 3 };
__device__ __forceinline__ constexpr int p_half_off(int type) {
  return type == P_A0 ? 0 : type == P_A1 ? QP_HALF : type == P_B0 ? 2 * QP_HALF : 3 * QP_HALF;
}

template <bool BF16>
__device__ __forceinline__ void qp2_mma(f32x4_t (&acc)[4][2], const u16x8_t (&a)[4][2],
                                        const u16x8_t (&b)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16<BF16>(a[i][ks], b[j][ks], acc[i][j]);
}

// Epilogue modes of the quadrant-phase kernel: EPI_STORE (score rows), EPI_FILTER (the fused
// screen's hit slots), EPI_POOL (the speculative screen's sample: per query and 64-row subgroup
// only the MAX score, S[q][4 ct + 2 ah + wa] -- 64x less output than the scores).
enum { EPI_STORE = 0, EPI_FILTER = 1, EPI_POOL = 2 };

template <bool BF16, int EPI>
__global__ __launch_bounds__(QP_THREADS, 2) void screen_gemm_qp2_kernel(
    const uint16_t* __restrict__ Q, const uint16_t* __restrict__ C, int64_t ld_img,
    int64_t n_rows, int n_qtiles, int64_t n_ctiles, int ktiles,
    const float* __restrict__ qscale, const float* __restrict__ cscale, EpiArgs e,
    int64_t cstride) {
  constexpr bool FILTER = EPI == EPI_FILTER;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t bid = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int64_t nwg = (int64_t)n_qtiles * n_ctiles;
  const int64_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int64_t L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int64_t per_group = (int64_t)QP_GROUP_C * n_qtiles;
  const int64_t g = L / per_group, w = L - g * per_group;
  const int64_t gc_rem = n_ctiles - g * QP_GROUP_C;
  const int64_t gc = gc_rem < QP_GROUP_C ? gc_rem : QP_GROUP_C;
  const int64_t ct = g * QP_GROUP_C + w % gc;
  const int64_t qt = w / gc;
  const int64_t c0 = ct * 256;
  // catalog row of the tile's first row: c0, or ct * cstride for a strided sample of full tiles
  // (store mode; n_rows then counts the sample's rows and the scores stay dense)
  const int64_t c0s = ct * cstride;
  const int64_t q0 = qt * 256;
  // after the K-tile ring: hits per query of the tile (filter mode), then the epilogue's
  // per-query scale / threshold and per-row scale, loaded before the prologue's LDS-DMA so they
  // retire with its first wait instead of stalling the epilogue
  uint32_t* lcnt = (uint32_t*)(smem + QP_LDS);
  float* lqs = (float*)(smem + QP_LDS + 1024);
  float* lth = lqs + QP_TILE;
  float* lcs = lth + QP_TILE;
  if constexpr (FILTER) {
    if (tid < QP_TILE) lcnt[tid] = 0u;
  }
  float pre_a = 1.f, pre_b = 0.f;
  if (tid < QP_TILE) {
    pre_a = qscale[q0 + tid];
    if constexpr (FILTER) pre_b = e.thr[q0 + tid];
  } else {
    const int64_t r = tid - QP_TILE;
    pre_a = (cscale && c0 + r < n_rows) ? cscale[c0s + r] : 1.f;
  }

  const int wa = wave >> 2;
  const int wb = wave & 3;
  const int fr = lane & 15;
  int a_off[4][2], b_off[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int c = ks * 4 + (lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wa * 64 + i * 16 + fr;
      a_off[i][ks] = r * 128 + ((c ^ (r & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wb * 32 + j * 16 + fr;
      b_off[j][ks] = r * 128 + ((c ^ (r & 7)) << 4);
    }
  }

  f32x4_t acc0[4][2], acc1[4][2], acc2[4][2], acc3[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc0[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      acc1[i][j] = acc0[i][j];
      acc2[i][j] = acc0[i][j];
      acc3[i][j] = acc0[i][j];
    }

  // LDS-DMA through buffer descriptors (T8): one 32-bit per-lane offset serves every half-tile;
  // rows past the end of the catalog fall outside num_records and read as 0 (never stored).
  const int64_t row_bytes = ld_img * 2;
  const int64_t c_rem = (n_rows - c0) * row_bytes;
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(C + c0s * ld_img), 0, (int)(c_rem < 0x7fffffffLL ? c_rem : 0x7fffffffLL),
      0x00020000);
  const __amdgpu_buffer_rsrc_t rsQ = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Q + q0 * ld_img), 0, (int)(256 * row_bytes), 0x00020000);
  // lane: row (wave*16 + (lane>>3)) of the half, 16-byte chunk (lane&7)^(lane>>3)
  const int voff = (int)((wave * 16 + (lane >> 3)) * row_bytes) + (((lane & 7) ^ (lane >> 3)) << 4);
  const int piece_step = (int)(8 * row_bytes);
  const int half_step = (int)(128 * row_bytes);
  const int total = 4 * ktiles;
  auto issue_u = [&](int idx) {  // no bounds check: the caller guarantees idx < total
    const int tile = idx >> 2, type = idx & 3;
    char* dst = smem + (tile & 1) * QP_BUF + p_half_off(type) + wave * 2048;
    const int soff = tile * 128 + ((type == P_A1 || type == P_B1) ? half_step : 0);
    const __amdgpu_buffer_rsrc_t rs = (type == P_A0 || type == P_A1) ? rsC : rsQ;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, voff, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 1024), 16, voff,
                                             soff + piece_step, 0, 0);
  };
  auto issue = [&](int idx) {
    if (idx < total) {
      const int tile = idx >> 2, type = idx & 3;
      char* dst = smem + (tile & 1) * QP_BUF + p_half_off(type) + wave * 2048;
      const int soff = tile * 128 + ((type == P_A1 || type == P_B1) ? half_step : 0);
      const __amdgpu_buffer_rsrc_t rs = (type == P_A0 || type == P_A1) ? rsC : rsQ;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, voff, soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 1024), 16, voff,
                                               soff + piece_step, 0, 0);
    }
  };
  auto wait_for = [&](int needed, int last_issued) {
    const int last = last_issued < total - 1 ? last_issued : total - 1;
    const int n = last - needed;
    wait_vm_halves(n > 0 ? n : 0);
  };
  auto read_a = [&](u16x8_t (&a)[4][2], const char* half) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][ks] = *(const u16x8_t*)(half + a_off[i][ks]);
  };
  auto read_b = [&](u16x8_t (&b)[2][2], const char* half) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j][ks] = *(const u16x8_t*)(half + b_off[j][ks]);
  };

  u16x8_t fa0[4][2], fa1[4][2], fbx[2][2], fby[2][2];
  // prologue: sequence indices 0..6; A0(0), B0(0) into the A0 / X sets
#pragma unroll
  for (int idx = 0; idx < 7; ++idx) issue(idx);
  wait_for(1, 6);
  if (tid < QP_TILE) {
    lqs[tid] = pre_a;
    lth[tid] = pre_b;
  } else {
    lcs[tid - QP_TILE] = pre_a;
  }
  qp_barrier();
  read_a(fa0, smem + p_half_off(P_A0));
  read_b(fbx, smem + p_half_off(P_B0));
  wait_for(2, 6);  // B1(0), read in Q1(0)

  // One tile of four phases. B0(t) lives in `s0`, B1(t) in `s1`; Q4 reads B0(t+1) into s1.
// GUARD = false in the steady state (every issued half-tile exists): the LDS-DMA pieces then
// live in the same basic block as the MFMAs and are spread between them by the
// sched_group_barrier patterns (masks: 0x008 MFMA, 0x100 DS read, 0x020 VMEM read) instead of
// sitting in front of the phase's first MFMA, where both waves of a SIMD stalled on their DMA
// issue at once.
#define QP2_ISSUE(IDX, GUARD)                                                                    \
  {                                                                                              \
    if (GUARD) issue(IDX);                                                                       \
    else issue_u(IDX);                                                                           \
  }
#define QP2_TILE(T, s0, s1, GUARD)                                                                \
  {                                                                                              \
    const int t_ = (T);                                                                          \
    const char* buf = smem + (t_ & 1) * QP_BUF;                                                  \
    const char* nbuf = smem + ((t_ + 1) & 1) * QP_BUF;                                           \
    /* Q1 (A0, B0): read B1(t) */                                                                \
    qp_barrier();                                                                                \
    QP2_ISSUE(4 * t_ + 7, GUARD);                                                                \
    qp2_mma<BF16>(acc0, fa0, s0);                                                                \
    read_b(s1, buf + p_half_off(P_B1));                                                          \
    if (!(GUARD)) {                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                         \
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
    } else {                                                                                     \
      _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_) {                                         \
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
    }                                                                                            \
    if (GUARD) wait_for(4 * t_ + 3, 4 * t_ + 7); else wait_vm<8>(); /* A1(t) for Q2 */           \
    /* Q2 (A0, B1): read A1(t) */                                                                \
    qp_barrier();                                                                                \
    QP2_ISSUE(4 * t_ + 8, GUARD);                                                                \
    qp2_mma<BF16>(acc1, fa0, s1);                                                                \
    read_a(fa1, buf + p_half_off(P_A1));                                                         \
    if (!(GUARD)) {                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < 5; ++i_) {                                         \
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
    } else {                                                                                     \
      _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) {                                         \
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
    }                                                                                            \
    /* Q3 (A1, B1): no reads */                                                                  \
    qp_barrier();                                                                                \
    QP2_ISSUE(4 * t_ + 9, GUARD);                                                                \
    qp2_mma<BF16>(acc2, fa1, s1);                                                                \
    if (!(GUARD)) {                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);                                        \
    }                                                                                            \
    if (GUARD) wait_for(4 * t_ + 5, 4 * t_ + 9); else wait_vm<8>(); /* A0(t+1), B0(t+1) for Q4 */\
    /* Q4 (A1, B0): read A0(t+1), B0(t+1) */                                                     \
    qp_barrier();                                                                                \
    QP2_ISSUE(4 * t_ + 10, GUARD);                                                               \
    qp2_mma<BF16>(acc3, fa1, s0);                                                                \
    if (!(GUARD) || t_ + 1 < ktiles) {                                                           \
      read_a(fa0, nbuf + p_half_off(P_A0));                                                      \
      read_b(s1, nbuf + p_half_off(P_B0));                                                       \
    }                                                                                            \
    if (!(GUARD)) {                                                                              \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < 3; ++i_) {                                         \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
      _Pragma("unroll") for (int i_ = 0; i_ < 7; ++i_) {                                         \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
    } else {                                                                                     \
      _Pragma("unroll") for (int i_ = 0; i_ < 12; ++i_) {                                        \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                       \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
      }                                                                                          \
    }                                                                                            \
    if (GUARD) wait_for(4 * t_ + 6, 4 * t_ + 10); else wait_vm<8>(); /* B1(t+1) for Q1(t+1) */   \
  }

  int t = 0;
  // steady state: the last half-tile issued by the pair (t, t+1) is 4 (t+1) + 10 < 4 ktiles
  for (; t + 4 < ktiles; t += 2) {
    QP2_TILE(t, fbx, fby, false);
    QP2_TILE(t + 1, fby, fbx, false);
  }
  for (; t + 1 < ktiles; t += 2) {
    QP2_TILE(t, fbx, fby, true);
    QP2_TILE(t + 1, fby, fbx, true);
  }
  if (t < ktiles) QP2_TILE(t, fbx, fby, true);
#undef QP2_TILE
#undef QP2_ISSUE

  // ---- epilogue: quadrant (ah, bh) = catalog half ah x query half bh ----
  const bool full = c0 + QP_TILE <= n_rows;  // uniform
  // Filter mode. Each lane holds 4 query columns (bh, j) x 32 catalog rows (2 halves x 4
  // accumulators x 4 rows); a block is one accumulator (4 consecutive rows of one query).
  //   1. column test (every tile): the max of each column's 32 values against the query's
  //      threshold -- 4 compares per lane, no per-block branches. SIMPLE (no row scales, a full
  //      tile): max_r fl(a_r qs) = fl(max_r(a_r) qs) for qs >= 0 (rounding is monotone), so the
  //      scale is applied once per column; NaNs drop out of fmaxf as they do out of >=.
  //   2. only if some lane of the wave passed: block bits m (bit c*8 + ah*4 + i) for the flagged
  //      columns.
  //   3. the lane's flagged blocks go to its 8 LDS slots in the dead K-tile ring (rounds of 8
  //      when a lane has more; only the wave's flagged columns are visited), and a ROLLED loop over the lane's own blocks computes the exact
  //      values, claims slots with one LDS atomic per block and writes the hits: the work
  //      follows the lane's hits, not the union of the wave's blocks (the earlier form executed
  //      every block any lane had flagged: ~600 VALU per wave with 2 hits, ~1500 with 60).
  // Every wave passed the last tile's final barrier after its last LDS read of the ring.
  auto filter_tile = [&](auto simple_tag) {
    constexpr bool SIMPLE = decltype(simple_tag)::value;
    float qs_r[2][2], th_r[2][2];
#pragma unroll
    for (int bh = 0; bh < 2; ++bh)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ql = bh * 128 + wb * 32 + j * 16 + fr;
        qs_r[bh][j] = lqs[ql];
        th_r[bh][j] = lth[ql];
      }
    // quadrant q = (ah, bh): acc0 (0, 0), acc1 (0, 1), acc2 (1, 1), acc3 (1, 0)
    auto acc_of = [&](int ah, int bh) -> const f32x4_t (&)[4][2] {
      return ah == 0 ? (bh == 0 ? acc0 : acc1) : (bh == 0 ? acc3 : acc2);
    };
    // row scales, register-resident (read from LDS once; 1 without scales)
    float4 cs_r[2][4];
    if constexpr (!SIMPLE) {
#pragma unroll
      for (int ah = 0; ah < 2; ++ah)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          cs_r[ah][i] = *(const float4*)(lcs + ah * 128 + wa * 64 + i * 16 + 4 * (lane >> 4));
    }
    // the exact epilogue values of block (ah, bh, i, j). Rows past n_rows are NOT masked here
    // (they read 0 through the buffer descriptor): the block bits are a superset, the exact
    // per-row test in the hit loop drops them.
    auto val4 = [&](int ah, int bh, int i, int j, float (&v)[4]) {
      const f32x4_t& a = acc_of(ah, bh)[i][j];
      const float qs = qs_r[bh][j];
      const float4 cs = cs_r[ah][i];
      v[0] = a[0] * qs * cs.x;
      v[1] = a[1] * qs * cs.y;
      v[2] = a[2] * qs * cs.z;
      v[3] = a[3] * qs * cs.w;
    };
    auto max4 = [](float a, float b, float c, float d) { return fmaxf(fmaxf(a, b), fmaxf(c, d)); };
    uint32_t m = 0;
    if constexpr (SIMPLE) {
      uint32_t colm = 0;
#pragma unroll
      for (int bh = 0; bh < 2; ++bh)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float mx = -__builtin_inff();
#pragma unroll
          for (int ah = 0; ah < 2; ++ah)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const f32x4_t& a = acc_of(ah, bh)[i][j];
              mx = fmaxf(mx, max4(a[0], a[1], a[2], a[3]));
            }
          colm |= (mx * qs_r[bh][j] >= th_r[bh][j] ? 1u : 0u) << (bh * 2 + j);
        }
      if (__builtin_expect(__ballot(colm != 0u) == 0ull, 1)) return;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int bh = c >> 1, j = c & 1;
        if (__ballot((colm >> c) & 1u) == 0ull) continue;
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4_t& a = acc_of(ah, bh)[i][j];
            const float mx = max4(a[0], a[1], a[2], a[3]) * qs_r[bh][j];
            m |= (mx >= th_r[bh][j] ? 1u : 0u) << (c * 8 + ah * 4 + i);
          }
      }
    } else {
      // row scales or a partial tile: the block bits directly (each block's values are used
      // at once; a column pass first would keep all 128 values live and spill)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v[4];
            val4(ah, c >> 1, i, c & 1, v);
            m |= (max4(v[0], v[1], v[2], v[3]) >= th_r[c >> 1][c & 1] ? 1u : 0u)
                 << (c * 8 + ah * 4 + i);
          }
      if (__builtin_expect(__ballot(m != 0u) == 0ull, 1)) return;
    }
    char* stg = smem + wave * 8192 + lane * 128;  // this lane's 8 slots of 16 B
    // columns with a flagged block in some lane of the wave (uniform): only their 8 blocks are
    // visited when staging
    uint32_t cols = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      cols |= (__ballot(((m >> (8 * c)) & 0xffu) != 0u) != 0ull ? 1u : 0u) << c;
    const int nblk = __popc(m);
    uint32_t rest = m;
#pragma unroll 1
    for (int round = 0;; ++round) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (!((cols >> c) & 1u)) continue;
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int g = c * 8 + ah * 4 + i;
            const int rank = __popc(m & ((1u << g) - 1u));
            if (((m >> g) & 1u) && (rank >> 3) == round)
              *(f32x4_t*)(stg + (rank & 7) * 16) = acc_of(ah, c >> 1)[i][c & 1];
          }
      }
#pragma unroll 1
      for (int s2 = 0; s2 < 8; ++s2) {
        if (__ballot(rest != 0u) == 0ull) break;
        if (rest != 0u && (nblk - __popc(rest)) >> 3 == round) {
          const int g = __builtin_ctz(rest);
          rest &= rest - 1u;
          const f32x4_t a = *(const f32x4_t*)(stg + s2 * 16);
          const int c = g >> 3, ah = (g >> 2) & 1, i = g & 3;
          const int ql = (c >> 1) * 128 + wb * 32 + (c & 1) * 16 + fr;
          const int il = ah * 128 + wa * 64 + i * 16 + 4 * (lane >> 4);
          const float qs = lqs[ql], th = lth[ql];
          const float4 cs = *(const float4*)(lcs + il);
          const float v[4] = {a[0] * qs * cs.x, a[1] * qs * cs.y, a[2] * qs * cs.z,
                              a[3] * qs * cs.w};
          uint32_t hb = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            hb |= (v[r] >= th && (full || c0 + il + r < n_rows) ? 1u : 0u) << r;
          if (hb) {
            const uint32_t base = atomicAdd(lcnt + ql, (uint32_t)__popc(hb));
            uint64_t* dst = e.cand + (q0 + ql) * e.ld_cand + ct * e.slots;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t p = base + (uint32_t)__popc(hb & ((1u << r) - 1u));
              if (((hb >> r) & 1u) && p < (uint32_t)e.slots) {
                const uint32_t row = (uint32_t)(e.idx_base + c0 + il + r);
                dst[p] = ((uint64_t)f2key(v[r]) << 32) | (uint64_t)(~row);
              }
            }
          }
        }
      }
      if (__ballot(nblk > 8 * (round + 1)) == 0ull) break;
    }
  };
  auto store_quadrant = [&](const f32x4_t (&acc)[4][2], int ah, int bh) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ql = bh * 128 + wb * 32 + j * 16 + fr;
      const float qs = lqs[ql];
      const float th = FILTER ? lth[ql] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int il = ah * 128 + wa * 64 + i * 16 + 4 * (lane >> 4);
        const float4 cs = *(const float4*)(lcs + il);
        epilogue4v<FILTER>(e, q0 + ql, c0 + il, n_rows, acc[i][j], qs, th, cs, lcnt + ql, ct);
      }
    }
  };
  // pool mode: max over the 64 rows (ah, wa) of each query: 4 accumulators x 4 values in the
  // lane, then the 4 lanes of the same fr (lane ^ 16, ^ 32); rows past n_rows are skipped
  auto pool_quadrant = [&](const f32x4_t (&acc)[4][2], int ah, int bh) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ql = bh * 128 + wb * 32 + j * 16 + fr;
      const float qs = lqs[ql];
      float mx = -__builtin_inff();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int il = ah * 128 + wa * 64 + i * 16 + 4 * (lane >> 4);
        const float4 cs = *(const float4*)(lcs + il);
        const f32x4_t& a = acc[i][j];
        const float v[4] = {a[0] * qs * cs.x, a[1] * qs * cs.y, a[2] * qs * cs.z, a[3] * qs * cs.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c0 + il + r < n_rows) mx = fmaxf(mx, v[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if ((lane >> 4) == 0) e.S[(q0 + ql) * e.ld_s + ct * 4 + ah * 2 + wa] = mx;
    }
  };
  if constexpr (EPI == EPI_POOL) {
    pool_quadrant(acc0, 0, 0);
    pool_quadrant(acc1, 0, 1);
    pool_quadrant(acc2, 1, 1);
    pool_quadrant(acc3, 1, 0);
  } else if constexpr (FILTER) {
    if (!cscale && full) filter_tile(std::true_type{});
    else filter_tile(std::false_type{});
  } else {
    store_quadrant(acc0, 0, 0);
    store_quadrant(acc1, 0, 1);
    store_quadrant(acc2, 1, 1);
    store_quadrant(acc3, 1, 0);
  }
  if constexpr (FILTER) filter_finish(e, lcnt, q0, QP_TILE, ct);
}


// Kernel choice: batches padded to a multiple of 256 queries take the 256 x 256 quadrant-phase
// kernel; smaller batches (B_pad = 128) the 128 x 128 one. Measured alternatives that lost on
// MI355X ("screening GEMM"): a 4-slot ring with k32 slices, one barrier per phase
// with two barriers (qp), a persistent one-workgroup-per-CU walk of the same tiles, and a
// 4-wave 128 x 128-per-wave tile (LDS-DMA issue cost with one wave per SIMD).
template <int EPI>
static int launch_gemm(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                       int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                       const float* cscale, const EpiArgs& e, hipStream_t stream,
                       int64_t cstride = 0) {
  const bool big = B_pad % QP_TILE == 0;
  if (cstride == 0) cstride = big ? QP_TILE : GBM;
  const int n_qtiles = (int)(B_pad / (big ? QP_TILE : GBN));
  const int64_t n_ctiles = ceil_div(n_rows, big ? QP_TILE : GBM);
  const int64_t nwg = n_ctiles * n_qtiles;
  if (nwg > 0x7fffffffLL) {
    set_error("screen gemm: grid too large");
    return EBT_EINVAL;
  }
  const uint16_t* Q = (const uint16_t*)qimg;
  const uint16_t* C = (const uint16_t*)cimg;
  if (big) {
    dim3 grid((unsigned)nwg), block(QP_THREADS);
    auto k = img_dtype == EBT_BF16 ? screen_gemm_qp2_kernel<true, EPI>
                                   : screen_gemm_qp2_kernel<false, EPI>;
    const int lds = QP_LDS + 1024 + 3 * QP_TILE * 4;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k, grid, block, lds, stream, Q, C, (int64_t)ld_img, n_rows, n_qtiles,
                       n_ctiles, d_pad / 64, qscale, cscale, e, cstride);
    return launch_check("screen_gemm_qp2_kernel");
  }
  if (cstride != GBM || EPI == EPI_POOL) {
    set_error("screen gemm: strided tiles / pooled scores need a batch padded to 256");
    return EBT_EINVAL;
  }
  constexpr bool FILTER = EPI == EPI_FILTER;
  dim3 grid((unsigned)nwg), block(GTHREADS);
  auto k = img_dtype == EBT_BF16 ? screen_gemm_kernel<true, FILTER>
                                 : screen_gemm_kernel<false, FILTER>;
  const int lds = GLDS_BYTES + (FILTER ? GBN * 4 : 0);
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(k, grid, block, lds, stream, Q, C, (int64_t)ld_img, n_rows, n_qtiles,
                     n_ctiles, d_pad / GBK, qscale, cscale, e);
  return launch_check("screen_gemm_kernel");
}

int64_t filter_group_rows(int64_t B_pad);

static int check_gemm_args(const char* who, const void* qimg, int64_t B_pad, const void* cimg,
                           int64_t n_rows, int32_t d_pad, int32_t ld_img, int img_dtype,
                           const float* qscale, const float* cscale) {
  if (!qimg || !cimg || !qscale) {
    set_error("%s: null pointer", who);
    return EBT_EINVAL;
  }
  if (B_pad <= 0 || B_pad % GBN != 0 || n_rows <= 0 || d_pad <= 0 || d_pad % GBK != 0 ||
      ld_img < d_pad || ld_img % 64 != 0 || (img_dtype != EBT_F16 && img_dtype != EBT_BF16)) {
    set_error("%s: bad shape (B_pad=%lld n=%lld d_pad=%d ld_img=%d)", who, (long long)B_pad,
              (long long)n_rows, d_pad, ld_img);
    return EBT_EINVAL;
  }
  if (cscale && ((uintptr_t)cscale & 15)) {
    set_error("%s: cscale must be 16-byte aligned", who);
    return EBT_EINVAL;
  }
  return EBT_OK;
}

int screen_gemm(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows, int32_t d_pad,
                int32_t ld_img, int img_dtype, const float* qscale, const float* cscale,
                float* scores, int64_t ld_scores, hipStream_t stream, int64_t cstride) {
  int rc = check_gemm_args("ebt_screen_scores", qimg, B_pad, cimg, n_rows, d_pad, ld_img,
                           img_dtype, qscale, cscale);
  if (rc) return rc;
  if (!scores || ld_scores < n_rows || ld_scores % 4 != 0) {
    set_error("ebt_screen_scores: bad score buffer (ld_s=%lld)", (long long)ld_scores);
    return EBT_EINVAL;
  }
  EpiArgs e{};
  e.S = scores;
  e.ld_s = ld_scores;
  if (cstride == 0) cstride = filter_group_rows(B_pad);
  if (cstride != filter_group_rows(B_pad) && (cstride < QP_TILE || n_rows % QP_TILE != 0)) {
    set_error("ebt_screen_scores: strided tiles must be full and non-overlapping");
    return EBT_EINVAL;
  }
  return launch_gemm<EPI_STORE>(qimg, B_pad, cimg, n_rows, d_pad, ld_img, img_dtype, qscale,
                                cscale, e, stream, cstride);
}

// The speculative screen's sample: P full 256-row tiles, cstride rows apart (P = n_rows / 256),
// -> pooled[q][g] = max score of query q over the sample's 64-row subgroup g (4P per query).
int screen_gemm_pool(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                     int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                     const float* cscale, int64_t cstride, float* pooled, int64_t ld_pooled,
                     hipStream_t stream) {
  int rc = check_gemm_args("screen_gemm_pool", qimg, B_pad, cimg, n_rows, d_pad, ld_img,
                           img_dtype, qscale, cscale);
  if (rc) return rc;
  if (!pooled || B_pad % QP_TILE != 0 || n_rows % QP_TILE != 0 || cstride < QP_TILE ||
      ld_pooled < n_rows / 64) {
    set_error("screen_gemm_pool: bad arguments");
    return EBT_EINVAL;
  }
  EpiArgs e{};
  e.S = pooled;
  e.ld_s = ld_pooled;
  return launch_gemm<EPI_POOL>(qimg, B_pad, cimg, n_rows, d_pad, ld_img, img_dtype, qscale,
                               cscale, e, stream, cstride);
}

int64_t filter_group_rows(int64_t B_pad) { return B_pad % QP_TILE == 0 ? QP_TILE : GBM; }

int screen_gemm_filter(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                       int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                       const float* cscale, const float* thr, uint64_t* cand, int64_t ld_cand,
                       int slots, uint8_t* counts, int64_t ld_counts, int* ovf, int64_t idx_base,
                       hipStream_t stream) {
  int rc = check_gemm_args("ebt_screen_filter", qimg, B_pad, cimg, n_rows, d_pad, ld_img,
                           img_dtype, qscale, cscale);
  if (rc) return rc;
  const int64_t groups = ceil_div(n_rows, filter_group_rows(B_pad));
  if (!thr || !cand || !counts || !ovf || slots < 1 || slots > EBT_FILTER_SLOTS_MAX ||
      ld_counts < groups || ld_cand < groups * slots || idx_base < 0 ||
      idx_base + n_rows > 0xffffffffLL) {
    set_error("ebt_screen_filter: bad candidate buffers (groups=%lld ld_cand=%lld ld_counts=%lld)",
              (long long)groups, (long long)ld_cand, (long long)ld_counts);
    return EBT_EINVAL;
  }
  EpiArgs e{};
  e.thr = thr;
  e.cand = cand;
  e.ld_cand = ld_cand;
  e.counts = counts;
  e.ld_counts = ld_counts;
  e.ovf = ovf;
  e.idx_base = idx_base;
  e.slots = slots;
  return launch_gemm<EPI_FILTER>(qimg, B_pad, cimg, n_rows, d_pad, ld_img, img_dtype, qscale,
                                 cscale, e, stream);
}

}  // namespace ebt
