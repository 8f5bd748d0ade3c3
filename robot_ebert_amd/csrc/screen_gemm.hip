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
#include <hip/hip_ext.h>

#include <atomic>
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
constexpr int QP_GROUP_C = 4;  // (tile_at's whole-group fast path shifts by 2)
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
// Persistent pipelined quadrant phases (qp2): ONE barrier per phase, the fragments of the NEXT
// phase are read while the current phase's 16 MFMAs run (interleaved by sched_group_barrier),
// and each workgroup walks several output tiles with the LDS-DMA stream running straight across
// the tile boundary: the last two K-tiles of tile s stage the first two K-tiles of tile s+1, so
// the next tile's operands are in flight during the epilogue (no per-tile prologue latency, no
// per-tile workgroup launch). Register sets: A0 / A1 fragments (32 VGPRs each) and two B sets
// whose roles swap every K-tile (B0(t) is read in Q4(t-1) and kept until Q4(t), B1(t) is read in
// Q1(t)), 224 VGPRs with the accumulators.
// Half-tile schedule (K-tile t issues A1(t+1) in Q1 and A0/B0/B1(t+2) in Q2/Q3/Q4; K-tile
// indices run on across tiles, an even K-tile count keeps buffer = K-tile & 1): a region is
// restaged >= 2 phases after its last ds_read issue and `s_waitcnt vmcnt(8)` before the barrier
// of every phase that reads retires exactly the half that phase reads (A0/B0 of t+1 in Q4(t),
// B1(t) in Q1(t), A1(t) in Q2(t)); every other load in the stream (the epilogue parameters)
// only makes a counted wait stricter. The last tile of a workgroup restages its own first
// K-tiles into dead regions (no branch in the MFMA blocks) and drains the stream before exit.
// Tile walk: the tiles of the launch are split into 8 contiguous ranges, one per XCD
// (workgroup b runs on XCD b & 7), and the n_x workgroups of an XCD take its range round-robin,
// so the tiles in flight on one XCD are consecutive -- groups of 4 catalog tiles walked
// query-tile-major, a catalog tile fetched about once per XCD and re-read from its L2.
// An odd K-tile count runs one extra all-zero K-tile (a descriptor with no records).
// =============================================================================================
enum { P_A0 = 0, P_B0 = 1, P_B1 = 2, P_A1 = 3 };
// Ring layout by half-tile, buffer innermost: A0 | A1 | B0 | B1, each [buffer 0 | buffer 1] of
// 16 KiB, so every catalog fragment lies within 64 KiB of one lane base and every query fragment
// within 64 KiB of another (ds_read_b128's 16-bit immediate covers both buffers).
__device__ __forceinline__ constexpr int p_half_addr(int type, int buf) {
  return (type == P_A0 ? 0 : type == P_A1 ? 2 : type == P_B0 ? 4 : 6) * QP_HALF + buf * QP_HALF;
}

template <bool BF16>
__device__ __forceinline__ void qp2_mma(f32x4_t (&acc)[4][2], const u16x8_t (&a)[4][2],
                                        const u16x8_t (&b)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = mfma16<BF16>(a[i][ks], b[j][ks], acc[i][j]);
}

// Epilogue modes of the quadrant-phase kernel: EPI_STORE (score rows), EPI_FILTER (the fused
// screen's hit slots), EPI_POOL (the speculative screen's sample: per query and 64-row subgroup
// only the MAX score, S[q][4 ct + 2 ah + wa] -- 64x less output than the scores).
enum { EPI_STORE = 0, EPI_FILTER = 1, EPI_POOL = 2 };

// LDS after the 128 KiB ring: hit counters (1 KiB), the tile's query scales / thresholds / row
// scales (3 KiB, LDS-DMA'd per tile), the filter epilogue's hit staging: per wave QP_STG_COLS
// flagged (lane, query column) pairs per round, each its 32 raw accumulators (128 B) and a
// 16-byte record {local query | row group << 8, query scale, threshold, -}.
constexpr int QP_PARAM = 1024 + 3 * QP_TILE * 4;
#ifndef EBT_HIT_STAGE_WHOLE
// half columns: 16 raw accumulators (64 B) + a 16-byte record per slot, 32 slots per wave
constexpr int QP_STG_COLS = 32;
constexpr int QP_STG_VAL = 64;
#else
constexpr int QP_STG_COLS = 16;
constexpr int QP_STG_VAL = 128;
#endif
constexpr int QP_STG_WAVE = QP_STG_COLS * (QP_STG_VAL + 16);
constexpr int QP_STG = 8 * QP_STG_WAVE;
#ifdef EBT_EPI_STAMP
// diagnostic build: per wave 8 u64 (phase cycle sums, tiles, last stamp) after the staging area
constexpr int QP_EPI_STAMP = 8 * 8 * 8;
#else
constexpr int QP_EPI_STAMP = 0;
#endif
constexpr int QP_LDS_TOTAL = QP_LDS + QP_PARAM + QP_STG + QP_EPI_STAMP;
static_assert(QP_LDS_TOTAL <= 160 * 1024, "LDS budget");

// Epilogue LDS reads in inline asm (each completes before it returns). The compiler treats any
// LDS read as possibly aliasing the LDS-DMA writes in flight and would put s_waitcnt vmcnt(0) in
// front of it, draining the next tile's operand stream (and the hit stores) in the epilogue; the
// parameter arrays and staging slots are disjoint from the ring by construction.
__device__ __forceinline__ float lds_f32(const void* p) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v) : "v"((uint32_t)(uintptr_t)p) : "memory");
  return v;
}
__device__ __forceinline__ f32x4_t lds_f32x4(const void* p) {
  f32x4_t v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(v) : "v"((uint32_t)(uintptr_t)p) : "memory");
  return v;
}
// Four query columns' scale and threshold (8 reads, one wait).
__device__ __forceinline__ void lds_qs_th4(const float* qs, const float* th, const int (&ql)[4],
                                           float (&q)[4], float (&t)[4]) {
  asm volatile(
      "ds_read_b32 %0, %8\n\tds_read_b32 %1, %9\n\tds_read_b32 %2, %10\n\tds_read_b32 %3, %11\n\t"
      "ds_read_b32 %4, %12\n\tds_read_b32 %5, %13\n\tds_read_b32 %6, %14\n\tds_read_b32 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]),
        "=&v"(t[3])
      : "v"((uint32_t)(uintptr_t)(qs + ql[0])), "v"((uint32_t)(uintptr_t)(qs + ql[1])),
        "v"((uint32_t)(uintptr_t)(qs + ql[2])), "v"((uint32_t)(uintptr_t)(qs + ql[3])),
        "v"((uint32_t)(uintptr_t)(th + ql[0])), "v"((uint32_t)(uintptr_t)(th + ql[1])),
        "v"((uint32_t)(uintptr_t)(th + ql[2])), "v"((uint32_t)(uintptr_t)(th + ql[3]))
      : "memory");
}
// The 8 row-scale vectors of a lane (rows base + ah * 128 + i * 16 .. + 3: byte offsets
// ah * 512 + i * 64 from one address, one wait).
__device__ __forceinline__ void lds_rowscales8(const float* p, f32x4_t (&c)[2][4]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:64\n\t"
      "ds_read_b128 %2, %8 offset:128\n\tds_read_b128 %3, %8 offset:192\n\t"
      "ds_read_b128 %4, %8 offset:512\n\tds_read_b128 %5, %8 offset:576\n\t"
      "ds_read_b128 %6, %8 offset:640\n\tds_read_b128 %7, %8 offset:704\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(c[0][0]), "=&v"(c[0][1]), "=&v"(c[0][2]), "=&v"(c[0][3]), "=&v"(c[1][0]),
        "=&v"(c[1][1]), "=&v"(c[1][2]), "=&v"(c[1][3])
      : "v"((uint32_t)(uintptr_t)p)
      : "memory");
}
// f2key (common.h) as selects instead of nested branches: one store block per hit value in the
// filter epilogue runs it under a divergent mask, where each branch level cost an exec save /
// skip pair.
__device__ __forceinline__ uint32_t f2key_select(float f) {
  const uint32_t u = __float_as_uint(f);
  uint32_t k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  k = f == 0.f ? 0x80000000u : k;
  return (f == f && f != -__builtin_inff()) ? k : 0u;
}
// Per-lane select by a lane mask (bit l: lane l takes t): v_cndmask_b32 on an SGPR pair.
__device__ __forceinline__ float vsel(uint64_t m, float t, float f) {
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}
__device__ __forceinline__ f32x4_t vsel4(uint64_t m, const f32x4_t& t, const f32x4_t& f) {
  return f32x4_t{vsel(m, t[0], f[0]), vsel(m, t[1], f[1]), vsel(m, t[2], f[2]),
                 vsel(m, t[3], f[3])};
}
// Staging writes (in asm: a plain LDS store would get the same vmcnt(0) as a plain read).
__device__ __forceinline__ void lds_put_col(uint32_t dst, const f32x4_t& a0, const f32x4_t& a1,
                                            const f32x4_t& a2, const f32x4_t& a3,
                                            const f32x4_t& a4, const f32x4_t& a5,
                                            const f32x4_t& a6, const f32x4_t& a7,
                                            uint32_t meta_dst, const f32x4_t& meta) {
  asm volatile(
      "ds_write_b128 %0, %2\n\tds_write_b128 %0, %3 offset:16\n\t"
      "ds_write_b128 %0, %4 offset:32\n\tds_write_b128 %0, %5 offset:48\n\t"
      "ds_write_b128 %0, %6 offset:64\n\tds_write_b128 %0, %7 offset:80\n\t"
      "ds_write_b128 %0, %8 offset:96\n\tds_write_b128 %0, %9 offset:112\n\t"
      "ds_write_b128 %1, %10"
      :
      : "v"(dst), "v"(meta_dst), "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6),
        "v"(a7), "v"(meta)
      : "memory");
}
// One 16-byte staging write (in asm, as lds_put_col).
__device__ __forceinline__ void lds_put_vec(uint32_t dst, const f32x4_t& v) {
  asm volatile("ds_write_b128 %0, %1" : : "v"(dst), "v"(v) : "memory");
}
// A staged column's record and 8 of its values (one wait).
__device__ __forceinline__ void lds_staged(uint32_t meta, uint32_t vals, f32x4_t& m, f32x4_t& v0,
                                          f32x4_t& v1) {
  asm volatile(
      "ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %4 offset:16\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(m), "=&v"(v0), "=&v"(v1)
      : "v"(meta), "v"(vals)
      : "memory");
}
__device__ __forceinline__ void lds_f32x4x2(const void* p, f32x4_t& c0, f32x4_t& c1) {
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:64\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(c0), "=&v"(c1)
               : "v"((uint32_t)(uintptr_t)p)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t* p, uint32_t v) {
  uint32_t r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(r) : "v"((uint32_t)(uintptr_t)p), "v"(v) : "memory");
  return r;
}
__device__ __forceinline__ float4 lds_float4(const void* p) {
  const f32x4_t v = lds_f32x4(p);
  return make_float4(v[0], v[1], v[2], v[3]);
}

// One output tile of the walk: catalog tile ct (rows c0.., image rows c0s..), query tile q0.
struct QpTile {
  int64_t ct, c0, c0s, q0;
};

// The kernel's arguments. The kernel re-reads them from the kernarg segment where they are used
// (scalar loads through an opaque copy of the segment pointer), so that none stays in SGPRs
// through the K-loop and the epilogue: the filter epilogue needs most of the 102 SGPRs.
struct QpArgs {
  const uint16_t* Q;
  const uint16_t* C;
  int64_t ld_img;
  int64_t n_rows;
  const float* qscale;
  const float* cscale;
  int64_t cstride;
  int n_qtiles, n_ctiles, ktiles;
  int pg_log2;  // log2(QP_GROUP_C * n_qtiles) when that is a power of two, else -1
  // pool mode: the sample's first `lead` tiles are the catalog's first tiles (contiguous), the
  // rest strided from there; the lead tiles' scores are also stored (S2, row pitch ld_s2)
  int lead;
  float* S2;
  int64_t ld_s2;
  EpiArgs e;
};
typedef const __attribute__((address_space(4))) QpArgs* QpArgsK;
__device__ __forceinline__ QpArgsK qp_args() {
  QpArgsK p = (QpArgsK)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

#ifdef EBT_EPI_STAMP
// Diagnostic build only: where a filter launch's cycles go, per wave. Lane 0 of every wave
// stamps the shader clock (s_memtime) at phase boundaries and adds the cycles since its previous
// stamp to that phase's sum in LDS: [0] K-loop (from the end of the previous tile's epilogue),
// [1] column test, [2] hit staging, [3] hit processing, [4] the rest of the epilogue up to the
// next tile (the workgroup barrier included: waiting for the slowest wave), [5] tiles, [6] tiles
// with hits in this wave; [7] the last stamp. Written to g_epi[(block * 8 + wave) * 8 ..] at exit.
__device__ unsigned long long* g_epi;
__device__ __forceinline__ void epi_stamp(char* smem, int wave, int phase) {
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* e = (unsigned long long*)(smem + QP_LDS + QP_PARAM + QP_STG) + wave * 8;
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (phase >= 0) e[phase] += t - e[7];
    e[7] = t;
  }
}
__device__ __forceinline__ void epi_count(char* smem, int wave, int slot) {
  if ((threadIdx.x & 63) == 0)
    ((unsigned long long*)(smem + QP_LDS + QP_PARAM + QP_STG) + wave * 8)[slot] += 1;
}
#define EPI_STAMP(ph) epi_stamp(smem, wave, (ph))
#define EPI_COUNT(sl) epi_count(smem, wave, (sl))
#else
#define EPI_STAMP(ph)
#define EPI_COUNT(sl)
#endif

#ifdef EBT_WALK_STAMP
// Diagnostic build only (the persistent walk's schedule, tools/walk_stamp.py): lane 0 of every
// workgroup of a filter-mode launch records (tile index L, 100 MHz real time) at the start of
// each of its tiles and (-1, time) at exit into g_walk[(block * WALK_MAX + t) * 2 ..] (vector
// stores; nothing else reads them). The shipped library has none of it.
constexpr int WALK_MAX = 4096;
__device__ unsigned long long* g_walk;
#endif
#ifdef EBT_CLOCK_STAMP
// Diagnostic build only (MI355X_MICROARCH.md "DVFS give-back" item 6): lane 0 of each workgroup
// of a filter-mode launch records the shader-clock and the 100 MHz real-time counters after the
// prologue and at exit into g_stamps[4 * blockIdx.x ..] (vector stores; nothing else reads them).
// The in-kernel clock is d(clock) / d(real time) x 100 MHz. The shipped library has none of it.
__device__ unsigned long long* g_stamps;
#endif

template <bool BF16, int EPI, bool ODD>
__global__ __launch_bounds__(QP_THREADS, 2) void screen_gemm_qp2_kernel(QpArgs args) {
  (void)args;  // read through qp_args()
  constexpr bool FILTER = EPI == EPI_FILTER;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bid = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // ---- the workgroup's tiles: L = Lbeg + j, + n_x, ... < Lend ----
  const int nwg = qp_args()->n_qtiles * qp_args()->n_ctiles;
  const int G = gridDim.x;
  const int xcd = bid & 7, j = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int Lbeg = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int Lend = Lbeg + q8 + (xcd < r8 ? 1 : 0);
  const int n_x = (G - xcd + 7) >> 3;  // workgroups on this XCD
  int L = Lbeg + j;
  if (L >= Lend) return;
  auto tile_at = [&](int Lt) {
    const QpArgsK A = qp_args();
    const int per_group = QP_GROUP_C * A->n_qtiles, n_ctiles = A->n_ctiles;
    QpTile T;
    // the walk's divisions are by launch constants: shifts when they are powers of two (every
    // BASELINE batch: 4..64 query tiles) and the group is whole (uniform branches), so the tile
    // boundary does not wait on scalar division sequences
    const int pl = A->pg_log2;
    const int g = pl >= 0 ? Lt >> pl : Lt / per_group, w = Lt - g * per_group;
    const int gc_rem = n_ctiles - g * QP_GROUP_C;
    const int gc = gc_rem < QP_GROUP_C ? gc_rem : QP_GROUP_C;
    int qt;
    if (gc == QP_GROUP_C) {
      T.ct = g * QP_GROUP_C + (w & (QP_GROUP_C - 1));
      qt = w >> 2;
    } else {
      T.ct = g * QP_GROUP_C + w % gc;
      qt = w / gc;
    }
    T.c0 = T.ct * QP_TILE;
    // catalog row of the tile's first row: c0, or ct * cstride for a strided sample of full
    // tiles (store / pool mode; n_rows then counts the sample's rows and the scores stay dense);
    // a pool-mode sample with a lead: tiles [0, lead) contiguous, the rest strided after them
    if constexpr (EPI == EPI_POOL)
      T.c0s = T.ct < A->lead ? T.c0 : (int64_t)A->lead * QP_TILE + (T.ct - A->lead) * A->cstride;
    else
      T.c0s = T.ct * A->cstride;
    T.q0 = (int64_t)qt * QP_TILE;
    return T;
  };
  // the buffer descriptors of a tile's operands (out-of-range catalog rows read as 0); only the
  // current tile's pair stays live through the K-loop, the next tile's is made for the last two
  // K-tiles, and the tile geometry is recomputed for the epilogue (SGPR budget)
  auto rsrc_c = [&](const QpTile& T) {
    const QpArgsK A = qp_args();
    const int64_t c_rem = (A->n_rows - T.c0) * A->ld_img * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(A->C + T.c0s * A->ld_img), 0,
                                             (int)(c_rem < 0x7fffffffLL ? c_rem : 0x7fffffffLL),
                                             0x00020000);
  };
  auto rsrc_q = [&](const QpTile& T) {
    const QpArgsK A = qp_args();
    return __builtin_amdgcn_make_buffer_rsrc((void*)(A->Q + T.q0 * A->ld_img), 0,
                                             (int)(QP_TILE * A->ld_img * 2), 0x00020000);
  };

  uint32_t* lcnt = (uint32_t*)(smem + QP_LDS);
  float* lqs = (float*)(smem + QP_LDS + 1024);
  float* lth = lqs + QP_TILE;
  float* lcs = lth + QP_TILE;
  if (tid < QP_TILE) {
    lcnt[tid] = 0u;
    if (!qp_args()->cscale) lcs[tid] = 1.f;
  }
#ifdef EBT_EPI_STAMP
  if (tid < 64) ((unsigned long long*)(smem + QP_LDS + QP_PARAM + QP_STG))[tid] = 0ull;
  __syncthreads();
  EPI_STAMP(-1);
#endif
  // the tile's epilogue parameters by LDS-DMA (one 1 KiB piece per array, waves 0..2): they
  // travel in the operand stream and are retired by its counted waits
  auto issue_params = [&](const QpTile& T) {
    const QpArgsK A = qp_args();
    // the lane offset from an opaque lane id: hoisted out of the tile loop, it would be spilled
    // at the K-loop's register peak and reloaded with a vmcnt(0) that drains the operand stream
    int lo = tid;
    asm volatile("" : "+v"(lo));
    lo = (lo & 63) * 16;
    if (wave == 0) {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(A->qscale + T.q0), 0, QP_TILE * 4, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lqs, 16, lo, 0, 0, 0);
    } else if (wave == 1 && FILTER) {
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(A->e.thr + T.q0), 0, QP_TILE * 4, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lth, 16, lo, 0, 0, 0);
    } else if (wave == 2 && A->cscale) {
      const int64_t rem = A->n_rows - T.c0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(A->cscale + T.c0s), 0, (int)(rem < QP_TILE ? rem * 4 : QP_TILE * 4), 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lcs, 16, lo, 0, 0, 0);
    }
  };

  const int wa = wave >> 2;
  const int wb = wave & 3;
  // Per-lane LDS fragment offsets (swizzled) and the LDS-DMA lane offset. They are recomputed at
  // the top of every tile from an opaque copy of the lane id: live through the K-loop only, not
  // through the epilogue (whose accumulators + temporaries need the rest of the 256 VGPRs).
  // Fragment (i, ks) of a half at row base + 16 i has row & 7 == fr & 7, so its swizzled offset
  // is base(ks) + i * 2048: one lane base per operand and k-step, the half, buffer and i are
  // ds_read immediates (p_half_addr).
  int a_base[2], b_base[2], voff, wdst, piece_step, half_step, kt, ktiles;
  auto set_geom = [&]() {
    // the wave's LDS-DMA destination offset, opaque too: the 16 destination addresses derived
    // from it stay out of the SGPRs held through the epilogue
    int w = wave * 2048;
    asm volatile("" : "+s"(w));
    wdst = w;
    int l = tid;
    asm volatile("" : "+v"(l));
    l &= 63;
    const int f = l & 15;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int sw = ((ks * 4 + (l >> 4)) ^ (f & 7)) << 4;
      a_base[ks] = (int)(uintptr_t)smem + (wa * 64 + f) * 128 + sw;
      b_base[ks] = (int)(uintptr_t)smem + p_half_addr(P_B0, 0) + (wb * 32 + f) * 128 + sw;
    }
    // LDS-DMA through buffer descriptors (T8): one 32-bit per-lane offset serves every
    // half-tile. lane: row (wave*16 + (lane>>3)) of the half, 16-byte chunk (lane&7)^(lane>>3)
    const QpArgsK A = qp_args();
    voff = (int)((wave * 16 + (l >> 3)) * A->ld_img * 2) + (((l & 7) ^ (l >> 3)) << 4);
    piece_step = (int)(8 * A->ld_img * 2);
    half_step = (int)(128 * A->ld_img * 2);
    kt = A->ktiles + (ODD ? 1 : 0);  // K-tiles per output tile (even)
    ktiles = A->ktiles;
  };

  f32x4_t acc0[4][2], acc1[4][2], acc2[4][2], acc3[4][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        acc0[i][jj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        acc1[i][jj] = acc0[i][jj];
        acc2[i][jj] = acc0[i][jj];
        acc3[i][jj] = acc0[i][jj];
      }
  };

  // half `type` of local K-tile kl of the tile with descriptors (rc, rq) into buffer `buf`
  auto issue_h = [&](const __amdgpu_buffer_rsrc_t& rc, const __amdgpu_buffer_rsrc_t& rq, int kl,
                     int type, int buf) {
    char* dst = smem + p_half_addr(type, buf) + wdst;
    const int soff = kl * 128 + ((type == P_A1 || type == P_B1) ? half_step : 0);
    __amdgpu_buffer_rsrc_t rs = (type == P_A0 || type == P_A1) ? rc : rq;
    if constexpr (ODD) rs = kl < ktiles ? rs : __builtin_amdgcn_make_buffer_rsrc((void*)0, 0, 0, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, voff, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 1024), 16, voff,
                                             soff + piece_step, 0, 0);
  };
  // fragments of half-tile `type` of buffer P (compile time)
  auto read_a = [&](u16x8_t (&a)[4][2], int P, int type) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i][ks] = *(const u16x8_t*)((lds_void*)(uintptr_t)(a_base[ks] + p_half_addr(type, P) + i * 2048));
  };
  auto read_b = [&](u16x8_t (&b)[2][2], int P, int type) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        b[jj][ks] = *(const u16x8_t*)((lds_void*)(uintptr_t)(b_base[ks] + p_half_addr(type, P) - p_half_addr(P_B0, 0) + jj * 2048));
  };

  u16x8_t fa0[4][2], fa1[4][2], fbx[2][2], fby[2][2];
  // prologue: the first tile's parameters, then K-tile 0 (A0, B0, B1, A1) and K-tile 1 (A0, B0,
  // B1) in stream order
  {
    set_geom();
    const QpTile T = tile_at(L);
    issue_params(T);
    const __amdgpu_buffer_rsrc_t rc = rsrc_c(T), rq = rsrc_q(T);
    issue_h(rc, rq, 0, P_A0, 0);
    issue_h(rc, rq, 0, P_B0, 0);
    issue_h(rc, rq, 0, P_B1, 0);
    issue_h(rc, rq, 0, P_A1, 0);
    issue_h(rc, rq, 1, P_A0, 1);
    issue_h(rc, rq, 1, P_B0, 1);
    issue_h(rc, rq, 1, P_B1, 1);
  }
  wait_vm<8>();  // A0(0), B0(0), B1(0)
  qp_barrier();
#ifdef EBT_CLOCK_STAMP
  unsigned long long st_t0 = 0, st_r0 = 0;
  if (EPI == EPI_FILTER && tid == 0) {
    st_t0 = __builtin_amdgcn_s_memtime();
    st_r0 = __builtin_amdgcn_s_memrealtime();
  }
#endif

  // One K-tile of four phases: P = buffer of this K-tile (compile time); (RC1, RQ1, K1): the tile
  // and local index of K-tile t+1 (its A1 is issued in Q1), (RC2, RQ2, K2): of K-tile t+2.
  // The LDS-DMA pieces live in the same basic block as the MFMAs and are spread between them by
  // the sched_group_barrier patterns (masks: 0x008 MFMA, 0x100 DS read, 0x020 VMEM read).
#define QP2_KTILE(P, s0, s1, RC1, RQ1, K1, RC2, RQ2, K2, READ_NEXT)                             \
  {                                                                                             \
    /* Q1 (A0, B0): read B1(t) */                                                               \
    qp_barrier();                                                                               \
    issue_h(RC1, RQ1, K1, P_A1, 1 - (P));                                                       \
    qp2_mma<BF16>(acc0, fa0, s0);                                                               \
    read_b(s1, (P), P_B1);                                                                      \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                          \
    _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_) {                                          \
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                        \
    }                                                                                           \
    wait_vm<8>(); /* A1(t) for Q2 */                                                            \
    /* Q2 (A0, B1): read A1(t) */                                                               \
    qp_barrier();                                                                               \
    issue_h(RC2, RQ2, K2, P_A0, (P));                                                           \
    qp2_mma<BF16>(acc1, fa0, s1);                                                               \
    read_a(fa1, (P), P_A1);                                                                     \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                          \
    _Pragma("unroll") for (int i_ = 0; i_ < 5; ++i_) {                                          \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                        \
    }                                                                                           \
    /* Q3 (A1, B1): no reads */                                                                 \
    qp_barrier();                                                                               \
    issue_h(RC2, RQ2, K2, P_B0, (P));                                                           \
    qp2_mma<BF16>(acc2, fa1, s1);                                                               \
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                          \
    __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);                                         \
    wait_vm<8>(); /* A0(t+1), B0(t+1) for Q4 */                                                 \
    /* Q4 (A1, B0): read A0(t+1), B0(t+1) */                                                    \
    qp_barrier();                                                                               \
    issue_h(RC2, RQ2, K2, P_B1, (P));                                                           \
    qp2_mma<BF16>(acc3, fa1, s0);                                                               \
    if (READ_NEXT) {                                                                            \
      read_a(fa0, 1 - (P), P_A0);                                                               \
      read_b(s1, 1 - (P), P_B0);                                                                \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                        \
      _Pragma("unroll") for (int i_ = 0; i_ < 3; ++i_) {                                        \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                      \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                      \
      }                                                                                         \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                        \
      _Pragma("unroll") for (int i_ = 0; i_ < 7; ++i_) {                                        \
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                      \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                      \
      }                                                                                         \
    } else {                                                                                    \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                                        \
      __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);                                       \
    }                                                                                           \
    wait_vm<8>(); /* B1(t+1) for Q1(t+1) */                                                     \
  }

#ifdef EBT_WALK_STAMP
  int walk_t = 0;
#endif
  for (;;) {
#ifdef EBT_WALK_STAMP
    if (EPI == EPI_FILTER && tid == 0 && g_walk && walk_t < WALK_MAX - 1) {
      unsigned long long* o = g_walk + ((int64_t)bid * WALK_MAX + walk_t) * 2;
      o[0] = (unsigned long long)L;
      o[1] = __builtin_amdgcn_s_memrealtime();
    }
    ++walk_t;
#endif
    const bool last = !(L + n_x < Lend);  // uniform
    // A0(0) / B0(0) of this tile landed before the last barrier (the prologue's, or the
    // previous tile's last phase)
    set_geom();
    read_a(fa0, 0, P_A0);
    read_b(fbx, 0, P_B0);
    {
      const QpTile T = tile_at(L);
      const __amdgpu_buffer_rsrc_t rc = rsrc_c(T), rq = rsrc_q(T);
      // K-tiles 0 .. kt-3 of the tile (pairs), then the boundary pair that stages the next tile
      zero_acc();
      for (int t = 0; t < kt - 2; t += 2) {
        QP2_KTILE(0, fbx, fby, rc, rq, t + 1, rc, rq, t + 2, true);
        QP2_KTILE(1, fby, fbx, rc, rq, t + 2, rc, rq, t + 3, true);
      }
      const QpTile N = tile_at(last ? L : L + n_x);
      const __amdgpu_buffer_rsrc_t nc = rsrc_c(N), nq = rsrc_q(N);
      QP2_KTILE(0, fbx, fby, rc, rq, kt - 1, nc, nq, 0, true);
      QP2_KTILE(1, fby, fbx, nc, nq, 0, nc, nq, 1, false);
    }
    __builtin_amdgcn_sched_barrier(0);
    EPI_STAMP(0);
    EPI_COUNT(5);
    // the epilogue's lane geometry is recomputed from an opaque copy of the lane id, so that
    // none of it is hoisted into registers held through the K-loop
    int lane_e = tid;
    asm volatile("" : "+v"(lane_e));
    const QpTile cur = tile_at(L);
    const QpArgsK A = qp_args();
    const int64_t n_rows = A->n_rows;
    const int tid_ = lane_e, lane_ = tid_ & 63, fr_ = lane_ & 15;
  // ---- epilogue helpers (quadrant (ah, bh) = catalog half ah x query half bh) ----
  // acc0 (0, 0), acc1 (0, 1), acc2 (1, 1), acc3 (1, 0)
  auto acc_of = [&](int ah, int bh) -> const f32x4_t (&)[4][2] {
    return ah == 0 ? (bh == 0 ? acc0 : acc1) : (bh == 0 ? acc3 : acc2);
  };
  // Filter mode. Each lane holds 4 query columns c = bh * 2 + jj, each 32 catalog rows (2 halves
  // x 4 accumulators x 4 rows).
  //   1. column test (every tile): one max per column against the query's threshold, 4 compares
  //      per lane. SIMPLE (no row scales): max_r fl(a_r qs) = fl(max_r(a_r) qs) for qs >= 0
  //      (rounding is monotone), exact. With row scales the max is over fl(a_r cs_r), and the
  //      threshold is lowered by a relative 2^-20 (+2^-120): fl(fl(a qs) cs) and fl(fl(a cs) qs)
  //      are both within (1 +- 2^-24)^2 of a qs cs, so the test is a superset of the exact one.
  //      NaNs drop out of fmaxf as they do out of >=; a column whose qs is not >= 0 is flagged.
  //   2. only if some lane passed: the wave's flagged (lane, column) pairs get consecutive
  //      indices (ballot + mbcnt per column) and are staged, QP_STG_COLS per round, into the
  //      wave's LDS region: the column's 32 raw accumulators + {query, row group, qs, th}.
  //   3. the whole wave processes the staged columns, 4 lanes x 8 values per column: exact
  //      values fl(fl(a qs) cs) (the store mode's), the exact test, one LDS atomic per lane with
  //      hits claims its slots, the hit stores. The cost follows the flagged columns, not the
  //      32 blocks of every lane.
  auto filter_tile = [&](const QpTile& T, auto simple_tag) {
    constexpr bool SIMPLE = decltype(simple_tag)::value;
    const bool full = T.c0 + QP_TILE <= n_rows;  // uniform
    const int g_ = lane_ >> 4;
    const int ql4[4] = {wb * 32 + fr_, wb * 32 + 16 + fr_, 128 + wb * 32 + fr_,
                        128 + wb * 32 + 16 + fr_};
    float q4[4], t4[4];
    lds_qs_th4(lqs, lth, ql4, q4, t4);
    auto max4 = [](float a, float b, float c, float d) { return fmaxf(fmaxf(a, b), fmaxf(c, d)); };
#ifndef EBT_HIT_STAGE_WHOLE
    // the test per HALF column (c, ah), 16 values: bit c * 2 + ah of colm8; colm = per column
    uint32_t colm8 = 0;
    if constexpr (SIMPLE) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int ah = 0; ah < 2; ++ah) {
          float mx = -__builtin_inff();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4_t& a = acc_of(ah, c >> 1)[i][c & 1];
            mx = fmaxf(mx, max4(a[0], a[1], a[2], a[3]));
          }
          colm8 |= (mx * q4[c] >= t4[c] || !(q4[c] >= 0.f) ? 1u : 0u) << (c * 2 + ah);
        }
    } else {
      f32x4_t cs[2][4];
      lds_rowscales8(lcs + wa * 64 + 4 * g_, cs);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float th_lo = t4[c] - fabsf(t4[c]) * 0x1p-20f - 0x1p-120f;
#pragma unroll
        for (int ah = 0; ah < 2; ++ah) {
          float mx = -__builtin_inff();
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4_t& a = acc_of(ah, c >> 1)[i][c & 1];
            const f32x4_t& s = cs[ah][i];
            mx = fmaxf(mx, max4(a[0] * s[0], a[1] * s[1], a[2] * s[2], a[3] * s[3]));
          }
          colm8 |= (mx * q4[c] >= th_lo || !(q4[c] >= 0.f) ? 1u : 0u) << (c * 2 + ah);
        }
      }
    }
    uint32_t colm = 0;  // per column c: either half flagged
#pragma unroll
    for (int c = 0; c < 4; ++c) colm |= (((colm8 >> (2 * c)) & 3u) != 0u ? 1u : 0u) << c;
#else
    uint32_t colm = 0;
    if constexpr (SIMPLE) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float mx = -__builtin_inff();
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4_t& a = acc_of(ah, c >> 1)[i][c & 1];
            mx = fmaxf(mx, max4(a[0], a[1], a[2], a[3]));
          }
        colm |= (mx * q4[c] >= t4[c] || !(q4[c] >= 0.f) ? 1u : 0u) << c;
      }
    } else {
      f32x4_t cs[2][4];
      lds_rowscales8(lcs + wa * 64 + 4 * g_, cs);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float mx = -__builtin_inff();
#pragma unroll
        for (int ah = 0; ah < 2; ++ah)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x4_t& a = acc_of(ah, c >> 1)[i][c & 1];
            const f32x4_t& s = cs[ah][i];
            mx = fmaxf(mx, max4(a[0] * s[0], a[1] * s[1], a[2] * s[2], a[3] * s[3]));
          }
        const float th_lo = t4[c] - fabsf(t4[c]) * 0x1p-20f - 0x1p-120f;
        colm |= (mx * q4[c] >= th_lo || !(q4[c] >= 0.f) ? 1u : 0u) << c;
      }
    }
#endif
#ifdef EBT_ABL_HIT_NONE  // ablation builds only: the column test without the hit path
    if (__ballot(colm != 0u) != 0ull || true) return;
#endif
    EPI_STAMP(1);
    if (__builtin_expect(__ballot(colm != 0u) == 0ull, 1)) return;
    EPI_COUNT(6);
#ifndef EBT_HIT_STAGE_WHOLE
    // 2. HALF columns (16 values, the half ah of a column with its own flag), by block b = (bh, p):
    //    the lane's p-th flagged half column of query half bh (combo k = jj * 2 + ah, in order);
    //    blocks in order, lanes in order within a block (n: uniform). A half is staged in 5
    //    writes (4 value vectors + the record) instead of a column's 9, only where its own max
    //    passes the test (a hit usually sits in one half), and 32 of them fit a round (the same
    //    LDS as 16 columns), so C2's waves stage theirs in one round instead of two. The (jj, ah)
    //    choice is a lane-mask v_cndmask per value, as for whole columns below.
    const uint32_t wst = (uint32_t)(uintptr_t)(smem + QP_LDS + QP_PARAM + wave * QP_STG_WAVE);
    const uint32_t wmeta = wst + QP_STG_COLS * QP_STG_VAL;
    uint64_t* cand = A->e.cand;
    const int64_t ld_cand = A->e.ld_cand;
    const int slots = A->e.slots;
    const int64_t rbase = A->e.idx_base + T.c0;
    // the lane's flagged halves not staged yet, per query half bh (bit jj * 2 + ah)
    uint32_t pend0 = colm8 & 0xFu, pend1 = (colm8 >> 4) & 0xFu;
#pragma unroll 1
    while (__ballot((pend0 | pend1) != 0u) != 0ull) {  // rounds (uniform)
      int nr = 0;  // slots filled in this round (uniform)
#pragma unroll
      for (int bh = 0; bh < 2; ++bh) {
        uint32_t& pend = bh ? pend1 : pend0;
#pragma unroll 1
        while (nr < QP_STG_COLS) {  // passes: each lane's next pending half of this bh
          const bool in = pend != 0u;
          const uint64_t bc = __ballot(in);
          if (bc == 0ull) break;
          const int pos = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bc >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)bc, 0u));
          if (in && nr + pos < QP_STG_COLS) {
            const int s = nr + pos;
            const int k = __builtin_ctz(pend);  // jj * 2 + ah
            pend &= pend - 1u;
            const bool j1 = (k >> 1) != 0, a1 = (k & 1) != 0;
            const uint64_t jm = __ballot(j1), am = __ballot(a1);
            const f32x4_t(&ac0)[4][2] = acc_of(0, bh);
            const f32x4_t(&ac1)[4][2] = acc_of(1, bh);
            const int ql = bh * 128 + wb * 32 + (j1 ? 16 : 0) + fr_;
            const float qs = vsel(jm, q4[bh * 2 + 1], q4[bh * 2]);
            const float th = vsel(jm, t4[bh * 2 + 1], t4[bh * 2]);
            const f32x4_t meta = {
                __builtin_bit_cast(float, (uint32_t)(ql | (g_ << 8) | ((a1 ? 1 : 0) << 12))), qs,
                th, 0.f};
            // one vector at a time (selected, then written): fewer registers live at once
            const uint32_t dst = wst + s * QP_STG_VAL;
#pragma unroll
            for (int i = 0; i < 4; ++i)
              lds_put_vec(dst + i * 16, vsel4(am, vsel4(jm, ac1[i][1], ac1[i][0]),
                                              vsel4(jm, ac0[i][1], ac0[i][0])));
            lds_put_vec(wmeta + s * 16, meta);
          }
          const int cnt = __popcll(bc);
          nr = nr + cnt < QP_STG_COLS ? nr + cnt : QP_STG_COLS;
        }
      }
      EPI_STAMP(2);
      // 3. lane: staged half s, values u * 8 .. u * 8 + 7 = accumulators i0, i0 + 1 (i0 = 2 u)
      // of half ah (the record), rows il0 .. il0 + 3 and il0 + 16 .. il0 + 19
      const int s = lane_ >> 1, u = lane_ & 1;
#ifdef EBT_ABL_HIT_STAGE_ONLY  // ablation builds only: the staging without the processing
      if (s < 0) {
#else
      if (s < nr) {
#endif
        f32x4_t m, v0, v1;
        lds_staged(wmeta + s * 16, wst + s * QP_STG_VAL + u * 32, m, v0, v1);
        const uint32_t mw = __builtin_bit_cast(uint32_t, m[0]);
        const int ql = (int)(mw & 255u), g = (int)((mw >> 8) & 15u), ah = (int)(mw >> 12);
        const float qs = m[1], th = m[2];
        const int il0 = ah * 128 + wa * 64 + u * 32 + 4 * g;
        f32x4_t c0 = {1.f, 1.f, 1.f, 1.f}, c1 = c0;
        if constexpr (!SIMPLE) lds_f32x4x2(lcs + il0, c0, c1);
        float v[8];
        uint32_t hb = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float a = k < 4 ? v0[k] : v1[k - 4];
          v[k] = SIMPLE ? a * qs : a * qs * (k < 4 ? c0[k] : c1[k - 4]);
          const int il = il0 + (k < 4 ? k : 12 + k);
          hb |= (v[k] >= th && (full || T.c0 + il < n_rows) ? 1u : 0u) << k;
        }
        if (hb) {
          const uint32_t base = lds_add_rtn(lcnt + ql, (uint32_t)__popc(hb));
          uint64_t* dst = cand + (T.q0 + ql) * ld_cand + T.ct * slots;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t pp = base + (uint32_t)__popc(hb & ((1u << k) - 1u));
            if (((hb >> k) & 1u) && pp < (uint32_t)slots) {
              const uint32_t row = (uint32_t)(rbase + il0 + (k < 4 ? k : 12 + k));
              uint32_t key = f2key_select(v[k]);
              asm volatile("" : "+v"(key));
#ifndef EBT_ABL_NO_HIT_STORES  // ablation builds only (timing of the epilogue's stores)
              dst[pp] = ((uint64_t)key << 32) | (uint64_t)(~row);
#else
              (void)dst;
              (void)row;
#endif
            }
          }
        }
      }
      EPI_STAMP(3);
    }
#else
    // 2. compact indices by BLOCK b = (bh, p): the lane's flagged columns of query half bh, one
    //    per pass p (p = 0: its first, jj = 0 if flagged else 1; p = 1: jj = 1 when both are);
    //    blocks in order, lanes in order within a block (n: uniform). A round writes one
    //    9-instruction block per (bh, p) it holds -- usually the two p = 0 blocks, where the
    //    per-column form wrote one per column c with a flagged lane (up to four): the staging is
    //    bound by those ds_write_b128 (profiles/r4/ab/epilogue_phases.jsonl). The jj choice is a
    //    lane-mask v_cndmask per value (a C select of two array elements would become a
    //    dynamically indexed array in scratch).
    int idx[4];
    bool inb[4];
    int n = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const bool f0 = (colm >> ((b >> 1) * 2)) & 1u, f1 = (colm >> ((b >> 1) * 2 + 1)) & 1u;
      inb[b] = (b & 1) ? (f0 && f1) : (f0 || f1);
      const uint64_t bc = __ballot(inb[b]);
      idx[b] = n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bc >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bc, 0u));
      n += __popcll(bc);
    }
    const uint32_t wst = (uint32_t)(uintptr_t)(smem + QP_LDS + QP_PARAM + wave * QP_STG_WAVE);
    const uint32_t wmeta = wst + QP_STG_COLS * 128;
    uint64_t* cand = A->e.cand;
    const int64_t ld_cand = A->e.ld_cand;
    const int slots = A->e.slots;
    const int64_t rbase = A->e.idx_base + T.c0;
#pragma unroll 1
    for (int r0 = 0; r0 < n; r0 += QP_STG_COLS) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int s = idx[b] - r0;
        if (inb[b] && s >= 0 && s < QP_STG_COLS) {
          const int bh = b >> 1;
          const f32x4_t(&ac0)[4][2] = acc_of(0, bh);
          const f32x4_t(&ac1)[4][2] = acc_of(1, bh);
          // jj = 1 for lanes whose first flagged column of this half is its second (or p = 1)
          const bool j1 = (b & 1) || !((colm >> (bh * 2)) & 1u);
          const uint64_t jm = __ballot(j1);
          const int ql = bh * 128 + wb * 32 + (j1 ? 16 : 0) + fr_;
          const float qs = vsel(jm, q4[bh * 2 + 1], q4[bh * 2]);
          const float th = vsel(jm, t4[bh * 2 + 1], t4[bh * 2]);
          const f32x4_t meta = {__builtin_bit_cast(float, (uint32_t)(ql | (g_ << 8))), qs, th, 0.f};
#ifndef EBT_ABL_STAGE_META_ONLY
          lds_put_col(wst + s * 128, vsel4(jm, ac0[0][1], ac0[0][0]), vsel4(jm, ac0[1][1], ac0[1][0]),
                      vsel4(jm, ac0[2][1], ac0[2][0]), vsel4(jm, ac0[3][1], ac0[3][0]),
                      vsel4(jm, ac1[0][1], ac1[0][0]), vsel4(jm, ac1[1][1], ac1[1][0]),
                      vsel4(jm, ac1[2][1], ac1[2][0]), vsel4(jm, ac1[3][1], ac1[3][0]),
                      wmeta + s * 16, meta);
#else  // ablation builds only: the staging's record write alone (values left stale)
          asm volatile("ds_write_b128 %0, %1" : : "v"(wmeta + s * 16), "v"(meta) : "memory");
#endif
        }
      }
      EPI_STAMP(2);
      // 3. lane: staged column s, values u * 8 .. u * 8 + 7 = half ah = u >> 1, accumulators
      // i0, i0 + 1 (i0 = (u & 1) * 2), rows il0 .. il0 + 3 and il0 + 16 .. il0 + 19
      const int nr = n - r0 < QP_STG_COLS ? n - r0 : QP_STG_COLS;
      const int s = lane_ >> 2, u = lane_ & 3;
#ifdef EBT_ABL_HIT_STAGE_ONLY  // ablation builds only: the staging without the processing
      if (s < 0) {
#else
      if (s < nr) {
#endif
        f32x4_t m, v0, v1;
        lds_staged(wmeta + s * 16, wst + s * 128 + u * 32, m, v0, v1);
        const uint32_t mw = __builtin_bit_cast(uint32_t, m[0]);
        const int ql = (int)(mw & 255u), g = (int)(mw >> 8);
        const float qs = m[1], th = m[2];
        const int il0 = (u >> 1) * 128 + wa * 64 + (u & 1) * 32 + 4 * g;
        f32x4_t c0 = {1.f, 1.f, 1.f, 1.f}, c1 = c0;
        if constexpr (!SIMPLE) lds_f32x4x2(lcs + il0, c0, c1);
        float v[8];
        uint32_t hb = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float a = k < 4 ? v0[k] : v1[k - 4];
          v[k] = SIMPLE ? a * qs : a * qs * (k < 4 ? c0[k] : c1[k - 4]);
          const int il = il0 + (k < 4 ? k : 12 + k);
          hb |= (v[k] >= th && (full || T.c0 + il < n_rows) ? 1u : 0u) << k;
        }
        if (hb) {
          const uint32_t base = lds_add_rtn(lcnt + ql, (uint32_t)__popc(hb));
          uint64_t* dst = cand + (T.q0 + ql) * ld_cand + T.ct * slots;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const uint32_t p = base + (uint32_t)__popc(hb & ((1u << k) - 1u));
            if (((hb >> k) & 1u) && p < (uint32_t)slots) {
              const uint32_t row = (uint32_t)(rbase + il0 + (k < 4 ? k : 12 + k));
              // opaque key: otherwise the compiler hoists a 64-bit constant of f2key's zero case
              // out of the tile loop, and at the K-loop's register peak spills it
              uint32_t key = f2key_select(v[k]);
              asm volatile("" : "+v"(key));
#ifndef EBT_ABL_NO_HIT_STORES  // ablation builds only (timing of the epilogue's stores)
              dst[p] = ((uint64_t)key << 32) | (uint64_t)(~row);
#else
              (void)dst;
              (void)row;
#endif
            }
          }
        }
      }
      EPI_STAMP(3);
    }
#endif
  };
  auto store_quadrant = [&](const QpTile& T, const f32x4_t (&acc)[4][2], int ah, int bh) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int ql = bh * 128 + wb * 32 + jj * 16 + fr_;
      const float qs = lds_f32(lqs + ql);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int il = ah * 128 + wa * 64 + i * 16 + 4 * (lane_ >> 4);
        const float4 cs = lds_float4(lcs + il);
        const f32x4_t& a = acc[i][jj];
        const float v[4] = {a[0] * qs * cs.x, a[1] * qs * cs.y, a[2] * qs * cs.z, a[3] * qs * cs.w};
        float* srow = A->e.S + (T.q0 + ql) * A->e.ld_s;
        const int64_t i0 = T.c0 + il;
        if (i0 + 3 < n_rows) {
          *(float4*)(srow + i0) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (i0 + r < n_rows) srow[i0 + r] = v[r];
        }
      }
    }
  };
  // pool mode: max over the 64 rows (ah, wa) of each query: 4 accumulators x 4 values in the
  // lane, then the 4 lanes of the same fr_ (lane ^ 16, ^ 32); rows past n_rows are skipped
  // (a lead tile, T.ct < lead: its full tile of scores is also stored, the filter's values, for
  // ebt's lead-hit extraction once the threshold is known -- the filter then skips those rows)
  auto pool_quadrant = [&](const QpTile& T, const f32x4_t (&acc)[4][2], int ah, int bh) {
    const bool lead_tile = T.ct < A->lead;  // uniform
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int ql = bh * 128 + wb * 32 + jj * 16 + fr_;
      const float qs = lds_f32(lqs + ql);
      float mx = -__builtin_inff();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int il = ah * 128 + wa * 64 + i * 16 + 4 * (lane_ >> 4);
        const float4 cs = lds_float4(lcs + il);
        const f32x4_t& a = acc[i][jj];
        const float v[4] = {a[0] * qs * cs.x, a[1] * qs * cs.y, a[2] * qs * cs.z, a[3] * qs * cs.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (T.c0 + il + r < n_rows) mx = fmaxf(mx, v[r]);
        if (lead_tile)
          *(float4*)(A->S2 + (T.q0 + ql) * A->ld_s2 + T.c0 + il) = make_float4(v[0], v[1], v[2], v[3]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if ((lane_ >> 4) == 0) A->e.S[(T.q0 + ql) * A->e.ld_s + T.ct * 4 + ah * 2 + wa] = mx;
    }
  };


    // ---- epilogue of `cur` (every wave passed the last phase's barrier after its last LDS
    // read of the tile's parameters' previous contents; the parameters landed: counted waits)
    if constexpr (EPI == EPI_POOL) {
      pool_quadrant(cur, acc0, 0, 0);
      pool_quadrant(cur, acc1, 0, 1);
      pool_quadrant(cur, acc2, 1, 1);
      pool_quadrant(cur, acc3, 1, 0);
    } else if constexpr (FILTER) {
      if (!A->cscale && cur.c0 + QP_TILE <= n_rows) filter_tile(cur, std::true_type{});
      else filter_tile(cur, std::false_type{});
    } else {
      store_quadrant(cur, acc0, 0, 0);
      store_quadrant(cur, acc1, 0, 1);
      store_quadrant(cur, acc2, 1, 1);
      store_quadrant(cur, acc3, 1, 0);
    }
    // every wave is past its reads of lcnt / lqs / lth / lcs (LDS-only barrier: the hit and
    // score stores need not drain here)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (FILTER) {
      if (tid_ < QP_TILE) {
        const uint32_t c = lcnt[tid_];
        const int64_t q = cur.q0 + tid_;
#ifndef EBT_ABL_NO_COUNT_STORES
        A->e.counts[q * A->e.ld_counts + cur.ct] = (uint8_t)(c < 255u ? c : 255u);
        if (c > (uint32_t)A->e.slots) A->e.ovf[q] = 1;
#else
        (void)q;
#endif
        lcnt[tid_] = 0u;
      }
    }
    EPI_STAMP(4);
    if (last) break;
    L += n_x;
    issue_params(tile_at(L));
  }
#undef QP2_KTILE
  // the last tile restaged its own first K-tiles: drain before the LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef EBT_EPI_STAMP
  if (EPI == EPI_FILTER && (tid & 63) == 0 && g_epi) {
    const unsigned long long* e =
        (const unsigned long long*)(smem + QP_LDS + QP_PARAM + QP_STG) + wave * 8;
    unsigned long long* o = g_epi + ((int64_t)bid * 8 + wave) * 8;
    for (int i = 0; i < 8; ++i) o[i] = e[i];
  }
#endif
#ifdef EBT_WALK_STAMP
  if (EPI == EPI_FILTER && tid == 0 && g_walk) {
    const int t = walk_t < WALK_MAX - 1 ? walk_t : WALK_MAX - 1;
    unsigned long long* o = g_walk + ((int64_t)bid * WALK_MAX + t) * 2;
    o[0] = ~0ull;
    o[1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
#ifdef EBT_CLOCK_STAMP
  if (EPI == EPI_FILTER && tid == 0 && g_stamps) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = g_stamps + 4 * (int64_t)bid;
    o[0] = st_t0;
    o[1] = st_r0;
    o[2] = t1;
    o[3] = r1;
  }
#endif
}

#ifdef EBT_EPI_STAMP
extern "C" int ebt_debug_epi_stamps(unsigned long long* buf) {
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_epi), &buf, sizeof(buf)), "hipMemcpyToSymbol");
}
#endif
#ifdef EBT_WALK_STAMP
extern "C" int ebt_debug_walk_stamps(unsigned long long* buf) {
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_walk), &buf, sizeof(buf)), "hipMemcpyToSymbol");
}
#endif
#ifdef EBT_CLOCK_STAMP
extern "C" int ebt_debug_clock_stamps(unsigned long long* buf) {
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)),
                   "hipMemcpyToSymbol");
}
#endif


// Kernel choice: batches padded to a multiple of 256 queries take the 256 x 256 quadrant-phase
// kernel; smaller batches (B_pad = 128) the 128 x 128 one. Measured alternatives that lost on
// MI355X ("screening GEMM"): a 4-slot ring with k32 slices, one barrier per phase
// with two barriers (qp), a persistent one-workgroup-per-CU walk of the same tiles, and a
// 4-wave 128 x 128-per-wave tile (LDS-DMA issue cost with one wave per SIMD).
// Compute units of the current device (the persistent grid size), cached per device: relaxed
// atomics (every writer stores the same value, so concurrent first calls from the serving
// threads race on nothing). The library's other process-wide state (api.hip: the LDS-attribute
// cache and the event pool; rccl_comm.hip: the RCCL entry points) is behind locks.
static int64_t n_cus() {
  static std::atomic<int64_t> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int64_t v = cache[dev].load(std::memory_order_relaxed);
  if (v == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    v = cus;
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

// The persistent grid's workgroups (one per CU) -- the planner's round size (api.hip)
int64_t gemm_cus() { return n_cus(); }

template <int EPI>
static int launch_gemm(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                       int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                       const float* cscale, const EpiArgs& e, hipStream_t stream,
                       int64_t cstride = 0, int lead = 0, float* S2 = nullptr,
                       int64_t ld_s2 = 0) {
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
    // persistent: one 148 KiB-LDS workgroup per CU walks ceil(tiles / CUs) tiles
    int64_t G = nwg < n_cus() ? nwg : n_cus();
#ifdef EBT_GRID_OVERRIDE
    // ablation build only: EBT_QP_GRID=<workgroups> runs the persistent grid on fewer CUs (the
    // GEMM's rate on a CU subset, for overlap experiments); never in the shipped library
    if (const char* g = getenv("EBT_QP_GRID")) {
      const int64_t v = atoll(g) & ~7LL;
      if (v >= 8 && v < G) G = v;
    }
#endif
    const int ktiles = d_pad / 64;
    dim3 grid((unsigned)G), block(QP_THREADS);
    auto k = (ktiles & 1) ? (img_dtype == EBT_BF16 ? screen_gemm_qp2_kernel<true, EPI, true>
                                                   : screen_gemm_qp2_kernel<false, EPI, true>)
                          : (img_dtype == EBT_BF16 ? screen_gemm_qp2_kernel<true, EPI, false>
                                                   : screen_gemm_qp2_kernel<false, EPI, false>);
    set_max_lds((const void*)k, QP_LDS_TOTAL);
    QpArgs a{};
    a.Q = Q;
    a.C = C;
    a.ld_img = ld_img;
    a.n_rows = n_rows;
    a.qscale = qscale;
    a.cscale = cscale;
    a.cstride = cstride;
    a.n_qtiles = n_qtiles;
    a.n_ctiles = (int)n_ctiles;
    a.ktiles = ktiles;
    const int per_group = QP_GROUP_C * n_qtiles;
    a.pg_log2 = (per_group & (per_group - 1)) == 0 ? __builtin_ctz((unsigned)per_group) : -1;
    a.lead = lead;
    a.S2 = S2;
    a.ld_s2 = ld_s2;
    a.e = e;
    hipEvent_t ev0, ev1;
    if (take_launch_events(&ev0, &ev1))   // a timed launch: the events ride on the dispatch
      hipExtLaunchKernelGGL(k, grid, block, QP_LDS_TOTAL, stream, ev0, ev1, 0, a);
    else
      hipLaunchKernelGGL(k, grid, block, QP_LDS_TOTAL, stream, a);
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
  set_max_lds((const void*)k, lds);
  hipEvent_t ev0, ev1;
  if (take_launch_events(&ev0, &ev1))
    hipExtLaunchKernelGGL(k, grid, block, lds, stream, ev0, ev1, 0, Q, C, (int64_t)ld_img,
                          n_rows, n_qtiles, n_ctiles, d_pad / GBK, qscale, cscale, e);
  else
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
// With lead > 0 the sample's first `lead` tiles are the catalog's first lead tiles and the rest
// start there (tile p >= lead at row lead * 256 + (p - lead) * cstride), and the lead tiles' f32
// scores -- the values the filter epilogue would test -- go to lead_scores[q][0, 256 lead)
// (row pitch ld_lead).
int screen_gemm_pool(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                     int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                     const float* cscale, int64_t cstride, float* pooled, int64_t ld_pooled,
                     hipStream_t stream, int64_t lead, float* lead_scores, int64_t ld_lead) {
  int rc = check_gemm_args("screen_gemm_pool", qimg, B_pad, cimg, n_rows, d_pad, ld_img,
                           img_dtype, qscale, cscale);
  if (rc) return rc;
  if (!pooled || B_pad % QP_TILE != 0 || n_rows % QP_TILE != 0 || cstride < QP_TILE ||
      ld_pooled < n_rows / 64 || lead < 0 || lead > n_rows / QP_TILE ||
      (lead > 0 && (!lead_scores || ld_lead < lead * QP_TILE || ld_lead % 4 != 0 ||
                    ((uintptr_t)lead_scores & 15)))) {
    set_error("screen_gemm_pool: bad arguments");
    return EBT_EINVAL;
  }
  EpiArgs e{};
  e.S = pooled;
  e.ld_s = ld_pooled;
  return launch_gemm<EPI_POOL>(qimg, B_pad, cimg, n_rows, d_pad, ld_img, img_dtype, qscale,
                               cscale, e, stream, cstride, (int)lead, lead_scores, ld_lead);
}



int64_t filter_group_rows(int64_t B_pad) { return B_pad % QP_TILE == 0 ? QP_TILE : GBM; }

// tiles per workgroup of one filter launch before it is split (EBT_FILTER_TPW in the
// environment at start, ebt_filter_split at run time; 0 = never split)
static std::atomic<int64_t>& filter_tpw_flag() {
  static std::atomic<int64_t> v([] {
    const char* s = getenv("EBT_FILTER_TPW");
    return s ? (int64_t)atoll(s) : (int64_t)32;
  }());
  return v;
}
static int64_t filter_tiles_per_wg() { return filter_tpw_flag().load(std::memory_order_relaxed); }

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

// Rows per part of a long filter screen (0: not split): at most filter_tiles_per_wg() tiles per
// workgroup, whole rounds. The persistent walk keeps its XCD's workgroups on neighbouring tiles
// only while they stay in step, and they drift apart over a long launch (tools/walk_stamp.py: a
// whole C5 launch, 2034 tiles per workgroup, ends with a median in-flight spread of 48 tiles
// instead of 32 and +45 % of modelled L2 miss traffic); every launch starts them together. The
// pipeline (api.hip filter_screen) launches a screen of more than 1.5 parts as consecutive
// parts over the same groups: the same tiles, hits and counts as one launch.
int64_t filter_split_rows(int64_t B_pad, int64_t n_rows) {
  const int64_t tpw = filter_tiles_per_wg();
  const int64_t qt = B_pad / QP_TILE;
  if (tpw <= 0 || B_pad % QP_TILE != 0 || qt < 1 || n_cus() % qt != 0) return 0;
  const int64_t round_rows = (n_cus() / qt) * QP_TILE;
  const int64_t cap_rows = tpw * round_rows;
  if (n_rows <= cap_rows + cap_rows / 2) return 0;
  const int64_t parts = (n_rows + cap_rows - 1) / cap_rows;
  return (n_rows / parts + round_rows - 1) / round_rows * round_rows;
}

}  // namespace ebt

extern "C" int64_t ebt_filter_split(int64_t tiles_per_workgroup) {
  if (tiles_per_workgroup < 0) return ebt::filter_tpw_flag().load();
  return ebt::filter_tpw_flag().exchange(tiles_per_workgroup);
}
