// Streaming top-k' select: one HBM pass over each score row.
//
// Replaces `movie_scores.loc[unrated].sort_values(ascending=False)[:k]` (lib.py:55; pandas
// core/series.py:3706-3716, a full O(N log N) argsort) with a single streaming pass per row
// segment. One 256-thread workgroup owns a (row, segment); it streams the segment in 4096-entry
// tiles (16 values per lane, float4 loads, the next two tiles prefetched into registers) and
// keeps a candidate buffer in LDS:
//   * an entry is admitted when its order-preserving key >= thr (initially every valid entry),
//     tested as a float compare against thr's float form; admission is wave-aggregated: the
//     lane counts' prefix from one ballot per count bit, one LDS atomic per wave and tile;
//   * when the buffer cannot take another full tile, it is compacted to exactly its k' best
//     entries by an adaptive-range radix select (11-bit histograms over the live [min, max] of
//     the 64-bit composite (key, ~index), so hot bins stay spread out), and thr rises to the
//     k'-th key -- after the first couple of tiles almost nothing passes the filter;
//   * at the end the k' survivors are bitonic-sorted in LDS by (value desc, index asc).
// Composites are unique (indices are), so the result is deterministic: exactly the k' largest
// (value, -index) pairs. NaN and -inf (masked / excluded) entries have key 0 and never enter.
#include "common.h"

namespace ebt {

constexpr int STHREADS = 256;
constexpr int SE = 16;                  // values per lane per tile
constexpr int STILE = STHREADS * SE;    // 4096 entries per tile
constexpr int SHIST = 2048;             // histogram bins (11 bits)
constexpr int KPRIME_MAX = 4096;

__host__ __device__ inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Buffer room beside the k' kept entries, in quarter tiles (> 4: a full tile's admissions must
// fit without compacting every tile; exactly one tile of room measured 1.7x slower). 1.25 tiles
// keep the LDS of k' <= ~500 at ~51 KiB, three workgroups per CU: 4096 x 1M, k' = 200 in
// 3.13 ms against 3.45 with two tiles of room and two workgroups per CU (-DEBT_SEL_ROOM=8
// -DEBT_SEL_WGS=2): each workgroup's per-tile admission is latency-bound, so more of them per
// CU shortens the pass.
#ifndef EBT_SEL_ROOM
#define EBT_SEL_ROOM 5
#endif
#ifndef EBT_SEL_WGS
#define EBT_SEL_WGS 3
#endif

struct SelLayout {
  int cap;       // buffer capacity (entries)
  int kpp;       // next pow2 >= kprime
  size_t off_key, off_idx, off_keep, off_misc, bytes;
};

__host__ __device__ inline SelLayout sel_layout(int kprime) {
  SelLayout L;
  L.cap = kprime + EBT_SEL_ROOM * (STILE / 4);
  L.kpp = next_pow2(kprime);
  L.off_key = 0;
  L.off_idx = L.off_key + 4 * (size_t)L.cap;
  L.off_keep = L.off_idx + 4 * (size_t)L.cap;
  L.off_keep = (L.off_keep + 15) & ~(size_t)15;
  size_t keep_bytes = 8 * (size_t)L.kpp;
  if (keep_bytes < 4 * (size_t)SHIST) keep_bytes = 4 * (size_t)SHIST;  // aliased with hist
  L.off_misc = L.off_keep + keep_bytes;
  L.bytes = L.off_misc + 256;
  return L;
}

__device__ __forceinline__ uint64_t comp_of(uint32_t key, uint32_t idx) {
  return ((uint64_t)key << 32) | (uint64_t)(~idx);
}

// block-wide min / max of u64 (all threads get the result). red: >= 8 u64 of LDS.
__device__ __forceinline__ void block_minmax_u64(uint64_t& mn, uint64_t& mx, uint64_t* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int w = threadIdx.x >> 6;
  lds_barrier();
  if ((threadIdx.x & 63) == 0) {
    red[w] = mn;
    red[4 + w] = mx;
  }
  lds_barrier();
  mn = red[0];
  mx = red[4];
#pragma unroll
  for (int i = 1; i < 4; ++i) {
    mn = red[i] < mn ? red[i] : mn;
    mx = red[4 + i] > mx ? red[4 + i] : mx;
  }
}

// theta = the rank-th largest composite among the n buffer entries (1 <= rank <= n).
__device__ uint64_t select_rank(const uint32_t* bkey, const uint32_t* bidx, int n, int rank,
                                uint32_t* hist, uint64_t* red, uint32_t* misc) {
  const int tid = threadIdx.x;
  uint64_t lo = 0, hi = ~0ull;
  int r = rank;
  for (int iter = 0; iter < 16; ++iter) {
    uint64_t mn = ~0ull, mx = 0;
    for (int i = tid; i < n; i += STHREADS) {
      const uint64_t c = comp_of(bkey[i], bidx[i]);
      if (c >= lo && c <= hi) {
        mn = c < mn ? c : mn;
        mx = c > mx ? c : mx;
      }
    }
    block_minmax_u64(mn, mx, red);
    if (mn == mx) return mn;
    const uint64_t span = mx - mn;
    const int bits = 64 - __builtin_clzll(span);
    const int shift = bits > 11 ? bits - 11 : 0;
#pragma unroll
    for (int j = 0; j < SHIST / STHREADS; ++j) hist[tid * (SHIST / STHREADS) + j] = 0;
    lds_barrier();
    for (int i = tid; i < n; i += STHREADS) {
      const uint64_t c = comp_of(bkey[i], bidx[i]);
      if (c >= mn && c <= mx) atomicAdd(&hist[(uint32_t)((c - mn) >> shift)], 1u);
    }
    lds_barrier();
    // suffix scan: thread t owns bins [8t, 8t+8)
    uint32_t hv[SHIST / STHREADS];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < SHIST / STHREADS; ++j) {
      hv[j] = hist[tid * (SHIST / STHREADS) + j];
      s += hv[j];
    }
    uint32_t x = s;  // inclusive suffix within the wave (lanes >= me)
    const int lane = tid & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t y = __shfl_down(x, o, 64);
      if (lane + o < 64) x += y;
    }
    uint32_t* wtot = misc + 8;
    if (lane == 0) wtot[tid >> 6] = x;
    lds_barrier();
    uint32_t above = x - s;
    for (int w2 = (tid >> 6) + 1; w2 < 4; ++w2) above += wtot[w2];
    if (above < (uint32_t)r && (uint32_t)r <= above + s) {
      uint32_t cum = above;
      for (int j = SHIST / STHREADS - 1; j >= 0; --j) {
        if (cum + hv[j] >= (uint32_t)r) {
          misc[0] = tid * (SHIST / STHREADS) + j;
          misc[1] = cum;
          break;
        }
        cum += hv[j];
      }
    }
    lds_barrier();
    const uint32_t b = misc[0];
    r -= (int)misc[1];
    lds_barrier();  // misc reused next iteration
    lo = mn + ((uint64_t)b << shift);
    const uint64_t w = (shift >= 64) ? ~0ull : ((1ull << shift) - 1);
    hi = (mx - lo) < w ? mx : lo + w;
    if (shift == 0) return lo;
  }
  return lo;  // not reached for unique composites
}

// Keep exactly min(rank, n) best entries: buffer -> keep (unordered) -> buffer[0..).
// Returns theta (rank-th composite). n > rank required.
__device__ uint64_t compact(uint32_t* bkey, uint32_t* bidx, int n, int rank, uint64_t* keep,
                            uint32_t* hist, uint64_t* red, uint32_t* misc) {
  const uint64_t theta = select_rank(bkey, bidx, n, rank, hist, red, misc);
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid == 0) misc[2] = 0;
  lds_barrier();  // hist (aliased with keep) is dead from here
  for (int base = 0; base < n; base += STHREADS) {
    const int i = base + tid;
    uint64_t c = 0;
    bool take = false;
    if (i < n) {
      c = comp_of(bkey[i], bidx[i]);
      take = c >= theta;
    }
    const uint64_t m = __ballot(take);
    if (m) {
      uint32_t wb = 0;
      if (lane == 0) wb = atomicAdd(&misc[2], (uint32_t)__popcll(m));
      wb = __shfl(wb, 0, 64);
      if (take) {
        const uint32_t pos = wb + (uint32_t)__popcll(m & ((1ull << lane) - 1));
        keep[pos] = c;
      }
    }
  }
  lds_barrier();
  for (int i = tid; i < rank; i += STHREADS) {
    const uint64_t c = keep[i];
    bkey[i] = (uint32_t)(c >> 32);
    bidx[i] = ~(uint32_t)c;
  }
  lds_barrier();
  return theta;
}

// Descending bitonic sort of keep[0..P) (P power of two).
__device__ void bitonic_desc(uint64_t* keep, int P) {
  const int tid = threadIdx.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (P >> 1); t += STHREADS) {
        // stride is a power of two: 2 stride (t / stride) + t % stride without a division
        const int lo = ((t & ~(stride - 1)) << 1) | (t & (stride - 1));
        const int hi = lo + stride;
        const uint64_t a = keep[lo], b = keep[hi];
        const bool desc = (lo & size) == 0;
        if ((a < b) == desc) {
          keep[lo] = b;
          keep[hi] = a;
        }
      }
      lds_barrier();
    }
  }
}

// TPI tiles per iteration: the next TPI tiles are loaded while the current TPI are admitted
// one tile at a time (the buffer check and the admission per tile as for TPI = 1), so a
// workgroup keeps TPI x 16 KiB in flight (TPI = 2: 1-2 % faster than 1; 3 is slower).
template <bool HAS_IDX, bool VEC, int TPI>
__global__ __launch_bounds__(STHREADS, EBT_SEL_WGS) void select_topk_kernel(
    const float* __restrict__ vals, const int64_t* __restrict__ idxs, int64_t ld, int64_t n,
    int64_t seg_len, int64_t idx_base, int kprime, float* __restrict__ out_vals,
    int64_t* __restrict__ out_idx, int64_t ld_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const SelLayout Lo = sel_layout(kprime);
  uint32_t* bkey = (uint32_t*)(smem + Lo.off_key);
  uint32_t* bidx = (uint32_t*)(smem + Lo.off_idx);
  uint64_t* keep = (uint64_t*)(smem + Lo.off_keep);
  uint32_t* hist = (uint32_t*)(smem + Lo.off_keep);  // aliased
  uint64_t* red = (uint64_t*)(smem + Lo.off_misc);
  uint32_t* misc = (uint32_t*)(smem + Lo.off_misc + 64);

  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t row = blockIdx.x;
  const int seg = blockIdx.y;
  const int64_t s0 = (int64_t)seg * seg_len;
  int64_t s1 = s0 + seg_len;
  s1 = s1 < n ? s1 : n;
  const float* vrow = vals + row * ld;
  const int64_t* irow = HAS_IDX ? idxs + row * ld : nullptr;

  if (tid == 0) misc[3] = 0;  // nbuf counter
  lds_barrier();
  uint32_t thr = 1;
  int nbuf = 0;
  // float form of "key >= thr" for the per-tile fast test: keys up to f2key(-FLT_MAX) admit
  // every finite value (-inf and NaN have key 0); above that key2f(thr) is a float (or a NaN
  // that admits nothing, as no float has such a key)
  auto thr_f = [](uint32_t t) {
    return t <= 0x00800000u ? -3.402823466e38f : key2f(t);
  };
  float tf = thr_f(thr);

  constexpr int TE = SE * TPI;  // values per lane in flight
  float cur[TE], nxt[TE];
  int64_t curi[HAS_IDX ? TE : 1], nxti[HAS_IDX ? TE : 1];
  // tiles t0, t0 + STILE, ... (TPI of them); element e of tile h at
  // t0 + h * STILE + (e >> 2) * (STHREADS * 4) + tid * 4 + (e & 3)
  auto load_tiles = [&](int64_t t0, float* v, int64_t* ix) {
#pragma unroll
    for (int j = 0; j < TE / 4; ++j) {
      const int64_t p = t0 + (j / (SE / 4)) * STILE + (j % (SE / 4)) * (STHREADS * 4) + tid * 4;
      if constexpr (VEC) {
        if (p < s1) {
          const float4 f = *(const float4*)(vrow + p);
          v[4 * j + 0] = f.x;
          v[4 * j + 1] = f.y;
          v[4 * j + 2] = f.z;
          v[4 * j + 3] = f.w;
          if constexpr (HAS_IDX) {
            const longlong2 a = *(const longlong2*)(irow + p);
            const longlong2 b = *(const longlong2*)(irow + p + 2);
            ix[4 * j + 0] = a.x;
            ix[4 * j + 1] = a.y;
            ix[4 * j + 2] = b.x;
            ix[4 * j + 3] = b.y;
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * j + e] = -__builtin_inff();
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t pe = p + e;
          v[4 * j + e] = pe < s1 ? vrow[pe] : -__builtin_inff();
          if constexpr (HAS_IDX) ix[4 * j + e] = pe < s1 ? irow[pe] : -1;
        }
      }
    }
  };

#if defined(EBT_SEL_DIAG)
  float dsum = 0.f;
#endif
  const int64_t ntiles = (s1 - s0 + STILE - 1) / STILE;
  const int64_t niter = (ntiles + TPI - 1) / TPI;
  if (ntiles > 0) load_tiles(s0, cur, curi);
  for (int64_t it = 0; it < niter; ++it) {
    const int64_t i0 = s0 + it * (int64_t)(TPI * STILE);
    if (it + 1 < niter) load_tiles(i0 + TPI * STILE, nxt, nxti);
#pragma unroll
    for (int h = 0; h < TPI; ++h) {
      const int64_t t0 = i0 + h * STILE;
      if (t0 >= s1) break;  // uniform: past the segment's last tile
#if defined(EBT_SEL_DIAG) && EBT_SEL_DIAG == 1
      // diagnostic build only: the stream alone (no admission, no barrier)
#pragma unroll
      for (int e = 0; e < SE; ++e) dsum += cur[h * SE + e];
      continue;
#elif defined(EBT_SEL_DIAG) && EBT_SEL_DIAG == 2
      // diagnostic build only: nothing is admitted, the per-tile test and barrier stay
      thr = 0xffffffffu;
      tf = __builtin_inff();
#endif
      if (nbuf + STILE > Lo.cap) {
        const uint64_t theta = compact(bkey, bidx, nbuf, kprime, keep, hist, red, misc);
        nbuf = kprime;
        const uint32_t tau = (uint32_t)(theta >> 32);
        thr = HAS_IDX ? tau : tau + 1u;
        tf = thr_f(thr);
        if (tid == 0) misc[3] = (uint32_t)nbuf;
        lds_barrier();
      }
      // fast test: once the threshold has risen, few tiles have a value to admit; a wave with
      // none skips the admission (a superset test: entries past the segment read -inf, excluded
      // (idx < 0) ones are dropped below)
      bool any = false;
#pragma unroll
      for (int e = 0; e < SE; ++e) any |= cur[h * SE + e] >= tf;
      if (__ballot(any) != 0ull) {
        // admission: a lane's admitted values as a bit mask, a wave scan of the lane counts and
        // ONE LDS atomic per wave for the wave's total; each lane then writes its own entries.
        // The threshold only rises at a compaction, so between two of them a wave admits a few
        // values in most tiles: a ballot + atomic per value slot cost ~16 LDS round trips per
        // wave and tile, the whole difference between this kernel and its bare stream.
        // The buffer order differs from a per-slot admission; the result does not (compaction
        // and the final sort order unique composites).
        // f2key(v) >= thr  <=>  v >= tf for every v (thr_f above; NaN compares false), so the
        // mask needs no key: a float compare and the segment end in 32 bits
        const int lim = (int)(s1 - t0 < STILE ? s1 - t0 : STILE);
        uint32_t msk = 0;
#pragma unroll
        for (int e = 0; e < SE; ++e) {
          const int o = (e >> 2) * (STHREADS * 4) + tid * 4 + (e & 3);
          bool take = o < lim && cur[h * SE + e] >= tf;
          if constexpr (HAS_IDX) take = take && curi[h * SE + e] >= 0;
          msk |= (take ? 1u : 0u) << e;
        }
        // exclusive prefix of the lane counts (0..16, five bits) from one ballot per bit: no
        // cross-lane LDS traffic (a shuffle scan is six dependent ds_bpermute round trips)
        const uint32_t cnt = (uint32_t)__popc(msk);
        uint32_t excl = 0, tot = 0;
#pragma unroll
        for (int bit = 0; bit < 5; ++bit) {
          const uint64_t bm = __ballot((cnt >> bit) & 1u);
          const uint32_t below = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
          excl += below << bit;
          tot += (uint32_t)__popcll(bm) << bit;
        }
        if (tot) {
          uint32_t wb = 0;
          if (lane == 0) wb = atomicAdd(&misc[3], tot);
          wb = (uint32_t)__builtin_amdgcn_readfirstlane((int)wb);  // lane 0: exec is full here
          uint32_t pos = wb + excl;
#pragma unroll
          for (int e = 0; e < SE; ++e) {
            if ((msk >> e) & 1u) {
              bkey[pos] = f2key(cur[h * SE + e]);
              if constexpr (HAS_IDX) bidx[pos] = (uint32_t)curi[h * SE + e];
              else bidx[pos] = (uint32_t)t0 + (uint32_t)((e >> 2) * (STHREADS * 4) + tid * 4 + (e & 3));
              ++pos;
            }
          }
        }
      }
      lds_barrier();
      nbuf = (int)misc[3];
    }
    if (it + 1 < niter) {
#pragma unroll
      for (int e = 0; e < TE; ++e) {
        cur[e] = nxt[e];
        if constexpr (HAS_IDX) curi[e] = nxti[e];
      }
    }
  }

#if defined(EBT_SEL_DIAG)
  if (dsum == 1.2345f) misc[3] = 0;  // keeps the diagnostic stream live
#endif
  // final: exactly min(kprime, nbuf) survivors, sorted
  int nk = nbuf;
  if (nbuf > kprime) {
    compact(bkey, bidx, nbuf, kprime, keep, hist, red, misc);
    nk = kprime;
  }
  const int P = Lo.kpp;
  for (int i = tid; i < P; i += STHREADS) keep[i] = i < nk ? comp_of(bkey[i], bidx[i]) : 0ull;
  lds_barrier();
  bitonic_desc(keep, P);
  float* ov = out_vals + row * ld_out + (int64_t)seg * kprime;
  int64_t* oi = out_idx + row * ld_out + (int64_t)seg * kprime;
  for (int i = tid; i < kprime; i += STHREADS) {
    const uint64_t c = keep[i];
    const uint32_t key = (uint32_t)(c >> 32);
    if (key == 0u) {
      ov[i] = -__builtin_inff();
      oi[i] = -1;
    } else {
      ov[i] = key2f(key);
      const uint32_t ix = ~(uint32_t)c;
      oi[i] = HAS_IDX ? (int64_t)(int32_t)ix : idx_base + (int64_t)ix;
    }
  }
}

size_t select_lds_bytes(int kprime) { return sel_layout(kprime).bytes; }

// tiles in flight per workgroup: two for a plain score row; one when int64 row ids travel with
// the values (three times the registers per value)
#ifndef EBT_SEL_TPI
#define EBT_SEL_TPI 2
#endif
#define SEL_TPI(H) ((H) ? 1 : EBT_SEL_TPI)

static int select_launch(const float* vals, const int64_t* idx, int64_t ld, int64_t B,
                         int64_t n, int64_t idx_base, int32_t kprime, int32_t segs,
                         float* out_vals, int64_t* out_idx, int64_t ld_out, hipStream_t stream) {
  if (!vals || !out_vals || !out_idx || B < 0 || n < 0 || ld < n || segs < 1 || kprime < 1 ||
      kprime > KPRIME_MAX || ld_out < (int64_t)segs * kprime || n >= 0x7fffffffLL ||
      segs > 65535 || B > 0x7fffffffLL) {
    set_error("ebt_select_topk: bad arguments (B=%lld n=%lld ld=%lld kprime=%d segs=%d)",
              (long long)B, (long long)n, (long long)ld, kprime, segs);
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  int64_t seg_len = ceil_div(n > 0 ? n : 1, segs);
  seg_len = (seg_len + 3) & ~(int64_t)3;
  const bool vec = (ld % 4 == 0) && (((uintptr_t)vals & 15) == 0) &&
                   (!idx || ((uintptr_t)idx & 15) == 0);
  const size_t lds = select_lds_bytes(kprime);
  dim3 grid((unsigned)B, (unsigned)segs), block(STHREADS);
#define EBT_SEL_LAUNCH(H, V)                                                                  \
  set_max_lds((const void*)select_topk_kernel<H, V, SEL_TPI(H)>, (int)lds);                    \
  hipLaunchKernelGGL((select_topk_kernel<H, V, SEL_TPI(H)>), grid, block, lds, stream, vals, \
                     idx, ld, n, seg_len, idx_base, (int)kprime, out_vals, out_idx, ld_out)
  if (idx) {
    if (vec) { EBT_SEL_LAUNCH(true, true); }
    else { EBT_SEL_LAUNCH(true, false); }
  } else {
    if (vec) { EBT_SEL_LAUNCH(false, true); }
    else { EBT_SEL_LAUNCH(false, false); }
  }
#undef EBT_SEL_LAUNCH
  return launch_check("select_topk_kernel");
}

int select_topk(const float* vals, const int64_t* idx, int64_t ld, int64_t B, int64_t n,
                int64_t idx_base, int32_t kprime, int32_t segs, float* out_vals,
                int64_t* out_idx, int64_t ld_out, hipStream_t stream) {
  return select_launch(vals, idx, ld, B, n, idx_base, kprime, segs, out_vals, out_idx, ld_out,
                       stream);
}

// ---------------------------------------------------------------------------------------------
// Fused screen, between segments. merge_segment: query b's list (its k' best so far, fv/fi
// sorted) plus the hits the last filter GEMM left in its per-group slots (screen_gemm.hip,
// EpiArgs) -> the k' best of both, written back over fv/fi. One workgroup per query: a block
// scan of the group counts places every hit, excluded rows (lib.py:48,55: binary search of the
// GLOBAL row in the query's sorted exclusion list) are dropped, and the union is sorted in LDS as
// u64 composites (key desc, row asc -- the order select_topk_kernel produces). About 2k'
// entries per query for a doubling segment. A slot overflow (count > SLOTS) or more hits than
// the LDS holds sets ovf[b]: the query's certificate becomes -1 and it is rerun unfused.
// ---------------------------------------------------------------------------------------------
constexpr int MERGE_MAX = 16384;  // LDS entries (128 KiB)
// dynamic LDS a merge workgroup may take: 160 KiB less the kernel's static LDS (its wsum / flag
// words and the bitonic sort's: 288 bytes on gfx950 -- read from the kernel, merge_lds_dyn())
constexpr size_t MERGE_LDS_CU = 160 * 1024;
constexpr int MERGE_DEFER = 1 << 4;  // ovf bit: the query waits for the full-size merge

static int merge_entries(int kprime) {
  int P = 2;
  while (P < kprime + 4 * kprime + 2048 && P < MERGE_MAX) P <<= 1;
  return P;
}

// One query's merge (the whole workgroup). tier 1 (P_max = a small LDS buffer, several
// workgroups per CU) defers a query whose union does not fit (ovf bit MERGE_DEFER, nothing
// written); tier 2 (the full buffer) merges a deferred one.
__device__ __forceinline__ void merge_segment_one(
    int64_t b, float* __restrict__ fv, int64_t* __restrict__ fi, int kprime,
    const uint64_t* __restrict__ cand, int64_t ld_cand, int slots,
    const uint8_t* __restrict__ counts, int64_t ld_counts, int n_groups, int P_max,
    int64_t row_offset, const int64_t* __restrict__ eo, const int64_t* __restrict__ er,
    int* __restrict__ ovf, int tier, uint64_t* mkeep, int* wsum, int& flag) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ovf_in = tier ? ovf[b] : 0;
  const uint8_t* cr = counts + b * ld_counts;
  const uint64_t* cb = cand + b * ld_cand;
  if (tid == 0) flag = 0;
  // this thread's groups: [g0, g0 + per16), per16 a multiple of 16, their counts read as
  // 16-byte vectors (one memory round trip, not one per group)
  const int per16 = ((n_groups + STHREADS - 1) / STHREADS + 15) & ~15;
  const int g0 = tid * per16;
  const int g1 = g0 + per16 < n_groups ? g0 + per16 : n_groups;
  const bool vec_counts = ((uintptr_t)cr & 15) == 0;
  auto counts16 = [&](int gv, uint32_t (&w)[4]) {  // counts of groups gv .. gv + 15 (0 past g1)
    if (vec_counts && gv + 16 <= g1) {
      const uint4 v = *(const uint4*)(cr + gv);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[q] = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int g = gv + q * 4 + e;
          w[q] |= (g < g1 ? (uint32_t)cr[g] : 0u) << (8 * e);
        }
      }
    }
  };
  int mine = 0;
  bool over = false;
  for (int gv = g0; gv < g1; gv += 16) {
    uint32_t w[4];
    counts16(gv, w);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int c = (w[e >> 2] >> (8 * (e & 3))) & 255;
      over |= c > slots;
      mine += c < slots ? c : slots;
    }
  }
  // block exclusive scan
  int incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < STHREADS / 64; ++w) {
    base += w < wave ? wsum[w] : 0;
    total += wsum[w];
  }
  const int room = P_max - kprime;
  if (tier == 1 && total > room) {  // block-uniform
    if (tid == 0) ovf[b] = ovf_in | MERGE_DEFER;
    return;
  }
  if (total > room) over = true;
  // the hits' slot positions: gbase[g] = the first position of group g's hits (exclusive prefix
  // over groups, LDS, u16: positions past `room` are dropped anyway), gbase[n_groups] = total
  uint16_t* gbase = (uint16_t*)(mkeep + P_max);
  {
    int run = base + incl - mine;  // this thread's exclusive prefix
    for (int gv = g0; gv < g1; gv += 16) {
      uint32_t w[4];
      counts16(gv, w);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int g = gv + e;
        const int c = (w[e >> 2] >> (8 * (e & 3))) & 255;
        if (g < g1) gbase[g] = (uint16_t)(run < 65535 ? run : 65535);
        run += c < slots ? c : slots;
      }
    }
    if (tid == 0) gbase[n_groups] = (uint16_t)(total < 65535 ? total : 65535);
  }
  __syncthreads();
  // every hit h < min(total, room): its group by binary search over gbase, four loads in flight
  // per thread before any is used
  const int nh = total < room ? total : room;
  const int64_t elo = eo ? eo[b] : 0, ehi = eo ? eo[b + 1] : 0;
  for (int h0 = tid; h0 < nh; h0 += 4 * STHREADS) {
    uint64_t comp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int h = h0 + u * STHREADS;
      comp[u] = 0ull;
      if (h < nh) {
        int lo = 0, hi = n_groups;  // the last g with gbase[g] <= h
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if ((int)gbase[mid] <= h) lo = mid;
          else hi = mid;
        }
        comp[u] = cb[(int64_t)lo * slots + (h - (int)gbase[lo])];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int h = h0 + u * STHREADS;
      if (h >= nh) continue;
      uint64_t cu = comp[u];
      if (ehi > elo) {
        const int64_t gr = (int64_t)(~(uint32_t)cu) + row_offset;
        int64_t lo = elo, hi = ehi;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (er[mid] < gr) lo = mid + 1;
          else hi = mid;
        }
        if (lo < ehi && er[lo] == gr) cu = 0ull;
      }
      mkeep[kprime + h] = cu;
    }
  }
  for (int i = tid; i < kprime; i += STHREADS) {
    const uint32_t key = f2key(fv[b * kprime + i]);
    const int64_t ix = fi[b * kprime + i];
    mkeep[i] = (key != 0u && ix >= 0) ? (((uint64_t)key << 32) | (uint64_t)(~(uint32_t)ix)) : 0ull;
  }
  if (over) flag = 1;
  const int used = kprime + nh;
  // A sorted list (the streaming select's, or this kernel's own output) merges with the hits
  // sorted alone: a bitonic sort of the next power of two >= nh, then a merge-path merge of the
  // two descending runs into the first kprime outputs -- instead of re-sorting list + hits
  // (the bitonic sort of P >= kprime + nh entries is LDS-bandwidth bound: ~16 B per entry and
  // stage). Anything else (a partitioned list) takes the full sort.
  int Ph = 2;
  while (Ph < nh) Ph <<= 1;
  __syncthreads();
  int bad = 0;
  for (int i = tid; i + 1 < kprime; i += STHREADS) bad |= mkeep[i] < mkeep[i + 1] ? 1 : 0;
  const bool sorted_list = !__syncthreads_or(bad) && kprime + Ph <= P_max;
  if (sorted_list) {
    uint64_t* hb = mkeep + kprime;
    for (int i = nh + tid; i < Ph; i += STHREADS) hb[i] = 0ull;
    __syncthreads();
    if (nh > 1) bitonic_desc(hb, Ph);
    // outputs [o0, o1) of this thread: the merge path's split at diagonal o0 (A = the list,
    // B = the hits, both descending; A first on equal composites -- only empty 0s can be equal)
    const int per = (kprime + STHREADS - 1) / STHREADS;
    const int o0 = tid * per < kprime ? tid * per : kprime;
    const int o1 = o0 + per < kprime ? o0 + per : kprime;
    if (o0 < o1) {
      int lo = o0 > nh ? o0 - nh : 0, hi = o0 < kprime ? o0 : kprime;
      while (lo < hi) {  // the number of list entries among the first o0 outputs
        const int mid = (lo + hi) >> 1;
        if (mkeep[mid] >= hb[o0 - 1 - mid]) lo = mid + 1;
        else hi = mid;
      }
      int i = lo, j = o0 - lo;
      for (int o = o0; o < o1; ++o) {
        const uint64_t a = i < kprime ? mkeep[i] : 0ull;
        const uint64_t c = j < nh ? hb[j] : 0ull;
        const bool take_a = j >= nh || (i < kprime && a >= c);
        const uint64_t comp = take_a ? a : c;
        i += take_a ? 1 : 0;
        j += take_a ? 0 : 1;
        const uint32_t key = (uint32_t)(comp >> 32);
        fv[b * kprime + o] = key ? key2f(key) : -__builtin_inff();
        fi[b * kprime + o] = key ? (int64_t)(~(uint32_t)comp) : -1;
      }
    }
  } else {
    int P = 2;
    while (P < used) P <<= 1;
    for (int i = used + tid; i < P; i += STHREADS) mkeep[i] = 0ull;
    __syncthreads();
    bitonic_desc(mkeep, P);
    for (int i = tid; i < kprime; i += STHREADS) {
      const uint64_t comp = mkeep[i];
      const uint32_t key = (uint32_t)(comp >> 32);
      fv[b * kprime + i] = key ? key2f(key) : -__builtin_inff();
      fi[b * kprime + i] = key ? (int64_t)(~(uint32_t)comp) : -1;
    }
  }
  if (tid == 0 && (flag || tier == 2)) ovf[b] = (ovf_in & ~MERGE_DEFER) | (flag ? 1 : 0);
}

// tier 0 / 1: one workgroup per query. tier 2: a grid of at most one workgroup per CU (the
// full LDS buffer) walks the queries and merges only those tier 1 deferred -- a handful per
// batch -- instead of launching B full-LDS workgroups that mostly exit at once (64 dispatch
// rounds of them at 16384 queries per merge).
__global__ __launch_bounds__(STHREADS) void merge_segment_kernel(
    float* __restrict__ fv, int64_t* __restrict__ fi, int kprime,
    const uint64_t* __restrict__ cand, int64_t ld_cand, int slots,
    const uint8_t* __restrict__ counts, int64_t ld_counts, int n_groups, int P_max,
    int64_t row_offset,
    const int64_t* __restrict__ eo, const int64_t* __restrict__ er, int* __restrict__ ovf,
    int tier, int64_t B) {
  extern __shared__ __attribute__((aligned(16))) uint64_t mkeep[];
  __shared__ int wsum[STHREADS / 64];
  __shared__ int flag;
  if (tier != 2) {
    merge_segment_one(blockIdx.x, fv, fi, kprime, cand, ld_cand, slots, counts, ld_counts,
                      n_groups, P_max, row_offset, eo, er, ovf, tier, mkeep, wsum, flag);
    return;
  }
  for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
    if (!(ovf[b] & MERGE_DEFER)) continue;  // uniform
    merge_segment_one(b, fv, fi, kprime, cand, ld_cand, slots, counts, ld_counts, n_groups,
                      P_max, row_offset, eo, er, ovf, tier, mkeep, wsum, flag);
    __syncthreads();  // LDS and the block's shared words are reused by the next query
  }
}

size_t merge_lds_dyn() {
  static size_t dyn = [] {
    hipFuncAttributes a{};
    size_t st = 1024;  // a safe static estimate if the attributes cannot be read
    if (hipFuncGetAttributes(&a, (const void*)merge_segment_kernel) == hipSuccess)
      st = (a.sharedSizeBytes + 15) & ~(size_t)15;
    return MERGE_LDS_CU - st;
  }();
  return dyn;
}

static int merge_segment_part(float* fv, int64_t* fi, int64_t B, int kprime,
                              const uint64_t* cand, int64_t ld_cand, int slots,
                              const uint8_t* counts, int64_t ld_counts, int64_t n_groups,
                              int64_t row_offset, const int64_t* eo, const int64_t* er, int* ovf,
                              hipStream_t st, double expect_hits) {
  const int P_max = merge_entries(kprime);
  // LDS: the P entries, then the u16 group positions (n_groups + 1)
  const size_t gb_bytes = ((size_t)(n_groups + 1) * 2 + 15) & ~(size_t)15;
  if ((size_t)P_max * 8 + gb_bytes > merge_lds_dyn()) {
    set_error("merge_segment: %lld groups do not fit the LDS", (long long)n_groups);
    return EBT_EINVAL;
  }
  set_max_lds((const void*)merge_segment_kernel, (int)((size_t)P_max * 8 + gb_bytes));
  // with an expected hit count (and an ovf array for the deferral bit): a first pass with room
  // for 3x the expected hits, at 4+ workgroups per CU instead of 1, then the full-size pass for
  // the (rare) queries that did not fit
  int P_small = 2;
  if (expect_hits > 0.0 && ovf) {
    const char* mv = getenv("EBT_MERGE_MARGIN");  // tests: 0 defers (nearly) every query
    const double margin = mv ? atof(mv) : 3.0;
    const double want = (double)kprime + margin * expect_hits + 256.0;
    while (P_small < want && P_small < P_max) P_small <<= 1;
  } else {
    P_small = P_max;
  }
  if (P_small < P_max) {
    hipLaunchKernelGGL(merge_segment_kernel, dim3((unsigned)B), dim3(STHREADS),
                       (size_t)P_small * 8 + gb_bytes, st, fv, fi, kprime, cand, ld_cand, slots,
                       counts, ld_counts, (int)n_groups, P_small, row_offset, eo, er, ovf, 1, B);
    int rc = launch_check("merge_segment_kernel");
    if (rc) return rc;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    const int64_t g2 = B < cus ? B : cus;
    hipLaunchKernelGGL(merge_segment_kernel, dim3((unsigned)g2), dim3(STHREADS),
                       (size_t)P_max * 8 + gb_bytes, st, fv, fi, kprime, cand, ld_cand, slots,
                       counts, ld_counts, (int)n_groups, P_max, row_offset, eo, er, ovf, 2, B);
    return launch_check("merge_segment_kernel");
  }
  hipLaunchKernelGGL(merge_segment_kernel, dim3((unsigned)B), dim3(STHREADS),
                     (size_t)P_max * 8 + gb_bytes, st, fv, fi, kprime, cand, ld_cand, slots,
                     counts, ld_counts, (int)n_groups, P_max, row_offset, eo, er, ovf, 0, B);
  return launch_check("merge_segment_kernel");
}

int64_t merge_block_max_groups(int kprime);

// More groups than one block merge can index (its u16 group positions share the LDS with the
// P_max entries): merge them in consecutive parts of whole 16-group blocks. Each part merges
// the list with the hits of its groups, so the parts together give the k' best of the list and
// every hit -- the same (key, row) composites, hence the same list, as one merge.
int merge_segment(float* fv, int64_t* fi, int64_t B, int kprime, const uint64_t* cand,
                  int64_t ld_cand, int slots, const uint8_t* counts, int64_t ld_counts,
                  int64_t n_groups,
                  int64_t row_offset, const int64_t* eo, const int64_t* er, int* ovf,
                  hipStream_t st, double expect_hits) {
  if (B < 0 || B > 0x7fffffffLL || kprime < 1 || kprime > KPRIME_MAX || n_groups < 1 ||
      n_groups > 0x7fffffffLL || ld_counts < n_groups ||
      ld_cand < n_groups * slots) {
    set_error("merge_segment: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const int64_t part = merge_block_max_groups(kprime) & ~(int64_t)15;
  for (int64_t g0 = 0; g0 < n_groups; g0 += part) {
    const int64_t ng = n_groups - g0 < part ? n_groups - g0 : part;
    const int rc = merge_segment_part(fv, fi, B, kprime, cand + g0 * slots, ld_cand, slots,
                                      counts + g0, ld_counts, ng, row_offset, eo, er, ovf, st,
                                      expect_hits * (double)ng / (double)n_groups);
    if (rc) return rc;
  }
  return EBT_OK;
}

// ---------------------------------------------------------------------------------------------
// The same merge with ONE WAVE per query (4 queries per workgroup, no block barriers) while
// k' + hits <= WTOP_N: the wave holds the union in registers (WTOP_E composites per lane) and
// selects with binary searches on the 32-bit key (a second one on the row part only when the
// key at the cut is tied), counting with ballot popcounts -- uniform (scalar) loops, 32-bit
// compares. The result is written PARTITIONED, not sorted (nothing downstream needs more):
//   [0, k-1) the k-1 best (any order), [k-1] the k-th best,
//   [k, n-1) the rest (any order),     [n-1] the smallest kept,   [n, k') empty (-inf / -1)
// with n = min(k', valid entries). Every consumer reads the list as a set plus those two
// positions: kth_threshold (the k-th), rescore (the k-th and the k'-th), the next merge (the
// k'-th). The block merge and the streaming select write fully sorted lists, a special case.
// Input either the per-group hit slots of the filter GEMM plus the list fv/fi, or (the fused
// screen's pilot) a dense score row with implicit rows idx_base + j and no list.
// ---------------------------------------------------------------------------------------------
constexpr int WTOP_E = 16;            // composites per lane
constexpr int WTOP_N = 64 * WTOP_E;   // union size per query
constexpr int WMERGE_K = 512;         // largest k'
constexpr int WMERGE_Q = STHREADS / 64;
constexpr int WCNT = 4;               // 16-byte count loads per lane: n_groups <= 64 * 64

// E: the leading entries per lane that can be nonzero (the union fills entry j = c / 64 of
// lane c % 64 in order, so every entry past ceil(used / 64) is 0 and counts nowhere)
template <int E>
__device__ __forceinline__ int wave_count_ge(const uint32_t (&kx)[WTOP_E], uint32_t t) {
  int c = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) c += __popcll(__ballot(kx[j] >= t));
  return c;
}

// The cut c (a composite) with exactly `want` entries of x >= c (1 <= want <= valid entries;
// composites are unique). lo: a key with count(key >= lo) >= want; hi: the largest key.
template <int E>
__device__ __forceinline__ uint64_t wave_cut(const uint64_t (&x)[WTOP_E],
                                             const uint32_t (&kx)[WTOP_E], int want, uint32_t lo,
                                             uint32_t hi) {
  uint32_t l = __builtin_amdgcn_readfirstlane(lo), h = __builtin_amdgcn_readfirstlane(hi);
  if (l > h) l = h;
  while (l < h) {  // largest t with count(key >= t) >= want
    const uint32_t mid = l + ((h - l) >> 1) + ((h - l) & 1u);  // l + ceil((h - l) / 2)
    if (wave_count_ge<E>(kx, mid) >= want) l = mid;
    else h = mid - 1;
  }
  const uint32_t t = l;
  int gt = 0, eq = 0;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    gt += __popcll(__ballot(kx[j] > t));
    eq += __popcll(__ballot(kx[j] == t));
  }
  const int need = want - gt;  // 1 <= need <= eq entries with key == t
  uint64_t u = 0;
  if (need < eq) {  // a tie at the cut: order the tied entries by row (rare)
    uint64_t l2 = 0, h2 = 0xffffffffull;  // largest u with count(key == t, low >= u) >= need
    while (l2 < h2) {
      const uint64_t mid = l2 + ((h2 - l2 + 1) >> 1);
      int c = 0;
#pragma unroll
      for (int j = 0; j < E; ++j)
        c += __popcll(__ballot(kx[j] == t && (uint32_t)x[j] >= (uint32_t)mid));
      if (c >= need) l2 = mid;
      else h2 = mid - 1;
    }
    u = l2;
  }
  return ((uint64_t)t << 32) | u;
}

// smallest nonzero composite >= cut over the wave (uniform result)
template <int E>
__device__ __forceinline__ uint64_t wave_min_at_least(const uint64_t (&x)[WTOP_E], uint64_t cut) {
  uint64_t m = ~0ull;
#pragma unroll
  for (int j = 0; j < E; ++j) m = (x[j] != 0ull && x[j] >= cut && x[j] < m) ? x[j] : m;
#ifdef EBT_MERGE_SHFL_RED
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t v = ((uint64_t)(uint32_t)__shfl_xor((int)(m >> 32), o, 64) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)m, o, 64);
    m = v < m ? v : m;
  }
  return m;
#else
  // the smallest high half, then the smallest low half among the lanes holding it
  const uint32_t mh = wave_min_u32((uint32_t)(m >> 32));
  const uint32_t ml = wave_min_u32((uint32_t)(m >> 32) == mh ? (uint32_t)m : 0xffffffffu);
  return ((uint64_t)mh << 32) | ml;
#endif
}

// The k' largest of the wave's composites x (0 = empty), written partitioned at k (see above)
// to ov/oi[0..kprime).
// Returns the value it wrote to position k-1 (uniform): the k-th best, -inf when fewer than k.
template <int E>
__device__ float wave_topk_write(const uint64_t (&x)[WTOP_E], int kprime, int k, float* ov,
                                 int64_t* oi, int lane, uint32_t key_lo) {
  float kth = -__builtin_inff();
  uint32_t kx[WTOP_E];
  int nvalid = 0;
  uint32_t kmax = 0u, kmin = 0xffffffffu;  // over the valid entries
#pragma unroll
  for (int j = E; j < WTOP_E; ++j) kx[j] = 0u;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    kx[j] = (uint32_t)(x[j] >> 32);
    nvalid += __popcll(__ballot(x[j] != 0ull));
    kmax = max(kmax, kx[j]);
    if (x[j] != 0ull) kmin = min(kmin, kx[j]);
  }
#ifdef EBT_MERGE_SHFL_RED
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
    kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o, 64));
  }
#else
  kmax = wave_max_u32(kmax);
  kmin = wave_min_u32(kmin);
#endif
  // every valid entry has key >= kmin, so count(key >= kmin) = nvalid >= want: a valid lower
  // end for the first bisection, ~8 steps shorter than 1 when the list started empty
  key_lo = key_lo > kmin ? key_lo : kmin;
  const int want = nvalid < kprime ? nvalid : kprime;
  const uint64_t below = (1ull << lane) - 1ull;
  if (want > 0) {
    // the kept set S = {x >= cw_cut} (want entries), its smallest cw; the top kk = min(k, want)
    // A = {x >= ck_cut}, its smallest ck (the kk-th best)
    const uint64_t cw_cut = wave_cut<E>(x, kx, want, key_lo > 1u ? key_lo : 1u, kmax);
    const uint64_t cw = wave_min_at_least<E>(x, cw_cut);
    const int kk = k < want ? k : want;
    uint64_t ck = cw;
    if (kk < want) {
      const uint64_t ck_cut = wave_cut<E>(x, kx, kk, (uint32_t)(cw_cut >> 32), kmax);
      ck = wave_min_at_least<E>(x, ck_cut);
    }
    if (kk == k) kth = key2f((uint32_t)(ck >> 32));
    int na = 0, nb = kk;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const uint64_t v = x[j];
      const bool inA = v > ck;                                  // the kk-1 best
      const bool inB = v != 0ull && v >= cw && v < ck && v != cw;  // between
      const uint64_t ma = __ballot(inA), mb = __ballot(inB);
      // (selects, not branches: the same precedence as an if / else chain)
      const int pa = na + __popcll(ma & below), pb = nb + __popcll(mb & below);
      const int pc = (v == ck && v != 0ull) ? kk - 1 : ((v == cw && v != 0ull) ? want - 1 : -1);
      const int pos = inA ? pa : (inB ? pb : pc);
      if (pos >= 0) {
        ov[pos] = key2f((uint32_t)(v >> 32));
        oi[pos] = (int64_t)(~(uint32_t)v);
      }
      na += __popcll(ma);
      nb += __popcll(mb);
    }
  }
  for (int i = want + lane; i < kprime; i += 64) {
    ov[i] = -__builtin_inff();
    oi[i] = -1;
  }
  return kth;
}

// The row-sharded step's floor entries (ebt_floor_pack's [w + 1] layout) from the wave merge's
// union, fused into the screen's last merge: the w largest keys of the union (= the w largest
// of the final list's k best, w <= k <= k'), keys above the w-th first, then as many equal to it
// as fit, -inf past them, then eps. The w-th key by bisection on ballot counts, as floor_pack.
template <int E>
__device__ void wave_floor_write(const uint64_t (&x)[WTOP_E], int w, float* dst, int lane,
                                 float eps) {
  uint32_t kx[E];
  int nvalid = 0;
  uint32_t kmax = 0u, kmin = 0xffffffffu;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    kx[j] = (uint32_t)(x[j] >> 32);
    nvalid += __popcll(__ballot(kx[j] != 0u));
    kmax = max(kmax, kx[j]);
    if (kx[j] != 0u) kmin = min(kmin, kx[j]);
  }
  kmax = wave_max_u32(kmax);
  kmin = wave_min_u32(kmin);
  uint32_t t = 0u;
  if (nvalid > w) {
    auto count_ge = [&](uint32_t v) {
      int c = 0;
#pragma unroll
      for (int j = 0; j < E; ++j) c += __popcll(__ballot(kx[j] >= v));
      return c;
    };
    uint32_t lo = kmin, hi = kmax;  // count_ge(kmin) = nvalid >= w
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1) + 1u;
      if (count_ge(mid) >= w) lo = mid;
      else hi = mid - 1u;
    }
    t = lo;
  }
  int base = 0;
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const bool pick = kx[j] != 0u && (pass == 0 ? (nvalid <= w || kx[j] > t)
                                                  : (nvalid > w && kx[j] == t));
      const uint64_t m = __ballot(pick);
      const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (pick && pos < w) dst[pos] = key2f(kx[j]);
      base += __popcll(m);
    }
  }
  for (int j = (base < w ? base : w) + lane; j < w; j += 64) dst[j] = -__builtin_inff();
  if (lane == 0) dst[w] = eps;
}

// (double)kth - 2 eps rounded down to a float (the segment threshold / speculative check value)
__device__ __forceinline__ float kth_minus_2eps_down(float kth, float eps) {
  const double t = (double)kth - 2.0 * (double)eps;
  float f = (float)t;
  if ((double)f > t && f == f && f != -__builtin_inff()) {  // one float step down
    const uint32_t u = __float_as_uint(f);
    f = f == 0.f ? -__uint_as_float(1u) : __uint_as_float(f > 0.f ? u - 1u : u + 1u);
  }
  return f;
}

#ifdef EBT_MERGE_STAMP
// Diagnostic build only: the shader cycles of each phase of a query's wave merge (hit mode):
// [0] list + counts loaded, [1] slot indices of the hits (LDS), [2] hits gathered, [3] the
// selection and the list written; g_mstamp[4 b ..] (vector stores; nothing else reads them).
__device__ unsigned long long* g_mstamp;
extern "C" int ebt_debug_merge_stamps(unsigned long long* buf) {
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_mstamp), &buf, sizeof(buf)), "hipMemcpyToSymbol");
}
#define MST(i) ms[i] = __builtin_amdgcn_s_memtime()
#else
#define MST(i)
#endif
template <bool DENSE>
__global__ __launch_bounds__(STHREADS, 4) void merge_wave_kernel(
    float* __restrict__ fv, int64_t* __restrict__ fi, int64_t B, int kprime, int k,
    const uint64_t* __restrict__ cand, int64_t ld_cand, int slots,
    const uint8_t* __restrict__ counts, int64_t ld_counts, int n_groups,
    const float* __restrict__ dense, int64_t ld_dense, int n_dense, int64_t idx_base,
    int64_t row_offset, const int64_t* __restrict__ eo, const int64_t* __restrict__ er,
    int* __restrict__ ovf, const float* __restrict__ veps, const float* __restrict__ vspec,
    float* __restrict__ fout, int fw, const float* __restrict__ feps, float* __restrict__ tout,
    const float* __restrict__ tin, const float* __restrict__ teps, int64_t B_pad) {
  __shared__ uint64_t stage[WMERGE_Q][WTOP_N];  // the union
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b = (int64_t)blockIdx.x * WMERGE_Q + w;
  if (b >= B) {
    if (tout && b < B_pad && lane == 0) tout[b] = __builtin_inff();  // padding: no hits
    return;
  }
  uint64_t* U = stage[w];
#ifdef EBT_MERGE_STAMP
  unsigned long long ms[5] = {0, 0, 0, 0, 0};
  MST(4);
#endif
  uint64_t x[WTOP_E];
  bool over = false;
  uint32_t key_lo = 1u;  // the new k'-th key is >= the list's k'-th key
  int used_n = WTOP_N;    // union entries (x[j] of lane l is entry l + 64 j; 0 past them)
  if constexpr (DENSE) {
    used_n = n_dense < WTOP_N ? n_dense : WTOP_N;
    const float* row = dense + b * ld_dense;
#pragma unroll
    for (int j = 0; j < WTOP_E; ++j) {
      const int c = lane + 64 * j;
      const uint32_t key = c < n_dense ? f2key(row[c]) : 0u;
      x[j] = key ? (((uint64_t)key << 32) | (uint64_t)(~(uint32_t)(idx_base + c))) : 0ull;
    }
  } else {
    const int64_t elo = eo ? eo[b] : 0, ehi = eo ? eo[b + 1] : 0;
    auto excluded = [&](uint64_t comp) {
      const int64_t gr = (int64_t)(~(uint32_t)comp) + row_offset;
      int64_t lo = elo, hi = ehi;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (er[mid] < gr) lo = mid + 1;
        else hi = mid;
      }
      return lo < ehi && er[lo] == gr;
    };
    key_lo = f2key(fv[b * kprime + kprime - 1]);
    // the list (U[0..kprime) below) and the hit counts are loaded together, before any of
    // them is used: one memory round trip instead of one per 64 list entries
    constexpr int LPL = WMERGE_K / 64;
    float lv[LPL];
    int64_t li[LPL];
#pragma unroll
    for (int u = 0; u < LPL; ++u) {
      const int i = lane + 64 * u;
      if (64 * u < kprime) {  // uniform
        lv[u] = i < kprime ? fv[b * kprime + i] : -__builtin_inff();
        li[u] = i < kprime ? fi[b * kprime + i] : -1;
      }
    }
    // the hits: U[kprime..), lane l owning groups [l*per, (l+1)*per), per a multiple of 16 so
    // its counts arrive as up to WCNT independent 16-byte loads (ld_counts is a multiple of 16)
    const uint8_t* cr = counts + b * ld_counts;
    const uint64_t* cb = cand + b * ld_cand;
    const int per = ((n_groups + 63) / 64 + 15) & ~15;
    const int g0 = lane * per;
    const int nv = per / 16;  // count vectors in use (uniform)
    uint4 cv4[WCNT];
#pragma unroll
    for (int v = 0; v < WCNT; ++v) {
      const int g = g0 + 16 * v;
      cv4[v] = (v < nv && g < n_groups) ? *(const uint4*)(cr + g) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < LPL; ++u) {
      const int i = lane + 64 * u;
      if (64 * u < kprime && i < kprime) {
        const uint32_t key = f2key(lv[u]);
        U[i] = (key != 0u && li[u] >= 0)
                   ? (((uint64_t)key << 32) | (uint64_t)(~(uint32_t)li[u])) : 0ull;
      }
    }
    auto cnt_at = [&](int v, int e) -> int {  // count of group g0 + 16 v + e (0 past the end)
      const uint32_t w4 = e < 4 ? cv4[v].x : e < 8 ? cv4[v].y : e < 12 ? cv4[v].z : cv4[v].w;
      const int c = (int)((w4 >> (8 * (e & 3))) & 0xffu);
      return g0 + 16 * v + e < n_groups ? c : 0;
    };
    int mine = 0;
#pragma unroll
    for (int v = 0; v < WCNT; ++v) {
      if (v >= nv) break;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = cnt_at(v, e);
        over |= c > slots;
        mine += c < slots ? c : slots;
      }
    }
    MST(0);
#ifdef EBT_MERGE_SLOT_LOOP
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int m = __shfl(incl, 63, 64);
#else
    const int incl = (int)wave_scan_add_u32((uint32_t)mine);
    const int m = __builtin_amdgcn_readlane(incl, 63);
#endif
    if (kprime + m > WTOP_N) over = true;
#ifndef EBT_MERGE_SLOT_LOOP
    // the hits without a per-lane loop over them: each group with hits marks its first hit's
    // position h0 (relative to kprime) with ((g + 1) << 16) | h0 -- increasing with h0 -- so that
    // an inclusive max scan over the positions gives every hit position h its group g and its
    // slot h - h0; the wave scans 64 positions at a time and issues each hit's load at once.
    // The same slots in the same order as the per-group loop below.
    const int mh = kprime + m < WTOP_N ? m : WTOP_N - kprime;
    uint32_t* M = (uint32_t*)(U + kprime);  // markers, in the hits' own LDS (rewritten below)
#pragma unroll
    for (int u = 0; u < WTOP_E; ++u) {
      const int h = u * 64 + lane;
      if (u * 64 < mh && h < mh) M[h] = 0u;
    }
    {
      int r = incl - mine;
#pragma unroll
      for (int v = 0; v < WCNT; ++v) {
        if (v >= nv) break;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          int c = cnt_at(v, e);
          c = c < slots ? c : slots;
          if (c > 0 && r < mh) M[r] = ((uint32_t)(g0 + 16 * v + e + 1) << 16) | (uint32_t)r;
          r += c;
        }
      }
    }
    MST(1);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    {
      uint64_t comp[WTOP_E];
      uint32_t carry = 0u;
#pragma unroll
      for (int u = 0; u < WTOP_E; ++u) {
        const int h = u * 64 + lane;
        if (u * 64 < mh) {  // uniform
          uint32_t mk = h < mh ? M[h] : 0u;
          mk = max(wave_scan_max_u32(mk), carry);
          carry = __builtin_amdgcn_readlane(mk, 63);
          const int64_t g = (int64_t)(mk >> 16) - 1;
          const int p = h - (int)(mk & 0xffffu);
          comp[u] = h < mh ? cb[g * slots + p] : 0ull;
        }
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // exclusions (lib.py:48,55): each hit's GLOBAL row looked up in the query's sorted
      // exclusion segment, a lane's hits 2 at a time in lockstep -- the segment's length sets a
      // wave-uniform step count, so every step issues those probes together (ceil(log2 L)
      // dependent loads, not one chain per hit). Branchless lower bound: bs advances by half
      // while seg[bs + half] < row; the row is excluded iff it sits at the lower bound.
      constexpr int XE = 2;
      if (ehi > elo && ehi - elo <= 0x7fffffffLL) {
        const int32_t L = (int32_t)(ehi - elo);
        const int64_t* seg = er + elo;
#pragma unroll
        for (int c0 = 0; c0 < WTOP_E; c0 += XE) {
          if (c0 * 64 >= mh) break;  // uniform
          int64_t gr[XE];
          int32_t bs[XE];
#pragma unroll
          for (int u = 0; u < XE; ++u) {
            gr[u] = (int64_t)(~(uint32_t)comp[c0 + u]) + row_offset;
            bs[u] = 0;
          }
          for (int32_t n = L; n > 1;) {
            const int32_t half = n >> 1;
            int64_t pv[XE];
#pragma unroll
            for (int u = 0; u < XE; ++u)
              if ((c0 + u) * 64 < mh) pv[u] = seg[bs[u] + half];
#pragma unroll
            for (int u = 0; u < XE; ++u)
              if ((c0 + u) * 64 < mh) bs[u] = pv[u] < gr[u] ? bs[u] + half : bs[u];
            n -= half;
          }
          int64_t a[XE], nx[XE];
#pragma unroll
          for (int u = 0; u < XE; ++u)
            if ((c0 + u) * 64 < mh) {
              a[u] = seg[bs[u]];
              nx[u] = bs[u] + 1 < L ? seg[bs[u] + 1] : gr[u] - 1;
            }
#pragma unroll
          for (int u = 0; u < XE; ++u) {
            const int h = (c0 + u) * 64 + lane;
            if ((c0 + u) * 64 < mh && h < mh) {
              const bool drop = a[u] < gr[u] ? nx[u] == gr[u] : a[u] == gr[u];
              U[kprime + h] = drop ? 0ull : comp[c0 + u];
            }
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < WTOP_E; ++u) {
          const int h = u * 64 + lane;
          if (u * 64 < mh && h < mh)
            U[kprime + h] = (ehi > elo && excluded(comp[u])) ? 0ull : comp[u];
        }
      }
    }
#else
    // the hits, in two passes: each lane writes the slot index of its hits (LDS only, so the
    // divergent per-group loop costs no memory latency), then the wave loads 64 hits at a time
    int pos = kprime + incl - mine;
    if (mine > 0) {
#pragma unroll
      for (int v = 0; v < WCNT; ++v) {
        if (v >= nv) break;
#pragma unroll 1
        for (int e = 0; e < 16; ++e) {
          int c = cnt_at(v, e);
          c = c < slots ? c : slots;
          const int64_t g = g0 + 16 * v + e;
          for (int p = 0; p < c; ++p, ++pos)
            if (pos < WTOP_N) U[pos] = (uint64_t)(g * slots + p);
        }
      }
    }
    MST(1);
    const int mh = kprime + m < WTOP_N ? m : WTOP_N - kprime;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    {  // every hit load issued before the first is used (mh <= WTOP_N: WTOP_E per lane)
      uint64_t comp[WTOP_E];
#pragma unroll
      for (int u = 0; u < WTOP_E; ++u) {
        const int h = u * 64 + lane;
        if (u * 64 < mh) comp[u] = h < mh ? cb[(int64_t)U[kprime + h]] : 0ull;  // uniform if
      }
#pragma unroll
      for (int u = 0; u < WTOP_E; ++u) {
        const int h = u * 64 + lane;
        if (u * 64 < mh && h < mh)
          U[kprime + h] = (ehi > elo && excluded(comp[u])) ? 0ull : comp[u];
      }
    }
#endif
    MST(2);
    const int used = kprime + m < WTOP_N ? kprime + m : WTOP_N;
    used_n = used;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < WTOP_E; ++j) {
      const int c = lane + 64 * j;
      x[j] = c < used ? U[c] : 0ull;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // entries in use per lane (uniform): the selection's counting loops stop there
  const int ne = (int)((used_n + 63) / 64);
  const float kth =
      ne <= 8 ? wave_topk_write<8>(x, kprime, k, fv + b * kprime, fi + b * kprime, lane, key_lo)
              : wave_topk_write<WTOP_E>(x, kprime, k, fv + b * kprime, fi + b * kprime, lane, key_lo);
  if (fout) {  // the floor entries of the row-sharded step (ebt_floor_pack folded in)
    const float fe = feps ? feps[b] : -__builtin_inff();
    if (ne <= 8) wave_floor_write<8>(x, fw, fout + b * (fw + 1), lane, fe);
    else wave_floor_write<WTOP_E>(x, fw, fout + b * (fw + 1), lane, fe);
  }
  const bool any_over = __ballot(over) != 0ull;
#ifdef EBT_MERGE_STAMP
  MST(3);
  if (!DENSE && lane == 0 && g_mstamp) {
    g_mstamp[4 * b + 0] = ms[0] - ms[4];
    g_mstamp[4 * b + 1] = ms[1] - ms[0];
    g_mstamp[4 * b + 2] = ms[2] - ms[1];
    g_mstamp[4 * b + 3] = ms[3] - ms[2];
  }
#endif
  if (lane == 0) {
    // tout: the next segment's threshold from the list just written (spec_threshold_kernel's
    // RAISE with tin = theta_spec, kth_threshold_kernel's value without), no launch of its own
    if (tout) {
      const float f = kth_minus_2eps_down(kth, teps[b]);
      tout[b] = tin ? (f > tin[b] ? f : tin[b]) : f;  // NaN f keeps theta_spec
    }
    // vspec: the speculative screen's VERIFY on the final list (spec_threshold_kernel,
    // SPEC_VERIFY) fused into the last merge: theta_spec > the k-th - 2 eps (rounded down), a
    // NaN or fewer than k entries fail with 2, as the separate launch would set after the merge
    if (vspec && !(vspec[b] <= kth_minus_2eps_down(kth, veps[b]))) ovf[b] = 2;
    else if (any_over) ovf[b] = 1;
  }
}

bool merge_wave_fits(int kprime) { return kprime <= WMERGE_K; }
// entries the block merge holds (list + hits) for this k'
int merge_block_capacity(int kprime) { return merge_entries(kprime); }
// groups one block merge can index: its LDS holds the P_max entries, then the u16 group
// positions (n_groups + 1, rounded to 16 bytes) -- merge_segment's own limit
int64_t merge_block_max_groups(int kprime) {
  return (int64_t)(merge_lds_dyn() - (size_t)merge_entries(kprime) * 8) / 2 - 8;
}
int64_t merge_wave_max_groups() { return 64 * 16 * WCNT; }
int merge_wave_capacity() { return WTOP_N; }

int merge_segment_wave(float* fv, int64_t* fi, int64_t B, int kprime, int k, const uint64_t* cand,
                       int64_t ld_cand, int slots, const uint8_t* counts, int64_t ld_counts,
                       int64_t n_groups, int64_t row_offset, const int64_t* eo,
                       const int64_t* er, int* ovf, hipStream_t st, const float* veps,
                       const float* vspec, float* fout, int fw, const float* feps,
                       float* tout, const float* tin, const float* teps, int64_t B_pad) {
  if (B < 0 || kprime < 1 || kprime > WMERGE_K || k < 1 || k > kprime || n_groups < 1 ||
      (fout && (fw < 1 || fw > k)) || (tout && (!teps || B_pad < B)) ||
      n_groups > 64 * 16 * WCNT ||
      ld_counts < n_groups || ld_counts % 16 != 0 || ((uintptr_t)counts & 15) ||
      ld_cand < n_groups * slots) {
    set_error("merge_segment_wave: bad arguments");
    return EBT_EINVAL;
  }
  const int64_t nq = tout ? B_pad : B;  // waves past B only write the padding's threshold
  if (nq == 0) return EBT_OK;
  hipLaunchKernelGGL(merge_wave_kernel<false>, dim3((unsigned)ceil_div(nq, WMERGE_Q)),
                     dim3(STHREADS), 0, st, fv, fi, B, kprime, k, cand, ld_cand, slots, counts, ld_counts, (int)n_groups, nullptr,
                     0, 0, 0, row_offset, eo, er, ovf, veps, vspec, fout, fw, feps, tout, tin, teps,
                     B_pad);
  return launch_check("merge_wave_kernel");
}

// Top-k' of a dense score block (n <= WTOP_N columns per row; masked entries -inf): the fused
// screen's pilot rows, straight into the list fv/fi.
int pilot_topk(const float* S, int64_t ld_s, int64_t B, int n, int64_t idx_base, int kprime,
               int k, float* fv, int64_t* fi, hipStream_t st) {
  if (B < 0 || n < 1 || n > WTOP_N || kprime < 1 || kprime > WMERGE_K || k < 1 || k > kprime ||
      ld_s < n) {
    set_error("pilot_topk: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  hipLaunchKernelGGL(merge_wave_kernel<true>, dim3((unsigned)ceil_div(B, WMERGE_Q)),
                     dim3(STHREADS), 0, st, fv, fi, B, kprime, k, nullptr, 0, 1, nullptr, 0, 0, S, ld_s, n, idx_base, 0, nullptr,
                     nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                     nullptr, B);
  return launch_check("merge_wave_kernel");
}

// thr[b] for the next fused segment: the k-th best approx score of query b's list so far minus
// 2 eps[b], rounded down. The list's k-th best only grows, so thr <= T - 2 eps for the FINAL
// k-th best T: a row the filter drops (approx < thr) cannot be in the exact top k -- the
// rescore's certificate covers it as it covers rows below the list's k'-th (rescore.hip).
// Padding queries get +inf (no hits); a list with fewer than k entries gives -inf (keep all).
__global__ void kth_threshold_kernel(const float* __restrict__ vals, int64_t ld, int64_t B,
                                     int64_t B_pad, int k, const float* __restrict__ eps,
                                     float* __restrict__ thr) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    thr[b] = kth_minus_2eps_down(vals[b * ld + k - 1], eps[b]);
  } else if (b < B_pad) {
    thr[b] = __builtin_inff();
  }
}
int kth_threshold(const float* vals, int64_t ld, int64_t B, int64_t B_pad, int k,
                  const float* eps, float* thr, hipStream_t st) {
  hipLaunchKernelGGL(kth_threshold_kernel, dim3((unsigned)ceil_div(B_pad, 256)), dim3(256), 0,
                     st, vals, ld, B, B_pad, k, eps, thr);
  return launch_check("kth_threshold_kernel");
}

// The speculative fused screen (api.hip, run_screen): a threshold theta_spec[b] estimated from a
// sample of the catalog filters the whole catalog in one pass. theta_spec is NOT a proven lower
// bound of T - 2 eps (T = the final list's k-th approx), so it is checked afterwards:
//   RAISE:  thr[b] = max(theta_spec[b], the list's k-th - 2 eps rounded down) for the next
//           segment (the second term is the rigorous kth_threshold value; padding rows +inf);
//   VERIFY: theta_spec[b] > the list's k-th - 2 eps (rounded down) sets ovf[b]: a row the filter
//           dropped might belong to the top k, so the query loses its certificate (-1) and is
//           rerun unfused. A list with fewer than k entries (-inf) or a NaN fails the test too.
//   INIT:   theta_spec[b] = vals[b][k-1] (the sample's j-th best as it is: the check is
//           theta_spec <= T - 2 eps, so no margin is subtracted here); padding rows +inf.
enum { SPEC_RAISE = 0, SPEC_VERIFY = 1, SPEC_INIT = 2 };
__global__ void spec_threshold_kernel(const float* __restrict__ vals, int64_t ld, int64_t B,
                                      int64_t B_pad, int k, const float* __restrict__ eps,
                                      const float* __restrict__ thr_spec, float* __restrict__ thr,
                                      int* __restrict__ ovf, int mode) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (mode == SPEC_INIT) {
    if (b < B_pad) thr[b] = b < B ? vals[b * ld + k - 1] : __builtin_inff();
    return;
  }
  if (b < B) {
    const float f = kth_minus_2eps_down(vals[b * ld + k - 1], eps[b]);
    const float s = thr_spec[b];
    if (mode == SPEC_RAISE) thr[b] = f > s ? f : s;  // NaN f keeps s
    else if (!(s <= f)) ovf[b] = 2;
  } else if (b < B_pad && mode == SPEC_RAISE) {
    thr[b] = __builtin_inff();
  }
}
// theta_spec[b] = the j-th largest of query b's G <= 2048 pooled sample maxima (one wave per
// query; the largest key t with count(key >= t) >= j, by bisection with ballot counts). A 64-row
// subgroup's max is >= x only if one of its rows is, so P(theta_spec > x) <= P(>= j sample rows
// >= x): spec_params' Poisson bound holds for the pooled estimate too. Fewer than j valid maxima
// -> -inf (keep everything: the merge overflows and the query is rerun unfused). E = maxima per
// lane (G <= 64 E): 4 for one shard's sample, up to 32 for the maxima of all shards
// (ebt_pool_kth over the all-gathered samples of a row-sharded catalog).
// Optionally (fv != null) the same wave also starts query b's empty list for the speculative
// screen (fv -inf / fi -1 over k' entries, ovf 0): three memsets fewer per batch.
// With a lead (the speculative screen's sample lead, lead > 0): the wave then takes its query's
// hits among the lead tiles' stored scores at the threshold just found -- what the filter
// epilogue writes for those tiles (screen_gemm.hip filter_tile: the same composites, counts
// and overflow flag), without a launch of its own.
struct LeadArgs {
  const float* s;
  int64_t ld;
  int lead;
  uint64_t* cand;
  int64_t ld_cand;
  int slots;
  uint8_t* counts;
  int64_t ld_counts;
};
// The lead tiles' scores are loaded LEAD_LB tiles at a time (4 x LEAD_LB floats per lane), every
// load of a batch issued before the first is used: one memory round trip per batch instead of
// one per tile. The first batch can be issued earlier still (lead_load, before pool_kth's
// bisection, whose ballot loop then hides its latency).
constexpr int LEAD_LB = 8;
struct LeadBatch {
  float v[LEAD_LB][4];
};
__device__ __forceinline__ void lead_load(const LeadArgs& la, int64_t b, int p0, LeadBatch& lb) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < LEAD_LB; ++q) {
    if (p0 + q < la.lead) {  // uniform
#pragma unroll
      for (int e = 0; e < 4; ++e)
        lb.v[q][e] = la.s[b * la.ld + (int64_t)(p0 + q) * 256 + e * 64 + lane];
    }
  }
}
__device__ __forceinline__ void lead_hits_wave(const LeadArgs& la, int64_t b, float th, int* ovf,
                                               LeadBatch& lb) {
  const int lane = threadIdx.x & 63;
  int over = 0;
  for (int p0 = 0; p0 < la.lead; p0 += LEAD_LB) {
    if (p0 > 0) lead_load(la, b, p0, lb);  // (batch 0: the caller's lead_load)
#pragma unroll
    for (int q = 0; q < LEAD_LB; ++q) {
      const int p = p0 + q;
      if (p >= la.lead) break;  // uniform
      uint32_t base = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = lb.v[q][e];
        const bool hit = v >= th;
        const uint64_t bm = __ballot(hit);
        const uint32_t pp = base + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
        if (hit && pp < (uint32_t)la.slots) {
          const uint32_t row = (uint32_t)(p * 256 + e * 64 + lane);
          la.cand[b * la.ld_cand + (int64_t)p * la.slots + pp] =
              ((uint64_t)f2key(v) << 32) | (uint64_t)(~row);
        }
        base += (uint32_t)__popcll(bm);
      }
      if (lane == 0) la.counts[b * la.ld_counts + p] = (uint8_t)(base < 255u ? base : 255u);
      over |= base > (uint32_t)la.slots ? 1 : 0;
    }
  }
  if (lane == 0 && over) ovf[b] = 1;
}
template <int E>
__global__ __launch_bounds__(256) void pool_kth_kernel(const float* __restrict__ pool, int64_t ld,
                                                       int64_t B, int64_t B_pad, int G, int j,
                                                       float* __restrict__ thr,
                                                       float* __restrict__ fv,
                                                       int64_t* __restrict__ fi, int kprime,
                                                       int* __restrict__ ovf, LeadArgs la,
                                                       int gj, int64_t rstride) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B_pad) return;
  if (fv) {
    if (lane == 0) ovf[b] = 0;
    if (b < B)
      for (int i = lane; i < kprime; i += 64) {
        fv[b * kprime + i] = -__builtin_inff();
        fi[b * kprime + i] = -1;
      }
  }
  LeadBatch lb;
  if (b >= B) {
    if (lane == 0) thr[b] = __builtin_inff();
    if (la.lead > 0) {   // zero counts
      lead_load(la, b, 0, lb);
      lead_hits_wave(la, b, __builtin_inff(), ovf, lb);
    }
    return;
  }
  if (la.lead > 0) lead_load(la, b, 0, lb);  // in flight during the bisection
  // gj > 0: the all-gathered [R][B][gj] layout of a row-sharded catalog's samples, read in place
  // (value g of query b at rank g / gj), instead of a [B][ld] row
  uint32_t kx[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int g = lane + 64 * e;
    const int gg = g < G ? g : 0;
    const int64_t off = gj > 0 ? (int64_t)(gg / gj) * rstride + b * gj + gg % gj : b * ld + gg;
    const float x = pool[off];
    kx[e] = g < G ? f2key(x) : 0u;
  }
  auto count_ge = [&](uint32_t t) {
    int c = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) c += __popcll(__ballot(kx[e] >= t));
    return c;
  };
  uint64_t lo = 1, hi = 0xffffffffull;  // largest t with count(key >= t) >= j
  float th = -__builtin_inff();
  if (count_ge(1u) >= j) {
    while (lo < hi) {
      const uint64_t mid = lo + ((hi - lo + 1) >> 1);
      if (count_ge((uint32_t)mid) >= j) lo = mid;
      else hi = mid - 1;
    }
    th = key2f((uint32_t)lo);
  }
  if (lane == 0) thr[b] = th;
  if (la.lead > 0) lead_hits_wave(la, b, th, ovf, lb);
}
int pool_kth(const float* pool, int64_t ld, int64_t B, int64_t B_pad, int G, int j, float* thr,
             hipStream_t st, float* fv, int64_t* fi, int kprime, int* ovf,
             const float* lead_s, int64_t ld_lead, int lead, uint64_t* cand, int64_t ld_cand,
             int slots, uint8_t* counts, int64_t ld_counts, int gj, int64_t rstride) {
  if (!pool || !thr || B < 0 || B_pad < B || G < 1 || G > 2048 || j < 1 ||
      (gj > 0 ? (G % gj != 0 || rstride < B * (int64_t)gj) : ld < G) ||
      (fv && (!fi || !ovf || kprime < 1)) ||
      (lead > 0 && (!lead_s || ld_lead < 256LL * lead || !cand || slots < 1 ||
                    ld_cand < (int64_t)lead * slots || !counts || ld_counts < lead || !ovf))) {
    set_error("pool_kth: bad arguments (G=%d j=%d ld=%lld lead=%d)", G, j, (long long)ld, lead);
    return EBT_EINVAL;
  }
  LeadArgs la{lead_s, ld_lead, lead > 0 ? lead : 0, cand, ld_cand, slots, counts, ld_counts};
  const dim3 grid((unsigned)ceil_div(B_pad, 4)), block(256);
  if (G <= 256)
    hipLaunchKernelGGL(pool_kth_kernel<4>, grid, block, 0, st, pool, ld, B, B_pad, G, j, thr, fv,
                       fi, kprime, ovf, la, gj, rstride);
  else
    hipLaunchKernelGGL(pool_kth_kernel<32>, grid, block, 0, st, pool, ld, B, B_pad, G, j, thr, fv,
                       fi, kprime, ovf, la, gj, rstride);
  return launch_check("pool_kth_kernel");
}

// The caller-threshold screen's set-up in one launch (it was a copy and three fills): the
// threshold (+inf on padding rows), the empty list (-inf / -1) and no overflow.
__global__ __launch_bounds__(256) void spec_given_init_kernel(const float* __restrict__ theta,
                                                              int64_t B, int64_t B_pad,
                                                              float* __restrict__ tspec,
                                                              float* __restrict__ fv,
                                                              int64_t* __restrict__ fi,
                                                              int64_t n_list, int* __restrict__ ovf) {
  const int64_t n = n_list > B_pad ? n_list : B_pad;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (i < B_pad) {
      tspec[i] = i < B ? theta[i] : __builtin_inff();
      ovf[i] = 0;
    }
    if (i < n_list) {
      fv[i] = -__builtin_inff();
      fi[i] = -1;
    }
  }
}

// The same with a lead (a row-sharded catalog's sample lead, ebt_cosine_screen_at_lead): one wave
// per query also takes its hits among the lead tiles' stored scores at the caller's threshold,
// as pool_kth_kernel does at its own.
__global__ __launch_bounds__(256) void spec_given_lead_kernel(const float* __restrict__ theta,
                                                              int64_t B, int64_t B_pad,
                                                              float* __restrict__ tspec,
                                                              float* __restrict__ fv,
                                                              int64_t* __restrict__ fi, int kprime,
                                                              int* __restrict__ ovf, LeadArgs la) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B_pad) return;
  if (lane == 0) ovf[b] = 0;
  const float th = b < B ? theta[b] : __builtin_inff();
  if (lane == 0) tspec[b] = th;
  if (b < B)
    for (int i = lane; i < kprime; i += 64) {
      fv[b * kprime + i] = -__builtin_inff();
      fi[b * kprime + i] = -1;
    }
  LeadBatch lb;
  lead_load(la, b, 0, lb);
  lead_hits_wave(la, b, th, ovf, lb);   // padding rows: +inf, zero counts
}

int spec_given_init(const float* theta, int64_t B, int64_t B_pad, float* tspec, float* fv,
                    int64_t* fi, int kprime, int* ovf, hipStream_t st, const float* lead_s,
                    int64_t ld_lead, int lead, uint64_t* cand, int64_t ld_cand, int slots,
                    uint8_t* counts, int64_t ld_counts) {
  if (lead > 0) {
    if (!lead_s || ld_lead < 256LL * lead || !cand || slots < 1 ||
        ld_cand < (int64_t)lead * slots || !counts || ld_counts < lead) {
      set_error("spec_given_init: bad lead arguments (lead=%d)", lead);
      return EBT_EINVAL;
    }
    LeadArgs la{lead_s, ld_lead, lead, cand, ld_cand, slots, counts, ld_counts};
    hipLaunchKernelGGL(spec_given_lead_kernel, dim3((unsigned)ceil_div(B_pad, 4)), dim3(256), 0,
                       st, theta, B, B_pad, tspec, fv, fi, kprime, ovf, la);
    return launch_check("spec_given_lead_kernel");
  }
  const int64_t n_list = B * (int64_t)kprime;
  const int64_t n = n_list > B_pad ? n_list : B_pad;
  int64_t blocks = ceil_div(n, 256);
  blocks = blocks < 4096 ? blocks : 4096;
  hipLaunchKernelGGL(spec_given_init_kernel, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(256),
                     0, st, theta, B, B_pad, tspec, fv, fi, n_list, ovf);
  return launch_check("spec_given_init_kernel");
}

int spec_threshold(const float* vals, int64_t ld, int64_t B, int64_t B_pad, int k,
                   const float* eps, const float* thr_spec, float* thr, int* ovf, int mode,
                   hipStream_t st) {
  hipLaunchKernelGGL(spec_threshold_kernel, dim3((unsigned)ceil_div(B_pad, 256)), dim3(256), 0,
                     st, vals, ld, B, B_pad, k, eps, thr_spec, thr, ovf, mode);
  return launch_check("spec_threshold_kernel");
}

}  // namespace ebt
