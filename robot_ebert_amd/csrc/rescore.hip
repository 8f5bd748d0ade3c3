// Exact float64 rescore of the screened candidates, final top-k, certification; and the
// cross-shard merge of partial top-k lists.
//
// The reference's arithmetic is float64 end to end (constants.py:56 builds a float64 DataFrame;
// sklearn keeps float64 unless both inputs are float32, metrics/pairwise.py:67). The screening
// GEMM runs in f16/bf16 MFMA, so its scores are approximations with a per-query error bound
// eps (prep.hip). Here every candidate is recomputed as (q64 . c) / gnorm64(c) in float64 --
// the same value as sklearn's normalize-then-dot up to float64 round-off -- and the k best are
// chosen by (score desc, row asc). The candidate set is PROVABLY a superset of the true top-k
// when approx[k'-1] < approx[k-1] - 2 eps ("certified-margin rescore");
// otherwise certified[b] = 0 and the host retries that query with a larger k'.
#include <atomic>
#include <cstdlib>

#include "common.h"

namespace ebt {

constexpr int RTHREADS = 256;
constexpr int RESCORE_RANK_MAX = 512;   // kept rows ordered by counting (else bitonic)

__device__ __forceinline__ bool pair_before(double sa, int64_t ra, double sb, int64_t rb) {
  return sa > sb || (sa == sb && ra < rb);
}

// Sort (score, row) pairs: score desc, row asc. P power of two.
__device__ void bitonic_pairs(double* sc, int64_t* rw, int P) {
  const int tid = threadIdx.x;
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (P >> 1); t += blockDim.x) {
        const int lo = ((t & ~(stride - 1)) << 1) | (t & (stride - 1));  // stride: a power of 2
        const int hi = lo + stride;
        const double a = sc[lo], b = sc[hi];
        const int64_t ra = rw[lo], rb = rw[hi];
        const bool first = (lo & size) == 0;  // this segment ends up in "before" order
        const bool swap = first ? pair_before(b, rb, a, ra) : pair_before(a, ra, b, rb);
        if (swap) {
          sc[lo] = b;
          sc[hi] = a;
          rw[lo] = rb;
          rw[hi] = ra;
        }
      }
      __syncthreads();
    }
  }
}

// Marks v as used here, unconditionally: a load feeding only a guarded store would otherwise be
// sunk into the guard's block and waited for there, one load at a time.
__device__ __forceinline__ void issued(double v) { asm volatile("" : : "v"(v)); }
__device__ __forceinline__ void issued(int64_t v) { asm volatile("" : : "v"(v)); }

// dst[0, d) = src[0, d) by the workgroup, eight loads per thread in flight (a plain strided loop
// waits for each load before the next); past-the-end slots load entry d - 1 and store nothing.
__device__ __forceinline__ void stage_f64(double* dst, const double* __restrict__ src, int d) {
  for (int j0 = threadIdx.x; j0 < d; j0 += 8 * RTHREADS) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * RTHREADS;
      v[u] = src[j < d ? j : d - 1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * RTHREADS;
      issued(v[u]);
      if (j < d) dst[j] = v[u];
    }
  }
}

static int next_pow2_h(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// Sum of q . row over one lane's share of the row (16-byte chunks ch = lane, lane+64, ...),
// accumulated in chunk order; the caller's wave_sum_f64 completes the dot product.
template <int DT>
__device__ __forceinline__ double chunk_dot(const double* qs, int j0, uint4 raw) {
  double s = 0.0;
  if constexpr (DT == EBT_F32) {
    const float* f = (const float*)&raw;
#pragma unroll
    for (int e = 0; e < 4; ++e) s += qs[j0 + e] * (double)f[e];
  } else if constexpr (DT == EBT_F64) {
    const double* f = (const double*)&raw;
    s += qs[j0] * f[0] + qs[j0 + 1] * f[1];
  } else {
    const uint16_t* h = (const uint16_t*)&raw;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      s += qs[j0 + e] * (DT == EBT_BF16 ? bf16_bits_to_f64(h[e]) : f16_bits_to_f64(h[e]));
  }
  return s;
}
// The same sum with the lane's query values in registers (q[e] = qs[j0 + e]): the same
// expression, so the same contracted FMA chain and the same bits.
template <int DT, int PER>
__device__ __forceinline__ double chunk_dot_reg(const double (&q)[PER], uint4 raw) {
  double s = 0.0;
  if constexpr (DT == EBT_F32) {
    const float* f = (const float*)&raw;
#pragma unroll
    for (int e = 0; e < 4; ++e) s += q[e] * (double)f[e];
  } else if constexpr (DT == EBT_F64) {
    const double* f = (const double*)&raw;
    s += q[0] * f[0] + q[1] * f[1];
  } else {
    const uint16_t* h = (const uint16_t*)&raw;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      s += q[e] * (DT == EBT_BF16 ? bf16_bits_to_f64(h[e]) : f16_bits_to_f64(h[e]));
  }
  return s;
}

// Rows per wave round trip of the register-query form, by chunks per lane (NU): about eight
// 16-byte loads per lane in flight (C2 / C4: NU = 2 -> 4 rows; C5: 3 -> 2; C3: 6 -> 2)
#ifndef EBT_RESCORE_NR_WIDE
#define EBT_RESCORE_NR_WIDE 2  // rows per trip at 3..6 chunks per lane (build knob for A/B)
#endif
#ifndef EBT_RESCORE_NR_NARROW
#define EBT_RESCORE_NR_NARROW 4  // rows per trip at <= 2 chunks per lane (build knob for A/B)
#endif
template <int NU>
constexpr int rescore_rows_per_trip() {
  return NU <= 2 ? EBT_RESCORE_NR_NARROW : (NU <= 6 ? EBT_RESCORE_NR_WIDE : 1);
}

// NU = 0: the query staged in LDS (any d), two rows per wave round trip. NU > 0 (VEC, d / PER
// <= 64 NU 16-byte chunks): each lane keeps its chunks' query values (chunks lane + 64 u) in
// registers for every row -- no LDS reads in the dot products, no query staging -- and gathers
// rescore_rows_per_trip<NU>() rows per round trip from per-pass row lists. Per row the same
// chunk order, the same per-chunk sums and the same wave butterfly: bitwise the same scores.
#ifdef EBT_RESCORE_STAMP
// Diagnostic build only: shader cycles of each phase of a query's rescore workgroup (wave 0's
// view): [0] query + list + compaction, [1] pass A, [2] s_min + pass B's list, [3] pass B,
// [4] order + write; g_rstamp[5 b ..] (vector stores; nothing else reads them).
__device__ unsigned long long* g_rstamp;
extern "C" int ebt_debug_rescore_stamps(unsigned long long* buf) {
  return hip_check(hipMemcpyToSymbol(HIP_SYMBOL(g_rstamp), &buf, sizeof(buf)), "hipMemcpyToSymbol");
}
#define RST(i) rs[i] = __builtin_amdgcn_s_memtime()
#else
#define RST(i)
#endif
// (f32 rows with the query held in registers at d = 1536, C3's variant: 138 VGPRs would give
// three waves per SIMD; bounded to 128 -- no spill -- it runs four, a quarter more row gathers
// in flight. The other variants are at four or more already, or would spill under the bound.)
template <int DT, bool VEC, int NU = 0>
__global__ __launch_bounds__(RTHREADS, (DT == EBT_F32 && NU == 6) ? 4 : 1) void rescore_kernel(
    const double* __restrict__ q64, int d, const void* __restrict__ cat, int64_t ld,
    const double* __restrict__ gnorm, int64_t row_offset, const float* __restrict__ cand_vals,
    const int64_t* __restrict__ cand_rows, int kprime, int kpp, int k, int64_t n_rows,
    const float* __restrict__ eps, const double* __restrict__ t_floor, double* __restrict__ out_s,
    int64_t* __restrict__ out_r, int32_t* __restrict__ certified, const int* __restrict__ ovf_cnt,
    int ovf_cap, unsigned long long* __restrict__ gathered, int64_t list_base,
    const float* __restrict__ theta, const int64_t* __restrict__ excl_off,
    const int64_t* __restrict__ excl_rows, const ShardPackOut pack) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* qs = (double*)smem;                           // d (NU = 0 only)
  double* sc = qs + (NU > 0 ? 0 : ((d + 1) & ~1));      // kpp: approx, then exact
  int64_t* rw = (int64_t*)(sc + kpp);         // kpp
  int* pl = (int*)(rw + kpp);                 // kpp: list position of each kept row
  int* ix = pl + kpp;                         // kpp (NU > 0): the rows of the current pass
  __shared__ int nvalid, corrupt, nkeep, ntop, nsel, ngath, xbad, npk;
  __shared__ unsigned long long smin_key;
  constexpr int NW = RTHREADS / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
#ifdef EBT_RESCORE_STAMP
  unsigned long long rs[6] = {0, 0, 0, 0, 0, 0};
#endif
  RST(0);
  if (tid == 0) {
    nvalid = 0;
    corrupt = 0;
    nkeep = 0;
    ntop = 0;
    nsel = 0;
    ngath = 0;
    xbad = 0;
    npk = 0;
    smin_key = ~0ull;
  }
  constexpr int ES = (DT == EBT_F64) ? 8 : (DT == EBT_F32 ? 4 : 2);
  constexpr int PER = 16 / ES;
  // the query's exclusion segment must be sorted ascending (the merges drop excluded rows by
  // binary search): checked here, one pass over its few rows, certified = -3 otherwise -- the
  // C entry's separate check kernel and flag memset folded into the kernel that writes the
  // certificate (set after the barrier below, read after the next)
  bool xb = false;
  if (excl_off) {
    const int64_t xs = excl_off[b], xe = excl_off[b + 1];
    xb = xe < xs;
    for (int64_t t = xs + tid; t + 1 < xe; t += RTHREADS) xb |= excl_rows[t] > excl_rows[t + 1];
  }
  // NU > 0: the lane's query values of chunks lane + 64 u (0 past the row)
  double qv[NU > 0 ? NU : 1][PER];
  if constexpr (NU > 0) {
    const int nch = d / PER;
    const double* qrow = q64 + b * d;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int ch = lane + 64 * u;
      const int cc = ch < nch ? ch : 0;  // clamped, so that every load is issued up front
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const double x = qrow[cc * PER + e];
        qv[u][e] = ch < nch ? x : 0.0;
      }
    }
  } else {
    stage_f64(qs, q64 + b * d, d);
  }
  const int64_t* cr = cand_rows + b * kprime;
  // Candidates whose approx score is below approx[k-1] - 2 eps cannot be in the top k (the k
  // best candidates all have exact >= approx[k-1] - eps > their exact), so their rows are not
  // gathered: about k + (rows in the 2 eps band) of the k' candidates are rescored.
  // t_floor (optional): a lower bound of the k-th best EXACT score over the whole (sharded)
  // catalog, e.g. max over shards of (shard's approx[k-1] - eps). A row of the global top k has
  // exact >= t_floor, so approx >= t_floor - eps: the cut may rise to that.
  const float* cv = cand_vals + b * kprime;
  double cut = (double)cv[k - 1] - 2.0 * (double)eps[b];
  if (t_floor && t_floor[b] - (double)eps[b] > cut) cut = t_floor[b] - (double)eps[b];
  __syncthreads();
  if (xb) xbad = 1;
  // 1. the whole list at once (no per-candidate load latency): count valid rows, flag corrupt
  //    ones, compact the rows above the cut into rw[0, nkeep)
  for (int c0 = 0; c0 < kprime; c0 += RTHREADS) {
    const int c = c0 + tid;
    int64_t row = -1;
    float v = 0.f;
    if (c < kprime) {
      row = cr[c];
      v = cv[c];
      row = row >= 0 ? row - list_base : -1;  // a list of GLOBAL rows (list_base = row_offset)
    }
    const bool bad = c < kprime && row >= n_rows;  // corrupt entry, never dereferenced
    const bool valid = c < kprime && row >= 0 && !bad;
    const bool keep = valid && !((double)v < cut);
    if (bad) corrupt = 1;
    const uint64_t vb = __ballot(valid), kb = __ballot(keep);
    int base = 0;
    if (lane == 0) {
      if (vb) atomicAdd(&nvalid, __popcll(vb));
      if (kb) base = atomicAdd(&nkeep, __popcll(kb));
    }
    base = __shfl(base, 0, 64);
    int at = -1;
    if (keep) {
      at = base + __popcll(kb & ((1ull << lane) - 1));
      rw[at] = row;
      sc[at] = (double)v;
      pl[at] = c;
    }
    if constexpr (NU > 0) {  // pass A's rows: the kept ones among the list's first k
      const bool top = keep && c < k;
      const uint64_t tb = __ballot(top);
      int tbase = 0;
      if (lane == 0 && tb) tbase = atomicAdd(&nsel, __popcll(tb));
      tbase = __shfl(tbase, 0, 64);
      if (top) ix[tbase + __popcll(tb & ((1ull << lane) - 1))] = at;
    }
  }
  __syncthreads();
  RST(1);
  const int nk = nkeep;
  // 2. exact scores in two passes. The list's first k positions hold its k best approx (a
  //    partitioned or sorted list): pass A scores those; their smallest exact score s_min
  //    bounds the k-th best exact score from below (k rows reach it), so a later candidate
  //    with approx < s_min - eps (exact < s_min) cannot enter the top k: pass B skips it. About
  //    half of the 2 eps band is never gathered.
  //    Two rows per wave at a time with all of a lane's loads for both rows issued before the
  //    arithmetic (chunk order per lane unchanged: bit-identical sums).
  auto exact_pass = [&](bool top, double cut2) {
    for (int j = wave; j < nk; j += 2 * NW) {
    const int jb = j + NW;
    const bool sel_a = (pl[j] < k) == top && (top || !(sc[j] < cut2));
    const bool sel_b = jb < nk && (pl[jb] < k) == top && (top || !(sc[jb] < cut2));
    if (!top) {  // skipped: below the two-stage cut, sorted last
      if (lane == 0 && pl[j] >= k && !sel_a) sc[j] = -__builtin_inf();
      if (lane == 0 && jb < nk && pl[jb] >= k && !sel_b) sc[jb] = -__builtin_inf();
    }
    if (!sel_a && !sel_b) continue;
    const int ja = sel_a ? j : jb;          // one selected row goes first
    const bool hb = sel_a && sel_b;         // a second one
    if (gathered && lane == 0) atomicAdd(&ngath, hb ? 2 : 1);
    const int64_t ra = rw[ja], rb = hb ? rw[jb] : ra;
    const double ga = gnorm[ra], gb = gnorm[rb];
    double sa = 0.0, sb = 0.0;
    if constexpr (VEC) {
      constexpr int ES = (DT == EBT_F64) ? 8 : (DT == EBT_F32 ? 4 : 2);
      constexpr int PER = 16 / ES;
      constexpr int U = 4;
      const int nch = d / PER;
      const char* pa = (const char*)cat + ra * ld * ES;
      const char* pb = (const char*)cat + rb * ld * ES;
      for (int ch0 = lane; ch0 < nch; ch0 += 64 * U) {
        uint4 xa[U], xb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ch = ch0 + 64 * u;
          if (ch < nch) {
            xa[u] = *(const uint4*)(pa + (int64_t)ch * 16);
            if (hb) xb[u] = *(const uint4*)(pb + (int64_t)ch * 16);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ch = ch0 + 64 * u;
          if (ch < nch) {
            sa += chunk_dot<DT>(qs, ch * PER, xa[u]);
            if (hb) sb += chunk_dot<DT>(qs, ch * PER, xb[u]);
          }
        }
      }
    } else {
      for (int e = lane; e < d; e += 64) {
        sa += qs[e] * load_as_f64<DT>(cat, ra * ld + e);
        if (hb) sb += qs[e] * load_as_f64<DT>(cat, rb * ld + e);
      }
    }
    sa = wave_sum_f64(sa);
    sb = wave_sum_f64(sb);
    if (lane == 0) {
      const double va = sa / ga;
      sc[ja] = (va == va) ? va : -__builtin_inf();
      if (hb) {
        const double vb2 = sb / gb;
        sc[jb] = (vb2 == vb2) ? vb2 : -__builtin_inf();
      }
    }
    }
  };
  // NU > 0: the wave's rows ix[i0 .. i0 + NR) of a pass list, all of their loads issued before
  // the arithmetic (the last row repeated past the list's end, not stored)
  auto exact_rows = [&](int n) {
    if constexpr (NU > 0) {
      constexpr int NR = rescore_rows_per_trip<NU>();
      const int nch = d / PER;
      for (int i0 = wave * NR; i0 < n; i0 += NW * NR) {
        int64_t r[NR];
        double g[NR];
        uint4 x[NR][NU];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) r[rr] = rw[ix[i0 + rr < n ? i0 + rr : n - 1]];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
          const char* p = (const char*)cat + r[rr] * ld * ES;
#pragma unroll
          for (int u = 0; u < NU; ++u) {
            const int ch = lane + 64 * u;
            x[rr][u] = *(const uint4*)(p + (int64_t)(ch < nch ? ch : 0) * 16);
          }
          g[rr] = gnorm[r[rr]];
        }
        double s[NR];
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
          s[rr] = 0.0;
#pragma unroll
          for (int u = 0; u < NU; ++u)
            if (lane + 64 * u < nch) s[rr] += chunk_dot_reg<DT, PER>(qv[u], x[rr][u]);
        }
        // the NR butterflies together; the first lane of each value's lane group stores it
        const double tot = wave_sum_f64_rows<NR>(s);
        const int own = wave_rows_owner<NR>(lane);
        double gown = g[0];
#pragma unroll
        for (int rr = 1; rr < NR; ++rr) gown = own == rr ? g[rr] : gown;
        if ((lane & (64 / NR - 1)) == 0 && i0 + own < n) {
          const double v = tot / gown;
          sc[ix[i0 + own]] = (v == v) ? v : -__builtin_inf();
        }
      }
    }
  };
  if constexpr (NU > 0) exact_rows(nsel);
  else exact_pass(true, 0.0);
  __syncthreads();
  RST(2);
  // pass B's row count restarts (every thread read pass A's before the barrier above)
  if (NU > 0 && tid == 0) {
    ngath = nsel;
    nsel = 0;
  }
  // s_min over the k top entries (all k present and valid), as an order-preserving key: a wave
  // count and a wave minimum (DPP), then one LDS atomic per wave instead of one per entry
  for (int j0 = 0; j0 < nk; j0 += RTHREADS) {
    const int j = j0 + tid;
    const bool top = j < nk && pl[j] < k;
    unsigned long long key = ~0ull;  // no valid key is all ones
    if (top) {
      const double x = sc[j];
      const unsigned long long u = (unsigned long long)__double_as_longlong(x);
      if (x == x) key = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
    }
    const uint64_t tb = __ballot(top);
    const uint32_t kh = wave_min_u32((uint32_t)(key >> 32));
    const uint32_t kl = wave_min_u32((uint32_t)(key >> 32) == kh ? (uint32_t)key : 0xffffffffu);
    const unsigned long long wk = ((unsigned long long)kh << 32) | kl;
    if (lane == 0) {
      if (tb) atomicAdd(&ntop, (int)__popcll(tb));
      if (wk != ~0ull) atomicMin(&smin_key, wk);
    }
  }
  __syncthreads();
  double cut2 = cut;
  // (eps = 0 means "rescore every candidate above the first cut", not an exact approx)
  if (ntop == k && smin_key != ~0ull && eps[b] > 0.f) {
    const unsigned long long key = smin_key;
    const double smin = __longlong_as_double(
        (long long)((key >> 63) ? (key & 0x7fffffffffffffffull) : ~key));
    if (smin - (double)eps[b] > cut2) cut2 = smin - (double)eps[b];
  }
  if constexpr (NU > 0) {
    // pass B's rows: past the list's first k and not below cut2; the others sorted last
    for (int j0 = 0; j0 < nk; j0 += RTHREADS) {
      const int j = j0 + tid;
      const bool rest = j < nk && pl[j] >= k;
      const bool sel = rest && !(sc[j] < cut2);
      if (rest && !sel) sc[j] = -__builtin_inf();
      const uint64_t sb = __ballot(sel);
      int sbase = 0;
      if (lane == 0 && sb) sbase = atomicAdd(&nsel, __popcll(sb));
      sbase = __shfl(sbase, 0, 64);
      if (sel) ix[sbase + __popcll(sb & ((1ull << lane) - 1))] = j;
    }
    __syncthreads();
    RST(3);
    exact_rows(nsel);
  } else {
    RST(3);
    exact_pass(false, cut2);
  }
  RST(4);
  if (pack.len) {
    // the sharded step's pack count: the entries of this query's top k with score >= t_floor
    // (ebt_shard_pack's prefix) are min(k, the kept rows scoring >= t_floor) -- those rank
    // before every other kept row; read from the exact scores in LDS, no second pass over the
    // written list. (A barrier first: the last pass's scores come from other waves.)
    __syncthreads();
    const double tf = t_floor ? t_floor[b] : -__builtin_inf();
    int c = 0;
    for (int j = tid; j < nk; j += RTHREADS) c += sc[j] >= tf ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0 && c) atomicAdd(&npk, c);   // read after the ordering's barriers
  }
  // 3. order the kept rows (score desc, row asc); positions past them read NaN / -1
  if (nk <= RESCORE_RANK_MAX) {
    // few rows (C2 / C3: ~120-150): each row's position is the number of rows before it,
    // counted over LDS broadcast reads -- one barrier instead of a bitonic network's ~36. The
    // reads go 8 rows at a time, all issued before the first compare (one LDS latency per 8
    // rows, not per row), and up to RTHREADS / 2 rows take two threads each, one per half of
    // the list (the upper half's count handed over in LDS): the same counts.
    __shared__ int part[RTHREADS / 2];
    auto count_before = [&](double s, int64_t r, int j, int lo, int hi) {
      int pos = 0;
      for (int i0 = lo; i0 < hi; i0 += 8) {
        double si[8];
        int64_t ri[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u < hi ? i0 + u : hi - 1;
          si[u] = sc[i];
          ri[u] = rw[i];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u;
          pos += (i < hi && (pair_before(si[u], ri[u], s, r) ||
                             (si[u] == s && ri[u] == r && i < j))) ? 1 : 0;
        }
      }
      return pos;
    };
    auto put = [&](double s, int64_t r, int pos) {
      if (pos < k) {
        out_s[b * k + pos] = s;
        out_r[b * k + pos] = r + row_offset;
      }
    };
    __syncthreads();
    if (nk <= RTHREADS / 2) {
      const int j = tid & (RTHREADS / 2 - 1);
      const bool upper = tid >= RTHREADS / 2;
      const int m = nk >> 1;
      double s = 0.0;
      int64_t r = 0;
      int pos = 0;
      if (j < nk) {
        s = sc[j];
        r = rw[j];
        pos = upper ? count_before(s, r, j, m, nk) : count_before(s, r, j, 0, m);
        if (upper) part[j] = pos;
      }
      __syncthreads();
      if (!upper && j < nk) put(s, r, pos + part[j]);
    } else {
      for (int j = tid; j < nk; j += RTHREADS) put(sc[j], rw[j], count_before(sc[j], rw[j], j, 0, nk));
    }
    for (int j = nk + tid; j < k; j += RTHREADS) {
      out_s[b * k + j] = __builtin_nan("");
      out_r[b * k + j] = -1;
    }
  } else {
    int P = 1;
    while (P < nk || P < k) P <<= 1;
    for (int c = nk + tid; c < P; c += RTHREADS) {
      sc[c] = -__builtin_inf();
      rw[c] = INT64_MAX;
    }
    __syncthreads();
    bitonic_pairs(sc, rw, P);
    for (int j = tid; j < k; j += RTHREADS) {
      const int64_t r = rw[j];
      if (r == INT64_MAX) {
        out_s[b * k + j] = __builtin_nan("");
        out_r[b * k + j] = -1;
      } else {
        out_s[b * k + j] = sc[j];
        out_r[b * k + j] = r + row_offset;
      }
    }
  }
  if (tid == 0) {
    int ok = 1;
    if (nvalid >= kprime && n_rows > kprime) {  // kprime >= n_rows: every row is a candidate
      // rows below the k'-th candidate have approx <= amin; none of them can enter the top k
      // when amin < cut (the local k-th - 2 eps, or t_floor - eps when that is higher)
      const double amin = (double)cv[kprime - 1];
      ok = amin < cut2;
    }
    if (ovf_cnt && ovf_cnt[b] > ovf_cap) ok = -1;  // fused screen dropped candidates
    // a caller's screening threshold above the floor's cut may have dropped a row of the
    // global top k (ebt_certify_cut's test, folded in)
    if (theta && t_floor && !((double)theta[b] <= t_floor[b] - (double)eps[b])) ok = -1;
    if (corrupt) ok = -2;                           // internal error: row out of range
    if (xbad) ok = -3;                              // caller error: unsorted exclusion segment
    certified[b] = ok;
    if (pack.len) pack.len[b] = (uint32_t)(npk < k ? npk : k);
    // rows gathered by the two passes (roofline accounting: ebt_timer_count_rows), spread over
    // 64 counters 128 bytes apart: one address taking every query's atomic serialised them and
    // slowed the measured kernel by ~9 % at C3
    if (gathered)
      atomicAdd(gathered + (b & 63) * 16, (unsigned long long)(ngath + (NU > 0 ? nsel : 0)));
  }
#ifdef EBT_RESCORE_STAMP
  RST(5);
  if (tid == 0 && g_rstamp) {
#pragma unroll
    for (int i = 0; i < 5; ++i) g_rstamp[5 * b + i] = rs[i + 1] - rs[i];
  }
#endif
}

// The same rescore with the candidate rows gathered into LDS by LDS-DMA
// (global_load_lds_dwordx4: per-lane source addresses, no VGPRs held by the data), R rows per
// batch: the workgroup keeps R * row_bytes (about 24 KiB) in flight per round trip instead of two
// rows per wave, so a query whose rows are gathered in ~15 dependent round trips needs ~8 (C2:
// ~123 rows of 1.5 KiB per query, latency-bound, not bandwidth-bound). Arithmetic, order of
// summation and every decision are those of rescore_kernel: bit-identical results.
typedef __attribute__((address_space(3))) void rs_lds_void;
typedef __attribute__((address_space(1))) const void rs_gbl_cvoid;

template <int DT>
__global__ __launch_bounds__(RTHREADS) void rescore_lds_kernel(
    const double* __restrict__ q64, int d, const void* __restrict__ cat, int64_t ld,
    const double* __restrict__ gnorm, int64_t row_offset, const float* __restrict__ cand_vals,
    const int64_t* __restrict__ cand_rows, int kprime, int kpp, int k, int64_t n_rows,
    const float* __restrict__ eps, const double* __restrict__ t_floor, double* __restrict__ out_s,
    int64_t* __restrict__ out_r, int32_t* __restrict__ certified, const int* __restrict__ ovf_cnt,
    int ovf_cap, int R) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ES = (DT == EBT_F64) ? 8 : (DT == EBT_F32 ? 4 : 2);
  constexpr int PER = 16 / ES;
  constexpr int NW = RTHREADS / 64;
  const int cpr = d / PER;                    // 16-byte chunks per row
  const int rb = cpr * 16;
  char* stage = smem;                         // R rows, padded to whole 1 KiB pieces
  const int stage_bytes = (R * cpr + 63) / 64 * 1024;
  double* qs = (double*)(smem + stage_bytes);
  double* sc = qs + ((d + 1) & ~1);
  int64_t* rw = (int64_t*)(sc + kpp);
  int* pl = (int*)(rw + kpp);
  int* sel = pl + ((kpp + 1) & ~1);
  double* gsc = (double*)(sel + ((kpp + 1) & ~1));  // the batch rows' gnorm (R)
  __shared__ int nvalid, corrupt, nkeep, ntop, nsel;
  __shared__ unsigned long long smin_key;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  if (tid == 0) {
    nvalid = 0;
    corrupt = 0;
    nkeep = 0;
    ntop = 0;
    smin_key = ~0ull;
  }
  stage_f64(qs, q64 + b * d, d);
  const int64_t* cr = cand_rows + b * kprime;
  const float* cv = cand_vals + b * kprime;
  double cut = (double)cv[k - 1] - 2.0 * (double)eps[b];
  if (t_floor && t_floor[b] - (double)eps[b] > cut) cut = t_floor[b] - (double)eps[b];
  __syncthreads();
  for (int c0 = 0; c0 < kprime; c0 += RTHREADS) {
    const int c = c0 + tid;
    int64_t row = -1;
    float v = 0.f;
    if (c < kprime) {
      row = cr[c];
      v = cv[c];
    }
    const bool bad = c < kprime && row >= n_rows;
    const bool valid = c < kprime && row >= 0 && !bad;
    const bool keep = valid && !((double)v < cut);
    if (bad) corrupt = 1;
    const uint64_t vb = __ballot(valid), kb = __ballot(keep);
    int base = 0;
    if (lane == 0) {
      if (vb) atomicAdd(&nvalid, __popcll(vb));
      if (kb) base = atomicAdd(&nkeep, __popcll(kb));
    }
    base = __shfl(base, 0, 64);
    if (keep) {
      const int at = base + __popcll(kb & ((1ull << lane) - 1));
      rw[at] = row;
      sc[at] = (double)v;
      pl[at] = c;
    }
  }
  __syncthreads();
  const int nk = nkeep;
  // the positions a pass scores, compacted into sel[0, nsel) (list order)
  auto select = [&](bool top, double cut2) {
    if (tid == 0) nsel = 0;
    __syncthreads();
    for (int j0 = 0; j0 < nk; j0 += RTHREADS) {
      const int j = j0 + tid;
      bool take = false;
      if (j < nk) {
        take = (pl[j] < k) == top && (top || !(sc[j] < cut2));
        if (!top && pl[j] >= k && !take) sc[j] = -__builtin_inf();  // below the two-stage cut
      }
      const uint64_t tb = __ballot(take);
      int base = 0;
      if (lane == 0 && tb) base = atomicAdd(&nsel, __popcll(tb));
      base = __shfl(base, 0, 64);
      if (take) sel[base + __popcll(tb & ((1ull << lane) - 1))] = j;
    }
    __syncthreads();
  };
  auto score = [&]() {
    const int m = nsel;
    for (int s0 = 0; s0 < m; s0 += R) {
      const int nr = m - s0 < R ? m - s0 : R;
      const int nch = nr * cpr;
      const int ninstr = (nch + 63) / 64;
      for (int it = wave; it < ninstr; it += NW) {
        int c = it * 64 + lane;
        c = c < nch ? c : nch - 1;  // lanes past the batch re-read its last chunk
        const int r = c / cpr, w = c - r * cpr;
        const char* src = (const char*)cat + (rw[sel[s0 + r]] * ld) * ES + (int64_t)w * 16;
        __builtin_amdgcn_global_load_lds((rs_gbl_cvoid*)src, (rs_lds_void*)(stage + it * 1024),
                                         16, 0, 0);
      }
      if (tid < nr) gsc[tid] = gnorm[rw[sel[s0 + tid]]];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int r = wave; r < nr; r += NW) {
        const char* rowp = stage + r * rb;
        double acc = 0.0;
        for (int ch = lane; ch < cpr; ch += 64)
          acc += chunk_dot<DT>(qs, ch * PER, *(const uint4*)(rowp + ch * 16));
        acc = wave_sum_f64(acc);
        if (lane == 0) {
          const double v = acc / gsc[r];
          sc[sel[s0 + r]] = (v == v) ? v : -__builtin_inf();
        }
      }
      __syncthreads();  // the stage is overwritten by the next batch
    }
  };
  select(true, 0.0);
  score();
  for (int j = tid; j < nk; j += RTHREADS) {
    if (pl[j] < k) {
      atomicAdd(&ntop, 1);
      const double x = sc[j];
      unsigned long long key = (unsigned long long)__double_as_longlong(x);
      key = (key >> 63) ? ~key : (key | 0x8000000000000000ull);
      if (x == x) atomicMin(&smin_key, key);
    }
  }
  __syncthreads();
  double cut2 = cut;
  if (ntop == k && smin_key != ~0ull && eps[b] > 0.f) {
    const unsigned long long key = smin_key;
    const double smin = __longlong_as_double(
        (long long)((key >> 63) ? (key & 0x7fffffffffffffffull) : ~key));
    if (smin - (double)eps[b] > cut2) cut2 = smin - (double)eps[b];
  }
  select(false, cut2);
  score();
  int P = 1;
  while (P < nk || P < k) P <<= 1;
  for (int c = nk + tid; c < P; c += RTHREADS) {
    sc[c] = -__builtin_inf();
    rw[c] = INT64_MAX;
  }
  __syncthreads();
  bitonic_pairs(sc, rw, P);
  for (int j = tid; j < k; j += RTHREADS) {
    const int64_t r = rw[j];
    if (r == INT64_MAX) {
      out_s[b * k + j] = __builtin_nan("");
      out_r[b * k + j] = -1;
    } else {
      out_s[b * k + j] = sc[j];
      out_r[b * k + j] = r + row_offset;
    }
  }
  if (tid == 0) {
    int ok = 1;
    if (nvalid >= kprime && n_rows > kprime) {
      const double amin = (double)cv[kprime - 1];
      ok = amin < cut2;
    }
    if (ovf_cnt && ovf_cnt[b] > ovf_cap) ok = -1;
    if (corrupt) ok = -2;
    certified[b] = ok;
  }
}

// LDS of rescore_lds_kernel for R rows per batch (0 when the layout does not apply)
static size_t rescore_lds_stage_total(int d, int es, int kprime, int R) {
  const int kpp = next_pow2_h(kprime);
  const int cpr = d * es / 16;
  const size_t stage = (size_t)(R * cpr + 63) / 64 * 1024;
  return stage + 8 * (size_t)((d + 1) & ~1) + 16 * (size_t)kpp + 8 * (size_t)((kpp + 1) & ~1) +
         8 * (size_t)R;
}

// ebt_rescore_form: 1 = register-query form (default; EBT_RESCORE_REG=0 in the environment
// starts the process with the LDS-query form)
static std::atomic<int>& rescore_form_flag() {
  static std::atomic<int> f([] {
    const char* v = getenv("EBT_RESCORE_REG");
    return v ? (atoi(v) != 0 ? 1 : 0) : 1;
  }());
  return f;
}
static bool rescore_form_reg() { return rescore_form_flag().load(std::memory_order_relaxed) != 0; }

__global__ void wave_sum_check_kernel(const double* __restrict__ in, int64_t n_waves,
                                      double* __restrict__ a, double* __restrict__ b) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n_waves) return;  // whole waves
  const double v = in[w * 64 + (threadIdx.x & 63)];
  a[w * 64 + (threadIdx.x & 63)] = wave_sum_f64(v);
  b[w * 64 + (threadIdx.x & 63)] = wave_sum_f64_shfl(v);
}

extern "C" int ebt_rescore_form(int form) {
  if (form < 0) return rescore_form_flag().load();
  return rescore_form_flag().exchange(form != 0 ? 1 : 0);
}

extern "C" int ebt_wave_sum_check(const double* in, int64_t n_waves, double* out_a, double* out_b,
                                  void* stream) {
  if (!in || !out_a || !out_b || n_waves < 0) {
    set_error("ebt_wave_sum_check: bad arguments");
    return EBT_EINVAL;
  }
  if (n_waves == 0) return EBT_OK;
  hipLaunchKernelGGL(wave_sum_check_kernel, dim3((unsigned)ceil_div(n_waves, 4)), dim3(256), 0,
                     (hipStream_t)stream, in, n_waves, out_a, out_b);
  return launch_check("wave_sum_check_kernel");
}

size_t rescore_lds_bytes(int d, int kprime) {
  const int kpp = next_pow2_h(kprime);
  return 8 * (size_t)((d + 1) & ~1) + 20 * (size_t)kpp;
}

int rescore(const double* q64, int64_t B, int32_t d, const void* cat, int dtype, int64_t ld,
            const double* gnorm, int64_t row_offset, const float* cand_vals,
            const int64_t* cand_rows, int32_t kprime, int32_t k, int64_t n_rows, const float* eps,
            const double* t_floor, double* out_s, int64_t* out_r, int32_t* certified,
            hipStream_t st, const int* ovf_cnt, int ovf_cap, unsigned long long* gathered,
            int64_t list_base, const float* theta, const int64_t* excl_off,
            const int64_t* excl_rows, const ShardPackOut* pack) {
  const ShardPackOut po = pack ? *pack : ShardPackOut{};
  if (!q64 || !cat || !gnorm || !cand_vals || !cand_rows || !eps || !out_s || !out_r ||
      !certified || B < 0 || d <= 0 || ld < d || k < 1 || kprime < k || kprime > 4096 ||
      dtype < 0 || dtype > 3) {
    set_error("ebt_rescore: bad arguments (d=%d k=%d kprime=%d)", d, k, kprime);
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const int kpp = next_pow2_h(kprime);
  const size_t lds = rescore_lds_bytes(d, kprime);
  if (lds > 150 * 1024) {
    set_error("ebt_rescore: d=%d with kprime=%d exceeds LDS", d, kprime);
    return EBT_EUNSUPPORTED;
  }
  const int es = dtype == EBT_F64 ? 8 : (dtype == EBT_F32 ? 4 : 2);
  const bool vec = (((uintptr_t)cat & 15) == 0) && ((ld * es) % 16 == 0) &&
                   (((int64_t)d * es) % 16 == 0);
  dim3 grid((unsigned)B), block(RTHREADS);
#ifdef EBT_RESCORE_LDS
  // Measured and not the default (profiles/r3/rescore_lds_ab.txt): the LDS-DMA batches
  // (16 rows of 1.5 KiB per round trip at C2) took 71-75 us per C2 step against 59-60 us for the
  // register gather, interleaved on one MI355X; C3 0.616 vs 0.564 ms. Kept for that A/B (it
  // takes neither the exclusion check nor the pack count: such calls use the register form).
  if (vec && !excl_off && !po.len) {
    const int row_bytes = d * es;
    int R = (24 << 10) / row_bytes;
    R = R > 64 ? 64 : R;
    while (R >= 2 && rescore_lds_stage_total(d, es, kprime, R) > (38u << 10)) --R;
    // only where it keeps more rows in flight than the register form (8 per workgroup)
    if (R > 8) {
      const size_t lds2 = rescore_lds_stage_total(d, es, kprime, R);
#define EBT_RSL(DT)                                                                             \
  set_max_lds((const void*)rescore_lds_kernel<DT>, (int)lds2);                                 \
  hipLaunchKernelGGL((rescore_lds_kernel<DT>), grid, block, lds2, st, q64, d, cat, ld, gnorm,   \
                     row_offset, cand_vals, cand_rows, kprime, kpp, k, n_rows, eps, t_floor,    \
                     out_s, out_r, certified, ovf_cnt, ovf_cap, R);
      switch (dtype) {
        case EBT_F32: EBT_RSL(EBT_F32) break;
        case EBT_BF16: EBT_RSL(EBT_BF16) break;
        case EBT_F16: EBT_RSL(EBT_F16) break;
        default: EBT_RSL(EBT_F64) break;
      }
#undef EBT_RSL
      return launch_check("rescore_lds_kernel");
    }
  }
#endif
  // the register-query form (chunks per lane NU, rounded up to an instantiated count) unless
  // the form is 0 (the LDS-query form, kept for A/B and for d beyond 512 chunks)
  const int nch = d * es / 16;
  const int nu_need = (nch + 63) / 64;
  const int nu = nu_need <= 4 ? nu_need : (nu_need <= 6 ? 6 : (nu_need <= 8 ? 8 : 0));
  if (vec && rescore_form_reg() && nu > 0) {
    const size_t lds_r = 24 * (size_t)kpp;
#define EBT_RSR(DT, NU)                                                                         \
  set_max_lds((const void*)rescore_kernel<DT, true, NU>, (int)lds_r);                          \
  hipLaunchKernelGGL((rescore_kernel<DT, true, NU>), grid, block, lds_r, st, q64, d, cat, ld,   \
                     gnorm, row_offset, cand_vals, cand_rows, kprime, kpp, k, n_rows, eps,      \
                     t_floor, out_s, out_r, certified, ovf_cnt, ovf_cap, gathered, list_base,   \
                     theta, excl_off, excl_rows, po);
#define EBT_RSR_NU(DT)                                                                          \
  switch (nu) {                                                                                 \
    case 1: EBT_RSR(DT, 1) break;                                                               \
    case 2: EBT_RSR(DT, 2) break;                                                               \
    case 3: EBT_RSR(DT, 3) break;                                                               \
    case 4: EBT_RSR(DT, 4) break;                                                               \
    case 6: EBT_RSR(DT, 6) break;                                                               \
    default: EBT_RSR(DT, 8) break;                                                              \
  }
    switch (dtype) {
      case EBT_F32: EBT_RSR_NU(EBT_F32) break;
      case EBT_BF16: EBT_RSR_NU(EBT_BF16) break;
      case EBT_F16: EBT_RSR_NU(EBT_F16) break;
      default: EBT_RSR_NU(EBT_F64) break;
    }
#undef EBT_RSR_NU
#undef EBT_RSR
    return launch_check("rescore_kernel");
  }
#define EBT_RS(DT)                                                                              \
  set_max_lds((const void*)rescore_kernel<DT, true>, (int)lds);                                \
  set_max_lds((const void*)rescore_kernel<DT, false>, (int)lds);                               \
  if (vec)                                                                                      \
    hipLaunchKernelGGL((rescore_kernel<DT, true>), grid, block, lds, st, q64, d, cat, ld,       \
                       gnorm, row_offset, cand_vals, cand_rows, kprime, kpp, k, n_rows, eps,    \
                       t_floor, out_s, out_r, certified, ovf_cnt, ovf_cap, gathered, list_base, \
                       theta, excl_off, excl_rows, po);                                                                  \
  else                                                                                          \
    hipLaunchKernelGGL((rescore_kernel<DT, false>), grid, block, lds, st, q64, d, cat, ld,      \
                       gnorm, row_offset, cand_vals, cand_rows, kprime, kpp, k, n_rows, eps,    \
                       t_floor, out_s, out_r, certified, ovf_cnt, ovf_cap, gathered, list_base, \
                       theta, excl_off, excl_rows, po);
  switch (dtype) {
    case EBT_F32: EBT_RS(EBT_F32) break;
    case EBT_BF16: EBT_RS(EBT_BF16) break;
    case EBT_F16: EBT_RS(EBT_F16) break;
    default: EBT_RS(EBT_F64) break;
  }
#undef EBT_RS
  return launch_check("rescore_kernel");
}

// ------------------------------------------------------------------------------- merge -----
// The k best of R sorted partial lists per query, (score desc, row asc). Up to MERGE_CAP
// entries are sorted in LDS at once: R k <= MERGE_CAP in one bitonic sort; more ranks in rounds
// that keep the running top k in slots [0, k) and bring the next (MERGE_CAP - k) / k ranks in
// behind it (k <= MERGE_CAP / 2).
constexpr int MERGE_CAP = 8192;

__global__ __launch_bounds__(RTHREADS) void merge_topk_kernel(const double* __restrict__ scores,
                                                               const int64_t* __restrict__ rows,
                                                               int R, int64_t B, int k, int P,
                                                               double* __restrict__ out_s,
                                                               int64_t* __restrict__ out_r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sc = (double*)smem;
  int64_t* rw = (int64_t*)(sc + P);
  const int64_t b = blockIdx.x;
  // fill slots [base, P) with ranks [r0, r0 + m), -inf past them
  auto fill = [&](int base, int r0, int m) {
    const int n = m * k;
    for (int i = base + threadIdx.x; i < P; i += RTHREADS) {
      double s = -__builtin_inf();
      int64_t r = INT64_MAX;
      const int e = i - base;
      if (e < n) {
        const int rr = r0 + e / k, j = e % k;
        const int64_t off = ((int64_t)rr * B + b) * k + j;
        const int64_t row = rows[off];
        if (row >= 0) {
          const double v = scores[off];
          s = (v == v) ? v : -__builtin_inf();
          r = row;
        }
      }
      sc[i] = s;
      rw[i] = r;
    }
    __syncthreads();
  };
  int r0 = R * k <= P ? R : P / k;
  fill(0, 0, r0);
  bitonic_pairs(sc, rw, P);
  const int per = (P - k) / k;
  while (r0 < R) {
    const int m = R - r0 < per ? R - r0 : per;
    fill(k, r0, m);
    bitonic_pairs(sc, rw, P);
    r0 += m;
  }
  for (int j = threadIdx.x; j < k; j += RTHREADS) {
    const int64_t r = rw[j];
    out_s[b * k + j] = r == INT64_MAX ? __builtin_nan("") : sc[j];
    out_r[b * k + j] = r == INT64_MAX ? -1 : r;
  }
}

// The same merge by co-ranks when every list is sorted (what ebt_cosine_topk returns): the
// position of entry j of list r in the merged order is j + the entries of the other lists that
// precede it (binary search in each: (score desc, row asc); equal keys -- the -inf/-1 padding --
// ordered by list). Only a prefix of each list can reach the top k: with kr = ceil(k / R), the
// R kr entries at list positions < kr all precede-or-equal m0 = the LAST of the R entries at
// position kr - 1, so the k-th best does too, and an entry after m0 is in no top k. Entries up
// to m0 (about k + R per query on untied data, of the R k) are placed by R - 1 searches within
// the other lists' prefixes, instead of a bitonic network over next_pow2(R k) slots (log^2
// stages of 16-byte LDS swaps). A list found unsorted sends the query down the bitonic network
// (same result).
constexpr int MERGE_CORANK_CAP = 8192;   // R k entries in LDS (16 B each)
constexpr int MERGE_CORANK_RMAX = 1024;  // lists (a 4-byte prefix length each in LDS)

__device__ __forceinline__ bool mt_before(double xs, int64_t xr, double es, int64_t er) {
  return xs > es || (xs == es && xr < er);
}

size_t merge_corank_lds(int R, int P) {
  return (size_t)P * 16 + RTHREADS * 16 + (((size_t)(2 * R + 1) * 4 + 15) & ~(size_t)15);
}

// The lists' sources. DenseSrc (merge_topk_corank_kernel): [R][B][k] f64 scores + i64 rows
// (row < 0 = padding). PackedSrc (merge_packed_kernel): every rank's packed list of
// ebt_shard_pack (one all-gathered byte buffer, `stride` bytes per rank): u32 start[B], u32
// len[B] (+ scratch), then f64 scores[cap], then i32 rows[cap]; query b's entries are
// [start[b], start[b] + len[b]) clipped to cap (the rest was not sent).
struct DenseSrc {
  const double* scores;
  const int64_t* rows;
};
struct PackedSrc {
  const char* recv;
  int64_t stride, cap;
};

__device__ __forceinline__ const uint32_t* pk_starts(const PackedSrc& p, int r) {
  return (const uint32_t*)(p.recv + (int64_t)r * p.stride);
}
__device__ __forceinline__ const uint32_t* pk_lens(const PackedSrc& p, int r, int64_t B) {
  return (const uint32_t*)(p.recv + (int64_t)r * p.stride) + B;
}
__device__ __forceinline__ const double* pk_scores(const PackedSrc& p, int r, int64_t B) {
  return (const double*)(p.recv + (int64_t)r * p.stride + shard_pack_hdr_bytes(B));
}
__device__ __forceinline__ const int32_t* pk_rows(const PackedSrc& p, int r, int64_t B) {
  return (const int32_t*)(p.recv + (int64_t)r * p.stride + shard_pack_hdr_bytes(B) + p.cap * 8);
}

template <class Src>
__global__ __launch_bounds__(RTHREADS) void merge_topk_corank_kernel(
    const Src src, int R, int64_t B, int k, int P, double* __restrict__ out_s,
    int64_t* __restrict__ out_r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = R * k;
  double* sc = (double*)smem;
  int64_t* rw = (int64_t*)(sc + P);   // P = next_pow2(n) >= n
  double* red_s = (double*)(rw + P);
  int64_t* red_r = (int64_t*)(red_s + RTHREADS / 2);
  int* plen = (int*)(red_r + RTHREADS / 2);
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  // four entries per thread in flight (a loop over e would wait for each load in turn: the
  // compiler peels the trip count's remainder into a serial loop)
  for (int e0 = tid; e0 < n; e0 += 4 * RTHREADS) {
    int64_t rv[4];
    double sv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * RTHREADS;
      const int ec = e < n ? e : n - 1;
      const int rr = ec / k, j = ec - rr * k;
      const int64_t off = ((int64_t)rr * B + b) * k + j;
      rv[u] = src.rows[off];
      sv[u] = src.scores[off];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * RTHREADS;
      issued(rv[u]);
      issued(sv[u]);
      if (e < n) {
        const bool pad = rv[u] < 0;
        sc[e] = pad || sv[u] != sv[u] ? -__builtin_inf() : sv[u];
        rw[e] = pad ? INT64_MAX : rv[u];
      }
    }
  }
  __syncthreads();
  int bad = 0;
  for (int e = tid; e < n; e += RTHREADS) {
    const int j = e % k;
    if (j + 1 < k && mt_before(sc[e + 1], rw[e + 1], sc[e], rw[e])) bad = 1;
  }
  if (__syncthreads_or(bad)) {
    // unsorted input: the bitonic network over P >= n slots
    for (int e = n + tid; e < P; e += RTHREADS) {
      sc[e] = -__builtin_inf();
      rw[e] = INT64_MAX;
    }
    __syncthreads();
    bitonic_pairs(sc, rw, P);
    for (int j = tid; j < k; j += RTHREADS) {
      const int64_t r = rw[j];
      out_s[b * k + j] = r == INT64_MAX ? __builtin_nan("") : sc[j];
      out_r[b * k + j] = r == INT64_MAX ? -1 : r;
    }
    return;
  }
  // m0: the last (in merged order) of the lists' entries at position kr - 1; then each list's
  // prefix of entries preceding-or-equal m0 (plen) and the prefixes' starts (cst) in the
  // compact enumeration of the candidates
  const int kr = (k + R - 1) / R;
  int* cst = plen + R;   // R + 1
  if (R <= 64) {
    // one wave, no barriers: lane r < R owns list r. Padding (row -1: a shard with fewer than
    // k rows above the floor cut -- at C3/8 about 18 of a list's 100) sorts last and is never a
    // candidate: V_r = the list's entries before its first padding entry. When at least k
    // entries lie in the "long" lists' first kr (V_r >= kr), m0 = the last of those lists'
    // kr-th entries bounds the k-th best as above; otherwise every non-padding entry is a
    // candidate (they are then few) and padding fills the positions past them.
    if (tid < 64) {
      int V = 0;
      if (tid < R) {
        const int64_t* orw = rw + tid * k;
        const double* os = sc + tid * k;
        int lo = 0, hi = k;   // first padding entry (sorted lists: padding is a suffix)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (!(orw[mid] == INT64_MAX && os[mid] == -__builtin_inf())) lo = mid + 1; else hi = mid;
        }
        V = lo;
      }
      const bool is_long = tid < R && V >= kr;
      const int n_long = __popcll(__ballot(is_long));
      double ms = __builtin_inf();
      int64_t mr = -1;   // "before everything": the identity of the max
      if (is_long) {
        ms = sc[tid * k + kr - 1];
        mr = rw[tid * k + kr - 1];
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double xs = __shfl_xor(ms, o, 64);
        const int64_t xr = __shfl_xor(mr, o, 64);
        if (mt_before(ms, mr, xs, xr)) {
          ms = xs;
          mr = xr;
        }
      }
      const bool bounded = n_long * kr >= k;
      int len = 0;
      if (tid < R) {
        len = V;
        if (bounded) {
          const double* os = sc + tid * k;
          const int64_t* orw = rw + tid * k;
          int lo = is_long ? kr : 0, hi = V;   // long lists: positions < kr are <= m0
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (!mt_before(ms, mr, os[mid], orw[mid])) lo = mid + 1; else hi = mid;
          }
          len = lo;
        }
      }
      int incl = len;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (tid >= o) incl += y;
      }
      if (tid < R) {
        plen[tid] = len;
        cst[tid] = incl - len;
      }
      if (tid == 63) cst[R] = incl;
    }
  } else {
    double ms = __builtin_inf();
    int64_t mr = -1;
    for (int r = tid; r < R; r += RTHREADS) {
      const double xs = sc[r * k + kr - 1];
      const int64_t xr = rw[r * k + kr - 1];
      if (mt_before(ms, mr, xs, xr)) {
        ms = xs;
        mr = xr;
      }
    }
    for (int h = RTHREADS / 2; h >= 1; h >>= 1) {
      if (tid >= h && tid < 2 * h) {
        red_s[tid - h] = ms;
        red_r[tid - h] = mr;
      }
      __syncthreads();
      if (tid < h && mt_before(ms, mr, red_s[tid], red_r[tid])) {
        ms = red_s[tid];
        mr = red_r[tid];
      }
      __syncthreads();
    }
    if (tid == 0) {
      red_s[0] = ms;
      red_r[0] = mr;
    }
    __syncthreads();
    ms = red_s[0];
    mr = red_r[0];
    for (int r = tid; r < R; r += RTHREADS) {
      const double* os = sc + r * k;
      const int64_t* orw = rw + r * k;
      int lo = kr, hi = k;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (!mt_before(ms, mr, os[mid], orw[mid])) lo = mid + 1; else hi = mid;
      }
      plen[r] = lo;
    }
    __syncthreads();
    if (tid == 0) {
      int c = 0;
      for (int r = 0; r < R; ++r) {
        cst[r] = c;
        c += plen[r];
      }
      cst[R] = c;
    }
  }
  __syncthreads();
  // candidate c -> (list rr, position j): one candidate per thread, so a wave's searches run
  // side by side instead of once per list position the wave strides over
  const int C = cst[R];
  for (int c = tid; c < C; c += RTHREADS) {
    int lo = 0, hi = R - 1;   // the last list whose start <= c
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (cst[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const int rr = lo, j = c - cst[rr];
    const int e = rr * k + j;
    const double es = sc[e];
    const int64_t er = rw[e];
    int pos = j;
    for (int o = 0; o < R && pos < k; ++o) {
      if (o == rr) continue;
      const double* os = sc + o * k;
      const int64_t* orw = rw + o * k;
      // entries of list o before e: those preceding it, and equal ones when o < rr
      int lo2 = 0, hi2 = plen[o];
      while (lo2 < hi2) {
        const int mid = (lo2 + hi2) >> 1;
        const bool before = mt_before(os[mid], orw[mid], es, er) ||
                            (o < rr && os[mid] == es && orw[mid] == er);
        if (before) lo2 = mid + 1; else hi2 = mid;
      }
      pos += lo2;
    }
    if (pos < k) {
      out_s[b * k + pos] = er == INT64_MAX ? __builtin_nan("") : es;
      out_r[b * k + pos] = er == INT64_MAX ? -1 : er;
    }
  }
  // fewer candidates than k (all of them non-padding): padding takes the rest
  for (int j = C + tid; j < k; j += RTHREADS) {
    out_s[b * k + j] = __builtin_nan("");
    out_r[b * k + j] = -1;
  }
}

// ebt_merge_packed: the co-rank merge over the packed lists as they are -- each rank's entries
// of query b (about k / R + the floor's band of them, instead of k slots mostly padding) staged
// compactly in LDS, then every entry placed at j + (entries of the other lists before it), by
// a binary search in each (score desc, row asc; equal keys ordered by list). A list found
// unsorted flags the batch incomplete (the caller merges the full lists instead): the packed
// lists come sorted from ebt_shard_pack.
// The entries one query's LDS holds: R k (every rank sending all of its k) is what a query can
// receive, but a query's entries above the catalog-wide floor number about k + the floor's band
// over all ranks together, so the room is min(R k, 2 k + 256) and a query with more (a band
// wider than k + 256: clustered data) flags the batch incomplete -- the caller's full exchange,
// as for a list cut by its capacity. At C5/8 (R 8, k 1000) that is 27 KiB instead of 94 KiB of
// LDS per query: five waves per CU instead of one for the binary searches' LDS latency.
__host__ __device__ inline int merge_packed_room(int R, int k) {
  const int64_t all = (int64_t)R * k, room = 2LL * k + 256;
  return (int)(all < room ? all : room);
}
size_t merge_packed_lds(int R, int k) {
  const size_t n = (size_t)merge_packed_room(R, k);
  return n * 8 + ((n * 4 + 15) & ~(size_t)15) + (((size_t)(3 * R + 1) * 4 + 15) & ~(size_t)15);
}

// one wave per query: 4096 queries all resident at once (16 workgroups per CU by their ~10 KiB of
// LDS at C3/8) instead of two rounds of 256-thread workgroups, each query's chain of dependent
// loads paid once
constexpr int MP_THREADS = 64;
__global__ __launch_bounds__(MP_THREADS) void merge_packed_kernel(
    const PackedSrc src, int R, int64_t B, int k, double* __restrict__ out_s,
    int64_t* __restrict__ out_r, int32_t* __restrict__ incomplete) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nmax = merge_packed_room(R, k);
  double* sc = (double*)smem;                                  // nmax
  int32_t* rw = (int32_t*)(sc + nmax);                         // nmax
  int* pst = (int*)((char*)rw + (((size_t)nmax * 4 + 15) & ~(size_t)15));  // R: packed start
  int* len = pst + R;                                          // R: entries sent
  int* off = len + R;                                          // R + 1: compact starts
  __shared__ int wsum[MP_THREADS / 64];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // 1. each rank's entries for this query (a list cut by its rank's capacity, or longer than
  //    k, makes the batch incomplete), and their compact starts (a block scan over the ranks)
  int carry = 0;
  for (int r0 = 0; r0 < R; r0 += MP_THREADS) {
    const int r = r0 + tid;
    int v = 0;
    if (r < R) {
      const int64_t s0 = pk_starts(src, r)[b], s1 = s0 + pk_lens(src, r, B)[b];
      const int64_t a = s0 < src.cap ? s0 : src.cap, e = s1 < src.cap ? s1 : src.cap;
      v = (int)(e - a < k ? e - a : k);
      pst[r] = (int)a;
      len[r] = v;
      if (s1 > src.cap || s1 - s0 > k) incomplete[0] = 1;
    }
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int base = carry, total = 0;
#pragma unroll
    for (int w = 0; w < MP_THREADS / 64; ++w) {
      base += w < wave ? wsum[w] : 0;
      total += wsum[w];
    }
    if (r < R) off[r] = base + incl - v;
    carry += total;
    __syncthreads();
  }
  if (tid == 0) off[R] = carry;
  __syncthreads();
  const int N = carry;
  if (N > nmax) {   // more than the query's room (merge_packed_room): the full exchange
    if (tid == 0) incomplete[0] = 1;
    return;
  }
  auto list_of = [&](int e) {   // the last list whose compact start is <= e (a non-empty one)
    int lo = 0, hi = R - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  // 2. the entries into LDS, four per thread in flight
  for (int e0 = tid; e0 < N; e0 += 4 * MP_THREADS) {
    double sv[4];
    int32_t rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * MP_THREADS;
      const int ec = e < N ? e : N - 1;
      const int rr = list_of(ec);
      const int64_t ix = (int64_t)pst[rr] + (ec - off[rr]);
      sv[u] = pk_scores(src, rr, B)[ix];
      rv[u] = pk_rows(src, rr, B)[ix];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * MP_THREADS;
      issued(sv[u]);
      if (e < N) {
        sc[e] = sv[u] != sv[u] ? -__builtin_inf() : sv[u];
        rw[e] = rv[u];
      }
    }
  }
  __syncthreads();
  // 3. sorted lists only
  int bad = 0;
  for (int e = tid; e < N; e += MP_THREADS) {
    const int rr = list_of(e);
    if (e + 1 < off[rr] + len[rr] && mt_before(sc[e + 1], rw[e + 1], sc[e], rw[e])) bad = 1;
  }
  if (__syncthreads_or(bad)) {
    if (tid == 0) incomplete[0] = 1;
    return;
  }
  // 4. positions: j + the entries of every other list before this one
  for (int e = tid; e < N; e += MP_THREADS) {
    const int rr = list_of(e);
    const double es = sc[e];
    const int64_t er = rw[e];
    int pos = e - off[rr];
    for (int o = 0; o < R && pos < k; ++o) {
      if (o == rr) continue;
      int lo = off[o], hi = off[o] + len[o];
      const int o0 = lo;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const bool before = mt_before(sc[mid], rw[mid], es, er) ||
                            (o < rr && sc[mid] == es && (int64_t)rw[mid] == er);
        if (before) lo = mid + 1; else hi = mid;
      }
      pos += lo - o0;
    }
    if (pos < k) {
      out_s[b * k + pos] = es;
      out_r[b * k + pos] = er;
    }
  }
  // fewer entries than k: padding takes the rest
  for (int j = N + tid; j < k; j += MP_THREADS) {
    out_s[b * k + j] = __builtin_nan("");
    out_r[b * k + j] = -1;
  }
}

int merge_topk(const double* scores, const int64_t* rows, int32_t R, int64_t B, int32_t k,
               double* out_s, int64_t* out_r, hipStream_t st) {
  if (!scores || !rows || !out_s || !out_r || R < 1 || B < 0 || k < 1 || k > MERGE_CAP / 2) {
    set_error("ebt_merge_topk: bad arguments (R=%d k=%d; k must be <= %d)", R, k, MERGE_CAP / 2);
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const int64_t n = (int64_t)R * k;
  if (R > 1 && R <= MERGE_CORANK_RMAX && n <= MERGE_CORANK_CAP) {
    const int P = next_pow2_h((int)n);
    const size_t lds = merge_corank_lds(R, P);
    set_max_lds((const void*)merge_topk_corank_kernel<DenseSrc>, (int)lds);
    hipLaunchKernelGGL(merge_topk_corank_kernel<DenseSrc>, dim3((unsigned)B), dim3(RTHREADS),
                       lds, st, DenseSrc{scores, rows}, R, B, k, P, out_s, out_r);
    return launch_check("merge_topk_corank_kernel");
  }
  const int P = next_pow2_h((int)(n < MERGE_CAP ? n : MERGE_CAP));
  set_max_lds((const void*)merge_topk_kernel, (int)(P * 16));
  hipLaunchKernelGGL(merge_topk_kernel, dim3((unsigned)B), dim3(RTHREADS), (size_t)P * 16, st,
                     scores, rows, R, B, k, P, out_s, out_r);
  return launch_check("merge_topk_kernel");
}

// ------------------------------------------------------------------------ compact exchange --
// ebt_shard_pack: per query the prefix of its sorted exact list with score >= t_floor[b] (a
// lower bound of the k-th best exact score over the whole catalog: every global top-k entry is
// in it), packed behind per-query starts. Two launches: (1) one thread per query counts its
// prefix (binary search: the predicate "real row and score >= floor" holds on a prefix of a
// sorted list), a workgroup scan gives the starts within its 256 queries and its total;
// (2) each workgroup adds the totals of the workgroups before it, writes the global starts and
// copies its entries (one per thread, the owning query found by binary search in LDS).
__global__ __launch_bounds__(SHARD_PACK_QPB) void shard_pack_count_kernel(
    const double* __restrict__ scores, const int64_t* __restrict__ rows, int64_t B, int k,
    const double* __restrict__ t_floor, uint32_t* __restrict__ hdr) {
  __shared__ int wsum[SHARD_PACK_QPB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = (int64_t)blockIdx.x * SHARD_PACK_QPB + tid;
  int cnt = 0;
  if (b < B) {
    const double tf = t_floor ? t_floor[b] : -__builtin_inf();
    const double* sr = scores + b * k;
    const int64_t* rr = rows + b * k;
    // the first position failing the predicate (it holds on a prefix), by an 8-way search:
    // each round trip loads up to 8 evenly spaced probes of [lo, hi) at once and keeps the gap
    // between the last probe passing and the first failing (k = 100: three round trips, not 7)
    int lo = 0, hi = k;
    while (lo < hi) {
      const int span = hi - lo, m = span < 8 ? span : 8;
      int p[8];
      int64_t pr[8];
      double ps[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        p[i] = lo + (int)((int64_t)(i + 1) * span / (m + 1));
        const int pc = i < m ? p[i] : lo;
        pr[i] = rr[pc];
        ps[i] = sr[pc];
      }
      int nlo = lo, nhi = hi;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (i >= m) continue;
        if (pr[i] >= 0 && ps[i] >= tf) nlo = p[i] + 1 > nlo ? p[i] + 1 : nlo;
        else nhi = p[i] < nhi ? p[i] : nhi;
      }
      lo = nlo;
      hi = nhi;
    }
    cnt = lo;
  }
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < SHARD_PACK_QPB / 64; ++w) {
    base += w < wave ? wsum[w] : 0;
    total += wsum[w];
  }
  if (b < B) hdr[b] = (uint32_t)(base + incl - cnt);  // start within the workgroup
  if (tid == 0) hdr[2 * B + blockIdx.x] = (uint32_t)total;
}

// (64 queries per workgroup -- 64 workgroups at B = 4096, not 16 -- and SHARD_PACK_COPY_THREADS
// threads: a workgroup's ~15 x 64 entries at C3/8 in four rounds)
constexpr int SHARD_PACK_COPY_THREADS = 256;
__global__ __launch_bounds__(SHARD_PACK_COPY_THREADS) void shard_pack_copy_kernel(
    const double* __restrict__ scores, const int64_t* __restrict__ rows, int64_t B, int k,
    int64_t cap, char* __restrict__ send) {
  __shared__ uint32_t lst[SHARD_PACK_QPB + 1];
  __shared__ uint32_t gbase;
  uint32_t* hdr = (uint32_t*)send;
  double* os = (double*)(send + shard_pack_hdr_bytes(B));
  int32_t* orow = (int32_t*)(send + shard_pack_hdr_bytes(B) + cap * 8);
  const int tid = threadIdx.x;
  const int64_t q0 = (int64_t)blockIdx.x * SHARD_PACK_QPB;
  const int nq = B - q0 < SHARD_PACK_QPB ? (int)(B - q0) : SHARD_PACK_QPB;
  const uint32_t* tot = hdr + 2 * B;
  if (tid < 64) {  // the totals of the workgroups before this one
    uint32_t s = 0;
    for (int i = tid; i < (int)blockIdx.x; i += 64) s += tot[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (tid == 0) gbase = s;
  }
  if (tid < nq) lst[tid] = hdr[q0 + tid];
  if (tid == 0) lst[nq] = tot[blockIdx.x];
  __syncthreads();
  const uint32_t g0 = gbase, n = lst[nq];
  if (tid < nq) {
    hdr[q0 + tid] = g0 + lst[tid];                // start
    hdr[B + q0 + tid] = lst[tid + 1] - lst[tid];  // len
  }
  for (uint32_t t = tid; t < n; t += SHARD_PACK_COPY_THREADS) {
    int lo = 0, hi = nq - 1;  // the last query whose start <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (lst[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const int64_t b = q0 + lo, j = t - lst[lo], pos = (int64_t)g0 + t;
    if (pos < cap) {
      os[pos] = scores[b * k + j];
      orow[pos] = (int32_t)rows[b * k + j];
    }
  }
}

// The pack's second half when the sharded rescore counted already (len[b] in the header): each
// workgroup's base is the sum of len over the queries before it (at most B values, L2-resident:
// no block totals, so no counting launch), then the starts and the copy as shard_pack_copy_kernel.
__global__ __launch_bounds__(SHARD_PACK_COPY_THREADS) void shard_pack_lens_kernel(
    const double* __restrict__ scores, const int64_t* __restrict__ rows, int64_t B, int k,
    int64_t cap, char* __restrict__ send) {
  __shared__ uint32_t lst[SHARD_PACK_QPB + 1];
  __shared__ uint32_t part[SHARD_PACK_COPY_THREADS / 64];
  uint32_t* hdr = (uint32_t*)send;
  const uint32_t* len = hdr + B;
  double* os = (double*)(send + shard_pack_hdr_bytes(B));
  int32_t* orow = (int32_t*)(send + shard_pack_hdr_bytes(B) + cap * 8);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t q0 = (int64_t)blockIdx.x * SHARD_PACK_QPB;
  const int nq = B - q0 < SHARD_PACK_QPB ? (int)(B - q0) : SHARD_PACK_QPB;
  uint32_t sum = 0;   // the queries before this workgroup's
  for (int64_t i = tid; i < q0; i += SHARD_PACK_COPY_THREADS) sum += len[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if (lane == 0) part[wave] = sum;
  if (wave == 0) {    // this workgroup's queries: an inclusive scan of their lens
    uint32_t v = lane < nq ? len[q0 + lane] : 0u;
    const uint32_t incl = wave_scan_add_u32(v);
    lst[lane + 1] = incl;
    if (lane == 0) lst[0] = 0u;
  }
  __syncthreads();
  uint32_t g0 = 0;
#pragma unroll
  for (int w = 0; w < SHARD_PACK_COPY_THREADS / 64; ++w) g0 += part[w];
  const uint32_t n = lst[nq];
  if (tid < nq) hdr[q0 + tid] = g0 + lst[tid];   // start
  for (uint32_t t = tid; t < n; t += SHARD_PACK_COPY_THREADS) {
    int lo = 0, hi = nq - 1;  // the last query whose start <= t (an empty one is skipped)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (lst[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const int64_t b = q0 + lo, j = t - lst[lo], pos = (int64_t)g0 + t;
    if (pos < cap) {
      os[pos] = scores[b * k + j];
      orow[pos] = (int32_t)rows[b * k + j];
    }
  }
}

int shard_pack_lens(const double* scores, const int64_t* rows, int64_t B, int32_t k,
                    int64_t cap, void* send, hipStream_t st) {
  hipLaunchKernelGGL(shard_pack_lens_kernel, dim3((unsigned)ceil_div(B, SHARD_PACK_QPB)),
                     dim3(SHARD_PACK_COPY_THREADS), 0, st, scores, rows, B, k, cap, (char*)send);
  return launch_check("shard_pack_lens_kernel");
}

int64_t shard_list_width(int32_t k, int32_t world) {
  const int64_t w = (3 * (int64_t)k + 2 * world - 1) / (2 * world) + 8;  // ceil(1.5 k / R) + 8
  return w < k ? w : k;
}

// ---------------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------------
// Exact screen (EBT_FLAG_EXACT): S[b][j] = (float)((q64_b . c_j) / gnorm64_j), the rescore's own
// float64 arithmetic rounded once to f32, for every row of a chunk. This is the last-resort
// screen for a query whose f16/bf16 screen cannot be certified even at k' = 4096 (a cluster of
// more than k' rows within the f16 error bound of the k-th score): its only error is the f32
// rounding (|score| <= 1, so <= 2^-25) plus float64 round-off, so EXACT_EPS certifies anything
// short of true f32-level ties. Plain FMA tiling (64 queries x 64 rows per workgroup, 4 x 4 per
// thread): it runs for a handful of queries, never on the hot path.
// ---------------------------------------------------------------------------------------------
constexpr int XT = 64, XK = 16;

template <int DT>
__global__ __launch_bounds__(256) void screen_exact_kernel(
    const double* __restrict__ q64, int64_t B, int d, const void* __restrict__ cat, int64_t ld,
    const double* __restrict__ gnorm, int64_t n_rows, float* __restrict__ S, int64_t ld_s) {
  __shared__ double qs[XK][XT + 1], cs[XK][XT + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * XT, b0 = (int64_t)blockIdx.y * XT;
  double acc[4][4] = {};
  for (int k0 = 0; k0 < d; k0 += XK) {
    // the tile's 4 elements per thread loaded before any is stored (guarded loads would each
    // be waited for in turn): out-of-range indices read a clamped in-range element, then 0
    constexpr int NE = XT * XK / 256;
    double cv[NE], qv[NE];
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      const int rr = e / XK, kk = e % XK;
      const int64_t row = r0 + rr, qb = b0 + rr;
      const int kc = k0 + kk < d ? k0 + kk : d - 1;
      cv[u] = load_as_f64<DT>(cat, (row < n_rows ? row : n_rows - 1) * ld + kc);
      qv[u] = q64[(qb < B ? qb : B - 1) * d + kc];
    }
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + 256 * u;
      const int rr = e / XK, kk = e % XK;
      const int64_t row = r0 + rr, qb = b0 + rr;
      const bool kin = k0 + kk < d;
      cs[kk][rr] = (kin && row < n_rows) ? cv[u] : 0.0;
      qs[kk][rr] = (kin && qb < B) ? qv[u] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < XK; ++kk) {
      double a[4], c[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = qs[kk][ty * 4 + i];
        c[i] = cs[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fma(a[i], c[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t qb = b0 + ty * 4 + i;
    if (qb >= B) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = r0 + tx * 4 + j;
      if (row < n_rows) {
        const double v = acc[i][j] / gnorm[row];
        S[qb * ld_s + row] = (v == v) ? (float)v : -__builtin_inff();
      }
    }
  }
}

int screen_exact(const double* q64, int64_t B, int32_t d, const void* cat, int dtype, int64_t ld,
                 const double* gnorm, int64_t n_rows, float* S, int64_t ld_s, hipStream_t st) {
  if (!q64 || !cat || !gnorm || !S || B < 0 || d < 1 || ld < d || n_rows < 0 || ld_s < n_rows ||
      dtype < 0 || dtype > 3) {
    set_error("ebt_screen_exact: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0 || n_rows == 0) return EBT_OK;
  if (ceil_div(B, XT) > 65535) {
    set_error("ebt_screen_exact: batch too large");
    return EBT_EINVAL;
  }
  dim3 grid((unsigned)ceil_div(n_rows, XT), (unsigned)ceil_div(B, XT)), block(256);
  switch (dtype) {
    case EBT_F32:
      hipLaunchKernelGGL(screen_exact_kernel<EBT_F32>, grid, block, 0, st, q64, B, d, cat, ld,
                         gnorm, n_rows, S, ld_s);
      break;
    case EBT_BF16:
      hipLaunchKernelGGL(screen_exact_kernel<EBT_BF16>, grid, block, 0, st, q64, B, d, cat, ld,
                         gnorm, n_rows, S, ld_s);
      break;
    case EBT_F16:
      hipLaunchKernelGGL(screen_exact_kernel<EBT_F16>, grid, block, 0, st, q64, B, d, cat, ld,
                         gnorm, n_rows, S, ld_s);
      break;
    default:
      hipLaunchKernelGGL(screen_exact_kernel<EBT_F64>, grid, block, 0, st, q64, B, d, cat, ld,
                         gnorm, n_rows, S, ld_s);
      break;
  }
  return launch_check("screen_exact_kernel");
}

// ---------------------------------------------------------------------------------------------
// Two-phase certification over a row-sharded catalog (distributed.py). Phase 1 on every rank:
// ebt_cosine_screen leaves the shard's k' best approx candidates (GLOBAL rows) -> all-gather ->
// the k' best of all shards (same on every rank). Phase 2: each rank computes the exact float64
// score of the merged candidates IT owns (rescore_owned: 0 elsewhere), an all-reduce (SUM)
// completes them, and finalize_topk sorts and certifies exactly like rescore_kernel. A row
// outside the merged list has approx <= the merged k'-th (it lost a merge or a shard's own
// selection, whose k'-th is <= the merged k'-th) or was dropped by a segment threshold below
// the list's k-th - 2 eps, so "merged[k'-1] < merged[k-1] - 2 eps" certifies the global top-k.
// ---------------------------------------------------------------------------------------------
__global__ void export_list_kernel(int64_t* __restrict__ rows, int64_t B, int kprime,
                                   int64_t row_offset, const int* __restrict__ ovf,
                                   const float* __restrict__ eps, int32_t* __restrict__ ovf_out,
                                   float* __restrict__ eps_out) {
  const int64_t b = blockIdx.x;
  for (int j = threadIdx.x; j < kprime; j += blockDim.x) {
    const int64_t r = rows[b * kprime + j];
    rows[b * kprime + j] = r >= 0 ? r + row_offset : -1;
  }
  if (threadIdx.x == 0) {
    ovf_out[b] = ovf ? (ovf[b] > 0 ? ovf[b] : 0) : 0;  // 1 overflow, 2 speculation failed
    eps_out[b] = eps[b];
  }
}

int export_list(int64_t* rows, int64_t B, int32_t kprime, int64_t row_offset, const int* ovf,
                const float* eps, int32_t* ovf_out, float* eps_out, hipStream_t st) {
  if (B <= 0) return EBT_OK;
  hipLaunchKernelGGL(export_list_kernel, dim3((unsigned)B), dim3(256), 0, st, rows, B, kprime,
                     row_offset, ovf, eps, ovf_out, eps_out);
  return launch_check("export_list_kernel");
}

template <int DT, bool VEC>
__global__ __launch_bounds__(RTHREADS) void rescore_owned_kernel(
    const double* __restrict__ q64, int d, const void* __restrict__ cat, int64_t ld,
    const double* __restrict__ gnorm, int64_t row_offset, int64_t n_local,
    const float* __restrict__ cand_vals, const int64_t* __restrict__ cand_rows, int kprime, int k,
    const float* __restrict__ eps, double* __restrict__ exact) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* qs = (double*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b = blockIdx.x;
  stage_f64(qs, q64 + b * d, d);
  __syncthreads();
  const float* cv = cand_vals + b * kprime;
  const double cut = (double)cv[k - 1] - 2.0 * (double)eps[b];
  for (int c = wave; c < kprime; c += RTHREADS / 64) {
    const int64_t g = cand_rows[b * kprime + c];
    const int64_t row = g - row_offset;
    const bool mine = g >= 0 && row >= 0 && row < n_local && !((double)cv[c] < cut);
    double s = 0.0;
    if (mine) {
      if constexpr (VEC) {
        constexpr int ES = (DT == EBT_F64) ? 8 : (DT == EBT_F32 ? 4 : 2);
        constexpr int PER = 16 / ES;
        const char* base = (const char*)cat + row * ld * ES;
        for (int ch = lane; ch < d / PER; ch += 64) {
          const uint4 raw = *(const uint4*)(base + (int64_t)ch * 16);
          const int j0 = ch * PER;
          if constexpr (DT == EBT_F32) {
            const float* f = (const float*)&raw;
#pragma unroll
            for (int e = 0; e < 4; ++e) s += qs[j0 + e] * (double)f[e];
          } else if constexpr (DT == EBT_F64) {
            const double* f = (const double*)&raw;
            s += qs[j0] * f[0] + qs[j0 + 1] * f[1];
          } else {
            const uint16_t* h = (const uint16_t*)&raw;
#pragma unroll
            for (int e = 0; e < 8; ++e)
              s += qs[j0 + e] * (DT == EBT_BF16 ? bf16_bits_to_f64(h[e]) : f16_bits_to_f64(h[e]));
          }
        }
      } else {
        for (int j = lane; j < d; j += 64) s += qs[j] * load_as_f64<DT>(cat, row * ld + j);
      }
      s = wave_sum_f64(s);
    }
    if (lane == 0) exact[b * kprime + c] = mine ? s / gnorm[row] : 0.0;
  }
}

int rescore_owned(const double* q64, int64_t B, int32_t d, const void* cat, int dtype, int64_t ld,
                  const double* gnorm, int64_t row_offset, int64_t n_local,
                  const float* cand_vals, const int64_t* cand_rows, int32_t kprime, int32_t k,
                  const float* eps, double* exact, hipStream_t st) {
  if (!q64 || !cat || !gnorm || !cand_vals || !cand_rows || !eps || !exact || B < 0 || d <= 0 ||
      ld < d || k < 1 || kprime < k || kprime > 4096 || dtype < 0 || dtype > 3 || n_local < 0) {
    set_error("ebt_rescore_owned: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const size_t lds = (size_t)((d + 1) & ~1) * 8;
  if (lds > 150 * 1024) {
    set_error("ebt_rescore_owned: d=%d exceeds LDS", d);
    return EBT_EUNSUPPORTED;
  }
  const int es = dtype == EBT_F64 ? 8 : (dtype == EBT_F32 ? 4 : 2);
  const bool vec = (((uintptr_t)cat & 15) == 0) && ((ld * es) % 16 == 0) &&
                   (((int64_t)d * es) % 16 == 0);
  dim3 grid((unsigned)B), block(RTHREADS);
#define EBT_RO(DT)                                                                              \
  set_max_lds((const void*)rescore_owned_kernel<DT, true>, (int)lds);                          \
  set_max_lds((const void*)rescore_owned_kernel<DT, false>, (int)lds);                         \
  if (vec)                                                                                      \
    hipLaunchKernelGGL((rescore_owned_kernel<DT, true>), grid, block, lds, st, q64, d, cat, ld, \
                       gnorm, row_offset, n_local, cand_vals, cand_rows, kprime, k, eps, exact); \
  else                                                                                          \
    hipLaunchKernelGGL((rescore_owned_kernel<DT, false>), grid, block, lds, st, q64, d, cat,    \
                       ld, gnorm, row_offset, n_local, cand_vals, cand_rows, kprime, k, eps,    \
                       exact);
  switch (dtype) {
    case EBT_F32: EBT_RO(EBT_F32) break;
    case EBT_BF16: EBT_RO(EBT_BF16) break;
    case EBT_F16: EBT_RO(EBT_F16) break;
    default: EBT_RO(EBT_F64) break;
  }
#undef EBT_RO
  return launch_check("rescore_owned_kernel");
}

// Sort the merged candidates above the cut by (exact desc, row asc), keep k, certify.
__global__ __launch_bounds__(RTHREADS) void finalize_topk_kernel(
    const float* __restrict__ cand_vals, const int64_t* __restrict__ cand_rows,
    const double* __restrict__ exact, int kprime, int kpp, int k, int64_t n_rows,
    const float* __restrict__ eps, const int32_t* __restrict__ ovf, double* __restrict__ out_s,
    int64_t* __restrict__ out_r, int32_t* __restrict__ certified) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* sc = (double*)smem;
  int64_t* rw = (int64_t*)(sc + kpp);
  __shared__ int nvalid;
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  if (tid == 0) nvalid = 0;
  __syncthreads();
  const float* cv = cand_vals + b * kprime;
  const double cut = (double)cv[k - 1] - 2.0 * (double)eps[b];
  int myvalid = 0;
  for (int c = tid; c < kpp; c += RTHREADS) {
    const int64_t r = c < kprime ? cand_rows[b * kprime + c] : -1;
    if (r >= 0) {
      ++myvalid;
      const double v = exact[b * kprime + c];
      sc[c] = ((double)cv[c] < cut || !(v == v)) ? -__builtin_inf() : v;
      rw[c] = r;
    } else {
      sc[c] = -__builtin_inf();
      rw[c] = INT64_MAX;
    }
  }
  if (myvalid) atomicAdd(&nvalid, myvalid);
  __syncthreads();
  bitonic_pairs(sc, rw, kpp);
  for (int j = tid; j < k; j += RTHREADS) {
    const int64_t r = rw[j];
    if (r == INT64_MAX) {
      out_s[b * k + j] = __builtin_nan("");
      out_r[b * k + j] = -1;
    } else {
      out_s[b * k + j] = sc[j];
      out_r[b * k + j] = r;
    }
  }
  if (tid == 0) {
    int ok = 1;
    if (nvalid >= kprime && n_rows > kprime)
      ok = (double)cv[kprime - 1] < (double)cv[k - 1] - 2.0 * (double)eps[b];
    if (ovf && ovf[b]) ok = -1;
    certified[b] = ok;
  }
}

int finalize_topk(const float* cand_vals, const int64_t* cand_rows, const double* exact,
                  int64_t B, int32_t kprime, int32_t k, int64_t n_rows, const float* eps,
                  const int32_t* ovf, double* out_s, int64_t* out_r, int32_t* certified,
                  hipStream_t st) {
  if (!cand_vals || !cand_rows || !exact || !eps || !out_s || !out_r || !certified || B < 0 ||
      k < 1 || kprime < k || kprime > 4096) {
    set_error("ebt_finalize_topk: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const int kpp = next_pow2_h(kprime);
  const size_t lds = (size_t)kpp * 16;
  set_max_lds((const void*)finalize_topk_kernel, (int)lds);
  hipLaunchKernelGGL(finalize_topk_kernel, dim3((unsigned)B), dim3(RTHREADS), lds, st, cand_vals,
                     cand_rows, exact, kprime, kpp, k, n_rows, eps, ovf, out_s, out_r, certified);
  return launch_check("finalize_topk_kernel");
}

// ---------------------------------------------------------------------------------------------
// Row-sharded per-shard path (distributed.py), after the floor all-gather: the catalog-wide floor
// and the certificate adjustment in two launches instead of ~17 small torch ops.
// union_floor: g = [R][B][ld] f32 (the shards' k best approx in columns [0, ld-1), their eps in
// column ld-1); t_floor[b] = the k-th largest of g[r][b][j] - g[r][b][ld-1] over r, j (float64,
// exact differences of two floats; NaN counts as -inf). One wave per query: bisection over the
// order-preserving 64-bit keys of the doubles, counts by a strided pass over the R*(ld-1) values.
__device__ __forceinline__ uint64_t d2key(double x) {
  if (!(x == x)) return 0ull;  // NaN -> below -inf
  uint64_t u = (uint64_t)__double_as_longlong(x);
  if (x == 0.0) u = 0ull;      // -0 == +0
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double key2d(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)u);
}

__global__ __launch_bounds__(256) void union_floor_kernel(const float* __restrict__ g, int R,
                                                          int64_t B, int ld, int k,
                                                          double* __restrict__ t_floor,
                                                          uint32_t* __restrict__ zero2) {
  if (zero2 && blockIdx.x == 0 && threadIdx.x < 2) zero2[threadIdx.x] = 0u;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const int per = ld - 1, n = R * per;
  auto val = [&](int i) {
    const int r = i / per, j = i - r * per;
    const float* row = g + ((int64_t)r * B + b) * ld;
    return (double)row[j] - (double)row[per];
  };
  auto count_ge = [&](uint64_t t) {
    int c = 0;
    for (int i = lane; i < n; i += 64) c += d2key(val(i)) >= t ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    return c;
  };
  // the largest key t with count(key >= t) >= k (key 0 = NaN / below everything)
  uint64_t lo = 0ull, hi = ~0ull;
  while (lo < hi) {
    const uint64_t mid = lo + ((hi - lo) >> 1) + 1;
    if (count_ge(mid) >= k) lo = mid;
    else hi = mid - 1;
  }
  if (lane == 0) t_floor[b] = lo == 0ull ? -__builtin_inf() : key2d(lo);
}

// The same bisection with the query's R*(ld-1) keys held in registers (up to 32 per lane), made
// once (all loads issued before the search), and the counts as ballot popcounts: W = 1 (one wave per query, n <= 2048: C3/8 has
// 8 x 100) or 4 (one 256-thread workgroup per query, n <= 8192: C5/8 has 8 x 1000; the waves'
// counts meet in LDS). The strided form above re-read every value from memory, with a
// division, in each of its 64 steps (0.39 ms per 4096-query C3/8 batch).
constexpr int UF_PL = 32;
// PL: key slots per lane, a compile-time bound (the launch picks the smallest of 4/8/16/32 that
// holds n): the count loop is then a fixed sequence of compare + popcount, no per-slot test.
// The bisection bounds are wave-uniform (readfirstlane): a scalar loop.
template <int W, int PL>
__global__ __launch_bounds__(256) void union_floor_reg_kernel(const float* __restrict__ g, int R,
                                                              int64_t B, int ld, int k,
                                                              double* __restrict__ t_floor,
                                                              uint32_t* __restrict__ zero2) {
  // (zero2: two words the caller needs zeroed before its next kernel -- the sharded step's pack
  // counter and "incomplete" flag, one memset launch less per step)
  if (zero2 && blockIdx.x == 0 && threadIdx.x < 2) zero2[threadIdx.x] = 0u;
  __shared__ int wc[2][4];
  __shared__ uint64_t wmm[2][4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t b = W == 1 ? (int64_t)blockIdx.x * 4 + (tid >> 6) : (int64_t)blockIdx.x;
  if (W == 1 && b >= B) return;
  const int per = ld - 1, n = R * per;
  const int t0 = W == 1 ? lane : tid;
  constexpr int STEP = 64 * W;
  if (n < k) {   // fewer values than k: no k-th largest
    if (t0 == 0) t_floor[b] = -__builtin_inf();
    return;
  }
  // every slot's two loads issued before any is used (a guarded load per slot would wait for
  // each in turn): indices past n re-read entry n - 1 and are masked to key 0 afterwards
  float v[PL], ev[PL];
#pragma unroll
  for (int e = 0; e < PL; ++e) {
    const int i0 = t0 + STEP * e, i = i0 < n ? i0 : n - 1;   // entry i: list i / per, i % per
    const int r = i / per, j = i - r * per;
    const float* row = g + ((int64_t)r * B + b) * ld;
    v[e] = row[j];
    ev[e] = row[per];
  }
  uint64_t key[PL];
  uint64_t mn = ~0ull, mx = 0ull;
#pragma unroll
  for (int e = 0; e < PL; ++e) {
    const bool in = t0 + STEP * e < n;
    key[e] = in ? d2key((double)v[e] - (double)ev[e]) : 0ull;
    if (in) {
      mn = key[e] < mn ? key[e] : mn;
      mx = key[e] > mx ? key[e] : mx;
    }
  }
  // the k-th largest key lies in [min key, max key]: bisect that bracket, not all 64 bits
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t a = __shfl_xor(mn, o, 64), c = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = c > mx ? c : mx;
  }
  if (W > 1) {
    if (lane == 0) {
      wmm[0][tid >> 6] = mn;
      wmm[1][tid >> 6] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      mn = wmm[0][w] < mn ? wmm[0][w] : mn;
      mx = wmm[1][w] > mx ? wmm[1][w] : mx;
    }
  }
  auto uni = [](uint64_t x) {
    const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi32 << 32) | lo32;
  };
  uint64_t lo = uni(mn), hi = uni(mx);   // count(key >= mn) = n >= k
  int parity = 0;
  while (lo < hi) {
    const uint64_t mid = lo + ((hi - lo) >> 1) + 1;
    int c = 0;
#pragma unroll
    for (int e = 0; e < PL; ++e) c += __popcll(__ballot(key[e] >= mid));
    if (W > 1) {
      if (lane == 0) wc[parity][tid >> 6] = c;
      __syncthreads();
      c = wc[parity][0] + wc[parity][1] + wc[parity][2] + wc[parity][3];
      parity ^= 1;   // the other buffer next step: no second barrier before the next write
    }
    c = __builtin_amdgcn_readfirstlane(c);
    if (c >= k) lo = mid;
    else hi = mid - 1;
  }
  if (t0 == 0) t_floor[b] = lo == 0ull ? -__builtin_inf() : key2d(lo);
}

// cert[b] = -1 (rerun unfused) when the fused screen overflowed (ovf[b] != 0) or the shared
// threshold may have dropped a global top-k row (theta[b] > t_floor[b] - eps[b]); -2 stays.
__global__ void certify_cut_kernel(int32_t* __restrict__ cert, const int32_t* __restrict__ ovf,
                                   const float* __restrict__ theta,
                                   const double* __restrict__ t_floor,
                                   const float* __restrict__ eps, int64_t B) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B || cert[b] == -2) return;
  bool drop = ovf[b] != 0;
  if (theta) drop |= !((double)theta[b] <= t_floor[b] - (double)eps[b]);
  if (drop) cert[b] = -1;
}

}  // namespace ebt

namespace ebt {
int union_floor(const float* gathered, int32_t R, int64_t B, int32_t ld, int32_t k,
                double* t_floor, hipStream_t stream, uint32_t* zero2);
}
extern "C" int ebt_union_floor(const float* gathered, int32_t R, int64_t B, int32_t ld, int32_t k,
                               double* t_floor, void* stream) {
  return ebt::union_floor(gathered, R, B, ld, k, t_floor, (hipStream_t)stream, nullptr);
}
int ebt::union_floor(const float* gathered, int32_t R, int64_t B, int32_t ld, int32_t k,
                     double* t_floor, hipStream_t stream, uint32_t* zero2) {
  if (!gathered || !t_floor || R < 1 || B < 0 || ld < 2 || k < 1 || (int64_t)R * (ld - 1) > (1 << 30)) {
    set_error("ebt_union_floor: bad arguments (R=%d B=%lld ld=%d k=%d)", R, (long long)B, ld, k);
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const int64_t n = (int64_t)R * (ld - 1);
  const hipStream_t st = (hipStream_t)stream;
  const dim3 g1((unsigned)ceil_div(B, 4)), g4((unsigned)B), blk(256);
#define EBT_UF(W, PL, G)                                                                       \
  {                                                                                           \
    hipLaunchKernelGGL((union_floor_reg_kernel<W, PL>), G, blk, 0, st, gathered, R, B, ld, k, \
                       t_floor, zero2);                                                       \
    return launch_check("union_floor_reg_kernel");                                            \
  }
  if (n <= 64 * 4) EBT_UF(1, 4, g1)
  if (n <= 64 * 8) EBT_UF(1, 8, g1)
  if (n <= 64 * 16) EBT_UF(1, 16, g1)
  if (n <= 64 * UF_PL) EBT_UF(1, 32, g1)
  if (n <= 256 * 16) EBT_UF(4, 16, g4)
  if (n <= 256 * UF_PL) EBT_UF(4, 32, g4)
#undef EBT_UF
  hipLaunchKernelGGL(union_floor_kernel, dim3((unsigned)ceil_div(B, 4)), dim3(256), 0,
                     (hipStream_t)stream, gathered, R, B, ld, k, t_floor, zero2);
  return launch_check("union_floor_kernel");
}

extern "C" int ebt_certify_cut(int32_t* cert, const int32_t* ovf, const float* theta,
                               const double* t_floor, const float* eps, int64_t B, void* stream) {
  using namespace ebt;
  if (!cert || !ovf || B < 0 || (theta && (!t_floor || !eps))) {
    set_error("ebt_certify_cut: bad arguments");
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  hipLaunchKernelGGL(certify_cut_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0,
                     (hipStream_t)stream, cert, ovf, theta, t_floor, eps, B);
  return launch_check("certify_cut_kernel");
}

extern "C" int64_t ebt_shard_list_width(int32_t k, int32_t world) {
  if (k < 1 || world < 1) return 0;
  return ebt::shard_list_width(k, world);
}

extern "C" int64_t ebt_shard_pack_cap(int64_t B, int32_t k, int32_t world, int64_t n_global) {
  using namespace ebt;
  // the packed merge holds R k entries in LDS; rows travel as int32
  // (the u32 starts count up to B k entries per rank)
  if (B < 1 || k < 1 || world < 2 || world > MERGE_CORANK_RMAX ||
      (int64_t)world * k > MERGE_CORANK_CAP || n_global >= (1LL << 31) ||
      B * (int64_t)k >= (1LL << 31))
    return 0;
  const int64_t cap = B * shard_list_width(k, world);
  return cap < (1LL << 31) ? cap : 0;
}

extern "C" size_t ebt_shard_pack_bytes(int64_t B, int64_t cap) {
  if (B < 1 || cap < 1) return 0;
  return (size_t)((ebt::shard_pack_hdr_bytes(B) + cap * 12 + 255) & ~(int64_t)255);
}

extern "C" int ebt_shard_pack(const double* scores, const int64_t* rows, int64_t B, int32_t k,
                              const double* t_floor, int64_t cap, void* send, void* stream) {
  using namespace ebt;
  if (!scores || !rows || !send || B < 1 || B >= (1LL << 31) || k < 1 || cap < 1 ||
      cap >= (1LL << 31)) {
    set_error("ebt_shard_pack: bad arguments (B=%lld k=%d cap=%lld)", (long long)B, k,
              (long long)cap);
    return EBT_EINVAL;
  }
  const hipStream_t st = (hipStream_t)stream;
  const unsigned grid = (unsigned)ceil_div(B, SHARD_PACK_QPB);
  hipLaunchKernelGGL(shard_pack_count_kernel, dim3(grid), dim3(SHARD_PACK_QPB), 0, st, scores,
                     rows, B, k, t_floor, (uint32_t*)send);
  int rc = launch_check("shard_pack_count_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(shard_pack_copy_kernel, dim3(grid), dim3(SHARD_PACK_COPY_THREADS), 0, st,
                     scores, rows, B, k, cap, (char*)send);
  return launch_check("shard_pack_copy_kernel");
}

extern "C" int ebt_merge_packed(const void* recv, int32_t R, int64_t B, int32_t k, int64_t cap,
                                double* out_scores, int64_t* out_rows, int32_t* incomplete,
                                void* stream) {
  using namespace ebt;
  if (!recv || !out_scores || !out_rows || !incomplete || R < 1 || R > MERGE_CORANK_RMAX ||
      B < 1 || k < 1 || cap < 1 || (int64_t)R * k > MERGE_CORANK_CAP) {
    set_error("ebt_merge_packed: bad arguments (R=%d B=%lld k=%d cap=%lld; R k <= %d)", R,
              (long long)B, k, (long long)cap, MERGE_CORANK_CAP);
    return EBT_EINVAL;
  }
  const size_t lds = merge_packed_lds(R, k);
  set_max_lds((const void*)merge_packed_kernel, (int)lds);
  const PackedSrc src{(const char*)recv, (int64_t)ebt_shard_pack_bytes(B, cap), cap};
  hipLaunchKernelGGL(merge_packed_kernel, dim3((unsigned)B), dim3(MP_THREADS), lds,
                     (hipStream_t)stream, src, R, B, k, out_scores, out_rows, incomplete);
  return launch_check("merge_packed_kernel");
}

// ------------------------------------------------------------------------ floor all-gather --
// ebt_floor_pack: out[b] = (the w largest of lv[b][0 .. n), n = min(k_eff, ld), then eps[b]) as
// [B][w + 1] f32 -- what each shard sends for the catalog-wide floor. The list may be
// partitioned (the wave merge's [0, k-1) in any order), so the w largest are selected: one wave
// per query, order-preserving keys in registers, the w-th largest key by bisection (ballot
// counts), then the keys above it and as many equal to it as fit, compacted by ballot prefix.
// Only the multiset of values matters to ebt_union_floor, so ties at the cut may go either way.
namespace ebt {
template <int PL>
__global__ __launch_bounds__(256) void floor_pack_kernel(const float* __restrict__ lv, int64_t ld,
                                                         int64_t B, int n, int w,
                                                         const float* __restrict__ eps,
                                                         float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* src = lv + b * ld;
  float* dst = out + b * (w + 1);
  uint32_t key[PL];
#pragma unroll
  for (int e = 0; e < PL; ++e) {  // clamped loads, all in flight, masked afterwards
    const int j = lane + 64 * e;
    const float v = n > 0 ? src[j < n ? j : n - 1] : 0.f;
    key[e] = j < n ? f2key(v) : 0u;
  }
  uint32_t t = 0u;  // the w-th largest key (0: fewer than w valid values)
  if (n > w) {
    uint32_t mn = ~0u, mx = 0u;
#pragma unroll
    for (int e = 0; e < PL; ++e) {
      if (key[e]) mn = key[e] < mn ? key[e] : mn;
      mx = key[e] > mx ? key[e] : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t a = __shfl_xor(mn, o, 64), c = __shfl_xor(mx, o, 64);
      mn = a < mn ? a : mn;
      mx = c > mx ? c : mx;
    }
    auto count_ge = [&](uint32_t x) {
      int c = 0;
#pragma unroll
      for (int e = 0; e < PL; ++e) c += __popcll(__ballot(key[e] >= x));
      return c;
    };
    mn = __builtin_amdgcn_readfirstlane(mn);
    mx = __builtin_amdgcn_readfirstlane(mx);
    if (count_ge(mn) >= w) {  // else fewer than w valid values: t = 0
      uint32_t lo = mn, hi = mx;  // invariant: count_ge(lo) >= w
      while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1) + 1u;
        if (count_ge(mid) >= w) lo = mid;
        else hi = mid - 1u;
      }
      t = lo;
    }
  }
  // keys > t first, then keys == t (t > 0), at most w in all; -inf past them
  int base = 0;
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int e = 0; e < PL; ++e) {
      const bool pick = key[e] != 0u && (pass == 0 ? (n <= w || key[e] > t) : (n > w && t != 0u && key[e] == t));
      const uint64_t m = __ballot(pick);
      const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (pick && pos < w) dst[pos] = key2f(key[e]);
      base += __popcll(m);
    }
  }
  for (int j = (base < w ? base : w) + lane; j < w; j += 64) dst[j] = -__builtin_inff();
  if (lane == 0) dst[w] = eps ? eps[b] : -__builtin_inff();
}
}  // namespace ebt

extern "C" int ebt_floor_pack(const float* list_vals, int64_t ld, int64_t B, int32_t k_eff,
                              int32_t w, const float* eps, float* out, void* stream) {
  using namespace ebt;
  if (!list_vals || !out || B < 0 || ld < 1 || k_eff < 0 || w < 1 || k_eff > 4096) {
    set_error("ebt_floor_pack: bad arguments (ld=%lld k_eff=%d w=%d; k_eff <= 4096)",
              (long long)ld, k_eff, w);
    return EBT_EINVAL;
  }
  if (B == 0) return EBT_OK;
  const int n = k_eff < ld ? k_eff : (int)ld;
  const hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)ceil_div(B, 4)), blk(256);
  if (n < 1) {  // nothing valid: -inf everywhere, then eps (PL = 1 over an empty list)
    hipLaunchKernelGGL((floor_pack_kernel<1>), grid, blk, 0, st, list_vals, ld, B, 0, w, eps, out);
    return launch_check("floor_pack_kernel");
  }
  if (n <= 64 * 4)
    hipLaunchKernelGGL((floor_pack_kernel<4>), grid, blk, 0, st, list_vals, ld, B, n, w, eps, out);
  else if (n <= 64 * 16)
    hipLaunchKernelGGL((floor_pack_kernel<16>), grid, blk, 0, st, list_vals, ld, B, n, w, eps, out);
  else
    hipLaunchKernelGGL((floor_pack_kernel<64>), grid, blk, 0, st, list_vals, ld, B, n, w, eps, out);
  return launch_check("floor_pack_kernel");
}
