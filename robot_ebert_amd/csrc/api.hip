// extern "C" entry points of libebert.so (declared in include/ebert.h), the pipeline
// orchestrator ebt_cosine_topk_prepared, the per-stage hipEvent timer and error reporting.
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

namespace ebt {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return EBT_OK;
  set_error("%s: %s", what, hipGetErrorString(e));
  return EBT_EHIP;
}

int launch_check(const char* what) { return hip_check(hipGetLastError(), what); }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device) and larger size:
// the launch paths ask before every launch, and the runtime call costs host time per batch
// (the attribute is a permission, not an allocation: a smaller launch after a larger one is
// unaffected).
void set_max_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::vector<std::pair<std::pair<const void*, int>, int>> seen;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  for (auto& e : seen)
    if (e.first.first == fn && e.first.second == dev) {
      if (e.second >= bytes) return;
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) ==
          hipSuccess)
        e.second = bytes;
      return;
    }
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess)
    seen.push_back({{fn, dev}, bytes});
}

// Completion events of submitted batches, recycled (creating and destroying one per batch is
// host time on every step): per device, a free list under a lock.
// The pool is keyed by the STREAM's device (a batch may be submitted and finished from threads
// whose current device differs from it: ADVICE r4), and an event is created under that device.
static int stream_device(hipStream_t st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (st) {
    hipDevice_t d = 0;
    if (hipStreamGetDevice(st, &d) == hipSuccess) dev = (int)d;
  }
  return dev;
}
hipEvent_t event_get(hipStream_t st) {
  static_assert(sizeof(hipEvent_t) == sizeof(void*), "event handle");
  const int dev = stream_device(st);
  {
    std::lock_guard<std::mutex> g(event_pool_mutex());
    auto& fl = event_pool()[dev & 63];
    if (!fl.empty()) {
      hipEvent_t e = fl.back();
      fl.pop_back();
      return e;
    }
  }
  int cur = dev;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
  if (cur != dev) (void)hipSetDevice(cur);
  return e;
}
void event_put(hipEvent_t e, hipStream_t st) {
  if (!e) return;
  const int dev = stream_device(st);
  std::lock_guard<std::mutex> g(event_pool_mutex());
  auto& fl = event_pool()[dev & 63];
  if (fl.size() < 64) fl.push_back(e);
  else (void)hipEventDestroy(e);
}
std::mutex& event_pool_mutex() {
  static std::mutex m;
  return m;
}
std::vector<hipEvent_t>* event_pool() {
  static std::vector<hipEvent_t> pools[64];
  return pools;
}

// kernels (defined in the other translation units)
int screen_gemm(const void*, int64_t, const void*, int64_t, int32_t, int32_t, int, const float*,
                const float*, float*, int64_t, hipStream_t, int64_t cstride = 0);
int select_topk(const float*, const int64_t*, int64_t, int64_t, int64_t, int64_t, int32_t,
                int32_t, float*, int64_t*, int64_t, hipStream_t);
int row_norms(const void*, int, int64_t, int32_t, int64_t, double*, float*, hipStream_t);
int screen_image(const void*, int, int64_t, int32_t, int64_t, const double*, int, int, void*,
                 int32_t, hipStream_t, unsigned int* err_max = nullptr);
int query_dense(const void*, int, int64_t, int32_t, int64_t, double*, hipStream_t);
int query_liked_sum(const void*, int, int32_t, int64_t, const double*, int64_t, const int64_t*,
                    const int64_t*, double*, hipStream_t, int64_t row_offset = 0,
                    int64_t n_local = 0);
int scale_rows_f64(double*, int64_t, int32_t, const double*, hipStream_t);
int query_image(const double*, int64_t, int64_t, int32_t, int, const void*, int64_t, int, float,
                void*, int32_t, float*, float*, hipStream_t);
int query_prep(const void*, int, int64_t, int64_t, int32_t, int64_t, int, int, float, double*,
               void*, int32_t, float*, float*, hipStream_t);
int mask_excluded(float*, int64_t, int64_t, int64_t, int64_t, const int64_t*, const int64_t*,
                  hipStream_t);
int rescore(const double*, int64_t, int32_t, const void*, int, int64_t, const double*, int64_t,
            const float*, const int64_t*, int32_t, int32_t, int64_t, const float*, const double*,
            double*, int64_t*, int32_t*, hipStream_t, const int*, int, unsigned long long*,
            int64_t list_base = 0, const float* theta = nullptr,
            const int64_t* excl_off = nullptr, const int64_t* excl_rows = nullptr,
            const ShardPackOut* pack = nullptr);
int screen_gemm_filter(const void*, int64_t, const void*, int64_t, int32_t, int32_t, int,
                       const float*, const float*, const float*, uint64_t*, int64_t, int,
                       uint8_t*, int64_t, int*, int64_t, hipStream_t);
int64_t filter_group_rows(int64_t);
int64_t filter_split_rows(int64_t B_pad, int64_t n_rows);

int spec_threshold(const float*, int64_t, int64_t, int64_t, int, const float*, const float*, float*,
                   int*, int, hipStream_t);
int kth_threshold(const float*, int64_t, int64_t, int64_t, int, const float*, float*,
                  hipStream_t);
int pool_kth(const float*, int64_t, int64_t, int64_t, int, int, float*, hipStream_t,
             float* fv = nullptr, int64_t* fi = nullptr, int kprime = 0, int* ovf = nullptr,
             const float* lead_s = nullptr, int64_t ld_lead = 0, int lead = 0,
             uint64_t* cand = nullptr, int64_t ld_cand = 0, int slots = 0,
             uint8_t* counts = nullptr, int64_t ld_counts = 0, int gj = 0,
             int64_t rstride = 0);
int spec_given_init(const float*, int64_t, int64_t, float*, float*, int64_t*, int, int*,
                    hipStream_t, const float* lead_s = nullptr, int64_t ld_lead = 0, int lead = 0,
                    uint64_t* cand = nullptr, int64_t ld_cand = 0, int slots = 0,
                    uint8_t* counts = nullptr, int64_t ld_counts = 0);
int screen_gemm_pool(const void*, int64_t, const void*, int64_t, int32_t, int32_t, int,
                     const float*, const float*, int64_t, float*, int64_t, hipStream_t,
                     int64_t lead = 0, float* lead_scores = nullptr, int64_t ld_lead = 0);
int64_t gemm_cus();
int merge_segment(float*, int64_t*, int64_t, int, const uint64_t*, int64_t, int, const uint8_t*,
                  int64_t, int64_t, int64_t, const int64_t*, const int64_t*, int*, hipStream_t,
                  double expect_hits = 0.0);
bool merge_wave_fits(int);
int merge_wave_capacity();
int merge_block_capacity(int);
int64_t merge_wave_max_groups();
int64_t merge_block_max_groups(int);
int merge_segment_wave(float*, int64_t*, int64_t, int, int, const uint64_t*, int64_t, int,
                       const uint8_t*, int64_t, int64_t, int64_t, const int64_t*, const int64_t*,
                       int*, hipStream_t, const float* veps = nullptr,
                       const float* vspec = nullptr, float* fout = nullptr, int fw = 0,
                       const float* feps = nullptr, float* tout = nullptr,
                       const float* tin = nullptr, const float* teps = nullptr,
                       int64_t B_pad = 0);
int pilot_topk(const float*, int64_t, int64_t, int, int64_t, int, int, float*, int64_t*,
               hipStream_t);
constexpr int64_t PILOT_ROWS = 1024;  // = WMERGE_H (select_topk.hip)
int merge_topk(const double*, const int64_t*, int32_t, int64_t, int32_t, double*, int64_t*,
               hipStream_t);
int screen_exact(const double*, int64_t, int32_t, const void*, int, int64_t, const double*, int64_t,
                 float*, int64_t, hipStream_t);
int export_list(int64_t*, int64_t, int32_t, int64_t, const int*, const float*, int32_t*, float*,
                hipStream_t);
int rescore_owned(const double*, int64_t, int32_t, const void*, int, int64_t, const double*,
                  int64_t, int64_t, const float*, const int64_t*, int32_t, int32_t, const float*,
                  double*, hipStream_t);
int finalize_topk(const float*, const int64_t*, const double*, int64_t, int32_t, int32_t, int64_t,
                  const float*, const int32_t*, double*, int64_t*, int32_t*, hipStream_t);

// EBT_FLAG_EXACT screening operands (the float64 catalog path), null for the MFMA screen
struct ExactScreen {
  const double* q64;
  int32_t d;
  const void* cat;
  int dtype;
  int64_t ld;
  const double* gnorm;
};

// ------------------------------------------------------------------------------ timer ------
struct Timer {
  struct Rec {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<Rec> recs;
  std::mutex mu;
  uint32_t mask = 0xffffffffu;  // stages recorded (ebt_timer_set_mask)
  std::vector<std::pair<int, hipEvent_t>> open;  // ebt_timer_begin without its _end yet
  // ebt_timer_count_rows: the rescore kernels add the candidate rows they gather here (device
  // memory of the device current at that call; one u64), for the top-K roofline's bytes
  unsigned long long* d_rows = nullptr;
  int rows_dev = -1;

  hipEvent_t get() {
    if (used == pool.size()) {
      // timing only (read after the batch's own completion event): no system-scope fence, i.e.
      // no cache writeback + invalidate around the measured kernels -- with the fence each
      // recorded stage cost the stream ~5 us of gaps (C2: ~4 % of a step)
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[used++];
  }
  ~Timer() {
    for (auto e : pool) (void)hipEventDestroy(e);
    if (d_rows) (void)hipFree(d_rows);
  }
};

// 64 row counters 128 bytes apart (the rescore's workgroup b adds to counter b % 64)
constexpr size_t TIMER_ROW_BYTES = 64 * 128;
// The row counters the rescore adds to, when counting is on, the rescore stage is recorded and
// the launch goes to the counters' own device (a rescore on another device's stream is not
// counted: its atomics would land in a peer's memory)
static unsigned long long* timer_rows(void* timer, hipStream_t st) {
  Timer* t = (Timer*)timer;
  if (!t || !t->d_rows || !((t->mask >> EBT_STAGE_RESCORE) & 1u)) return nullptr;
  int dev = -1;
  if (st ? hipStreamGetDevice(st, &dev) != hipSuccess : hipGetDevice(&dev) != hipSuccess)
    return nullptr;
  return dev == t->rows_dev ? t->d_rows : nullptr;
}

// runs f with the timer's counter device current (restored afterwards)
template <class F>
static int on_rows_dev(const Timer* t, F f) {
  int cur = -1;
  int rc = hip_check(hipGetDevice(&cur), "hipGetDevice");
  if (rc) return rc;
  if (cur != t->rows_dev && (rc = hip_check(hipSetDevice(t->rows_dev), "hipSetDevice"))) return rc;
  rc = f();
  if (cur != t->rows_dev) (void)hipSetDevice(cur);
  return rc;
}

struct StageScope {
  Timer* t;
  int stage;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  StageScope(void* timer, int s, hipStream_t stream) : t((Timer*)timer), stage(s), st(stream) {
    // an unrecorded stage adds no event (each recorded pair costs the stream ~5 us of gaps)
    if (t && !((t->mask >> s) & 1u)) t = nullptr;
    if (t) {
      std::lock_guard<std::mutex> g(t->mu);
      a = t->get();
      b = t->get();
      if (a) (void)hipEventRecord(a, st);
    }
  }
  ~StageScope() {
    if (t && a && b) {
      (void)hipEventRecord(b, st);
      std::lock_guard<std::mutex> g(t->mu);
      t->recs.push_back({stage, a, b});
    }
  }
};

// A stage that is exactly one kernel launch (the filter GEMM's, the roofline's dominant kernel):
// its event pair is handed to the launch (take_launch_events -> hipExtLaunchKernelGGL), which
// binds the events to the dispatch -- no marker packets between the launches of the timed
// region, where StageScope's two hipEventRecords cost the stream gaps of their own. A launch that
// does not take them (an argument error before it) records nothing. EBT_TIMER_MARKERS=1: the
// StageScope form (A/B).
static thread_local hipEvent_t tl_launch_ev[2] = {nullptr, nullptr};
bool take_launch_events(hipEvent_t* start, hipEvent_t* stop) {
  *start = tl_launch_ev[0];
  *stop = tl_launch_ev[1];
  tl_launch_ev[0] = tl_launch_ev[1] = nullptr;
  return *start != nullptr;
}
static bool timer_markers() {
  static const bool on = [] {
    const char* v = getenv("EBT_TIMER_MARKERS");
    return v && v[0] == '1';
  }();
  return on;
}
struct KernelStage {
  Timer* t;
  int stage;
  hipEvent_t a = nullptr, b = nullptr;
  StageScope* markers = nullptr;
  KernelStage(void* timer, int s, hipStream_t stream) : t((Timer*)timer), stage(s) {
    if (t && !((t->mask >> s) & 1u)) t = nullptr;
    if (!t) return;
    if (timer_markers()) {
      markers = new StageScope(timer, s, stream);
      t = nullptr;
      return;
    }
    std::lock_guard<std::mutex> g(t->mu);
    a = t->get();
    b = t->get();
    if (a && b) {
      tl_launch_ev[0] = a;
      tl_launch_ev[1] = b;
    }
  }
  ~KernelStage() {
    delete markers;
    if (!t || !a || !b) return;
    const bool taken = tl_launch_ev[0] == nullptr;
    tl_launch_ev[0] = tl_launch_ev[1] = nullptr;
    if (!taken) return;
    std::lock_guard<std::mutex> g(t->mu);
    t->recs.push_back({stage, a, b});
  }
};

// --------------------------------------------------------------------- workspace layout ----
// Unfused:  [S: B_pad x chunk f32][seg tmp][per-chunk candidates][final candidates]
// Fused:    the same for the HEAD rows [0, H) (chunked), plus the candidate rows
//           [B][kprime + cap] (head top-k' then appended tail candidates), counters and
//           thresholds. The tail rows [H, n) never materialise scores.
struct WsLayout {
  int64_t chunk, ld_s, n_chunks, head, seg_max, group_rows, ld_cand, ld_counts;
  int segs;
  bool fused, pilot;
  // speculative fused screen: `spec_tiles` 256-row sample tiles, `spec_stride` tiles apart;
  // threshold = the spec_j-th best sample score - 2 eps; ~spec_hits expected hits per query
  bool spec;
  int64_t spec_tiles, spec_stride;
  int spec_j;
  double spec_hits;
  // the sample's LEAD: its first spec_lead tiles are the catalog's first tiles, their scores are
  // kept (ld_lead floats per query at off_lead) and their hits extracted once theta_spec is
  // known, so the filter GEMM starts after them and covers whole rounds of the persistent grid
  // (spec_lead_tiles); round_rows = the rows of one such round (0: no rounding)
  int64_t spec_lead, ld_lead, round_rows;
  size_t off_s, off_segv, off_segi, off_chv, off_chi, off_fv, off_fi, off_cand, off_counts,
      off_thr, off_ovf, off_eps, off_tspec, off_lead, bytes;
};

constexpr int SPEC_KPRIME_MAX = 2048;

// P(Poisson(lam) > m)
static double poisson_tail(double lam, int m) {
  double pmf = exp(-lam), cdf = pmf;
  for (int i = 1; i <= m; ++i) {
    pmf *= lam / i;
    cdf += pmf;
  }
  const double t = 1.0 - cdf;
  // 1 - cdf loses everything below ~1e-16: bound the tail by its first terms instead
  if (t < 1e-12) {
    double term = pmf * lam / (m + 1), sum = 0.0;
    for (int i = m + 1; i < m + 64 && term > 0.0; ++i) {
      sum += term;
      term *= lam / (i + 1);
    }
    return sum;
  }
  return t;
}

// Speculative screen parameters (see run_screen). The sample: P evenly spaced full 256-row tiles
// (P = min(64, tiles / 24), so at most ~4 % of the rows are screened twice, or one workgroup per
// CU for small batches); lambda = the expected
// number of sample rows at or above the rank-k' score, taking the sample as a uniform draw of
// the rows; j = the smallest rank with P(Poisson(lambda) >= j) <= 1e-6, so a speculative
// threshold is too high (caught by the VERIFY check -> unfused rerun) about once per million
// queries on data in no particular order. Expected hits per query ~ j n / m.
static bool spec_params(int64_t B_pad, int64_t n_rows, int32_t kprime, int64_t* tiles,
                        int64_t* stride, int* j, double* hits) {
  static const int enabled = [] {
    const char* v = getenv("EBT_SPEC");
    return v ? atoi(v) : 1;
  }();
  // k' <= 512: one wave per query merges the hits; up to 2048: the block merge
  if (!enabled || B_pad % 256 != 0 || kprime > SPEC_KPRIME_MAX) return false;
  const int64_t full = n_rows / 256;
  int64_t P = full / 24;
  // a sample that leaves CUs idle costs one tile's latency whatever its size: with few query
  // tiles take up to one workgroup per CU (MI355X: 256) while that stays within 1/6 of the rows
  // (C2: 64 tiles instead of 16 -> ~300 instead of ~565 hits per query, one filter launch)
  const int64_t fill = 256 / (B_pad / 256 > 0 ? B_pad / 256 : 1);
  if (P < fill && fill <= full / 6) P = fill;
  // at most 64 tiles, or 1/200 of the rows of a large catalog (up to 512 tiles: 2048 pooled
  // maxima, ebt_pool_kth's limit). A sample of m rows puts the k'-th best score near sample rank
  // lambda = k' m / n, and the threshold at the j-th (j ~ lambda + 5 sqrt(lambda) + 6), so the
  // hits per query ~ j n / m fall roughly as 1 / m while lambda is small: C5 (50M rows, k' = 1256)
  // 64 -> 512 tiles takes ~21.6K hits per query to ~5.4K for 0.3 % more GEMM rows
#ifndef EBT_SPEC_SAMPLE_DIV
#define EBT_SPEC_SAMPLE_DIV 200
#endif
  // at least 16 tiles (round 5: C3 16 instead of 64, one round of the pool GEMM instead of four:
  // +0.4 % at 32, +0.5-0.8 % more at 16, profiles/r5/ab/sample32_*, sample16_*), and at least
  // one workgroup per CU (C2 keeps 64)
#ifndef EBT_SPEC_SAMPLE_MIN
#define EBT_SPEC_SAMPLE_MIN 16  // (build knob for A/B)
#endif
  const int64_t pdiv = full / EBT_SPEC_SAMPLE_DIV;
  // (k' > 512, the block merges: 32 -- their cost grows with the hits a smaller sample lets in)
  const int64_t smin = merge_wave_fits(kprime) ? EBT_SPEC_SAMPLE_MIN : 32;
  const int64_t pmin = fill > smin ? fill : smin;
  const int64_t pmax = pdiv > pmin ? (pdiv < 512 ? pdiv : 512) : pmin;
  P = P > pmax ? pmax : P;
  // whole rounds of workgroups: P x (query tiles) a multiple of 256 when that keeps >= 8 tiles
  const int64_t per = 256 / (B_pad / 256) > 0 ? 256 / (B_pad / 256) : 1;
  if (P / per * per >= 8) P = P / per * per;
  if (P < 8) return false;
  const double m = 256.0 * P;
  const double lam = (double)kprime * m / (double)n_rows;
  // upper tail of Poisson(lam): 1 - sum_{i<j} pmf(i)
  double pmf = exp(-lam), cdf = 0.0;
  int jj = 0;
  for (; jj < 100000; ++jj) {
    if (1.0 - cdf <= 1e-6) break;
    cdf += pmf;
    pmf *= lam / (jj + 1);
  }
  if (jj < 1) jj = 1;
  if (jj > (int)(m / 64) / 2) return false;  // the pooled estimate: 4P maxima per query
  *tiles = P;
  // an odd stride: the sample tiles visit every 256-row phase of 1024-row (and larger
  // power-of-two) blocks instead of one -- with an even stride a generated catalog whose rows
  // repeat structure per block was sampled at one phase only (a C4 query got 3.8x its expected
  // hits from an unrepresentative sample)
  *stride = full / P;
  if (*stride > 1 && *stride % 2 == 0) *stride -= 1;
  *j = jj;
  // the j-th of the 4P pooled maxima sits ~j^2 / (2 * 4P) sample ranks lower (two of the top j
  // sample rows in one 64-row subgroup count once)
  *hits = ((double)jj + (double)jj * jj / (8.0 * P)) * (double)n_rows / m;
  return true;
}

static size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

// ebt_spec_lead: 1 = the speculative screen's lead tiles (default; EBT_SPEC_LEAD=0 in the
// environment starts the process without them)
static std::atomic<int>& spec_lead_flag() {
  static std::atomic<int> f([] {
    const char* v = getenv("EBT_SPEC_LEAD");
    return v ? (atoi(v) != 0 ? 1 : 0) : 1;
  }());
  return f;
}

// The persistent screening GEMM runs one 256 x 256 output tile per CU and round: a launch of T
// catalog tiles x Q query tiles takes ceil(T Q / CUs) rounds, the last one partly idle. Catalog
// tiles per whole round (CUs / Q; 0 when Q does not divide the CU count), and the lead: the
// catalog tiles the sample takes over from the filter so that the rest, n_tiles - lead, is a
// whole number of rounds (C2: 391 tiles x 4 query tiles on 256 CUs -> lead 7, the filter's 7th
// round of 28 tiles disappears; C3: 3907 x 16 -> lead 3).
static int64_t round_tiles(int64_t B_pad) {
  const int64_t q = B_pad / 256, cus = gemm_cus();
  return (q > 0 && cus % q == 0) ? cus / q : 0;
}
// (the room for it regardless of ebt_spec_lead, so that a workspace sized before the knob
// changes still fits: the layout's offsets never depend on the knob)
static int64_t spec_lead_room(int64_t B_pad, int64_t n_rows, int64_t sample_tiles) {
  const int64_t rt = round_tiles(B_pad);
  if (rt <= 1) return 0;
  const int64_t lead = ceil_div(n_rows, 256) % rt;
  // a lead of at most half the sample (its strided part keeps the spread), and full tiles only
  return (lead <= sample_tiles / 2 && lead * 256 <= n_rows - 256) ? lead : 0;
}
static int64_t spec_lead_tiles(int64_t B_pad, int64_t n_rows, int64_t sample_tiles) {
  return spec_lead_flag().load(std::memory_order_relaxed)
             ? spec_lead_room(B_pad, n_rows, sample_tiles) : 0;
}

// A row-sharded catalog's sample lead (ebt_cosine_sample_lead / ebt_cosine_screen_at_lead): the
// shard's filter then covers whole rounds too. The shards' samples together spread over the
// catalog, so a shard's lead may take all but 4 of its sample tiles (C3 on 8 ranks: 489 tiles
// per shard, 16 sample tiles of which the first 9 are the lead; the filter's 31st round of 9 x 16
// tiles disappears).
int64_t shard_lead_room(int64_t B_pad, int64_t n_rows, int64_t sample_tiles) {
  const int64_t rt = round_tiles(B_pad);
  if (rt <= 1) return 0;
  const int64_t lead = ceil_div(n_rows, 256) % rt;
  return (lead <= sample_tiles - 4 && lead * 256 <= n_rows - 256) ? lead : 0;
}
int64_t shard_lead_tiles(int64_t B_pad, int64_t n_rows, int64_t sample_tiles) {
  return spec_lead_flag().load(std::memory_order_relaxed)
             ? shard_lead_room(B_pad, n_rows, sample_tiles) : 0;
}

static WsLayout ws_layout(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                          int64_t chunk_rows, int flags) {
  WsLayout L{};
  // fused screen: the head rows give each query its first list and threshold; the tail is
  // filtered inside the GEMM epilogue in doubling segments (each as large as all rows before
  // it, so ~k' hits per query per segment), capped so the per-group hit slots
  // (B_pad x groups x slots u64) stay within 1 GiB. For k' <= 512 the head is a
  // 1024-row PILOT (scores sorted per query by one wave); larger k' take H = max(65536, 256 k')
  // rows through the streaming select.
  static const int64_t h_min = [] {
    const char* v = getenv("EBT_FUSE_HEAD");
    return v ? atoll(v) : 65536LL;
  }();
  L.pilot = merge_wave_fits(kprime);
  L.spec = !(flags & (EBT_FLAG_NO_FUSE | EBT_FLAG_EXACT)) &&
           spec_params(B_pad, n_rows, kprime, &L.spec_tiles, &L.spec_stride, &L.spec_j,
                       &L.spec_hits);
  if ((flags & EBT_FLAG_THETA) && !(flags & (EBT_FLAG_NO_FUSE | EBT_FLAG_EXACT)) &&
      merge_wave_fits(kprime)) {
    // the caller's threshold (ebt_cosine_screen_at): no sample of our own; the spec layout
    // (hit slots, threshold buffer) is kept, the sample scores buffer shrinks to one tile
    if (!L.spec) L.spec_tiles = 1;
    L.spec = true;
  }
  int64_t H = 256LL * kprime;
  H = H < h_min ? h_min : H;
  H = (H + 255) / 256 * 256;
  if (L.pilot) H = PILOT_ROWS;
  if (L.spec) H = 256 * L.spec_tiles;  // the sample (its rows are filtered again with the rest)
  L.fused = L.spec || (!(flags & (EBT_FLAG_NO_FUSE | EBT_FLAG_EXACT)) && n_rows >= 2 * H);
  L.head = L.fused ? H : n_rows;
  if (L.fused) {
    // hit slots: up to 1 GiB of u64 per call, never more than the whole tail at the minimum of
    // 16 slots per group (plus the pilot segment's few groups at up to 128 slots)
    L.group_rows = filter_group_rows(B_pad);
    // 1 GiB at B_pad <= 4096, growing with the batch up to 8 GiB (C5: 16384 queries): larger
    // segments, fewer merges
    static const int64_t small_budget = [] {   // EBT_SLOT_BUDGET_MB: A/B knob, B_pad <= 4096
      const char* v = getenv("EBT_SLOT_BUDGET_MB");
      return (v ? atoll(v) : 1024LL) << 20;
    }();
    int64_t bytes = B_pad * (512LL << 10);
    bytes = bytes < (1LL << 30) ? (1LL << 30) : (bytes > (8LL << 30) ? (8LL << 30) : bytes);
    if (B_pad <= 4096) bytes = small_budget;
    const int64_t budget = bytes / (B_pad * 8);
    const int64_t need = ceil_div(n_rows - (L.spec ? 0 : H), L.group_rows) * 16 +
                         8 * EBT_FILTER_SLOTS_MAX;
    L.ld_cand = budget < need ? budget : need;
    L.ld_cand = L.ld_cand < 8 * EBT_FILTER_SLOTS_MAX ? 8 * EBT_FILTER_SLOTS_MAX : L.ld_cand;
    L.seg_max = L.ld_cand / 16 * L.group_rows;
    // the speculative screen may use 8 slots per group: counts for ld_cand / 8 groups
    L.ld_counts = (L.ld_cand / 8 + 15) / 16 * 16;
  }
  if (L.spec && !(flags & EBT_FLAG_THETA)) {
    L.spec_lead = spec_lead_tiles(B_pad, n_rows, L.spec_tiles);
    L.ld_lead = spec_lead_room(B_pad, n_rows, L.spec_tiles) * 256;
  }
  if (L.spec) {
    const int64_t rt = round_tiles(B_pad);
    L.round_rows = rt > 1 ? rt * 256 : 0;
  }
  L.chunk = chunk_rows < L.head ? chunk_rows : L.head;
  if (L.spec) L.chunk = L.head / 64;  // the sample's pooled maxima (4 per tile)
  if (L.chunk < 1) L.chunk = 1;
  L.ld_s = (L.chunk + 3) & ~(int64_t)3;
  // score rows >= 4 KiB: pitch = 64 floats past a multiple of 64, so the store epilogue's 16
  // query rows per instruction and the select's concurrent rows do not all start on the same
  // HBM channel (a power-of-two pitch measured 5x slower writes and reads)
  if (L.ld_s >= 1024) L.ld_s = (L.ld_s + 63) / 64 * 64 + 64;
  L.n_chunks = ceil_div(L.head, L.chunk);
  // enough select workgroups to fill the chip: >= 512 (2 per CU)
  int64_t segs = B > 0 ? ceil_div(512, B) : 1;
  int64_t max_segs = L.chunk / (2 * 4096);
  if (max_segs < 1) max_segs = 1;
  if (segs > max_segs) segs = max_segs;
  if (segs < 1) segs = 1;
  L.segs = (int)segs;
  size_t o = 0;
  L.off_s = o;
  o = align_up(o + (size_t)B_pad * L.ld_s * 4);
  // the streaming select's per-segment and per-chunk lists: only head_topk (the unfused path,
  // the float64 screen and the progressive screen's head) selects from score rows; the
  // speculative screen's sample writes pooled maxima instead, so its layout has none of them
  // (round 6: C5's first pass carried 14.7 GiB of unused chunk lists, 16384 queries x 64 sample
  // "chunks" x k' 1256 x 12 bytes -- 23.2 -> 8.4 GiB per batch)
  const bool selects = !L.spec;
  L.off_segv = o;
  if (selects && L.segs > 1) o = align_up(o + (size_t)B * L.segs * kprime * 4);
  L.off_segi = o;
  if (selects && L.segs > 1) o = align_up(o + (size_t)B * L.segs * kprime * 8);
  L.off_chv = o;
  if (selects && L.n_chunks > 1) o = align_up(o + (size_t)B * L.n_chunks * kprime * 4);
  L.off_chi = o;
  if (selects && L.n_chunks > 1) o = align_up(o + (size_t)B * L.n_chunks * kprime * 8);
  L.off_fv = o;
  o = align_up(o + (size_t)B * kprime * 4);
  L.off_fi = o;
  o = align_up(o + (size_t)B * kprime * 8);
  if (L.fused) {
    L.off_cand = o;
    o = align_up(o + (size_t)B_pad * L.ld_cand * 8);
    L.off_counts = o;
    o = align_up(o + (size_t)B_pad * L.ld_counts);
    L.off_thr = o;
    o = align_up(o + (size_t)B_pad * 4);
    L.off_ovf = o;
    o = align_up(o + (size_t)B_pad * 4);
  }
  L.off_eps = o;
  if (flags & EBT_FLAG_EXACT) o = align_up(o + (size_t)B_pad * 4);
  if (L.spec) {
    L.off_tspec = o;
    o = align_up(o + (size_t)B_pad * 4);
  }
  L.off_lead = o;
  if (L.ld_lead) o = align_up(o + (size_t)B_pad * L.ld_lead * 4);
  L.bytes = o;
  return L;
}

// Top-k' of rows [r0, r0+nrows) of the (shard-local) catalog into dv/di (row stride ld_d), the
// unfused way: chunked GEMM -> mask -> streaming select (-> select across chunks).
static int head_topk(const WsLayout& L, char* ws, const void* qimg, const float* qscale,
                     int64_t B, int64_t B_pad, const void* cimg, const float* cscale,
                     int img_dtype, int32_t ld_img, int64_t r0, int64_t nrows, int32_t d_pad,
                     int64_t row_offset, const int64_t* excl_off, const int64_t* excl_rows,
                     int32_t kprime, float* dv_final, int64_t* di_final, int64_t ld_final,
                     void* timer, hipStream_t st, const ExactScreen* ex = nullptr) {
  float* S = (float*)(ws + L.off_s);
  float* segv = (float*)(ws + L.off_segv);
  int64_t* segi = (int64_t*)(ws + L.off_segi);
  float* chv = (float*)(ws + L.off_chv);
  int64_t* chi = (int64_t*)(ws + L.off_chi);
  const int64_t n_chunks = ceil_div(nrows, L.chunk);
  int rc;
  for (int64_t c = 0; c < n_chunks; ++c) {
    const int64_t c0 = r0 + c * L.chunk;
    const int64_t nc = (r0 + nrows - c0) < L.chunk ? (r0 + nrows - c0) : L.chunk;
    {
      StageScope s(timer, EBT_STAGE_GEMM, st);
      if (ex) {
        const int es = ex->dtype == EBT_F64 ? 8 : (ex->dtype == EBT_F32 ? 4 : 2);
        rc = screen_exact(ex->q64, B, ex->d, (const char*)ex->cat + c0 * ex->ld * es, ex->dtype,
                          ex->ld, ex->gnorm + c0, nc, S, L.ld_s, st);
      } else {
        rc = screen_gemm(qimg, B_pad, (const char*)cimg + c0 * ld_img * 2, nc, d_pad, ld_img,
                         img_dtype, qscale, cscale ? cscale + c0 : nullptr, S, L.ld_s, st);
      }
    }
    if (rc) return rc;
    if (excl_off) {
      StageScope s(timer, EBT_STAGE_MASK, st);
      rc = mask_excluded(S, L.ld_s, B, row_offset + c0, row_offset + c0 + nc, excl_off,
                         excl_rows, st);
      if (rc) return rc;
    }
    float* dv = n_chunks == 1 ? dv_final : chv + c * kprime;
    int64_t* di = n_chunks == 1 ? di_final : chi + c * kprime;
    const int64_t ld_d = n_chunks == 1 ? ld_final : n_chunks * kprime;
    {
      StageScope s(timer, EBT_STAGE_SELECT, st);
      if (L.segs == 1) {
        rc = select_topk(S, nullptr, L.ld_s, B, nc, c0, kprime, 1, dv, di, ld_d, st);
      } else {
        rc = select_topk(S, nullptr, L.ld_s, B, nc, c0, kprime, L.segs, segv, segi,
                         (int64_t)L.segs * kprime, st);
        if (!rc)
          rc = select_topk(segv, segi, (int64_t)L.segs * kprime, B, (int64_t)L.segs * kprime, 0,
                           kprime, 1, dv, di, ld_d, st);
      }
    }
    if (rc) return rc;
  }
  if (n_chunks > 1) {
    StageScope s(timer, EBT_STAGE_MERGE_SELECT, st);
    rc = select_topk(chv, chi, n_chunks * kprime, B, n_chunks * kprime, 0, kprime, 1, dv_final,
                     di_final, ld_final, st);
    if (rc) return rc;
  }
  return EBT_OK;
}

// The rescore of the row-sharded step (driver.hip): the shard's list holds GLOBAL rows
// (list_base = row_offset: no local-rows pass), and the certificate also takes ebt_certify_cut's
// tests (an overflowed fused list, a caller's threshold above the floor's cut) -- two launches
// fewer per step. Timed and row-counted as ebt_rescore.
int rescore_sharded(const double* q64, int64_t B, int32_t d, const void* cat, int dtype,
                    int64_t ld, const double* gnorm64, int64_t row_offset, const float* cand_vals,
                    const int64_t* cand_rows, int32_t kprime, int32_t k, int64_t n_rows,
                    const float* eps, const double* t_floor, double* out_s, int64_t* out_r,
                    int32_t* certified, const int* ovf, const float* theta, void* timer,
                    hipStream_t st, int64_t list_base, const int64_t* excl_off,
                    const int64_t* excl_rows, const ShardPackOut* pack) {
  StageScope sc(timer, EBT_STAGE_RESCORE, st);
  return rescore(q64, B, d, cat, dtype, ld, gnorm64, row_offset, cand_vals, cand_rows,
                 kprime, k, n_rows, eps, t_floor, out_s, out_r, certified, st, ovf, 0,
                 timer_rows(timer, st), list_base, theta, excl_off, excl_rows, pack);
}

}  // namespace ebt

using namespace ebt;

extern "C" {

int ebt_version(void) { return 303; }  // 0.3.3: certificates into pinned host buffers (ebert.h)

const char* ebt_last_error(void) { return g_err; }

int ebt_row_norms(const void* x, int dtype, int64_t n, int32_t d, int64_t ld, double* gnorm64,
                  float* inv32, void* stream) {
  return row_norms(x, dtype, n, d, ld, gnorm64, inv32, (hipStream_t)stream);
}

int ebt_screen_image(const void* x, int dtype, int64_t n, int32_t d, int64_t ld,
                     const double* gnorm64, int normalize, int img_dtype, void* img,
                     int32_t ld_img, void* stream) {
  return screen_image(x, dtype, n, d, ld, gnorm64, normalize, img_dtype, img, ld_img,
                      (hipStream_t)stream);
}

int ebt_query_dense(const void* q, int dtype, int64_t B, int32_t d, int64_t ldq, double* q64,
                    void* stream) {
  return query_dense(q, dtype, B, d, ldq, q64, (hipStream_t)stream);
}

int ebt_query_liked_sum(const void* cat, int dtype, int32_t d, int64_t ld,
                        const double* gnorm64_cat, int64_t B, const int64_t* liked_off,
                        const int64_t* liked_rows, double* q64, void* stream) {
  return query_liked_sum(cat, dtype, d, ld, gnorm64_cat, B, liked_off, liked_rows, q64,
                         (hipStream_t)stream);
}

int ebt_query_prep(const void* q, int dtype, int64_t B, int64_t B_pad, int32_t d, int64_t ldq,
                   int img_dtype, int native_q, float u_cat, double* q64, void* qimg,
                   int32_t ld_img, float* qscale, float* eps, void* stream) {
  return query_prep(q, dtype, B, B_pad, d, ldq, img_dtype, native_q, u_cat, q64, qimg, ld_img,
                    qscale, eps, (hipStream_t)stream);
}

int ebt_scale_rows_f64(double* q64, int64_t B, int32_t d, const double* scale, void* stream) {
  return scale_rows_f64(q64, B, d, scale, (hipStream_t)stream);
}

int ebt_query_image(const double* q64, int64_t B, int64_t B_pad, int32_t d, int img_dtype,
                    const void* q_native, int64_t ldq, int native_q, float u_cat, void* qimg,
                    int32_t ld_img, float* qscale, float* eps, void* stream) {
  return query_image(q64, B, B_pad, d, img_dtype, q_native, ldq, native_q, u_cat, qimg, ld_img,
                     qscale, eps, (hipStream_t)stream);
}

int ebt_screen_scores(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                      int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                      const float* cscale, float* scores, int64_t ld_scores, void* stream) {
  return screen_gemm(qimg, B_pad, cimg, n_rows, d_pad, ld_img, img_dtype, qscale, cscale, scores,
                     ld_scores, (hipStream_t)stream);
}

int64_t ebt_filter_group_rows(int64_t B_pad) { return filter_group_rows(B_pad); }

int64_t ebt_merge_block_max_groups(int32_t kprime) {
  return kprime < 1 || kprime > 4096 ? -1 : merge_block_max_groups(kprime);
}

int ebt_screen_filter(const void* qimg, int64_t B_pad, const void* cimg, int64_t n_rows,
                      int32_t d_pad, int32_t ld_img, int img_dtype, const float* qscale,
                      const float* cscale, const float* thr, uint64_t* cand, int64_t ld_cand,
                      int32_t slots, uint8_t* counts, int64_t ld_counts, int32_t* ovf,
                      int64_t idx_base, void* stream) {
  return screen_gemm_filter(qimg, B_pad, cimg, n_rows, d_pad, ld_img, img_dtype, qscale, cscale,
                            thr, cand, ld_cand, slots, counts, ld_counts, ovf, idx_base,
                            (hipStream_t)stream);
}

int ebt_mask_excluded(float* scores, int64_t ld_scores, int64_t B, int64_t col_begin,
                      int64_t col_end, const int64_t* excl_off, const int64_t* excl_rows,
                      void* stream) {
  return mask_excluded(scores, ld_scores, B, col_begin, col_end, excl_off, excl_rows,
                       (hipStream_t)stream);
}

int ebt_select_topk(const float* vals, const int64_t* idx, int64_t ld, int64_t B, int64_t n,
                    int64_t idx_base, int32_t kprime, int32_t segs, float* out_vals,
                    int64_t* out_idx, int64_t ld_out, void* stream) {
  return select_topk(vals, idx, ld, B, n, idx_base, kprime, segs, out_vals, out_idx, ld_out,
                     (hipStream_t)stream);
}

int ebt_rescore(const double* q64, int64_t B, int32_t d, const void* cat, int dtype, int64_t ld,
                const double* gnorm64, int64_t row_offset, const float* cand_vals,
                const int64_t* cand_rows, int32_t kprime, int32_t k, int64_t n_rows, const float* eps,
                const double* t_floor, double* out_scores, int64_t* out_rows, int32_t* certified,
                void* timer, void* stream) {
  StageScope sc(timer, EBT_STAGE_RESCORE, (hipStream_t)stream);
  return rescore(q64, B, d, cat, dtype, ld, gnorm64, row_offset, cand_vals, cand_rows, kprime, k,
                 n_rows, eps, t_floor, out_scores, out_rows, certified, (hipStream_t)stream,
                 nullptr, 0, timer_rows(timer, (hipStream_t)stream));
}

int ebt_screen_exact(const double* q64, int64_t B, int32_t d, const void* cat, int dtype,
                     int64_t ld, const double* gnorm64, int64_t n_rows, float* scores,
                     int64_t ld_scores, void* stream) {
  return screen_exact(q64, B, d, cat, dtype, ld, gnorm64, n_rows, scores, ld_scores,
                      (hipStream_t)stream);
}

int ebt_merge_hits(float* fv, int64_t* fi, int64_t B, int32_t kprime, int32_t k,
                   const uint64_t* cand,
                   int64_t ld_cand, int32_t slots, const uint8_t* counts, int64_t ld_counts,
                   int64_t n_groups, int64_t row_offset, const int64_t* excl_off,
                   const int64_t* excl_rows, int32_t* ovf, void* stream) {
  if (!fv || !fi || !cand || !counts || !ovf || ((excl_off == nullptr) != (excl_rows == nullptr))) {
    set_error("ebt_merge_hits: null pointer");
    return EBT_EINVAL;
  }
  if (k < 1 || k > kprime) {
    set_error("ebt_merge_hits: k=%d outside [1, kprime=%d]", k, kprime);
    return EBT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (merge_wave_fits(kprime) && n_groups <= merge_wave_max_groups() && ld_counts % 16 == 0)
    return merge_segment_wave(fv, fi, B, kprime, k, cand, ld_cand, slots, counts, ld_counts,
                              n_groups, row_offset, excl_off, excl_rows, ovf, st);
  return merge_segment(fv, fi, B, kprime, cand, ld_cand, slots, counts, ld_counts, n_groups,
                       row_offset, excl_off, excl_rows, ovf, st);
}

int ebt_merge_topk(const double* scores, const int64_t* rows, int32_t R, int64_t B, int32_t k,
                   double* out_scores, int64_t* out_rows, void* stream) {
  return merge_topk(scores, rows, R, B, k, out_scores, out_rows, (hipStream_t)stream);
}

size_t ebt_cosine_topk_workspace(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                                 int64_t chunk_rows, int flags) {
  if (B < 0 || B_pad < B || n_rows < 1 || kprime < 1 || chunk_rows < 1) return 0;
  return ws_layout(B, B_pad, n_rows, kprime, chunk_rows, flags).bytes;
}

int ebt_cosine_topk_plan(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                         int64_t chunk_rows, int flags, int64_t* head_rows, int64_t* cap,
                         int64_t* chunk, int32_t* fused) {
  if (B < 0 || B_pad < B || n_rows < 1 || kprime < 1 || chunk_rows < 1 || !head_rows || !cap ||
      !chunk || !fused) {
    set_error("ebt_cosine_topk_plan: bad arguments");
    return EBT_EINVAL;
  }
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, chunk_rows, flags);
  *head_rows = L.head;
  *cap = L.fused ? L.seg_max : 0;
  *chunk = L.chunk;
  *fused = L.fused ? 1 : 0;
  return EBT_OK;
}

int ebt_cosine_topk_spec_plan(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                              int flags, int64_t* sample_tiles, int64_t* tile_stride,
                              int32_t* rank, double* hits) {
  if (B < 0 || B_pad < B || n_rows < 1 || kprime < 1 || !sample_tiles || !tile_stride || !rank ||
      !hits) {
    set_error("ebt_cosine_topk_spec_plan: bad arguments");
    return EBT_EINVAL;
  }
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, 1024, flags);
  *sample_tiles = L.spec ? L.spec_tiles : 0;
  *tile_stride = L.spec ? L.spec_stride : 0;
  *rank = L.spec ? L.spec_j : 0;
  *hits = L.spec ? L.spec_hits : 0.0;
  return EBT_OK;
}

int64_t ebt_cosine_topk_spec_lead(int64_t B, int64_t B_pad, int64_t n_rows, int32_t kprime,
                                  int flags) {
  if (B < 0 || B_pad < B || n_rows < 1 || kprime < 1) return -1;
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, 1024, flags);
  return L.spec ? L.spec_lead : 0;
}

int ebt_spec_lead(int on) {
  if (on < 0) return spec_lead_flag().load();
  return spec_lead_flag().exchange(on != 0 ? 1 : 0);
}

}  // extern "C"

namespace ebt {

// What the rescore needs from the screen: the eps the certificate uses (the caller's, or the
// exact screen's constant) and the fused screen's overflow flags (null when not fused).
struct ScreenOut {
  const float* eps;
  const int* ovf;
};

struct PipeArgs {
  const double* q64;
  const void* qimg;
  const float* qscale;
  const float* eps;
  int64_t B, B_pad;
  const void* cat;
  int dtype;
  int64_t ld;
  const double* gnorm64;
  const void* cimg;
  const float* cscale;
  int img_dtype;
  int32_t ld_img;
  int64_t n_rows;
  int32_t d, d_pad;
  int64_t row_offset;
  const int64_t* excl_off;
  const int64_t* excl_rows;
  int32_t k, kprime;
  int64_t chunk_rows;
  int flags;
  // ebt_cosine_screen_at: the caller's per-query threshold [B] and expected hits per query
  const float* theta = nullptr;
  double hits = 0.0;
  // ebt_cosine_screen_at_lead: the caller's sample lead -- the shard's first `lead` 256-row tiles,
  // their scores [B_pad][ld_lead] stored by ebt_cosine_sample_lead
  int64_t lead = 0;
  const float* lead_s = nullptr;
  int64_t ld_lead = 0;
  // screen_at_local: the threshold as the gs_j-th of the all-gathered sample maxima ([R][B][gj],
  // rank stride gs_rstride floats, gs_G values per query), taken by the same launch that starts
  // the list and takes the lead's hits (instead of a caller's theta)
  const float* gsamp = nullptr;
  int64_t gs_rstride = 0;
  int gs_G = 0, gs_gj = 0, gs_j = 0;
  // screen_at_local: the row-sharded step's floor entries ([B][floor_w + 1], ebt_floor_pack's
  // layout) written by the screen's last wave merge
  float* floor_out = nullptr;
  int floor_w = 0;
};

static int check_pipe(const PipeArgs& a, const char* who) {
  const bool exact = a.flags & EBT_FLAG_EXACT;
  if (!a.q64 || (!exact && (!a.qimg || !a.qscale || !a.eps || !a.cimg)) || !a.cat ||
      !a.gnorm64) {
    set_error("%s: null pointer", who);
    return EBT_EINVAL;
  }
  if (a.B < 1 || a.B_pad < a.B || a.B_pad % 128 != 0 || a.n_rows < 1 || a.d < 1 ||
      a.d_pad < a.d || a.d_pad % 64 != 0 || a.ld_img < a.d_pad || a.k < 1 || a.kprime < a.k ||
      a.kprime > 4096 || a.kprime % 4 != 0 || a.chunk_rows < 128 || a.chunk_rows % 128 != 0 ||
      ((a.excl_off == nullptr) != (a.excl_rows == nullptr))) {
    set_error("%s: bad arguments (B=%lld B_pad=%lld n=%lld d=%d d_pad=%d k=%d kprime=%d "
              "chunk=%lld)", who, (long long)a.B, (long long)a.B_pad, (long long)a.n_rows, a.d,
              a.d_pad, a.k, a.kprime, (long long)a.chunk_rows);
    return EBT_EINVAL;
  }
  return EBT_OK;
}

// The speculative fused screen. The progressive pilot/segment screen below pays for its rising
// threshold with ~k' ln(n / 1024) hits per query (measured ~2850 at C3 over 6 filter launches,
// each hit a cold epilogue path while the tile's MFMAs idle). Here:
//   1. sample: P full 256-row tiles spread evenly over the catalog through the GEMM with the
//      POOL epilogue (strided tiles; per query only the max of each 64-row subgroup leaves the
//      kernel); theta_spec = the j-th largest of those 4P maxima (spec_params: the rank whose
//      estimate exceeds the k'-th best catalog score with probability <= 1e-6 on unordered data);
//   2. the whole catalog through the filter GEMM with theta_spec in few large segments (the list
//      starts empty; later segments raise the threshold to max(theta_spec, list k-th - 2 eps)),
//      each followed by the wave merge (exclusions dropped there);
//   3. VERIFY: theta_spec <= the final list's k-th - 2 eps, else ovf = 2 -> certificate -1 ->
//      the query is rerun unfused. So theta_spec needs no proof: a wrong guess costs a rerun.
// Sample rows are screened twice (in the sample and in the filter pass); they enter the list
// only through the filter, so nothing is counted twice.
// One fused segment's filter screen over rows [r0, r0 + seg): one launch, or consecutive
// launches of whole rounds when the segment is long (filter_split_rows, screen_gemm.hip), each
// its own timed launch (the roofline's per-launch average stays a kernel's). The hits and counts
// of group g of the segment land at cand + g * slots / counts + g, whatever the parts.
static int filter_screen(const PipeArgs& a, int64_t r0, int64_t seg, const float* thr,
                         uint64_t* cand, int64_t ld_cand, int slots, uint8_t* counts,
                         int64_t ld_counts, int* ovf, void* timer, hipStream_t st) {
  const int64_t part = filter_split_rows(a.B_pad, seg);
  const int64_t step = part > 0 ? part : seg;
  for (int64_t p0 = 0; p0 < seg; p0 += step) {
    const int64_t nr = seg - p0 < step ? seg - p0 : step;
    const int64_t r = r0 + p0, g = p0 / 256;  // part boundaries are whole 256-row groups
    KernelStage s(timer, EBT_STAGE_GEMM_FILTER, st);
    const int rc = screen_gemm_filter(a.qimg, a.B_pad, (const char*)a.cimg + r * a.ld_img * 2, nr,
                                      a.d_pad, a.ld_img, a.img_dtype, a.qscale,
                                      a.cscale ? a.cscale + r : nullptr, thr, cand + g * slots,
                                      ld_cand, slots, counts + g, ld_counts, ovf, r, st);
    if (rc) return rc;
  }
  return EBT_OK;
}

static int run_screen_spec(const PipeArgs& a, const WsLayout& L, char* ws, float* fv,
                           int64_t* fi, void* timer, hipStream_t st) {
  int rc;
  const int64_t B = a.B, B_pad = a.B_pad, n_rows = a.n_rows;
  const int32_t k = a.k, kprime = a.kprime;
  uint64_t* cand = (uint64_t*)(ws + L.off_cand);
  uint8_t* counts = (uint8_t*)(ws + L.off_counts);
  float* thr = (float*)(ws + L.off_thr);
  int* ovf = (int*)(ws + L.off_ovf);
  float* pooled = (float*)(ws + L.off_s);
  float* tspec = (float*)(ws + L.off_tspec);
  const int64_t m = L.head;
  // ebt_cosine_screen_at: the caller's threshold (or screen_at_local's gathered samples)
  const bool given = a.theta != nullptr || a.gsamp != nullptr;
  const double spec_hits = given ? (a.hits > 0.0 ? a.hits : 1.0) : L.spec_hits;
  // hits per group ~ H group_rows / n (per query; its threshold's own spread ~ 1/sqrt(j) on
  // top): slots for 4x that + 4, and at least enough that a group overflow (which costs its
  // query an unfused rerun of the whole catalog) is expected less than once per thousand batches
  const double per_group = spec_hits * (double)L.group_rows / (double)n_rows;
  const double n_cells = (double)B * (double)ceil_div(n_rows, L.group_rows);
  int slots = 8;
  while (slots < EBT_FILTER_SLOTS_MAX &&
         (slots < 4.0 * per_group + 4.0 || n_cells * poisson_tail(1.5 * per_group, slots) > 1e-3))
    slots *= 2;
  // the lead tiles (the sample's first tiles, their scores kept by the pool GEMM): their hits
  // at theta_spec go into the first segment's first groups, taken by the same launch that finds
  // theta_spec (pool_kth); the filter then starts after them
  const int64_t lead = given ? a.lead : L.spec_lead;
  if (lead > 0 && (lead * slots > L.ld_cand || lead > L.ld_counts || L.group_rows != 256)) {
    set_error("run_screen_spec: the lead does not fit the hit slots");
    return EBT_EINVAL;
  }
  if (given) {
    // the threshold, the empty list (-inf / -1), no overflow yet: one launch
    // (+ the caller's lead hits at theta into the first groups' slots)
    if (a.gsamp)   // the threshold from the gathered samples, in the same launch
      rc = pool_kth(a.gsamp, a.gs_G, B, B_pad, a.gs_G, a.gs_j, tspec, st, fv, fi, kprime, ovf,
                    a.lead_s, a.ld_lead, (int)lead, cand, L.ld_cand, slots, counts, L.ld_counts,
                    a.gs_gj, a.gs_rstride);
    else
      rc = spec_given_init(a.theta, B, B_pad, tspec, fv, fi, kprime, ovf, st, a.lead_s,
                           a.ld_lead, (int)lead, cand, L.ld_cand, slots, counts, L.ld_counts);
    if (rc) return rc;
  } else {
    {
      StageScope s(timer, EBT_STAGE_GEMM, st);
      rc = screen_gemm_pool(a.qimg, B_pad, a.cimg, m, a.d_pad, a.ld_img, a.img_dtype, a.qscale,
                            a.cscale, 256 * L.spec_stride, pooled, L.ld_s, st, lead,
                            (float*)(ws + L.off_lead), L.ld_lead);
    }
    if (rc) return rc;
    {
      StageScope s(timer, EBT_STAGE_SELECT, st);
      // theta_spec, the empty list (-inf / -1) with no overflow yet, the lead's hits
      rc = pool_kth(pooled, L.ld_s, B, B_pad, (int)(m / 64), L.spec_j, tspec, st, fv, fi, kprime,
                    ovf, (const float*)(ws + L.off_lead), L.ld_lead, (int)lead, cand, L.ld_cand,
                    slots, counts, L.ld_counts);
    }
    if (rc) return rc;
  }
  const bool wave = merge_wave_fits(kprime);
  int64_t seg_cap = L.ld_cand / slots;
  const int64_t max_groups = wave ? merge_wave_max_groups() : merge_block_max_groups(kprime);
  seg_cap = seg_cap < max_groups ? seg_cap : max_groups;
  seg_cap *= L.group_rows;
  const double cap = (double)(wave ? merge_wave_capacity() : merge_block_capacity(kprime));
  // A query's hits are ~ Gamma(j) n / m around the expected H = j n / m (its threshold is the
  // j-th of its own sample): the merge's room beside the list must hold f times the expected
  // hits, f = the Gamma(j) quantile at 1e-2 / B over its mean (P(Gamma(j) > x) = P(Poisson(x)
  // < j)), so that an overflow -- an unfused rerun of the query -- is expected less than once
  // per hundred batches (f = 2.6 at j = 16, B = 4096; 3.0 at j = 12, B = 8192; floor 2.5).
  double f_spread = 2.5;
  if (!given && L.spec_j > 0) {
    const double target = 1e-2 / (double)(B > 0 ? B : 1);
    double x = (double)L.spec_j;
    while (x < 8.0 * L.spec_j) {
      double pmf = exp(-x), cdf = pmf;
      for (int i = 1; i < L.spec_j; ++i) {
        pmf *= x / i;
        cdf += pmf;
      }
      if (cdf <= target) break;
      x += 0.25;
    }
    f_spread = x / (double)L.spec_j;
    f_spread = f_spread < 2.5 ? 2.5 : f_spread;
  }
  int64_t r0 = 256 * lead;
  bool first = true, verified = false, thr_raised = false;
  while (r0 < n_rows) {
    // expected hits <= 1 / f_spread of the merge's room beside the list. Hits per row: at
    // theta_spec H / n; after r0 rows the raised threshold (the list's k-th - 2 eps) keeps at
    // most ~k' / r0 of the rows. A remainder of less than half a segment joins the last one.
    // The first segment also merges the lead's groups: its cap is that much smaller.
    const int64_t g0 = first ? lead : 0;  // groups of the lead in front of this segment's
    const int64_t cap_rows = seg_cap - g0 * L.group_rows;
    const double room = (cap - kprime) / f_spread;
    // after r0 rows the raised threshold keeps about k + (the 2 eps band) of every r0 rows; k'
    // budgets that band at k' - k, so (k + k') / 2 per r0 rows still leaves the band twice its
    // budget (round 5; k' per r0 before: C3 took four filter launches per batch instead of three)
    const double kept = 0.5 * ((double)k + (double)kprime);
    double rate = spec_hits / (double)n_rows;
    if (!first && kept / (double)r0 < rate) rate = kept / (double)r0;
    int64_t seg = (int64_t)(room / (rate > 1e-12 ? rate : 1e-12));
    seg = (seg + 255) / 256 * 256;
    // whole rounds of the persistent grid (every segment but a remainder): no partly idle
    // last round per launch
    if (L.round_rows > 0 && seg >= L.round_rows) seg = seg / L.round_rows * L.round_rows;
    seg = seg < 256 ? 256 : seg;
    const int64_t cap_r = L.round_rows > 0 && cap_rows >= L.round_rows
                              ? cap_rows / L.round_rows * L.round_rows : cap_rows;
    seg = seg < cap_r ? seg : cap_r;
    if (!first && n_rows - r0 - seg < seg / 2) seg = n_rows - r0;
    if (seg > cap_rows) seg = cap_rows;
    if (seg > n_rows - r0) seg = n_rows - r0;
    if (seg < 1) {
      set_error("run_screen_spec: no room for a segment");
      return EBT_EINVAL;
    }
    const float* t = tspec;
    if (!first) {
      if (!thr_raised) {  // (the previous wave merge wrote it: no launch)
        rc = spec_threshold(fv, kprime, B, B_pad, k, a.eps, tspec, thr, ovf, 0, st);
        if (rc) return rc;
      }
      t = thr;
    }
    rc = filter_screen(a, r0, seg, t, cand + g0 * slots, L.ld_cand, slots, counts + g0,
                       L.ld_counts, ovf, timer, st);
    if (rc) return rc;
    // the last wave merge also runs the final VERIFY of theta_spec (no separate launch)
    const bool fuse_verify = wave && !given && r0 + seg == n_rows;
    verified |= fuse_verify;
    const int64_t groups = g0 + ceil_div(seg, L.group_rows);
    const bool last = r0 + seg == n_rows;
    // the wave merge of a segment that is not the last also writes the next one's threshold
    // (spec_threshold's RAISE folded in)
    thr_raised = wave && !last;
    {
      StageScope s(timer, EBT_STAGE_MERGE_SELECT, st);
      if (wave)
        rc = merge_segment_wave(fv, fi, B, kprime, k, cand, L.ld_cand, slots, counts,
                                L.ld_counts, groups, a.row_offset, a.excl_off, a.excl_rows, ovf,
                                st, fuse_verify ? a.eps : nullptr, fuse_verify ? tspec : nullptr,
                                last ? a.floor_out : nullptr, a.floor_w, a.eps,
                                thr_raised ? thr : nullptr, tspec, a.eps, B_pad);
      else  // sorted lists (the block merge sorts the union)
        rc = merge_segment(fv, fi, B, kprime, cand, L.ld_cand, slots, counts, L.ld_counts,
                           groups, a.row_offset, a.excl_off, a.excl_rows, ovf, st,
                           rate * (double)(seg + g0 * L.group_rows));
    }
    if (rc) return rc;
    r0 += seg;
    first = false;
  }
  // a caller's threshold is verified by the caller against the catalog-wide floor (the local
  // list may hold fewer than k rows: most of the global top k live on other shards)
  if (given || verified) return EBT_OK;
  return spec_threshold(fv, kprime, B, B_pad, k, a.eps, tspec, nullptr, ovf, 1, st);
}

// The screen: the k' best approx candidates per query into fv/fi (LOCAL rows, sorted), by the
// exact (float64) screen, the unfused chunked screen or the fused pilot/segment screen.
static int run_screen(const PipeArgs& a, const WsLayout& L, char* ws, float* fv, int64_t* fi,
                      void* timer, hipStream_t st, ScreenOut* so) {
  int rc;
  so->eps = a.eps;
  so->ovf = nullptr;
  const int64_t B = a.B, B_pad = a.B_pad, n_rows = a.n_rows, row_offset = a.row_offset;
  const int32_t k = a.k, kprime = a.kprime, d_pad = a.d_pad, ld_img = a.ld_img;
  if (a.flags & EBT_FLAG_EXACT) {  // float64 screen; its bound replaces the caller's eps
    const ExactScreen ex{a.q64, a.d, a.cat, a.dtype, a.ld, a.gnorm64};
    float* xeps = (float*)(ws + L.off_eps);
    const float e = EBT_EXACT_EPS;
    uint32_t bits;
    memcpy(&bits, &e, 4);
    rc = hip_check(hipMemsetD32Async((hipDeviceptr_t)xeps, (int)bits, (size_t)B, st),
                   "hipMemsetD32Async");
    if (rc) return rc;
    so->eps = xeps;
    return head_topk(L, ws, nullptr, nullptr, B, B_pad, nullptr, nullptr, a.img_dtype, ld_img, 0,
                     n_rows, d_pad, row_offset, a.excl_off, a.excl_rows, kprime, fv, fi, kprime,
                     timer, st, &ex);
  }
  if (!L.fused)
    return head_topk(L, ws, a.qimg, a.qscale, B, B_pad, a.cimg, a.cscale, a.img_dtype, ld_img, 0,
                     n_rows, d_pad, row_offset, a.excl_off, a.excl_rows, kprime, fv, fi, kprime,
                     timer, st);
  uint64_t* cand = (uint64_t*)(ws + L.off_cand);
  uint8_t* counts = (uint8_t*)(ws + L.off_counts);
  float* thr = (float*)(ws + L.off_thr);
  int* ovf = (int*)(ws + L.off_ovf);
  so->ovf = ovf;
  if (L.spec) return run_screen_spec(a, L, ws, fv, fi, timer, st);
  // 1. head rows [0, H): exact top-k' per query (the list fv/fi)
  if (L.pilot) {
    float* S = (float*)(ws + L.off_s);
    {
      StageScope s(timer, EBT_STAGE_GEMM, st);
      rc = screen_gemm(a.qimg, B_pad, a.cimg, L.head, d_pad, ld_img, a.img_dtype, a.qscale,
                       a.cscale, S, L.ld_s, st);
    }
    if (rc) return rc;
    if (a.excl_off) {
      StageScope s(timer, EBT_STAGE_MASK, st);
      rc = mask_excluded(S, L.ld_s, B, row_offset, row_offset + L.head, a.excl_off, a.excl_rows,
                         st);
      if (rc) return rc;
    }
    StageScope s(timer, EBT_STAGE_SELECT, st);
    rc = pilot_topk(S, L.ld_s, B, (int)L.head, 0, kprime, k, fv, fi, st);
  } else {
    rc = head_topk(L, ws, a.qimg, a.qscale, B, B_pad, a.cimg, a.cscale, a.img_dtype, ld_img, 0,
                   L.head, d_pad, row_offset, a.excl_off, a.excl_rows, kprime, fv, fi, kprime,
                   timer, st);
  }
  if (rc) return rc;
  rc = hip_check(hipMemsetAsync(ovf, 0, (size_t)B_pad * 4, st), "hipMemsetAsync");
  if (rc) return rc;
  // 2. tail rows [H, n) in segments: threshold = the list's k-th approx - 2 eps, GEMM with the
  //    filter epilogue, merge of list + hits (exclusions dropped) back into the list
  int64_t r0 = L.head;
  while (r0 < n_rows) {
    // hits per group ~ G k' / r0 when the segment's rows are like the r0 before it: slots for
    // 4x that (+8), so a group overflows (-> unfused rerun of the query) only on skewed data
    const double per_group = (double)L.group_rows * kprime / (double)r0;
    int slots = 16;
    while (slots < 4.0 * per_group + 8.0 && slots < EBT_FILTER_SLOTS_MAX) slots *= 2;
    // segment = GROW x the rows so far: ~GROW k' hits per query at most (the threshold sits 2 eps
    // below the list's k-th best, so typically ~GROW (k + the 2 eps band)); the wave merge holds
    // 1024 hits, the block merge 4 k' + 2048
    int64_t grow = 2;
    if (L.pilot) {  // the wave merge holds k' + hits <= its capacity
      grow = (merge_wave_capacity() - kprime) / kprime;
      grow = grow < 1 ? 1 : (grow > 3 ? 3 : grow);
    }
    int64_t seg = n_rows - r0 < grow * r0 ? n_rows - r0 : grow * r0;
    if (n_rows - (r0 + seg) < seg / 2 && n_rows - r0 <= (grow + 1) * r0)
      seg = n_rows - r0;  // no small last segment
    int64_t seg_cap = L.ld_cand / slots * L.group_rows;
    const int64_t max_groups = L.pilot ? merge_wave_max_groups() : merge_block_max_groups(kprime);
    if (seg_cap > max_groups * L.group_rows) seg_cap = max_groups * L.group_rows;
    seg = seg < seg_cap ? seg : seg_cap;
    const int64_t groups = ceil_div(seg, L.group_rows);
    rc = kth_threshold(fv, kprime, B, B_pad, k, a.eps, thr, st);
    if (rc) return rc;
    rc = filter_screen(a, r0, seg, thr, cand, L.ld_cand, slots, counts, L.ld_counts, ovf,
                       timer, st);
    if (rc) return rc;
    {
      StageScope s(timer, EBT_STAGE_MERGE_SELECT, st);
      rc = L.pilot ? merge_segment_wave(fv, fi, B, kprime, k, cand, L.ld_cand, slots, counts,
                                        L.ld_counts, groups, row_offset, a.excl_off, a.excl_rows,
                                        ovf, st)
                   : merge_segment(fv, fi, B, kprime, cand, L.ld_cand, slots, counts,
                                   L.ld_counts, groups, row_offset, a.excl_off, a.excl_rows, ovf,
                                   st);
    }
    if (rc) return rc;
    r0 += seg;
  }
  return EBT_OK;
}

}  // namespace ebt

extern "C" {

int ebt_cosine_topk_prepared(const double* q64, const void* qimg, const float* qscale, const float* eps,
                    int64_t B, int64_t B_pad, const void* cat, int dtype, int64_t ld,
                    const double* gnorm64, const void* cimg, const float* cscale, int img_dtype,
                    int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad, int64_t row_offset,
                    const int64_t* excl_off, const int64_t* excl_rows, int32_t k, int32_t kprime,
                    int64_t chunk_rows, int flags, void* workspace, size_t ws_bytes,
                    double* out_scores, int64_t* out_rows, int32_t* certified, void* timer,
                    void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const PipeArgs a{q64, qimg, qscale, eps, B, B_pad, cat, dtype, ld, gnorm64, cimg, cscale,
                   img_dtype, ld_img, n_rows, d, d_pad, row_offset, excl_off, excl_rows, k, kprime,
                   chunk_rows, flags};
  int rc = check_pipe(a, "ebt_cosine_topk_prepared");
  if (rc) return rc;
  if (!workspace || !out_scores || !out_rows || !certified) {
    set_error("ebt_cosine_topk_prepared: null pointer");
    return EBT_EINVAL;
  }
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, chunk_rows, flags);
  if (ws_bytes < L.bytes) {
    set_error("ebt_cosine_topk_prepared: workspace %zu < %zu bytes", ws_bytes, L.bytes);
    return EBT_ENOMEM;
  }
  char* ws = (char*)workspace;
  float* fv = (float*)(ws + L.off_fv);
  int64_t* fi = (int64_t*)(ws + L.off_fi);
  ScreenOut so{};
  rc = run_screen(a, L, ws, fv, fi, timer, st, &so);
  if (rc) return rc;
  StageScope s(timer, EBT_STAGE_RESCORE, st);
  // (the rescore also checks each query's exclusion segment: certified = -3 when it is not
  // sorted ascending -- the check the C entry used to launch on its own, with a flag memset)
  return rescore(q64, B, d, cat, dtype, ld, gnorm64, row_offset, fv, fi, kprime, k, n_rows,
                 so.eps, nullptr, out_scores, out_rows, certified, st, so.ovf, 0,
                 timer_rows(timer, st), 0, nullptr, excl_off, excl_rows);
}

int ebt_cosine_screen(const double* q64, const void* qimg, const float* qscale, const float* eps,
                      int64_t B, int64_t B_pad, const void* cat, int dtype, int64_t ld,
                      const double* gnorm64, const void* cimg, const float* cscale, int img_dtype,
                      int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad, int64_t row_offset,
                      const int64_t* excl_off, const int64_t* excl_rows, int32_t k, int32_t kprime,
                      int64_t chunk_rows, int flags, void* workspace, size_t ws_bytes,
                      float* list_vals, int64_t* list_rows, int32_t* ovf_out, float* eps_out,
                      void* timer, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const PipeArgs a{q64, qimg, qscale, eps, B, B_pad, cat, dtype, ld, gnorm64, cimg, cscale,
                   img_dtype, ld_img, n_rows, d, d_pad, row_offset, excl_off, excl_rows, k, kprime,
                   chunk_rows, flags};
  int rc = check_pipe(a, "ebt_cosine_screen");
  if (rc) return rc;
  if (!workspace || !list_vals || !list_rows || !ovf_out || !eps_out) {
    set_error("ebt_cosine_screen: null pointer");
    return EBT_EINVAL;
  }
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, chunk_rows, flags);
  if (ws_bytes < L.bytes) {
    set_error("ebt_cosine_screen: workspace %zu < %zu bytes", ws_bytes, L.bytes);
    return EBT_ENOMEM;
  }
  char* ws = (char*)workspace;
  ScreenOut so{};
  rc = run_screen(a, L, ws, list_vals, list_rows, timer, st, &so);
  if (rc) return rc;
  return export_list(list_rows, B, kprime, row_offset, so.ovf, so.eps, ovf_out, eps_out, st);
}

int ebt_cosine_screen_at(const double* q64, const void* qimg, const float* qscale,
                         const float* eps, int64_t B, int64_t B_pad, const void* cat, int dtype,
                         int64_t ld, const double* gnorm64, const void* cimg, const float* cscale,
                         int img_dtype, int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad,
                         int64_t row_offset, const int64_t* excl_off, const int64_t* excl_rows,
                         int32_t k, int32_t kprime, int64_t chunk_rows, int flags,
                         void* workspace, size_t ws_bytes, float* list_vals, int64_t* list_rows,
                         int32_t* ovf_out, float* eps_out, const float* theta, double hits,
                         void* timer, void* stream) {
  return ebt_cosine_screen_at_lead(q64, qimg, qscale, eps, B, B_pad, cat, dtype, ld, gnorm64,
                                   cimg, cscale, img_dtype, ld_img, n_rows, d, d_pad, row_offset,
                                   excl_off, excl_rows, k, kprime, chunk_rows, flags, workspace,
                                   ws_bytes, list_vals, list_rows, ovf_out, eps_out, theta, hits,
                                   0, nullptr, 0, timer, stream);
}

int ebt_cosine_screen_at_lead(const double* q64, const void* qimg, const float* qscale,
                              const float* eps, int64_t B, int64_t B_pad, const void* cat,
                              int dtype, int64_t ld, const double* gnorm64, const void* cimg,
                              const float* cscale, int img_dtype, int32_t ld_img, int64_t n_rows,
                              int32_t d, int32_t d_pad, int64_t row_offset,
                              const int64_t* excl_off, const int64_t* excl_rows, int32_t k,
                              int32_t kprime, int64_t chunk_rows, int flags, void* workspace,
                              size_t ws_bytes, float* list_vals, int64_t* list_rows,
                              int32_t* ovf_out, float* eps_out, const float* theta, double hits,
                              int64_t lead, const float* lead_scores, int64_t ld_lead,
                              void* timer, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  flags |= EBT_FLAG_THETA;
  PipeArgs a{q64, qimg, qscale, eps, B, B_pad, cat, dtype, ld, gnorm64, cimg, cscale,
             img_dtype, ld_img, n_rows, d, d_pad, row_offset, excl_off, excl_rows, k, kprime,
             chunk_rows, flags};
  a.theta = theta;
  a.hits = hits;
  a.lead = lead;
  a.lead_s = lead_scores;
  a.ld_lead = ld_lead;
  int rc = check_pipe(a, "ebt_cosine_screen_at");
  if (rc) return rc;
  if (lead < 0 || (lead > 0 && (!lead_scores || ld_lead < 256 * lead || 256 * lead >= n_rows))) {
    set_error("ebt_cosine_screen_at_lead: bad lead (lead=%lld, ld_lead=%lld, n_rows=%lld)",
              (long long)lead, (long long)ld_lead, (long long)n_rows);
    return EBT_EINVAL;
  }
  if (!workspace || !list_vals || !list_rows || !ovf_out || !eps_out || !theta) {
    set_error("ebt_cosine_screen_at: null pointer");
    return EBT_EINVAL;
  }
  if ((flags & (EBT_FLAG_NO_FUSE | EBT_FLAG_EXACT)) || !merge_wave_fits(kprime) ||
      !(hits >= 0.0)) {
    set_error("ebt_cosine_screen_at: needs the fused screen with kprime <= 512 (kprime=%d, "
              "flags=%d, hits=%g)", kprime, flags, hits);
    return EBT_EINVAL;
  }
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, chunk_rows, flags);
  if (ws_bytes < L.bytes) {
    set_error("ebt_cosine_screen_at: workspace %zu < %zu bytes", ws_bytes, L.bytes);
    return EBT_ENOMEM;
  }
  char* ws = (char*)workspace;
  ScreenOut so{};
  rc = run_screen(a, L, ws, list_vals, list_rows, timer, st, &so);
  if (rc) return rc;
  return export_list(list_rows, B, kprime, row_offset, so.ovf, so.eps, ovf_out, eps_out, st);
}

}  // extern "C"

namespace ebt {
// The sharded step's screen at the shared threshold without ebt_cosine_screen_at_lead's export
// launch (driver.hip): the list keeps LOCAL rows (the sharded rescore reads them with list base
// 0), and the screen's own overflow flags and eps stay where the pipeline wrote them (*ovf_dev,
// *eps_dev point into the workspace / the prepared queries).
int screen_at_local(const double* q64, const void* qimg, const float* qscale, const float* eps,
                    int64_t B, int64_t B_pad, const void* cat, int dtype, int64_t ld,
                    const double* gnorm64, const void* cimg, const float* cscale, int img_dtype,
                    int32_t ld_img, int64_t n_rows, int32_t d, int32_t d_pad, int64_t row_offset,
                    const int64_t* excl_off, const int64_t* excl_rows, int32_t k, int32_t kprime,
                    int64_t chunk_rows, void* workspace, size_t ws_bytes, float* list_vals,
                    int64_t* list_rows, const float* gsamp, int64_t gs_rstride, int gs_G,
                    int gs_gj, int gs_j, double hits, int64_t lead, const float* lead_scores,
                    int64_t ld_lead, const float** theta_dev, const int** ovf_dev,
                    const float** eps_dev, void* timer, hipStream_t st, float* floor_out,
                    int floor_w) {
  const int flags = EBT_FLAG_THETA;
  PipeArgs a{q64, qimg, qscale, eps, B, B_pad, cat, dtype, ld, gnorm64, cimg, cscale,
             img_dtype, ld_img, n_rows, d, d_pad, row_offset, excl_off, excl_rows, k, kprime,
             chunk_rows, flags};
  a.hits = hits;
  a.lead = lead;
  a.lead_s = lead_scores;
  a.ld_lead = ld_lead;
  a.gsamp = gsamp;
  a.gs_rstride = gs_rstride;
  a.gs_G = gs_G;
  a.gs_gj = gs_gj;
  a.gs_j = gs_j;
  a.floor_out = floor_out;
  a.floor_w = floor_w;
  int rc = check_pipe(a, "screen_at_local");
  if (rc) return rc;
  if (!workspace || !list_vals || !list_rows || !gsamp || !theta_dev || !ovf_dev || !eps_dev ||
      !merge_wave_fits(kprime) || !(hits >= 0.0) || lead < 0 || gs_G < 1 || gs_G > 2048 ||
      (floor_out && (floor_w < 1 || floor_w > k)) ||
      gs_gj < 1 || gs_G % gs_gj != 0 || gs_rstride < B * (int64_t)gs_gj || gs_j < 1 ||
      (lead > 0 && (!lead_scores || ld_lead < 256 * lead || 256 * lead >= n_rows))) {
    set_error("screen_at_local: bad arguments (kprime=%d, lead=%lld, G=%d, gj=%d, j=%d)", kprime,
              (long long)lead, gs_G, gs_gj, gs_j);
    return EBT_EINVAL;
  }
  const WsLayout L = ws_layout(B, B_pad, n_rows, kprime, chunk_rows, flags);
  if (ws_bytes < L.bytes) {
    set_error("screen_at_local: workspace %zu < %zu bytes", ws_bytes, L.bytes);
    return EBT_ENOMEM;
  }
  ScreenOut so{};
  rc = run_screen(a, L, (char*)workspace, list_vals, list_rows, timer, st, &so);
  if (rc) return rc;
  *ovf_dev = so.ovf;
  *eps_dev = so.eps;
  *theta_dev = (const float*)((char*)workspace + L.off_tspec);
  return EBT_OK;
}
}  // namespace ebt

extern "C" {

int ebt_cosine_sample(const void* qimg, const float* qscale, int64_t B_pad, const void* cimg,
                      const float* cscale, int img_dtype, int32_t ld_img, int64_t n_rows,
                      int32_t d_pad, int64_t tiles, int64_t tile_stride, float* pooled,
                      int64_t ld_pooled, void* timer, void* stream) {
  return ebt_cosine_sample_lead(qimg, qscale, B_pad, cimg, cscale, img_dtype, ld_img, n_rows,
                                d_pad, tiles, tile_stride, pooled, ld_pooled, 0, nullptr, 0, timer,
                                stream);
}

int ebt_cosine_sample_lead(const void* qimg, const float* qscale, int64_t B_pad,
                           const void* cimg, const float* cscale, int img_dtype, int32_t ld_img,
                           int64_t n_rows, int32_t d_pad, int64_t tiles, int64_t tile_stride,
                           float* pooled, int64_t ld_pooled, int64_t lead, float* lead_scores,
                           int64_t ld_lead, void* timer, void* stream) {
  // tiles 0 .. lead-1 are the first tiles, tile t >= lead starts at row 256 (lead + (t - lead)
  // tile_stride): the last one ends within (tiles - 1) tile_stride + 1 tiles
  const int64_t last = tiles > lead ? lead + (tiles - lead - 1) * tile_stride : lead - 1;
  if (tiles < 1 || tile_stride < 1 || lead < 0 || lead > tiles || 256 * (last + 1) > n_rows ||
      (lead > 0 && (!lead_scores || ld_lead < 256 * lead))) {
    set_error("ebt_cosine_sample: %lld tiles %lld apart (lead %lld) do not fit %lld rows",
              (long long)tiles, (long long)tile_stride, (long long)lead, (long long)n_rows);
    return EBT_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  StageScope s(timer, EBT_STAGE_GEMM, st);
  return screen_gemm_pool(qimg, B_pad, cimg, 256 * tiles, d_pad, ld_img, img_dtype, qscale, cscale,
                          256 * tile_stride, pooled, ld_pooled, st, lead, lead_scores, ld_lead);
}

int ebt_pool_kth(const float* pooled, int64_t ld, int64_t B, int64_t B_pad, int32_t G, int32_t j,
                 float* theta, void* stream) {
  return pool_kth(pooled, ld, B, B_pad, G, j, theta, (hipStream_t)stream);
}

int ebt_rescore_owned(const double* q64, int64_t B, int32_t d, const void* cat, int dtype,
                      int64_t ld, const double* gnorm64, int64_t row_offset, int64_t n_rows,
                      const float* cand_vals, const int64_t* cand_rows, int32_t kprime, int32_t k,
                      const float* eps, double* exact, void* stream) {
  return rescore_owned(q64, B, d, cat, dtype, ld, gnorm64, row_offset, n_rows, cand_vals,
                       cand_rows, kprime, k, eps, exact, (hipStream_t)stream);
}

int ebt_finalize_topk(const float* cand_vals, const int64_t* cand_rows, const double* exact,
                      int64_t B, int32_t kprime, int32_t k, int64_t n_rows_global,
                      const float* eps, const int32_t* ovf, double* out_scores, int64_t* out_rows,
                      int32_t* certified, void* stream) {
  return finalize_topk(cand_vals, cand_rows, exact, B, kprime, k, n_rows_global, eps, ovf,
                       out_scores, out_rows, certified, (hipStream_t)stream);
}

void* ebt_timer_create(void) { return new (std::nothrow) Timer(); }

void ebt_timer_destroy(void* timer) { delete (Timer*)timer; }

int ebt_timer_set_mask(void* timer, uint32_t stage_mask) {
  if (!timer) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  t->mask = stage_mask;
  return EBT_OK;
}

int ebt_timer_reset(void* timer) {
  if (!timer) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  t->recs.clear();
  t->open.clear();
  t->used = 0;
  if (t->d_rows)
    return on_rows_dev(t, [&] {
      return hip_check(hipMemset(t->d_rows, 0, TIMER_ROW_BYTES), "hipMemset");
    });
  return EBT_OK;
}

int ebt_timer_count_rows(void* timer, int on) {
  if (!timer) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  if (!on) {
    if (t->d_rows) (void)on_rows_dev(t, [&] { return hip_check(hipFree(t->d_rows), "hipFree"); });
    t->d_rows = nullptr;
    return EBT_OK;
  }
  if (t->d_rows) return EBT_OK;
  int rc = hip_check(hipMalloc((void**)&t->d_rows, TIMER_ROW_BYTES), "hipMalloc");
  if (rc) return rc;
  (void)hipGetDevice(&t->rows_dev);
  return hip_check(hipMemset(t->d_rows, 0, TIMER_ROW_BYTES), "hipMemset");
}

int ebt_timer_rows(void* timer, int64_t* rows) {
  if (!timer || !rows) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  *rows = 0;
  if (!t->d_rows) return EBT_OK;
  unsigned long long v[TIMER_ROW_BYTES / 8];
  // hipMemcpy waits for the work before it on the null stream; the caller synchronises the
  // launch streams first (as for ebt_timer_query)
  int rc = on_rows_dev(t, [&] {
    return hip_check(hipMemcpy(v, t->d_rows, TIMER_ROW_BYTES, hipMemcpyDeviceToHost), "hipMemcpy");
  });
  int64_t tot = 0;
  for (int i = 0; i < 64; ++i) tot += (int64_t)v[i * 16];
  *rows = tot;
  return rc;
}

int ebt_timer_begin(void* timer, int stage, void* stream) {
  if (!timer || stage < 0 || stage >= EBT_NUM_STAGES) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  if (!((t->mask >> stage) & 1u)) return EBT_OK;
  for (auto& o : t->open)
    if (o.first == stage) {
      set_error("ebt_timer_begin: stage %d is already open", stage);
      return EBT_EINVAL;
    }
  hipEvent_t a = t->get();
  if (!a) return hip_check(hipErrorOutOfMemory, "hipEventCreate");
  int rc = hip_check(hipEventRecord(a, (hipStream_t)stream), "hipEventRecord");
  if (rc) return rc;
  t->open.push_back({stage, a});
  return EBT_OK;
}

int ebt_timer_end(void* timer, int stage, void* stream) {
  if (!timer || stage < 0 || stage >= EBT_NUM_STAGES) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  for (size_t i = 0; i < t->open.size(); ++i) {
    if (t->open[i].first != stage) continue;
    hipEvent_t a = t->open[i].second;
    t->open.erase(t->open.begin() + (long)i);
    hipEvent_t b = t->get();
    if (!b) return hip_check(hipErrorOutOfMemory, "hipEventCreate");
    int rc = hip_check(hipEventRecord(b, (hipStream_t)stream), "hipEventRecord");
    if (rc) return rc;
    t->recs.push_back({stage, a, b});
    return EBT_OK;
  }
  return EBT_OK;  // not open: the stage was masked at ebt_timer_begin
}

int ebt_timer_query(void* timer, int stage, double* total_ms, int64_t* launches) {
  if (!timer || !total_ms || !launches) return EBT_EINVAL;
  Timer* t = (Timer*)timer;
  std::lock_guard<std::mutex> g(t->mu);
  double tot = 0.0;
  int64_t cnt = 0;
  for (auto& r : t->recs) {
    if (r.stage != stage) continue;
    int rc = hip_check(hipEventSynchronize(r.b), "hipEventSynchronize");
    if (rc) return rc;
    float ms = 0.f;
    rc = hip_check(hipEventElapsedTime(&ms, r.a, r.b), "hipEventElapsedTime");
    if (rc) return rc;
    tot += ms;
    ++cnt;
  }
  *total_ms = tot;
  *launches = cnt;
  return EBT_OK;
}

}  // extern "C"
