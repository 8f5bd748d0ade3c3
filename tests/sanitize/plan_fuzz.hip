// Host-only sanitizer run (ASan + UBSan) of libebert's planning arithmetic: the workspace
// layouts of the prepared pipeline (api.hip: ws_layout, spec_params) and of the self-contained
// path (driver.hip: ebt_workspace_bytes), the plan / spec-plan queries and the catalog state
// sizing, over a grid of batch sizes, catalog sizes, k', chunk sizes and flags. No GPU call is
// made (the layouts are pure host code). Built by `make -C robot_ebert_amd/csrc sanitize` with
// -fsanitize=address,undefined on the host side only; run by tests/test_sanitize_host.py.
// Checks, besides the sanitizers: every region of a layout lies inside its byte count, regions
// are 256-byte aligned and in increasing order, the plan agrees with the layout.
#include "../../robot_ebert_amd/csrc/api.hip"

#include <cstdio>

static int failures = 0;
#define CHECK(c, ...)                                                   \
  do {                                                                  \
    if (!(c)) {                                                         \
      if (failures++ < 20) {                                            \
        fprintf(stderr, "FAIL %s:%d %s: ", __FILE__, __LINE__, #c);     \
        fprintf(stderr, __VA_ARGS__);                                   \
        fprintf(stderr, "\n");                                          \
      }                                                                 \
    }                                                                   \
  } while (0)

static int64_t pad_b(int64_t B) { return B <= 128 ? 128 : (B + 255) / 256 * 256; }

int main() {
  const int64_t Bs[] = {1, 2, 64, 127, 128, 129, 255, 256, 1000, 1024, 4096, 8192, 16384};
  const int64_t ns[] = {1, 2, 5, 100, 1023, 1024, 2269, 4096, 5000, 65536, 100000, 131072,
                        1000000, 1250000, 6250000, 10000000, 50000000};
  const int32_t kps[] = {4, 8, 16, 104, 128, 200, 512, 516, 1256, 2048, 2052, 4096};
  const int flagset[] = {0, EBT_FLAG_NO_FUSE, EBT_FLAG_EXACT, EBT_FLAG_THETA,
                         EBT_FLAG_THETA | EBT_FLAG_NO_FUSE};
  long cases = 0;
  for (int64_t B : Bs)
    for (int64_t n : ns)
      for (int32_t kp : kps) {
        if (kp > (n + 3) / 4 * 4) continue;
        const int64_t chunks[] = {128, 4096, 262144, (n + 127) / 128 * 128};
        for (int64_t ch : chunks)
          for (int fl : flagset) {
            const int64_t Bp = pad_b(B);
            const ebt::WsLayout L = ebt::ws_layout(B, Bp, n, kp, ch, fl);
            ++cases;
            const size_t offs[] = {L.off_s,   L.off_segv, L.off_segi, L.off_chv, L.off_chi,
                                   L.off_fv,  L.off_fi};
            size_t prev = 0;
            for (size_t o : offs) {
              CHECK(o % 256 == 0 && o >= prev && o <= L.bytes, "B=%lld n=%lld kp=%d ch=%lld fl=%d",
                    (long long)B, (long long)n, kp, (long long)ch, fl);
              prev = o;
            }
            // (a caller's threshold, EBT_FLAG_THETA: the one-tile sample buffer is never read)
            const bool theta = L.spec && (fl & EBT_FLAG_THETA);
            CHECK(L.head >= 1 && (L.head <= n || theta) && L.chunk >= 1 && L.n_chunks >= 1,
                  "head=%lld chunk=%lld n=%lld", (long long)L.head, (long long)L.chunk,
                  (long long)n);
            CHECK(L.bytes >= (size_t)Bp * L.ld_s * 4, "score area");
            if (L.fused) {
              CHECK(L.off_cand % 256 == 0 && L.off_cand + (size_t)Bp * L.ld_cand * 8 <= L.bytes,
                    "cand");
              CHECK(L.off_ovf + (size_t)Bp * 4 <= L.bytes && L.ld_cand >= 8 * 128 &&
                        L.ld_counts * 8 >= L.ld_cand && L.seg_max >= L.group_rows,
                    "fused layout B=%lld n=%lld kp=%d", (long long)B, (long long)n, kp);
            }
            if (L.spec && !theta) {
              CHECK(L.spec_tiles >= 1 && L.spec_stride >= 1 && L.spec_j >= 1 &&
                        L.spec_hits > 0.0 && L.off_tspec + (size_t)Bp * 4 <= L.bytes,
                    "spec B=%lld n=%lld kp=%d fl=%d", (long long)B, (long long)n, kp, fl);
              CHECK((L.spec_tiles - 1) * L.spec_stride + 1 <= n / 256, "sample tiles in range");
            }
            int64_t h = 0, cap = 0, chunk = 0;
            int32_t fused = 0;
            CHECK(ebt_cosine_topk_plan(B, Bp, n, kp, ch, fl, &h, &cap, &chunk, &fused) == 0 &&
                      h == L.head && fused == (L.fused ? 1 : 0),
                  "plan");
            CHECK(ebt_cosine_topk_workspace(B, Bp, n, kp, ch, fl) == L.bytes, "workspace");
          }
      }
  // the self-contained path: catalog state and driver workspace over dtypes / k
  for (int64_t n : ns)
    for (int dt = 0; dt < 4; ++dt)
      for (int32_t d : {32, 77, 768, 1536}) {
        const size_t st = ebt_catalog_state_bytes((const void*)0x100000, dt, n, d, d);
        CHECK(st >= (size_t)n * 12, "state n=%lld", (long long)n);
        ebt_catalog c{};
        c.data = c.image = (const void*)0x100000;
        c.gnorm64 = (double*)0x200000;
        c.inv32 = (float*)0x300000;
        c.dtype = dt;
        c.d = d;
        c.n = n;
        c.ld = d;
        c.d_pad = (d + 63) / 64 * 64;
        c.ld_img = c.d_pad;
        c.img_dtype = dt == EBT_BF16 ? EBT_BF16 : EBT_F16;
        c.native = dt == EBT_BF16 || dt == EBT_F16;
        for (int64_t B : {1, 129, 4096})
          for (int32_t k : {1, 10, 100, 1000, 4096, 5000}) {
            ++cases;
            const size_t ws = ebt_workspace_bytes(&c, B, k, nullptr);
            // min(k, n) <= 4096: the screen; beyond it the full-sort path (large_k.hip), whose
            // sizing is host arithmetic since round 6 (no device query): every case is valid
            const bool ok = (k < n ? k : n) <= 4096;
            CHECK(ws > 0, "driver ws n=%lld B=%lld k=%d -> %zu", (long long)n, (long long)B, k,
                  ws);
            ebt_options o{};
            o.kprime = 4 * k;
            o.chunk_rows = 4096;
            o.flags = EBT_FLAG_NO_FUSE;
            if (ok) CHECK(ebt_workspace_bytes(&c, B, k, &o) > 0, "driver ws with options");
          }
      }
  printf("plan_fuzz: %ld layouts checked, %d failures\n", cases, failures);
  return failures ? 1 : 0;
}
