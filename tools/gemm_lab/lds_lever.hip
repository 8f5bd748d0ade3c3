// LDS-read bytes per MFMA as a clock lever (cdna_hip_programming.md rule 28's
// third lever): the screening GEMM's inner loop without its global stream or epilogue, on random
// f16 operands, at several (operand fragments read from LDS) : (MFMAs) ratios. A wave of the
// production kernel (screen_gemm.hip qp2, 256 x 256 tile, 8 waves) reads 12 fragments of 1 KiB
// per 32 v_mfma_f32_16x16x32_f16 (a 4 x 8 block outer product per 32-deep k step): 384 B/MFMA.
// A larger per-wave register tile reads fewer bytes per MFMA, but at 2 waves per SIMD the
// 128 accumulator VGPRs of 4 x 8 blocks are the most a wave can hold beside its operands; an
// 8 x 8 register tile (256 accumulators) needs 1 wave per SIMD. This lab measures the loop
// alone, so the question "would fewer LDS bytes per MFMA raise the clock / throughput on random
// operands" is answered without the production kernel's other constraints:
//
//   v_4x8_w8    4 x 8 blocks, 8 waves per CU (2 per SIMD), 384 B/MFMA  -- the production loop
//   v_4x8_half  the same MFMA stream, fragments re-read from LDS every 2nd k step: 192 B/MFMA
//   v_4x8_none  the same MFMA stream, operands rotated in registers, no LDS reads: 0 B/MFMA
//   v_8x8_w4    8 x 8 blocks, 4 waves per CU (1 per SIMD), 256 B/MFMA  -- the larger tile
//   v_8x8_w4_pipe  the same with the next step's fragments read under the current MFMAs
//   v_4x4_w8    4 x 4 blocks, 8 waves, 512 B/MFMA
//
// Each variant runs back to back for ~2.5 s (the clock settles, MI355X_MICROARCH.md "DVFS
// give-back"), then 10 timed launches (hipEvents); lane 0 of every workgroup stamps the shader
// clock (s_memtime) and the 100 MHz real-time counter (s_memrealtime) at its start and end, so
// each line reports TFLOP/s, the fraction of the 2.5 PFLOP/s dense f16 peak and the clock.
// Output: one JSON line per variant. Build: hipcc -O3 --offload-arch=gfx950 (tools/gemm_lab/gpu.sh).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NFRAG = 32;  // fragments resident in LDS (32 KiB)

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// READ_EVERY: fragments re-read from LDS every READ_EVERY k steps (0: never -- rotated in
// registers instead)
template <int FA, int FB, int WAVES, int READ_EVERY>
__global__ __launch_bounds__(64 * WAVES) void lever_kernel(const half8* __restrict__ src,
                                                           int iters, float* __restrict__ out,
                                                           unsigned long long* __restrict__ st) {
  __shared__ half8 lds[NFRAG * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < NFRAG * 64; i += 64 * WAVES) lds[i] = src[(blockIdx.x * 7 + i) % (NFRAG * 64 * 8)];
  __syncthreads();
  unsigned long long c0 = 0, r0 = 0;
  if (tid == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f32x4 acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  half8 a[FA], b[FB];
#pragma unroll
  for (int i = 0; i < FA; ++i) a[i] = lds[(i & (NFRAG - 1)) * 64 + lane];
#pragma unroll
  for (int j = 0; j < FB; ++j) b[j] = lds[((FA + j) & (NFRAG - 1)) * 64 + lane];
  const int wv = tid >> 6;
  for (int it = 0; it < iters; ++it) {
    if (READ_EVERY > 0 && it % (READ_EVERY > 0 ? READ_EVERY : 1) == 0) {
      const int base = (it + wv) & (NFRAG - 1);
#pragma unroll
      for (int i = 0; i < FA; ++i) a[i] = lds[((base + i) & (NFRAG - 1)) * 64 + lane];
#pragma unroll
      for (int j = 0; j < FB; ++j) b[j] = lds[((base + FA + j) & (NFRAG - 1)) * 64 + lane];
    } else if (READ_EVERY == 0) {
      // operands change every step without LDS: rotate the fragment registers
      const half8 t = a[0];
#pragma unroll
      for (int i = 0; i + 1 < FA; ++i) a[i] = a[i + 1];
      a[FA - 1] = b[0];
#pragma unroll
      for (int j = 0; j + 1 < FB; ++j) b[j] = b[j + 1];
      b[FB - 1] = t;
    }
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        if constexpr (FA * FB > 32)
          // 256 accumulators: pinned to AGPRs (the builtin lets the compiler shuttle them
          // between AGPRs and VGPRs -- 100 v_accvgpr moves per k step); each accumulator's next
          // use is FA * FB MFMAs later, so no dependency hazard needs a wait
          asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[i]), "v"(b[j]));
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[(size_t)blockIdx.x * 64 * WAVES + tid] = s;
  if (tid == 0) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    st[2 * blockIdx.x] = c1 - c0;
    st[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// The 8 x 8 register tile with the next k step's fragments read under the current step's MFMAs
// (double-buffered operand registers: 2 x 16 fragments = 128 VGPRs beside 256 AGPR
// accumulators): one wave per SIMD has no second wave to hide the ds_read latency behind, so
// its own pipeline must.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void lever_pipe_kernel(const half8* __restrict__ src,
                                                                int iters, float* __restrict__ out,
                                                                unsigned long long* __restrict__ st) {
  constexpr int FA = 8, FB = 8;
  __shared__ half8 lds[NFRAG * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < NFRAG * 64; i += 64 * WAVES) lds[i] = src[(blockIdx.x * 7 + i) % (NFRAG * 64 * 8)];
  __syncthreads();
  unsigned long long c0 = 0, r0 = 0;
  if (tid == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  f32x4 acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wv = tid >> 6;
  half8 a[FA], b[FB], an[FA], bn[FB];
#pragma unroll
  for (int i = 0; i < FA; ++i) a[i] = lds[(i & (NFRAG - 1)) * 64 + lane];
#pragma unroll
  for (int j = 0; j < FB; ++j) b[j] = lds[((FA + j) & (NFRAG - 1)) * 64 + lane];
  for (int it = 0; it < iters; ++it) {
    const int base = (it + 1 + wv) & (NFRAG - 1);
#pragma unroll
    for (int i = 0; i < FA; ++i) an[i] = lds[((base + i) & (NFRAG - 1)) * 64 + lane];
#pragma unroll
    for (int j = 0; j < FB; ++j) bn[j] = lds[((base + FA + j) & (NFRAG - 1)) * 64 + lane];
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j)
        asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(a[i]), "v"(b[j]));
#pragma unroll
    for (int i = 0; i < FA; ++i) a[i] = an[i];
#pragma unroll
    for (int j = 0; j < FB; ++j) b[j] = bn[j];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[(size_t)blockIdx.x * 64 * WAVES + tid] = s;
  if (tid == 0) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    st[2 * blockIdx.x] = c1 - c0;
    st[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int FA, int FB, int WAVES, int RE, bool PIPE = false>
void run(const char* name, const half8* src, float* out, unsigned long long* st, int cus,
         double settle_s) {
  const double bytes_per_mfma = RE == 0 ? 0.0 : (double)(FA + FB) * 1024.0 / (FA * FB) / RE;
  // ~2 ms per launch
  const int iters = (int)(2.0e-3 * 1.9e15 / ((double)cus * WAVES * FA * FB * 16384.0));
  auto launch = [&] {
    if constexpr (PIPE)
      hipLaunchKernelGGL((lever_pipe_kernel<WAVES>), dim3(cus), dim3(64 * WAVES), 0, 0, src,
                         iters, out, st);
    else
      hipLaunchKernelGGL((lever_kernel<FA, FB, WAVES, RE>), dim3(cus), dim3(64 * WAVES), 0, 0,
                         src, iters, out, st);
  };
  launch();
  CHECK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < settle_s) {
    for (int i = 0; i < 20; ++i) launch();
    CHECK(hipDeviceSynchronize());
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 10;
  CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * cus);
  CHECK(hipMemcpy(h.data(), st, 16 * (size_t)cus, hipMemcpyDeviceToHost));
  std::vector<double> ghz(cus);
  for (int i = 0; i < cus; ++i) ghz[i] = (double)h[2 * i] / ((double)h[2 * i + 1] / 100e6) / 1e9;
  std::sort(ghz.begin(), ghz.end());
  const double flops = (double)cus * WAVES * FA * FB * 16384.0 * iters * reps;
  const double tf = flops / (ms * 1e-3) / 1e12;
  printf("{\"variant\": \"%s\", \"blocks\": \"%dx%d\", \"waves_per_cu\": %d, "
         "\"lds_bytes_per_mfma\": %.1f, \"iters\": %d, \"ms_per_launch\": %.4f, "
         "\"tflops\": %.1f, \"frac_of_2500\": %.4f, \"clock_ghz_median\": %.3f, "
         "\"tflops_at_2p4ghz\": %.1f}\n",
         name, FA, FB, WAVES, bytes_per_mfma, iters, ms / reps, tf, tf / 2500.0,
         ghz[cus / 2], tf * 2.4 / ghz[cus / 2]);
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const double settle = argc > 1 ? atof(argv[1]) : 2.5;
  const int rounds = argc > 2 ? atoi(argv[2]) : 2;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const size_t n = (size_t)NFRAG * 64 * 8;  // 8 distinct LDS images over the workgroups
  std::vector<_Float16> h(n * 8);
  unsigned s = 12345u;
  for (auto& v : h) {  // random operands in (-1, 1): the switching energy of real data
    s = s * 1664525u + 1013904223u;
    v = (_Float16)(((double)(s >> 8) / (double)(1u << 24)) * 2.0 - 1.0);
  }
  half8* src;
  float* out;
  unsigned long long* st;
  CHECK(hipMalloc(&src, n * sizeof(half8)));
  CHECK(hipMemcpy(src, h.data(), n * sizeof(half8), hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, (size_t)cus * 512 * sizeof(float)));
  CHECK(hipMalloc(&st, (size_t)cus * 16));
  for (int r = 0; r < rounds; ++r) {  // interleaved rounds
    run<4, 8, 8, 1>("v_4x8_w8", src, out, st, cus, settle);
    run<4, 8, 8, 2>("v_4x8_half", src, out, st, cus, settle);
    run<4, 8, 8, 0>("v_4x8_none", src, out, st, cus, settle);
    run<8, 8, 4, 1>("v_8x8_w4", src, out, st, cus, settle);
    run<8, 8, 4, 1, true>("v_8x8_w4_pipe", src, out, st, cus, settle);
    run<4, 4, 8, 1>("v_4x4_w8", src, out, st, cus, settle);
  }
  return 0;
}
