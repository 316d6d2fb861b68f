// Practical fp16 MFMA ceiling of this MI355X under its clock management: back-to-back
// v_mfma_f32_32x32x16_f16 on random operands held in registers (8 A and 8 B fragments per wave,
// consecutive MFMAs on different random pairs, 8 independent accumulators), one or two waves per SIMD on every CU,
// no memory traffic in the loop. Reports TFLOP/s and the in-kernel clock (s_memtime cycles over
// s_memrealtime at 100 MHz, MI355X_MICROARCH.md 'DVFS give-back' item 6) after >= 2 s of
// back-to-back launches. The gap between 2.5 PF (2.4 GHz) and this number is what no schedule of
// the tiled scan can recover; DESIGN.md §6 prices the scan against both.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_ceiling.hip -o tools/probes/mfma_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ half8 rnd8(uint32_t seed) {
  half8 h;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    h[i] = (_Float16)((float)(mix(seed * 8 + i) & 0xffff) * (1.0f / 32768.0f) - 1.0f);
  return h;
}

__global__ __launch_bounds__(256) void mfma_loop(int iters, float* out, long long* stamps) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  half8 a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = rnd8(g * 16 + i);
    b[i] = rnd8(g * 16 + 8 + i);
  }
  f32x16 acc[8] = {};
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[j], b[(j + 3) & 7], acc[j], 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  out[g] = s;
  if ((threadIdx.x & 63) == 0) {
    const int w = g / 64;
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  for (int waves_per_simd = 1; waves_per_simd <= 2; ++waves_per_simd) {
    const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
    const int threads = blocks * 256;
    float* out;
    long long* st;
    CHECK(hipMalloc(&out, threads * sizeof(float)));
    CHECK(hipMalloc(&st, (threads / 64) * 2 * sizeof(long long)));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // >= 2 s of back-to-back launches before the timed one (the clock settles under load)
    float warm_ms = 0.f;
    while (warm_ms < 2000.f) {
      CHECK(hipEventRecord(e0));
      mfma_loop<<<blocks, 256>>>(iters, out, st);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      warm_ms += ms;
    }
    const int reps = 10;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) mfma_loop<<<blocks, 256>>>(iters, out, st);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> h((threads / 64) * 2);
    CHECK(hipMemcpy(h.data(), st, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    for (size_t w = 0; w < h.size() / 2; ++w)
      if (h[2 * w + 1] > 0) ghz.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);
    std::sort(ghz.begin(), ghz.end());
    const double flops = (double)(threads / 64) * iters * 8 * 32768.0 * reps;
    printf("waves_per_simd=%d cus=%d iters=%d: %.1f TFLOP/s (%.1f %% of 2.5 PF), in-kernel clock "
           "median %.2f GHz (min %.2f, max %.2f), %.3f ms per launch\n",
           waves_per_simd, cus, iters, flops / (ms * 1e-3) / 1e12,
           flops / (ms * 1e-3) / 2.5e15 * 100.0, ghz[ghz.size() / 2], ghz.front(), ghz.back(),
           ms / reps);
    CHECK(hipFree(out));
    CHECK(hipFree(st));
  }
  return 0;
}
