// HBM read-pattern probe for the dense scan (diagnostic, not part of the library).
// Streams a 2 GB buffer of 1M x 1024 fp16 rows with one 512-thread workgroup per CU and reports
// TB/s for: (0) the scan's lane->row mapping (lane r of a half reads row r: 32 rows x 2 x 16 B
// per instruction), (1) the same bytes fully coalesced (1 KB contiguous per instruction),
// at prefetch depths 4 and 8 groups.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int DIM = 1024;
constexpr int64_t N = 1 << 20;
constexpr int TILE = 32;

template <int MODE, int DEPTH>
__global__ __launch_bounds__(512) void probe(const uint16_t* __restrict__ rows, int tiles_per_wg,
                                             int64_t n_tiles, u32x4* __restrict__ sink) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t t1 = min(t0 + (int64_t)tiles_per_wg, n_tiles);
  u32x4 acc = {0, 0, 0, 0};
  constexpr int GROUPS = DIM / 64;
  for (int64_t t = t0 + wave; t < t1; t += 8) {
    const u32x4* base;
    if (MODE == 0) base = reinterpret_cast<const u32x4*>(rows + (t * TILE + r) * DIM) + 4 * h;
    else base = reinterpret_cast<const u32x4*>(rows + t * TILE * DIM) + lane;
    u32x4 buf[DEPTH][4];
#pragma unroll
    for (int g = 0; g < DEPTH; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        buf[g][i] = MODE == 0 ? base[8 * g + i] : base[64 * (4 * g + i)];
#pragma unroll
    for (int g = 0; g < GROUPS; ++g) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc ^= buf[g % DEPTH][i];
      if (g + DEPTH < GROUPS) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          buf[g % DEPTH][i] = MODE == 0 ? base[8 * (g + DEPTH) + i] : base[64 * (4 * (g + DEPTH) + i)];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int MODE, int DEPTH>
void run(const uint16_t* d, u32x4* sink, int cus) {
  const int64_t n_tiles = N / TILE;
  const int tpw = (int)((n_tiles + cus - 1) / cus);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) probe<MODE, DEPTH><<<cus, 512>>>(d, tpw, n_tiles, sink);
  hipEventRecord(a);
  const int iters = 20;
  for (int it = 0; it < iters; ++it) probe<MODE, DEPTH><<<cus, 512>>>(d, tpw, n_tiles, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= iters;
  printf("mode %d depth %d: %.3f ms  %.2f TB/s\n", MODE, DEPTH, ms, N * DIM * 2.0 / ms / 1e9);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  uint16_t* d;
  u32x4* sink;
  hipMalloc(&d, N * DIM * 2);
  hipMalloc(&sink, 4096 * 16);
  hipMemset(d, 1, N * DIM * 2);
  run<0, 4>(d, sink, p.multiProcessorCount);
  run<0, 8>(d, sink, p.multiProcessorCount);
  run<1, 4>(d, sink, p.multiProcessorCount);
  run<1, 8>(d, sink, p.multiProcessorCount);
  run<0, 4>(d, sink, 2 * p.multiProcessorCount);
  run<1, 4>(d, sink, 2 * p.multiProcessorCount);
  hipFree(d);
  hipFree(sink);
  return 0;
}
