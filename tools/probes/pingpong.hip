// Microbenchmark of the two-waves-per-SIMD ping-pong (tiled scan design): per phase every wave
// does LOAD (NREAD ds_read_b128 + lgkmcnt(0)) -> s_barrier -> MATH (8 v_mfma_f32_32x32x16_f16)
// -> s_barrier, waves 4-7 one barrier behind waves 0-3 (they share SIMDs with 0-3). Variants:
//   acc=v : accumulators in ArchVGPRs (what hipcc picks for a <= 256-register kernel)
//   acc=a : accumulators pinned to AccVGPRs a[0:31] by inline asm
//   nread : ds_read_b128 per LOAD (0 = none); stagger 0/1; mfma 0/1
// Prints cycles per phase (s_memtime around the loop, wave 0 of each workgroup, median).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int ACC_A, int NREAD, int STAGGER, int MFMA, int GLDS = 0, int INFL = 3>
__global__ __launch_bounds__(512) void pingpong(long long* out, int iters, float* sink,
                                                const uint16_t* src, long long src_elems) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 65536 / 4; i += 512) reinterpret_cast<float*>(smem)[i] = 0.001f * i;
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)smem +
                        (uint32_t)(((wave * 64 + lane) * 16) & 65535);
  u32x4 fr[12];
  for (int j = 0; j < 12; ++j) fr[j] = u32x4{(uint32_t)j, 1u, 2u, 3u};
  f32x16 c0 = {}, c1 = {};
  u32x4 stage0 = {0u, 0u, 0u, 0u}, stage1 = {0u, 0u, 0u, 0u};
  if (STAGGER && wave >= 4) __builtin_amdgcn_s_barrier();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (GLDS == 2) {
      // register staging of the same 2 KB: 2 x global_load_dwordx4 (16 B / lane) -> 2 x
      // ds_write_b128 into the upper 64 KB, the loads issued one phase ahead of their write
      const long long e = ((((long long)blockIdx.x * iters + it) * 16 + wave * 2) * 512 + lane * 8) &
                          (src_elems - 1);
      u32x4 x0 = *reinterpret_cast<const u32x4*>(src + e);
      u32x4 x1 = *reinterpret_cast<const u32x4*>(src + ((e + 512) & (src_elems - 1)));
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      const uint32_t wa = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(smem + 65536 + ((it & 3) * 16 + wave * 2) * 1024) + lane * 16;
      asm volatile("ds_write_b128 %0, %1" :: "v"(wa), "v"(stage0) : "memory");
      asm volatile("ds_write_b128 %0, %1 offset:1024" :: "v"(wa), "v"(stage1) : "memory");
      stage0 = x0;
      stage1 = x1;
    } else if (GLDS) {
      // 2 x 1 KB LDS-DMA per wave into the upper 64 KB (8 rows x 128 B each, like the scan's
      // pieces), streaming through `src`; then keep 3 phases (6 instructions) in flight
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const long long e = ((((long long)blockIdx.x * iters + it) * 16 + wave * 2 + i) * 512 +
                             lane * 8) & (src_elems - 1);  // power-of-two sizes
        __builtin_amdgcn_global_load_lds(src + e,
                                         (__attribute__((address_space(3))) void*)(smem + 65536 + ((it & 3) * 16 + wave * 2 + i) * 1024),
                                         16, 0, 0);
      }
      if constexpr (INFL == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      if constexpr (INFL == 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      if constexpr (INFL == 7) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
      if constexpr (INFL == 11) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
    }
#pragma unroll
    for (int j = 0; j < NREAD; ++j)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fr[j]) : "v"(base), "i"(j * 1024 % 65536));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    if (MFMA) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (ACC_A) {
          asm volatile("v_mfma_f32_32x32x16_f16 a[0:15], %0, %1, a[0:15]" ::"v"(fr[2 * k]), "v"(fr[8 + k])
                       : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11",
                         "a12", "a13", "a14", "a15");
          asm volatile("v_mfma_f32_32x32x16_f16 a[16:31], %0, %1, a[16:31]" ::"v"(fr[2 * k + 1]), "v"(fr[8 + k])
                       : "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25",
                         "a26", "a27", "a28", "a29", "a30", "a31");
        } else {
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, fr[2 * k]),
                                                      __builtin_bit_cast(half8, fr[8 + k]), c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, fr[2 * k + 1]),
                                                      __builtin_bit_cast(half8, fr[8 + k]), c1, 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (STAGGER && wave < 4) __builtin_amdgcn_s_barrier();
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j];
  for (int j = 0; j < 12; ++j) s += __uint_as_float(fr[j].x);
  s += __uint_as_float(stage0.x) + __uint_as_float(stage1.y);
  if (s == 123.456f) sink[threadIdx.x] = s;
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int A, int R, int S, int M, int G = 0, int I = 3>
void run(const char* name, int iters, long long src_elems = 1 << 20) {
  const int nb = 256;
  long long* d;
  float* sink;
  (void)hipMalloc(&d, nb * sizeof(long long));
  (void)hipMalloc(&sink, 512 * sizeof(float));
  uint16_t* src;
  (void)hipMalloc(&src, src_elems * 2);
  (void)hipMemset(src, 0, src_elems * 2);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pingpong<A, R, S, M, G, I>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  for (int rep = 0; rep < 2; ++rep) pingpong<A, R, S, M, G, I><<<nb, 512, 131072>>>(d, iters, sink, src, src_elems);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  pingpong<A, R, S, M, G, I><<<nb, 512, 131072>>>(d, iters, sink, src, src_elems);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> h(nb);
  (void)hipMemcpy(h.data(), d, nb * sizeof(long long), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH.md constants table)
  printf("%-34s %8.1f ticks/phase  %7.3f ms  (%.0f ns/phase)\n", name, (double)h[nb / 2] / iters,
         ms, ms * 1e6 / iters);
  (void)hipFree(d);
  (void)hipFree(sink);
  (void)hipFree(src);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  run<0, 8, 1, 1>("nread=8 no staging", iters);
  run<0, 8, 1, 1, 1, 3>("nread=8 glds L2", iters, 1 << 20);
  run<0, 8, 1, 1, 2, 3>("nread=8 regstage L2", iters, 1 << 20);
  run<0, 8, 1, 1, 1, 3>("nread=8 glds HBM", iters, 1LL << 30);
  run<0, 8, 1, 1, 2, 3>("nread=8 regstage HBM", iters, 1LL << 30);
  run<0, 8, 1, 0, 2, 3>("nread=8 regstage L2 mfma=0", iters, 1 << 20);
  run<0, 8, 0, 1, 2, 3>("nread=8 regstage L2 stagger=0", iters, 1 << 20);
  return 0;
}
