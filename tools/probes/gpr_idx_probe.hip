// Micro-benchmark of the register scan's accumulate step (sparse.hip, sparse_scan_reg_kernel):
// cycles per (weight, slot) pair for
//   A: packed multiply + packed add into a statically chosen accumulator pair,
//   B: the same add through VGPR index mode with the slot in an SGPR (s_set_gpr_idx_on),
//   C: B with the slot first moved from a VGPR by v_readfirstlane (as the LDS-fed pair loop).
// One workgroup of 256 threads per CU, 4096 pairs per wave; prints cycles per pair per wave.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(const float* __restrict__ in, float* __restrict__ out,
                                             long long* __restrict__ cyc, int iters) {
  const int lane = threadIdx.x & 63;
  f2 v = f2{in[lane], in[lane + 64]};
  v16f acc = 0.f;
  int qv = (lane * 0) + 2;  // VGPR copy of the slot (all lanes equal)
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
    const float w = __int_as_float(0x3f000000 + (i & 7));
    const f2 x = v * f2{w, w};
    if constexpr (MODE == 0) {
      const int s = i & 7;
      // static slot via a switch on the low bits (the compiler emits straight-line adds per case)
      switch (s) {
        case 0: acc.s01 += x; break;
        case 1: acc.s23 += x; break;
        case 2: acc.s45 += x; break;
        case 3: acc.s67 += x; break;
        case 4: acc.s89 += x; break;
        case 5: acc.sab += x; break;
        case 6: acc.scd += x; break;
        default: acc.sef += x; break;
      }
    } else {
      int q2;
      if constexpr (MODE == 1) {
        q2 = (i * 2) & 14;
      } else {
        q2 = __builtin_amdgcn_readfirstlane(qv);
        qv = (qv + 2) & 14;
      }
      asm volatile(
          "s_set_gpr_idx_on %1, gpr_idx(SRC0,DST)\n\t"
          "v_pk_add_f32 v[64:65], v[64:65], %2\n\t"
          "s_set_gpr_idx_off"
          : "+{v[64:79]}"(acc)
          : "s"(q2), "v"(x));
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int blocks = 256, iters = 4096;
  float *in, *out;
  long long* cyc;
  hipMalloc(&in, 128 * 4);
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 8);
  float h[128];
  for (int i = 0; i < 128; ++i) h[i] = 0.01f * (i + 1);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[3] = {"A static add", "B index-mode add, slot in SGPR",
                          "C index-mode add, slot via v_readfirstlane"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) probe<0><<<blocks, 256>>>(in, out, cyc, iters);
      if (mode == 1) probe<1><<<blocks, 256>>>(in, out, cyc, iters);
      if (mode == 2) probe<2><<<blocks, 256>>>(in, out, cyc, iters);
      hipDeviceSynchronize();
    }
    long long hc[blocks];
    hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int b = 0; b < blocks; ++b) avg += (double)hc[b];
    avg /= blocks;
    printf("%-45s %.1f clock64 ticks per pair (one wave per SIMD)\n", names[mode], avg / iters);
  }
  return 0;
}
