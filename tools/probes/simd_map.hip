// Which SIMD each wave of a 512-thread workgroup lands on (HW_ID.SIMD_ID), to check the
// pairing the phase-pipelined scan's stagger assumes (waves w and w + 4 on one SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void simd_map(int* out) {
  // s_getreg_b32 HW_REG_HW_ID (id 4), bits [5:4] = SIMD_ID, [11:8] = CU_ID
  const int hw = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);  // 2 bits at offset 4
  const int cu = __builtin_amdgcn_s_getreg((3 << 11) | (8 << 6) | 4);  // 4 bits at offset 8
  __shared__ int pad[40000];  // 160 KB-ish: one workgroup per CU, like the scan
  pad[threadIdx.x] = hw;
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
    out[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 2] = pad[threadIdx.x] | (cu << 8);
}

int main() {
  const int nb = 256;
  int* d;
  hipMalloc(&d, nb * 8 * 2 * sizeof(int));
  simd_map<<<nb, 512>>>(d);
  std::vector<int> h(nb * 8 * 2);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  int same4 = 0, same1 = 0, same2 = 0;
  for (int b = 0; b < nb; ++b) {
    int s[8];
    for (int w = 0; w < 8; ++w) s[w] = h[(b * 8 + w) * 2] & 3;
    for (int w = 0; w < 4; ++w) same4 += s[w] == s[w + 4];
    for (int w = 0; w < 8; w += 2) same1 += s[w] == s[w + 1];
    for (int w = 0; w < 8; ++w) same2 += s[w] == s[w ^ 2];
    if (b < 6) {
      printf("block %d:", b);
      for (int w = 0; w < 8; ++w) printf(" w%d->simd%d", w, s[w]);
      printf("\n");
    }
  }
  printf("pairs sharing a SIMD: (w, w+4) %d/%d, (2i, 2i+1) %d/%d, (w, w^2) %d/%d\n", same4,
         nb * 4, same1, nb * 4, same2, nb * 8);
  return 0;
}
