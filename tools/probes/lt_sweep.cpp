// Sweep of every hipBLASLt solution for the cross-encoder's four projection GEMMs at the
// hybrid_rerank shape (1280 pairs x 256 tokens = 327,680 rows, d 768, FFN 3072), fp16 in/out,
// fp32 accumulate, TN layout as F.linear issues it (y[M,N] = x[M,K] W[N,K]^T + bias).
// Prints the heuristic's first choice and the fastest supported solutions per shape (TFLOP/s),
// with the epilogue used by the forward (BIAS) and, for FFN-up, GELU_BIAS for comparison.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    auto _s = (x);                                                         \
    if ((int)_s != 0) {                                                    \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)_s); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

// random fp16 in [-1/32, 1/32) (a hash per element), so the MFMA operands toggle as real data does
__global__ void fill(uint16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13;
    p[i] = (uint16_t)(0x2000u | (x & 0x83ffu));  // exponent 8 (2^-7..), random mantissa and sign
  }
}

struct Shape {
  const char* name;
  long M, N, K;
};

static float time_algo(hipblasLtHandle_t h, hipblasLtMatmulDesc_t desc, hipblasLtMatrixLayout_t la,
                       hipblasLtMatrixLayout_t lb, hipblasLtMatrixLayout_t lc, const void* A,
                       const void* B, void* C, hipblasLtMatmulAlgo_t* algo, void* ws, size_t wsz,
                       int reps) {
  const float alpha = 1.f, beta = 0.f;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  if (hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, C, lc, C, lc, algo, ws, wsz, 0) != 0)
    return -1.f;
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r)
    (void)hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, C, lc, C, lc, algo, ws, wsz, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / reps;
}

int main(int argc, char** argv) {
  const long M = argc > 1 ? atol(argv[1]) : 327680;
  const int top = argc > 2 ? atoi(argv[2]) : 6;
  const int max_try = argc > 3 ? atoi(argv[3]) : 400;
  const bool scan = argc > 4 && argv[4][0] == 's';  // Q x C scan shapes instead
  const hipDataType out_t = argc > 5 && argv[5][0] == 'f' ? HIP_R_32F : HIP_R_16F;
  const Shape enc[] = {{"qkv", M, 2304, 768}, {"attn_out", M, 768, 768},
                       {"ffn_up", M, 3072, 768}, {"ffn_down", M, 768, 3072}};
  const Shape scn[] = {{"scan512", M, 512, 1024}, {"scan256", M, 256, 1024},
                       {"scan128", M, 128, 1024}, {"scan64", M, 64, 1024}};
  const Shape* shapes = scan ? scn : enc;
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  const size_t wsz = 256ull << 20;
  void* ws;
  CK(hipMalloc(&ws, wsz));
  void *A, *B, *C, *bias;
  CK(hipMalloc(&A, 3072L * 3072 * 2));
  CK(hipMalloc(&B, M * 3072 * 2));
  CK(hipMalloc(&C, M * 3072 * 4));
  CK(hipMalloc(&bias, 3072 * 2));
  fill<<<4096, 256>>>((uint16_t*)A, 3072L * 3072, 1u);
  fill<<<4096, 256>>>((uint16_t*)B, M * 3072, 2u);
  CK(hipDeviceSynchronize());
  CK(hipMemset(bias, 0, 3072 * 2));
  std::vector<hipblasLtMatmulHeuristicResult_t> all;
  CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, HIPBLAS_OP_T,
                                HIPBLAS_OP_N, HIP_R_16F, HIP_R_16F, out_t, out_t,
                                HIPBLAS_COMPUTE_32F, all));
  printf("solutions listed: %zu\n", all.size());
  for (int variant = 0; variant < (scan ? 4 : 5); ++variant) {
    const Shape& s = shapes[variant < 4 ? variant : 2];
    const bool gelu = variant == 4;
    const double flop = 2.0 * s.M * s.N * s.K;
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
    hipblasLtEpilogue_t ep = gelu ? HIPBLASLT_EPILOGUE_GELU_BIAS
                             : scan ? HIPBLASLT_EPILOGUE_DEFAULT : HIPBLASLT_EPILOGUE_BIAS;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    hipDataType bt = HIP_R_16F;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    hipblasLtMatrixLayout_t la, lb, lc;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16F, s.K, s.N, s.K));
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16F, s.K, s.M, s.K));
    CK(hipblasLtMatrixLayoutCreate(&lc, out_t, s.N, s.M, s.N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsz,
                                             sizeof(wsz)));
    hipblasLtMatmulHeuristicResult_t heur[8];
    int got = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 8, heur, &got));
    const int reps = 8;
    float t_h = time_algo(h, desc, la, lb, lc, A, B, C, &heur[0].algo, ws, wsz, reps);
    printf("%-9s%s M=%ld N=%ld K=%ld heuristic#0 %.3f ms %.0f TF/s  %s\n", s.name,
           gelu ? "+gelu" : "", s.M, s.N, s.K, t_h, flop / t_h * 1e-9,
           hipblaslt_ext::getKernelNameFromAlgo(h, heur[0].algo).c_str());
    std::vector<std::pair<float, int>> res;
    const float alpha = 1.f, beta = 0.f;
    int tried = 0;
    for (size_t i = 0; i < all.size() && tried < max_try; ++i) {
      size_t need = 0;
      if (hipblaslt_ext::matmulIsAlgoSupported(h, desc, &alpha, la, lb, &beta, lc, lc, all[i].algo,
                                               need) != HIPBLAS_STATUS_SUCCESS ||
          need > wsz)
        continue;
      ++tried;
      float t = time_algo(h, desc, la, lb, lc, A, B, C, &all[i].algo, ws, wsz, 3);
      if (t > 0) res.emplace_back(t, (int)i);
    }
    std::sort(res.begin(), res.end());
    printf("  supported+timed %d\n", tried);
    for (int j = 0; j < top && j < (int)res.size(); ++j) {
      auto& a = all[res[j].second].algo;
      float t = time_algo(h, desc, la, lb, lc, A, B, C, &a, ws, wsz, reps);
      printf("  idx %6d %.3f ms %.0f TF/s  %s\n", hipblaslt_ext::getIndexFromAlgo(a), t,
             flop / t * 1e-9, hipblaslt_ext::getKernelNameFromAlgo(h, a).c_str());
    }
    fflush(stdout);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(desc);
  }
  return 0;
}
