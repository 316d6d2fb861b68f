// Device-resident chunk-store layouts shared by the index builders and the search kernels.
#pragma once

#include "armi_common.h"

// Dense store. Rows stay caller-owned fp16 [n_rows][dim]; the index owns the per-row norm
// arrays, padded to a whole number of 32-row tiles so the scan never reads past them.
struct armi_index {
  int device = 0;
  const uint16_t* rows = nullptr;
  int64_t n_rows = 0;
  int64_t n_tiles = 0;       // ceil(n_rows / 32)
  int dim = 0;
  int64_t ordinal_base = 0;
  int num_cus = 0;
  int64_t* norm2 = nullptr;  // [n_tiles*32] exact sum of squares of the 2^24-scaled row (-1 = invalid)
  double* inv_norm = nullptr;    // [n_tiles*32] 1/sqrt(norm2)
  float* inv_norm32 = nullptr;   // [n_tiles*32] inv_norm * 2^24 as fp32 (NaN = invalid / padding)
  unsigned long long* invalid = nullptr;  // [1] count of rows outside the fp16 domain
};

// Sparse store: caller-owned CSR plus a device inverted index (postings) built at create time.
struct armi_sparse_index {
  int device = 0;
  int64_t n_rows = 0;
  int64_t nnz = 0;
  int32_t vocab = 0;
  int64_t ordinal_base = 0;
  int num_cus = 0;
  const int64_t* indptr = nullptr;
  const int32_t* indices = nullptr;
  const float* values = nullptr;
};

namespace armi {
constexpr int TILE_ROWS = 32;
constexpr float kTwoPow24 = 16777216.0f;
}  // namespace armi
