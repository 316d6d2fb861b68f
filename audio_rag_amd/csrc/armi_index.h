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
  int num_cus = 0;           // CUs of the device: the dense scans launch one workgroup each
  int device_cus = 0;        // CUs of the device
  int64_t* norm2 = nullptr;  // [n_tiles*32] exact sum of squares of the 2^24-scaled row (-1 = invalid)
  double* inv_norm = nullptr;    // [n_tiles*32] 1/sqrt(norm2)
  float* inv_norm32 = nullptr;   // [n_tiles*32] inv_norm * 2^24 as fp32 (NaN = invalid / padding)
  unsigned long long* invalid = nullptr;  // [1] count of rows outside the fp16 domain
  // int8 filter image of the rows (the first pass of the 64-query scan reads these 1-byte
  // components instead of the 2-byte fp16 ones): row r ~= s_r * rows8[r], s_r = max_i |x_ri| / 127
  int8_t* rows8 = nullptr;       // [n_tiles][dim / 16][32][16] round(x / s_r) (0 for invalid /
                                 // padding): 16-B chunk c of row r at tile r/32, chunk c, lane r%32
  float* a32 = nullptr;          // [n_tiles*32] s_r / |x_r| (score scale; NaN = invalid / padding)
  float* e32 = nullptr;          // [n_tiles*32] >= ||x_r - s_r rows8[r]||_2 / |x_r| (per unit |q|)
  // The int8 image (rows8, a32, e32) is stored in a SCATTERED row order: ordinal i sits at image
  // position img_pos(i) = 32 * ((i % T) * perm_mul % T) + i / T (T = n_tiles), so consecutive
  // ordinals (overlapping chunks of one recording: near-duplicate vectors) land in tiles about
  // 0.618 T apart, i.e. in different scan workgroups and lane lists, and a run of near-duplicates
  // never crowds one lane list. perm_inv = perm_mul^-1 mod T.
  int64_t perm_mul = 1;
  int64_t perm_inv = 1;
  int32_t* tile_ord = nullptr;   // [n_tiles] ordinal of image tile tau's row 0 = tau * perm_inv mod T
};

namespace armi {
// image position -> ordinal (may be >= n_rows for padding positions)
__host__ __device__ inline int64_t img_to_ord(int64_t pos, int64_t T, int64_t perm_inv) {
  const int64_t tau = pos >> 5;
  return (pos & 31) * T + (tau * perm_inv) % T;
}
__host__ __device__ inline int64_t ord_to_img(int64_t i, int64_t T, int64_t perm_mul) {
  return 32 * (((i % T) * perm_mul) % T) + i / T;
}
}  // namespace armi

// Sparse store: a device inverted index built at create time from the caller's CSR. Term t's
// postings (row, value) sit in [term_ptr[t], term_ptr[t+1]),
// ascending by row, the last slot a sentinel row (INT32_MAX); 64 sentinel slots pad the end.
// The rows are split into n_ranges contiguous ranges of range_rows rows (a multiple of 64), one
// scan workgroup each; terms with >= 256 postings carry start_tab[long_of[t]][range] = offset of
// their first posting at or after the range start.
struct armi_sparse_index {
  int device = 0;
  int64_t n_rows = 0;
  int64_t nnz = 0;
  int32_t vocab = 0;
  int64_t ordinal_base = 0;
  int num_cus = 0;
  int64_t range_rows = 0;
  int n_ranges = 0;
  int64_t n_postings = 0;        // valid postings + one sentinel per term
  int64_t n_long = 0;
  int32_t* term_ptr = nullptr;   // [vocab+1]
  int32_t* post = nullptr;       // [n_postings + 128][2]: (row, value bits) per posting
  int32_t* long_of = nullptr;    // [vocab] index into start_tab, -1 for short terms
  int32_t* start_tab = nullptr;  // [n_long][n_ranges]
  // Dense columns (round 4): a term in at least 1/8 of the rows also keeps its value bits per row
  // (0 = no posting, a zero value as -0.0, like the postings), so the scan stages its tile by one
  // coalesced load instead of cursor, ballot and scatter work.
  int32_t n_dense = 0;
  int64_t dense_stride = 0;      // words per column (rows rounded up, + one tile of zeros)
  int32_t* dense_of = nullptr;   // [vocab] column of the term, -1
  uint32_t* dense_val = nullptr; // [n_dense][dense_stride]
  // MFMA filter (round 6): every term in >= 1/32 of the rows has a u8 column of quantisation levels
  // a = ceil(v / term_scale[t]) in [0, 255] (a * term_scale >= v exactly; 0 = no posting or a zero
  // value), so a pass streams 1 B per row and term and scores upper bounds on the matrix cores;
  // the candidates are rescored exactly from the fp32 columns and the rare-value tables.
  bool filter_ok = false;        // every value >= 0 (the bound needs non-negative products)
  bool filter_on = true;         // armi_sparse_index_set_filter
  float* term_scale = nullptr;   // [vocab] RU(max value of the term / 255), 0 for empty terms
  int32_t n_col8 = 0;            // terms with a u8 column: df >= rows / 32
  int32_t* col8_of = nullptr;    // [vocab] u8 column of the term, -1
  int64_t dense8_stride = 0;     // bytes per u8 column (rows rounded up to a filter tile, + one)
  uint8_t* dense_u8 = nullptr;   // [n_col8][dense8_stride]
  int2* rare_of = nullptr;       // [vocab] rare-value table {first bucket, mask} or {-1, 0}
  uint2* rare_tab = nullptr;     // the filter rescore's (row, value bits) tables, 8 per bucket
  int64_t rare_slots = 0;
};

namespace armi {
constexpr int TILE_ROWS = 32;
constexpr float kTwoPow24 = 16777216.0f;
}  // namespace armi
