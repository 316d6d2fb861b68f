// Dense chunk-store construction: validation and exact per-row norms.
//
// Reference behaviour restated: Qdrant's COSINE distance normalises every vector at insert
// (QdrantRetriever._ensure_collection, src/audio_rag/retrieval/qdrant.py:93-109, and the
// per-point upserts of QdrantRetriever.add, qdrant.py:183-220). Instead of storing a rounded
// normalised copy, the store keeps the fp16 vector the encoder produced and an exact norm, so
// the search ranks by the exact cosine of those fp16 values.
#include <cmath>
#include <type_traits>

#include <vector>

#include "armi_index.h"

namespace {

// One wave per row: exact int64 sum of squares of the fixed-point (x * 2^24) image.
__global__ __launch_bounds__(256) void row_norms_kernel(const uint16_t* __restrict__ rows,
                                                        int64_t n_rows, int64_t n_padded,
                                                        int dim, int64_t* __restrict__ norm2,
                                                        double* __restrict__ inv_norm,
                                                        float* __restrict__ inv_norm32,
                                                        unsigned long long* __restrict__ invalid) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (row >= n_padded) return;
  if (row >= n_rows) {  // tile padding: never a result
    if (lane == 0) {
      norm2[row] = -1;
      inv_norm[row] = 0.0;
      inv_norm32[row] = __builtin_nanf("");
    }
    return;
  }
  const uint16_t* src = rows + row * (int64_t)dim;
  int64_t acc = 0;
  bool ok = true;
  for (int i = lane; i < dim; i += 64) {
    const uint32_t h = src[i];
    ok &= armi::fp16_in_domain(h);
    const int64_t v = armi::fp16_to_fixed24(h);
    acc += v * v;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  const bool row_ok = __all(ok);
  if (lane == 0) {
    if (!row_ok) {
      norm2[row] = -1;
      inv_norm[row] = 0.0;
      inv_norm32[row] = __builtin_nanf("");
      atomicAdd(invalid, 1ull);
    } else {
      norm2[row] = acc;
      const double inv = acc > 0 ? 1.0 / sqrt((double)acc) : 0.0;
      inv_norm[row] = inv;
      inv_norm32[row] = (float)(inv * 16777216.0);
    }
  }
}

// One wave per image position: the int8 filter image. s = max |x_i| / 127 (fp32),
// q_i = rint(x_i / s), a32 = s / |x|, e32 = ||x - s q||_2 / |x| rounded up (the quantisation term
// of the filter's score bound: |q.(x - s q)| / |x| <= |q| e32 by Cauchy-Schwarz). Image position
// pos holds ordinal img_to_ord(pos) (armi_index.h: the scattered order).
template <int DIM>
__global__ __launch_bounds__(256) void row_filter_kernel(const uint16_t* __restrict__ rows,
                                                         int64_t n_rows, int64_t n_padded,
                                                         int64_t n_tiles, int64_t perm_inv,
                                                         const double* __restrict__ inv_norm,
                                                         const int64_t* __restrict__ norm2,
                                                         int8_t* __restrict__ rows8,
                                                         float* __restrict__ a32,
                                                         float* __restrict__ e32) {
  constexpr int E = DIM / 64;
  const int lane = threadIdx.x & 63;
  const int64_t pos = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (pos >= n_padded) return;
  const int64_t row = n_tiles > 0 ? armi::img_to_ord(pos, n_tiles, perm_inv) : n_rows;
  // tile-blocked layout: 16-B chunk c of image row p sits at (p / 32) * 32 * DIM + c * 512 +
  // (p % 32) * 16, so the scan's wave-wide chunk loads (32 rows x 16 B per lane half) are
  // contiguous 512-B runs
  int8_t* tile = rows8 + (pos >> 5) * 32 * DIM + (pos & 31) * 16;
  auto dst_at = [&](int i) -> int8_t& { return tile[(i >> 4) * 512 + (i & 15)]; };
  if (row >= n_rows || norm2[row] < 0) {  // padding or invalid: never a result
#pragma unroll
    for (int i = 0; i < E; ++i) dst_at(lane + 64 * i) = 0;
    if (lane == 0) {
      a32[pos] = __builtin_nanf("");
      e32[pos] = 0.0f;
    }
    return;
  }
  const uint16_t* src = rows + row * DIM;
  float x[E];
  float mx = 0.0f;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    x[i] = (float)__builtin_bit_cast(_Float16, src[lane + 64 * i]);
    mx = fmaxf(mx, fabsf(x[i]));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
  const float s = mx > 0.0f ? mx / 127.0f : 1.0f;
  double err = 0.0;
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const float qv = fminf(fmaxf(rintf(x[i] / s), -127.0f), 127.0f);
    dst_at(lane + 64 * i) = (int8_t)qv;
    const double d = (double)x[i] - (double)s * (double)qv;  // exact in fp64
    err += d * d;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) err += __shfl_xor(err, off);
  if (lane == 0) {
    const double inv = inv_norm[row] * 16777216.0;  // 1 / |x|
    a32[pos] = (float)((double)s * inv);
    e32[pos] = (float)(sqrt(err) * inv * (1.0 + 1.0 / 1048576.0)) ;
  }
}

__global__ __launch_bounds__(256) void tile_ord_kernel(int64_t T, int64_t perm_inv,
                                                       int32_t* __restrict__ out) {
  const int64_t tau = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (tau < T) out[tau] = (int32_t)((tau * perm_inv) % T);
}

int64_t gcd64(int64_t a, int64_t b) {
  while (b) {
    const int64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// Modular inverse of a mod m (gcd(a, m) = 1), extended Euclid.
int64_t inv_mod(int64_t a, int64_t m) {
  if (m == 1) return 0;
  int64_t t = 0, nt = 1, r = m, nr = a % m;
  while (nr) {
    const int64_t q = r / nr;
    int64_t tmp = t - q * nt; t = nt; nt = tmp;
    tmp = r - q * nr; r = nr; nr = tmp;
  }
  return t < 0 ? t + m : t;
}

}  // namespace

extern "C" {

int armi_index_create(int device, const uint16_t* rows, int64_t n_rows, int dim,
                      int64_t ordinal_base, armi_index** out, hipStream_t stream) {
  ARMI_REQUIRE(out != nullptr, "armi_index_create: out is null");
  *out = nullptr;
  ARMI_REQUIRE(rows != nullptr || n_rows == 0, "armi_index_create: rows is null");
  ARMI_REQUIRE(n_rows >= 0 && n_rows < (int64_t(1) << 31) - 64,
               "armi_index_create: n_rows must be in [0, 2^31 - 64)");
  ARMI_REQUIRE(dim == 256 || dim == 512 || dim == 768 || dim == 1024,
               "armi_index_create: dim must be 256, 512, 768 or 1024");
  ARMI_HIP(hipSetDevice(device));
  armi_index* idx = new armi_index();
  idx->device = device;
  idx->rows = rows;
  idx->n_rows = n_rows;
  idx->n_tiles = (n_rows + armi::TILE_ROWS - 1) / armi::TILE_ROWS;
  idx->dim = dim;
  idx->ordinal_base = ordinal_base;
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) { delete idx; return armi::hip_fail(e, "hipGetDeviceProperties"); }
  idx->num_cus = prop.multiProcessorCount;
  idx->device_cus = prop.multiProcessorCount;
  // scattered image order: multiplier ~ 0.618 T, coprime with T (armi_index.h)
  if (idx->n_tiles > 1) {
    const int64_t T = idx->n_tiles;
    int64_t p = std::max<int64_t>(1, (int64_t)((double)T * 0.6180339887498949));
    while (gcd64(p, T) != 1) ++p;
    idx->perm_mul = p % T;
    idx->perm_inv = inv_mod(idx->perm_mul, T);
  } else {
    idx->perm_mul = idx->perm_inv = 1;
  }
  const int64_t padded = std::max<int64_t>(idx->n_tiles * armi::TILE_ROWS, 1);
  e = hipMalloc(&idx->norm2, padded * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&idx->inv_norm, padded * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&idx->inv_norm32, padded * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&idx->invalid, sizeof(unsigned long long));
  // whole 32-row tiles (the tile-blocked layout), also for an empty store
  const int64_t tiled = std::max<int64_t>(idx->n_tiles, 1) * armi::TILE_ROWS;
  if (e == hipSuccess) e = hipMalloc(&idx->rows8, tiled * dim);
  if (e == hipSuccess) e = hipMalloc(&idx->a32, padded * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&idx->e32, padded * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&idx->tile_ord, std::max<int64_t>(idx->n_tiles, 1) * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemsetAsync(idx->invalid, 0, sizeof(unsigned long long), stream);
  if (e != hipSuccess) { armi_index_destroy(idx); return armi::hip_fail(e, "armi_index_create alloc"); }
  {
    const int64_t T = std::max<int64_t>(idx->n_tiles, 1);
    tile_ord_kernel<<<dim3((unsigned)((T + 255) / 256)), dim3(256), 0, stream>>>(
        idx->n_tiles > 0 ? T : 1, idx->perm_inv, idx->tile_ord);
    e = hipGetLastError();
    if (e != hipSuccess) { armi_index_destroy(idx); return armi::hip_fail(e, "tile_ord_kernel"); }
  }
  const int64_t blocks = (padded + 3) / 4;
  row_norms_kernel<<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(
      rows, n_rows, padded, dim, idx->norm2, idx->inv_norm, idx->inv_norm32, idx->invalid);
  e = hipGetLastError();
  if (e != hipSuccess) { armi_index_destroy(idx); return armi::hip_fail(e, "row_norms_kernel"); }
  auto filt = [&](auto D) {
    row_filter_kernel<decltype(D)::value><<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(
        rows, n_rows, padded, idx->n_tiles, idx->perm_inv, idx->inv_norm, idx->norm2, idx->rows8,
        idx->a32, idx->e32);
  };
  switch (dim) {
    case 256: filt(std::integral_constant<int, 256>{}); break;
    case 512: filt(std::integral_constant<int, 512>{}); break;
    case 768: filt(std::integral_constant<int, 768>{}); break;
    default: filt(std::integral_constant<int, 1024>{}); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) { armi_index_destroy(idx); return armi::hip_fail(e, "row_filter_kernel"); }
  *out = idx;
  return ARMI_OK;
}

int armi_index_destroy(armi_index* idx) {
  if (!idx) return ARMI_OK;
  hipFree(idx->norm2);
  hipFree(idx->inv_norm);
  hipFree(idx->inv_norm32);
  hipFree(idx->invalid);
  hipFree(idx->rows8);
  hipFree(idx->a32);
  hipFree(idx->e32);
  hipFree(idx->tile_ord);
  delete idx;
  return ARMI_OK;
}

int64_t armi_index_rows(const armi_index* idx) { return idx ? idx->n_rows : -1; }

int armi_index_dim(const armi_index* idx) { return idx ? idx->dim : -1; }


int64_t armi_index_invalid_rows(const armi_index* idx) {
  if (!idx) return -1;
  unsigned long long v = 0;
  if (hipMemcpy(&v, idx->invalid, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int64_t)v;
}

int armi_index_norms(const armi_index* idx, const int64_t** norm2, const double** inv_norm,
                     const float** inv_norm32) {
  ARMI_REQUIRE(idx != nullptr, "armi_index_norms: index is null");
  if (norm2) *norm2 = idx->norm2;
  if (inv_norm) *inv_norm = idx->inv_norm;
  if (inv_norm32) *inv_norm32 = idx->inv_norm32;
  return ARMI_OK;
}

}  // extern "C"
