// Certified MFMA filter of the sparse search (round 6). Included by sparse.hip inside its
// anonymous namespace: uses its pass layout (QTerm lists per query slot, the pass's ascending
// distinct terms uterm[u]), range partition, range_cursor, ord_key_f and the candidate-list
// workspace of the exact scan.
//
// Restates the same search as sparse.hip (Qdrant's sparse dot product, qdrant.py:289-312):
// score(q, d) = fp32 sum, ascending shared index, of fl32(q_i * d_i). The exact scan computes it
// for every row with one VALU multiply and add per (query, term, row), and three rounds of tuning
// left it issue-bound at ~0.18 ms per 64-query pass. Here every row instead gets an
// UPPER BOUND of its score from the matrix cores, and only the best few rows per query are
// scored exactly:
//
//   index build: every value v >= 0 of a term in >= 1/32 of the rows (a u8 column) is stored as
//     the u8 level a = ceil(v / s_t), s_t = RU(max_t / 255), so a * s_t >= v exactly (1 B per row
//     and term, half of the fp16 bytes and a quarter of the fp32 columns the exact scan reads);
//     posting terms (df < rows / 32) get their levels from the same rule while they are staged.
//   per pass (prep): B[u][q] = RU16(w_qu * s_u * 2^e) >= w * s * 2^e, one fp16 per (term, query),
//     e chosen per pass to keep B well inside fp16's range (never subnormal: clamped to 2^-14).
//   scan: rows in 1024-row tiles, the pass's terms in 16-term steps. Each step stages the u8
//     column tiles (one 16-B load per lane, prefetched four steps ahead in registers; a posting
//     term's next 128 postings, scattered) into a [16 term][1024 row] fp16 LDS image, and
//     v_mfma_f32_32x32x16_f16 multiplies it (A operand by ds_read_b64_tr_b16: the image is
//     term-major, the operand wants 8 terms of one row per lane) with the step's B slice. key =
//     acc * scale_up >= the row's exact fp32 score: every product a * B >= w * v, and the fp32
//     roundings of both the reference's sum and the MFMA accumulation are covered by
//     scale_up = 2^-e (1 + (nU + 600) 2^-22) (at most 2 (256 + 2 nU) roundings of 2^-23 each).
//     Per lane x query a 3-deep list of (key, row) plus the largest key it dropped; per
//     workgroup and query the best 16 entries and a bound on everything else.
//   merge (per query): the pool's entries from the kc-th largest list maximum up are rescored
//     exactly (the value of each query term in the row from the term's fp32 column, df >= rows/8,
//     or its postings; the products of the shared terms added in ascending
//     term order: the oracle's and the exact scan's arithmetic); the query is CERTIFIED when its
//     k-th exact score exceeds every bound of a row not rescored (keys never under-state a
//     score), and then answered. Queries that cannot be certified (ties at the boundary, fewer
//     than k sharing rows, negative weights) keep their flags and take the exact scan, which
//     skips certified queries and exits at once when none is left.
//
// Limits: an index with a negative value, a pass of more than 512 distinct terms or k > 128
// does not use the filter (the exact scan answers), and neither does a query with a negative or
// non-finite weight.

constexpr int kFT = 1024;                      // rows per filter tile
constexpr int kFK = 16;                        // terms per step (one MFMA k-step)
constexpr int kFWaves = 8;
constexpr int kFThreads = kFWaves * 64;
constexpr int kFDepth = 4;                     // steps in flight (register ring)
constexpr int kFMaxSeg = 32;                   // a held term per lane pair: 32 steps of 16 terms
constexpr int kFMaxU = kFMaxSeg * kFK;         // distinct terms of a filtered pass, at most 512
constexpr int kFImgStride = kFT * 2 + 64;      // bytes per term row of the image (+64: the
                                               // transposed reads of a half-wave hit 64 banks)
constexpr int kFImgBytes = kFK * kFImgStride;
constexpr int kFBBytes = kQB * kFK * 2;        // one B slice [q][16] fp16 (2 KB), in the
constexpr int kFBSlice = kQB * kFK;            // workspace and, for every step, in LDS
constexpr int kFList = 3;                      // lane list depth
constexpr int kFLanes = 2 * kFWaves;           // lane lists per query and workgroup
constexpr int kFPool = kFLanes * kFList;       // their entries (48)
constexpr size_t kFLds = (size_t)2 * kFImgBytes + (size_t)kFMaxSeg * kFBBytes + 256;
constexpr int kFSel = 1024;                    // rescored candidates per query, at most
constexpr int kFVal = 8192;                    // (row, term) value slots of one rescore chunk
constexpr int kFMaxK = 128;
constexpr int32_t kFNone = (int32_t)0x80000000;  // held-term cursor of "no term"
static_assert(kQB * kFPool * 8 + kQB * kFLanes * 4 <= 2 * kFImgBytes, "merge overlays the images");
static_assert(2 * kFImgBytes + kFMaxSeg * kFBBytes + 256 <= 160 * 1024, "LDS of the filter scan");
static_assert(kFMaxSeg * 2 <= 64, "one lane per held term");

#ifdef ARMI_SPARSE_PROFILE
// Profiling build only (ARMI_BUILD_FLAGS=-DARMI_SPARSE_PROFILE, ARMI_SPARSE_DBG=8): 100 MHz stamps
// per scan wave (issue, compute, epilogue, finish, barrier, prologue, steps) and per merge query
// (phase ends: pool, selection, rescore, rank, rounds)
__device__ unsigned long long g_fscan_prof[kMaxRanges * kFWaves * 8];
__device__ unsigned long long g_fmerge_prof[kQB * 16];
#define ARMI_FP_T(x) x = wall_clock64()
#else
#define ARMI_FP_T(x) (void)0
#endif

__host__ __device__ inline int filter_segments(int n_u) {
  const int s = (n_u + kFK - 1) / kFK;
  return s > kFDepth - 1 ? s : kFDepth - 1;  // a term's next tile issues after its last finish
}

typedef _Float16 fhalf2 __attribute__((ext_vector_type(2)));
typedef _Float16 fhalf8 __attribute__((ext_vector_type(8)));
typedef float ff32x16 __attribute__((ext_vector_type(16)));
typedef short fs4 __attribute__((ext_vector_type(4)));
typedef uint32_t fu32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t fu32x2 __attribute__((ext_vector_type(2)));
typedef int32_t fp4 __attribute__((ext_vector_type(4), aligned(8)));

// A posting window loaded and waited for inside one asm block: the rare continuation loads of
// a tile that holds more than 128 postings of a term. As a plain load the compiler's wait-count
// pass cannot tell whether it ran, and waited vmcnt(0) for it at the top of every step, i.e. for
// the whole prefetch ring (the scan then ran one memory round trip per step).
__device__ __forceinline__ fp4 load_window_sync(const int2* p) {
  fp4 v;
  asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// Quantisation level of a value: the least integer a with a * s >= v (a in [0, 255] since
// 255 s >= the term's largest value; 0 for v = 0 or -0.0). The fixup makes the bound exact
// whatever the rounding of the division (the product is exact in fp64).
__host__ __device__ inline float u8_level(float v, float s) {
  if (!(v > 0.f) || !(s > 0.f)) return 0.f;
  float a = ceilf(v / s);
  if ((double)a * (double)s < (double)v) a += 1.f;
  return a > 255.f ? 255.f : a;
}

// The scan's level of a posting value (v >= 0, s > 0, inv ~ 1/s): a valid bound like u8_level
// (a * s >= v, a <= 255) without a division: ceil(v * inv) is at most one below ceil(v / s)
// (v / s <= 255, two roundings of 2^-24), and the sign of fma(a, s, -v) (one rounding of the
// exact a * s - v) says whether a * s >= v; on equality (or an underflowed difference) one level
// more keeps the bound safe. It may exceed u8_level's level by one; any a with a * s >= v is a
// valid bound, and 255 s >= v for every value of the term.
__device__ __forceinline__ float u8_level_fast(float v, float s, float inv) {
  float a = ceilf(v * inv);
  a += fmaf(a, s, -v) <= 0.f && v > 0.f ? 1.f : 0.f;
  return fminf(a, 255.f);
}

// 4 bytes -> 4 fp16 (exact): byte b as fp16 bits 0x64bb = 1024 + b, minus 1024.
__device__ __forceinline__ fu32x2 u8x4_f16(uint32_t x) {
  const fhalf2 l = __builtin_bit_cast(fhalf2, __builtin_amdgcn_perm(0x64646464u, x, 0x04010400u));
  const fhalf2 h = __builtin_bit_cast(fhalf2, __builtin_amdgcn_perm(0x64646464u, x, 0x04030402u));
  const fhalf2 o = {(_Float16)1024.0f, (_Float16)1024.0f};
  return fu32x2{__builtin_bit_cast(uint32_t, l - o), __builtin_bit_cast(uint32_t, h - o)};
}

// Smallest fp16 >= p (p >= 0; +inf above the fp16 range), never subnormal (>= 2^-14 for p > 0):
// the MFMA operand of a weight * scale product.
__device__ __forceinline__ uint16_t ru_half(double p) {
  if (!(p > 0.0)) return 0;
  float f = (float)p;
  if ((double)f < p) f = __uint_as_float(__float_as_uint(f) + 1u);
  uint16_t b = __builtin_bit_cast(uint16_t, (_Float16)f);
  if ((float)__builtin_bit_cast(_Float16, b) < f) b = (uint16_t)(b + 1);
  return b < 0x0400 ? (uint16_t)0x0400 : b;
}

// ---------------------------------------------------------------------------- index build

// tmax[t] = bit pattern of the largest value of term t (values >= 0 order as their bits;
// -0.0 counts as 0), n_neg = values < 0. Over the postings sorted by term (sorted entry i: see
// dense_fill): a wave reduces its runs of one term first, so only the first lane of a run issues
// the atomic (the CSR-order form's atomics on the hot terms took 21 ms per 96M values).
__global__ void term_max_kernel(const uint32_t* __restrict__ skeys, const int2* __restrict__ post,
                                int64_t nnz, int32_t vocab, uint32_t* __restrict__ tmax,
                                unsigned long long* __restrict__ n_neg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  uint32_t t = 0xffffffffu, m = 0u;
  bool neg = false;
  if (i < nnz) {
    t = skeys[i];
    if (t < (uint32_t)vocab) {
      const float v = __int_as_float(post[i + t].y);
      neg = v < 0.f;
      m = v > 0.f ? __float_as_uint(v) : 0u;
    } else {
      t = 0xffffffffu;
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {  // segmented max over the wave's run of term t
    const uint32_t mo = __shfl_down(m, d), to = __shfl_down(t, d);
    if (lane + d < 64 && to == t) m = max(m, mo);
  }
  const uint32_t tp = __shfl_up(t, 1);
  if ((lane == 0 || tp != t) && t != 0xffffffffu && m) atomicMax(&tmax[t], m);
  const unsigned long long b = __ballot(neg);
  if (lane == 0 && b) atomicAdd(n_neg, (unsigned long long)__popcll(b));
}

// s_t = the least fp32 >= max_t / 255 with 255 s_t >= max_t (checked in fp64)
__global__ void term_scale_kernel(const uint32_t* __restrict__ tmax, int32_t vocab,
                                  float* __restrict__ scale) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= vocab) return;
  const float m = __uint_as_float(tmax[t]);
  float s = m / 255.f;
  while (255.0 * (double)s < (double)m) s = __uint_as_float(__float_as_uint(s) + 1u);
  scale[t] = m > 0.f ? s : 0.f;
}

// terms with a u8 column: df >= rows / kCol8Frac (a wider set than the exact scan's fp32
// columns: a posting term then holds <= ~32 postings per 1024-row tile on average, so a tile
// almost never needs a second 128-posting window, whose synchronous load stalls the workgroup)
constexpr int kCol8Frac = 32;
__global__ void col8_flag_kernel(const int32_t* __restrict__ term_ptr, int32_t vocab,
                                 int64_t n_rows, int32_t* __restrict__ flag) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < vocab) {
    const int64_t df = term_ptr[t + 1] - 1 - term_ptr[t];
    flag[t] = (df > 0 && df * kCol8Frac >= n_rows) ? 1 : 0;
  } else if (t == vocab) {
    flag[t] = 0;
  }
}

// u8 level of every posting of a u8-column term into its column (sorted entry i: see dense_fill)
__global__ void dense_u8_fill_kernel(const int32_t* __restrict__ dense_of,
                                     const int2* __restrict__ post,
                                     const uint32_t* __restrict__ skeys, int64_t nnz, int32_t vocab,
                                     const float* __restrict__ scale, int64_t stride,
                                     uint8_t* __restrict__ dense_u8) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint32_t t = skeys[i];
  if (t >= (uint32_t)vocab) return;
  const int32_t d = dense_of[t];
  if (d < 0) return;
  const int2 pv = post[i + t];
  dense_u8[(size_t)d * stride + pv.x] = (uint8_t)u8_level(__int_as_float(pv.y), scale[t]);
}

// The rescore's values of the terms without an fp32 column (df < rows / 8): per term t an
// open-addressed table of 2^m buckets of 8 (row, value bits) slots (64 B), a row in one of two
// buckets (two-choice: the emptier at insert), so a lookup is two independent 64-B loads, whatever
// the term's df (a search of its postings was a chain of ~10 dependent loads, ~25 us a query).
// Empty slots hold row -1. rare_of[t] = {first bucket, 2^m - 1}, {-1, 0} for no table.
constexpr int kRareSlots = 8;

__host__ __device__ inline uint32_t rare_hash1(uint32_t row, uint32_t t) {
  uint32_t h = row * 0x9E3779B1u ^ (t * 0x85EBCA77u + 0x165667B1u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

__host__ __device__ inline uint32_t rare_hash2(uint32_t h1) {
  uint32_t h = h1 ^ 0x68E31DA4u;
  h *= 0xB5297A4Du;
  h ^= h >> 13;
  h *= 0x1B56C4E9u;
  h ^= h >> 16;
  return h;
}

// buckets of term t: the least power of two >= df / div (div = 4: 2-4 rows per bucket on average)
__global__ void rare_buckets_kernel(const int32_t* __restrict__ term_ptr,
                                    const int32_t* __restrict__ dense_of, int32_t vocab, int div,
                                    int32_t* __restrict__ nb) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > vocab) return;
  int32_t b = 0;
  if (t < vocab && dense_of[t] < 0) {
    const int64_t df = term_ptr[t + 1] - 1 - term_ptr[t];
    if (df > 0) {
      b = 1;
      while ((int64_t)b * div < df) b <<= 1;
    }
  }
  nb[t] = b;
}

__global__ void rare_of_kernel(const int32_t* __restrict__ nb, const int32_t* __restrict__ scan,
                               int32_t vocab, int2* __restrict__ rare_of) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= vocab) return;
  rare_of[t] = nb[t] > 0 ? make_int2(scan[t], nb[t] - 1) : make_int2(-1, 0);
}

// every posting of a table term into the emptier of its two buckets; when both are full, into
// the first bucket after the second (cyclically in the term's table) that has room (a chain the
// lookup follows only when both of a row's buckets are full); fail counts postings that found the
// whole table full (never at these loads; the build then retries with more buckets)
__global__ void rare_insert_kernel(const int2* __restrict__ rare_of, const int2* __restrict__ post,
                                   const uint32_t* __restrict__ skeys, int64_t nnz, int32_t vocab,
                                   int32_t* __restrict__ fill, uint2* __restrict__ tab,
                                   int32_t* __restrict__ fail) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const uint32_t t = skeys[i];
  if (t >= (uint32_t)vocab) return;
  const int2 ro = rare_of[t];
  if (ro.x < 0) return;
  const int2 pv = post[i + t];
  const uint32_t h1 = rare_hash1((uint32_t)pv.x, t);
  const uint32_t c1 = h1 & (uint32_t)ro.y, c2 = rare_hash2(h1) & (uint32_t)ro.y;
  const uint32_t first = fill[ro.x + c2] < fill[ro.x + c1] ? c2 : c1;
  uint32_t c = first;
  int s = atomicAdd(&fill[ro.x + c], 1);
  if (s >= kRareSlots) {
    c = first == c1 ? c2 : c1;
    s = atomicAdd(&fill[ro.x + c], 1);
  }
  for (uint32_t step = 1; s >= kRareSlots && step <= (uint32_t)ro.y; ++step) {
    c = (c2 + step) & (uint32_t)ro.y;
    s = atomicAdd(&fill[ro.x + c], 1);
  }
  if (s >= kRareSlots) {
    atomicAdd(fail, 1);
    return;
  }
  tab[((int64_t)ro.x + c) * kRareSlots + s] = make_uint2((uint32_t)pv.x, (uint32_t)pv.y);
}

// the value bits of row r in term table {base, mask} (t the term), 0 when r has no posting (a
// zero value is stored as -0.0): its two buckets in one round of loads; only when both are full
// (slot 7 taken) and neither holds r, the chain after the second bucket up to a bucket with room
__device__ __forceinline__ uint32_t rare_value(const uint2* __restrict__ tab, int32_t base,
                                               int32_t mask, uint32_t t, int32_t r) {
  const uint32_t h1 = rare_hash1((uint32_t)r, t);
  const uint32_t c2 = rare_hash2(h1) & (uint32_t)mask;
  const uint4* p1 = reinterpret_cast<const uint4*>(tab + (base + (int64_t)(h1 & (uint32_t)mask)) * kRareSlots);
  const uint4* p2 = reinterpret_cast<const uint4*>(tab + (base + (int64_t)c2) * kRareSlots);
  uint4 v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = p1[i];
    v[4 + i] = p2[i];
  }
  uint32_t bits = 0u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    bits = v[i].x == (uint32_t)r ? v[i].y : bits;
    bits = v[i].z == (uint32_t)r ? v[i].w : bits;
  }
  if (bits || v[3].z == 0xffffffffu || v[7].z == 0xffffffffu) return bits;
  for (uint32_t step = 1; step <= (uint32_t)mask; ++step) {  // both full: the overflow chain
    const uint4* p = reinterpret_cast<const uint4*>(
        tab + (base + (int64_t)((c2 + step) & (uint32_t)mask)) * kRareSlots);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 w = p[i];
      if (w.x == (uint32_t)r) return w.y;
      if (w.z == (uint32_t)r) return w.w;
    }
    if (p[3].z == 0xffffffffu) return 0u;
  }
  return 0u;
}

// ---------------------------------------------------------------------------- per pass

// The tail of the pass_terms block (1024 threads, after its lists are written and a barrier):
// the pass's B slices fB[seg][q][16] (fp16 bits), scale_up, and per query whether the filter
// may answer it (felig). A query is eligible when the pass has at most 512 distinct terms and
// every weight of the query is finite and >= 0. A slot whose list the pass_terms wave holds in
// registers (cap.regs: <= 64 entries, entry j in lane j) is read from there, the others from the
// lists in global memory; one barrier (the pass's largest w * s for the exponent e).
__device__ __forceinline__ void filter_prep_block(int nU, const QTerm* __restrict__ ql,
                                                  const int32_t* __restrict__ qu,
                                                  const PrepCapture& cap, const FilterPrep& fp) {
  uint16_t* __restrict__ fB = fp.fB;
  const float* __restrict__ fs = fp.fs;
  __shared__ double wmax[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = armi::wave_id();
  const bool pass_ok = nU <= kFMaxU;
  const int nSeg = filter_segments(nU);
  if (pass_ok) {
    uint4* b4 = reinterpret_cast<uint4*>(fB);
    for (int i = tid; i < nSeg * kFBSlice / 8; i += 1024) b4[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  double mx = 0.0;
  bool ok[kQW];
#pragma unroll
  for (int i = 0; i < kQW; ++i) {
    const int slot = wave * kQW + i;
    const int q = cap.q[i];
    const int n = q >= 0 ? cap.n[i] : 0;
    bool bad = false;
    double m = 0.0;
    if (cap.regs[i]) {  // uniform
      if (lane < n) {
        bad = !(cap.w[i] >= 0.f) || !isfinite(cap.w[i]);  // NaN fails w >= 0
        m = (double)cap.w[i] * (double)cap.s[i];
      }
    } else {
      for (int j = lane; j < n; j += 64) {
        const float w = ql[slot * kQStride + j].w;
        const float sc = fs[slot * kQStride + j];
        bad |= !(w >= 0.f) || !isfinite(w);
        m = fmax(m, (double)w * (double)sc);
      }
    }
    ok[i] = pass_ok && q >= 0 && __ballot(bad) == 0ull;
    if (ok[i]) mx = fmax(mx, m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if (lane == 0) wmax[wave] = mx;
  __syncthreads();
  double m = 0.0;
  for (int w = 0; w < 16; ++w) m = fmax(m, wmax[w]);
  int x = 0;
  if (m > 0.0) (void)frexp(m, &x);  // m < 2^x
  int e = 14 - x;                   // every B < 2^14
  e = e < -100 ? -100 : (e > 110 ? 110 : e);
  if (tid == 0) {
    const double d = ldexp(1.0 + (double)(nU + 600) * 0x1p-22, -e);
    float f = (float)d;
    if ((double)f < d) f = __uint_as_float(__float_as_uint(f) + 1u);
    *fp.fscale = f;
  }
#pragma unroll
  for (int i = 0; i < kQW; ++i) {
    const int slot = wave * kQW + i;
    const int q = cap.q[i];
    if (q < 0) continue;  // wave-uniform
    if (lane == 0) fp.felig[q] = ok[i] ? 1 : 0;
    if (!ok[i]) continue;
    const int n = cap.n[i];
    if (cap.regs[i]) {
      if (lane < n)
        fB[(size_t)(cap.u[i] / kFK) * kFBSlice + q * kFK + (cap.u[i] % kFK)] =
            ru_half(ldexp((double)cap.w[i] * (double)cap.s[i], e));
    } else {
      for (int j = lane; j < n; j += 64) {
        const int u = qu[slot * kQStride + j];
        const float w = ql[slot * kQStride + j].w;
        const float sc = fs[slot * kQStride + j];
        fB[(size_t)(u / kFK) * kFBSlice + q * kFK + (u % kFK)] = ru_half(ldexp((double)w * (double)sc, e));
      }
    }
  }
}

// The filter scan: one 512-thread workgroup per row range (the exact scan's ranges), steps =
// (1024-row tile, 16 terms). Wave w stages terms 16 seg + 2 w + j (j = 0, 1) of every step:
// its held terms' cursors sit in lane 2 seg + j of creg (x: posting cursor, or -(d + 1) for
// dense column d, or kFNone; y: row of the cursor's posting) and their scales in sreg. The
// MFMAs: wave w owns row blocks 4 w .. 4 w + 3 (32 rows each) x both 32-query halves.
__global__ __launch_bounds__(kFThreads) void sparse_filter_scan_kernel(
    const int32_t* __restrict__ term_ptr, const int2* __restrict__ post,
    const int32_t* __restrict__ long_of, const int32_t* __restrict__ start_tab, int64_t n_rows,
    int64_t range_rows, int n_ranges, const uint64_t* __restrict__ row_mask,
    const int32_t* __restrict__ uterm, const int32_t* __restrict__ n_terms,
    const int32_t* __restrict__ col8_of, const uint8_t* __restrict__ dense_u8, int64_t stride8,
    const float* __restrict__ term_scale, const uint16_t* __restrict__ fB,
    const float* __restrict__ fscale, float* __restrict__ cand_key,
    int32_t* __restrict__ cand_row, float* __restrict__ cand_bound) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  const int g = blockIdx.x;
  const int wave = armi::wave_id();
  const int lane = threadIdx.x & 63;
  const int nU = *n_terms;
  if (nU == 0 || nU > kFMaxU) return;  // workgroup-uniform: the merge / exact scan answer
  const int nSeg = filter_segments(nU);
  const int64_t lo = (int64_t)g * range_rows;
  const int64_t hi = min(lo + range_rows, n_rows);
  const int n_tiles = hi > lo ? (int)((hi - lo + kFT - 1) / kFT) : 0;
  const int S = n_tiles * nSeg;
  const float scale = *fscale;
  // the pass's B slices, all of them for the whole scan: [seg][q][16] fp16, the two 16-B halves
  // of query q's row swapped when q & 8 (conflict-free 16-lane ds_read_b128 groups)
  unsigned char* const bimg = fsm + 2 * kFImgBytes;
  unsigned char* const trash = bimg + (size_t)kFMaxSeg * kFBBytes;  // scatter sink
  for (int i = threadIdx.x; i < nSeg * (kFBBytes / 16); i += kFThreads) {
    const int q = (i >> 1) & (kQB - 1), h = i & 1;
    *reinterpret_cast<uint4*>(bimg + (i >> 1) * 32 + 16 * (h ^ ((q >> 3) & 1))) =
        reinterpret_cast<const uint4*>(fB)[i];
  }

  int2 creg = make_int2(kFNone, 0);
  float sreg = 0.f, ireg = 0.f;
  {
    const int sg = lane >> 1, u = sg * kFK + 2 * wave + (lane & 1);
    if (sg < nSeg && u < nU) {
      const int32_t t = uterm[u];
      const int32_t d = col8_of[t];
      sreg = term_scale[t];
      ireg = sreg > 0.f ? 1.f / sreg : 0.f;
      creg = d >= 0 ? make_int2(-(d + 1), 0)
                    : range_cursor(t, g, lo, n_ranges, term_ptr, long_of, start_tab, post);
    }
  }
  const int rev2 = 2 * (63 - lane);
  fp4 ring[kFDepth][2];
  auto tile_hi = [&](int tile) { return (int32_t)min(lo + (int64_t)(tile + 1) * kFT, hi); };
  // step s's loads into ring slot `slot`: every lane issues the same two loads per step (steps
  // past the end and absent terms read a fixed in-bounds address), so the waits the compiler
  // counts stay exact
  auto issue = [&](int s, int slot) {
    const bool live = s < S;
    const int tile = live ? s / nSeg : 0;
    const int seg = live ? s - tile * nSeg : 0;
    const int64_t tlo = lo + (int64_t)tile * kFT;
    const int32_t thi = tile_hi(tile);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = 2 * seg + j;
      const int cx = rl_i(creg.x, c), cy = rl_i(creg.y, c);
      const fp4* src = reinterpret_cast<const fp4*>(post + rev2);
      if (live && cx != kFNone) {
        if (cx < 0)
          src = reinterpret_cast<const fp4*>(dense_u8 + (size_t)(-cx - 1) * stride8 + tlo + 16 * lane);
        else if (cy < thi)
          src = reinterpret_cast<const fp4*>(post + cx + rev2);
      }
      ring[slot][j] = *src;
    }
  };
  // step s from ring slot `slot` into LDS buffer par: the held terms' rows of the image (u8
  // levels as fp16; a posting term's row cleared and its in-tile postings scattered; an absent
  // term's row zero)
  auto finish = [&](int s, int slot, int par) {
    // the slot's loads are waited for here, once, on every path (a use inside the branches
    // below made the compiler's wait counts conservative: a whole step drained per step)
    asm volatile("" ::"v"(ring[slot][0]), "v"(ring[slot][1]));
    if (s >= S) return;  // uniform
    const int tile = s / nSeg, seg = s - tile * nSeg;
    const int32_t tlo = (int32_t)(lo + (int64_t)tile * kFT);
    const int32_t thi = tile_hi(tile);
    unsigned char* img = fsm + par * kFImgBytes;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = 2 * seg + j;
      const int cx = rl_i(creg.x, c), cy = rl_i(creg.y, c);
      unsigned char* rowp = img + (2 * wave + j) * kFImgStride;
      fu32x4* dst = reinterpret_cast<fu32x4*>(rowp + 32 * lane);
      if (cx != kFNone && cx < 0) {
        const fp4 v = ring[slot][j];
        const fu32x2 a = u8x4_f16((uint32_t)v.x), b = u8x4_f16((uint32_t)v.y);
        const fu32x2 cc = u8x4_f16((uint32_t)v.z), dd = u8x4_f16((uint32_t)v.w);
        dst[0] = fu32x4{a.x, a.y, b.x, b.y};
        dst[1] = fu32x4{cc.x, cc.y, dd.x, dd.y};
        continue;
      }
      dst[0] = fu32x4{0u, 0u, 0u, 0u};
      dst[1] = fu32x4{0u, 0u, 0u, 0u};
      if (cx == kFNone || cy >= thi) continue;  // no posting of the term in this tile
      const float sc = rl_f(sreg, c), isc = rl_f(ireg, c);
      fp4 v = ring[slot][j];
      int adv = 0;  // postings consumed before v
      while (true) {  // wave-uniform trip count
        const uint64_t be = __ballot(v.x < thi), bo = __ballot(v.z < thi);
        const int ne = be == ~0ull ? 64 : __builtin_clzll(~be);
        const int no = bo == ~0ull ? 64 : __builtin_clzll(~bo);
        const int n = min(2 * ne, 2 * no + 1);  // postings of v inside the tile
        const _Float16 a0 = (_Float16)u8_level_fast(__int_as_float(v.y), sc, isc);
        const _Float16 a1 = (_Float16)u8_level_fast(__int_as_float(v.w), sc, isc);
        unsigned char* d0 = rev2 < n ? rowp + 2 * (v.x - tlo) : trash + 2 * lane;
        unsigned char* d1 = rev2 + 1 < n ? rowp + 2 * (v.z - tlo) : trash + 2 * lane;
        *reinterpret_cast<_Float16*>(d0) = a0;
        *reinterpret_cast<_Float16*>(d1) = a1;
        if (n < 128) {
          const int nl = 63 - (n >> 1);
          const int32_t re = rl_i(v.x, nl), ro = rl_i(v.z, nl);
          if (lane == c) {
            creg.x = cx + adv + n;
            creg.y = (n & 1) ? ro : re;
          }
          break;
        }
        adv += 128;
        v = load_window_sync(post + cx + adv + rev2);
      }
    }
  };

  ff32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    acc[i][0] = ff32x16{};
    acc[i][1] = ff32x16{};
  }
  // transposed-read addresses of the A operand (T10): lane 4 q + p of each 16-lane group
  // supplies term row kb + q (+ 4 for the second read), data rows rb + 4 p .. + 3
  const int li = lane & 15;
  const int a_off = (8 * (lane >> 5) + (li >> 2)) * kFImgStride + 2 * (16 * ((lane >> 4) & 1) + 4 * (li & 3));
  const int b_off = (lane & 31) * 32 + 16 * ((lane >> 5) ^ ((lane >> 3) & 1));
  auto compute = [&](int par, int seg) {
    const unsigned char* img = fsm + par * kFImgBytes;
    const unsigned char* bb = bimg + seg * kFBBytes;
    const fu32x4 b0 = *reinterpret_cast<const fu32x4*>(bb + b_off);
    const fu32x4 b1 = *reinterpret_cast<const fu32x4*>(bb + 32 * 32 + b_off);
    fhalf8 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const unsigned char* p = img + a_off + 2 * 32 * (4 * wave + i);
      typedef __attribute__((address_space(3))) fs4 lds_fs4;
      const fs4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_fs4*)(p));
      const fs4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_fs4*)(p + 4 * kFImgStride));
      const fu32x2 l2 = __builtin_bit_cast(fu32x2, lo4), h2 = __builtin_bit_cast(fu32x2, hi4);
      a[i] = __builtin_bit_cast(fhalf8, fu32x4{l2.x, l2.y, h2.x, h2.y});
    }
    // a tile's first segment starts its sums from the MFMA's zero operand (no 128 register
    // clears per tile in the epilogue)
    if (seg == 0) {  // uniform
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], __builtin_bit_cast(fhalf8, b0), ff32x16{}, 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], __builtin_bit_cast(fhalf8, b1), ff32x16{}, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], __builtin_bit_cast(fhalf8, b0), acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], __builtin_bit_cast(fhalf8, b1), acc[i][1], 0, 0, 0);
      }
    }
  };

  // per lane and query half: a 3-deep (key, row) list and the best key it dropped
  float ls[2][kFList], disc[2];
  int32_t lr[2][kFList];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    disc[h] = kNegInf;
#pragma unroll
    for (int e = 0; e < kFList; ++e) {
      ls[h][e] = kNegInf;
      lr[h][e] = kEndRow;
    }
  }
  auto insert = [&](int h, float x, int32_t r) {
#pragma unroll
    for (int e = 0; e < kFList; ++e) {
      const bool c = x > ls[h][e];
      const float ts = c ? x : ls[h][e];
      const int32_t tr = c ? r : lr[h][e];
      x = c ? ls[h][e] : x;
      r = c ? lr[h][e] : r;
      ls[h][e] = ts;
      lr[h][e] = tr;
    }
    disc[h] = fmaxf(disc[h], x);
  };
  // The tile's keys into the lane lists; accumulators cleared. Row of register v of block i:
  // 32 (4 w + i) + 8 (v / 4) + 4 (lane / 32) + v % 4 (the 32x32 MFMA output layout).
  // Per lane and query half, a compare-free network keeps the tile's four best raw accumulators
  // (descending), each carrying its code 16 i + v in the low 6 mantissa bits (v_and_or): per
  // score one max and three med3 (on the bit patterns), no row arithmetic and no selects (a 3-deep insertion with row
  // selects cost ~17 VALU per score and was half the kernel's time: 64 M scores per pass). At the
  // tile's end the best three enter the lane list with their rows, the fourth joins the dropped
  // bound. A code lowers a key by < 2^-17 relative, so the keys leaving the tile are scaled by
  // scale * (1 + 2^-16). A row that does not count (past the range, masked out) scores 0, and an
  // entry whose value is 0 apart from its code never enters a list (its score is <= 0: it
  // cannot be certified into a top-k, see the merge's bound).
  const float scale_x = scale * (1.0f + 0x1p-16f);
  auto epilogue = [&](int tile) {
    const int32_t tlo = (int32_t)(lo + (int64_t)tile * kFT);
    const int32_t thi = tile_hi(tile);
    const bool full = thi - tlo == kFT && !row_mask;  // uniform
    // (as their bit patterns: every key is >= +0, so the unsigned order is the float order, and
    // integer max / med3 need no canonicalising copies of bit-built floats)
    uint32_t top[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) top[h][e] = 0u;
    auto net = [&](int h, float xf, uint32_t code) {
      const uint32_t x = (__float_as_uint(xf) & 0xffffffc0u) | code;
      const uint32_t a = top[h][0], b = top[h][1], c = top[h][2], d = top[h][3];
      top[h][0] = max(a, x);
      top[h][1] = max(min(a, b), min(max(a, b), x));  // med3: v_med3_u32
      top[h][2] = max(min(b, c), min(max(b, c), x));
      top[h][3] = max(min(c, d), min(max(c, d), x));
    };
    if (full) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          net(0, acc[i][0][v], 16 * i + v);
          net(1, acc[i][1][v], 16 * i + v);
        }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t rb = tlo + 32 * (4 * wave + i);
        uint32_t mb = 0xffffffffu;
        if (row_mask) {
          const uint64_t w64 = rb < thi ? row_mask[rb >> 6] : 0ull;
          mb = (uint32_t)(w64 >> (rb & 32));
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int off = 8 * (v >> 2) + 4 * (lane >> 5) + (v & 3);
          const bool ok = rb + off < thi && ((mb >> off) & 1u);
          net(0, ok ? acc[i][0][v] : 0.f, 16 * i + v);
          net(1, ok ? acc[i][1][v] : 0.f, 16 * i + v);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const uint32_t bits = top[h][e];
        const uint32_t code = bits & 63u;
        const int32_t r = tlo + 32 * (4 * wave + (int)(code >> 4)) + 8 * (int)((code >> 2) & 3) +
                          4 * (lane >> 5) + (int)(code & 3);
        insert(h, (bits & ~63u) ? __uint_as_float(bits) * scale_x : kNegInf, r);
      }
      const uint32_t b4 = top[h][3];
      disc[h] = fmaxf(disc[h], (b4 & ~63u) ? __uint_as_float(b4) * scale_x : kNegInf);
    }
  };

  unsigned long long tp[6] = {0, 0, 0, 0, 0, 0}, ta = 0, tb = 0;
  (void)tp;
  (void)ta;
  (void)tb;
  ARMI_FP_T(ta);
  // prologue: the first kFDepth - 1 steps in flight, step 0 staged
#pragma unroll
  for (int p = 0; p < kFDepth - 1; ++p) issue(p, p);
  finish(0, 0, 0);
  __syncthreads();
#ifdef ARMI_SPARSE_PROFILE
  ARMI_FP_T(tb);
  tp[5] = tb - ta;
#define ARMI_FP_ADD(i) ARMI_FP_T(tb); tp[i] += tb - ta; ta = tb
#else
#define ARMI_FP_ADD(i) (void)0
#endif
  ARMI_FP_T(ta);
  // step s: issue s + 3 (ring slot (s + 3) % 4), multiply image s % 2, epilogue at a tile's last
  // step, stage s + 1 (slot (s + 1) % 4) into the other image, one barrier
  // (the four steps of a round run whole, past S too: their loads are dummies, their products
  // unused and their stores skipped, so every path issues the same loads in the same order and
  // the compiler's wait counts stay exact)
  for (int s0 = 0; s0 < S; s0 += kFDepth) {
#pragma clang loop unroll(full)
    for (int d = 0; d < kFDepth; ++d) {
      const int s = s0 + d;
      issue(s + kFDepth - 1, (d + kFDepth - 1) % kFDepth);
      // keep the step's loads at the top: the scheduler otherwise sinks them below this step's
      // waits, and only one step stays in flight
      __builtin_amdgcn_sched_barrier(0);
      ARMI_FP_ADD(0);
      const int tile = s / nSeg, seg = s - tile * nSeg;
      compute(d & 1, seg);
      ARMI_FP_ADD(1);
      if (s < S && seg == nSeg - 1) epilogue(tile);  // uniform
      ARMI_FP_ADD(2);
      finish(s + 1, (d + 1) % kFDepth, (d + 1) & 1);
      ARMI_FP_ADD(3);
      __syncthreads();
      ARMI_FP_ADD(4);
    }
  }

#ifdef ARMI_SPARSE_PROFILE
  if (lane == 0) {
    unsigned long long* pr = g_fscan_prof + ((size_t)g * kFWaves + wave) * 8;
    for (int i = 0; i < 6; ++i) pr[i] = tp[i];
    pr[6] = S;
  }
#endif
#undef ARMI_FP_ADD
  // workgroup merge: per query the 48 lane-list entries and 16 dropped bounds through LDS (over
  // the images), then one wave per 8 queries keeps the best 16 and the bound of the rest
  float* mkey = reinterpret_cast<float*>(fsm);                        // [kQB][kFPool]
  int32_t* mrow = reinterpret_cast<int32_t*>(fsm + kQB * kFPool * 4);  // [kQB][kFPool]
  float* mdisc = reinterpret_cast<float*>(fsm + kQB * kFPool * 8);     // [kQB][kFLanes]
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int q = 32 * h + (lane & 31);
    const int base = q * kFPool + 2 * kFList * wave + kFList * (lane >> 5);
#pragma unroll
    for (int e = 0; e < kFList; ++e) {
      mkey[base + e] = ls[h][e];
      mrow[base + e] = lr[h][e];
    }
    mdisc[q * kFLanes + 2 * wave + (lane >> 5)] = disc[h];
  }
  __syncthreads();
  float key[8], bq[8];
  int32_t row[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int q = 8 * wave + n;
    key[n] = lane < kFPool ? mkey[q * kFPool + lane] : kNegInf;
    row[n] = lane < kFPool ? mrow[q * kFPool + lane] : kEndRow;
    bq[n] = lane < kFLanes ? mdisc[q * kFLanes + lane] : kNegInf;
  }
  armi::wave_sort_approx_desc_n<8>(key, row);
#pragma unroll
  for (int n = 0; n < 8; ++n) bq[n] = fmaxf(bq[n], lane == kKW ? key[n] : kNegInf);
  armi::wave_max_all_n<8>(bq);
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const size_t base = (size_t)g * kQB + 8 * wave + n;
    if (lane < kKW) {
      cand_key[base * kKW + lane] = key[n];
      cand_row[base * kKW + lane] = row[n];
    }
    if (lane == 0) cand_bound[base] = bq[n];
  }
}

// Per query of the pass, in up to two rounds. Round 1: the kc best keys of the pool (the entries
// from the kc-th largest list maximum up, ranked by key) are rescored exactly from the caller's
// fp32 columns / postings and ranked (score desc, row asc); certified when the k-th exact score
// exceeds the bound
// of every row left out (the lists' bounds, the pool keys below the threshold, the (kc+1)-th key).
// Round 2 (when round 1 cannot certify): every pool entry whose key reaches round 1's k-th exact
// score, rescored and ranked again: a row outside it has key < that score <= the true k-th, so
// only the lists' bounds and the pool keys below it remain. (Round 2 certifies the queries whose
// scores crowd the top, e.g. two terms present in every row: ~100 rows within the keys' slack of
// the 40th score.) Certified queries are answered and flagged (CERTIFIED | FILTERED) with
// kth = +inf, so the exact scan and its collect pass skip them; the others are left to it.
// Rankings are rank counts (each entry counts the entries better than it, split over 2 or 4
// threads when few: 16-B LDS reads, no barrier per stage) instead of bitonic sorts. The query's
// terms come from the pass_terms block's per-query table (fterm / fw / fnt).
__global__ __launch_bounds__(256) void sparse_filter_merge_kernel(
    const float* __restrict__ cand_key, const int32_t* __restrict__ cand_row,
    const float* __restrict__ cand_bound, int n_wg, int q_first, int k, int kc,
    int64_t ordinal_base, const int32_t* __restrict__ felig, const int4* __restrict__ fterm,
    const float* __restrict__ fw, const int32_t* __restrict__ fnt,
    const uint2* __restrict__ rare_tab,
    const uint32_t* __restrict__ dense_val, int64_t dense_stride, float* __restrict__ out_scores,
    int64_t* __restrict__ out_ids, int32_t* __restrict__ out_count, uint32_t* __restrict__ flags,
    float* __restrict__ kth_out) {
  __shared__ __attribute__((aligned(16))) float skey[kFSel];  // selected: key, then exact score
  __shared__ __attribute__((aligned(16))) int32_t srow[kFSel];
  __shared__ __attribute__((aligned(16))) float tkey[kFSel];  // ranked copies
  __shared__ __attribute__((aligned(16))) int32_t trow[kFSel];
  __shared__ float vals[kFVal];    // (row, query term) values of a rescore chunk
  __shared__ int4 tinfo[kMaxTerms];  // {fp32 column or -1, table base, table mask, term}
  __shared__ float tw[kMaxTerms];
  __shared__ uint32_t umax[256];
  __shared__ float red[8];
  __shared__ float t0s;
  __shared__ int sh[4];  // [0] selected, [2] members, [3] terms without a column
  const int ql = blockIdx.x;
  const int qg = q_first + ql;
  const int tid = threadIdx.x, lane = tid & 63, wave = armi::wave_id();
  unsigned long long ts[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int pn_all = 0, pn_sel = 0;
  (void)ts;
  (void)pn_all;
  (void)pn_sel;
  ARMI_FP_T(ts[0]);
  if (!felig[ql]) return;  // uniform: the exact scan answers
  const int nt = fnt[ql];
#ifdef ARMI_SPARSE_PROFILE
  auto prof_out = [&](int rounds) {
    if (tid == 0) {
      ARMI_FP_T(ts[7]);
      for (int i = 1; i < 8; ++i) g_fmerge_prof[ql * 16 + i] = ts[i] ? ts[i] - ts[0] : 0;
      g_fmerge_prof[ql * 16] = rounds;
      g_fmerge_prof[ql * 16 + 8] = nt;
      g_fmerge_prof[ql * 16 + 9] = sh[3];
      g_fmerge_prof[ql * 16 + 10] = pn_all;
      g_fmerge_prof[ql * 16 + 11] = pn_sel;
      for (int i = 8; i < 11; ++i) g_fmerge_prof[ql * 16 + 4 + i] = ts[i] ? ts[i] - ts[0] : 0;
    }
  };
#else
  auto prof_out = [&](int) {};
#endif
  auto answer = [&](int count) {  // tkey / trow ranked, count valid entries
    if (wave != 0) return;
    for (int c = lane; c < k; c += 64) {
      const size_t o = (size_t)qg * k + c;
      out_scores[o] = c < count ? tkey[c] : kNegInf;
      out_ids[o] = c < count ? ordinal_base + trow[c] : -1;
    }
    if (lane == 0) {
      out_count[qg] = count;
      flags[ql] |= ARMI_FLAG_CERTIFIED | ARMI_FLAG_FILTERED;
      kth_out[ql] = std::numeric_limits<float>::infinity();
    }
  };
  if (nt == 0) {  // no terms: no row shares an index (every pool key is a stand-in)
    answer(0);
    return;
  }
  // the pool (16 sorted entries per range list), its list bounds and maxima
  const int pool = n_wg * kKW;
  float kk[kSmPer];
  int32_t rw[kSmPer];
#pragma unroll
  for (int j = 0; j < kSmPer; ++j) {
    const int e = tid + 256 * j;
    const size_t src = ((size_t)(e / kKW) * kQB + ql) * kKW + (e % kKW);
    kk[j] = e < pool ? cand_key[src] : kNegInf;
    rw[j] = e < pool ? cand_row[src] : 0;
  }
  float b = tid < n_wg ? cand_bound[(size_t)tid * kQB + ql] : kNegInf;
#pragma unroll
  for (int j = 0; j < kSmPer; ++j) {
    const int e = tid + 256 * j;
    if (e < pool && e % kKW == 0) umax[e / kKW] = ord_key_f(kk[j]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b = fmaxf(b, armi::xor_stride(b, off));
  if (lane == 0) red[wave] = b;
  if (tid == 0) sh[3] = 0;
  __syncthreads();
  for (int j = tid; j < nt; j += 256) {
    const int4 ti = fterm[ql * kMaxTerms + j];
    tinfo[j] = ti;
    tw[j] = fw[ql * kMaxTerms + j];
    if (ti.x < 0) atomicAdd(&sh[3], 1);
  }
  __syncthreads();
  const bool rare = sh[3] > 0;  // terms without an fp32 column: values from their postings
  ARMI_FP_T(ts[1]);
  const float list_bound = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  if (wave == 0) {  // t0 = kc-th largest list maximum (one-wave radix select)
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gg = lane + 64 * i;
      u[i] = gg < n_wg ? umax[gg] : ord_key_f(kNegInf);
    }
    float t0 = kNegInf;
    if (n_wg >= kc) {
      uint32_t prefix = 0;
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = prefix | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) cnt += __popcll(__ballot(u[i] >= cand));
        if (cnt >= kc) prefix = cand;
      }
      t0 = from_ord_key_f(prefix);
    }
    if (lane == 0) t0s = t0;
    ARMI_FP_T(ts[8]);
  }
  // rank of each of n entries of (key, row) by (key desc, row asc): tpe threads per entry each
  // count a slice of the others (16-B LDS reads), summed across the tpe lanes; emit(i, rank)
  auto rank_all = [&](const float* key, const int32_t* row, int n, auto&& emit) {
    const int lt = n <= 64 ? 2 : (n <= 128 ? 1 : 0);  // log2 tpe
    const int tpe = 1 << lt;
    const int per = (((n + tpe - 1) >> lt) + 3) & ~3;
    for (int f0 = 0; f0 < (n << lt); f0 += 256) {
      const int f = f0 + tid;
      const int i = f >> lt, part = f & (tpe - 1);
      int r = 0;
      if (i < n) {
        const float ki = key[i];
        const int32_t ri = row[i];
        const int j1 = min(n, (part + 1) * per);
        for (int j = part * per; j < j1; j += 4) {
          const float4 k4 = *reinterpret_cast<const float4*>(key + j);
          const int4 r4 = *reinterpret_cast<const int4*>(row + j);
          r += armi::approx_better(k4.x, r4.x, ki, ri) ? 1 : 0;
          r += ((j + 1 < j1) && armi::approx_better(k4.y, r4.y, ki, ri)) ? 1 : 0;
          r += ((j + 2 < j1) && armi::approx_better(k4.z, r4.z, ki, ri)) ? 1 : 0;
          r += ((j + 3 < j1) && armi::approx_better(k4.w, r4.w, ki, ri)) ? 1 : 0;
        }
      }
      if (lt >= 1) r += __shfl_xor(r, 1);
      if (lt >= 2) r += __shfl_xor(r, 2);
      if (i < n && part == 0) emit(i, r);
    }
  };
  float thr = kNegInf;
  for (int round = 0; round < 2; ++round) {
    __syncthreads();  // (t0s written; the previous round is done with the arrays)
    if (tid == 0) {
      sh[0] = 0;
      sh[2] = 0;
    }
    if (round == 0) thr = t0s;
    __syncthreads();
    // the pool entries >= thr into skey / srow: per-thread counts, a wave prefix sum and one LDS
    // atomic per wave (no per-entry atomic round trips); the others' maximum joins the bound
    float dmax = kNegInf;
    int c = 0;
#pragma unroll
    for (int j = 0; j < kSmPer; ++j) {
      const bool sel = kk[j] != kNegInf && kk[j] >= thr;
      c += sel ? 1 : 0;
      dmax = fmaxf(dmax, sel ? kNegInf : kk[j]);
    }
    int incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d);
      if (lane >= d) incl += y;
    }
    int wbase = 0;
    if (lane == 63 && incl > 0) wbase = atomicAdd(&sh[0], incl);
    int pos = __shfl(wbase, 63) + incl - c;
    if (c > 0) {
#pragma unroll
      for (int j = 0; j < kSmPer; ++j) {
        if (kk[j] != kNegInf && kk[j] >= thr) {
          if (pos < kFSel) {
            skey[pos] = kk[j];
            srow[pos] = rw[j];
          }
          ++pos;
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dmax = fmaxf(dmax, armi::xor_stride(dmax, off));
    if (lane == 0) red[4 + wave] = dmax;
    __syncthreads();
    if (round == 0) ARMI_FP_T(ts[9]);
    const int n_all = sh[0];
    if (n_all > kFSel) return;  // uniform: too many ties for the rescore, the exact scan answers
    float bound = fmaxf(list_bound, fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7])));
    int n_sel = n_all;
    if (round == 0 && n_all > kc) {
      // the kc best keys only; the (kc+1)-th joins the bound of the rows left out
      rank_all(skey, srow, n_all, [&](int i, int r) {
        if (r <= kc) {
          tkey[r] = skey[i];
          trow[r] = srow[i];
        }
      });
      __syncthreads();
      bound = fmaxf(bound, tkey[kc]);
      for (int i = tid; i < kc; i += 256) {
        skey[i] = tkey[i];
        srow[i] = trow[i];
      }
      n_sel = kc;
      __syncthreads();
      if (round == 0) ARMI_FP_T(ts[10]);
    }
    ARMI_FP_T(ts[2]);
    pn_all = n_all;
    pn_sel = n_sel;
    // exact scores of the selected rows, in chunks of rows whose (row, term) slots fit vals
    const int chunk = max(1, min(kFSel, kFVal / nt));
    for (int c0 = 0; c0 < n_sel; c0 += chunk) {
      const int nr = min(chunk, n_sel - c0);
      // a term in >= 1/8 of the rows: its value from the exact scan's fp32 column (value bits,
      // 0 = no posting), one independent load per (row, term) (rows of a few 4-MB columns:
      // reading the same values from the rows' CSR entries took ~29 us of the merge's 47);
      // sentinel (NaN bits) = no value yet
      for (int f = tid; f < nr * nt; f += 256) {
        const int i = f / nt, j = f - i * nt;
        const int32_t d = tinfo[j].x;
        uint32_t bits = 0u;
        if (d >= 0) bits = dense_val[(size_t)d * dense_stride + srow[c0 + i]];
        vals[f] = __uint_as_float(bits ? bits : 0xffffffffu);
      }
      if (rare) {  // uniform: a term without a column (df < rows / 8)
        // its value for each selected row from the term's rare-value table (two independent
        // 64-B bucket loads), one (row, term) pair per thread
        __syncthreads();  // (the column loads' vals writes before these)
        ARMI_FP_T(ts[6]);
        for (int f = tid; f < nr * nt; f += 256) {
          const int i = f / nt, j = f - i * nt;
          const int4 ti = tinfo[j];
          if (ti.x >= 0 || ti.y < 0) continue;  // a column, or no posting at all
          const uint32_t bits = rare_value(rare_tab, ti.y, ti.z, (uint32_t)ti.w, srow[c0 + i]);
          if (bits) vals[f] = __uint_as_float(bits);
        }
      }
      __syncthreads();
      for (int i = tid; i < nr; i += 256) {
        float sc = 0.f;
        bool hit = false;
        for (int p = 0; p < nt; ++p) {
          const float v = vals[i * nt + p];
          if (__float_as_uint(v) != 0xffffffffu) {
            sc = __fadd_rn(sc, __fmul_rn(tw[p], v));  // the reference's order and rounding
            hit = true;
          }
        }
        skey[c0 + i] = hit ? sc : kNegInf;
      }
      __syncthreads();
    }
    ARMI_FP_T(ts[3]);
    // rank the exact scores (score desc, row asc); the best k go to tkey / trow
    int mem = 0;
    for (int i = tid; i < n_sel; i += 256) mem += skey[i] != kNegInf;
    if (mem) atomicAdd(&sh[2], mem);
    rank_all(skey, srow, n_sel, [&](int i, int r) {
      if (r < k) {
        tkey[r] = skey[i];
        trow[r] = srow[i];
      }
    });
    __syncthreads();
    const int members = sh[2];
    const bool certified = members >= k ? tkey[k - 1] > bound : bound == kNegInf;
    ARMI_FP_T(ts[4 + round]);
    if (certified) {
      answer(min(members, k));
      prof_out(round + 1);
      return;
    }
    if (members < k) {  // uniform: no k-th score to widen the rescore with
      prof_out(-1);
      return;
    }
    thr = tkey[k - 1];  // round 2: every pool row whose key reaches it
  }
}
