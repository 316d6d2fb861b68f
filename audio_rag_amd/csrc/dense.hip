// Dense cosine top-k over a fp16 chunk store (gfx950).
//
// Restates Qdrant's COSINE search as called by QdrantRetriever.search
// (src/audio_rag/retrieval/qdrant.py:284-288 dense prefetch of hybrid search, 316-332 dense
// query) over vectors produced by BGEM3Embedder (src/audio_rag/embeddings/bge.py:104-157,
// fp16 on GPU: bge.py:54). Ranking is the exact cosine of the fp16 inputs; ties are broken by
// ascending chunk ordinal.
//
// Pipeline per call (all on one stream, no host synchronisation):
//   1. dense_scan: one 512-thread workgroup per CU streams a contiguous range of 32-row tiles
//      straight from HBM into VGPRs (each corpus byte is read once and used by exactly one
//      wave), multiplies it against up to 64 queries held in LDS with
//      v_mfma_f32_32x32x16_f16 (fp32 accumulate), scales by the fp32 inverse norm and keeps a
//      4-deep top list per lane and query in registers. The 16 lane lists of a query are merged
//      in LDS by a wave bitonic sort into 16 candidates per workgroup, plus the largest score
//      any list discarded ("bound").
//   2. dense_merge: one workgroup per query pools all workgroup candidates, keeps the KC best
//      approximate scores, rescores them EXACTLY (int64 dot of the 2^24 fixed-point images),
//      sorts by (exact key desc, ordinal asc) and certifies the answer: every discarded row has
//      approximate score <= bound and |approx - exact| <= delta, so when the k-th exact key
//      exceeds bound + delta no discarded row can belong to the top-k.
//   3. dense_exact_scan + merge_lists: for queries that could not be certified, an exhaustive
//      exact scan (workgroups of certified queries exit immediately).
#include <cmath>
#include <cstdlib>
#include <limits>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "armi_index.h"

namespace {

using armi::TILE_ROWS;

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kQB = 64;       // queries per scan pass (LDS holds their fragment image)
constexpr int kLaneList = 4;  // top entries kept per lane and query
constexpr int kKW = 16;       // candidates per workgroup and query
constexpr int kDepth = 4;     // 64-byte groups in flight per lane
constexpr float kNegInf = -std::numeric_limits<float>::infinity();
constexpr double kNegInfD = -std::numeric_limits<double>::infinity();
constexpr int64_t kNoOrd = std::numeric_limits<int64_t>::max();
constexpr int kMaxK = 240;
constexpr int kMergeThreads = 256;
constexpr int kDenseMergeThreads = 512;  // dense_merge_kernel: 8 waves share the exact rescore
constexpr int kMaxPool = 4096;  // pooled candidates per query in the merge kernels
// delta = kDeltaSafety * dim * 2^-24 * |q|: the fp32 accumulation error bound gamma_dim * |q|
// (|sum| <= sum |q_i x_i| <= |q||x|) with a 4x allowance for the MFMA's internal ordering.
constexpr double kDeltaSafety = 4.0;
// The four-wave scan's approximate scores carry a row code in their 6 low mantissa bits: up to
// 2^-18 |score| more (scores are at most |q| (1 + 2^-10) in the certificate's units); 2^-17 |q|.
constexpr double kEncodeSlack = 1.0 / 131072.0;

template <int M>
__device__ __forceinline__ void topm_insert(float x, int32_t id, float (&s)[M], int32_t (&ix)[M],
                                            float& disc) {
#pragma unroll
  for (int j = 0; j < M; ++j) {
    const bool c = x > s[j];
    const float ts = c ? x : s[j];
    const int32_t ti = c ? id : ix[j];
    x = c ? s[j] : x;
    id = c ? ix[j] : id;
    s[j] = ts;
    ix[j] = ti;
  }
  disc = fmaxf(disc, x);
}

// The same MFMA with the accumulator pinned to AGPRs (inline asm: hipcc otherwise keeps it in
// ArchVGPRs when the kernel fits in 256 of them).
__device__ __forceinline__ void mfma16_acc(f32x16& c, u32x4 a, u32x4 b) {
  asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

__device__ __forceinline__ f32x16 mfma16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a),
                                                __builtin_bit_cast(half8, b), c, 0, 0, 0);
}

// Corpus row loads use the default cache policy: measured, non-temporal (nt) register loads of
// this access shape ran the scan at 3.3 TB/s instead of 5.4 TB/s.
__device__ __forceinline__ u32x4 stream_load(const u32x4* p) { return *p; }

// LDS bytes of the scan kernel: the query fragment image, later overlaid by the merge scratch.
template <int DIM>
constexpr int scan_lds_bytes() {
  constexpr int img = (DIM / 16) * 2 * kQB * 16;
  constexpr int scratch = kQB * 64 * 4 * 2 + kQB * 16 * 4;
  return img > scratch ? img : scratch;
}

// dense_scan_i8_kernel's query image (round 6): the 64 fp16 query rows as they are in memory,
// row q at q * (2 DIM + 16) B (the 16-B pad: the MFMA B reads of 16 lanes, queries r .. r + 15 at
// one chunk, fall on 16 distinct 4-bank groups), copied by LDS-DMA (1-KB global_load_lds_dwordx4
// pieces of one row, no register staging); the workgroup merge reuses the region.
template <int DIM>
constexpr int i8_qstride() { return DIM * 2 + 16; }
template <int DIM>
constexpr int i8_img_bytes() {
  constexpr int img = kQB * i8_qstride<DIM>();
  constexpr int scratch = kQB * 64 * 4 * 2 + kQB * 16 * 4;
  return img > scratch ? img : scratch;
}

template <int DIM>
__global__ __launch_bounds__(kThreads) void dense_scan_kernel(
    const uint16_t* __restrict__ rows, const float* __restrict__ inv_norm32,
    const uint64_t* __restrict__ row_mask, int64_t n_rows, int64_t n_tiles, int tiles_per_wg,
    int n_ranges, int n_qb, const uint16_t* __restrict__ queries_all, int q_stride,
    float* __restrict__ cand_key, int32_t* __restrict__ cand_row, float* __restrict__ cand_bound) {
  constexpr int KSTEPS = DIM / 16;
  // workgroup -> (64-query block qb, tile range rp). With several blocks, the blocks of one range
  // get workgroup ids congruent mod 8, i.e. the same XCD: they stream the same rows at about the
  // same time, so one block's HBM read is the others' L2 hit.
  int qb = 0, rp = blockIdx.x;
  if (n_qb > 1) {
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    qb = j % n_qb;
    rp = (j / n_qb) * 8 + xcd;
  }
  if (rp >= n_ranges) return;  // workgroup-uniform, before any barrier
  const int q0 = qb * kQB;
  const int nq = min(kQB, q_stride - q0);
  const uint16_t* __restrict__ queries = queries_all + (size_t)q0 * DIM;
  constexpr int GROUPS = DIM / 64;
  static_assert(GROUPS % kDepth == 0, "prefetch ring must divide the tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  u32x4* qimg = reinterpret_cast<u32x4*>(smem);  // [KSTEPS][2][kQB] 16-byte fragments

  const int wave = armi::wave_id();
  const int lane = threadIdx.x & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t t_begin = (int64_t)rp * tiles_per_wg;
  const int64_t t_end = min(t_begin + (int64_t)tiles_per_wg, n_tiles);
  int64_t t = t_begin + wave;
  auto row_ptr = [&](int64_t tile) -> const u32x4* {
    int64_t rr = tile * TILE_ROWS + r;
    rr = rr < n_rows ? rr : n_rows - 1;
    return reinterpret_cast<const u32x4*>(rows + rr * DIM) + 4 * h;
  };
  // the first tile's loads go out before the query image is staged: the HBM latency of the
  // first groups overlaps the image fill
  const u32x4* cur = row_ptr(t < t_end ? t : t_begin);
  u32x4 buf[kDepth][4];
  if (t < t_end) {
#pragma unroll
    for (int g = 0; g < kDepth; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[g][i] = stream_load(cur + 8 * g + i);
  }

  // 1. Query fragment image. K-step s, lane half h takes the 8 elements of chunk
  //    c = 8*(s/4) + 4*h + s%4, matching the corpus chunk that lane half loads (any k order
  //    is valid for a dot product as long as A and B agree).
  for (int e = threadIdx.x; e < KSTEPS * 2 * kQB; e += kThreads) {
    const int q = e & (kQB - 1);
    const int sh = e >> 6;
    const int h = sh & 1;
    const int s = sh >> 1;
    const int c = 8 * (s >> 2) + 4 * h + (s & 3);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (q < nq) v = *reinterpret_cast<const u32x4*>(queries + (size_t)q * DIM + 8 * c);
    qimg[e] = v;
  }
  __syncthreads();

  float s0[kLaneList], s1[kLaneList];
  int32_t i0[kLaneList], i1[kLaneList];
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    s0[j] = kNegInf; s1[j] = kNegInf; i0[j] = -1; i1[j] = -1;
  }
  float d0 = kNegInf, d1 = kNegInf;

  if (t < t_end) {
    for (; t < t_end; t += kWaves) {
      const int64_t tn = (t + kWaves < t_end) ? t + kWaves : 0;  // (tile 0: shared, L2-hot)
      const u32x4* nxt = row_ptr(tn);
      // The fragment image is loop-invariant; an opaque per-tile offset keeps the compiler from
      // hoisting all 2*KSTEPS fragment reads out of the tile loop (512 VGPRs -> scratch).
      int qoff = h * kQB + r;
      asm volatile("" : "+v"(qoff));
      const u32x4* qv = qimg + qoff;
      f32x16 acc0 = {}, acc1 = {};
      float4 iv4[4];  // inverse norms of the lane's 16 rows, loaded before the next tile's loads
#pragma unroll
      for (int g = 0; g < GROUPS; ++g) {
        u32x4 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = buf[g % kDepth][i];
        if (g == GROUPS - kDepth) {
          // (an epilogue load issued after the prefetch would be waited for with a vmcnt(0)
          // that drains the prefetch at every tile)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            iv4[q] = *reinterpret_cast<const float4*>(inv_norm32 + t * TILE_ROWS + 8 * q + 4 * h);
        }
        if (g + kDepth < GROUPS) {
#pragma unroll
          for (int i = 0; i < 4; ++i) buf[g % kDepth][i] = stream_load(cur + 8 * (g + kDepth) + i);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            buf[g % kDepth][i] = stream_load(nxt + 8 * (g + kDepth - GROUPS) + i);
        }
        // Pin the refill here: without it the scheduler sinks each load next to its first use
        // (kDepth groups later) and every group waits a full HBM round trip.
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int s = 4 * g + i;
          const u32x4 b0 = qv[s * 2 * kQB];
          const u32x4 b1 = qv[s * 2 * kQB + 32];
          acc0 = mfma16(a[i], b0, acc0);
          acc1 = mfma16(a[i], b1, acc1);
        }
      }
      cur = nxt;

      // Epilogue: lane holds rows (j&3) + 8*(j>>2) + 4*h of the tile, queries r and 32 + r.
      const int64_t row0 = t * TILE_ROWS;
      float inv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = iv4[q];
        inv[4 * q + 0] = v.x; inv[4 * q + 1] = v.y; inv[4 * q + 2] = v.z; inv[4 * q + 3] = v.w;
      }
      // Invalid rows carry a NaN inverse norm, filtered rows get one here: a NaN score never
      // enters a lane list (x > s is false) and fmaxf ignores it in the maxima and the bound,
      // i.e. the lists and bounds of a -inf score without per-score tests.
      if (row_mask) {
        const uint32_t mbits = (uint32_t)(row_mask[row0 >> 6] >> (row0 & 63));
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (!((mbits >> ((j & 3) + 8 * (j >> 2) + 4 * h)) & 1u)) inv[j] = __builtin_nanf("");
      }
      float x0[16], x1[16];
      float mx0 = kNegInf, mx1 = kNegInf;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        x0[j] = acc0[j] * inv[j];
        x1[j] = acc1[j] * inv[j];
        mx0 = fmaxf(mx0, x0[j]);
        mx1 = fmaxf(mx1, x1[j]);
      }
      const int32_t rbase = (int32_t)row0 + 4 * h;
      if (__any(mx0 > s0[kLaneList - 1])) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (!__any(x0[j] > s0[kLaneList - 1])) {
            d0 = fmaxf(d0, x0[j]);  // = topm_insert of a value no lane list takes
            continue;
          }
          topm_insert<kLaneList>(x0[j], rbase + (j & 3) + 8 * (j >> 2), s0, i0, d0);
        }
      } else {
        d0 = fmaxf(d0, mx0);
      }
      if (__any(mx1 > s1[kLaneList - 1])) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (!__any(x1[j] > s1[kLaneList - 1])) {
            d1 = fmaxf(d1, x1[j]);  // = topm_insert of a value no lane list takes
            continue;
          }
          topm_insert<kLaneList>(x1[j], rbase + (j & 3) + 8 * (j >> 2), s1, i1, d1);
        }
      } else {
        d1 = fmaxf(d1, mx1);
      }
    }
  }

  // 2. Workgroup merge (the query image is dead: overlay it).
  __syncthreads();
  float* lkey = reinterpret_cast<float*>(smem);                           // [kQB][65]
  int32_t* lrow = reinterpret_cast<int32_t*>(smem + kQB * 65 * 4);        // [kQB][65]
  float* ldisc = reinterpret_cast<float*>(smem + kQB * 65 * 8);           // [kQB][17]
  const int slot = wave * 2 + h;
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    lkey[r * 65 + slot * kLaneList + j] = s0[j];
    lrow[r * 65 + slot * kLaneList + j] = i0[j];
    lkey[(32 + r) * 65 + slot * kLaneList + j] = s1[j];
    lrow[(32 + r) * 65 + slot * kLaneList + j] = i1[j];
  }
  ldisc[r * 17 + slot] = d0;
  ldisc[(32 + r) * 17 + slot] = d1;
  __syncthreads();
  // each wave merges its kQB / kWaves queries together (interleaved shuffle chains)
  constexpr int QW = kQB / kWaves;
  float key[QW], b[QW];
  int32_t row[QW];
#pragma unroll
  for (int qq = 0; qq < QW; ++qq) {
    const int q = wave * QW + qq;
    key[qq] = lkey[q * 65 + lane];
    row[qq] = lrow[q * 65 + lane];
    b[qq] = (lane < 16) ? ldisc[q * 17 + lane] : kNegInf;
  }
  armi::wave_sort_approx_desc_n<QW>(key, row);
#pragma unroll
  for (int qq = 0; qq < QW; ++qq)
    if (lane == kKW) b[qq] = fmaxf(b[qq], key[qq]);
  armi::wave_max_all_n<QW>(b);
#pragma unroll
  for (int qq = 0; qq < QW; ++qq) {
    const int q = wave * QW + qq;
    if (q >= nq) break;
    const size_t base = (size_t)rp * q_stride + q0 + q;
    if (lane < kKW) {
      cand_key[base * kKW + lane] = key[qq];
      cand_row[base * kKW + lane] = row[qq];
    }
    if (lane == 0) cand_bound[base] = b[qq];
  }
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef _Float16 half2v __attribute__((ext_vector_type(2)));

// 4 int8 components (one dword) -> 4 fp16 fragments components (two dwords), exactly: the
// biased byte u = b + 128 becomes the fp16 1024 + u (bits 0x64uu), minus 1152 = b.
__device__ __forceinline__ void i8x4_to_f16(uint32_t d, uint32_t& lo, uint32_t& hi) {
  const uint32_t u = d ^ 0x80808080u;
  const half2v bias = {(_Float16)1152.0f, (_Float16)1152.0f};
  const half2v l = __builtin_bit_cast(half2v, __builtin_amdgcn_perm(0x64646464u, u, 0x04010400u));
  const half2v h = __builtin_bit_cast(half2v, __builtin_amdgcn_perm(0x64646464u, u, 0x04030402u));
  lo = __builtin_bit_cast(uint32_t, l - bias);
  hi = __builtin_bit_cast(uint32_t, h - bias);
}

// NT: nontemporal loads (images larger than the Infinity Cache, use_nt_stream)
template <bool NT>
__device__ __forceinline__ u32x4 i8_load(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// Int8-filter form of dense_scan_kernel: the default 64-query scan (round 2). Each row's first
// pass reads its 1-byte int8 image (rows8, one 1 KB row at dim 1024) instead of its 2-byte fp16
// components: half the HBM bytes of the HBM-bound pass. Lane half h loads 16-B chunks 8g+4h+i of
// its row (16 int8 each), converts them exactly to fp16 (i8x4_to_f16) and runs the same
// v_mfma_f32_32x32x16_f16 against the fp16 query image (k-step s, half h = query components
// 128(s>>3) + 64h + 8(s&7) .. +7, the corpus chunk's order). The lane-list key is an UPPER
// BOUND of the fp16 row's cosine: acc * a32[row] + e32[row] * |q| (a32 = s/|x|; e32 bounds the
// quantisation term |q.(x - s x8)|/|x| by Cauchy-Schwarz; |q| rounded up), so the rows
// dense_merge_kernel discards still satisfy exact <= bound + delta (delta: the fp32 accumulation
// term, unchanged) and its certificate holds as for the fp16 scan; it rescoring more of the pool
// (kc_i8) absorbs the looser keys.

// Probe builds only (-DARMI_PROBE_BUILD -DARMI_I8_STAMPS): per (workgroup, wave) s_memrealtime
// (100 MHz, chip-wide) at kernel entry, after the query image, after the tile loop and at the
// end of the workgroup merge, read back by armi_probe_i8_stamps (not part of the ABI).
#if defined(ARMI_PROBE_BUILD) && defined(ARMI_I8_STAMPS)
__device__ uint64_t g_i8_stamps[256 * kWaves * 4];
#define I8_STAMP(slot)                                                                \
  do {                                                                                \
    if (!COLLECT && lane == 0 && blockIdx.x < 256)                                    \
      g_i8_stamps[(blockIdx.x * kWaves + wave) * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define I8_STAMP(slot) do {} while (0)
#endif

// COLLECT: the second pass for the queries the merge could not certify (replaces the per-query
// exhaustive exact scan of round 2). The call's uncertified queries, in query order, are dealt
// 64 per block; each gets its merge-computed threshold thr[q] = (k-th exact key found) - delta,
// rounded down. Every row whose key (the same upper bound as the scan's, exact <= key + delta)
// reaches it is appended to the query's list: a row of the true top-k has exact >= k-th found,
// hence key >= thr, so the list holds the whole top-k whatever the corpus looks like (runs of
// near-duplicates, one-ulp neighbours, exact duplicates). dense_collect_merge_kernel rescores it.
template <int DIM, bool COLLECT, bool NT>
__device__ __forceinline__ void scan_i8_body(
    const int bid, const int8_t* __restrict__ rows8, const float* __restrict__ a32, const float* __restrict__ e32,
    const uint64_t* __restrict__ row_mask, int64_t n_rows, int64_t n_tiles, int tiles_per_wg,
    int n_ranges, int n_qb, const uint16_t* __restrict__ queries_all, int q_stride,
    float* __restrict__ cand_key, int32_t* __restrict__ cand_row, float* __restrict__ cand_bound,
    const int32_t* __restrict__ tile_ord, const uint32_t* __restrict__ flags,
    const float* __restrict__ thr, int32_t* __restrict__ col_cnt, int32_t* __restrict__ col_list,
    int col_cap){
  constexpr int KSTEPS = DIM / 16;  // MFMA k-steps
  constexpr int GROUPS = DIM / 128;  // 128-B groups of a row: 4 chunks per lane half
  constexpr int DEPTH = GROUPS % 4 == 0 ? 4 : 2;  // groups in flight per lane
  int qb = 0, rp = bid;
  if (n_qb > 1) {
    const int xcd = bid & 7, j = bid >> 3;
    qb = j % n_qb;
    rp = (j / n_qb) * 8 + xcd;
  }
  if (rp >= n_ranges) return;  // workgroup-uniform, before any barrier
  const int q0 = qb * kQB;
  int nq = min(kQB, q_stride - q0);
  const uint16_t* __restrict__ queries = queries_all + (size_t)q0 * DIM;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int QS = i8_qstride<DIM>();  // query row stride of the image (B)
  float* qnorm = reinterpret_cast<float*>(smem + (size_t)i8_img_bytes<DIM>());  // [kQB] |q| up
  float* qscale = qnorm + kQB;  // (unused slot, keeps the layout of scan_i8_lds_bytes)
  // (qscale + kQB: [8][kQB] unused slots, keep the layout of scan_i8_lds_bytes)
  int32_t* qsel = reinterpret_cast<int32_t*>(qscale + kQB + kQB * (kThreads / kQB));  // [kQB] COLLECT
  float* qthr = reinterpret_cast<float*>(qsel + kQB);                        // [kQB] COLLECT
  int32_t* wcnt = reinterpret_cast<int32_t*>(qthr + kQB);                    // [kWaves]

  const int wave = armi::wave_id();
  const int lane = threadIdx.x & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  I8_STAMP(0);
  // first pass, static split: the workgroup's waves take its tiles from an LDS counter (each
  // wave's first tile is t_begin + wave; the counter hands out the rest in order). Round-3 stamps
  // (profiles/r03i_i8_stamps_*): with a fixed tile-per-wave split the 8 waves of a workgroup
  // ended their loops ~32 us apart on average at 1M rows (wave speed differs by ~15 % inside a
  // CU), and the workgroup merge waits for the last of them. An LDS atomic returns in ~100 cycles
  // through lgkmcnt, so unlike a device-scope dequeue it never drains the vmcnt prefetch queue.
  int32_t* const wtile = wcnt;  // wcnt[0]: next tile offset of the workgroup (non-COLLECT)
  if constexpr (!COLLECT) {
    if (threadIdx.x == 0) wtile[0] = kWaves;  // published by the image phase's barriers
  }
  if constexpr (COLLECT) {
    // this block's slice [q0, q0 + 64) of the ordered list of uncertified queries
    for (int e = threadIdx.x; e < kQB; e += kThreads) {
      qsel[e] = 0;
      qthr[e] = __builtin_inff();
    }
    int base = 0;
    for (int c0 = 0; c0 < q_stride; c0 += kThreads) {
      const int q = c0 + (int)threadIdx.x;
      const bool u = q < q_stride && !(flags[q] & ARMI_FLAG_CERTIFIED);
      const uint64_t bal = __ballot(u);
      if (lane == 0) wcnt[wave] = __popcll(bal);
      __syncthreads();
      int pre = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const int c = wcnt[w];
        pre += w < wave ? c : 0;
        tot += c;
      }
      const int p = base + pre + __popcll(bal & ((1ull << lane) - 1ull));
      if (u && p >= q0 && p < q0 + kQB) {
        qsel[p - q0] = q;
        qthr[p - q0] = thr[q];
      }
      base += tot;
      __syncthreads();
    }
    nq = min(kQB, base - q0);
    if (nq <= 0) return;  // workgroup-uniform
  }
  auto qrow = [&](int q) -> const uint16_t* {
    if constexpr (COLLECT) return queries_all + (size_t)qsel[q] * DIM;
    return queries + (size_t)q * DIM;
  };
  // Tile schedule: workgroup rp owns tiles [rp * tiles_per_wg, ...); wave w starts on tile
  // t_begin + w, then takes the next tile of the range from the workgroup's LDS counter (first
  // pass) or every kWaves-th (collect pass). Measured and not adopted: a dynamic cross-workgroup
  // dequeue (round 3: profiles/r03d_*, r03e_*; round 4 tail form: r04ah_dense_tail_ab.txt) and
  // fewer tiles for the odd XCDs, whose waves stream ~5 % slower (r04aj / r04ak: +1.3 % without
  // the nontemporal stream, none with it).
  const int64_t t_begin = (int64_t)rp * tiles_per_wg;
  const int64_t t_end = min(t_begin + (int64_t)tiles_per_wg, n_tiles);
  int64_t t = t_begin + wave < t_end ? t_begin + wave : -1;
  // tile-blocked int8 image (armi_index.h): chunk c of the tile's row r at c * 512 + r * 16, so
  // chunk c of the lane's row is cur[32 c]; the padded tail tile is allocated (zero rows, NaN a32)
  auto row_ptr = [&](int64_t tile) -> const u32x4* {
    return reinterpret_cast<const u32x4*>(rows8 + tile * TILE_ROWS * DIM) + r + 4 * h * 32;
  };
  const u32x4* cur = row_ptr(t >= 0 ? t : 0);
  u32x4 buf[DEPTH][4];
  // the first tile's first DEPTH groups. The fp16 query image issues its own (L2-resident) loads
  // first: vmcnt counts in issue order, so an image behind this 16-load HBM burst would wait for
  // all of it before writing LDS (round 3: the image phase took ~11 us of every launch).
  auto prefetch_first = [&]() {
    if (t >= 0) {
#pragma unroll
      for (int g = 0; g < DEPTH; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) buf[g][i] = i8_load<NT>(cur + 32 * (8 * g + i));
    }
  };

  // 1. The query image by LDS-DMA: wave w copies queries 8w .. 8w + 7, each row as 1-KB pieces
  //    (lane l: bytes 16 l of the piece; a short last piece masks its lanes off), all in flight
  //    with the first tile's row loads issued behind them. Rows past the call's queries stay
  //    unwritten (their MFMA columns are never read). Then |q| rounded up (fp32 sum of DIM squares,
  //    relative error < 2^-13) from the image: lane l sums chunks (l >> 3) + 8 i of query
  //    8w + (l & 7). (Round 4-5: register-staged copy into a chunk-major image, 7.5-8.2 us of
  //    every launch; profiles/r06_i8_image_dma_ab.txt.)
  {
    constexpr int PIECES = (DIM * 2 + 1023) / 1024;  // 1-KB pieces per query row
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
      const int q = 8 * wave + qq;
      if (q < nq) {  // wave-uniform
        const unsigned char* src = reinterpret_cast<const unsigned char*>(qrow(q));
#pragma unroll
        for (int pc = 0; pc < PIECES; ++pc) {
          constexpr int kTail = (DIM * 2) % 1024;
          if (kTail == 0 || pc < PIECES - 1 || lane * 16 < kTail)
            __builtin_amdgcn_global_load_lds(src + pc * 1024 + lane * 16,
                                             (lds_ptr_t)(smem + q * QS + pc * 1024), 16, 0, 0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    prefetch_first();
    __builtin_amdgcn_sched_barrier(0);
    // this wave's pieces are in LDS (it reads only its own rows below; the barrier after this
    // block publishes them to the other waves)
    if (t >= 0)  // (wave-uniform: the row loads behind the pieces were issued)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH * 4) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    constexpr int CH = DIM / 8;  // 16-B chunks per row
    const int q = 8 * wave + (lane & 7);
    float ss = 0.0f;
#pragma unroll
    for (int i = 0; i < CH / 8; ++i) {
      const int j = 8 * i + (lane >> 3);
      const u32x4 v = *reinterpret_cast<const u32x4*>(smem + q * QS + j * 16);
      const half8 hv = __builtin_bit_cast(half8, v);
#pragma unroll
      for (int c = 0; c < 8; ++c) ss += (float)hv[c] * (float)hv[c];
    }
    ss += armi::xor_stride(ss, 8);
    ss += armi::xor_stride(ss, 16);
    ss += armi::xor_stride(ss, 32);
    if (lane < 8) qnorm[q] = sqrtf(ss) * (1.0f + 1.0f / 4096.0f);
  }
  __syncthreads();
  I8_STAMP(1);
  const float qn0 = qnorm[r], qn1 = qnorm[32 + r];
  float th0 = __builtin_inff(), th1 = __builtin_inff();
  int qi0 = 0, qi1 = 0;
  if constexpr (COLLECT) {
    th0 = qthr[r];
    th1 = qthr[32 + r];
    qi0 = qsel[r];
    qi1 = qsel[32 + r];
  }

  float s0[kLaneList], s1[kLaneList];
  int32_t i0[kLaneList], i1[kLaneList];
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    s0[j] = kNegInf; s1[j] = kNegInf; i0[j] = -1; i1[j] = -1;
  }
  float d0 = kNegInf, d1 = kNegInf;

  if (t >= 0) {
    int64_t tn = -1;
    for (; t >= 0; t = tn) {
      // first pass: the next tile of the workgroup's range from the LDS counter (one lane's
      // ds_add_rtn in asm, waited for at group GROUPS - DEPTH: the compiler's form waits
      // lgkmcnt(0) at once, i.e. also for the tile's scalar loads)
      int wgot = 0;
      if constexpr (!COLLECT) {
        const uint32_t a = (uint32_t)(uintptr_t)(lds_ptr_t)wtile;
        uint64_t saved;
        asm volatile(
            "s_mov_b64 %1, exec\n\ts_mov_b64 exec, 1\n\t"
            "ds_add_rtn_u32 %0, %2, %3\n\ts_mov_b64 exec, %1"
            : "=&v"(wgot), "=&s"(saved)
            : "v"(a), "v"(1)
            : "memory");
      }
      const u32x4* nxt = cur;
      bool has_next = false;
      float4 sv[4], ev[4];  // a32 / e32 of the lane's 16 rows (loaded mid-tile)
      const int32_t tord = tile_ord[t];  // ordinal of the tile's image row 0 (wave-uniform)
      // the lane's two query rows in the image (queries r and 32 + r, chunk half h)
      int qoff = r * QS + h * 128;
      asm volatile("" : "+v"(qoff));
      const unsigned char* qb0 = smem + qoff;
      const unsigned char* qb1 = qb0 + 32 * QS;
      // k-step s: chunk 16 (s >> 3) + 8 h + (s & 7) of the row (the corpus chunks' order)
      auto qfrag = [&](const unsigned char* b, int s) {
        return *reinterpret_cast<const u32x4*>(b + (s >> 3) * 256 + (s & 7) * 16);
      };
      f32x16 acc0 = {}, acc1 = {};
#pragma unroll
      for (int g = 0; g < GROUPS; ++g) {
        if (g == GROUPS - DEPTH) {  // the next tile, whose loads start now
          if constexpr (COLLECT) {
            tn = t + kWaves < t_end ? t + kWaves : -1;
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wgot)::"memory");
            const int wnext = __builtin_amdgcn_readfirstlane(wgot);
            tn = t_begin + wnext < t_end ? t_begin + wnext : -1;
          }
          has_next = tn >= 0;
          // (no next tile: the loads go to image tile 0 instead, which every wave's last tile
          // shares, so they hit L2 once it is there; re-reading the wave's own tile cost ~33 MB of
          // HBM / Infinity-Cache fetches per launch, 1.33 x the algorithmic bytes at 100k rows)
          nxt = row_ptr(has_next ? tn : 0);
          // the epilogue's row scales, issued before the next tile's loads: waiting for them
          // then leaves those in flight (issued after the prefetch, their wait was a vmcnt(0)
          // that drained it at every tile)
          const int64_t r0s = t * TILE_ROWS;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            sv[q] = *reinterpret_cast<const float4*>(a32 + r0s + 8 * q + 4 * h);
            ev[q] = *reinterpret_cast<const float4*>(e32 + r0s + 8 * q + 4 * h);
          }
        }
        u32x4 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = buf[g % DEPTH][i];
        if (g + DEPTH < GROUPS) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            buf[g % DEPTH][i] = i8_load<NT>(cur + 32 * (8 * (g + DEPTH) + i));
        } else {  // (no next tile: tile 0, so every path issues the same loads)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            buf[g % DEPTH][i] = i8_load<NT>(nxt + 32 * (8 * (g + DEPTH - GROUPS) + i));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint32_t c[8];  // fp16 pairs of components 0-7 (c[0..3]) and 8-15 (c[4..7])
          i8x4_to_f16(a[i].x, c[0], c[1]);
          i8x4_to_f16(a[i].y, c[2], c[3]);
          i8x4_to_f16(a[i].z, c[4], c[5]);
          i8x4_to_f16(a[i].w, c[6], c[7]);
#if defined(ARMI_PROBE_BUILD) && ARMI_I8_ABL == 1  // timing only: no conversion
          const u32x4 f0 = a[i], f1 = a[i];
          (void)c;
#else
          const u32x4 f0 = {c[0], c[1], c[2], c[3]}, f1 = {c[4], c[5], c[6], c[7]};
#endif
          const int s = 8 * g + 2 * i;
#if defined(ARMI_PROBE_BUILD) && ARMI_I8_ABL == 2  // timing only: no MFMAs
          asm volatile("" :: "v"(f0), "v"(f1), "v"(qfrag(qb0, s)), "v"(qfrag(qb1, s + 1)));
#else
          acc0 = mfma16(f0, qfrag(qb0, s), acc0);
          acc1 = mfma16(f0, qfrag(qb1, s), acc1);
          acc0 = mfma16(f1, qfrag(qb0, s + 1), acc0);
          acc1 = mfma16(f1, qfrag(qb1, s + 1), acc1);
#endif
        }
      }
      cur = nxt;

      // Epilogue: lane holds rows (j&3) + 8*(j>>2) + 4*h of the tile, queries r and 32 + r.
      const int64_t row0 = t * TILE_ROWS;
      float sc[16], ec[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = sv[q], w = ev[q];
        sc[4 * q + 0] = v.x; sc[4 * q + 1] = v.y; sc[4 * q + 2] = v.z; sc[4 * q + 3] = v.w;
        ec[4 * q + 0] = w.x; ec[4 * q + 1] = w.y; ec[4 * q + 2] = w.z; ec[4 * q + 3] = w.w;
      }
      // invalid and filtered rows: NaN scale (never a lane-list entry, ignored by the bound)
      if (row_mask) {
        const uint32_t mbits = (uint32_t)(row_mask[row0 >> 6] >> (row0 & 63));
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (!((mbits >> ((j & 3) + 8 * (j >> 2) + 4 * h)) & 1u)) sc[j] = __builtin_nanf("");
      }
      float x0[16], x1[16];
      float mx0 = kNegInf, mx1 = kNegInf;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        x0[j] = __builtin_fmaf(acc0[j], sc[j], ec[j] * qn0);
        x1[j] = __builtin_fmaf(acc1[j], sc[j], ec[j] * qn1);
        mx0 = fmaxf(mx0, x0[j]);
        mx1 = fmaxf(mx1, x1[j]);
      }
      // image row p of the tile holds ordinal tord + p * T (armi_index.h): lists and the collect
      // lists carry ordinals
      const int32_t T32 = (int32_t)n_tiles;
      const int32_t obase = tord + 4 * h * T32;
      if constexpr (COLLECT) {
        // append every image position whose key reaches the query's threshold (NaN keys of
        // invalid / filtered rows never do)
        if (__any(mx0 >= th0 || mx1 >= th1)) {
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int32_t pos = obase + ((j & 3) + 8 * (j >> 2)) * T32;
            if (x0[j] >= th0) {
              const int s = atomicAdd(col_cnt + qi0, 1);
              if (s < col_cap) col_list[(size_t)qi0 * col_cap + s] = pos;
            }
            if (x1[j] >= th1) {
              const int s = atomicAdd(col_cnt + qi1, 1);
              if (s < col_cap) col_list[(size_t)qi1 * col_cap + s] = pos;
            }
          }
        }
        continue;
      }
      if (__any(mx0 > s0[kLaneList - 1])) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (!__any(x0[j] > s0[kLaneList - 1])) {
            d0 = fmaxf(d0, x0[j]);
            continue;
          }
          topm_insert<kLaneList>(x0[j], obase + ((j & 3) + 8 * (j >> 2)) * T32, s0, i0, d0);
        }
      } else {
        d0 = fmaxf(d0, mx0);
      }
      if (__any(mx1 > s1[kLaneList - 1])) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (!__any(x1[j] > s1[kLaneList - 1])) {
            d1 = fmaxf(d1, x1[j]);
            continue;
          }
          topm_insert<kLaneList>(x1[j], obase + ((j & 3) + 8 * (j >> 2)) * T32, s1, i1, d1);
        }
      } else {
        d1 = fmaxf(d1, mx1);
      }
    }
  }

  I8_STAMP(2);
  if constexpr (COLLECT) return;
  // 2. Workgroup merge (as dense_scan_kernel; the query image is dead: overlay it). Rows of 65
  // dwords: lanes r = 0..31 write query r's row at the same column, so a 64-dword stride put all
  // 32 stores of an instruction in one bank
  constexpr int kLS = 65;
  __syncthreads();
  float* lkey = reinterpret_cast<float*>(smem);                           // [kQB][kLS]
  int32_t* lrow = reinterpret_cast<int32_t*>(smem + kQB * kLS * 4);       // [kQB][kLS]
  float* ldisc = reinterpret_cast<float*>(smem + kQB * kLS * 8);          // [kQB][17]
  const int slot = wave * 2 + h;
#pragma unroll
  for (int j = 0; j < kLaneList; ++j) {
    lkey[r * kLS + slot * kLaneList + j] = s0[j];
    lrow[r * kLS + slot * kLaneList + j] = i0[j];
    lkey[(32 + r) * kLS + slot * kLaneList + j] = s1[j];
    lrow[(32 + r) * kLS + slot * kLaneList + j] = i1[j];
  }
  ldisc[r * 17 + slot] = d0;
  ldisc[(32 + r) * 17 + slot] = d1;
  __syncthreads();
  constexpr int QW = kQB / kWaves;
  float key[QW], b[QW];
  int32_t row[QW];
#pragma unroll
  for (int qq = 0; qq < QW; ++qq) {
    const int q = wave * QW + qq;
    key[qq] = lkey[q * kLS + lane];
    row[qq] = lrow[q * kLS + lane];
    b[qq] = (lane < 16) ? ldisc[q * 17 + lane] : kNegInf;
  }
  armi::wave_sort_approx_desc_n<QW>(key, row);
#pragma unroll
  for (int qq = 0; qq < QW; ++qq)
    if (lane == kKW) b[qq] = fmaxf(b[qq], key[qq]);
  armi::wave_max_all_n<QW>(b);
#pragma unroll
  for (int qq = 0; qq < QW; ++qq) {
    const int q = wave * QW + qq;
    if (q >= nq) break;
    const size_t base = (size_t)rp * q_stride + q0 + q;
    if (lane < kKW) {
      cand_key[base * kKW + lane] = key[qq];
      cand_row[base * kKW + lane] = row[qq];
    }
    if (lane == 0) cand_bound[base] = b[qq];
  }
  I8_STAMP(3);
}

template <int DIM, bool COLLECT, bool NT>
__global__ __launch_bounds__(kThreads) void dense_scan_i8_kernel(
    const int8_t* __restrict__ rows8, const float* __restrict__ a32, const float* __restrict__ e32,
    const uint64_t* __restrict__ row_mask, int64_t n_rows, int64_t n_tiles, int tiles_per_wg,
    int n_ranges, int n_qb, const uint16_t* __restrict__ queries_all, int q_stride,
    float* __restrict__ cand_key, int32_t* __restrict__ cand_row, float* __restrict__ cand_bound,
    const int32_t* __restrict__ tile_ord, const uint32_t* __restrict__ flags,
    const float* __restrict__ thr, int32_t* __restrict__ col_cnt, int32_t* __restrict__ col_list,
    int col_cap, int xcd_step) {
  // xcd_step > 1 (small shards, plan_scan): only workgroups whose id is a multiple of xcd_step
  // work, i.e. those on XCDs 0, xcd_step, ... (workgroup i runs on XCD i mod 8)
  if (blockIdx.x % xcd_step != 0) return;
  scan_i8_body<DIM, COLLECT, NT>(blockIdx.x / xcd_step, rows8, a32, e32, row_mask, n_rows, n_tiles, tiles_per_wg, n_ranges, n_qb,
      queries_all, q_stride, cand_key, cand_row, cand_bound, tile_ord, flags, thr, col_cnt,
      col_list, col_cap);
}


template <int DIM>
constexpr int scan_i8_lds_bytes() {
  return i8_img_bytes<DIM>() + kQB * 8 + kQB * 4 * (kThreads / kQB) + kQB * 8 + kWaves * 4;
}

// Multi-block scan for calls with more than 2 * kQB queries (the all-gathered batch of a sharded
// step: G * 64 queries over a 1/G shard): dense_gemm_scan_w4_kernel below. Corpus rows are read
// from HBM once per 256-query block; the output is the candidate layout dense_merge_kernel reads
// (n_wg = number of row ranges). Round 1-2 forms (register-staged, eight-wave LDS-DMA, phase
// pipelined) and the round-3 16x16x32 form were measured slower and removed in round 4
// (profiles/r02_w4_scan_ab.txt, r02_p8_scan_ab.txt).
constexpr int kGQB = 256;           // queries per block
constexpr int kGRT = 128;           // smallest row range of the plan
constexpr int kG2Rows = 256;  // rows per tile

// Four-wave tiled scan: one wave per SIMD, each wave owning a 128-row x 128-query block of the
// 256 x 256 tile (16 v_mfma_f32_32x32x16_f16 accumulators = 256 AccVGPRs), so a k-step carries
// twice the MFMA work per wave of the eight-wave kernels and half their fragment reads per MFMA
// (4 + 4 ds_read_b128 per 16 MFMAs). Same candidate output as dense_gemm_scan_glds_kernel.
//   * LDS ring of four 32-wide k-step stages (512 image rows x 64 B = 32 KB each: 256 corpus
//     rows, then the 256-query block; chunk c of image row ir at slot c ^ ((ir >> 2) & 3)) plus
//     two 1-KB inverse-norm copies (tile parity), issued by wave 0 with the tile's first stage;
//   * per k-step s: [first half] the 16 MFMAs of sub-step 0 with pieces 0-3 of stage s+3 and the
//     sub-step 1 fragment reads of stage s between them -> vmcnt(12) retires stage s+1 ->
//     s_barrier -> [second half] the 16 MFMAs of sub-step 1 with pieces 4-7 of stage s+3 and the
//     sub-step 0 fragment reads of stage s+1 between them; the tile epilogue after the last k-step;
//   * a wave's 8 pieces per stage are 1-KB LDS-DMA instructions whose per-lane source offsets
//     are fixed (the swizzle of a piece depends on the lane only), so an issue is one
//     instruction over a scalar base.
constexpr int kW4Threads = 256;
constexpr int kW4Img = (kG2Rows + kGQB) * 64;  // one 32-wide k-step stage
constexpr int kW4Norm = 4 * kW4Img;            // the two row-scale copies follow the ring

template <int DIM>
constexpr size_t gemm_w4_lds_bytes() {
  constexpr size_t lists = (size_t)kGQB * 16 * 8 + kGQB * 4 * 4;
  constexpr size_t ring = (size_t)kW4Norm + 4096;
  return ring > lists ? ring : lists;
}

// I8 (round 4): the int8 x int8 form for k <= 64. Rows come from the index's int8 filter image
// (rows8, tile-blocked, scattered row order; n_rows / ranges / row_mask in IMAGE positions) and
// the queries from their per-call int8 quantisation (query_i8_kernel: q ~= s_q q8), both staged
// by the same LDS-DMA pieces: a stage holds 64 components instead of 32 in the same 32 KB, and
// v_mfma_i32_32x32x32_i8 (the fp16 MFMA's cycles at twice the K) takes the same fragment reads,
// so a row tile costs half the k-loop. Each score is an UPPER BOUND of the fp16 row's cosine
// (times |q|, the units of the int8 64-query scan): with D = x8.q8 (exact int32),
//   x.q/|x| <= D s_q a32 + e32 (|q| + eq) + eq,   eq >= ||q - s_q q8||, e32 >= ||x - s_x x8||/|x|
// (x.q = s_x s_q D + s_x x8.(q - s_q q8) + (x - s_x x8).q, Cauchy-Schwarz, s_x |x8| <= |x| +
// ||x - s_x x8||), so dense_merge_kernel's exact rescore and certificate apply as for the int8
// 64-query scan; the candidates' rows are converted to ordinals when the lists are written.
// ABL (probe build only, results wrong): 1 no LDS-DMA pieces in the k-loop, 2 no tile
// epilogue, 4 no MFMAs, 8 no mid-step barrier.
template <int DIM, int ABL, bool I8>
__global__ __launch_bounds__(kW4Threads) __attribute__((amdgpu_waves_per_eu(1, 1)))
void dense_gemm_scan_w4_kernel(
    const uint16_t* __restrict__ rows, const float* __restrict__ inv_norm32,
    const uint64_t* __restrict__ row_mask, int64_t n_rows, int64_t rows_per_range, int n_ranges,
    int n_qb, const uint16_t* __restrict__ queries, int nq, float* __restrict__ cand_key,
    int32_t* __restrict__ cand_row, float* __restrict__ cand_bound,
    const int8_t* __restrict__ rows8, const float* __restrict__ a32, const float* __restrict__ e32,
    const int32_t* __restrict__ tile_ord, const int8_t* __restrict__ q8,
    const float4* __restrict__ qsc) {
  constexpr int KT = I8 ? DIM / 64 : DIM / 32;  // k-steps (stages) per row tile
  typedef typename std::conditional<I8, i32x16, f32x16>::type acc_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int id = blockIdx.x;
  int qb, rp;
  if (n_qb == 2) {
    qb = (id >> 3) & 1;
    rp = (id >> 4) * 8 + (id & 7);
  } else {
    qb = id % n_qb;
    rp = id / n_qb;
  }
  if (rp >= n_ranges) return;  // workgroup-uniform, before any barrier
  const int64_t lo = (int64_t)rp * rows_per_range;
  const int64_t hi = min(lo + rows_per_range, n_rows);
  const int q_base = qb * kGQB;
  const int n_here = (int)(hi - lo);
  const int last_row = (int)(n_rows - 1 - lo);                   // clamp target (row offset)
  const int last4 = (int)(((n_rows + 31) / 32) * 32 - 4 - lo);  // last 16-B group of the norms
  const unsigned char* __restrict__ rsrc =
      I8 ? reinterpret_cast<const unsigned char*>(rows8 + lo * DIM)
         : reinterpret_cast<const unsigned char*>(rows + lo * DIM);
  const unsigned char* __restrict__ qsrc =
      I8 ? reinterpret_cast<const unsigned char*>(q8 + (size_t)q_base * DIM)
         : reinterpret_cast<const unsigned char*>(queries + (size_t)q_base * DIM);
  const float* __restrict__ inv_r = (I8 ? a32 : inv_norm32) + lo;

  const int tid = threadIdx.x;
  const int wave = armi::wave_id();
  const int lane = tid & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int wr = wave >> 1;  // row group: rows wr*128 + m*32 + ...
  const int wq = wave & 1;   // query group: queries wq*128 + n*32 + r

  float sl[4][kLaneList];
  int32_t il[4][kLaneList];
  float dl[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    dl[n] = kNegInf;
#pragma unroll
    for (int j = 0; j < kLaneList; ++j) { sl[n][j] = kNegInf; il[n][j] = -1; }
  }

  const int n_tiles = (n_here + kG2Rows - 1) / kG2Rows;
  // piece p of a stage, this wave: image rows p*64 + prow (p < 4: corpus rows of the tile,
  // p >= 4: queries (p-4)*64 + prow of the block); lane slot lane % 4 holds chunk c. Corpus rows
  // are clamped to the store (the last tile of a range, and the tail stages nobody reads); the
  // byte offsets are 32-bit (the host keeps a range below 4 GiB) over a scalar base.
  const int prow = wave * 16 + (lane >> 2);
  const int c = (lane & 3) ^ ((lane >> 4) & 3);
  const uint32_t c16 = (uint32_t)(c * 16);
  uint32_t b_off[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int q = min(q_base + p * 64 + prow, nq - 1);
    b_off[p] = (uint32_t)((q - q_base) * DIM * (I8 ? 1 : 2)) + c16;
  }
  auto issue_piece = [&](int st, int p) {
    const int tn = st / KT;
    const int t = st - tn * KT;
    lds_ptr_t dst = (lds_ptr_t)(smem + (st & 3) * kW4Img + (p * 4 + wave) * 1024);
    if (p < 4) {
      const uint32_t row = (uint32_t)min(tn * kG2Rows + p * 64 + prow, last_row);
      if constexpr (I8) {
        // tile-blocked image: 16-B chunk cc of the 32-row tile's row rr at cc * 512 + rr * 16;
        // stage t = chunks 4t .. 4t + 3
        __builtin_amdgcn_global_load_lds(
            rsrc + t * 2048 + ((row >> 5) * (uint32_t)(32 * DIM) + (row & 31) * 16 + c * 512), dst,
            16, 0, 0);
      } else {
        __builtin_amdgcn_global_load_lds(rsrc + t * 64 + (row * (uint32_t)(DIM * 2) + c16), dst,
                                         16, 0, 0);
      }
    } else {
      __builtin_amdgcn_global_load_lds(qsrc + t * 64 + b_off[p - 4], dst, 16, 0, 0);
    }
  };
  // row scales of row tile tn -> LDS [kW4Norm + (tn & 1) 2 KB] (wave 0, 4 rows per lane;
  // clamped to the padded arrays, rows past the range are masked anyway): the inverse norms, or
  // for I8 a32 then e32
  auto issue_norms = [&](int tn) {
    if (wave == 0) {
      const int rr = min(tn * kG2Rows + 4 * lane, last4);
      __builtin_amdgcn_global_load_lds(inv_r + rr, (lds_ptr_t)(smem + kW4Norm + (tn & 1) * 2048),
                                       16, 0, 0);
      if constexpr (I8)
        __builtin_amdgcn_global_load_lds(e32 + lo + rr,
                                         (lds_ptr_t)(smem + kW4Norm + (tn & 1) * 2048 + 1024), 16,
                                         0, 0);
    }
  };

  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  const int swz = (r >> 2) & 3;
  const uint32_t a_lane = lds0 + (uint32_t)(wr * 128 + r) * 64;
  const uint32_t b_lane = lds0 + (uint32_t)(kG2Rows + wq * 128 + r) * 64;
  const uint32_t co0 = (uint32_t)(((0 + h) ^ swz) << 4);
  const uint32_t co1 = (uint32_t)(((2 + h) ^ swz) << 4);
  u32x4 fa[2][4], fb[2][4];  // [sub-step][row block m / query block n]
  // fragment item i of sub-step `sub` of stage st: i < 4 row block i, else query block i - 4
  auto read_item = [&](int st, int sub, int i) {
    const uint32_t stage = (uint32_t)((st & 3) * kW4Img) + (sub ? co1 : co0);
    if (i < 4) {
      const uint32_t addr = a_lane + stage;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[sub][i]) : "v"(addr), "i"(i * 2048));
    } else {
      const uint32_t addr = b_lane + stage;
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(fb[sub][i - 4]) : "v"(addr), "i"((i - 4) * 2048));
    }
  };
  // the fragment reads of a sub-step have landed (ties the registers to the wait)
  auto frags_ready = [&](int sub) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[sub][0]), "+v"(fa[sub][1]), "+v"(fa[sub][2]), "+v"(fa[sub][3]),
                   "+v"(fb[sub][0]), "+v"(fb[sub][1]), "+v"(fb[sub][2]), "+v"(fb[sub][3])
                 :: "memory");
  };

  {
    // an AGPR operand anywhere in the kernel makes hipcc select the AGPR form of the MFMAs
    // (accumulators in AccVGPRs); the ArchVGPR form would need all 512 registers for them
    int zero = 0;
    asm volatile("; agpr-form hint %0" ::"a"(zero));
  }
  acc_t acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = acc_t{};
  auto mma = [&](u32x4 a, u32x4 b, acc_t c) -> acc_t {
    if constexpr (I8)
      return __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, a),
                                                   __builtin_bit_cast(i32x4, b), c, 0, 0, 0);
    else
      return mfma16(a, b, c);
  };
  // I8: the lane's queries (q = q_base + wq 128 + n 32 + r). Scores are kept divided by s_q
  // (one query per (lane, n), so the lane's and the workgroup's comparisons see one scale):
  // u = D a32 + e32 c1 + c2 with c1 = (|q| + eq) / s_q, c2 = eq / s_q, and s_q u is written to
  // the candidate lists. A zero query (s_q = 0: D = eq = |q| = 0) keeps scale 1, c1 = 1, c2 = 0
  // (e32 >= 0 still bounds its 0 cosine). For an fp16 query 1 <= c1 < 2^20 (s_q >= max|q_i| / 254,
  // |q| <= sqrt(DIM) max|q_i|), so a dead row's key (bias -1e30) stays finite and below -1e30;
  // scales that are not finite (a query holding inf/NaN) fall back to the zero query's.
  float qs_s[4] = {1.f, 1.f, 1.f, 1.f}, qs_c1[4] = {1.f, 1.f, 1.f, 1.f},
        qs_c2[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (I8) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int q = q_base + wq * 128 + n * 32 + r;
      if (q < nq) {
        const float4 v = qsc[q];
        const float c1 = v.z / v.x, c2 = v.y / v.x;
        if (v.x > 0.0f && c1 < 1.0e20f && c2 < 1.0e20f) {
          qs_s[n] = v.x;
          qs_c1[n] = c1;
          qs_c2[n] = c2;
        }
      }
    }
  }

  // Tile epilogue without compares (one wave per SIMD: nothing overlaps it, so no wave-divergent
  // insertion per score and no lane masks): each score carries its row code m*16 + j in its 6 low
  // mantissa bits (a perturbation below 2^-18 |score|, covered by the certificate's kEncodeSlack),
  // so per lane and query block a max/min chain keeps the tile's best two scores WITH their rows
  // and the largest score below them ("third"): three v_med3_f32 per score. Rows outside the range
  // or dropped by the filter (and rows the index marks invalid: NaN inverse norm) score -FLT_MAX
  // (I8: -1e30 c1 + c2) instead: every score is finite, so a coded score is never a NaN and the
  // v_med3_f32 chain needs no clamp or canonicalising copy. The two best join the lane list, third the discarded bound; a row leaves the
  // candidates only at or below its lane-tile's third or by eviction from the list, both covered by
  // the bound, so dense_merge_kernel's certificate holds (it fails only where one lane-tile of 64
  // rows holds three of the top k).
  auto epilogue = [&](int tile) {
    float b1[4], b2[4], b3[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) { b1[n] = kNegInf; b2[n] = kNegInf; b3[n] = kNegInf; }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      __builtin_amdgcn_sched_barrier(0);
      const int ro = tile * kG2Rows + wr * 128 + m * 32;  // row offset of the 32-row block
      const int64_t rb = lo + ro;
      uint32_t linv = lds0 + (uint32_t)(kW4Norm + (tile & 1) * 2048 +
                                        (wr * 128 + m * 32 + 4 * h) * 4);
      // block m's norms are read after block m-1's scores are folded (else hipcc hoists the
      // four blocks' norms and masks together)
      asm volatile("" : "+v"(linv) : "v"(b3[0]), "v"(b3[1]), "v"(b3[2]), "v"(b3[3]));
      u32x4 invw[4], errw[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(invw[g]) : "v"(linv), "i"(32 * g));
      if constexpr (I8) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(errw[g]) : "v"(linv), "i"(1024 + 32 * g));
      }
      uint32_t valid = ro + 32 <= n_here ? 0xffffffffu
                                         : (ro >= n_here ? 0u : (1u << (n_here - ro)) - 1u);
      if (row_mask && valid) valid &= (uint32_t)(row_mask[rb >> 6] >> (rb & 63));
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(invw[0]), "+v"(invw[1]), "+v"(invw[2]), "+v"(invw[3]), "+v"(errw[0]),
                     "+v"(errw[1]), "+v"(errw[2]), "+v"(errw[3])::"memory");
      // score = fma(acc, inv, bias): (inv, 0) for a live row, (0, -FLT_MAX) otherwise; I8:
      // inv = a32, bias = e32 (dead: e32 = -1e30, folded per query below)
      float inv[16], bias[16];
      const uint32_t vb = valid >> (4 * h);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t w4v[4] = {invw[g].x, invw[g].y, invw[g].z, invw[g].w};
        const uint32_t e4v[4] = {errw[g].x, errw[g].y, errw[g].z, errw[g].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 4 * g + e;
          const float iv = __uint_as_float(w4v[e]);
          const bool live = ((vb >> ((j & 3) + 8 * (j >> 2))) & 1u) && iv == iv;
          inv[j] = live ? iv : 0.0f;
          if constexpr (I8)
            bias[j] = live ? __uint_as_float(e4v[e]) : -1.0e30f;
          else
            bias[j] = live ? 0.0f : -3.4028234663852886e38f;
        }
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        __builtin_amdgcn_sched_barrier(0);
        // read here from AccVGPRs (else hipcc copies all 256 accumulators out at the loop exit),
        // after the previous block is folded (else the four blocks of m are read out together)
        asm volatile("" : "+a"(acc[m][n]) : "v"(b3[(n + 3) & 3]));
        // scores two rows at a time (v_pk_fma_f32)
        float y[16];
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          const f32x2 iv2 = {inv[j], inv[j + 1]}, bs2 = {bias[j], bias[j + 1]};
          f32x2 y2;
          if constexpr (I8) {
            // D a32 + e32 c1 + c2 (divided by s_q). A dead row (inv 0, bias -1e30) gives a
            // finite score <= -1e30 (1 <= c1 < 2^20)
            const f32x2 a2 = {(float)acc[m][n][j], (float)acc[m][n][j + 1]};
            y2 = __builtin_elementwise_fma(
                a2, iv2, __builtin_elementwise_fma(bs2, f32x2{qs_c1[n], qs_c1[n]},
                                                   f32x2{qs_c2[n], qs_c2[n]}));
          } else {
            y2 = __builtin_elementwise_fma(f32x2{acc[m][n][j], acc[m][n][j + 1]}, iv2, bs2);
          }
          y[j] = y2.x;
          y[j + 1] = y2.y;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          // code m*16 + j (an inline constant) in the low 6 mantissa bits (y is finite: the
          // coded score is too). b1 >= b2 >= b3: three v_med3_f32 keep the best two and the
          // third (the max as med3 against +FLT_MAX: the intrinsic takes the and-or's result
          // as it is, where max / maximumnum insert a canonicalising copy)
          const float e = __uint_as_float((__float_as_uint(y[j]) & ~63u) | (uint32_t)(m * 16 + j));
          const float nb3 = __builtin_amdgcn_fmed3f(b2[n], b3[n], e);
          b2[n] = __builtin_amdgcn_fmed3f(b1[n], b2[n], e);
          b1[n] = __builtin_amdgcn_fmed3f(b1[n], e, 3.4028234663852886e38f);
          b3[n] = nb3;
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const int32_t rbase = (int32_t)(lo + tile * kG2Rows + wr * 128) + 4 * h;
    // code m*16 + j -> row rbase + m*32 + (j & 3) + 8 (j >> 2); dead scores (no live row:
    // <= -1e30, where live ones are below 2^40 in magnitude) stay out of the lists and the bound
    constexpr float kDead = -1.0e29f;
    auto row_of = [&](float b) {
      const int32_t code = (int32_t)(__float_as_uint(b) & 63u);
      return rbase + ((code >> 4) << 5) + (code & 3) + ((code & 12) << 1);
    };
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      if (b1[n] > kDead) topm_insert<kLaneList>(b1[n], row_of(b1[n]), sl[n], il[n], dl[n]);
      if (b2[n] > kDead) topm_insert<kLaneList>(b2[n], row_of(b2[n]), sl[n], il[n], dl[n]);
      if (b3[n] > kDead) dl[n] = fmaxf(dl[n], b3[n]);
    }
  };

  const int n_steps = n_tiles * KT;
  if (n_steps > 0) {
    // prologue: stages 0-2 whole; stage 0 retired (the 16 younger pieces stay in flight)
#pragma unroll
    for (int st = 0; st < 3; ++st) {
      if (st % KT == 0) issue_norms(st / KT);
#pragma unroll
      for (int p = 0; p < 8; ++p) issue_piece(st, p);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i) read_item(0, 0, i);
    frags_ready(0);
    __builtin_amdgcn_sched_barrier(0);
    for (int tile = 0; tile < n_tiles; ++tile) {
      // one k-step; the tile's first starts the accumulators from the MFMAs' zero C operand (no
      // 256 AccVGPR writes per tile)
      auto kstep = [&](const int kt, auto first) {
        const int s = tile * KT + kt;
        // Stages past the last k-step are issued too (rows clamped into the store, never read),
        // so every wait keeps the same count and the loop carries no issue branches.
        const int s3 = s + 3;
        if (s3 % KT == 0) issue_norms(s3 / KT);
        // ---- first half: sub-step 0 MFMAs; sub-step 1 reads of stage s (between the first 8
        // MFMAs, so their latency hides behind the last 8); pieces 0-3 of stage s+3
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if constexpr (!(ABL & 4)) {
            if constexpr (decltype(first)::value)
              acc[i >> 2][i & 3] = mma(fa[0][i >> 2], fb[0][i & 3], acc_t{});
            else
              acc[i >> 2][i & 3] = mma(fa[0][i >> 2], fb[0][i & 3], acc[i >> 2][i & 3]);
          }
          if (i < 8) read_item(s, 1, i);
          if (!(ABL & 1) && i >= 8 && (i & 1)) issue_piece(s3, (i - 8) >> 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        frags_ready(1);
        // retire stage s+1 (younger: stage s+2 whole, the first half of s+3)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(ABL & 8)) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // ---- second half: sub-step 1 MFMAs; sub-step 0 reads of stage s+1; pieces 4-7 of s+3
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          if constexpr (!(ABL & 4))
            acc[i >> 2][i & 3] = mma(fa[1][i >> 2], fb[1][i & 3], acc[i >> 2][i & 3]);
          if (i < 8) read_item(s + 1, 0, i);
          if (!(ABL & 1) && i >= 8 && (i & 1)) issue_piece(s3, 4 + ((i - 8) >> 1));
          __builtin_amdgcn_sched_barrier(0);
        }
        frags_ready(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n) asm volatile("" : "+a"(acc[m][n]));
        __builtin_amdgcn_sched_barrier(0);
      };
      kstep(0, std::true_type{});
      for (int kt = 1; kt < KT; ++kt) kstep(kt, std::false_type{});
      if constexpr (!(ABL & 2)) epilogue(tile);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // workgroup lists (the layout of dense_gemm_scan_glds_kernel); the tail stages' DMA must land
  // before the ring is reused
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* lkey = reinterpret_cast<float*>(smem);                       // [256][16]
  int32_t* lrow = reinterpret_cast<int32_t*>(smem + kGQB * 16 * 4);   // [256][16]
  float* ldisc = reinterpret_cast<float*>(smem + kGQB * 16 * 8);      // [256][4]
  {
    const int slot = (wr * 2 + h) * kLaneList;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int q = wq * 128 + n * 32 + r;
#pragma unroll
      for (int j = 0; j < kLaneList; ++j) {
        lkey[q * 16 + slot + j] = sl[n][j] * qs_s[n];  // I8: back to key units (else * 1)
        lrow[q * 16 + slot + j] = il[n][j];
      }
      ldisc[q * 4 + wr * 2 + h] = dl[n] * qs_s[n];
    }
  }
  __syncthreads();
  for (int round = 0; round < kGQB / 16; ++round) {  // 4 waves x 4 queries per round
    const int ql = (round * 4 + wave) * 4 + (lane >> 4);
    float key = lkey[ql * 16 + (lane & 15)];
    int32_t row = lrow[ql * 16 + (lane & 15)];
#pragma unroll
    for (int size = 2; size <= 16; size <<= 1) {
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const float ok = armi::xor_stride(key, stride);
        const int32_t orow = armi::xor_stride(row, stride);
        const bool lower = (lane & stride) == 0;
        const bool desc = (lane & size) == 0;
        const bool other_better = armi::approx_better(ok, orow, key, row);
        const bool take_other = (lower == desc) ? other_better : !other_better;
        if (take_other) { key = ok; row = orow; }
      }
    }
    const int rank = (lane & 16) ? 15 - (lane & 15) : (lane & 15);
    const int qg = q_base + ql;
    if constexpr (I8) {
      // image position -> ordinal (armi_index.h: row rr of image tile tau is ordinal
      // rr * T + tile_ord[tau])
      const int64_t T = n_rows / 32;
      if (row >= 0) row = (int32_t)((int64_t)(row & 31) * T + tile_ord[row >> 5]);
    }
    if (qg < nq) {
      const size_t base = (size_t)rp * nq + qg;
      cand_key[base * kKW + rank] = key;
      cand_row[base * kKW + rank] = row;
      if (rank == 0) {
        const float* dd = ldisc + ql * 4;
        cand_bound[base] = fmaxf(fmaxf(dd[0], dd[1]), fmaxf(dd[2], dd[3]));
      }
    }
  }
}

// Per-call int8 quantisation of the queries for the int8 tiled scan (one wave per query):
// s_q = f max|q_i| / 127 with the f of {1, 0.8, 0.65, 0.5} whose clamped rounding
// q8 = clamp(round(q / s_q), +-127) leaves the smallest residual (clipping a few large components
// buys a finer step for the rest: the residual is in the bound whatever it is), and the scales
// qsc[q] = (s_q, eq, |q| + eq, 0) with eq >= ||q - s_q q8||_2 and |q| rounded up. Rounding: the
// computed residual r_i = fl(q_i - fl(s_q q8_i)) is within 2^-23 (|q_i| + |rho_i|) of the true
// one, and the fp32 sum of DIM squares within DIM 2^-24 relative, so
// eq = sqrt(sum r^2) (1 + 2^-10) + |q| 2^-20 bounds ||rho|| (DIM <= 1024).
template <int DIM>
__global__ __launch_bounds__(256) void query_i8_kernel(const uint16_t* __restrict__ queries,
                                                       int nq, int8_t* __restrict__ q8,
                                                       float4* __restrict__ qsc) {
  const int q = blockIdx.x * 4 + armi::wave_id();
  if (q >= nq) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  constexpr int CH = DIM / 8;               // 16-B chunks of 8 components
  constexpr int PER = (CH + 63) / 64;
  float v[PER][8];
  float amax = 0.0f, ss = 0.0f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    u32x4 w = {0u, 0u, 0u, 0u};
    if (c < CH) w = *reinterpret_cast<const u32x4*>(queries + (size_t)q * DIM + 8 * c);
    const half8 hv = __builtin_bit_cast(half8, w);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[i][e] = (float)hv[e];
      amax = fmaxf(amax, fabsf(v[i][e]));
      ss += v[i][e] * v[i][e];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    amax = fmaxf(amax, armi::xor_stride(amax, off));
    ss += armi::xor_stride(ss, off);
  }
  constexpr float kF[4] = {1.0f, 0.8f, 0.65f, 0.5f};
  float err[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float sf = amax * kF[f] / 127.0f;
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = sf > 0.0f ? rintf(v[i][e] / sf) : 0.0f;
        t = fminf(fmaxf(t, -127.0f), 127.0f);
        const float res = v[i][e] - sf * t;
        err[f] += res * res;
      }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) err[f] += armi::xor_stride(err[f], off);
  }
  int best = 0;
#pragma unroll
  for (int f = 1; f < 4; ++f) best = err[f] < err[best] ? f : best;
  const float sq = amax * kF[best] / 127.0f;
  float er = 0.0f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    uint32_t packed[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = sq > 0.0f ? rintf(v[i][e] / sq) : 0.0f;
      t = fminf(fmaxf(t, -127.0f), 127.0f);
      const float res = v[i][e] - sq * t;
      er += res * res;
      packed[e >> 2] |= ((uint32_t)(int32_t)t & 0xffu) << (8 * (e & 3));
    }
    if (c < CH)
      *reinterpret_cast<u32x2*>(q8 + (size_t)q * DIM + 8 * c) = u32x2{packed[0], packed[1]};
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) er += armi::xor_stride(er, off);
  if (lane == 0) {
    const float qn = sqrtf(ss) * (1.0f + 1.0f / 4096.0f);
    const float eq = sqrtf(er) * (1.0f + 1.0f / 1024.0f) + qn * (1.0f / 1048576.0f);
    qsc[q] = make_float4(sq, eq, qn + eq, 0.0f);
  }
}

// This lane's DIM/64 contiguous fp16 elements of a vector, as raw 8-byte words.
template <int DIM>
__device__ __forceinline__ void load_raw(const uint16_t* __restrict__ v, int lane,
                                         u32x2 (&raw)[DIM / 256]) {
  constexpr int E = DIM / 64;
  const u32x2* p = reinterpret_cast<const u32x2*>(v + lane * E);
#pragma unroll
  for (int i = 0; i < E / 4; ++i) raw[i] = p[i];
}

template <int DIM>
__device__ __forceinline__ void raw_to_fixed(const u32x2 (&raw)[DIM / 256],
                                             int32_t (&out)[DIM / 64]) {
#pragma unroll
  for (int i = 0; i < DIM / 256; ++i) {
    out[4 * i + 0] = armi::fp16_to_fixed24(raw[i][0] & 0xffffu);
    out[4 * i + 1] = armi::fp16_to_fixed24(raw[i][0] >> 16);
    out[4 * i + 2] = armi::fp16_to_fixed24(raw[i][1] & 0xffffu);
    out[4 * i + 3] = armi::fp16_to_fixed24(raw[i][1] >> 16);
  }
}

// Exact 2^24 fixed-point image of this lane's DIM/64 contiguous elements.
template <int DIM>
__device__ __forceinline__ void load_fixed(const uint16_t* __restrict__ v, int lane,
                                           int32_t (&out)[DIM / 64]) {
  u32x2 raw[DIM / 256];
  load_raw<DIM>(v, lane, raw);
  raw_to_fixed<DIM>(raw, out);
}

// Exact int64 dot of this lane's slice, reduced over the wave.
template <int DIM>
__device__ __forceinline__ int64_t dot_fixed(const int32_t (&qf)[DIM / 64],
                                             const u32x2 (&raw)[DIM / 256]) {
  int32_t xf[DIM / 64];
  raw_to_fixed<DIM>(raw, xf);
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < DIM / 64; ++i) acc += (int64_t)qf[i] * (int64_t)xf[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += armi::xor_stride(acc, off);
  return acc;
}

template <int DIM>
__device__ __forceinline__ int64_t wave_dot_exact(const int32_t (&qf)[DIM / 64],
                                                  const uint16_t* __restrict__ row, int lane) {
  u32x2 raw[DIM / 256];
  load_raw<DIM>(row, lane, raw);
  return dot_fixed<DIM>(qf, raw);
}

// Per-query exact norm: writes 1/sqrt(norm2) (0 for a zero query) and |q| in real units.
template <int DIM>
__global__ __launch_bounds__(64) void query_norms_kernel(const uint16_t* __restrict__ queries,
                                                         int nq, double* __restrict__ inv_q,
                                                         double* __restrict__ qnorm_real) {
  const int q = blockIdx.x;
  if (q >= nq) return;
  const int lane = threadIdx.x;
  int32_t qf[DIM / 64];
  load_fixed<DIM>(queries + (size_t)q * DIM, lane, qf);
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < DIM / 64; ++i) acc += (int64_t)qf[i] * (int64_t)qf[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += armi::xor_stride(acc, off);
  if (lane == 0) {
    inv_q[q] = acc > 0 ? 1.0 / sqrt((double)acc) : 0.0;
    qnorm_real[q] = sqrt((double)acc) * (1.0 / 16777216.0);
  }
}

// Order-preserving map of a float to uint32 (larger float -> larger key; -inf lowest).
__device__ __forceinline__ uint32_t ord_key(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_ord_key(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// One workgroup per query (all passes of the call): exact query norm, select, exact rescore,
// certify, emit.
//   Each scan workgroup's list is sorted, so its first entry is its maximum. The kc-th largest of
//   those maxima, t0 (a radix select over the 256 maxima in one wave), is a lower bound of the
//   pooled kc-th best, hence every entry of the pooled top-kc is >= t0: only entries >= t0 are
//   kept (typically ~2*kc of n_wg*kKW) and sorted. Entries below t0 are discards and join the
//   bound. Small sorts run inside one wave (shuffles, no barriers).
constexpr int kSelCap = 1024;  // kept entries per query; overflow -> uncertified (exact fallback)
constexpr int kRescoreBatch = 8;

// Exact keys of 8 rows at once by one wave: each row's inverse norm is loaded with the row (same
// round trip), and the 8 per-lane partial dots are reduced together (a halving butterfly: 10 int64
// shuffles for 8 rows instead of 48). rr[j] = ordinal of row j or -1. Lane 8r (r = 0..7) ends
// with row r's exact key in `key` (-inf for rr[r] < 0) and its ordinal in `row` (integer sums:
// any order gives the same bits).
template <int DIM>
__device__ __forceinline__ void exact_keys8(const int32_t (&qf)[DIM / 64],
                                            const uint16_t* __restrict__ rows,
                                            const double* __restrict__ inv_norm,
                                            const int32_t (&rr)[8], int lane, double& key,
                                            int32_t& row) {
  u32x2 raw[8][DIM / 256];
  double inv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int32_t src = rr[j] >= 0 ? rr[j] : 0;
    load_raw<DIM>(rows + (size_t)src * DIM, lane, raw[j]);
    inv[j] = inv_norm[src];
  }
  int64_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int32_t xf[DIM / 64];
    raw_to_fixed<DIM>(raw[j], xf);
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < DIM / 64; ++i) acc += (int64_t)qf[i] * (int64_t)xf[i];
    v[j] = acc;
  }
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
#pragma unroll
  for (int m = 0; m < 4; ++m) {  // lanes with bit 5 keep rows 4..7, the others rows 0..3
    const int64_t mine = b5 ? v[4 + m] : v[m];
    const int64_t give = b5 ? v[m] : v[4 + m];
    v[m] = mine + armi::xor_stride(give, 32);
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int64_t mine = b4 ? v[2 + m] : v[m];
    const int64_t give = b4 ? v[m] : v[2 + m];
    v[m] = mine + armi::xor_stride(give, 16);
  }
  int64_t dot = (b3 ? v[1] : v[0]) + armi::xor_stride(b3 ? v[0] : v[1], 8);
  dot += armi::xor_stride(dot, 4);
  dot += armi::xor_stride(dot, 2);
  dot += armi::xor_stride(dot, 1);
  const int r = (lane >> 3) & 7;  // = 4 b5 + 2 b4 + b3
  row = -1;
  double myinv = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j == r) {
      row = rr[j];
      myinv = inv[j];
    }
  }
  key = row >= 0 ? (double)dot * myinv : kNegInfD;
}

// fp32 keys of 8 rows at once, in exact_keys8's layout and key units (2^24 |q| cos). Each lane's
// DIM/64 products q_i x_i are exact in fp32 (fp16 significands: 11 x 11 bits, |q_i x_i| < 4 and
// >= 2^-48, no under- or overflow), summed by FMA in element order, then the 8 rows' 64 lane
// partials by the same halving butterfly; key_f = dot_f * 2^48 * inv_norm[row] in double, stored
// as float. |key_f - key| <= (DIM + 66) 2^-24 |q| |x| * 2^24 / |x| + |key| 2^-24
// <= (DIM + 67) |q| (standard FMA-sum error bound over <= DIM + 6 roundings, Cauchy-Schwarz;
// the last term the float store).
template <int DIM>
__device__ __forceinline__ void approx_keys8(const float (&qh)[DIM / 64],
                                             const uint16_t* __restrict__ rows,
                                             const double* __restrict__ inv_norm,
                                             const int32_t (&rr)[8], int lane, float& key,
                                             int32_t& row) {
  u32x2 raw[8][DIM / 256];
  double inv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int32_t src = rr[j] >= 0 ? rr[j] : 0;
    load_raw<DIM>(rows + (size_t)src * DIM, lane, raw[j]);
    inv[j] = inv_norm[src];
  }
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < DIM / 256; ++i) {
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const uint32_t word = raw[j][i][w];
        const float x0 = (float)__builtin_bit_cast(_Float16, (uint16_t)(word & 0xffffu));
        const float x1 = (float)__builtin_bit_cast(_Float16, (uint16_t)(word >> 16));
        acc = __builtin_fmaf(qh[4 * i + 2 * w], x0, acc);
        acc = __builtin_fmaf(qh[4 * i + 2 * w + 1], x1, acc);
      }
    }
    v[j] = acc;
  }
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const float mine = b5 ? v[4 + m] : v[m];
    const float give = b5 ? v[m] : v[4 + m];
    v[m] = mine + armi::xor_stride(give, 32);
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const float mine = b4 ? v[2 + m] : v[m];
    const float give = b4 ? v[m] : v[2 + m];
    v[m] = mine + armi::xor_stride(give, 16);
  }
  float dot = (b3 ? v[1] : v[0]) + armi::xor_stride(b3 ? v[0] : v[1], 8);
  dot += armi::xor_stride(dot, 4);
  dot += armi::xor_stride(dot, 2);
  dot += armi::xor_stride(dot, 1);
  const int r = (lane >> 3) & 7;
  row = -1;
  double myinv = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j == r) {
      row = rr[j];
      myinv = inv[j];
    }
  }
  key = row >= 0 ? (float)((double)dot * 281474976710656.0 * myinv) : kNegInf;
  if (key != key) key = __builtin_inff();  // NaN: always rescored exactly
}

// Largest float <= x (x finite or infinite).
__device__ __forceinline__ float f32_round_down(double x) {
  float f = (float)x;
  if ((double)f > x) {  // one ulp toward -inf (f is finite here)
    const uint32_t u = __float_as_uint(f);
    f = f > 0.0f ? __uint_as_float(u - 1u) : (f == 0.0f ? -1.17549435e-38f : __uint_as_float(u + 1u));
  }
  return f;
}

// sel_col (J) / sel_rank (r): t0 = the r-th largest of the workgroup lists' J-th entries. r lists
// hold >= J entries >= t0 each, so the pool holds >= r J >= kc entries >= t0 and its kc-th best is
// >= t0 (host: the smallest J with r = ceil(kc / J) <= n_wg; with r > n_wg, t0 = -inf).
// Probe builds only (-DARMI_PROBE_BUILD -DARMI_I8_STAMPS): s_memrealtime per merge workgroup
// (thread 0) at entry and after each phase, read back with the scan's stamps.
#if defined(ARMI_PROBE_BUILD) && defined(ARMI_I8_STAMPS)
__device__ uint64_t g_merge_stamps[64 * 8];
#define MERGE_STAMP(slot)                                                            \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 64)                                         \
      g_merge_stamps[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
#else
#define MERGE_STAMP(slot) do {} while (0)
#endif

template <int DIM>
__device__ __forceinline__ void merge_body(
    const int qg, const float* __restrict__ cand_key, const int32_t* __restrict__ cand_row,
    const float* __restrict__ cand_bound, int n_wg, int q_stride, const uint16_t* __restrict__ rows,
    const double* __restrict__ inv_norm, const uint16_t* __restrict__ queries,
    double* __restrict__ inv_q_out, double* __restrict__ qnorm_out, int k, int kc, int sel_col,
    int sel_rank, int64_t ordinal_base,
    float* __restrict__ out_scores, int64_t* __restrict__ out_ids, double* __restrict__ out_rank,
    int32_t* __restrict__ out_count, uint32_t* __restrict__ out_flags, float* __restrict__ thr_out,
    int32_t* __restrict__ col_cnt, int32_t* __restrict__ help_done, int two_stage){
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* skey = reinterpret_cast<float*>(smem);                              // [kSelCap]
  int32_t* srow = reinterpret_cast<int32_t*>(smem + kSelCap * 4);            // [kSelCap]
  double* rkey = reinterpret_cast<double*>(smem + kSelCap * 8);              // [256]
  int64_t* rord = reinterpret_cast<int64_t*>(smem + kSelCap * 8 + 256 * 8);  // [256]
  float* red = reinterpret_cast<float*>(smem + kSelCap * 8 + 256 * 16);      // [16]
  int* ctr = reinterpret_cast<int*>(smem + kSelCap * 8 + 256 * 16 + 64);     // [4]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  const int pool = n_wg * kKW;
  MERGE_STAMP(0);

  // One memory round trip for everything the selection needs: the pool (8 entries per thread;
  // pool <= kMaxPool = 8 * 512, so one round), the workgroup lists' bounds and the query are all
  // in flight before anything waits. Entry g * kKW is workgroup g's maximum (its list is sorted).
  constexpr int kFilterBatch = 8;
  static_assert(kFilterBatch * kDenseMergeThreads >= kMaxPool, "one filter round");
  float kk[kFilterBatch];
  int32_t rw[kFilterBatch];
#pragma unroll
  for (int j = 0; j < kFilterBatch; ++j) {
    const int e = tid + j * kDenseMergeThreads;
    const size_t src = ((size_t)(e / kKW) * q_stride + qg) * kKW + (e % kKW);
    kk[j] = e < pool ? cand_key[src] : kNegInf;
    rw[j] = e < pool ? cand_row[src] : 0;
  }
  float b = tid < n_wg ? cand_bound[(size_t)tid * q_stride + qg] : kNegInf;
  // exact query norm (every wave holds the fixed-point query for the rescore anyway)
  int32_t qf[DIM / 64];
  load_fixed<DIM>(queries + (size_t)qg * DIM, lane, qf);
  int64_t n2q = 0;
#pragma unroll
  for (int i = 0; i < DIM / 64; ++i) n2q += (int64_t)qf[i] * (int64_t)qf[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) n2q += armi::xor_stride(n2q, off);
  const double inv_q = n2q > 0 ? 1.0 / sqrt((double)n2q) : 0.0;
  const double qnorm_real = sqrt((double)n2q) * (1.0 / 16777216.0);
  if (tid == 0) {
    // read by the collect merge (agent-scope stores: past this XCD's L2)
    __hip_atomic_store(inv_q_out + qg, inv_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(qnorm_out + qg, qnorm_real, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ctr[0] = 0;
  }
#if defined(ARMI_PROBE_BUILD) && defined(ARMI_MERGE_ABL) && ARMI_MERGE_ABL == 3
  if (kk[0] == 12345.f && rw[kFilterBatch - 1] == -7 && b == 1.f) out_flags[qg] = 0;  // keep loads
  return;  // probe: loads + query norm only
#endif
  // workgroup maxima and bound partials to LDS (rkey is free until the rescore)
  uint32_t* umax = reinterpret_cast<uint32_t*>(rkey);         // [256]
  float* bpart = reinterpret_cast<float*>(rkey) + 256;        // [kDenseMergeThreads / 64]
#pragma unroll
  for (int j = 0; j < kFilterBatch; ++j) {
    const int e = tid + j * kDenseMergeThreads;
    if (sel_col > 0 && e < pool && e % kKW == sel_col - 1) umax[e / kKW] = ord_key(kk[j]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b = fmaxf(b, armi::xor_stride(b, off));
  if (lane == 0) bpart[wave] = b;
  __syncthreads(); MERGE_STAMP(1);

  // wave 0: t0 = kc-th largest workgroup maximum, and the workgroup lists' own bounds
  if (wave == 0) {
    float bb = kNegInf;
#pragma unroll
    for (int w = 0; w < kDenseMergeThreads / 64; ++w) bb = fmaxf(bb, bpart[w]);
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int g = lane + 64 * i;
      u[i] = g < n_wg ? umax[g] : ord_key(kNegInf);
    }
    float t0 = kNegInf;
    if (sel_col > 0 && n_wg >= sel_rank) {
      uint32_t prefix = 0;  // largest v with #{u >= v} >= r, i.e. the r-th largest key
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = prefix | (1u << bit);
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) cnt += __popcll(__ballot(u[i] >= cand));
        if (cnt >= sel_rank) prefix = cand;
      }
      t0 = from_ord_key(prefix);
    }
    if (lane == 0) {
      red[8] = bb;
      red[9] = t0;
    }
  }
  __syncthreads(); MERGE_STAMP(2);
  float t0 = red[9];
  if (sel_col == 0) {
    // exact selection (the int8 tiled scan): t0 = the kc-th largest key of the whole pool, by a
    // workgroup radix select over the keys held in registers (one barrier per bit; the per-wave
    // counts alternate between two LDS slots). Its looser upper bounds make many list entries
    // clear a list-statistics threshold, which overflowed kSelCap at 256 lists (r04w: every
    // query of a 1M x 256 call uncertified); the exact threshold keeps ~kc entries.
    int* wcnt = reinterpret_cast<int*>(rkey) + 320;  // [2][kMW], past umax / bpart
    uint32_t kq[kFilterBatch];
#pragma unroll
    for (int j = 0; j < kFilterBatch; ++j) kq[j] = ord_key(kk[j]);
    uint32_t prefix = 0;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t cand = prefix | (1u << bit);
      int c = 0;
#pragma unroll
      for (int j = 0; j < kFilterBatch; ++j) c += __popcll(__ballot(kq[j] >= cand));
      if (lane == 0) wcnt[(bit & 1) * 8 + wave] = c;
      __syncthreads();
      int tot = 0;
#pragma unroll
      for (int w = 0; w < kDenseMergeThreads / 64; ++w) tot += wcnt[(bit & 1) * 8 + w];
      if (tot >= kc) prefix = cand;
    }
    const uint32_t lowest = ord_key(kNegInf);
    t0 = from_ord_key(prefix > lowest ? prefix : lowest);
  }

  // filter the pool held in registers
  float dmax = kNegInf;
#pragma unroll
  for (int j = 0; j < kFilterBatch; ++j) {
    if (kk[j] == kNegInf) continue;
    if (kk[j] >= t0) {
      const int slot = atomicAdd(&ctr[0], 1);
      if (slot < kSelCap) {
        skey[slot] = kk[j];
        srow[slot] = rw[j];
      }
    } else {
      dmax = fmaxf(dmax, kk[j]);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dmax = fmaxf(dmax, armi::xor_stride(dmax, off));
  if (lane == 0) red[wave] = dmax;
  __syncthreads(); MERGE_STAMP(3);
  const int n_sel = ctr[0];
  const bool overflow = n_sel > kSelCap;
  const int n_keep = overflow ? kSelCap : n_sel;
  int n2;
  if (n_keep <= 64 && kc <= 64) {
    if (wave == 0) {
      float key = lane < n_keep ? skey[lane] : kNegInf;
      int32_t row = lane < n_keep ? srow[lane] : 0x7fffffff;
      armi::wave_sort_approx_desc(key, row);
      skey[lane] = key;
      srow[lane] = row;
    }
    __syncthreads();
    n2 = 64;
  } else if (n_keep <= 4 * 64 && kc <= 64) {
    // Top 64 of up to 256 kept entries without a workgroup-wide bitonic sort (one barrier per
    // stage): each wave sorts a run of 64 in registers, then wave 0 folds the runs pairwise (run
    // A against run B reversed: the lane-wise better entries are the top 64 of both, a bitonic
    // sequence that 6 half-cleaner stages sort). Everything folded away joins the bound.
    {
      float key = 64 * wave + lane < n_keep ? skey[64 * wave + lane] : kNegInf;
      int32_t row = 64 * wave + lane < n_keep ? srow[64 * wave + lane] : 0x7fffffff;
      armi::wave_sort_approx_desc(key, row);
      skey[64 * wave + lane] = key;
      srow[64 * wave + lane] = row;
    }
    __syncthreads();
    if (wave == 0) {
      float key = skey[lane];
      int32_t row = srow[lane];
      float lost = kNegInf;
      for (int run = 1; run < 4 && 64 * run < n_keep; ++run) {
        const float okey = skey[64 * run + 63 - lane];
        const int32_t orow = srow[64 * run + 63 - lane];
        const bool other = armi::approx_better(okey, orow, key, row);
        lost = fmaxf(lost, other ? key : okey);
        if (other) { key = okey; row = orow; }
#pragma unroll
        for (int stride = 32; stride > 0; stride >>= 1) {
          const float k2 = armi::xor_stride(key, stride);
          const int32_t r2 = armi::xor_stride(row, stride);
          const bool lower = (lane & stride) == 0;
          const bool better = armi::approx_better(k2, r2, key, row);
          if (lower == better) { key = k2; row = r2; }
        }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) lost = fmaxf(lost, armi::xor_stride(lost, off));
      skey[lane] = key;
      srow[lane] = row;
      if (lane == 0) red[10] = lost;
    }
    __syncthreads();
    n2 = 64;
  } else {
    n2 = armi::pow2_at_least(n_keep > kc ? n_keep : kc);
    for (int e = n_keep + tid; e < n2; e += kDenseMergeThreads) {
      skey[e] = kNegInf;
      srow[e] = 0x7fffffff;
    }
    armi::lds_sort_approx_desc(skey, srow, n2);
  }
#if defined(ARMI_PROBE_BUILD) && defined(ARMI_MERGE_ABL) && ARMI_MERGE_ABL == 2
  if (tid == 0) out_flags[qg] = 0;
  return;  // probe: up to the sorted selection
#endif
  MERGE_STAMP(4);
  float bound = red[8];
#pragma unroll
  for (int w = 0; w < kDenseMergeThreads / 64; ++w) bound = fmaxf(bound, red[w]);
  if (n_keep > 64 && n_keep <= 4 * 64 && kc <= 64) bound = fmaxf(bound, red[10]);
  if (kc < n2) bound = fmaxf(bound, skey[kc]);

  static_assert(kRescoreBatch == 8, "exact_keys8 reduces 8 rows");
  constexpr int kMW = kDenseMergeThreads / 64;
  const int per_wave = (kc + kMW - 1) / kMW;
  // Two-stage rescore (default; two_stage = 0: every one of the kc exactly, the round-3 form).
  // Stage 1: fp32 keys key_f of the kc best (approx_keys8), |key_f - key| <= e_f. Every row with
  // key_f >= cut = (k-th largest key_f) - 2 e_f is rescored exactly; a row below cut has
  // key < k-th key_f - e_f <= the exact key of each of the k rows with key_f >= k-th key_f, so
  // the exactly rescored rows hold the top-k of the kc (ties at the k-th included), and only
  // ~k + a few of the kc pay the int64 arithmetic.
  int32_t* xlist = reinterpret_cast<int32_t*>(smem + kSelCap * 8 + 256 * 16 + 64 + 16);  // [256]
  int n_x = kc;  // rows rescored exactly (entries of xlist when two_stage)
  if (two_stage) {
    float qh[DIM / 64];
    {
      u32x2 qraw[DIM / 256];
      load_raw<DIM>(queries + (size_t)qg * DIM, lane, qraw);
#pragma unroll
      for (int i = 0; i < DIM / 256; ++i)
#pragma unroll
        for (int w = 0; w < 2; ++w) {
          qh[4 * i + 2 * w] = (float)__builtin_bit_cast(_Float16, (uint16_t)(qraw[i][w] & 0xffffu));
          qh[4 * i + 2 * w + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(qraw[i][w] >> 16));
        }
    }
    for (int i0 = 0; i0 < per_wave; i0 += kRescoreBatch) {
      int32_t rr[kRescoreBatch];
#pragma unroll
      for (int j = 0; j < kRescoreBatch; ++j) {
        const int c = wave + kMW * (i0 + j);
        const bool live = (i0 + j < per_wave) && c < kc && skey[c] != kNegInf;
        rr[j] = live ? srow[c] : -1;
      }
      float key;
      int32_t myrow;
      approx_keys8<DIM>(qh, rows, inv_norm, rr, lane, key, myrow);
      const int r = (lane >> 3) & 7;
      if ((lane & 7) == 0 && i0 + r < per_wave) {
        const int c = wave + kMW * (i0 + r);
        if (c < kc) skey[c] = key;  // (this wave's own entries: read above, then replaced)
      }
    }
    __syncthreads();
    if (wave == 0) {
      // k-th largest key_f (radix select over <= 256 entries), the cut, the list of rows >= cut
      uint32_t u[4];
      int live = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        u[i] = c < kc ? ord_key(skey[c]) : ord_key(kNegInf);
        live += c < kc && skey[c] != kNegInf;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) live += armi::xor_stride(live, off);
      double cut = kNegInfD;
      if (live >= k) {
        uint32_t prefix = 0;
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t cand = prefix | (1u << bit);
          int cnt = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) cnt += __popcll(__ballot(u[i] >= cand));
          if (cnt >= k) prefix = cand;
        }
        const double e_f = (double)(DIM + 67) * qnorm_real * 1.0625;  // key units, 6 % margin
        cut = (double)from_ord_key(prefix) - 2.0 * e_f;
      }
      int m = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = lane + 64 * i;
        const float kf = c < kc ? skey[c] : kNegInf;
        const bool take = kf != kNegInf && (double)kf >= cut;
        const unsigned long long bm = __ballot(take);
        if (take) xlist[m + __popcll(bm & ((1ull << lane) - 1ull))] = c;
        m += __popcll(bm);
      }
      if (lane == 0) ctr[1] = m;
    }
    __syncthreads();
    n_x = ctr[1];
  }
  // exact rescore, kRescoreBatch rows in flight per wave (exact_keys8): entry i of the exact set
  // is xlist[i] (two_stage) or i
  const int per_wave_x = (n_x + kMW - 1) / kMW;
  for (int i0 = 0; i0 < per_wave_x; i0 += kRescoreBatch) {
    int32_t rr[kRescoreBatch];
#pragma unroll
    for (int j = 0; j < kRescoreBatch; ++j) {
      const int i = wave + kMW * (i0 + j);
      bool live = i0 + j < per_wave_x && i < n_x;
      int c = 0;
      if (live) {
        c = two_stage ? xlist[i] : i;
        live = skey[c] != kNegInf;
      }
      rr[j] = live ? srow[c] : -1;
    }
    double key;
    int32_t myrow;
    exact_keys8<DIM>(qf, rows, inv_norm, rr, lane, key, myrow);
    const int r = (lane >> 3) & 7;
    if ((lane & 7) == 0 && i0 + r < per_wave_x) {
      const int i = wave + kMW * (i0 + r);
      if (i < n_x) {
        rkey[i] = key;
        rord[i] = myrow >= 0 ? ordinal_base + myrow : kNoOrd;
      }
    }
  }
  // sort the exact set: n_s = its size padded to a power of two (<= kc)
  const int n_s = n_x <= 64 ? 64 : armi::pow2_at_least(n_x);
  for (int i = n_x + tid; i < n_s; i += kDenseMergeThreads) {
    rkey[i] = kNegInfD;
    rord[i] = kNoOrd;
  }
  __syncthreads();
  MERGE_STAMP(5);
  if (n_s <= 64) {
    if (wave == 0) {
      double key = rkey[lane];
      int64_t ord = rord[lane];
      armi::wave_sort_rank_desc(key, ord);
      rkey[lane] = key;
      rord[lane] = ord;
    }
    __syncthreads();
  } else {
    armi::lds_sort_rank_desc(rkey, rord, n_s);
  }

  MERGE_STAMP(6);
  if (wave != 0) return;
  // valid entries form a prefix of the sorted list
  int n_valid = 0;
  for (int c = lane; c < n_s; c += 64) n_valid += rord[c] != kNoOrd;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) n_valid += armi::xor_stride(n_valid, off);
  bool certified;
  int n_out;
  const double delta =
      (kDeltaSafety * (double)DIM * (1.0 / 16777216.0) + kEncodeSlack) * qnorm_real;
  // second-pass threshold: every row of the true top-k has exact >= this k-th exact key (found
  // rows are real rows), hence int8 key >= kth - delta; fewer than k valid rows: collect them all
  float thr = kNegInf;
  if (n_valid >= k) {
    const double kth = rkey[k - 1] * (1.0 / 16777216.0);
    certified = kth > (double)bound + delta;
    thr = f32_round_down(kth - delta);
    n_out = k;
  } else {
    certified = (bound == kNegInf);
    n_out = n_valid;
  }
  certified = certified && !overflow;
  if (certified) {
    for (int c = lane; c < k; c += 64) {
      const size_t o = (size_t)qg * k + c;
      if (c < n_out) {
        out_scores[o] = (float)(rkey[c] * inv_q);
        out_ids[o] = rord[c];
        if (out_rank) out_rank[o] = rkey[c];
      } else {
        out_scores[o] = kNegInf;
        out_ids[o] = -1;
        if (out_rank) out_rank[o] = kNegInfD;
      }
    }
  }
  if (lane == 0) {
    // an uncertified query's count is the collect merge's to write (one writer per address: two
    // XCDs' L2s writing the same line back in either order could leave this one's 0 last)
    if (certified) out_count[qg] = n_out;
    // what the collect pass reads, stored past this XCD's L2 (agent scope: `sc1`)
    __hip_atomic_store(out_flags + qg, certified ? ARMI_FLAG_CERTIFIED : 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(thr_out + qg, certified ? __builtin_inff() : thr, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(col_cnt + qg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(help_done + qg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  MERGE_STAMP(7);
}

template <int DIM>
__global__ __launch_bounds__(kDenseMergeThreads) void dense_merge_kernel(
    const float* __restrict__ cand_key, const int32_t* __restrict__ cand_row,
    const float* __restrict__ cand_bound, int n_wg, int q_stride, const uint16_t* __restrict__ rows,
    const double* __restrict__ inv_norm, const uint16_t* __restrict__ queries,
    double* __restrict__ inv_q_out, double* __restrict__ qnorm_out, int k, int kc, int sel_col,
    int sel_rank, int64_t ordinal_base,
    float* __restrict__ out_scores, int64_t* __restrict__ out_ids, double* __restrict__ out_rank,
    int32_t* __restrict__ out_count, uint32_t* __restrict__ out_flags, float* __restrict__ thr_out,
    int32_t* __restrict__ col_cnt, int32_t* __restrict__ help_done, int two_stage) {
  merge_body<DIM>(blockIdx.x, cand_key, cand_row, cand_bound, n_wg, q_stride, rows, inv_norm, queries,
      inv_q_out, qnorm_out, k, kc, sel_col, sel_rank, ordinal_base, out_scores, out_ids,
      out_rank, out_count, out_flags, thr_out, col_cnt, help_done, two_stage);
}


constexpr size_t kMergeLds = kSelCap * 8 + 256 * 16 + 64 + 16 + 256 * 4;

// Second-pass merge, one workgroup per query (certified queries exit at once): exact keys of the
// rows dense_scan_i8_kernel<COLLECT> appended (local rows -> ordinals), top-k by (key desc,
// ordinal asc). The list holds every row of the true top-k (see the collect pass), so this top-k
// is the exact answer. Rows go through LDS 512 at a time: [0, 512) the best so far, [512, 1024)
// the next chunk, one bitonic sort per chunk; a list of <= 512 rows is scored and sorted once.
// A query whose list overflowed (more than cap rows within delta + the int8 slack of its k-th key:
// a pile of near-duplicates) is answered by the grid's n_help helper workgroups instead: helper h
// scores its 1/n_help of the shard exactly and writes its slice's top-k rows into the query's
// list (slot h * k ...), and the last helper to finish (a per-query counter, zeroed by
// dense_merge_kernel) merges those n_help * k <= cap rows as above. The shard is read once per
// such query, spread over n_help CUs. Helpers find nothing to do, and exit, on every other call.
constexpr int kColChunk = 512;
constexpr size_t kColMergeLds = 2 * kColChunk * 16 + 16;
constexpr int kMaxHelp = 64;
// Per-query capacity of the collect pass's row list (beyond it the second-pass merge scores every
// row itself: a pathological pile of > 4096 rows within the bound slack of the k-th key).
constexpr int kCollectCap = 4096;

// Top of n rows (list entries, or rows r0 .. r0 + n - 1 of the shard when list == nullptr) left
// sorted by (key desc, ordinal asc) in key / ord [0, max(n, k)); filtered / invalid rows skipped.
template <int DIM>
__device__ void collect_top_rows(const int32_t* __restrict__ list, int64_t r0, int64_t n, int k,
                                 const int32_t (&qf)[DIM / 64], const uint16_t* __restrict__ rows,
                                 const double* __restrict__ inv_norm,
                                 const int64_t* __restrict__ norm2,
                                 const uint64_t* __restrict__ row_mask, int64_t ordinal_base,
                                 double* key, int64_t* ord) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  __syncthreads();  // the caller's previous use of key / ord is over
  for (int e = tid; e < 2 * kColChunk; e += kDenseMergeThreads) {
    key[e] = kNegInfD;
    ord[e] = kNoOrd;
  }
  const bool single = n <= kColChunk;
  constexpr int kPerWave = kColChunk / (kDenseMergeThreads / 64);  // 64 rows per wave and chunk
  for (int64_t c0 = 0; c0 < n; c0 += kColChunk) {
    const int base = single ? 0 : kColChunk;
    const int m = (int)min<int64_t>(kColChunk, n - c0);
    __syncthreads();  // the previous sort is done with [base, base + kColChunk)
    for (int b = 0; b < kPerWave; b += 8) {
      int32_t rr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = kPerWave * wave + b + j;
        int32_t o = -1;
        if (e < m) {
          if (list == nullptr) {
            const int64_t row = r0 + c0 + e;
            const bool on = norm2[row] >= 0 &&
                            (!row_mask || ((row_mask[row >> 6] >> (row & 63)) & 1ull));
            o = on ? (int32_t)row : -1;
          } else {
            o = list[c0 + e];
          }
        }
        rr[j] = o;
      }
      double kk;
      int32_t myrow;
      exact_keys8<DIM>(qf, rows, inv_norm, rr, lane, kk, myrow);
      if ((lane & 7) == 0) {
        const int e = base + kPerWave * wave + b + ((lane >> 3) & 7);
        key[e] = kk;
        ord[e] = myrow >= 0 ? ordinal_base + myrow : kNoOrd;
      }
    }
    armi::lds_sort_rank_desc(key, ord,
                             single ? armi::pow2_at_least(m > k ? m : k) : 2 * kColChunk);
  }
  __syncthreads();
}

template <int DIM>
__device__ __forceinline__ void collect_merge_body(
    const int bid, const int n_help, const int32_t* __restrict__ col_cnt, int32_t* __restrict__ col_list, int col_cap,
    int32_t* __restrict__ help_done, int nq, const uint16_t* __restrict__ rows,
    const double* __restrict__ inv_norm, const int64_t* __restrict__ norm2,
    const uint64_t* __restrict__ row_mask, int64_t n_rows, const uint16_t* __restrict__ queries,
    const double* __restrict__ inv_q, int k, int64_t ordinal_base, float* __restrict__ out_scores,
    int64_t* __restrict__ out_ids, double* __restrict__ out_rank, int32_t* __restrict__ out_count,
    uint32_t* __restrict__ flags){
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* key = reinterpret_cast<double*>(smem);                            // [2 * kColChunk]
  int64_t* ord = reinterpret_cast<int64_t*>(smem + 2 * kColChunk * 8);       // [2 * kColChunk]
  int* s_last = reinterpret_cast<int*>(smem + 2 * kColChunk * 16);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  auto write_out = [&](int qg) {
    if (wave != 0) return;
    int n_valid = 0;
    for (int c = lane; c < k; c += 64) n_valid += ord[c] != kNoOrd;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) n_valid += armi::xor_stride(n_valid, off);
    const double iq = inv_q[qg];
    for (int c = lane; c < k; c += 64) {
      const size_t o = (size_t)qg * k + c;
      const bool v = ord[c] != kNoOrd;
      out_scores[o] = v ? (float)(key[c] * iq) : kNegInf;
      out_ids[o] = v ? ord[c] : -1;
      out_rank[o] = v ? key[c] : kNegInfD;
    }
    if (lane == 0) {
      out_count[qg] = n_valid;
      flags[qg] = ARMI_FLAG_FALLBACK;
    }
  };
  if (bid < nq) {  // the query's own workgroup
    const int qg = bid;
    if (flags[qg] & ARMI_FLAG_CERTIFIED) return;  // workgroup-uniform
    const int cnt = col_cnt[qg];
    if (cnt > col_cap) return;  // overflowed: the helpers answer it
    int32_t qf[DIM / 64];
    load_fixed<DIM>(queries + (size_t)qg * DIM, lane, qf);
    collect_top_rows<DIM>(col_list + (size_t)qg * col_cap, 0, cnt, k, qf, rows, inv_norm, norm2,
                          row_mask, ordinal_base, key, ord);
    write_out(qg);
    return;
  }
  const int h = bid - nq;
  const int64_t lo = n_rows * h / n_help, hi = n_rows * (h + 1) / n_help;
  // Nearly every call has no overflowed query: every thread checks its share of the queries at
  // once (one load round trip, one barrier) before the per-query walk, whose dependent flag /
  // count loads cost ~nq round trips (10 us at nq = 64, profiles/r04p: the helpers were the
  // collect merge's whole time on certified calls).
  bool any = false;
  for (int q = tid; q < nq; q += kDenseMergeThreads)
    any |= !(flags[q] & ARMI_FLAG_CERTIFIED) && col_cnt[q] > col_cap;
  if (!__syncthreads_or(any)) return;  // workgroup-uniform
  for (int qg = 0; qg < nq; ++qg) {
    if ((flags[qg] & ARMI_FLAG_CERTIFIED) || col_cnt[qg] <= col_cap) continue;  // uniform
    int32_t qf[DIM / 64];
    load_fixed<DIM>(queries + (size_t)qg * DIM, lane, qf);
    collect_top_rows<DIM>(nullptr, lo, hi - lo, k, qf, rows, inv_norm, norm2, row_mask,
                          ordinal_base, key, ord);
    int32_t* list = col_list + (size_t)qg * col_cap;
    for (int c = tid; c < k; c += kDenseMergeThreads)
      list[h * k + c] = ord[c] != kNoOrd ? (int32_t)(ord[c] - ordinal_base) : -1;
    __threadfence();
    __syncthreads();
    if (tid == 0) *s_last = atomicAdd(help_done + qg, 1) == n_help - 1;
    __syncthreads();
    if (*s_last) {  // every helper's slice is in the list
      __threadfence();
      collect_top_rows<DIM>(list, 0, (int64_t)n_help * k, k, qf, rows, inv_norm, norm2, row_mask,
                            ordinal_base, key, ord);
      write_out(qg);
    }
  }
}

template <int DIM>
__global__ __launch_bounds__(kDenseMergeThreads) void dense_collect_merge_kernel(
    const int32_t* __restrict__ col_cnt, int32_t* __restrict__ col_list, int col_cap,
    int32_t* __restrict__ help_done, int nq, const uint16_t* __restrict__ rows,
    const double* __restrict__ inv_norm, const int64_t* __restrict__ norm2,
    const uint64_t* __restrict__ row_mask, int64_t n_rows, const uint16_t* __restrict__ queries,
    const double* __restrict__ inv_q, int k, int64_t ordinal_base, float* __restrict__ out_scores,
    int64_t* __restrict__ out_ids, double* __restrict__ out_rank, int32_t* __restrict__ out_count,
    uint32_t* __restrict__ flags) {
  collect_merge_body<DIM>(blockIdx.x, (int)gridDim.x - nq, col_cnt, col_list, col_cap, help_done, nq, rows,
      inv_norm, norm2, row_mask, n_rows, queries, inv_q, k, ordinal_base, out_scores, out_ids,
      out_rank, out_count, flags);
}


// First kernel of a filtered int8-scan call: the caller's row filter in int8 image order: bit p
// of the output = bit img_to_ord(p) of the caller's ordinal mask (0 for padding positions), one
// wave per 64 image positions.
__global__ __launch_bounds__(256) void scan_prep_kernel(const uint64_t* __restrict__ mask,
                                                        int64_t n_rows, int64_t T,
                                                        const int32_t* __restrict__ tile_ord,
                                                        uint64_t* __restrict__ out) {
  const int64_t pos = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool bit = false;
  if (pos < T * 32) {
    const int64_t i = (pos & 31) * T + tile_ord[pos >> 5];
    bit = i < n_rows && ((mask[i >> 6] >> (i & 63)) & 1ull);
  }
  const uint64_t b = __ballot(bit);
  if ((threadIdx.x & 63) == 0 && pos < T * 32) out[pos >> 6] = b;
}

// Exhaustive exact scan: grid (n_blocks, nq); block b scores rows [b*rpb, (b+1)*rpb) and keeps
// its best `cap` (power of two) entries. Queries whose flag says CERTIFIED are skipped.
template <int DIM>
__global__ __launch_bounds__(256) void dense_exact_scan_kernel(
    const uint16_t* __restrict__ rows, const double* __restrict__ inv_norm,
    const int64_t* __restrict__ norm2, const uint64_t* __restrict__ row_mask, int64_t n_rows,
    int64_t rows_per_block, const uint16_t* __restrict__ queries, const uint32_t* __restrict__ flags,
    int cap, int64_t ordinal_base, double* __restrict__ ex_key, int64_t* __restrict__ ex_ord) {
  const int q = blockIdx.y;
  if (flags && (flags[q] & ARMI_FLAG_CERTIFIED)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* key = reinterpret_cast<double*>(smem);               // [2*cap]
  int64_t* ord = reinterpret_cast<int64_t*>(smem + 2 * cap * 8);  // [2*cap]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  for (int e = tid; e < 2 * cap; e += 256) {
    key[e] = kNegInfD;
    ord[e] = kNoOrd;
  }
  int32_t qf[DIM / 64];
  load_fixed<DIM>(queries + (size_t)q * DIM, lane, qf);
  const int64_t lo = (int64_t)blockIdx.x * rows_per_block;
  const int64_t hi = min(lo + rows_per_block, n_rows);
  __syncthreads();
  for (int64_t c0 = lo; c0 < hi; c0 += cap) {
    for (int i = wave; i < cap; i += 4) {
      const int64_t row = c0 + i;
      double kk = kNegInfD;
      int64_t oo = kNoOrd;
      if (row < hi) {
        const bool on = (!row_mask || ((row_mask[row >> 6] >> (row & 63)) & 1ull)) && norm2[row] >= 0;
        if (on) {
          const int64_t dot = wave_dot_exact<DIM>(qf, rows + (size_t)row * DIM, lane);
          kk = (double)dot * inv_norm[row];
          oo = ordinal_base + row;
        }
      }
      if (lane == 0) {
        key[cap + i] = kk;
        ord[cap + i] = oo;
      }
    }
    armi::lds_sort_rank_desc(key, ord, 2 * cap);
  }
  const size_t base = ((size_t)q * gridDim.x + blockIdx.x) * cap;
  for (int e = tid; e < cap; e += 256) {
    ex_key[base + e] = key[e];
    ex_ord[base + e] = ord[e];
  }
}

// Byte strides of the lists merge_lists_kernel reads: element j of list s for query q sits at
// s*s8 + q*q8 + 8j (key, ordinal) and s*s4 + q*q4 + 4j (score); its count at s*cs + q*cq. Plain
// [S][B][k] arrays and the packed rows of the sharded exchange (every field of a (shard, query)
// row in one byte row, read in place) are both such layouts.
struct ListLayout {
  int64_t s8, q8, s4, q4, cs, cq;
};

// Generic merge of sorted-or-unsorted (key, ordinal) lists (layout above); lists hold `width`
// slots of which counts (nullable) say how many are valid (otherwise ordinal == kNoOrd marks an
// empty slot).
// only_uncertified: skip queries whose flag has CERTIFIED, mark the others FALLBACK.
__global__ __launch_bounds__(kMergeThreads) void merge_lists_kernel(
    const unsigned char* __restrict__ in_key, const unsigned char* __restrict__ in_score,
    const unsigned char* __restrict__ in_ord, const unsigned char* __restrict__ in_count,
    ListLayout lay, int n_lists, int width,
    int pool2, const double* __restrict__ inv_q, int k_out, double* __restrict__ out_key,
    float* __restrict__ out_score, int64_t* __restrict__ out_ord, int32_t* __restrict__ out_count,
    uint32_t* __restrict__ flags, int only_uncertified) {
  const int q = blockIdx.x;
  if (only_uncertified && (flags[q] & ARMI_FLAG_CERTIFIED)) return;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* key = reinterpret_cast<double*>(smem);
  int64_t* ord = reinterpret_cast<int64_t*>(smem + pool2 * 8);
  float* sc = reinterpret_cast<float*>(smem + pool2 * 16);
  const int tid = threadIdx.x;
  const int pool = n_lists * width;
  // sort (key, ord) and look scores up afterwards through a (list, slot) payload packed in ord's
  // companion array: keep scores in LDS addressed by the pooled index.
  int32_t* src = reinterpret_cast<int32_t*>(smem + pool2 * 20);
  for (int e = tid; e < pool2; e += kMergeThreads) {
    double kk = kNegInfD;
    int64_t oo = kNoOrd;
    float ss = kNegInf;
    if (e < pool) {
      const int s = e / width, j = e % width;
      const int cnt = in_count ? *reinterpret_cast<const int32_t*>(
                                     in_count + s * lay.cs + q * lay.cq)
                               : width;
      if (j < cnt) {
        const int64_t at = s * lay.s8 + q * lay.q8 + 8 * (int64_t)j;
        oo = *reinterpret_cast<const int64_t*>(in_ord + at);
        if (oo != kNoOrd && oo >= 0) {
          kk = *reinterpret_cast<const double*>(in_key + at);
          ss = in_score ? *reinterpret_cast<const float*>(in_score + s * lay.s4 + q * lay.q4 +
                                                          4 * (int64_t)j)
                        : 0.0f;
        } else {
          oo = kNoOrd;
        }
      }
    }
    key[e] = kk;
    ord[e] = oo;
    sc[e] = ss;
    src[e] = e;
  }
  __syncthreads();
  // bitonic sort carrying the source index (so scores follow their entry)
  for (int size = 2; size <= pool2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < pool2 / 2; t += kMergeThreads) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const bool hi_better = armi::rank_better(key[hi], ord[hi], key[lo], ord[lo]);
        if (hi_better == desc) {
          const double tk = key[lo]; key[lo] = key[hi]; key[hi] = tk;
          const int64_t to = ord[lo]; ord[lo] = ord[hi]; ord[hi] = to;
          const int32_t ts = src[lo]; src[lo] = src[hi]; src[hi] = ts;
        }
      }
      __syncthreads();
    }
  }
  int* s_valid_p = reinterpret_cast<int*>(smem + pool2 * 24);
  if (tid == 0) {
    int nv = 0;
    while (nv < pool2 && nv < k_out && ord[nv] != kNoOrd) ++nv;
    *s_valid_p = nv;
  }
  __syncthreads();
  const int nv = *s_valid_p;
  const double iq = inv_q ? inv_q[q] : 0.0;
  for (int c = tid; c < k_out; c += kMergeThreads) {
    const size_t o = (size_t)q * k_out + c;
    if (c < nv) {
      out_key[o] = key[c];
      out_ord[o] = ord[c];
      out_score[o] = in_score ? sc[src[c]] : (float)(key[c] * iq);
    } else {
      out_key[o] = kNegInfD;
      out_ord[o] = -1;
      out_score[o] = kNegInf;
    }
  }
  if (tid == 0) {
    out_count[q] = nv;
    if (only_uncertified) flags[q] = ARMI_FLAG_FALLBACK;
  }
}

size_t merge_lds_bytes(int pool2) { return (size_t)pool2 * 24 + 16; }

struct ScanPlan {
  int n_qb = 1;   // 64-query blocks of the call
  int grid = 0;   // workgroups launched
  int xcd_step = 1;  // single block on few workgroups: the working ones sit on 8 / xcd_step XCDs
  int n_wg = 0;   // tile ranges (candidate lists per query)
  int tiles_per_wg = 0;
  int pool2 = 0;
  int kc = 0;
};

ScanPlan plan_scan(const armi_index* idx, int k, int nq) {
  ScanPlan p;
  const int64_t tiles = std::max<int64_t>(idx->n_tiles, 1);
  const int cus = std::min(std::max(idx->num_cus, 1), 256);
  p.n_qb = std::max(1, (nq + kQB - 1) / kQB);
  // one block: at least one tile per wave of a workgroup (round 5). A small shard (10k rows: 313
  // tiles) otherwise spread over 157 workgroups of 2 tiles, each paying the query-image phase and
  // writing 64 x 16 candidates (2 MB of lists = 27 % over the 10 MB image, and a 2.5k-entry merge
  // pool); 40 workgroups of 8 tiles finish as early and write a quarter of that.
  int64_t want = p.n_qb > 1 ? cus : std::min<int64_t>(cus, (tiles + kWaves - 1) / kWaves);
  if (p.n_qb > 1) want = std::max<int64_t>(8, ((cus + p.n_qb - 1) / p.n_qb + 7) / 8 * 8);
  const int64_t wgs = std::min<int64_t>(want, tiles);
  p.tiles_per_wg = (int)((tiles + wgs - 1) / wgs);
  p.n_wg = (int)((tiles + p.tiles_per_wg - 1) / p.tiles_per_wg);
  p.grid = p.n_qb == 1 ? p.n_wg : p.n_qb * 8 * ((p.n_wg + 7) / 8);
  // Probe builds only (ARMI_BUILD_FLAGS=-DARMI_XCD_COMPACT): a single block of <= 64 workgroups
  // on two XCDs (workgroup i runs on XCD i mod 8; the others exit at once), so only two L2s fetch
  // the fp16 queries (128 KB each). At 10k rows that takes the scan's HBM traffic from 1.18 to
  // 1.06 x (one XCD) of its 10.4 MB but the step from 0.0518 to 0.0535-0.0537 ms: the 20
  // workgroups' query-image reads then share one or two L2s (profiles/r05p_xcd_ab.txt).
#ifdef ARMI_XCD_COMPACT
  if (p.n_qb == 1 && p.n_wg <= 2 * std::max(1, cus / 8)) {
    p.xcd_step = 4;
    p.grid = p.n_wg * p.xcd_step;
  }
#endif
  p.pool2 = armi::pow2_at_least(p.n_wg * kKW);
  p.kc = std::max(4, std::min(armi::pow2_at_least(k + 8), 256));
  return p;
}

// Multi-block calls (more than kQB queries): up to 2 blocks the XCD-grouped dense_scan_kernel
// (HBM-bound, rows shared through L2), beyond that the LDS-DMA tiled dense_gemm_scan_w4_kernel
// (rows read once per 256 queries). Measured per-GPU call times, 1M rows / G with G*64 queries
// (profiles/r01f_scan_form_ab.txt, r02_w4_scan_ab.txt): the grouped scan wins at G = 2, the
// tiled one from G = 4 on.
bool use_gemm_scan(int nq) { return nq > 2 * kQB; }

// The 64-query scan reads the int8 filter image (dense_scan_i8_kernel) for k <= 64, with the
// merge rescoring the kc_i8 best upper bounds; larger k takes the fp16 scan (dense_scan_kernel).
// k = 40 is the reference's default hybrid prefetch (QueryPipeline.query -> search(top_k=20) ->
// dense prefetch limit 2 * 20, src/audio_rag/retrieval/qdrant.py:281-293).
constexpr int kI8MaxK = 64;
bool use_i8_filter(const armi_index* idx, int k) { return idx->rows8 != nullptr && k <= kI8MaxK; }
// The int8 passes stream the image with nontemporal loads when it exceeds ARMI_I8_NT_MIN_MB: an
// image that the Infinity Cache (256 MB) cannot hold is re-read from HBM every call anyway, and
// the nontemporal form ran 4 % faster at 1M rows (1 GB image); at 100k rows (100 MB, cache
// resident across calls) it ran 2-5 % slower (profiles/r04aj_dense_nt_skew_ab.txt).
#ifndef ARMI_I8_NT_MIN_MB
#define ARMI_I8_NT_MIN_MB 192
#endif
bool use_nt_stream(const armi_index* idx) {
  return (double)idx->n_tiles * TILE_ROWS * idx->dim > ARMI_I8_NT_MIN_MB * 1048576.0;
}
// Rows rescored per query after the int8 pass: the rows whose key (an upper bound) reaches the
// k-th exact cosine are about 15-35 for k = 5 at 1M random unit rows (bound slack ~0.008). k <= 10
// rescores 64 (hybrid's dense prefetch of 10: 6 400 of 6 400 queries certified at 1M rows, step
// 0.255 vs 0.273 ms with 128, tools/probes/kc_ab.sh); a query whose k-th cosine sits among more
// near-equal bounds takes the exact fallback, so only its time depends on this choice.
// k = 40 at 1M random unit rows: ~110 rows reach the 40th cosine (bound slack 0.26 sigma at
// 3.94 sigma), so 256; the collect pass catches whatever a smaller pool misses.
int kc_i8(int k) { return k <= 10 ? 64 : (k <= 20 ? 128 : 256); }
// The int8 x int8 tiled scan's bound adds the query's quantisation term (eq ~ ||q|| 0.006-0.009 at
// dim 1024): about twice the slack of the 64-query int8 scan, so the merge rescores 256 rows,
// selected exactly from the pool. One uncertified query costs the call a collect pass over the
// shard, so the form runs where its certificate holds and its halved k-loop pays
// (tools/probes/tiled_i8_cert.py, random unit rows, top-5; profiles/r04y_tiled_i8_threshold.txt):
// 100 % certified from 250k rows up (250k x 256: 201 vs 229 us per call on the fp16 form; 1.25M x
// 512: 1.10 vs ~1.45 ms), 98.6-99.2 % at 65k-125k rows (then slower than the fp16 form). At k = 40
// too many rows reach the 40th cosine through the slack (10 % of 1.25M-row calls certified, r04s).
// So: k <= 5 (the metric's top-5) on shards of >= 200k rows; otherwise the fp16 tiled scan.
constexpr int kTiledI8MaxK = 5;
constexpr int64_t kTiledI8MinRows = 200000;
int kc_tiled_i8(int) { return 256; }
bool use_tiled_i8(const armi_index* idx, int k) {
  return idx->rows8 != nullptr && k <= kTiledI8MaxK && idx->n_rows >= kTiledI8MinRows;
}

// dense_merge_kernel's rescore: fp32 keys of the kc best, exact keys only for the rows within the
// fp32 error of the k-th, when kc > 64 (k > 10: hybrid's prefetch of 40 rescores 256); else every
// one of the kc exactly. Measured (profiles/r03y_*): kc 256 two-stage 0.274 vs 0.280 ms per 1M
// step at k = 40 and hybrid 0.568 vs 0.575-0.589 ms; kc 64 two-stage 0.2585 vs 0.2557 ms (k = 5)
// and 0.0775 vs 0.0724 ms at 100k rows, where the fp32 pass's extra round trip and barrier cost
// more than the int64 work it saves. ARMI_MERGE_RESCORE=exact|two forces either (A/B, tests).
bool merge_two_stage(int kc) {
  const char* e = getenv("ARMI_MERGE_RESCORE");  // (read per call: tests switch in-process)
  if (e && e[0] == 'e') return false;
  if (e && e[0] == 't') return true;
  return kc > 64;
}

// Threshold column of the merge's pool selection (dense_merge_kernel): the smallest J (power of
// two, <= kKW) with r = ceil(kc / J) <= n_wg. (sel_col = 0 instead selects the pool's exact kc-th
// key: the int8 tiled scan.)
void merge_select(int kc, int n_wg, int& col, int& rank) {
  int j = 1;
  while (j < kKW && (kc + j - 1) / j > n_wg) j <<= 1;
  col = j;
  rank = (kc + j - 1) / j;
}

struct GemmPlan {
  int n_qb = 0;
  int n_ranges = 0;
  int64_t rows_per_range = 0;
  int grid = 0;
};

// rows scanned by the tiled form: image positions (T * 32) for the int8 form, else the rows
int64_t gemm_rows(const armi_index* idx, int k) {
  return use_tiled_i8(idx, k) ? std::max<int64_t>(idx->n_tiles, 1) * 32 : idx->n_rows;
}

GemmPlan plan_gemm(const armi_index* idx, int nq, int64_t n_scan) {
  GemmPlan p;
  p.n_qb = (nq + kGQB - 1) / kGQB;
  const int cus = std::min(std::max(idx->num_cus, 1), 256);
  const int64_t rows = std::max<int64_t>(n_scan, 1);
  int want = std::max(1, (cus + p.n_qb - 1) / p.n_qb);
  want = (int)std::min<int64_t>(want, (rows + kGRT - 1) / kGRT);  // >= one row tile per range
  // dense_gemm_scan_w4_kernel addresses a range's rows (plus one tile of clamped reads) with
  // 32-bit byte offsets: enough ranges that every range stays below 4 GiB (<= 256 ranges, the
  // merge's pool, cover 512M rows at dim 1024 - more than 288 GB of HBM holds)
  const int64_t max_rows = ((int64_t(1) << 32) / (2 * (int64_t)idx->dim) - 2 * kG2Rows) / 32 * 32;
  want = (int)std::max<int64_t>(want, (rows + max_rows - 1) / max_rows);
  p.rows_per_range = ((rows + want - 1) / want + 31) / 32 * 32;
  p.n_ranges = (int)((rows + p.rows_per_range - 1) / p.rows_per_range);
  p.grid = p.n_qb == 2 ? 16 * ((p.n_ranges + 7) / 8) : p.n_qb * p.n_ranges;
  return p;
}

struct ExactPlan {
  int cap = 0;
  int n_blocks = 0;
  int64_t rows_per_block = 0;
  int pool2 = 0;
};

ExactPlan plan_exact(const armi_index* idx, int k) {
  ExactPlan p;
  p.cap = std::max(64, armi::pow2_at_least(k));
  const int max_blocks = std::max(1, kMaxPool / p.cap);
  const int64_t want = (idx->n_rows + 4095) / 4096;  // >= 4k rows per block
  p.n_blocks = (int)std::max<int64_t>(1, std::min<int64_t>(max_blocks, want));
  p.rows_per_block = (idx->n_rows + p.n_blocks - 1) / p.n_blocks;
  if (p.rows_per_block == 0) p.rows_per_block = 1;
  p.pool2 = armi::pow2_at_least(p.n_blocks * p.cap);
  return p;
}

struct Workspace {
  float* cand_key;
  int32_t* cand_row;
  float* cand_bound;
  double* inv_q;
  double* qnorm;
  double* ex_key;
  int64_t* ex_ord;
  float* thr;          // [nq] collect threshold (+inf: certified)
  int32_t* col_cnt;    // [nq] rows appended by the collect pass
  int32_t* col_list;   // [nq][kCollectCap] local rows
  int32_t* help_done;  // [nq] helper workgroups done with an overflowed query
  uint64_t* mask_img;  // row filter in int8 image order
  int8_t* q8;          // [nq][dim] int8 queries of the int8 tiled scan
  float4* qsc;         // [nq] their scales (query_i8_kernel)
  size_t bytes;
};

Workspace carve(void* base, const armi_index* idx, int nq, int k, bool fast) {
  armi::Carver cv(base);
  Workspace w{};
  if (fast) {
    const int n_wg = use_gemm_scan(nq) ? plan_gemm(idx, nq, gemm_rows(idx, k)).n_ranges
                                       : plan_scan(idx, k, nq).n_wg;
    w.cand_key = cv.take<float>((size_t)n_wg * nq * kKW);
    w.cand_row = cv.take<int32_t>((size_t)n_wg * nq * kKW);
    w.cand_bound = cv.take<float>((size_t)n_wg * nq);
    w.thr = cv.take<float>(nq);
    w.col_cnt = cv.take<int32_t>(nq);
    w.col_list = cv.take<int32_t>((size_t)nq * kCollectCap);
    w.help_done = cv.take<int32_t>(nq);
    w.mask_img = cv.take<uint64_t>((size_t)(std::max<int64_t>(idx->n_tiles, 1) * 32 + 63) / 64);
    if (use_gemm_scan(nq) && use_tiled_i8(idx, k)) {
      w.q8 = cv.take<int8_t>((size_t)nq * idx->dim);
      w.qsc = cv.take<float4>(nq);
    }
  }
  w.inv_q = cv.take<double>(nq);
  w.qnorm = cv.take<double>(nq);
  if (!fast) {
    const ExactPlan ep = plan_exact(idx, k);
    w.ex_key = cv.take<double>((size_t)nq * ep.n_blocks * ep.cap);
    w.ex_ord = cv.take<int64_t>((size_t)nq * ep.n_blocks * ep.cap);
  }
  w.bytes = cv.off + 256;
  return w;
}

using armi::allow_lds;

// out_rank must be non-null (callers substitute workspace scratch).
template <int DIM>
int launch_exact(const armi_index* idx, const uint16_t* queries, int nq, int k,
                 const uint64_t* row_mask, float* out_scores, int64_t* out_ids, double* out_rank,
                 int32_t* out_count, uint32_t* flags, int only_uncertified, const Workspace& w,
                 hipStream_t stream) {
  const ExactPlan ep = plan_exact(idx, k);
  const size_t lds_merge = merge_lds_bytes(ep.pool2);
  if (int rc = allow_lds(merge_lists_kernel, lds_merge)) return rc;
  dense_exact_scan_kernel<DIM><<<dim3(ep.n_blocks, nq), dim3(256), (size_t)ep.cap * 32, stream>>>(
      idx->rows, idx->inv_norm, idx->norm2, row_mask, idx->n_rows, ep.rows_per_block, queries,
      only_uncertified ? flags : nullptr, ep.cap, idx->ordinal_base, w.ex_key, w.ex_ord);
  ARMI_LAUNCHED("dense_exact_scan_kernel");
  const ListLayout lay{/*s8=*/8 * (int64_t)ep.cap, /*q8=*/8 * (int64_t)ep.n_blocks * ep.cap, 0, 0,
                       0, 0};
  merge_lists_kernel<<<dim3(nq), dim3(kMergeThreads), lds_merge, stream>>>(
      reinterpret_cast<const unsigned char*>(w.ex_key), nullptr,
      reinterpret_cast<const unsigned char*>(w.ex_ord), nullptr, lay, ep.n_blocks, ep.cap,
      ep.pool2, w.inv_q, k, out_rank, out_scores, out_ids, out_count, flags, only_uncertified);
  ARMI_LAUNCHED("merge_lists_kernel(exact)");
  return ARMI_OK;
}

template <int DIM>
int dense_second_pass(const armi_index* idx, const uint16_t* queries, int nq, int k,
                      const uint64_t* row_mask, const uint64_t* mask_i8, float* out_scores,
                      int64_t* out_ids, double* out_rank, int32_t* out_count, uint32_t* out_flags,
                      const Workspace& w, hipStream_t stream);

template <int DIM>
int dense_topk_impl(const armi_index* idx, const uint16_t* queries, int nq, int k,
                    const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                    double* out_rank, int32_t* out_count, uint32_t* out_flags,
                    const Workspace& w, hipStream_t stream) {
  const ScanPlan sp = plan_scan(idx, k, nq);
  int n_wg = sp.n_wg;
  int kc = sp.kc;
  const int64_t T = std::max<int64_t>(idx->n_tiles, 1);
  // the int8 passes (first pass and collect pass) read the filter in image order
  const uint64_t* mask_i8 = nullptr;
  if (row_mask) {
    scan_prep_kernel<<<dim3((unsigned)std::max<int64_t>(1, (T * 32 + 255) / 256)), dim3(256), 0,
                       stream>>>(row_mask, idx->n_rows, T, idx->tile_ord, w.mask_img);
    ARMI_LAUNCHED("scan_prep_kernel");
    mask_i8 = w.mask_img;
  }
  if (use_gemm_scan(nq)) {
    const bool i8 = use_tiled_i8(idx, k);
    const int64_t n_scan = gemm_rows(idx, k);
    const GemmPlan gp = plan_gemm(idx, nq, n_scan);
    n_wg = gp.n_ranges;
    ARMI_REQUIRE((gp.rows_per_range + kG2Rows) * (int64_t)DIM * 2 < (int64_t(1) << 32),
                 "armi_dense_topk: row range too large for the tiled scan");
    if (i8) {
      kc = kc_tiled_i8(k);
      query_i8_kernel<DIM><<<dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, stream>>>(queries, nq,
                                                                                     w.q8, w.qsc);
      ARMI_LAUNCHED("query_i8_kernel");
    }
#if defined(ARMI_PROBE_BUILD) && defined(ARMI_W4_ABL)  // timing-only ablations (results wrong)
    auto kern = i8 ? dense_gemm_scan_w4_kernel<DIM, ARMI_W4_ABL, true>
                   : dense_gemm_scan_w4_kernel<DIM, ARMI_W4_ABL, false>;
#else
    auto kern = i8 ? dense_gemm_scan_w4_kernel<DIM, 0, true> : dense_gemm_scan_w4_kernel<DIM, 0, false>;
#endif
    if (int rc = allow_lds(kern, gemm_w4_lds_bytes<DIM>())) return rc;
    const int rc_l = armi::timed_kernel(
        ARMI_TIMING_DENSE_SCAN, kern, dim3(gp.grid), dim3(kW4Threads), gemm_w4_lds_bytes<DIM>(),
        stream, idx->rows, idx->inv_norm32, i8 ? mask_i8 : row_mask, n_scan, gp.rows_per_range,
        gp.n_ranges, gp.n_qb, queries, nq, w.cand_key, w.cand_row, w.cand_bound,
        (const int8_t*)idx->rows8, (const float*)idx->a32, (const float*)idx->e32,
        (const int32_t*)idx->tile_ord, (const int8_t*)w.q8, (const float4*)w.qsc);
    ARMI_LAUNCHED("dense_gemm_scan_w4_kernel");
    if (rc_l) return rc_l;
  } else if (use_i8_filter(idx, k)) {
    kc = kc_i8(k);
    auto kern = use_nt_stream(idx) ? dense_scan_i8_kernel<DIM, false, true>
                                   : dense_scan_i8_kernel<DIM, false, false>;
    if (int rc = allow_lds(kern, scan_i8_lds_bytes<DIM>())) return rc;
    const int rc_l = armi::timed_kernel(
        ARMI_TIMING_DENSE_SCAN, kern, dim3(sp.grid), dim3(kThreads), scan_i8_lds_bytes<DIM>(),
        stream, (const int8_t*)idx->rows8, (const float*)idx->a32, (const float*)idx->e32,
        mask_i8, idx->n_rows, idx->n_tiles, sp.tiles_per_wg, sp.n_wg, sp.n_qb, queries, nq,
        w.cand_key, w.cand_row, w.cand_bound, (const int32_t*)idx->tile_ord,
        (const uint32_t*)nullptr, (const float*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, 0,
        sp.xcd_step);
    ARMI_LAUNCHED("dense_scan_i8_kernel");
    if (rc_l) return rc_l;
  } else {
    if (int rc = allow_lds(dense_scan_kernel<DIM>, scan_lds_bytes<DIM>())) return rc;
    const int rc_l = armi::timed_kernel(
        ARMI_TIMING_DENSE_SCAN, dense_scan_kernel<DIM>, dim3(sp.grid), dim3(kThreads),
        scan_lds_bytes<DIM>(), stream, (const uint16_t*)idx->rows, (const float*)idx->inv_norm32,
        row_mask, idx->n_rows, idx->n_tiles, sp.tiles_per_wg, sp.n_wg, sp.n_qb, queries, nq,
        w.cand_key, w.cand_row, w.cand_bound);
    ARMI_LAUNCHED("dense_scan_kernel");
    if (rc_l) return rc_l;
  }
  // one merge for every query of the call: per-pass merges would serialise a latency-bound
  // kernel per 64 queries (the multi-GPU step scans G*64 queries)
  ARMI_REQUIRE(n_wg >= 1 && n_wg * kKW <= kMaxPool,
               "dense merge: the candidate pool must fit one filter round (<= 256 lists)");
  int sel_col = 1, sel_rank = kc;
  merge_select(kc, n_wg, sel_col, sel_rank);
  if (use_gemm_scan(nq) && use_tiled_i8(idx, k)) sel_col = 0;  // exact pool selection
  dense_merge_kernel<DIM><<<dim3(nq), dim3(kDenseMergeThreads), kMergeLds, stream>>>(
      w.cand_key, w.cand_row, w.cand_bound, n_wg, nq, idx->rows, idx->inv_norm, queries,
      w.inv_q, w.qnorm, k, kc, sel_col, sel_rank,
      idx->ordinal_base, out_scores, out_ids, out_rank, out_count, out_flags, w.thr, w.col_cnt,
      w.help_done, merge_two_stage(kc) ? 1 : 0);
  ARMI_LAUNCHED("dense_merge_kernel");
  return dense_second_pass<DIM>(idx, queries, nq, k, row_mask, mask_i8, out_scores, out_ids,
                                out_rank, out_count, out_flags, w, stream);
}

// Second pass for the uncertified queries (both kernels exit at once when every query of the
// call is certified): int8 collect over the whole shard, then exact rescore of the lists.
template <int DIM>
int dense_second_pass(const armi_index* idx, const uint16_t* queries, int nq, int k,
                      const uint64_t* row_mask, const uint64_t* mask_i8, float* out_scores,
                      int64_t* out_ids, double* out_rank, int32_t* out_count, uint32_t* out_flags,
                      const Workspace& w, hipStream_t stream) {
  {
    const ScanPlan cp = plan_scan(idx, k, 1);  // one block's ranges; blocks of one range share an XCD
    const int n_qb = (nq + kQB - 1) / kQB;
    const int grid = n_qb == 1 ? cp.n_wg : n_qb * 8 * ((cp.n_wg + 7) / 8);
    auto kern = use_nt_stream(idx) ? dense_scan_i8_kernel<DIM, true, true>
                                   : dense_scan_i8_kernel<DIM, true, false>;
    if (int rc = allow_lds(kern, scan_i8_lds_bytes<DIM>())) return rc;
    kern<<<dim3(grid), dim3(kThreads), scan_i8_lds_bytes<DIM>(), stream>>>(
        idx->rows8, idx->a32, idx->e32, mask_i8, idx->n_rows, idx->n_tiles, cp.tiles_per_wg,
        cp.n_wg, n_qb, queries, nq, nullptr, nullptr, nullptr, idx->tile_ord,
        out_flags, w.thr, w.col_cnt, w.col_list, kCollectCap, 1);
    ARMI_LAUNCHED("dense_scan_i8_kernel(collect)");
  }
  if (int rc = allow_lds(dense_collect_merge_kernel<DIM>, kColMergeLds)) return rc;
  // helpers for overflowed lists: each writes k rows into the list, so n_help * k <= the cap
  const int n_help = std::max(1, std::min<int>(kMaxHelp, kCollectCap / k));
  dense_collect_merge_kernel<DIM><<<dim3(nq + n_help), dim3(kDenseMergeThreads), kColMergeLds,
                                    stream>>>(
      w.col_cnt, w.col_list, kCollectCap, w.help_done, nq, idx->rows, idx->inv_norm, idx->norm2,
      row_mask, idx->n_rows, queries, w.inv_q, k, idx->ordinal_base, out_scores, out_ids,
      out_rank, out_count, out_flags);
  ARMI_LAUNCHED("dense_collect_merge_kernel");
  return ARMI_OK;
}

template <typename F>
int dispatch_dim(int dim, F&& f) {
  switch (dim) {
    case 256: return f(std::integral_constant<int, 256>{});
    case 512: return f(std::integral_constant<int, 512>{});
    case 768: return f(std::integral_constant<int, 768>{});
    case 1024: return f(std::integral_constant<int, 1024>{});
    default: return armi::fail(ARMI_ERR_INVALID, "unsupported dim");
  }
}

}  // namespace

extern "C" {

// Workspace layout: [carved buffers][rank scratch nq*k doubles][flags nq u32]
int armi_dense_scan_form(const armi_index* idx, int n_queries, int k) {
  if (!idx || n_queries <= 0 || k <= 0) return -1;
  k = std::min(k, kMaxK);
  if (use_gemm_scan(n_queries))
    return use_tiled_i8(idx, k) ? ARMI_SCAN_TILED_INT8 : ARMI_SCAN_TILED_FP16;
  return use_i8_filter(idx, k) ? ARMI_SCAN_INT8_FILTER : ARMI_SCAN_FP16;
}

int armi_dense_scan_nontemporal(const armi_index* idx, int n_queries, int k) {
  const int form = armi_dense_scan_form(idx, n_queries, k);
  if (form < 0) return -1;
  return form == ARMI_SCAN_INT8_FILTER && use_nt_stream(idx) ? 1 : 0;
}

size_t armi_dense_workspace_bytes(const armi_index* idx, int n_queries, int k) {
  if (!idx || n_queries <= 0 || k <= 0) return 0;
  k = std::min(k, kMaxK);
  const Workspace w = carve(nullptr, idx, n_queries, k, true);
  return armi::align_up(w.bytes, 256) + armi::align_up((size_t)n_queries * k * 8, 256) +
         armi::align_up((size_t)n_queries * 4, 256);
}

int armi_dense_topk(const armi_index* idx, const uint16_t* queries, int n_queries, int k,
                    const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                    double* out_rank, int32_t* out_count, uint32_t* out_flags, void* workspace,
                    size_t workspace_bytes, hipStream_t stream) {
  ARMI_REQUIRE(idx != nullptr, "armi_dense_topk: index is null");
  ARMI_REQUIRE(n_queries >= 0, "armi_dense_topk: n_queries < 0");
  ARMI_REQUIRE(k >= 1 && k <= kMaxK, "armi_dense_topk: k must be in [1, 240]");
  if (n_queries == 0) return ARMI_OK;
  ARMI_REQUIRE(queries && out_scores && out_ids && out_count && out_flags && workspace,
               "armi_dense_topk: null pointer argument");
  ARMI_REQUIRE(workspace_bytes >= armi_dense_workspace_bytes(idx, n_queries, k),
               "armi_dense_topk: workspace too small");
  ARMI_HIP(hipSetDevice(idx->device));
  if (idx->n_rows == 0) {
    ARMI_HIP(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_queries, stream));
    ARMI_HIP(hipMemsetAsync(out_flags, 0, sizeof(uint32_t) * n_queries, stream));
    ARMI_HIP(hipMemsetAsync(out_ids, 0xff, sizeof(int64_t) * n_queries * k, stream));
    return ARMI_OK;
  }
  const Workspace w = carve(workspace, idx, n_queries, k, true);
  double* rank = out_rank;
  if (!rank)
    rank = reinterpret_cast<double*>(static_cast<char*>(workspace) + armi::align_up(w.bytes, 256));
  return dispatch_dim(idx->dim, [&](auto D) {
    constexpr int DIM = decltype(D)::value;
    return dense_topk_impl<DIM>(idx, queries, n_queries, k, row_mask, out_scores, out_ids, rank,
                                out_count, out_flags, w, stream);
  });
}

size_t armi_dense_exact_workspace_bytes(const armi_index* idx, int n_queries, int k) {
  if (!idx || n_queries <= 0 || k <= 0) return 0;
  k = std::min(k, kMaxK);
  const Workspace w = carve(nullptr, idx, n_queries, k, false);
  return armi::align_up(w.bytes, 256) + armi::align_up((size_t)n_queries * k * 8, 256) +
         armi::align_up((size_t)n_queries * 4, 256);
}

int armi_dense_exact_topk(const armi_index* idx, const uint16_t* queries, int n_queries, int k,
                          const uint64_t* row_mask, float* out_scores, int64_t* out_ids,
                          double* out_rank, int32_t* out_count, void* workspace,
                          size_t workspace_bytes, hipStream_t stream) {
  ARMI_REQUIRE(idx != nullptr, "armi_dense_exact_topk: index is null");
  ARMI_REQUIRE(k >= 1 && k <= kMaxK, "armi_dense_exact_topk: k must be in [1, 240]");
  if (n_queries <= 0) return ARMI_OK;
  ARMI_REQUIRE(queries && out_scores && out_ids && out_count && workspace,
               "armi_dense_exact_topk: null pointer argument");
  ARMI_REQUIRE(workspace_bytes >= armi_dense_exact_workspace_bytes(idx, n_queries, k),
               "armi_dense_exact_topk: workspace too small");
  ARMI_HIP(hipSetDevice(idx->device));
  if (idx->n_rows == 0) {
    ARMI_HIP(hipMemsetAsync(out_count, 0, sizeof(int32_t) * n_queries, stream));
    ARMI_HIP(hipMemsetAsync(out_ids, 0xff, sizeof(int64_t) * n_queries * k, stream));
    return ARMI_OK;
  }
  const Workspace w = carve(workspace, idx, n_queries, k, false);
  char* tail = static_cast<char*>(workspace) + armi::align_up(w.bytes, 256);
  double* rank = out_rank ? out_rank : reinterpret_cast<double*>(tail);
  uint32_t* flags =
      reinterpret_cast<uint32_t*>(tail + armi::align_up((size_t)n_queries * k * 8, 256));
  ARMI_HIP(hipMemsetAsync(flags, 0, sizeof(uint32_t) * n_queries, stream));
  return dispatch_dim(idx->dim, [&](auto D) {
    constexpr int DIM = decltype(D)::value;
    query_norms_kernel<DIM><<<dim3(n_queries), dim3(64), 0, stream>>>(queries, n_queries,
                                                                      w.inv_q, w.qnorm);
    ARMI_LAUNCHED("query_norms_kernel");
    return launch_exact<DIM>(idx, queries, n_queries, k, row_mask, out_scores, out_ids, rank,
                             out_count, flags, 0, w, stream);
  });
}

#if defined(ARMI_PROBE_BUILD) && defined(ARMI_I8_STAMPS)
int armi_probe_i8_stamps(uint64_t* out) {
  ARMI_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_i8_stamps), sizeof(g_i8_stamps)));
  return ARMI_OK;
}
int armi_probe_merge_stamps(uint64_t* out) {
  ARMI_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_merge_stamps), sizeof(g_merge_stamps)));
  return ARMI_OK;
}
#endif

int armi_topk_merge_shards(const double* in_rank, const float* in_scores, const int64_t* in_ids,
                           const int32_t* in_count, int n_shards, int n_queries, int k_in,
                           int k_out, double* out_rank, float* out_scores, int64_t* out_ids,
                           int32_t* out_count, hipStream_t stream) {
  ARMI_REQUIRE(n_shards >= 1 && k_in >= 1 && k_out >= 1, "armi_topk_merge_shards: bad sizes");
  ARMI_REQUIRE((int64_t)n_shards * k_in <= kMaxPool,
               "armi_topk_merge_shards: n_shards * k_in must be <= 4096");
  if (n_queries <= 0) return ARMI_OK;
  ARMI_REQUIRE(in_rank && in_scores && in_ids && in_count && out_rank && out_scores && out_ids &&
                   out_count,
               "armi_topk_merge_shards: null pointer argument");
  const int pool2 = armi::pow2_at_least(n_shards * k_in);
  if (int rc = allow_lds(merge_lists_kernel, merge_lds_bytes(pool2))) return rc;
  const int64_t nk = (int64_t)n_queries * k_in;
  const ListLayout lay{8 * nk, 8 * (int64_t)k_in, 4 * nk, 4 * (int64_t)k_in,
                       4 * (int64_t)n_queries, 4};
  using B = const unsigned char*;
  merge_lists_kernel<<<dim3(n_queries), dim3(kMergeThreads), merge_lds_bytes(pool2), stream>>>(
      reinterpret_cast<B>(in_rank), reinterpret_cast<B>(in_scores), reinterpret_cast<B>(in_ids),
      reinterpret_cast<B>(in_count), lay, n_shards, k_in, pool2, nullptr, k_out, out_rank,
      out_scores, out_ids, out_count, nullptr, 0);
  ARMI_LAUNCHED("merge_lists_kernel(shards)");
  return ARMI_OK;
}

int armi_topk_merge_shards_packed(const void* packed, int64_t shard_stride,
                                  int64_t query_stride, int64_t off_rank, int64_t off_scores,
                                  int64_t off_ids, int64_t off_count, int n_shards,
                                  int n_queries, int k_in, int k_out, double* out_rank,
                                  float* out_scores, int64_t* out_ids, int32_t* out_count,
                                  hipStream_t stream) {
  ARMI_REQUIRE(n_shards >= 1 && k_in >= 1 && k_out >= 1,
               "armi_topk_merge_shards_packed: bad sizes");
  ARMI_REQUIRE((int64_t)n_shards * k_in <= kMaxPool,
               "armi_topk_merge_shards_packed: n_shards * k_in must be <= 4096");
  if (n_queries <= 0) return ARMI_OK;
  ARMI_REQUIRE(packed && out_rank && out_scores && out_ids && out_count,
               "armi_topk_merge_shards_packed: null pointer argument");
  const uintptr_t base = reinterpret_cast<uintptr_t>(packed);
  ARMI_REQUIRE((base + off_rank) % 8 == 0 && (base + off_ids) % 8 == 0 &&
                   (base + off_scores) % 4 == 0 && (base + off_count) % 4 == 0 &&
                   query_stride % 8 == 0 && shard_stride % 8 == 0,
               "armi_topk_merge_shards_packed: fields and strides must be naturally aligned "
               "(8-byte rank / ids, 4-byte scores / count, strides multiples of 8)");
  const int pool2 = armi::pow2_at_least(n_shards * k_in);
  if (int rc = allow_lds(merge_lists_kernel, merge_lds_bytes(pool2))) return rc;
  const ListLayout lay{shard_stride, query_stride, shard_stride, query_stride, shard_stride,
                       query_stride};
  using B = const unsigned char*;
  B p = static_cast<B>(packed);
  merge_lists_kernel<<<dim3(n_queries), dim3(kMergeThreads), merge_lds_bytes(pool2), stream>>>(
      p + off_rank, p + off_scores, p + off_ids, p + off_count, lay, n_shards, k_in, pool2,
      nullptr, k_out, out_rank, out_scores, out_ids, out_count, nullptr, 0);
  ARMI_LAUNCHED("merge_lists_kernel(shards, packed)");
  return ARMI_OK;
}

}  // extern "C"
