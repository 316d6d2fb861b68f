// fp16 linear layers of the XLM-RoBERTa cross-encoder with fused epilogues (gfx950).
//
// Replaces the nn.Linear calls of XLMRobertaLayer that sentence-transformers' CrossEncoder runs
// for BGEReranker (src/audio_rag/reranking/bge.py:119-123): out = x . W^T + b, and for the FFN's
// intermediate dense the exact-erf GELU of XLMRobertaIntermediate fused into the GEMM epilogue,
// so the [tokens][3072] activation is written once (fp16) instead of written, read and written
// again by a separate GELU pass.
//
// Operands (row-major fp16 bit patterns, nn.Linear layout): x [m][k], w [n][k] (both K-contiguous),
// bias [n] fp32, out [m][n] fp16. n % 256 == 0, k % 64 == 0.
//
// Kernel (persistent, one 512-thread workgroup per CU, 128 KB LDS):
//   tile = 256 features (P = rows of w) x 256 tokens (Q = rows of x); D[p][q] = sum_k P[p][k] Q[q][k]
//   with v_mfma_f32_16x16x32_f16: lane (l & 15) holds row l & 15 of a 16-row block, 8 k values
//   8 (l >> 4) .. +7 of a 32-wide k-step for both operands; the accumulator register j of lane l
//   is D[p = 4 (l >> 4) + j][q = l & 15], i.e. four consecutive features of one token (8-byte
//   fp16 stores). 8 waves = 2 (features, 128 each) x 4 (tokens, 64 each): per wave 8 x 4 blocks
//   of 16 x 16 (128 fp32 accumulators).
//   K-tiles of 64, four phases each; phase = one quadrant (4 feature blocks x 2 token blocks) over
//   the whole K-tile (16 MFMAs), quadrant order (0,0) (0,1) (1,1) (1,0), so the fragment reads per
//   phase are 12 / 4 / 8 / 4 ds_read_b128. Each phase is a load segment (reads + one staged
//   half-tile), a barrier, the MFMA segment and a barrier; the two feature groups run one barrier
//   apart, so on every SIMD one wave multiplies while its partner loads (round 4).
//   Staging: global_load_lds_dwordx4 (LDS-DMA, 1 KB = 8 rows x 128 B per wave instruction) into two
//   64-KB buffers; each operand image is split into two "halves" (the rows its phases read:
//   feature half h = rows 64h..64h+63 and 128+64h..; token half h = rows 64 wq + 32h..+31), and one
//   half-tile (2 instructions per wave) is issued per phase: phase 0 feature half 1 of K-tile s+1,
//   phase 1 token half 0 of s+1, phase 2 feature half 0 of s+2, phase 3 token half 1 of s+2 -- each
//   half is restaged two phases after its last read, and lands >= 4 phases before it is read;
//   one counted s_waitcnt vmcnt(4) per K-tile, never 0 in steady state, raw
//   s_barrier (a __syncthreads would drain the DMA). 16-B chunk c of row r sits at chunk
//   c ^ (r & 7) (swizzle applied to the global source address), so every ds_read_b128 lane group
//   hits 16 distinct bank slots.
//   The K-tile stream runs across the workgroup's tiles: the next tile's first K-tiles are in
//   flight while a tile's epilogue (bias [+ GELU], fp16 stores) runs.
#include <cmath>

#include "armi_common.h"

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kT = 256;                 // tile rows of each operand
constexpr int kBK = 64;                 // K per K-tile
constexpr int kThreads = 512;
constexpr int kImg = kT * kBK * 2;      // one operand image (32 KB)
constexpr int kBuf = 2 * kImg;          // P + Q images of one K-tile (64 KB)
constexpr int kBias = 2 * kBuf;         // two 1-KB bias slots (tile parity)
constexpr size_t kLds = 2 * kBuf + 2 * 1024;

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
  half2v v = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// Exact-erf GELU of XLMRobertaIntermediate, x Phi(x), for the GEMM epilogue: with z = |x| / sqrt 2
// and E = erfc(z) = t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) exp(-z^2), t = 1 / (1 + p z)
// (Abramowitz & Stegun 7.1.26, |erf error| <= 1.5e-7), Phi(x) = 1/2 + sign(x) (1/2 - E/2).
// 16 VALU slots per element (one v_rcp, one v_exp) against ~25 for 0.5 x (1 + erf_f32(x / sqrt 2))
// with both erf branches evaluated; GELU output error <= 4.7e-7 absolute over [-12, 12] in fp32
// (checked against float64 erf), far below the fp16 rounding of the stored value (2^-11 relative).
__device__ __forceinline__ float gelu_erf(float x) {
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(x), 0.2316419f, 1.0f));  // p / sqrt 2
  float h = fmaf(0.5307027145f, t, -0.7265760135f);  // a_i / 2
  h = fmaf(h, t, 0.7107068705f);
  h = fmaf(h, t, -0.142248368f);
  h = fmaf(h, t, 0.127414796f);
  const float e = __builtin_amdgcn_exp2f((x * x) * -0.72134752044448170368f);  // exp(-x^2 / 2)
  const float half_erfc = (t * h) * e;
  return x * fmaf(copysignf(1.0f, x), 0.5f - half_erfc, 0.5f);
}

// sources of one tile of a workgroup's stream (linear_f16_kernel)
struct TileSrc {
  const unsigned char* p;  // feature block of w (scalar base)
  const unsigned char* q;  // token block of x
  uint32_t oq[2][2];       // per-lane token row offsets [half][piece] (clamped for a partial block)
  int tp;                  // feature block index
  int64_t q0;              // first token row
};

template <int EPI>
__global__ __launch_bounds__(kThreads) void linear_f16_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, const float* __restrict__ bias,
    uint16_t* __restrict__ out, int64_t m, int n, int k, int n_tiles_p, int64_t n_tiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int wave = armi::wave_id();
  const int lane = tid & 63;
  const int wp = wave >> 2;  // feature group (128 rows)
  const int wq = wave & 3;   // token group (64 rows)
  const int nK = k / kBK;

  // workgroup -> tiles: slot s (XCD-major: the workgroups of one XCD take consecutive tiles, so a
  // token block's feature tiles share that XCD's L2), tiles s, s + G, s + 2G, ...
  const int G = gridDim.x;
  const int b = blockIdx.x;
  int slot;
  {
    const int q8 = G / 8, r8 = G % 8, xcd = b % 8;
    slot = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + b / 8;
  }
  const int64_t my_tiles = slot < n_tiles ? (n_tiles - 1 - slot) / G + 1 : 0;
  const int64_t total = my_tiles * nK;  // K-tiles of this workgroup's stream
  if (total == 0) return;

  // per-lane staging offsets (bytes, relative to the tile's first row, K-tile 0): piece i of a
  // half-tile = 8 rows; lane -> row base + (lane >> 3), logical chunk (lane & 7) ^ (lane >> 3)
  const int prow = lane >> 3;
  const int pchunk = (lane & 7) ^ prow;
  uint32_t offP[2][2];              // [half][piece of this wave]
  uint32_t dstP[2][2], dstQ[2][2];  // LDS byte offsets of the pieces inside an image
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * wave + j;
      const int bp = i < 8 ? 64 * h + 8 * i : 128 + 64 * h + 8 * (i - 8);
      const int bq = 64 * (i >> 2) + 32 * h + 8 * (i & 3);
      offP[h][j] = (uint32_t)((bp + prow) * k + 8 * pchunk) * 2u;
      dstP[h][j] = (uint32_t)bp * 128u;
      dstQ[h][j] = (uint32_t)bq * 128u;
    }

  // Tiles of the stream: the current one and the next one (K-tiles s + 1 and s + 2 of the stream
  // belong to one of the two: nK >= 2). Per tile: scalar bases of its operand blocks and, for a
  // partial token block, the per-lane row offsets clamped to the last row (rows past m are read
  // from row m - 1 and never stored).
  auto tile_src = [&](int64_t j) {
    TileSrc ts;
    const int64_t t = (int64_t)slot + j * G;
    const int tp = (int)(t % n_tiles_p);
    const int64_t q0 = (t / n_tiles_p) * kT;
    ts.tp = tp;
    ts.q0 = q0;
    ts.p = reinterpret_cast<const unsigned char*>(w + (size_t)tp * kT * k);
    ts.q = reinterpret_cast<const unsigned char*>(x + (size_t)q0 * k);
    const int64_t qlim = m - 1 - q0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int i = 2 * wave + jj;
        const int bq = 64 * (i >> 2) + 32 * h + 8 * (i & 3);
        const int64_t rq = bq + prow;
        const int row = (int)(rq < qlim ? rq : qlim);
        ts.oq[h][jj] = (uint32_t)((row * k + 8 * pchunk) * 2);
      }
    return ts;
  };
  TileSrc cur = tile_src(0), nxt = tile_src(1);
  // K-tile sidx = s + d of the stream (kt = K-tile of s within its tile): operand op, half h
  auto issue_half = [&](int64_t sidx, int kt_s, int d, int op, int h) {
    if (sidx >= total) return;  // uniform
    int kt2 = kt_s + d;
    const bool next = kt2 >= nK;
    kt2 -= next ? nK : 0;
    unsigned char* buf = smem + (sidx & 1) * kBuf + op * kImg;
    if (op == 0) {
      const unsigned char* src = (next ? nxt.p : cur.p) + kt2 * (kBK * 2);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        __builtin_amdgcn_global_load_lds(src + offP[h][jj], (lds_ptr_t)(buf + dstP[h][jj]), 16, 0,
                                         0);
    } else {
      const unsigned char* src = (next ? nxt.q : cur.q) + kt2 * (kBK * 2);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        __builtin_amdgcn_global_load_lds(src + (next ? nxt.oq[h][jj] : cur.oq[h][jj]),
                                         (lds_ptr_t)(buf + dstQ[h][jj]), 16, 0, 0);
    }
  };
  // bias of the tile j's features -> LDS slot j & 1 (one 1-KB LDS-DMA by wave 0); tp = its block
  auto issue_bias = [&](int64_t j, int tp) {
    if (wave == 0 && j < my_tiles)
      __builtin_amdgcn_global_load_lds(bias + tp * kT + 4 * lane,
                                       (lds_ptr_t)(smem + kBias + (j & 1) * 1024), 16, 0, 0);
  };

  // fragment addresses: row (l & 15) of a 16-row block, logical chunk 4 s + (l >> 4) at physical
  // chunk ^ (l & 7)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  const uint32_t co0 = (uint32_t)((((lane >> 4)) ^ (lane & 7)) << 4);
  const uint32_t co1 = co0 ^ 64u;
  const uint32_t rowP = (uint32_t)(128 * wp + (lane & 15)) * 128u;
  const uint32_t rowQ = (uint32_t)(64 * wq + (lane & 15)) * 128u + kImg;

  u32x4 pf[4][2];  // feature blocks of the current quadrant half x k-step
  u32x4 qf[2][2];  // token blocks of the current quadrant half x k-step
  auto read_p = [&](int par, int ph) {
    const uint32_t a0 = lds0 + par * kBuf + rowP + co0 + ph * 64 * 128;
    const uint32_t a1 = lds0 + par * kBuf + rowP + co1 + ph * 64 * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(pf[i][0]) : "v"(a0), "i"(i * 2048));
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(pf[i][1]) : "v"(a1), "i"(i * 2048));
    }
  };
  auto read_q = [&](int par, int qh) {
    const uint32_t a0 = lds0 + par * kBuf + rowQ + co0 + qh * 32 * 128;
    const uint32_t a1 = lds0 + par * kBuf + rowQ + co1 + qh * 32 * 128;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(qf[i][0]) : "v"(a0), "i"(i * 2048));
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(qf[i][1]) : "v"(a1), "i"(i * 2048));
    }
  };
  auto frags_ready = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(pf[0][0]), "+v"(pf[0][1]), "+v"(pf[1][0]), "+v"(pf[1][1]),
                   "+v"(pf[2][0]), "+v"(pf[2][1]), "+v"(pf[3][0]), "+v"(pf[3][1]),
                   "+v"(qf[0][0]), "+v"(qf[0][1]), "+v"(qf[1][0]), "+v"(qf[1][1])::"memory");
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto quadrant = [&](int ph, int qh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[4 * ph + i][2 * qh + jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
              __builtin_bit_cast(half8, pf[i][s]), __builtin_bit_cast(half8, qf[jj][s]),
              acc[4 * ph + i][2 * qh + jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // bias (+ GELU) and fp16 stores of tile j (= cur); the bias comes from LDS by an asm read (a
  // compiler-visible LDS read after the bias DMA would be preceded by a vmcnt(0) that drains the
  // next tile's staging). Stores are 16 B per lane: lane row g = lane >> 4 holds features
  // 4g..4g+3 of its token in two token blocks; one v_permlane16_swap per dword pair regroups them
  // so that row g stores features 8 (g >> 1)..+7 of token block 2 jp + (g & 1) (half the store
  // instructions of 8-B stores: the epilogue's store issue is its tail).
  const uint32_t bias_lane = lds0 + kBias + (uint32_t)(128 * wp + 4 * (lane >> 4)) * 4u;
  const int g16 = lane >> 4;
  auto epilogue = [&](int64_t j) {
    const bool full = cur.q0 + kT <= m;
    const int64_t qb = cur.q0 + 64 * wq + (lane & 15) + 16 * (g16 & 1);
    uint16_t* orow = out + (size_t)cur.tp * kT + 128 * wp + 8 * (g16 >> 1);
    const uint32_t ba = bias_lane + (uint32_t)(j & 1) * 1024u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f32x4 bv;
      asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(bv) : "v"(ba), "i"(i * 64) : "memory");
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        uint32_t pk[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int jj = 2 * jp + h;
          float v0 = acc[i][jj][0] + bv[0], v1 = acc[i][jj][1] + bv[1];
          float v2 = acc[i][jj][2] + bv[2], v3 = acc[i][jj][3] + bv[3];
          if constexpr (EPI == 1) {
            v0 = gelu_erf(v0);
            v1 = gelu_erf(v1);
            v2 = gelu_erf(v2);
            v3 = gelu_erf(v3);
          }
          pk[h][0] = pack_h2(v0, v1);
          pk[h][1] = pack_h2(v2, v3);
          acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
        const int64_t q = qb + 32 * jp;
        if (full || q < m)
          *reinterpret_cast<u32x4*>(orow + (size_t)q * n + 16 * i) =
              u32x4{(uint32_t)s0[0], (uint32_t)s1[0], (uint32_t)s0[1], (uint32_t)s1[1]};
      }
    }
  };

  // prologue: K-tile 0 whole, K-tile 1's feature half 0 and token half 1 (the phase-2/3 issues
  // of the K-tile before it), the first tile's bias
  issue_bias(0, cur.tp);
  issue_half(0, 0, 0, 0, 0);
  issue_half(0, 0, 0, 1, 0);
  issue_half(0, 0, 0, 1, 1);
  issue_half(0, 0, 0, 0, 1);
  issue_half(1, 0, 1, 0, 0);
  issue_half(1, 0, 1, 1, 1);
  if (total > 1) {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  // Phase = load segment (the quadrant's fragment reads + one staged half-tile) | s_barrier |
  // MFMA segment (16 MFMAs) | s_barrier. The feature group wp = 1 runs ONE barrier behind group 0
  // (the extra s_barrier below, balanced by group 0's after the loop): waves w and w + 4 share a
  // SIMD, so each SIMD pairs one wave's MFMA segment with its partner's load segment (or epilogue)
  // instead of both waves loading, then both multiplying.
  // LDS hazards under the one-barrier lag: a half-tile is restaged >= 2 phases after its last
  // read (WAR), and a K-tile is read >= 1 phase after the counted vmcnt that retires it, which
  // sits in phase 3's load segment before its first barrier (RAW); bias slot j & 1 is re-staged
  // at K-tile 1 of tile j - 1 + 2, long after epilogue(j - 2) read it.
  auto mfma_segment = [&](int ph, int qh) {
    __builtin_amdgcn_s_barrier();
    frags_ready();
    __builtin_amdgcn_sched_barrier(0);
    quadrant(ph, qh);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };
  if (wp == 1) __builtin_amdgcn_s_barrier();
  int64_t j = 0;   // tile of the stream
  int kt = 0;      // K-tile within the tile
  for (int64_t s = 0; s < total; ++s) {
    const int par = (int)(s & 1);
    // phase 0: quadrant (0, 0); K-tile s + 1's feature half 1
    read_p(par, 0);
    read_q(par, 0);
    issue_half(s + 1, kt, 1, 0, 1);
    if (kt == 1) issue_bias(j + 1, nxt.tp);  // slot (j+1)&1 was last read by epilogue(j-1)
    mfma_segment(0, 0);
    // phase 1: quadrant (0, 1); K-tile s + 1's token half 0
    read_q(par, 1);
    issue_half(s + 1, kt, 1, 1, 0);
    mfma_segment(0, 1);
    // phase 2: quadrant (1, 1); K-tile s + 2's feature half 0 (read last in phase 0)
    read_p(par, 1);
    issue_half(s + 2, kt, 2, 0, 0);
    mfma_segment(1, 1);
    // phase 3: quadrant (1, 0); K-tile s + 2's token half 1 (read last in phase 1); K-tile s + 1
    // complete (only s + 2's two halves, 4 pieces, may stay in flight)
    read_q(par, 0);
    issue_half(s + 2, kt, 2, 1, 1);
    if (s + 2 < total) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mfma_segment(1, 0);
    if (++kt == nK) {
      epilogue(j);
      kt = 0;
      ++j;
      cur = nxt;
      nxt = tile_src(j + 1);
    }
  }
  if (wp == 0) __builtin_amdgcn_s_barrier();
}


// out[m][n] = epi(x . w^T + bias) for a few token rows (the query encodes of BGE-M3,
// embeddings/xlmr_f16.py), where the GEMM is a weight stream: workgroup (j, b) owns output
// columns 16j .. 16j + 15 of token rows 32b .. 32b + 31 and its WAVES waves split K evenly; each
// wave runs v_mfma_f32_16x16x32_f16 over its slice with the weight rows read straight from HBM
// (lane l: column l & 15, k 8 (l >> 4) .. + 7 of each 32-step, i.e. 16 contiguous bytes of the
// [n][k] row), the token rows from L2; the partial tiles are summed in LDS in wave order (the
// same result every run), then bias (+ exact GELU) and the fp16 store. A row's arithmetic
// depends only on k (the wave split), never on m or on the other rows: a query encoded alone
// and inside a batch gets the same bits (round 5: the batched query encode uses this too).
template <int EPI, int STEPS, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void linear_small_m_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, const float* __restrict__ bias,
    uint16_t* __restrict__ out, int m, int n, int k) {
  __shared__ float part[WAVES][2][16][17];  // [wave][row tile][row][col] (+1: bank spread)
  x += (size_t)blockIdx.y * 32 * k;
  out += (size_t)blockIdx.y * 32 * n;
  m = min(m - 32 * (int)blockIdx.y, 32);
  const int wave = armi::wave_id();
  const int lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 16;
  const int kw = k / WAVES;
  const int kb = wave * kw;
  const int c = lane & 15, kq = 8 * (lane >> 4);
  const uint16_t* wp = w + (size_t)(n0 + c) * k + kb + kq;
  const uint16_t* xp0 = x + (size_t)c * k + kb + kq;
  const uint16_t* xp1 = x + (size_t)(c + 16) * k + kb + kq;
  const bool r0 = c < m, r1 = c + 16 < m, two = m > 16;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  auto step = [&](const u32x4& b, int s) {
    const u32x4 a0 = r0 ? *reinterpret_cast<const u32x4*>(xp0 + s) : u32x4{0u, 0u, 0u, 0u};
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a0),
                                                  __builtin_bit_cast(half8, b), acc0, 0, 0, 0);
    if (two) {
      const u32x4 a1 = r1 ? *reinterpret_cast<const u32x4*>(xp1 + s) : u32x4{0u, 0u, 0u, 0u};
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, a1),
                                                    __builtin_bit_cast(half8, b), acc1, 0, 0, 0);
    }
  };
  if constexpr (STEPS > 0) {
    // the slice's weight pieces (the HBM stream) all in flight before the first MFMA; the token
    // rows are L2 hits
    u32x4 b[STEPS];
#pragma unroll
    for (int i = 0; i < STEPS; ++i) b[i] = *reinterpret_cast<const u32x4*>(wp + 32 * i);
#pragma unroll
    for (int i = 0; i < STEPS; ++i) step(b[i], 32 * i);
  } else {
    for (int s = 0; s < kw; s += 32) step(*reinterpret_cast<const u32x4*>(wp + s), s);
  }
  // D layout of the 16x16 tile: lane l holds column l & 15, rows 4 (l >> 4) + j
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    part[wave][0][4 * (lane >> 4) + j][c] = acc0[j];
    part[wave][1][4 * (lane >> 4) + j][c] = acc1[j];
  }
  __syncthreads();
  const int t = threadIdx.x;  // output (tile, row, col) = (t >> 8, (t >> 4) & 15, t & 15)
  const int tile = t >> 8, row = 16 * tile + ((t >> 4) & 15), col = t & 15;
  if (t < 512 && row < m) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) v += part[q][tile][(t >> 4) & 15][col];
    v += bias[n0 + col];
    if (EPI == ARMI_EPI_BIAS_GELU) v = gelu_erf(v);
    out[(size_t)row * n + n0 + col] = __builtin_bit_cast(uint16_t, (_Float16)v);
  }
}



}  // namespace

extern "C" {

int armi_enc_linear_f16(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* out,
                        int64_t m, int n, int k, int epilogue, hipStream_t stream) {
  ARMI_REQUIRE(n >= 256 && n % 256 == 0, "enc_linear_f16: n must be a multiple of 256");
  ARMI_REQUIRE(k >= 128 && k % 64 == 0 && k <= 8192,
               "enc_linear_f16: k must be a multiple of 64 in [128, 8192]");
  ARMI_REQUIRE(epilogue == ARMI_EPI_BIAS || epilogue == ARMI_EPI_BIAS_GELU,
               "enc_linear_f16: unknown epilogue");
  if (m <= 0) return ARMI_OK;
  ARMI_REQUIRE(x && w && bias && out, "enc_linear_f16: null pointer argument");
  ARMI_REQUIRE((int64_t)kT * k * 2 < (int64_t(1) << 31) && (int64_t)n * k * 2 < (int64_t(1) << 32),
               "enc_linear_f16: operand too large for 32-bit tile offsets");
  const int n_tp = n / kT;
  const int64_t n_tq = (m + kT - 1) / kT;
  const int64_t n_tiles = n_tq * n_tp;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    ARMI_HIP(hipGetDevice(&dev));
    ARMI_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int grid = (int)std::min<int64_t>(n_tiles, cus);
  auto kern = epilogue == ARMI_EPI_BIAS_GELU ? linear_f16_kernel<1> : linear_f16_kernel<0>;
  if (int rc = armi::allow_lds(kern, kLds)) return rc;
  const int rc_l = armi::timed_kernel(ARMI_TIMING_ENCODER_GEMM, kern, dim3(grid), dim3(kThreads),
                                      kLds, stream, x, w, bias, out, m, n, k, n_tp, n_tiles);
  ARMI_LAUNCHED("linear_f16_kernel");
  return rc_l;
}


int armi_enc_linear_small_f16(const uint16_t* x, const uint16_t* w, const float* bias,
                              uint16_t* out, int m, int n, int k, int epilogue,
                              hipStream_t stream) {
  ARMI_REQUIRE(m >= 0 && m <= 32 * 65535, "enc_linear_small_f16: m must be in [0, 32 * 65535]");
  ARMI_REQUIRE(n >= 16 && n % 16 == 0, "enc_linear_small_f16: n must be a multiple of 16");
  ARMI_REQUIRE(k >= 256 && k % 256 == 0 && (int64_t)n * k < (int64_t(1) << 31),
               "enc_linear_small_f16: k must be a multiple of 256 (n * k < 2^31)");
  ARMI_REQUIRE(epilogue == ARMI_EPI_BIAS || epilogue == ARMI_EPI_BIAS_GELU,
               "enc_linear_small_f16: unknown epilogue");
  if (m == 0) return ARMI_OK;
  ARMI_REQUIRE(x && w && bias && out, "enc_linear_small_f16: null pointer argument");
  const bool g = epilogue == ARMI_EPI_BIAS_GELU;
  // K = 4096 / 3072 (the output dense: 64 or 48 workgroups for 8 or 6 MB of weights): 16 waves
  // per workgroup, twice the loads in flight per CU
  if (k == 4096 || k == 3072) {
    auto kern = k == 4096 ? (g ? linear_small_m_kernel<1, 8, 16> : linear_small_m_kernel<0, 8, 16>)
                          : (g ? linear_small_m_kernel<1, 6, 16> : linear_small_m_kernel<0, 6, 16>);
    kern<<<dim3(n / 16, (m + 31) / 32), dim3(1024), 0, stream>>>(x, w, bias, out, m, n, k);
    ARMI_LAUNCHED("linear_small_m_kernel");
    return ARMI_OK;
  }
  auto kern = k == 1024 ? (g ? linear_small_m_kernel<1, 4, 8> : linear_small_m_kernel<0, 4, 8>)
              : k == 768  ? (g ? linear_small_m_kernel<1, 3, 8> : linear_small_m_kernel<0, 3, 8>)
                          : (g ? linear_small_m_kernel<1, 0, 8> : linear_small_m_kernel<0, 0, 8>);
  kern<<<dim3(n / 16, (m + 31) / 32), dim3(512), 0, stream>>>(x, w, bias, out, m, n, k);
  ARMI_LAUNCHED("linear_small_m_kernel");
  return ARMI_OK;
}

}  // extern "C"
