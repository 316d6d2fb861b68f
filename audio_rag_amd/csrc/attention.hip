// Fused masked self-attention + fp16 glue kernels of the XLM-RoBERTa cross-encoder that
// BGEReranker runs through sentence-transformers' CrossEncoder.predict
// (src/audio_rag/reranking/bge.py:119-123; BAAI/bge-reranker-base: 12 heads x 64, L <= 512 at
// bge.py:53). Replaces the eager QK^T -> masked softmax -> PV of XLMRobertaSelfAttention, which
// materialises an fp32 [n, H, L, L] score tensor per layer (4 GB at 1280 pairs x L 256), with
// one pass that keeps K and V^T of a (sequence, head) in LDS and the scores in registers.
//
// Layout (row-major, fp16 bit patterns):
//   qkv  [n_seq][L][3][H][64]   the fused QKV projection output ([n*L][3*H*64])
//   mask [n_seq][L] int32       key mask (0 = padding key)
//   ctx  [n_seq][L][H][64]      attention output, already in the layout the output projection
//                               consumes ([n*L][H*64]); no permute/copy
//
// Per workgroup: one (sequence, head, block of 256 queries), 8 waves x 32 queries, so K and V of
// a (sequence, head) are read from HBM once for L <= 256.
//   S^T = K . Q^T with v_mfma_f32_32x32x16_f16 puts one query on each lane (16 of a 32-key block
//   per lane half): row max / row sum are in-lane plus one cross-half shuffle.
//   O^T = V^T . P^T takes the S^T accumulator (P^T after exp, packed to fp16) as its B operand
//   with no lane movement, and O^T keeps the query on the lane, so the online-softmax rescale of
//   O is an in-lane multiply: a single pass over the keys, one exp per score.
#include <cmath>
#include <limits>

#include "armi_common.h"

namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kDh = 64;           // head dim (XLM-R base and large)
constexpr int kQPerWave = 32;
constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kQPerWg = kQPerWave * kWaves;
constexpr int kKStride = kDh + 8;  // K row stride in halves (144 B: conflict-free b128 reads)
constexpr int kMaxL = 512;
// Probe builds only (ARMI_BUILD_FLAGS=-DARMI_ATT_ABL=n): 1 = stage K / V / Q but skip the
// softmax / P.V loop, 2 = skip the HBM loads (stage zeros) but compute, 0 = the product kernel
// (tools/probes/att_pmc.sh: at 1280 x 256 the product kernel takes the SUM of the two)
#ifndef ARMI_ATT_ABL
#define ARMI_ATT_ABL 0
#endif

__device__ __forceinline__ int vt_stride(int lp) { return lp + 4; }  // V^T row stride (halves)

__device__ __forceinline__ f32x16 mfma16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a),
                                                __builtin_bit_cast(half8, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
  half2v v = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// S^T block (32 keys x 32 queries) of key block kb: lane (r, h) gets keys (i&3)+8(i>>2)+4h of
// the block for query r in register i.
__device__ __forceinline__ f32x16 score_block(const uint16_t* __restrict__ ks, int kb, int r,
                                              int h, const u32x4 (&qf)[kDh / 16]) {
  f32x16 acc = {};
  const uint16_t* krow = ks + (kb * 32 + r) * kKStride + 8 * h;
#pragma unroll
  for (int t = 0; t < kDh / 16; ++t) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(krow + 16 * t);
    acc = mfma16(a, qf[t], acc);
  }
  return acc;
}

// maximumNumber: lowers to v_max3_f32 without the canonicalising v_max_f32 copies that fmaxf
// gets on MFMA results (no NaN reaches these maxima)
__device__ __forceinline__ float fmax2(float a, float b) {
  return __builtin_elementwise_maximumnum(a, b);
}

// max over the two lanes r and r + 32 (the two key halves of query r): one permlane32 swap
__device__ __forceinline__ float halves_max(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmax2(fmax2(x, __builtin_bit_cast(float, (uint32_t)sw[0])),
               __builtin_bit_cast(float, (uint32_t)sw[1]));
}

__device__ __forceinline__ float halves_sum(float x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, x);
  const auto sw = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  // lanes < 32: sw[1] is the partner; lanes >= 32: sw[0]
  return x + __builtin_bit_cast(float, (uint32_t)((threadIdx.x & 32) ? sw[0] : sw[1]));
}

// Online softmax of one wave's 32 queries over key blocks [0, kb_end) of the staged K / V^T
// images (the kernels' comment). Lane kb of live_v holds block kb's live-key bits (bit j = key
// 32 kb + j is unmasked; read with v_readlane, no LDS round trip per block); a block
// with no live key is skipped, a full block needs no masking.
// Per block the VALU work is kept to what the math needs: the block maximum on the raw scores
// (8 v_max3 + one permlane32 swap), p = exp2(s * c - m * c) as one FMA + one v_exp, the row-sum
// adds and 8 packs. The running maximum m is only raised when a score exceeds it by more than
// 2^kRescaleLog2 in P (deferred rescale, cdna_hip_programming.md T13; the decision is taken
// before this block's P is formed and after the previous block's P.V, so O, l and P always share
// one m): P stays <= 2^8, well inside fp16, and the O / l rescale runs on the rare blocks that
// raise m instead of every block. Returns O^T (unnormalised) and this lane half's row sum.
constexpr float kRescaleLog2 = 8.f;

__device__ __forceinline__ float addf(float a, float b) {
  float d;  // (asm: keeps the row sums single adds; -O3 SLP-packs them into v_pk_add_f32, which
            // costs more than two v_add_f32 beside MFMAs, MI355X_MICROARCH.md constants table)
  asm("v_add_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

// one key block of attend_keys: mask, deferred-rescale online softmax, P.V
__device__ __forceinline__ void attend_block(f32x16 acc, uint32_t lv, int kb, int h, float c,
                                             float thr, const uint16_t* __restrict__ v0,
                                             const uint16_t* __restrict__ v1, float& m, float& mc,
                                             float& l, f32x16& o0, f32x16& o1) {
  if (lv == 0u) return;  // workgroup-uniform: every key of the block is padding
  if (lv != ~0u) {
    const uint32_t lh = lv >> (4 * h);  // this lane half's keys at bits (i & 3) + 8 (i >> 2)
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (!(lh & (1u << ((i & 3) + 8 * (i >> 2))))) acc[i] = -INFINITY;
  }
  float m5[5];
#pragma unroll
  for (int g = 0; g < 5; ++g) m5[g] = fmax2(fmax2(acc[3 * g], acc[3 * g + 1]), acc[3 * g + 2]);
  const float t0 = fmax2(fmax2(m5[0], m5[1]), m5[2]);
  const float t1 = fmax2(fmax2(m5[3], m5[4]), acc[15]);
  const float bm = halves_max(fmax2(t0, t1));
  if (__builtin_amdgcn_ballot_w64(bm > m + thr)) {  // wave-uniform
    const float mn = fmax2(m, bm);
    const float alpha = __builtin_amdgcn_exp2f((m - mn) * c);  // 0 on the first live block
    o0 *= alpha;
    o1 *= alpha;
    l *= alpha;
    m = mn;
    mc = mn * c;
  }
  float p[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) p[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i], c, -mc));
  float s4[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) s4[g] = addf(addf(p[4 * g], p[4 * g + 1]), addf(p[4 * g + 2], p[4 * g + 3]));
  l = addf(l, addf(addf(s4[0], s4[1]), addf(s4[2], s4[3])));
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    // B fragment of k-step st: registers 8st..8st+7 = keys 16st + 8(j>>2) + 4h + (j&3)
    u32x4 pb;
    pb[0] = pack_h2(p[8 * st + 0], p[8 * st + 1]);
    pb[1] = pack_h2(p[8 * st + 2], p[8 * st + 3]);
    pb[2] = pack_h2(p[8 * st + 4], p[8 * st + 5]);
    pb[3] = pack_h2(p[8 * st + 6], p[8 * st + 7]);
    const int key0 = kb * 32 + 16 * st;
    const u32x2 a0 = *reinterpret_cast<const u32x2*>(v0 + key0);
    const u32x2 a1 = *reinterpret_cast<const u32x2*>(v0 + key0 + 8);
    const u32x2 b0 = *reinterpret_cast<const u32x2*>(v1 + key0);
    const u32x2 b1 = *reinterpret_cast<const u32x2*>(v1 + key0 + 8);
    o0 = mfma16(u32x4{a0[0], a0[1], a1[0], a1[1]}, pb, o0);
    o1 = mfma16(u32x4{b0[0], b0[1], b1[0], b1[1]}, pb, o1);
  }
}

__device__ __forceinline__ void attend_keys(const uint16_t* __restrict__ ks,
                                            const uint16_t* __restrict__ vt, int vts,
                                            uint32_t live_v, int kb_end, int r,
                                            int h, const u32x4 (&qf)[kDh / 16], float c,
                                            f32x16& o0, f32x16& o1, float& l) {
  const float thr = kRescaleLog2 / c;  // the threshold in raw score units
  float m = -INFINITY, mc = 0.f;       // running max (raw units) and m * c
  l = 0.f;
  o0 = f32x16{};
  o1 = f32x16{};
  const uint16_t* v0 = vt + r * vts + 4 * h;
  const uint16_t* v1 = vt + (32 + r) * vts + 4 * h;
  // two named score buffers, blocks taken in pairs: S^T of the next block is issued before this
  // block's softmax (its MFMAs run under that VALU work) with no register rotation
  f32x16 sa = score_block(ks, 0, r, h, qf), sb;
  for (int kb = 0; kb < kb_end; kb += 2) {
    if (kb + 1 < kb_end) sb = score_block(ks, kb + 1, r, h, qf);
    attend_block(sa, __builtin_amdgcn_readlane(live_v, kb), kb, h, c, thr, v0, v1, m, mc, l, o0, o1);
    if (kb + 1 >= kb_end) break;
    if (kb + 2 < kb_end) sa = score_block(ks, kb + 2, r, h, qf);
    attend_block(sb, __builtin_amdgcn_readlane(live_v, kb + 1), kb + 1, h, c, thr, v0, v1, m, mc, l,
                 o0, o1);
  }
}

// Lane i < nkb of the result holds block i's live-key bits; *kb_end = one past the last block
// holding a live key (workgroup-uniform; 0 when every key is padding).
__device__ __forceinline__ uint32_t live_lanes(const uint32_t* live, int nkb, int& kb_end) {
  const int lane = threadIdx.x & 63;
  const uint32_t v = lane < nkb ? live[lane] : 0u;
  const uint64_t nz = __builtin_amdgcn_ballot_w64(v != 0u);
  kb_end = nz ? 64 - __builtin_clzll(nz) : 0;
  return v;
}

__global__ __launch_bounds__(kThreads, 4) void attention_f16_kernel(
    const uint16_t* __restrict__ qkv, const int32_t* __restrict__ mask, uint16_t* __restrict__ ctx,
    int L, int heads, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lp = (L + 31) & ~31;
  const int vts = vt_stride(lp);
  uint16_t* ks = reinterpret_cast<uint16_t*>(smem);               // [lp][kKStride]
  uint16_t* vt = ks + lp * kKStride;                               // [kDh][vts]
  uint32_t* live = reinterpret_cast<uint32_t*>(vt + kDh * vts);   // [lp / 32] live-key bits

  const int qblk = blockIdx.x;
  const int head = blockIdx.y;
  const int seq = blockIdx.z;
  const int tid = threadIdx.x;
  const int row_stride = 3 * heads * kDh;  // halves between consecutive tokens
  const uint16_t* base = qkv + (size_t)seq * L * row_stride + head * kDh;

  const int wave = armi::wave_id();
  const int lane = tid & 63;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int qw0 = qblk * kQPerWg + wave * kQPerWave;
  const int q = qw0 + r;
  // The Q fragments and every K / V load of a 256-key round are issued before the first LDS
  // store, so a workgroup waits for HBM once per round instead of once per load.
  u32x4 qf[kDh / 16];
#pragma unroll
  for (int t = 0; t < kDh / 16; ++t) {
    qf[t] = u32x4{0u, 0u, 0u, 0u};
    if (ARMI_ATT_ABL != 2 && q < L)
      qf[t] = *reinterpret_cast<const u32x4*>(base + (size_t)q * row_stride + 16 * t + 8 * h);
  }
  // Stage K (row-major) and V^T (two keys per 32-bit LDS word) of this (seq, head). Per round of
  // 256 keys thread tid loads K chunks e = tid + 512u (u < 4) and V key pairs e = tid + 512u
  // (u < 2): chunk e & 7 (8 halves) of key (pair) e >> 3.
  const uint16_t* kbase = base + heads * kDh;
  const uint16_t* vbase = base + 2 * heads * kDh;
  for (int j0 = 0; j0 < lp; j0 += 256) {
    u32x4 kv[4], va[2], vb[2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + kThreads * u;
      const int j = j0 + (e >> 3);
      kv[u] = u32x4{0u, 0u, 0u, 0u};
      if (ARMI_ATT_ABL != 2 && j < L)
        kv[u] = *reinterpret_cast<const u32x4*>(kbase + (size_t)j * row_stride + 8 * (e & 7));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + kThreads * u;
      const int j = j0 + 2 * (e >> 3);
      const uint16_t* vp = vbase + 8 * (e & 7);
      va[u] = u32x4{0u, 0u, 0u, 0u};
      vb[u] = u32x4{0u, 0u, 0u, 0u};
      if (ARMI_ATT_ABL != 2 && j < L) va[u] = *reinterpret_cast<const u32x4*>(vp + (size_t)j * row_stride);
      if (ARMI_ATT_ABL != 2 && j + 1 < L)
        vb[u] = *reinterpret_cast<const u32x4*>(vp + (size_t)(j + 1) * row_stride);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + kThreads * u;
      const int j = j0 + (e >> 3);
      if (j < lp) *reinterpret_cast<u32x4*>(ks + j * kKStride + 8 * (e & 7)) = kv[u];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + kThreads * u;
      const int j = j0 + 2 * (e >> 3);
      const int c = e & 7;
      if (j < lp) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t lo = (va[u][i] & 0xffffu) | (vb[u][i] << 16);
          const uint32_t hi = (va[u][i] >> 16) | (vb[u][i] & 0xffff0000u);
          *reinterpret_cast<uint32_t*>(vt + (8 * c + 2 * i) * vts + j) = lo;
          *reinterpret_cast<uint32_t*>(vt + (8 * c + 2 * i + 1) * vts + j) = hi;
        }
      }
    }
  }
  {  // key j = tid (L <= 512 = kThreads): one ballot per wave gives two blocks' live bits
    const bool lk = tid < L && mask[(size_t)seq * L + tid] != 0;
    const uint64_t bits = __builtin_amdgcn_ballot_w64(lk);
    if (lane == 0 && 64 * wave < lp) {
      live[2 * wave] = (uint32_t)bits;
      if (64 * wave + 32 < lp) live[2 * wave + 1] = (uint32_t)(bits >> 32);
    }
  }
  __syncthreads();
  if (qw0 >= L) return;  // wave-uniform: no query of this wave exists (after the only barrier)
  int kb_end;
  const uint32_t live_v = live_lanes(live, lp / 32, kb_end);

  // One pass, online softmax in the exp2 domain (s' = s * scale * log2 e). O is accumulated
  // transposed, O^T = V^T . P^T: the P^T accumulator of S^T is the B operand as it stands and
  // O^T's column (the query) is the lane, so the running max, sum and rescale are all in-lane.
  f32x16 o0, o1;
  float l;
  if (ARMI_ATT_ABL == 1) {
    o0 = f32x16{};
    o1 = f32x16{};
    l = 1.f;
  } else {
    attend_keys(ks, vt, vts, live_v, kb_end, r, h, qf, scale_log2, o0, o1, l);
  }
  l = halves_sum(l);  // both lane halves share the running max
  const float inv_l = l > 0.f ? 1.0f / l : 0.f;

  // lane (r, h) holds query r, dims 8g + 4h + (0..3) (o0) and 32 + those (o1): 8-byte stores
  if (q < L) {
    uint16_t* dst = ctx + ((size_t)seq * L + q) * (heads * kDh) + head * kDh + 4 * h;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u32x2 w0 = {pack_h2(o0[4 * g] * inv_l, o0[4 * g + 1] * inv_l),
                        pack_h2(o0[4 * g + 2] * inv_l, o0[4 * g + 3] * inv_l)};
      const u32x2 w1 = {pack_h2(o1[4 * g] * inv_l, o1[4 * g + 1] * inv_l),
                        pack_h2(o1[4 * g + 2] * inv_l, o1[4 * g + 3] * inv_l)};
      *reinterpret_cast<u32x2*>(dst + 8 * g) = w0;
      *reinterpret_cast<u32x2*>(dst + 32 + 8 * g) = w1;
    }
  }
}


// out = LayerNorm(x + res) (x fp16, res fp32 nullable) -> fp32 out and fp16 out16 (nullable).
constexpr int kMaxPerLane = 16;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__global__ __launch_bounds__(256) void layernorm_residual_f16_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ res, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ out, uint16_t* __restrict__ out16,
    int64_t n_rows, int width, float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const uint16_t* xr = x + row * width;
  const float* rr = res ? res + row * width : nullptr;
  float v[kMaxPerLane];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    v[i] = 0.f;
    if (c < width) {
      v[i] = (float)__builtin_bit_cast(_Float16, xr[c]) + (rr ? rr[c] : 0.f);
      s += v[i];
    }
  }
  const float mean = wave_sum(s) / (float)width;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i)
    if (lane + 64 * i < width) {
      const float d = v[i] - mean;
      ss += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)width + eps);
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    if (c < width) {
      const float y = (v[i] - mean) * rstd * gamma[c] + beta[c];
      out[row * width + c] = y;
      if (out16) out16[row * width + c] = __builtin_bit_cast(uint16_t, (_Float16)y);
    }
  }
}

// Vectorised form for width = 256 * CPL: lane owns elements 4c .. 4c+3 of chunks c = lane + 64 i,
// so every access is an 8-byte (fp16) or 16-byte (fp32) vector; same arithmetic as above.
template <int CPL>
__global__ __launch_bounds__(256) void layernorm_residual_f16_vec_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ res, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ out, uint16_t* __restrict__ out16,
    int64_t n_rows, float eps) {
  constexpr int W = 256 * CPL;
  const int64_t row = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  float v[CPL][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    const u32x2 xv = *reinterpret_cast<const u32x2*>(x + row * W + 4 * c);
    const half2v h0 = __builtin_bit_cast(half2v, (uint32_t)xv[0]);
    const half2v h1 = __builtin_bit_cast(half2v, (uint32_t)xv[1]);
    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (res) rv = *reinterpret_cast<const float4*>(res + row * W + 4 * c);
    v[i][0] = (float)h0[0] + rv.x;
    v[i][1] = (float)h0[1] + rv.y;
    v[i][2] = (float)h1[0] + rv.z;
    v[i][3] = (float)h1[1] + rv.w;
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mean = wave_sum(s) / (float)W;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      ss += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)W + eps);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    const float4 g = *reinterpret_cast<const float4*>(gamma + 4 * c);
    const float4 b = *reinterpret_cast<const float4*>(beta + 4 * c);
    const float4 y = make_float4((v[i][0] - mean) * rstd * g.x + b.x, (v[i][1] - mean) * rstd * g.y + b.y,
                                 (v[i][2] - mean) * rstd * g.z + b.z, (v[i][3] - mean) * rstd * g.w + b.w);
    *reinterpret_cast<float4*>(out + row * W + 4 * c) = y;
    if (out16)
      *reinterpret_cast<u32x2*>(out16 + row * W + 4 * c) = u32x2{pack_h2(y.x, y.y), pack_h2(y.z, y.w)};
  }
}

// out16 = LayerNorm(x16 + res16): the all-fp16 residual stream variant (statistics in fp32),
// width = 256 * CPL; 6 bytes of HBM traffic per element instead of 12.
template <int CPL>
__global__ __launch_bounds__(256) void add_layernorm_f16_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
    const float* __restrict__ gamma, const float* __restrict__ beta, uint16_t* __restrict__ out16,
    int64_t n_rows, float eps) {
  constexpr int W = 256 * CPL;
  const int64_t row = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  float v[CPL][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    const u32x2 xv = *reinterpret_cast<const u32x2*>(x + row * W + 4 * c);
    const u32x2 rv = *reinterpret_cast<const u32x2*>(res + row * W + 4 * c);
#pragma unroll
    for (int w = 0; w < 2; ++w) {
      const uint32_t xw = xv[w], rw = rv[w];
      const half2v hx = __builtin_bit_cast(half2v, xw);
      const half2v hr = __builtin_bit_cast(half2v, rw);
      v[i][2 * w] = (float)hx[0] + (float)hr[0];
      v[i][2 * w + 1] = (float)hx[1] + (float)hr[1];
    }
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mean = wave_sum(s) / (float)W;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[i][e] - mean;
      ss += d * d;
    }
  const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)W + eps);
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    const float4 g = *reinterpret_cast<const float4*>(gamma + 4 * c);
    const float4 b = *reinterpret_cast<const float4*>(beta + 4 * c);
    *reinterpret_cast<u32x2*>(out16 + row * W + 4 * c) =
        u32x2{pack_h2((v[i][0] - mean) * rstd * g.x + b.x, (v[i][1] - mean) * rstd * g.y + b.y),
              pack_h2((v[i][2] - mean) * rstd * g.z + b.z, (v[i][3] - mean) * rstd * g.w + b.w)};
  }
}

// in-place exact-erf GELU of fp16 x (+ fp32 bias[col], nullable), computed in fp32
__global__ __launch_bounds__(256) void gelu_f16_kernel(uint16_t* __restrict__ x,
                                                       const float* __restrict__ bias, int64_t n,
                                                       int width) {
  const int64_t i8 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i8 >= n) return;
  u32x4 v = *reinterpret_cast<const u32x4*>(x + i8);
  const int c0 = (int)(i8 % width);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t word = v[w];  // (bit_cast of a vector-element lvalue miscompiles)
    const half2v hv = __builtin_bit_cast(half2v, word);
    float t0 = (float)hv[0] + (bias ? bias[c0 + 2 * w] : 0.f);
    float t1 = (float)hv[1] + (bias ? bias[c0 + 2 * w + 1] : 0.f);
    t0 = 0.5f * t0 * (1.0f + armi::erf_f32(t0 * 0.70710678118654752440f));
    t1 = 0.5f * t1 * (1.0f + armi::erf_f32(t1 * 0.70710678118654752440f));
    v[w] = pack_h2(t0, t1);
  }
  *reinterpret_cast<u32x4*>(x + i8) = v;
}

// Attention of one query token per sequence (the <s> token, position 0) over all its keys: the
// last encoder layer of the cross-encoder, whose only consumer is the classification head on the
// <s> row (XLMRobertaClassificationHead reads features[:, 0, :]), needs no other query row.
// One workgroup per (head, sequence), 4 waves. A key's 64 channels are 8 chunks of 16 B, so a wave
// covers 8 keys per load instruction (lane = key slot (lane >> 3) x chunk (lane & 7)): every load
// is a full 128-B line. Scores: chunk partial dots reduced over the 8 chunk lanes, masked softmax
// in fp32; P.V: each lane accumulates its chunk's 8 channels over its keys, then the key slots
// (shuffles) and the waves (LDS) are summed.
// Layout as attention_f16_kernel: qkv [n_seq][L][3][H][64]; ctx [n_seq][H][64] (= [n_seq][d]).
constexpr int kClsThreads = 256;
constexpr int kClsKeySlots = kClsThreads / 8;             // keys per round (8 lanes per key)
constexpr int kClsRounds = kMaxL / kClsKeySlots;          // rounds at L = kMaxL
__global__ __launch_bounds__(kClsThreads) void attention_cls_f16_kernel(
    const uint16_t* __restrict__ qkv, const int32_t* __restrict__ mask, uint16_t* __restrict__ ctx,
    int L, int heads, float scale) {
  __shared__ float p[kMaxL];
  __shared__ float red[kClsThreads / 64];
  __shared__ float part[kClsThreads / 64][kDh];
  const int head = blockIdx.x, seq = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int ch = lane & 7;                   // 16-B chunk: channels 8 ch .. 8 ch + 7
  const int slot = wave * 8 + (lane >> 3);   // key slot: keys slot, slot + 32, ...
  const int d3 = 3 * heads * kDh;
  const uint16_t* __restrict__ base = qkv + (size_t)seq * L * d3;
  float qv[8];
  {
    const half8 hq = __builtin_bit_cast(half8, *reinterpret_cast<const u32x4*>(
                                                   base + head * kDh + 8 * ch));
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[e] = (float)hq[e] * scale;
  }
  const int rounds = (L + kClsKeySlots - 1) / kClsKeySlots;
  // scores: all of this lane's K chunks in flight before any is used
  u32x4 kc[kClsRounds];
#pragma unroll
  for (int r = 0; r < kClsRounds; ++r) {
    const int j = slot + r * kClsKeySlots;
    if (r < rounds && j < L)
      kc[r] = *reinterpret_cast<const u32x4*>(base + (size_t)j * d3 + (heads + head) * kDh + 8 * ch);
  }
  float m = -INFINITY;
#pragma unroll
  for (int r = 0; r < kClsRounds; ++r) {
    const int j = slot + r * kClsKeySlots;
    float sc = 0.f;
    if (r < rounds && j < L) {
      const half8 hk = __builtin_bit_cast(half8, kc[r]);
#pragma unroll
      for (int e = 0; e < 8; ++e) sc += qv[e] * (float)hk[e];
    }
    sc += __shfl_xor(sc, 1);
    sc += __shfl_xor(sc, 2);
    sc += __shfl_xor(sc, 4);
    if (r < rounds && j < L) {
      sc = mask[(size_t)seq * L + j] != 0 ? sc : -INFINITY;
      if (ch == 0) p[j] = sc;
      m = fmaxf(m, sc);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();  // red is reused for the sum
  float sum = 0.f;
  for (int j = tid; j < L; j += kClsThreads) {
    const float e = p[j] == -INFINITY ? 0.f : expf(p[j] - m);
    p[j] = e;
    sum += e;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  const float total = red[0] + red[1] + red[2] + red[3];
  // P.V: this lane's chunk of its keys' V rows, all loads in flight first
  u32x4 vc[kClsRounds];
#pragma unroll
  for (int r = 0; r < kClsRounds; ++r) {
    const int j = slot + r * kClsKeySlots;
    if (r < rounds && j < L)
      vc[r] = *reinterpret_cast<const u32x4*>(base + (size_t)j * d3 + (2 * heads + head) * kDh +
                                              8 * ch);
  }
  float acc[8] = {};
#pragma unroll
  for (int r = 0; r < kClsRounds; ++r) {
    const int j = slot + r * kClsKeySlots;
    if (r < rounds && j < L) {
      const float w = p[j];
      const half8 hv = __builtin_bit_cast(half8, vc[r]);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += w * (float)hv[e];
    }
  }
#pragma unroll
  for (int off = 8; off < 64; off <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], off);
  if (lane < 8)
#pragma unroll
    for (int e = 0; e < 8; ++e) part[wave][8 * ch + e] = acc[e];
  __syncthreads();
  if (tid < kDh) {
    const float o = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    ctx[((size_t)seq * heads + head) * kDh + tid] =
        __builtin_bit_cast(uint16_t, (_Float16)(total > 0.f ? o / total : 0.f));
  }
}

size_t attention_lds_bytes(int L) {
  const int lp = (L + 31) & ~31;
  return (size_t)lp * kKStride * 2 + (size_t)kDh * (lp + 4) * 2 + (size_t)lp * 4;
}

}  // namespace

extern "C" {

int armi_enc_attention_f16(const uint16_t* qkv, const int32_t* mask, uint16_t* ctx, int n_seq,
                           int L, int heads, int head_dim, float scale, hipStream_t stream) {
  ARMI_REQUIRE(head_dim == kDh, "attention_f16: head_dim must be 64");
  ARMI_REQUIRE(L >= 1 && L <= kMaxL, "attention_f16: L must be in [1, 512]");
  ARMI_REQUIRE(heads >= 1 && heads <= 65535, "attention_f16: bad head count");
  if (n_seq <= 0) return ARMI_OK;
  ARMI_REQUIRE(n_seq <= 65535, "attention_f16: n_seq must be <= 65535 per call");
  ARMI_REQUIRE(qkv && mask && ctx, "attention_f16: null pointer argument");
  const size_t lds = attention_lds_bytes(L);
  // raise the dynamic-LDS limit once per device, to the largest L (not per call: keeps the
  // launch path free of non-stream runtime calls, so it can be captured in a HIP graph)
  if (int rc = armi::allow_lds(attention_f16_kernel, attention_lds_bytes(kMaxL))) return rc;
  const float scale_log2 = scale * 1.4426950408889634f;
  attention_f16_kernel<<<dim3((L + kQPerWg - 1) / kQPerWg, heads, n_seq), dim3(kThreads), lds,
                         stream>>>(qkv, mask, ctx, L, heads, scale_log2);
  ARMI_LAUNCHED("attention_f16_kernel");
  return ARMI_OK;
}

int armi_enc_attention_cls_f16(const uint16_t* qkv, const int32_t* mask, uint16_t* ctx,
                               int n_seq, int L, int heads, int head_dim, float scale,
                               hipStream_t stream) {
  ARMI_REQUIRE(head_dim == kDh, "attention_cls_f16: head_dim must be 64");
  ARMI_REQUIRE(L >= 1 && L <= kMaxL, "attention_cls_f16: L must be in [1, 512]");
  ARMI_REQUIRE(heads >= 1 && heads <= 65535, "attention_cls_f16: bad head count");
  if (n_seq <= 0) return ARMI_OK;
  ARMI_REQUIRE(n_seq <= 65535, "attention_cls_f16: n_seq must be <= 65535 per call");
  ARMI_REQUIRE(qkv && mask && ctx, "attention_cls_f16: null pointer argument");
  attention_cls_f16_kernel<<<dim3(heads, n_seq), dim3(kClsThreads), 0, stream>>>(qkv, mask, ctx,
                                                                                   L, heads, scale);
  ARMI_LAUNCHED("attention_cls_f16_kernel");
  return ARMI_OK;
}

int armi_enc_layernorm_residual_f16(const uint16_t* x, const float* res, const float* gamma,
                                    const float* beta, float* out, uint16_t* out16,
                                    int64_t n_rows, int width, float eps, hipStream_t stream) {
  ARMI_REQUIRE(width >= 1 && width <= 64 * kMaxPerLane,
               "layernorm_f16: width must be in [1, 1024]");
  if (n_rows <= 0) return ARMI_OK;
  ARMI_REQUIRE(x && gamma && beta && out, "layernorm_f16: null pointer argument");
  const dim3 grid((unsigned)((n_rows + 3) / 4));
  switch (width) {  // the XLM-R widths take the vectorised kernel
    case 768:
      layernorm_residual_f16_vec_kernel<3><<<grid, dim3(256), 0, stream>>>(x, res, gamma, beta,
                                                                          out, out16, n_rows, eps);
      break;
    case 1024:
      layernorm_residual_f16_vec_kernel<4><<<grid, dim3(256), 0, stream>>>(x, res, gamma, beta,
                                                                          out, out16, n_rows, eps);
      break;
    default:
      layernorm_residual_f16_kernel<<<grid, dim3(256), 0, stream>>>(x, res, gamma, beta, out,
                                                                    out16, n_rows, width, eps);
  }
  ARMI_LAUNCHED("layernorm_residual_f16_kernel");
  return ARMI_OK;
}

int armi_enc_add_layernorm_f16(const uint16_t* x, const uint16_t* res, const float* gamma,
                               const float* beta, uint16_t* out16, int64_t n_rows, int width,
                               float eps, hipStream_t stream) {
  ARMI_REQUIRE(width == 768 || width == 1024, "add_layernorm_f16: width must be 768 or 1024");
  if (n_rows <= 0) return ARMI_OK;
  ARMI_REQUIRE(x && res && gamma && beta && out16, "add_layernorm_f16: null pointer argument");
  const dim3 grid((unsigned)((n_rows + 3) / 4));
  if (width == 768)
    add_layernorm_f16_kernel<3><<<grid, dim3(256), 0, stream>>>(x, res, gamma, beta, out16, n_rows,
                                                                eps);
  else
    add_layernorm_f16_kernel<4><<<grid, dim3(256), 0, stream>>>(x, res, gamma, beta, out16, n_rows,
                                                                eps);
  ARMI_LAUNCHED("add_layernorm_f16_kernel");
  return ARMI_OK;
}

int armi_enc_gelu_f16(uint16_t* x, const float* bias, int64_t n_rows, int width,
                      hipStream_t stream) {
  ARMI_REQUIRE(width >= 8 && width % 8 == 0, "gelu_f16: width must be a multiple of 8");
  if (n_rows <= 0) return ARMI_OK;
  ARMI_REQUIRE(x != nullptr, "gelu_f16: x is null");
  const int64_t n = n_rows * width;
  gelu_f16_kernel<<<dim3((unsigned)((n / 8 + 255) / 256)), dim3(256), 0, stream>>>(x, bias, n,
                                                                                   width);
  ARMI_LAUNCHED("gelu_f16_kernel");
  return ARMI_OK;
}

}  // extern "C"
