// Non-GEMM ops of the XLM-RoBERTa cross-encoder that BGEReranker runs through
// sentence-transformers' CrossEncoder.predict (src/audio_rag/reranking/bge.py:119-123;
// model BAAI/bge-reranker-base, max_length=512 at bge.py:53; num_labels=1 => sigmoid).
// fp32 activations, row-major, one wave per row (widths up to 1024, rows up to 512 keys).
#include <cmath>
#include <limits>

#include "armi_common.h"

namespace {

constexpr int kMaxPerLane = 16;  // width <= 1024

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}

// LayerNorm of a row held as kMaxPerLane strided values per lane (two-pass mean / variance,
// as torch.nn.functional.layer_norm computes it).
template <typename OutT = float>
__device__ __forceinline__ void layernorm_row(float (&v)[kMaxPerLane], int width, int lane,
                                              const float* __restrict__ gamma,
                                              const float* __restrict__ beta, float eps,
                                              OutT* __restrict__ out) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i)
    if (lane + 64 * i < width) s += v[i];
  const float mean = wave_sum(s) / (float)width;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i)
    if (lane + 64 * i < width) {
      const float d = v[i] - mean;
      ss += d * d;
    }
  const float var = wave_sum(ss) / (float)width;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    if (c < width) out[c] = (OutT)((v[i] - mean) * rstd * gamma[c] + beta[c]);
  }
}

__global__ __launch_bounds__(256) void layernorm_residual_kernel(
    const float* __restrict__ x, const float* __restrict__ res, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ out, int64_t n_rows, int width, float eps) {
  const int64_t row = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const float* xr = x + row * width;
  const float* rr = res ? res + row * width : nullptr;
  float v[kMaxPerLane];
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    v[i] = 0.f;
    if (c < width) v[i] = xr[c] + (rr ? rr[c] : 0.f);
  }
  layernorm_row(v, width, lane, gamma, beta, eps, out + row * width);
}

// scores [n_seq][heads][L][L]; one wave per (seq, head, query row)
__global__ __launch_bounds__(256) void masked_softmax_kernel(float* __restrict__ scores,
                                                             const int32_t* __restrict__ mask,
                                                             int n_seq, int heads, int L,
                                                             float scale) {
  const int64_t row = (int64_t)blockIdx.x * 4 + armi::wave_id();
  const int64_t n_rows = (int64_t)n_seq * heads * L;
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const int seq = (int)(row / ((int64_t)heads * L));
  float* p = scores + row * L;
  const int32_t* m = mask + (int64_t)seq * L;
  constexpr int kMaxKeys = 512 / 64;
  float v[kMaxKeys];
  float mx = -std::numeric_limits<float>::infinity();
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    const int c = lane + 64 * i;
    v[i] = -std::numeric_limits<float>::infinity();
    if (c < L && m[c] != 0) v[i] = p[c] * scale;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < L && v[i] != -std::numeric_limits<float>::infinity()) ? expf(v[i] - mx) : 0.f;
    s += v[i];
  }
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.0f / s : 0.f;
#pragma unroll
  for (int i = 0; i < kMaxKeys; ++i) {
    const int c = lane + 64 * i;
    if (c < L) p[c] = v[i] * inv;
  }
}

__global__ __launch_bounds__(256) void bias_gelu_kernel(float* __restrict__ x,
                                                        const float* __restrict__ bias,
                                                        int64_t n, int width) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  float4* p = reinterpret_cast<float4*>(x + i4);
  float4 v = *p;
  float e[4] = {v.x, v.y, v.z, v.w};
  const int c0 = (int)(i4 % width);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float t = e[j] + (bias ? bias[c0 + j] : 0.f);
    e[j] = 0.5f * t * (1.0f + erff(t * 0.70710678118654752440f));
  }
  *p = make_float4(e[0], e[1], e[2], e[3]);
}

// XLM-R embeddings (transformers create_position_ids_from_input_ids): position id of token t is
// padding_idx + number of non-pad tokens in [0, t] for a non-pad token, padding_idx for a pad.
// T = float (fp32 tables) or _Float16 (the fp16 model's own tables, no fp32 copy; the sums are
// the same fp32 operations on the same values)
template <typename T, typename OutT>
__global__ __launch_bounds__(256) void embed_kernel(const int32_t* __restrict__ ids,
                                                    const T* __restrict__ word,
                                                    const T* __restrict__ pos,
                                                    const T* __restrict__ type0,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta,
                                                    OutT* __restrict__ out, int n_seq, int L,
                                                    int width, int pad_id, int vocab, int n_pos,
                                                    float eps) {
  const int64_t tok = (int64_t)blockIdx.x * 4 + armi::wave_id();
  if (tok >= (int64_t)n_seq * L) return;
  const int lane = threadIdx.x & 63;
  const int seq = (int)(tok / L);
  const int t = (int)(tok % L);
  const int32_t* row_ids = ids + (int64_t)seq * L;
  int count = 0;
  for (int c0 = 0; c0 <= t; c0 += 64) {
    const int c = c0 + lane;
    const bool nonpad = (c <= t) && (row_ids[c] != pad_id);
    count += __popcll(__ballot(nonpad));
  }
  int id = row_ids[t];
  int pid = (id != pad_id) ? pad_id + count : pad_id;
  if (id < 0 || id >= vocab) id = 3;  // <unk>
  pid = pid < n_pos ? pid : n_pos - 1;
  const T* w = word + (int64_t)id * width;
  const T* pp = pos + (int64_t)pid * width;
  float v[kMaxPerLane];
#pragma unroll
  for (int i = 0; i < kMaxPerLane; ++i) {
    const int c = lane + 64 * i;
    v[i] = 0.f;
    if (c < width) v[i] = (float)w[c] + (float)pp[c] + (float)type0[c];
  }
  layernorm_row(v, width, lane, gamma, beta, eps, out + tok * width);
}

// The fp16 embedding for widths that are multiples of 256 (XLM-R base 768, large 1024), round 5:
// workgroup = kEmbTok consecutive tokens of one sequence, one wave per token in turn. The
// position ids come from one count of the sequence's non-pad tokens before the chunk
// (__syncthreads_count over its ids) plus a ballot prefix inside it (embed_kernel recounted the
// sequence prefix per token: a chain of dependent loads per row); each lane owns four contiguous
// components per 256 (8-B loads and stores instead of one 2-B access per component), type0,
// gamma and beta stay in registers across the wave's tokens. Same fp32 arithmetic per component
// as embed_kernel ((word + pos) + type0, two-pass LayerNorm); the lane sums run over another
// component order, so the outputs agree to fp32 rounding of the statistics, not bitwise.
constexpr int kEmbTok = 32;
template <int NC>  // NC = width / 256
__global__ __launch_bounds__(256) void embed_seq_f16_kernel(
    const int32_t* __restrict__ ids, const _Float16* __restrict__ word,
    const _Float16* __restrict__ pos, const _Float16* __restrict__ type0,
    const float* __restrict__ gamma, const float* __restrict__ beta, _Float16* __restrict__ out,
    int L, int pad_id, int vocab, int n_pos, float eps) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  constexpr int width = 256 * NC;
  __shared__ int32_t pid_s[kEmbTok], id_s[kEmbTok];
  const int chunks = (L + kEmbTok - 1) / kEmbTok;
  const int seq = blockIdx.x / chunks;
  const int t0 = (blockIdx.x % chunks) * kEmbTok;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t* row_ids = ids + (int64_t)seq * L;
  int before = 0;  // non-pad tokens in [0, t0)
  for (int c = 0; c < t0; c += 256) {
    const int i = c + tid;
    before += __syncthreads_count(i < t0 && row_ids[i] != pad_id);
  }
  if (wave == 0) {
    const int t = t0 + lane;
    const int32_t id = (lane < kEmbTok && t < L) ? row_ids[t] : pad_id;
    const uint64_t nonpad = __ballot(lane < kEmbTok && t < L && id != pad_id);
    const int count = before + __popcll(nonpad & ((2ull << lane) - 1ull));  // [0, t]
    if (lane < kEmbTok) {
      int p = id != pad_id ? pad_id + count : pad_id;
      pid_s[lane] = p < n_pos ? p : n_pos - 1;
      id_s[lane] = (id < 0 || id >= vocab) ? 3 : id;  // <unk>
    }
  }
  __syncthreads();
  float ty[NC][4], ga[NC][4], be[NC][4];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = 256 * j + 4 * lane;
    const h4 tv = *reinterpret_cast<const h4*>(type0 + c);
    const float4 g4 = *reinterpret_cast<const float4*>(gamma + c);
    const float4 b4 = *reinterpret_cast<const float4*>(beta + c);
    ty[j][0] = (float)tv[0], ty[j][1] = (float)tv[1], ty[j][2] = (float)tv[2], ty[j][3] = (float)tv[3];
    ga[j][0] = g4.x, ga[j][1] = g4.y, ga[j][2] = g4.z, ga[j][3] = g4.w;
    be[j][0] = b4.x, be[j][1] = b4.y, be[j][2] = b4.z, be[j][3] = b4.w;
  }
  for (int k = wave; k < kEmbTok && t0 + k < L; k += 4) {
    const _Float16* w = word + (int64_t)id_s[k] * width;
    const _Float16* pp = pos + (int64_t)pid_s[k] * width;
    h4 wv[NC], pv[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      wv[j] = *reinterpret_cast<const h4*>(w + 256 * j + 4 * lane);
      pv[j] = *reinterpret_cast<const h4*>(pp + 256 * j + 4 * lane);
    }
    float v[NC][4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[j][e] = (float)wv[j][e] + (float)pv[j][e] + ty[j][e];
        s += v[j][e];
      }
    const float mean = wave_sum(s) / (float)width;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mean;
        ss += d * d;
      }
    const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)width + eps);
    _Float16* o = out + ((int64_t)seq * L + t0 + k) * width;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      h4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = (_Float16)((v[j][e] - mean) * rstd * ga[j][e] + be[j][e]);
      *reinterpret_cast<h4*>(o + 256 * j + 4 * lane) = r;
    }
  }
}

// Classification head on <s> (RobertaClassificationHead + sigmoid): h = tanh(W1 x0 + b1),
// logit = w2 . h + b2, out = sigmoid(logit). kHeadSeq sequences per workgroup, one thread per
// output feature (blockDim = width rounded up to 64): thread o walks the transposed dense weight
// W1^T [in][out] down its column (coalesced across the workgroup's threads, each weight read
// from L2 once per workgroup) against the kHeadSeq <s> rows broadcast from LDS as float4s, so
// every weight load feeds kHeadSeq fp32 FMAs. Then tanh, the out_proj products and one
// workgroup reduction per sequence. (Round 3's form, a wave reduction per output and sequence,
// took 1.23 ms per 1,280-pair forward.)
constexpr int kHeadSeq = 8;

__global__ __launch_bounds__(1024) void cls_head_kernel(const float* __restrict__ hidden,
                                                        const float* __restrict__ dense_wt,
                                                        const float* __restrict__ dense_b,
                                                        const float* __restrict__ out_w,
                                                        const float* __restrict__ out_b,
                                                        float* __restrict__ out, int n_seq, int L,
                                                        int width) {
  extern __shared__ __attribute__((aligned(16))) float sh[];  // [kHeadSeq][width] x0; red
  const int seq0 = blockIdx.x * kHeadSeq;
  const int nseq = min(kHeadSeq, n_seq - seq0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = armi::wave_id();
  const int n_waves = blockDim.x >> 6;
  float* xs = sh;
  float* red = sh + kHeadSeq * width;  // [kHeadSeq][n_waves]
  for (int e = tid; e < kHeadSeq * width; e += blockDim.x) {
    const int q = e / width, c = e - q * width;
    xs[e] = q < nseq ? hidden[(int64_t)(seq0 + q) * L * width + c] : 0.f;
  }
  __syncthreads();
  const int o = tid;
  const bool live = o < width;
  float acc[kHeadSeq];
#pragma unroll
  for (int q = 0; q < kHeadSeq; ++q) acc[q] = 0.f;
  if (live) {
    const float* wc = dense_wt + o;
    int c = 0;
    for (; c + 4 <= width; c += 4) {
      const float w0 = wc[(int64_t)c * width], w1 = wc[(int64_t)(c + 1) * width];
      const float w2 = wc[(int64_t)(c + 2) * width], w3 = wc[(int64_t)(c + 3) * width];
#pragma unroll
      for (int q = 0; q < kHeadSeq; ++q) {
        const float4 x = *reinterpret_cast<const float4*>(xs + q * width + c);
        acc[q] = fmaf(w0, x.x, acc[q]);
        acc[q] = fmaf(w1, x.y, acc[q]);
        acc[q] = fmaf(w2, x.z, acc[q]);
        acc[q] = fmaf(w3, x.w, acc[q]);
      }
    }
    for (; c < width; ++c) {
      const float w = wc[(int64_t)c * width];
#pragma unroll
      for (int q = 0; q < kHeadSeq; ++q) acc[q] = fmaf(w, xs[q * width + c], acc[q]);
    }
  }
  const float bo = live ? dense_b[o] : 0.f, wo = live ? out_w[o] : 0.f;
#pragma unroll
  for (int q = 0; q < kHeadSeq; ++q) {
    const float t = live ? wo * tanhf(acc[q] + bo) : 0.f;
    const float ws = wave_sum(t);
    if (lane == 0) red[q * n_waves + wave] = ws;
  }
  __syncthreads();
  if (tid < nseq) {
    float logit = out_b[0];
    for (int w = 0; w < n_waves; ++w) logit += red[tid * n_waves + w];
    out[seq0 + tid] = 1.0f / (1.0f + expf(-logit));
  }
}

}  // namespace

extern "C" {

int armi_enc_layernorm_residual(const float* x, const float* res, const float* gamma,
                                const float* beta, float* out, int64_t n_rows, int width,
                                float eps, hipStream_t stream) {
  ARMI_REQUIRE(width >= 1 && width <= 64 * kMaxPerLane, "layernorm: width must be in [1, 1024]");
  if (n_rows <= 0) return ARMI_OK;
  ARMI_REQUIRE(x && gamma && beta && out, "layernorm: null pointer argument");
  layernorm_residual_kernel<<<dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, stream>>>(
      x, res, gamma, beta, out, n_rows, width, eps);
  ARMI_LAUNCHED("layernorm_residual_kernel");
  return ARMI_OK;
}

int armi_enc_masked_softmax(float* scores, const int32_t* mask, int n_seq, int heads, int L,
                            float scale, hipStream_t stream) {
  ARMI_REQUIRE(L >= 1 && L <= 512, "masked_softmax: L must be in [1, 512]");
  if (n_seq <= 0 || heads <= 0) return ARMI_OK;
  ARMI_REQUIRE(scores && mask, "masked_softmax: null pointer argument");
  const int64_t rows = (int64_t)n_seq * heads * L;
  masked_softmax_kernel<<<dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream>>>(
      scores, mask, n_seq, heads, L, scale);
  ARMI_LAUNCHED("masked_softmax_kernel");
  return ARMI_OK;
}

int armi_enc_bias_gelu(float* x, const float* bias, int64_t n_rows, int width,
                       hipStream_t stream) {
  ARMI_REQUIRE(width >= 4 && width % 4 == 0, "bias_gelu: width must be a multiple of 4");
  if (n_rows <= 0) return ARMI_OK;
  ARMI_REQUIRE(x != nullptr, "bias_gelu: x is null");
  const int64_t n = n_rows * width;
  bias_gelu_kernel<<<dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, stream>>>(x, bias, n,
                                                                                     width);
  ARMI_LAUNCHED("bias_gelu_kernel");
  return ARMI_OK;
}

int armi_enc_embed(const int32_t* ids, const float* word, const float* pos, const float* type0,
                   const float* gamma, const float* beta, float* out, int n_seq, int L,
                   int width, int pad_id, int vocab, int n_pos, float eps, hipStream_t stream) {
  ARMI_REQUIRE(width >= 1 && width <= 64 * kMaxPerLane, "embed: width must be in [1, 1024]");
  ARMI_REQUIRE(vocab > 3 && n_pos > pad_id + 1 && pad_id >= 0, "embed: bad vocab / n_pos / pad_id");
  ARMI_REQUIRE(L >= 1, "embed: L must be >= 1");
  if (n_seq <= 0) return ARMI_OK;
  ARMI_REQUIRE(ids && word && pos && type0 && gamma && beta && out,
               "embed: null pointer argument");
  const int64_t toks = (int64_t)n_seq * L;
  embed_kernel<float, float><<<dim3((unsigned)((toks + 3) / 4)), dim3(256), 0, stream>>>(
      ids, word, pos, type0, gamma, beta, out, n_seq, L, width, pad_id, vocab, n_pos, eps);
  ARMI_LAUNCHED("embed_kernel");
  return ARMI_OK;
}

int armi_enc_embed_f16(const int32_t* ids, const uint16_t* word, const uint16_t* pos,
                       const uint16_t* type0, const float* gamma, const float* beta, uint16_t* out,
                       int n_seq, int L, int width, int pad_id, int vocab, int n_pos, float eps,
                       hipStream_t stream) {
  ARMI_REQUIRE(width >= 1 && width <= 64 * kMaxPerLane, "embed_f16: width must be in [1, 1024]");
  ARMI_REQUIRE(vocab > 3 && n_pos > pad_id + 1 && pad_id >= 0,
               "embed_f16: bad vocab / n_pos / pad_id");
  ARMI_REQUIRE(L >= 1, "embed_f16: L must be >= 1");
  if (n_seq <= 0) return ARMI_OK;
  ARMI_REQUIRE(ids && word && pos && type0 && gamma && beta && out,
               "embed_f16: null pointer argument");
  const int64_t toks = (int64_t)n_seq * L;
  if (width % 256 == 0) {
    const int64_t blocks = (int64_t)n_seq * ((L + kEmbTok - 1) / kEmbTok);
    ARMI_REQUIRE(blocks < (int64_t(1) << 31), "embed_f16: too many sequences");
    auto* w16 = reinterpret_cast<const _Float16*>(word);
    auto* p16 = reinterpret_cast<const _Float16*>(pos);
    auto* t16 = reinterpret_cast<const _Float16*>(type0);
    auto* o16 = reinterpret_cast<_Float16*>(out);
    switch (width / 256) {
      case 1:
        embed_seq_f16_kernel<1><<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(
            ids, w16, p16, t16, gamma, beta, o16, L, pad_id, vocab, n_pos, eps);
        break;
      case 2:
        embed_seq_f16_kernel<2><<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(
            ids, w16, p16, t16, gamma, beta, o16, L, pad_id, vocab, n_pos, eps);
        break;
      case 3:
        embed_seq_f16_kernel<3><<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(
            ids, w16, p16, t16, gamma, beta, o16, L, pad_id, vocab, n_pos, eps);
        break;
      default:
        embed_seq_f16_kernel<4><<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(
            ids, w16, p16, t16, gamma, beta, o16, L, pad_id, vocab, n_pos, eps);
        break;
    }
    ARMI_LAUNCHED("embed_seq_f16_kernel");
    return ARMI_OK;
  }
  embed_kernel<_Float16, _Float16><<<dim3((unsigned)((toks + 3) / 4)), dim3(256), 0, stream>>>(
      ids, reinterpret_cast<const _Float16*>(word), reinterpret_cast<const _Float16*>(pos),
      reinterpret_cast<const _Float16*>(type0), gamma, beta, reinterpret_cast<_Float16*>(out),
      n_seq, L, width, pad_id, vocab, n_pos, eps);
  ARMI_LAUNCHED("embed_kernel");
  return ARMI_OK;
}

int armi_enc_cls_head_sigmoid(const float* hidden, const float* dense_wt, const float* dense_b,
                              const float* out_w, const float* out_b, float* out, int n_seq,
                              int L, int width, hipStream_t stream) {
  ARMI_REQUIRE(width >= 4 && width <= 1024 && width % 4 == 0,
               "cls_head: width must be a multiple of 4 in [4, 1024]");
  if (n_seq <= 0) return ARMI_OK;
  ARMI_REQUIRE(hidden && dense_wt && dense_b && out_w && out_b && out,
               "cls_head: null pointer argument");
  const int threads = (width + 63) / 64 * 64;
  const size_t lds = ((size_t)kHeadSeq * width + (size_t)kHeadSeq * (threads / 64)) * sizeof(float);
  if (int rc = armi::allow_lds(cls_head_kernel,
                               ((size_t)kHeadSeq * 1024 + kHeadSeq * 16) * sizeof(float)))
    return rc;
  cls_head_kernel<<<dim3((n_seq + kHeadSeq - 1) / kHeadSeq), dim3(threads), lds, stream>>>(
      hidden, dense_wt, dense_b, out_w, out_b, out, n_seq, L, width);
  ARMI_LAUNCHED("cls_head_kernel");
  return ARMI_OK;
}

}  // extern "C"
