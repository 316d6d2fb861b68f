// Shared host + device helpers of libarmi (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string>

#include "../../include/armi.h"

namespace armi {

// ----------------------------------------------------------------------------------- errors

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define ARMI_HIP(call)                                   \
  do {                                                   \
    hipError_t _e = (call);                              \
    if (_e != hipSuccess) return armi::hip_fail(_e, #call); \
  } while (0)

#define ARMI_LAUNCHED(what)                              \
  do {                                                   \
    hipError_t _e = hipGetLastError();                   \
    if (_e != hipSuccess) return armi::hip_fail(_e, what); \
  } while (0)

#define ARMI_REQUIRE(cond, msg)                          \
  do {                                                   \
    if (!(cond)) return armi::fail(ARMI_ERR_INVALID, msg); \
  } while (0)

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Live kernel timing (armi_scan_timing_enable / armi_kernel_timing_read): TimedLaunch brackets
// one launch on `stream` with a HIP event pair when timing is enabled, else costs nothing.
struct TimedLaunch {
  int slot = -1;
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipStream_t stream = nullptr;
  int begin(int slot, hipStream_t stream);  // 0 = not timed, 1 = timed, <0 = error (set)
  int end();
};

// One kernel's duration into a timing slot without marker packets around it: begin() hands out
// the slot's event pair when timing is on (ev[0] = ev[1] = nullptr when off), the caller passes
// them to hipExtLaunchKernelGGL, which binds them to the dispatch's own start / end timestamps,
// and commit() files them. (Two hipEventRecord markers per launch cost ~6 us of a 61-us step at
// 100k rows: each waits for the pipe to drain.)
struct TimedKernel {
  int slot = -1;
  hipEvent_t ev[2] = {nullptr, nullptr};
  // 0 = not timed (timing off, or the stream is being captured into a graph), 1 = timed,
  // <0 = error (set)
  int begin(int slot, hipStream_t stream);
  int commit();
};

// kern<<<grid, block, lds, stream>>>(args...), its duration filed under `slot` when timing is on
template <typename K, typename... Args>
int timed_kernel(int slot, K kern, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                 Args... args) {
  TimedKernel tk;
  const int on = tk.begin(slot, stream);
  if (on < 0) return ARMI_ERR_HIP;
  if (on)
    hipExtLaunchKernelGGL(kern, grid, block, (std::uint32_t)lds, stream, tk.ev[0], tk.ev[1], 0u,
                          args...);
  else
    kern<<<grid, block, lds, stream>>>(args...);
  return tk.commit();
}

// Raises a kernel's dynamic-LDS limit to `bytes` (> 64 KiB needs it) on the current device, once
// per (device, kernel): later searches issue stream work only (no runtime call per search, so the
// calls stay graph-capturable). The attribute is per device, hence the device in the key.
int allow_lds_raw(const void* kernel, size_t bytes);
template <typename K>
inline int allow_lds(K kernel, size_t bytes) {
  return allow_lds_raw(reinterpret_cast<const void*>(kernel), bytes);
}

// Carves consecutive 256-B aligned sub-buffers out of one caller workspace.
struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  template <typename T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
    off += count * sizeof(T);
    return p;
  }
};

// ------------------------------------------------------------------------------- numerics

// Exact integer image of an IEEE binary16 value: x * 2^24 (every finite fp16 is an integer
// multiple of 2^-24). Callers guarantee exponent field <= 15 (|x| < 2), so |result| < 2^25.
// Through fp32: the fp16 -> fp32 conversion is exact (subnormals included), x * 2^24 is an
// integer of at most 11 significant bits (exact in fp32) and the conversion to int32 exact:
// 3 instructions instead of the bit-field form's ~9 (every in-domain fp16 bit pattern checked
// against the bit-field form, the same integers).
__device__ __forceinline__ int32_t fp16_to_fixed24(uint32_t h) {
  const float x = (float)__builtin_bit_cast(_Float16, (uint16_t)(h & 0xffffu));
  return (int32_t)(x * 16777216.0f);
}

__device__ __forceinline__ bool fp16_in_domain(uint32_t h) { return ((h >> 10) & 31) <= 15; }

// Total order used by every dense ranking: key descending, then ordinal ascending.
// (bitwise, not short-circuit: the || / && form compiled to exec-mask branches inside the wave
// sorts, one waited shuffle at a time; round-3 ISA of dense_scan_i8_kernel's workgroup merge)
__device__ __forceinline__ bool rank_better(double ka, int64_t ia, double kb, int64_t ib) {
  return (ka > kb) | ((ka == kb) & (ia < ib));
}
__device__ __forceinline__ bool approx_better(float ka, int32_t ia, float kb, int32_t ib) {
  return (ka > kb) | ((ka == kb) & (ia < ib));
}

// Lane l reads lane l ^ S, without the LDS pipe (ds_bpermute): S = 1, 2 one DPP quad
// permutation, 4 a half-row mirror then a quad reversal ((l ^ 7) ^ 3), 8 a row rotation by 8,
// 16 / 32 one v_permlane16/32_swap of the value with itself (the swapped row of the other half)
// and a select.
#ifndef ARMI_SORT_DPP
#define ARMI_SORT_DPP 1  // 0: ds_bpermute (__shfl_xor) as before round 4 (r04ai: 100k step -2 %)
#endif
template <int S>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  static_assert(S == 1 || S == 2 || S == 4 || S == 8 || S == 16 || S == 32, "lane xor");
  if constexpr (S == 1) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  } else if constexpr (S == 2) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  } else if constexpr (S == 4) {
    const int t = __builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, t, 0x1B, 0xF, 0xF, false);
  } else if constexpr (S == 8) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
  } else if constexpr (S == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? (uint32_t)p[0] : (uint32_t)p[1];
  } else {
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? (uint32_t)p[0] : (uint32_t)p[1];
  }
}

// v of lane l ^ stride for any 4- or 8-byte type (stride: a compile-time constant after the
// sorts' full unrolling, so the switch folds)
template <typename T>
__device__ __forceinline__ T xor_stride(T v, int stride) {
#if ARMI_SORT_DPP
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte lane values");
  auto one = [&](uint32_t u) -> uint32_t {
    switch (stride) {
      case 1: return xor_lane<1>(u);
      case 2: return xor_lane<2>(u);
      case 4: return xor_lane<4>(u);
      case 8: return xor_lane<8>(u);
      case 16: return xor_lane<16>(u);
      default: return xor_lane<32>(u);
    }
  };
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, one(__builtin_bit_cast(uint32_t, v)));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t lo = one((uint32_t)u), hi = one((uint32_t)(u >> 32));
    return __builtin_bit_cast(T, lo | (hi << 32));
  }
#else
  return __shfl_xor(v, stride);
#endif
}

// In-LDS bitonic sort of n (power of two) entries into descending rank order, executed by the
// whole workgroup. Entries: (double key, int64 ordinal).
__device__ inline void lds_sort_rank_desc(double* key, int64_t* ord, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = threadIdx.x; t < n / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const double klo = key[lo], khi = key[hi];
        const int64_t olo = ord[lo], ohi = ord[hi];
        const bool hi_better = rank_better(khi, ohi, klo, olo);
        if (hi_better == desc) {
          key[lo] = khi; key[hi] = klo;
          ord[lo] = ohi; ord[hi] = olo;
        }
      }
    }
  }
  __syncthreads();
}

// Same for (float approx key, int32 row) entries.
__device__ inline void lds_sort_approx_desc(float* key, int32_t* row, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int t = threadIdx.x; t < n / 2; t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const float klo = key[lo], khi = key[hi];
        const int32_t rlo = row[lo], rhi = row[hi];
        const bool hi_better = approx_better(khi, rhi, klo, rlo);
        if (hi_better == desc) {
          key[lo] = khi; key[hi] = klo;
          row[lo] = rhi; row[hi] = rlo;
        }
      }
    }
  }
  __syncthreads();
}

// Wave-level (64 lanes) bitonic sort, one entry per lane, descending by (key, row asc).
__device__ __forceinline__ void wave_sort_approx_desc(float& key, int32_t& row) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float ok = xor_stride(key, stride);
      const int32_t orow = xor_stride(row, stride);
      const bool lower = (lane & stride) == 0;
      const bool desc = (lane & size) == 0;
      const bool other_better = approx_better(ok, orow, key, row);
      // lower lane of a descending pair keeps the better entry (selects, no branch)
      const bool take_other = other_better ^ (lower != desc);
      key = take_other ? ok : key;
      row = take_other ? orow : row;
    }
  }
}

// Wave-level bitonic sort of (double key, int64 ordinal), one entry per lane, into descending
// rank order (key desc, ordinal asc).
__device__ __forceinline__ void wave_sort_rank_desc(double& key, int64_t& ord) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const double ok = xor_stride(key, stride);
      const int64_t oo = xor_stride(ord, stride);
      const bool lower = (lane & stride) == 0;
      const bool desc = (lane & size) == 0;
      const bool other_better = rank_better(ok, oo, key, ord);
      const bool take_other = other_better ^ (lower != desc);
      key = take_other ? ok : key;
      ord = take_other ? oo : ord;
    }
  }
}

template <int S, int N>
__device__ __forceinline__ void xor_exchange_n(const float (&key)[N], const int32_t (&row)[N],
                                               float (&ok)[N], int32_t (&orow)[N]) {
#pragma unroll
  for (int n = 0; n < N; ++n) {
#if ARMI_SORT_DPP
    ok[n] = __uint_as_float(xor_lane<S>(__float_as_uint(key[n])));
    orow[n] = (int32_t)xor_lane<S>((uint32_t)row[n]);
#else
    ok[n] = __shfl_xor(key[n], S);
    orow[n] = __shfl_xor(row[n], S);
#endif
  }
}

// b[n] = max over the wave of b[n], for N values at once (all lanes get it).
template <int N>
__device__ __forceinline__ void wave_max_all_n(float (&b)[N]) {
#if ARMI_SORT_DPP
#define ARMI_MAX_STEP(S)                                                                    \
  _Pragma("unroll") for (int n = 0; n < N; ++n)                                            \
      b[n] = fmaxf(b[n], __uint_as_float(xor_lane<S>(__float_as_uint(b[n]))));
  ARMI_MAX_STEP(32) ARMI_MAX_STEP(16) ARMI_MAX_STEP(8) ARMI_MAX_STEP(4) ARMI_MAX_STEP(2)
  ARMI_MAX_STEP(1)
#undef ARMI_MAX_STEP
#else
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int n = 0; n < N; ++n) b[n] = fmaxf(b[n], __shfl_xor(b[n], off));
#endif
}

// N independent wave sorts at once: every stage issues all N lists' shuffles before using any,
// so the N dependent shuffle chains overlap instead of running back to back.
template <int N>
__device__ __forceinline__ void wave_sort_approx_desc_n(float (&key)[N], int32_t (&row)[N]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      float ok[N];
      int32_t orow[N];
      switch (stride) {  // (unrolled: one case per stage)
        case 1: xor_exchange_n<1>(key, row, ok, orow); break;
        case 2: xor_exchange_n<2>(key, row, ok, orow); break;
        case 4: xor_exchange_n<4>(key, row, ok, orow); break;
        case 8: xor_exchange_n<8>(key, row, ok, orow); break;
        case 16: xor_exchange_n<16>(key, row, ok, orow); break;
        default: xor_exchange_n<32>(key, row, ok, orow); break;
      }
      const bool lower = (lane & stride) == 0;
      const bool desc = (lane & size) == 0;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        const bool other_better = approx_better(ok[n], orow[n], key[n], row[n]);
        const bool take_other = other_better ^ (lower != desc);
        key[n] = take_other ? ok[n] : key[n];
        row[n] = take_other ? orow[n] : row[n];
      }
    }
  }
}

// Wave index within the workgroup as a wave-uniform (SGPR) value: the compiler cannot prove
// threadIdx.x >> 6 uniform by itself, and everything derived from a "divergent" wave index
// (list pointers, loop bounds, loaded metadata) would otherwise go to VGPRs and exec-masked flow.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// erf in fp32 without branches (|error| <= 1.2 ulp, 6.9e-8 absolute over [-10, 10], checked
// against float64 erf): the minimax fits of the well-known branch-split erff (|x| <= 0.9277:
// odd polynomial in x; above: 1 - exp(-(|x| + poly(|x|) |x|))), both evaluated and selected, so the
// 8 values of a thread never diverge. The library erff spends ~3x the instructions in branches;
// the GELU pass was instruction-bound on it.
__device__ __forceinline__ float erf_f32(float a) {
  const float t = fabsf(a), s = a * a;
  float r = fmaf(-1.72853470e-5f, t, 3.83197126e-4f);
  const float u = fmaf(-3.88396438e-3f, t, 2.42546219e-2f);
  r = fmaf(r, s, u);
  r = fmaf(r, t, -1.06777877e-1f);
  r = fmaf(r, t, -6.34846687e-1f);
  r = fmaf(r, t, -1.28717512e-1f);
  r = fmaf(r, t, -t);
  const float big = copysignf(1.0f - __expf(r), a);
  float q = -5.96761703e-4f;
  q = fmaf(q, s, 4.99119423e-3f);
  q = fmaf(q, s, -2.67681349e-2f);
  q = fmaf(q, s, 1.12819925e-1f);
  q = fmaf(q, s, -3.76125336e-1f);
  q = fmaf(q, s, 1.28379166e-1f);
  q = fmaf(q, a, a);
  return t > 0.927734375f ? big : q;
}

__host__ __device__ inline int pow2_at_least(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace armi
