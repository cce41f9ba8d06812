// Shared device helpers for the DETRPose gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../include/detrpose_hip.h"

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- error reporting
void dp_set_error(const char* fmt, ...);
int dp_check_launch(const char* what);
// stream-ordered zero fill of `bytes` bytes (a kernel: graph-capturable); 0 on success
int dp_zero_async(void* p, size_t bytes, hipStream_t s);

// dp_conv2d_describe: while a describe buffer is set (this thread), the conv launch sites
// write the kernel instantiation they would launch and return 0 instead of launching
char* dp_describe_buf(int* len);
void dp_describe_set(char* buf, int len);
#define DP_DESCRIBE(...)                      \
  do {                                        \
    int dp_dlen_ = 0;                         \
    if (char* dp_dbuf_ = dp_describe_buf(&dp_dlen_)) { \
      snprintf(dp_dbuf_, dp_dlen_, __VA_ARGS__); \
      return 0;                               \
    }                                         \
  } while (0)
#define DP_TF(b) ((b) ? "true" : "false")

#define DP_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      dp_set_error(__VA_ARGS__);              \
      return DP_EINVAL;                       \
    }                                         \
  } while (0)

// ---------------------------------------------------------------- scalar conversions
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16_t x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float x) { return (bf16_t)x; }

// 16-byte vector of T: 8 bf16 or 4 f32
template <typename T> struct Vec16;
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  bf16x8 v;
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = (bf16_t)x; }
};
template <> struct Vec16<float> {
  static constexpr int N = 4;
  f32x4 v;
  __device__ __forceinline__ float get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = x; }
};

template <typename T>
__device__ __forceinline__ Vec16<T> load16(const T* p) {
  Vec16<T> r;
  *reinterpret_cast<uint4*>(&r.v) = *reinterpret_cast<const uint4*>(p);
  return r;
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const Vec16<T>& r) {
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(&r.v);
}
// non-temporal (streaming) 16-byte store: the halo convs' outputs (A/B on the L b64 3x3
// shapes: -2..-4 %; on the 1x1 / decoder GEMMs, whose outputs the next kernel re-reads from
// L2, it cost up to +13 %, so only conv_halo uses it)
template <typename T>
__device__ __forceinline__ void store16_nt(T* p, const Vec16<T>& r) {
  typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(*reinterpret_cast<const u32x4_nt*>(&r.v), reinterpret_cast<u32x4_nt*>(p));
}

// ---------------------------------------------------------------- activations
// sigmoid / SiLU through v_exp_f32 + v_rcp_f32 (1 ulp): a plain `/` compiles to the IEEE
// division sequence (div_scale x2, div_fmas, div_fixup + Newton steps), which made SiLU the
// most expensive part of the conv epilogues
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float silu_f(float x) { return x * sigmoidf_(x); }

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case DP_ACT_RELU: return fmaxf(x, 0.f);
    case DP_ACT_SILU: return silu_f(x);
    case DP_ACT_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    default: return x;
  }
}


// ---------------------------------------------------------------- wave reductions (64 lanes)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// row r < 2^31 (every launch checks its row count): 32-bit division, 64-bit offsets
__device__ __forceinline__ int64_t rowmap_off(const dp_rowmap& m, int64_t r) {
  const unsigned ri = (unsigned)r, gs = (unsigned)m.group;
  const unsigned g = ri / gs;
  const unsigned i = ri - g * gs;
  return m.base + (int64_t)g * m.stride_g + (int64_t)i * m.stride_r;
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
