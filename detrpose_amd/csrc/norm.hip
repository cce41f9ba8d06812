// Row-wise kernels: residual add, LayerNorm (+residual, +post-add, +masked rows) and the
// decoder Gate.  One 64-lane wave per row; each lane owns E = c/64 contiguous elements,
// moved with one vector load/store where E*sizeof(T) is 4/8/16 bytes; statistics in f32
// with wave shuffles (no LDS).  HBM-bound: ~3 row passes of c elements each.
//   nn.LayerNorm post-norm residuals: hybrid_encoder.py:281-296, transformer.py:405-442
//   Gate: transformer.py:222-235
//   two-stage masked_fill + enc_output + enc_output_norm: transformer.py:1232-1236
#include "common.h"

namespace {

template <typename T, int E>
__device__ __forceinline__ void vload(const T* p, float* v) {
  constexpr int BYTES = E * (int)sizeof(T);
  if constexpr (BYTES == 16) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const T* q = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int t = 0; t < E; ++t) v[t] = to_f32(q[t]);
  } else if constexpr (BYTES == 8) {
    uint2 u = *reinterpret_cast<const uint2*>(p);
    const T* q = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int t = 0; t < E; ++t) v[t] = to_f32(q[t]);
  } else if constexpr (BYTES == 4) {
    uint32_t u = *reinterpret_cast<const uint32_t*>(p);
    const T* q = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int t = 0; t < E; ++t) v[t] = to_f32(q[t]);
  } else {
#pragma unroll
    for (int t = 0; t < E; ++t) v[t] = to_f32(p[t]);
  }
}

template <typename T, int E>
__device__ __forceinline__ void vstore(T* p, const float* v) {
  constexpr int BYTES = E * (int)sizeof(T);
  if constexpr (BYTES == 16 || BYTES == 8 || BYTES == 4) {
    T q[E];
#pragma unroll
    for (int t = 0; t < E; ++t) q[t] = from_f32<T>(v[t]);
    if constexpr (BYTES == 16) *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(q);
    else if constexpr (BYTES == 8) *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(q);
    else *reinterpret_cast<uint32_t*>(p) = *reinterpret_cast<const uint32_t*>(q);
  } else {
#pragma unroll
    for (int t = 0; t < E; ++t) p[t] = from_f32<T>(v[t]);
  }
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void add_rows_kernel(T* out, dp_rowmap om, const T* a, dp_rowmap am, const T* b,
                                                       dp_rowmap bm, int rows, int c) {
  const unsigned nch = (unsigned)(c / VEC);
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (unsigned)rows * nch) return;
  const unsigned r = gid / nch;
  const int i = (int)(gid - r * nch) * VEC;
  float x[VEC], y[VEC];
  vload<T, VEC>(a + rowmap_off(am, r) + i, x);
  if (b) {   // b == NULL: a row copy through the maps
    vload<T, VEC>(b + rowmap_off(bm, r) + i, y);
#pragma unroll
    for (int t = 0; t < VEC; ++t) x[t] += y[t];
  }
  vstore<T, VEC>(out + rowmap_off(om, r) + i, x);
}

template <int E>
__device__ __forceinline__ void ln_apply(float* v, const float* __restrict__ g, const float* __restrict__ bta, int c0,
                                         int c, float eps) {
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < E; ++t) s += v[t];
  const float mean = wave_sum(s) / c;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < E; ++t) {
    const float dlt = v[t] - mean;
    q += dlt * dlt;
  }
  const float rstd = rsqrtf(wave_sum(q) / c + eps);
#pragma unroll
  for (int t = 0; t < E; ++t) v[t] = (v[t] - mean) * rstd * g[c0 + t] + bta[c0 + t];
}

// R rows per wave, all of their loads issued before the first reduction: one row per wave
// left a single 512-byte load in flight per wave, far too few bytes in flight for HBM
// (Little's law), and the row statistics of R rows now overlap in the shuffle chains. Rows
// past the end are clamped for the loads (legal addresses, no divergent branches around
// them) and skipped at the store; masked rows are selected at the end.
template <typename T, int E, int R>
__global__ __launch_bounds__(256) void layernorm_kernel(T* out, dp_rowmap om, const T* x, dp_rowmap xm, const T* res,
                                                        dp_rowmap rm, const float* __restrict__ g,
                                                        const float* __restrict__ bta, float eps, int rows,
                                                        const T* post, dp_rowmap pm, int post_group, int post_skip,
                                                        const uint8_t* mask, int mask_period, const float* masked_row) {
  constexpr int c = 64 * E;
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (r0 >= rows) return;
  const int c0 = lane * E;
  float v[R][E];
#pragma unroll
  for (int i = 0; i < R; ++i) vload<T, E>(x + rowmap_off(xm, min(r0 + i, rows - 1)) + c0, v[i]);
  if (res) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float rv[E];
      vload<T, E>(res + rowmap_off(rm, min(r0 + i, rows - 1)) + c0, rv);
#pragma unroll
      for (int t = 0; t < E; ++t) v[i][t] += rv[t];
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) ln_apply<E>(v[i], g, bta, c0, c, eps);
  if (post) {
    // every row's post-add is read before the first store (out may alias the post rows)
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = min(r0 + i, rows - 1);
      const int grp = (unsigned)r / (unsigned)post_group;
      const int w = r - grp * post_group;
      if (w >= post_skip) {
        const int pr = grp * (post_group - post_skip) + (w - post_skip);
        float pv[E];
        vload<T, E>(post + rowmap_off(pm, pr) + c0, pv);
#pragma unroll
        for (int t = 0; t < E; ++t) v[i][t] += pv[t];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    if (r >= rows) break;
    if (mask && mask[(unsigned)r % (unsigned)mask_period]) {
#pragma unroll
      for (int t = 0; t < E; ++t) v[i][t] = masked_row[c0 + t];
    }
    vstore<T, E>(out + rowmap_off(om, r) + c0, v[i]);
  }
}

// Two-stage selection head in one pass (transformer.py:1232-1240): LayerNorm of contiguous
// rows (+ border mask: masked rows take masked_row), the row stored in T, and
// cls_out[r] = max_j (y . w_j + b_j) over the STORED (T-rounded) row y, so the class scores
// equal what dp_class_max would compute from the written rows, without reading them again.
template <typename T, int E, int R>
__global__ __launch_bounds__(256) void ln_classmax_kernel(T* out, const T* x, const float* __restrict__ g,
                                                          const float* __restrict__ bta, float eps, int rows,
                                                          const uint8_t* mask, int mask_period,
                                                          const float* masked_row, const float* __restrict__ cw,
                                                          const float* __restrict__ cb, int ncls, float* cls_out) {
  constexpr int c = 64 * E;
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (r0 >= rows) return;
  const int c0 = lane * E;
  float v[R][E];
#pragma unroll
  for (int i = 0; i < R; ++i) vload<T, E>(x + (int64_t)min(r0 + i, rows - 1) * c + c0, v[i]);
#pragma unroll
  for (int i = 0; i < R; ++i) ln_apply<E>(v[i], g, bta, c0, c, eps);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + i;
    if (r >= rows) break;
    if (mask && mask[(unsigned)r % (unsigned)mask_period]) {
#pragma unroll
      for (int t = 0; t < E; ++t) v[i][t] = masked_row[c0 + t];
    }
#pragma unroll
    for (int t = 0; t < E; ++t) v[i][t] = to_f32(from_f32<T>(v[i][t]));   // the stored value
    vstore<T, E>(out + (int64_t)r * c + c0, v[i]);
    float best = -INFINITY;
    for (int j = 0; j < ncls; ++j) {
      float sj = 0.f;
#pragma unroll
      for (int t = 0; t < E; ++t) sj = fmaf(v[i][t], cw[j * c + c0 + t], sj);
      best = fmaxf(best, wave_sum(sj) + cb[j]);
    }
    if (lane == 0) cls_out[r] = best;
  }
}

template <typename T, int E>
__global__ __launch_bounds__(256) void gate_ln_kernel(T* out, int out_ld, const T* gates, const T* xcat,
                                                      const float* __restrict__ g, const float* __restrict__ bta,
                                                      float eps, int rows) {
  constexpr int c = 64 * E;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int c0 = lane * E;
  const T* gr = gates + (int64_t)r * 2 * c;
  const T* xr = xcat + (int64_t)r * 2 * c;
  float g1[E], g2[E], x1[E], x2[E], v[E];
  vload<T, E>(gr + c0, g1);
  vload<T, E>(gr + c + c0, g2);
  vload<T, E>(xr + c0, x1);
  vload<T, E>(xr + c + c0, x2);
#pragma unroll
  for (int t = 0; t < E; ++t) v[t] = sigmoidf_(g1[t]) * x1[t] + sigmoidf_(g2[t]) * x2[t];
  ln_apply<E>(v, g, bta, c0, c, eps);
  vstore<T, E>(out + (int64_t)r * out_ld + c0, v);
}

constexpr int LN_ROWS = 4;   // rows per wave of layernorm_kernel

template <typename T>
int launch_ln(int e, dim3 grid, hipStream_t s, T* out, dp_rowmap om, const T* x, dp_rowmap xm, const T* res,
              dp_rowmap rm, const float* g, const float* b, float eps, int rows, const T* post, dp_rowmap pm, int pg,
              int ps, const uint8_t* mask, int mp, const float* mrow) {
#define DP_LN(E_)                                                                                                   \
  case E_:                                                                                                          \
    hipLaunchKernelGGL((layernorm_kernel<T, E_, LN_ROWS>), grid, dim3(256), 0, s, out, om, x, xm, res, rm, g, b, eps, \
                       rows,                                                                                        \
                       post, pm, pg, ps, mask, mp, mrow);                                                            \
    break;
  switch (e) {
    DP_LN(2) DP_LN(4) DP_LN(6) DP_LN(8)
    default: dp_set_error("dp_layernorm: c=%d unsupported (128/256/384/512)", 64 * e); return DP_EINVAL;
  }
#undef DP_LN
  return dp_check_launch("dp_layernorm");
}

template <typename T>
int launch_gate(int e, dim3 grid, hipStream_t s, T* out, int ld, const T* gates, const T* xcat, const float* g,
                const float* b, float eps, int rows) {
  switch (e) {
    case 2: hipLaunchKernelGGL((gate_ln_kernel<T, 2>), grid, dim3(256), 0, s, out, ld, gates, xcat, g, b, eps, rows); break;
    case 4: hipLaunchKernelGGL((gate_ln_kernel<T, 4>), grid, dim3(256), 0, s, out, ld, gates, xcat, g, b, eps, rows); break;
    case 6: hipLaunchKernelGGL((gate_ln_kernel<T, 6>), grid, dim3(256), 0, s, out, ld, gates, xcat, g, b, eps, rows); break;
    case 8: hipLaunchKernelGGL((gate_ln_kernel<T, 8>), grid, dim3(256), 0, s, out, ld, gates, xcat, g, b, eps, rows); break;
    default: dp_set_error("dp_gate_layernorm: c=%d unsupported", 64 * e); return DP_EINVAL;
  }
  return dp_check_launch("dp_gate_layernorm");
}

bool rm_aligned(const dp_rowmap& m, int vec) {
  return m.base % vec == 0 && m.stride_g % vec == 0 && m.stride_r % vec == 0;
}

}  // namespace

extern "C" int dp_add_rows(void* out, dp_rowmap om, const void* a, dp_rowmap am, const void* b, dp_rowmap bm,
                           int32_t rows, int32_t c, int32_t dtype, void* stream) {
  DP_REQUIRE(om.group > 0 && am.group > 0 && bm.group > 0, "dp_add_rows: row map group must be > 0");
  const int vec = dtype == DP_BF16 ? 8 : 4;
  const bool al = c % vec == 0 && rm_aligned(om, vec) && rm_aligned(am, vec) && rm_aligned(bm, vec) &&
                  ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(a) |
                    reinterpret_cast<uintptr_t>(b)) & 15) == 0;
  DP_REQUIRE(al, "dp_add_rows: rows must be 16-byte aligned (c=%d)", c);
  DP_REQUIRE((int64_t)rows * c < (1ll << 31), "dp_add_rows: %d rows x %d too large", rows, c);
  const int64_t total = (int64_t)rows * (c / vec);
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL((add_rows_kernel<bf16_t, 8>), grid, block, 0, as_stream(stream), (bf16_t*)out, om,
                       (const bf16_t*)a, am, (const bf16_t*)b, bm, rows, c);
  else
    hipLaunchKernelGGL((add_rows_kernel<float, 4>), grid, block, 0, as_stream(stream), (float*)out, om,
                       (const float*)a, am, (const float*)b, bm, rows, c);
  return dp_check_launch("dp_add_rows");
}

extern "C" int dp_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, const void* res, dp_rowmap rm,
                            const float* gamma, const float* beta, float eps, int32_t rows, int32_t c,
                            const void* post, dp_rowmap pm, int32_t post_group, int32_t post_skip,
                            const uint8_t* row_mask, int32_t mask_period, const float* masked_row, int32_t dtype,
                            void* stream) {
  DP_REQUIRE(c % 64 == 0 && c / 64 <= 8, "dp_layernorm: c=%d must be a multiple of 64 and <= 512", c);
  DP_REQUIRE(om.group > 0 && xm.group > 0 && (!res || rm.group > 0), "dp_layernorm: row map group must be > 0");
  DP_REQUIRE(!post || (post_group > post_skip && pm.group > 0), "dp_layernorm: bad post map");
  DP_REQUIRE(!row_mask || (mask_period > 0 && masked_row), "dp_layernorm: bad mask");
  const int e = c / 64;
  dim3 grid((unsigned)((rows + 4 * LN_ROWS - 1) / (4 * LN_ROWS)));
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    return launch_ln<bf16_t>(e, grid, s, (bf16_t*)out, om, (const bf16_t*)x, xm, (const bf16_t*)res, rm, gamma, beta,
                             eps, rows, (const bf16_t*)post, pm, post_group, post_skip, row_mask, mask_period,
                             masked_row);
  return launch_ln<float>(e, grid, s, (float*)out, om, (const float*)x, xm, (const float*)res, rm, gamma, beta, eps,
                          rows, (const float*)post, pm, post_group, post_skip, row_mask, mask_period, masked_row);
}

extern "C" int dp_layernorm_classmax(void* out, const void* x, const float* gamma, const float* beta, float eps,
                                     int32_t rows, int32_t c, const uint8_t* row_mask, int32_t mask_period,
                                     const float* masked_row, const float* cls_w, const float* cls_b, int32_t nclass,
                                     float* cls_out, int32_t dtype, void* stream) {
  DP_REQUIRE(out && x && gamma && beta && cls_w && cls_b && cls_out, "dp_layernorm_classmax: null pointer");
  DP_REQUIRE(c % 64 == 0 && c / 64 <= 8 && nclass >= 1 && nclass <= 4,
             "dp_layernorm_classmax: c=%d (multiple of 64, <= 512), nclass=%d (1..4)", c, nclass);
  DP_REQUIRE(!row_mask || (mask_period > 0 && masked_row), "dp_layernorm_classmax: bad mask");
  DP_REQUIRE((int64_t)rows * c < (1ll << 40), "dp_layernorm_classmax: too many rows");
  const int e = c / 64;
  dim3 grid((unsigned)((rows + 4 * LN_ROWS - 1) / (4 * LN_ROWS)));
  hipStream_t s = as_stream(stream);
#define DP_LNC(T_, E_)                                                                                          \
  case E_:                                                                                                      \
    hipLaunchKernelGGL((ln_classmax_kernel<T_, E_, LN_ROWS>), grid, dim3(256), 0, s, (T_*)out, (const T_*)x,    \
                       gamma, beta, eps, rows, row_mask, mask_period, masked_row, cls_w, cls_b, nclass, cls_out); \
    break;
  if (dtype == DP_BF16) {
    switch (e) { DP_LNC(bf16_t, 2) DP_LNC(bf16_t, 4) DP_LNC(bf16_t, 6) DP_LNC(bf16_t, 8) default: return DP_EINVAL; }
  } else {
    switch (e) { DP_LNC(float, 2) DP_LNC(float, 4) DP_LNC(float, 6) DP_LNC(float, 8) default: return DP_EINVAL; }
  }
#undef DP_LNC
  return dp_check_launch("dp_layernorm_classmax");
}

extern "C" int dp_gate_layernorm(void* out, int32_t out_ld, const void* gates, const void* xcat, const float* gamma,
                                 const float* beta, float eps, int32_t rows, int32_t c, int32_t dtype, void* stream) {
  DP_REQUIRE(c % 64 == 0 && c / 64 <= 8, "dp_gate_layernorm: c=%d must be a multiple of 64 and <= 512", c);
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    return launch_gate<bf16_t>(c / 64, grid, s, (bf16_t*)out, out_ld, (const bf16_t*)gates, (const bf16_t*)xcat,
                               gamma, beta, eps, rows);
  return launch_gate<float>(c / 64, grid, s, (float*)out, out_ld, (const float*)gates, (const float*)xcat, gamma, beta,
                            eps, rows);
}
