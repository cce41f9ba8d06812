// Row-wise kernels: residual add, LayerNorm (+residual, +post-add, +masked rows) and the
// decoder Gate.  One 64-lane wave per row, each lane owns c/64 contiguous elements,
// statistics in f32 with wave shuffles (no LDS).
//   nn.LayerNorm post-norm residuals: hybrid_encoder.py:281-296, transformer.py:405-442
//   Gate: transformer.py:222-235
//   two-stage masked_fill + enc_output + enc_output_norm: transformer.py:1232-1236
#include "common.h"

namespace {

constexpr int MAXE = 8;  // c <= 512

template <typename T>
__device__ __forceinline__ void load_row(const T* p, int e, float* v) {
  for (int t = 0; t < e; ++t) v[t] = to_f32(p[t]);
}

template <typename T>
__global__ __launch_bounds__(256) void add_rows_kernel(T* out, dp_rowmap om, const T* a, dp_rowmap am, const T* b,
                                                       dp_rowmap bm, int rows, int c) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)rows * c) return;
  const int64_t r = gid / c;
  const int i = (int)(gid - r * c);
  out[rowmap_off(om, r) + i] = from_f32<T>(to_f32(a[rowmap_off(am, r) + i]) + to_f32(b[rowmap_off(bm, r) + i]));
}

template <typename T>
__global__ __launch_bounds__(256) void layernorm_kernel(T* out, dp_rowmap om, const T* x, dp_rowmap xm, const T* res,
                                                        dp_rowmap rm, const float* __restrict__ g,
                                                        const float* __restrict__ bta, float eps, int rows, int c,
                                                        const T* post, dp_rowmap pm, int post_group, int post_skip,
                                                        const uint8_t* mask, int mask_period, const float* masked_row) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int e = c >> 6;
  const int c0 = lane * e;
  float v[MAXE];
  T* o = out + rowmap_off(om, r) + c0;
  if (mask && mask[r % mask_period]) {
    for (int t = 0; t < e; ++t) o[t] = from_f32<T>(masked_row[c0 + t]);
    return;
  }
  load_row(x + rowmap_off(xm, r) + c0, e, v);
  if (res) {
    float rv[MAXE];
    load_row(res + rowmap_off(rm, r) + c0, e, rv);
    for (int t = 0; t < e; ++t) v[t] += rv[t];
  }
  float s = 0.f;
  for (int t = 0; t < e; ++t) s += v[t];
  const float mean = wave_sum(s) / c;
  float q = 0.f;
  for (int t = 0; t < e; ++t) {
    const float dlt = v[t] - mean;
    q += dlt * dlt;
  }
  const float rstd = rsqrtf(wave_sum(q) / c + eps);
  for (int t = 0; t < e; ++t) v[t] = (v[t] - mean) * rstd * g[c0 + t] + bta[c0 + t];
  if (post) {
    const int64_t grp = r / post_group;
    const int w = (int)(r - grp * post_group);
    if (w >= post_skip) {
      const int64_t pr = grp * (post_group - post_skip) + (w - post_skip);
      float pv[MAXE];
      load_row(post + rowmap_off(pm, pr) + c0, e, pv);
      for (int t = 0; t < e; ++t) v[t] += pv[t];
    }
  }
  for (int t = 0; t < e; ++t) o[t] = from_f32<T>(v[t]);
}

template <typename T>
__global__ __launch_bounds__(256) void gate_ln_kernel(T* out, int out_ld, const T* gates, const T* xcat,
                                                      const float* __restrict__ g, const float* __restrict__ bta,
                                                      float eps, int rows, int c) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int e = c >> 6;
  const int c0 = lane * e;
  const T* gr = gates + r * 2 * c;
  const T* xr = xcat + r * 2 * c;
  float v[MAXE];
  float s = 0.f;
  for (int t = 0; t < e; ++t) {
    const float g1 = sigmoidf_(to_f32(gr[c0 + t])), g2 = sigmoidf_(to_f32(gr[c + c0 + t]));
    v[t] = g1 * to_f32(xr[c0 + t]) + g2 * to_f32(xr[c + c0 + t]);
    s += v[t];
  }
  const float mean = wave_sum(s) / c;
  float q = 0.f;
  for (int t = 0; t < e; ++t) {
    const float dlt = v[t] - mean;
    q += dlt * dlt;
  }
  const float rstd = rsqrtf(wave_sum(q) / c + eps);
  T* o = out + r * out_ld + c0;
  for (int t = 0; t < e; ++t) o[t] = from_f32<T>((v[t] - mean) * rstd * g[c0 + t] + bta[c0 + t]);
}

}  // namespace

extern "C" int dp_add_rows(void* out, dp_rowmap om, const void* a, dp_rowmap am, const void* b, dp_rowmap bm,
                           int32_t rows, int32_t c, int32_t dtype, void* stream) {
  DP_REQUIRE(om.group > 0 && am.group > 0 && bm.group > 0, "dp_add_rows: row map group must be > 0");
  const int64_t total = (int64_t)rows * c;
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(add_rows_kernel<bf16_t>, grid, block, 0, as_stream(stream), (bf16_t*)out, om, (const bf16_t*)a,
                       am, (const bf16_t*)b, bm, rows, c);
  else
    hipLaunchKernelGGL(add_rows_kernel<float>, grid, block, 0, as_stream(stream), (float*)out, om, (const float*)a, am,
                       (const float*)b, bm, rows, c);
  return dp_check_launch("dp_add_rows");
}

extern "C" int dp_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, const void* res, dp_rowmap rm,
                            const float* gamma, const float* beta, float eps, int32_t rows, int32_t c,
                            const void* post, dp_rowmap pm, int32_t post_group, int32_t post_skip,
                            const uint8_t* row_mask, int32_t mask_period, const float* masked_row, int32_t dtype,
                            void* stream) {
  DP_REQUIRE(c % 64 == 0 && c / 64 <= MAXE, "dp_layernorm: c=%d must be a multiple of 64 and <= 512", c);
  DP_REQUIRE(om.group > 0 && xm.group > 0 && (!res || rm.group > 0), "dp_layernorm: row map group must be > 0");
  DP_REQUIRE(!post || (post_group > post_skip && pm.group > 0), "dp_layernorm: bad post map");
  DP_REQUIRE(!row_mask || (mask_period > 0 && masked_row), "dp_layernorm: bad mask");
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(layernorm_kernel<bf16_t>, grid, block, 0, as_stream(stream), (bf16_t*)out, om, (const bf16_t*)x,
                       xm, (const bf16_t*)res, rm, gamma, beta, eps, rows, c, (const bf16_t*)post, pm, post_group,
                       post_skip, row_mask, mask_period, masked_row);
  else
    hipLaunchKernelGGL(layernorm_kernel<float>, grid, block, 0, as_stream(stream), (float*)out, om, (const float*)x, xm,
                       (const float*)res, rm, gamma, beta, eps, rows, c, (const float*)post, pm, post_group, post_skip,
                       row_mask, mask_period, masked_row);
  return dp_check_launch("dp_layernorm");
}

extern "C" int dp_gate_layernorm(void* out, int32_t out_ld, const void* gates, const void* xcat, const float* gamma,
                                 const float* beta, float eps, int32_t rows, int32_t c, int32_t dtype, void* stream) {
  DP_REQUIRE(c % 64 == 0 && c / 64 <= MAXE, "dp_gate_layernorm: c=%d must be a multiple of 64 and <= 512", c);
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(gate_ln_kernel<bf16_t>, grid, block, 0, as_stream(stream), (bf16_t*)out, out_ld,
                       (const bf16_t*)gates, (const bf16_t*)xcat, gamma, beta, eps, rows, c);
  else
    hipLaunchKernelGGL(gate_ln_kernel<float>, grid, block, 0, as_stream(stream), (float*)out, out_ld,
                       (const float*)gates, (const float*)xcat, gamma, beta, eps, rows, c);
  return dp_check_launch("dp_gate_layernorm");
}
