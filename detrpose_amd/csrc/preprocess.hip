// Input pipeline of the reference benchmark on the GPU:
// tools/benchmark/dataset.py:56-61 = T.Resize(size=639, max_size=640) -> PadToSize((640, 640),
// fill=114) -> ToTensor -> ConvertImageDtype(float), applied to an image already decoded to a
// uint8 RGB (3, h, w) tensor on the device (dataset.py:74-75 decodes onto `self.device`).
//
// Resize on a uint8 tensor with antialias (torchvision's tensor path off the CPU): float
// bilinear interpolation with the antialias triangle filter, then round + clamp back to
// uint8. The filter is ATen's _upsample_bilinear2d_aa: for output index i at scale
// s = in/out, center = s (i + 0.5), support = s >= 1 ? s : 1, taps j in
// [int(center - support + 0.5), int(center + support + 0.5)) clipped to the input, weight
// max(0, 1 - |(j - center + 0.5) / max(s, 1)|) normalised to sum 1. Per output pixel the
// horizontal sum of every tap row is formed first, then the vertical sum (the order of the
// reference kernel, so float rounding matches up to ties). Then pad with `fill` to
// out_h x out_w (right / bottom) and divide by 255: one (3, out_h, out_w) f32 slot of the
// model's input batch.
#include "common.h"

namespace {

constexpr int MAXTAP = 64;   // taps per axis: supports downscales up to ~31x

struct AxisW {
  int first, n;
  float w[MAXTAP];
};

__device__ __forceinline__ void axis_weights(int i, int in_size, int out_size, AxisW& a) {
  const float scale = (float)in_size / (float)out_size;
  const float center = scale * (i + 0.5f);
  const float support = scale >= 1.f ? scale : 1.f;
  const float invscale = scale >= 1.f ? 1.f / scale : 1.f;
  int xmin = (int)(center - support + 0.5f);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5f);
  if (xmax > in_size) xmax = in_size;
  int n = xmax - xmin;
  if (n > MAXTAP) n = MAXTAP;
  float total = 0.f;
  for (int j = 0; j < n; ++j) {
    float x = fabsf((j + xmin - center + 0.5f) * invscale);
    const float w = x < 1.f ? 1.f - x : 0.f;
    a.w[j] = w;
    total += w;
  }
  if (total != 0.f)
    for (int j = 0; j < n; ++j) a.w[j] /= total;   // divided, as the reference normalises
  a.first = xmin, a.n = n;
}

// one thread per output pixel (y, x), all 3 channels
__global__ __launch_bounds__(256) void resize_pad_kernel(const uint8_t* __restrict__ img, int h, int w, int nh, int nw,
                                                         float* __restrict__ out, int oh, int ow, float fill) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= oh * ow) return;
  const int y = idx / ow, x = idx - y * ow;
  const int64_t plane = (int64_t)oh * ow;
  if (y >= nh || x >= nw) {
    const float f = fill / 255.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) out[c * plane + idx] = f;
    return;
  }
  AxisW ax, ay;
  axis_weights(x, w, nw, ax);
  axis_weights(y, h, nh, ay);
  for (int c = 0; c < 3; ++c) {
    const uint8_t* src = img + (int64_t)c * h * w;
    float acc = 0.f;
    for (int i = 0; i < ay.n; ++i) {
      const uint8_t* row = src + (int64_t)(ay.first + i) * w + ax.first;
      float hs = 0.f;
      for (int j = 0; j < ax.n; ++j) hs += ax.w[j] * (float)row[j];
      acc += ay.w[i] * hs;
    }
    float v = rintf(acc);   // round half to even, as torch.round
    v = fminf(fmaxf(v, 0.f), 255.f);
    out[c * plane + idx] = v / 255.f;
  }
}

}  // namespace

extern "C" int dp_resize_pad(const uint8_t* img, int32_t h, int32_t w, int32_t new_h, int32_t new_w, float* out,
                             int32_t out_h, int32_t out_w, float fill, void* stream) {
  DP_REQUIRE(img && out, "dp_resize_pad: null pointer");
  DP_REQUIRE(h > 0 && w > 0 && new_h > 0 && new_w > 0 && new_h <= out_h && new_w <= out_w,
             "dp_resize_pad: bad sizes (%dx%d -> %dx%d in %dx%d)", h, w, new_h, new_w, out_h, out_w);
  DP_REQUIRE((float)h / new_h < MAXTAP / 2 - 1 && (float)w / new_w < MAXTAP / 2 - 1,
             "dp_resize_pad: downscale %dx%d -> %dx%d beyond %d taps", h, w, new_h, new_w, MAXTAP);
  DP_REQUIRE((int64_t)out_h * out_w < (1ll << 31) && (int64_t)3 * h * w < (1ll << 31), "dp_resize_pad: too large");
  const int n = out_h * out_w;
  hipLaunchKernelGGL(resize_pad_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream), img, h, w, new_h,
                     new_w, out, out_h, out_w, fill);
  return dp_check_launch("dp_resize_pad");
}
