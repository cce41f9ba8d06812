// Row ops of the HGNetv2 backbone's training step (BASELINE config 5: freeze_at=-1 trains every
// backbone parameter, freeze_norm=True keeps its norms FrozenBatchNorm2d): the backward of
// ConvBNAct's epilogue (frozen BN affine, ReLU, LearnableAffineBlock), the input gradient of a
// strided dense conv as col2im of dz W, and the StemBlock max-pool's backward. The convs run on
// dp_conv2d / dp_dwconv2d (forward, stride-1 input gradient) and dp_gemm (weight gradients over
// dp_im2col); see detrpose_amd/backbone_train.py for the tape.
#include <algorithm>

#include "common.h"
#include <stdlib.h>

namespace {

template <typename T>
__device__ __forceinline__ float ldf(const T* p) {
  return to_f32(*p);
}

// ConvBNAct backward from its stored output y = lab(act(u)) [+ res], u = s z + b (hgnetv2.py:129-134):
// dz = dy * a * act'(u) * s[ch]; with LAB (scale a, bias cb) also d a += dy r, d cb += dy where r =
// relu(u) = (y - res - cb) / a. relu'(u) is read off y: the unit counts as on where a r exceeds
// the stored output's rounding (exact zero test without LAB and residual).
// A block = 256 threads = (256 / cw) rows x cw channels (cw = c rounded up to a power of two, at
// most 256), so narrow maps (the stem's 16 / 32 channels) fill the lanes; each thread does RU rows
// per step with all their loads issued first. RELU / RES / LAB are template flags: no branch
// around a load.
template <typename T, bool RELU, bool RES, bool LAB>
__global__ __launch_bounds__(256) void frozen_act_bwd_kernel(const T* __restrict__ y, int64_t ldy,
                                                             const T* __restrict__ res, int64_t ldr,
                                                             const T* __restrict__ dy, int64_t lddy, T* __restrict__ dz,
                                                             int64_t lddz, int rows, int c, int cw_log2,
                                                             const float* __restrict__ lab_a,
                                                             const float* __restrict__ lab_b,
                                                             const float* __restrict__ scale, float* __restrict__ dlab_a,
                                                             float* __restrict__ dlab_b) {
  constexpr int RU = 4;
  const int cw = 1 << cw_log2, rpb = 256 >> cw_log2;
  const int ch = blockIdx.y * cw + (threadIdx.x & (cw - 1));
  const int rsub = threadIdx.x >> cw_log2;
  const bool active = ch < c;
  const int chc = active ? ch : c - 1;
  // relative rounding of the stored output (f32: 2^-23, bf16: 2^-8): y = round(a r + cb + res),
  // so r == 0 is told from r > 0 only up to that
  const float eps = sizeof(T) == 2 ? 3.90625e-3f : 1.1920929e-7f;
  float a = 1.f, cb = 0.f;
  if (LAB) {
    a = *lab_a;
    cb = *lab_b;
  }
  const float sc_ch = scale ? scale[chc] : 1.f;
  float sa = 0.f, sc = 0.f;
  const int step = gridDim.x * rpb * RU;
  for (int r0 = blockIdx.x * rpb * RU + rsub; r0 < rows; r0 += step) {
    float g[RU], yv[RU], rv[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t r = min(r0 + u * rpb, rows - 1);
      g[u] = ldf(dy + r * lddy + chc);
      yv[u] = RELU ? ldf(y + r * ldy + chc) : 0.f;
      rv[u] = RES ? ldf(res + r * ldr + chc) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const bool ok = active && r0 + u * rpb < rows;
      float d = g[u];
      if (RELU) {
        // the stored output holds lab(act(u)) + res (the HG block's identity, added after the act)
        const float v = yv[u] - rv[u] - cb;   // a * relu(u), up to the output's rounding
        const float tol = (RES || LAB) ? eps * (fabsf(yv[u]) + fabsf(rv[u]) + fabsf(cb)) : 0.f;
        const bool on = LAB ? (a > 0.f ? v > tol : v < -tol) : v > tol;
        if (LAB) {
          const float rr = on ? v / a : 0.f;
          sa = fmaf(ok ? g[u] : 0.f, rr, sa);
          sc += ok ? g[u] : 0.f;
          d = on ? g[u] * a : 0.f;
        } else {
          d = on ? g[u] : 0.f;
        }
      }
      if (ok) dz[(int64_t)(r0 + u * rpb) * lddz + ch] = from_f32<T>(d * sc_ch);
    }
  }
  if (!LAB) return;
  __shared__ float red[2][4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sa += __shfl_xor(sa, o);
    sc += __shfl_xor(sc, o);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = sa;
    red[1][wv] = sc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(dlab_a, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(dlab_b, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// 16-byte vectors of channels: 8 bf16 or 4 f32 (VC), or one element (VC = 1)
template <typename T, int VC>
__device__ __forceinline__ void ld16v(const T* p, float (&v)[VC]) {
  if constexpr (VC == 1) {
    v[0] = ldf(p);
  } else {
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    const u32x4_t u = *reinterpret_cast<const u32x4_t*>(p);
    if constexpr (VC == 8) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[2 * q] = __uint_as_float(u[q] << 16), v[2 * q + 1] = __uint_as_float(u[q] & 0xffff0000u);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = __uint_as_float(u[q]);
    }
  }
}
template <typename T, int VC>
__device__ __forceinline__ void st16v(T* p, const float (&v)[VC]) {
  if constexpr (VC == 1) {
    *p = from_f32<T>(v[0]);
  } else if constexpr (VC == 8) {
    bf16x8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = (bf16_t)v[e];
    *reinterpret_cast<bf16x8*>(p) = r;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// The bf16 non-LAB case (every DETRPose-L / X backbone conv) over 16-byte channel vectors: a
// thread owns 8 channels of RU rows; a block = (256 / cw) rows x cw chunks (cw = c / 8 rounded
// up to a power of two).
template <bool RELU, bool RES>
__global__ __launch_bounds__(256) void frozen_act_bwd_vec_kernel(const bf16_t* __restrict__ y, int64_t ldy,
                                                                 const bf16_t* __restrict__ res, int64_t ldr,
                                                                 const bf16_t* __restrict__ dy, int64_t lddy,
                                                                 bf16_t* __restrict__ dz, int64_t lddz, int rows, int c,
                                                                 int cw_log2, const float* __restrict__ scale) {
  constexpr int RU = 4;
  const int cw = 1 << cw_log2, rpb = 256 >> cw_log2;
  const int ck = blockIdx.y * cw + (threadIdx.x & (cw - 1));
  const int rsub = threadIdx.x >> cw_log2;
  if (ck * 8 >= c) return;
  const int ch = ck * 8;
  constexpr float eps = 3.90625e-3f;   // bf16 rounding of the stored output (see above)
  float sc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sc[e] = scale ? scale[ch + e] : 1.f;
  const int step = gridDim.x * rpb * RU;
  for (int r0 = blockIdx.x * rpb * RU + rsub; r0 < rows; r0 += step) {
    float g[RU][8], yv[RU][8], rv[RU][8];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t r = min(r0 + u * rpb, rows - 1);
      ld16v<bf16_t, 8>(dy + r * lddy + ch, g[u]);
      if (RELU) ld16v<bf16_t, 8>(y + r * ldy + ch, yv[u]);
      if (RES) ld16v<bf16_t, 8>(res + r * ldr + ch, rv[u]);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (r0 + u * rpb >= rows) continue;
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        d[e] = g[u][e];
        if (RELU) {
          const float v = yv[u][e] - (RES ? rv[u][e] : 0.f);
          const float tol = RES ? eps * (fabsf(yv[u][e]) + fabsf(rv[u][e])) : 0.f;
          d[e] = v > tol ? g[u][e] : 0.f;
        }
        d[e] *= sc[e];
      }
      st16v<bf16_t, 8>(dz + (int64_t)(r0 + u * rpb) * lddz + ch, d);
    }
  }
}

// dx[b][y][x][ci] (+)= sum over the (ky, kx) whose output (oy, ox) = ((y + pad - ky) / s, ...) is
// whole and in range of col[(b*oh + oy)*ow + ox][(ky*kw + kx)*cin + ci]: the input gradient of a
// stride-s conv from dcol = dz W (W^T packed tap-major, dp_conv_pack mode 4), so the lanes of a
// wave (consecutive ci) read consecutive column entries. The (ky, oy) / (kx, ox) pairs of a pixel
// are enumerated directly (ky = (y + pad) mod s + s*i) instead of testing every tap.
template <typename T>
__global__ void col2im_kernel(const T* __restrict__ col, int h, int w, int cin, int kh, int kw, int s, int pad,
                              int oh, int ow, T* __restrict__ dx, int64_t bs, int ps, int acc, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int ci = (int)(e % cin);
  const int64_t p = e / cin;
  const int x = (int)(p % w);
  const int64_t t = p / w;
  const int yy = (int)(t % h), b = (int)(t / h);
  const int64_t K = (int64_t)cin * kh * kw;
  float sum = 0.f;
  for (int ky = (yy + pad) % s; ky < kh; ky += s) {
    const int ny = yy + pad - ky;
    if (ny < 0) break;
    const int oy = ny / s;
    if (oy >= oh) continue;
    const T* crow = col + ((int64_t)b * oh + oy) * ow * K + (int64_t)ky * kw * cin + ci;
    for (int kx = (x + pad) % s; kx < kw; kx += s) {
      const int nx = x + pad - kx;
      if (nx < 0) break;
      const int ox = nx / s;
      if (ox >= ow) continue;
      sum += ldf(crow + ox * K + kx * cin);
    }
  }
  T* o = dx + (int64_t)b * bs + ((int64_t)yy * w + x) * ps + ci;
  *o = from_f32<T>(acc ? ldf(o) + sum : sum);
}

// The same with 16-byte channel vectors (VC channels per thread: 8 bf16 / 4 f32) and 32-bit
// index arithmetic (total / VC < 2^31, host-checked): the scalar form spends most of its time in
// 64-bit divisions, one thread per element.
template <typename T, int VC>
__global__ __launch_bounds__(256) void col2im_vec_kernel(const T* __restrict__ col, int h, int w, int cin, int kh,
                                                         int kw, int s, int pad, int oh, int ow, T* __restrict__ dx,
                                                         int64_t bs, int ps, int acc, unsigned total) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const unsigned e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const unsigned nch = (unsigned)(cin / VC);
  const unsigned p = e / nch;
  const int ci = (int)(e - p * nch) * VC;
  const unsigned t = p / (unsigned)w;
  const int x = (int)(p - t * (unsigned)w);
  const unsigned b_ = t / (unsigned)h;
  const int yy = (int)(t - b_ * (unsigned)h), b = (int)b_;
  const int64_t K = (int64_t)cin * kh * kw;
  float sum[VC];
#pragma unroll
  for (int v = 0; v < VC; ++v) sum[v] = 0.f;
  for (int ky = (yy + pad) % s; ky < kh; ky += s) {
    const int ny = yy + pad - ky;
    if (ny < 0) break;
    const int oy = ny / s;
    if (oy >= oh) continue;
    const T* crow = col + ((int64_t)b * oh + oy) * ow * K + (int64_t)ky * kw * cin + ci;
    for (int kx = (x + pad) % s; kx < kw; kx += s) {
      const int nx = x + pad - kx;
      if (nx < 0) break;
      const int ox = nx / s;
      if (ox >= ow) continue;
      const u32x4_t u = *reinterpret_cast<const u32x4_t*>(crow + ox * K + kx * cin);
      if constexpr (VC == 8) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sum[2 * q] += __uint_as_float(u[q] << 16);
          sum[2 * q + 1] += __uint_as_float(u[q] & 0xffff0000u);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) sum[q] += __uint_as_float(u[q]);
      }
    }
  }
  T* o = dx + (int64_t)b * bs + ((int64_t)yy * w + x) * ps + ci;
  if (acc) {
    const u32x4_t u = *reinterpret_cast<const u32x4_t*>(o);
    if constexpr (VC == 8) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sum[2 * q] += __uint_as_float(u[q] << 16);
        sum[2 * q + 1] += __uint_as_float(u[q] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) sum[q] += __uint_as_float(u[q]);
    }
  }
  if constexpr (VC == 8) {
    bf16x8 r;
#pragma unroll
    for (int v = 0; v < 8; ++v) r[v] = (bf16_t)sum[v];
    *reinterpret_cast<bf16x8*>(o) = r;
  } else {
    *reinterpret_cast<float4*>(o) = make_float4(sum[0], sum[1], sum[2], sum[3]);
  }
}

// F.pad(x, (0,1,0,1)) + MaxPool2d(2, 1, ceil_mode=True) backward (hgnetv2.py:215, 217): each
// output's gradient goes to its window's first maximum in scan order (max_pool2d's argmax, the
// pad zeros included: a pad maximum takes the gradient out of the map); gathered per input.
// VC channels per thread (16-byte vectors when the rows allow: 8x fewer load instructions);
// I32: total / VC < 2^31, the index split in 32-bit unsigned arithmetic
template <typename T, bool I32, int VC>
__global__ void maxpool_bwd_kernel(const T* __restrict__ x, int64_t xbs, int xps, const T* __restrict__ dout,
                                   int64_t obs, int ops, int h, int w, int c, T* __restrict__ dx, int64_t dbs, int dps,
                                   int64_t total) {
  // every load unconditional (clamped address, value selected away): the 3x3 neighbourhood of
  // x and the 2x2 of dout are in flight together
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int nch = c / VC;
  int ch, px, py, b;
  if constexpr (I32) {
    const unsigned e32 = (unsigned)e, p = e32 / (unsigned)nch, t = p / (unsigned)w, b_ = t / (unsigned)h;
    ch = (int)(e32 - p * (unsigned)nch) * VC, px = (int)(p - t * (unsigned)w), py = (int)(t - b_ * (unsigned)h);
    b = (int)b_;
  } else {
    ch = (int)(e % nch) * VC;
    const int64_t p = e / nch;
    px = (int)(p % w);
    const int64_t t = p / w;
    py = (int)(t % h), b = (int)(t / h);
  }
  const T* xb = x + (int64_t)b * xbs + ch;
  float xv[3][3][VC];   // x at rows py-1 .. py+1, columns px-1 .. px+1 (0 past the right / bottom edge)
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dxx = 0; dxx < 3; ++dxx) {
      const int yy = py - 1 + dy, xx = px - 1 + dxx;
      ld16v<T, VC>(xb + ((int64_t)min(max(yy, 0), h - 1) * w + min(max(xx, 0), w - 1)) * xps, xv[dy][dxx]);
      if (!(yy < h && xx < w))   // yy, xx >= 0 wherever a window reads them
#pragma unroll
        for (int v = 0; v < VC; ++v) xv[dy][dxx][v] = 0.f;
    }
  float acc[VC];
#pragma unroll
  for (int v = 0; v < VC; ++v) acc[v] = 0.f;
#pragma unroll
  for (int oy = 0; oy < 2; ++oy)
#pragma unroll
    for (int ox = 0; ox < 2; ++ox) {
      // output (py - 1 + oy, px - 1 + ox): window rows oy .. oy+1, columns ox .. ox+1 of xv
      const int qy = py - 1 + oy, qx = px - 1 + ox;
      float g[VC];
      ld16v<T, VC>(dout + (int64_t)b * obs + ((int64_t)max(qy, 0) * w + max(qx, 0)) * ops + ch, g);
#pragma unroll
      for (int v = 0; v < VC; ++v) {
        float best = -INFINITY;
        int arg = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float xq = xv[oy + (q >> 1)][ox + (q & 1)][v];
          if (xq > best) {
            best = xq;
            arg = q;
          }
        }
        // this pixel is the window's (1 - oy, 1 - ox) element
        if (qy >= 0 && qx >= 0 && arg == ((1 - oy) << 1 | (1 - ox))) acc[v] += g[v];
      }
    }
  T* o = dx + (int64_t)b * dbs + ((int64_t)py * w + px) * dps + ch;
  float prev[VC];
  ld16v<T, VC>(o, prev);
#pragma unroll
  for (int v = 0; v < VC; ++v) prev[v] += acc[v];
  st16v<T, VC>(o, prev);
}

int grid_of(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace

#define DP_DT(CALL)         \
  do {                      \
    if (dtype == DP_BF16) { \
      using T = bf16_t;     \
      CALL;                 \
    } else {                \
      using T = float;      \
      CALL;                 \
    }                       \
  } while (0)

extern "C" int dp_frozen_act_bwd(const void* y, int64_t ld_y, const void* res, int64_t ld_res, const void* dy,
                                 int64_t ld_dy, void* dz, int64_t ld_dz,
                                 int32_t rows, int32_t c, int32_t act, const float* lab_a, const float* lab_b,
                                 const float* scale, float* dlab_a, float* dlab_b, int32_t dtype, void* stream) {
  DP_REQUIRE(dy && dz && rows > 0 && c > 0 && (act == DP_ACT_NONE || (act == DP_ACT_RELU && y)) &&
                 (!lab_a || (lab_b && act == DP_ACT_RELU && dlab_a && dlab_b)),
             "dp_frozen_act_bwd: bad arguments");
  int lg = 0;
  while ((1 << lg) < c && lg < 8) ++lg;
  const int cw = 1 << lg, rpb = 256 / cw, gy = (c + cw - 1) / cw;
  const int gx = std::max(1, std::min((rows + rpb * 4 - 1) / (rpb * 4), std::max(1, 4096 / gy)));
  const bool relu = act == DP_ACT_RELU, hres = relu && res, lab = lab_a != nullptr;
  hipStream_t s = as_stream(stream);
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  static const bool vec_off = getenv("DETRPOSE_FAB_VEC") && atoi(getenv("DETRPOSE_FAB_VEC")) == 0;   // A/B
  if (!vec_off && dtype == DP_BF16 && !lab && c % 8 == 0 && ld_dy % 8 == 0 && ld_dz % 8 == 0 &&
      (!relu || ld_y % 8 == 0) && (!hres || ld_res % 8 == 0) && a16(dy) && a16(dz) && a16(relu ? y : nullptr) &&
      a16(hres ? res : nullptr)) {
    const int nck = c / 8;
    int lv = 0;
    while ((1 << lv) < nck && lv < 8) ++lv;
    const int cwv = 1 << lv, rpv = 256 / cwv, gyv = (nck + cwv - 1) / cwv;
    const int gxv = std::max(1, std::min((rows + rpv * 4 - 1) / (rpv * 4), std::max(1, 4096 / gyv)));
#define FABV(R_, S_)                                                                                           \
  hipLaunchKernelGGL((frozen_act_bwd_vec_kernel<R_, S_>), dim3(gxv, gyv), dim3(256), 0, s, (const bf16_t*)y, ld_y, \
                     (const bf16_t*)res, ld_res, (const bf16_t*)dy, ld_dy, (bf16_t*)dz, ld_dz, rows, c, lv, scale)
    if (!relu) FABV(false, false);
    else if (!hres) FABV(true, false);
    else FABV(true, true);
#undef FABV
    return dp_check_launch("dp_frozen_act_bwd");
  }
#define FAB(T_, R_, S_, L_)                                                                                      \
  hipLaunchKernelGGL((frozen_act_bwd_kernel<T_, R_, S_, L_>), dim3(gx, gy), dim3(256), 0, s, (const T_*)y, ld_y, \
                     (const T_*)res, ld_res, (const T_*)dy, ld_dy, (T_*)dz, ld_dz, rows, c, lg, lab_a, lab_b, scale, \
                     dlab_a, dlab_b)
#define FAB_T(T_)                                      \
  if (!relu) FAB(T_, false, false, false);             \
  else if (!hres && !lab) FAB(T_, true, false, false); \
  else if (!hres) FAB(T_, true, false, true);          \
  else if (!lab) FAB(T_, true, true, false);           \
  else FAB(T_, true, true, true)
  if (dtype == DP_BF16) {
    FAB_T(bf16_t);
  } else {
    FAB_T(float);
  }
#undef FAB_T
#undef FAB
  return dp_check_launch("dp_frozen_act_bwd");
}

extern "C" int dp_col2im(const void* col, int32_t batch, int32_t h, int32_t w, int32_t cin, int32_t kh, int32_t kw,
                         int32_t stride, int32_t pad, int32_t oh, int32_t ow, void* dx, int64_t dx_bstride,
                         int32_t dx_pstride, int32_t accumulate, int32_t dtype, void* stream) {
  DP_REQUIRE(col && dx && batch > 0 && h > 0 && w > 0 && cin > 0 && kh > 0 && kw > 0 && stride > 0 && oh > 0 && ow > 0,
             "dp_col2im: bad arguments");
  const int64_t total = (int64_t)batch * h * w * cin;
  const int vc = dtype == DP_BF16 ? 8 : 4, esz = dtype == DP_BF16 ? 2 : 4;
  const bool vec = cin % vc == 0 && dx_pstride % vc == 0 && dx_bstride % vc == 0 && total / vc < (1ll << 31) &&
                   (reinterpret_cast<uintptr_t>(col) & 15) == 0 && (reinterpret_cast<uintptr_t>(dx) & 15) == 0 &&
                   vc * esz == 16;
  if (vec) {
    const unsigned n = (unsigned)(total / vc);
    if (dtype == DP_BF16)
      hipLaunchKernelGGL((col2im_vec_kernel<bf16_t, 8>), dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                         (const bf16_t*)col, h, w, cin, kh, kw, stride, pad, oh, ow, (bf16_t*)dx, dx_bstride,
                         dx_pstride, accumulate, n);
    else
      hipLaunchKernelGGL((col2im_vec_kernel<float, 4>), dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                         (const float*)col, h, w, cin, kh, kw, stride, pad, oh, ow, (float*)dx, dx_bstride,
                         dx_pstride, accumulate, n);
    return dp_check_launch("dp_col2im");
  }
  DP_DT(hipLaunchKernelGGL(col2im_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                           (const T*)col, h, w, cin, kh, kw, stride, pad, oh, ow, (T*)dx, dx_bstride, dx_pstride,
                           accumulate, total));
  return dp_check_launch("dp_col2im");
}

extern "C" int dp_maxpool2x2_pad_rb_bwd(const void* x, int64_t x_bstride, int32_t x_pstride, const void* dout,
                                        int64_t dout_bstride, int32_t dout_pstride, int32_t batch, int32_t h,
                                        int32_t w, int32_t c, void* dx, int64_t dx_bstride, int32_t dx_pstride,
                                        int32_t dtype, void* stream) {
  DP_REQUIRE(x && dout && dx && batch > 0 && h > 0 && w > 0 && c > 0, "dp_maxpool2x2_pad_rb_bwd: bad arguments");
  const int64_t total = (int64_t)batch * h * w * c;
  const int vc = dtype == DP_BF16 ? 8 : 4;
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool vec = c % vc == 0 && x_pstride % vc == 0 && dout_pstride % vc == 0 && dx_pstride % vc == 0 &&
                   x_bstride % vc == 0 && dout_bstride % vc == 0 && dx_bstride % vc == 0 && a16(x) && a16(dout) &&
                   a16(dx) && total / vc < (1ll << 31);
  const dim3 blk(256);
  if (vec) {
    const int64_t n = total / vc;
    if (dtype == DP_BF16)
      hipLaunchKernelGGL((maxpool_bwd_kernel<bf16_t, true, 8>), dim3((unsigned)((n + 255) / 256)), blk, 0,
                         as_stream(stream), (const bf16_t*)x, x_bstride, x_pstride, (const bf16_t*)dout, dout_bstride,
                         dout_pstride, h, w, c, (bf16_t*)dx, dx_bstride, dx_pstride, n);
    else
      hipLaunchKernelGGL((maxpool_bwd_kernel<float, true, 4>), dim3((unsigned)((n + 255) / 256)), blk, 0,
                         as_stream(stream), (const float*)x, x_bstride, x_pstride, (const float*)dout, dout_bstride,
                         dout_pstride, h, w, c, (float*)dx, dx_bstride, dx_pstride, n);
  } else if (total < (1ll << 31)) {
    DP_DT(hipLaunchKernelGGL((maxpool_bwd_kernel<T, true, 1>), dim3((unsigned)((total + 255) / 256)), blk, 0,
                             as_stream(stream), (const T*)x, x_bstride, x_pstride, (const T*)dout, dout_bstride,
                             dout_pstride, h, w, c, (T*)dx, dx_bstride, dx_pstride, total));
  } else {
    DP_DT(hipLaunchKernelGGL((maxpool_bwd_kernel<T, false, 1>), dim3((unsigned)((total + 255) / 256)), blk, 0,
                             as_stream(stream), (const T*)x, x_bstride, x_pstride, (const T*)dout, dout_bstride,
                             dout_pstride, h, w, c, (T*)dx, dx_bstride, dx_pstride, total));
  }
  return dp_check_launch("dp_maxpool2x2_pad_rb_bwd");
}
