// Row ops of the HybridEncoder's training step (BASELINE config 5): the
// encoder's BatchNorm2d layers on batch statistics (sync_bn), the ConvNormLayer / VGGBlock
// epilogues with their backward, the pieces of conv backward that are not GEMMs or convs
// themselves, and the nearest-x2 / activation / add rows. Convolutions run on dp_conv2d
// (forward and 3x3 input gradient with flipped weights) and dp_gemm (1x1 input gradient,
// every weight gradient over an im2col); see detrpose_amd/encoder_train.py for the tape.
//
// Layout: NHWC activations as [rows][c] with a row stride (channel slices of concat buffers),
// rows = batch * h * w. f32 statistics. Activations / activation gradients of dtype.
#include <algorithm>
#include <stdlib.h>
#include <type_traits>

#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ float ld_(const T* p) {
  return to_f32(*p);
}

// act(pre) and d act / d pre (hybrid_encoder.py get_activation: silu / relu / gelu (erf))
__device__ __forceinline__ float act_f(float x, int act) {
  if (act == DP_ACT_RELU) return fmaxf(x, 0.f);
  if (act == DP_ACT_SILU) return x / (1.f + __expf(-x));
  if (act == DP_ACT_GELU) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  return x;
}
__device__ __forceinline__ float act_d(float x, int act) {
  if (act == DP_ACT_RELU) return x > 0.f ? 1.f : 0.f;
  if (act == DP_ACT_SILU) {
    const float s = 1.f / (1.f + __expf(-x));
    return s * (1.f + x * (1.f - s));
  }
  if (act == DP_ACT_GELU)
    return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
  return 1.f;
}

// ---------------------------------------------------------------- BatchNorm statistics
// Column sums over a block of rows, shifted by the column's first-row value K (single-pass
// variance without the E[x^2] - mean^2 cancellation): part[y][0] = sum (x - K), part[y][1] =
// sum (x - K)^2 over row slice y. Block: 64 channels (lane) x 4 row phases (wave), `slice` rows
// (a multiple of 32; see bn_slice_rows: enough slices to fill the chip, few enough for a short reduction).
// No float atomics: bn_stats_reduce_kernel sums the slices in a fixed order, so the forward
// is deterministic run to run.
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* __restrict__ x, int64_t ld, int rows, int c, int slice,
                                                       float* __restrict__ part) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  const int chc = min(ch, c - 1);
  const int r0 = blockIdx.y * slice;
  float s1 = 0.f, s2 = 0.f;
  const float k = ld_(x + chc);
  const int r1 = min(r0 + slice, rows);
  for (int r = r0 + wv; r < r1; r += 32) {   // 8 rows per step, loads issued together
    float d[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) d[u] = ld_(x + (int64_t)min(r + 4 * u, r1 - 1) * ld + chc) - k;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (r + 4 * u < r1) {
        s1 += d[u];
        s2 = fmaf(d[u], d[u], s2);
      }
  }
  red[0][wv][lane] = s1;
  red[1][wv][lane] = s2;
  __syncthreads();
  if (wv == 0 && ch < c) {
    float* pp = part + (int64_t)blockIdx.y * 2 * c;
    pp[ch] = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
    pp[c + ch] = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
  }
}

// out [3][c] = (K, sum over the ny slices of part[y][0], of part[y][1]): wave w of 16 adds
// slices w, w + 16, ... in order, then the 16 wave sums are added in order.
// parts [np][3][c] (one per rank: K, S1, S2 over `count` rows each) -> mr [2][c] = (mean, rstd)
// of the union (Chan's parallel combination), biased variance; running statistics updated as
// F.batch_norm does (momentum, unbiased variance). One channel.
__device__ __forceinline__ void bn_finalize_ch(const float* __restrict__ parts, int np, float count, int c, int ch,
                                               float eps, float momentum, float* __restrict__ rmean,
                                               float* __restrict__ rvar, float* __restrict__ mr) {
  double n = 0.0, mean = 0.0, m2 = 0.0;
  for (int p = 0; p < np; ++p) {
    const float* q = parts + (int64_t)p * 3 * c;
    const double k = q[ch], s1 = q[c + ch], s2 = q[2 * c + ch];
    const double mi = k + s1 / count, m2i = s2 - s1 * s1 / count;
    const double nn = n + count, delta = mi - mean;
    mean += delta * count / nn;
    m2 += m2i + delta * delta * n * count / nn;
    n = nn;
  }
  const double var = m2 / n;
  mr[ch] = (float)mean;
  mr[c + ch] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    rmean[ch] = (float)((1.0 - momentum) * rmean[ch] + momentum * mean);
    rvar[ch] = (float)((1.0 - momentum) * rvar[ch] + momentum * (n > 1.0 ? m2 / (n - 1.0) : var));
  }
}

struct BnFin {   // the finalize of dp_bn_stats_finalize (mr == nullptr: none)
  float count, eps, momentum;
  float *rmean, *rvar, *mr;
};

template <typename T>
__global__ __launch_bounds__(1024) void bn_stats_reduce_kernel(const T* __restrict__ x, const float* __restrict__ part,
                                                               int ny, int c, float* __restrict__ out, BnFin fin) {
  constexpr int NWV = 16;
  __shared__ float red[2][NWV][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  const int chc = min(ch, c - 1);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int y = wv; y < ny; y += NWV) {
    s1 += part[(int64_t)y * 2 * c + chc];
    s2 += part[(int64_t)y * 2 * c + c + chc];
  }
  red[0][wv][lane] = s1;
  red[1][wv][lane] = s2;
  __syncthreads();
  if (wv == 0 && ch < c) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int k = 0; k < NWV; ++k) t1 += red[0][k][lane], t2 += red[1][k][lane];
    out[ch] = ld_(x + ch);
    out[c + ch] = t1;
    out[2 * c + ch] = t2;
    // one rank (no SyncBN exchange between the statistics and their finalize): finalize here, from
    // the values this thread just stored (the same arithmetic as bn_finalize_kernel's)
    if (fin.mr) bn_finalize_ch(out, 1, fin.count, c, ch, fin.eps, fin.momentum, fin.rmean, fin.rvar, fin.mr);
  }
}

__global__ void bn_finalize_kernel(const float* __restrict__ parts, int np, float count, int c, float eps,
                                   float momentum, float* __restrict__ rmean, float* __restrict__ rvar,
                                   float* __restrict__ mr) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  bn_finalize_ch(parts, np, count, c, ch, eps, momentum, rmean, rvar, mr);
}

// VC-element vector loads / stores of a row chunk (VC = 1, or 16 / 8 bytes)
template <typename T, int VC>
__device__ __forceinline__ void ld_vec(const T* p, float (&v)[VC]) {
  if constexpr (VC == 1) {
    v[0] = to_f32(*p);
  } else if constexpr (std::is_same<T, bf16_t>::value && VC == 8) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const unsigned w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) v[2 * q] = __uint_as_float(w4[q] << 16), v[2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
  } else if constexpr (std::is_same<T, bf16_t>::value) {
    static_assert(VC == 4, "bf16 vectors of 4 or 8");
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16), v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16), v[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
    static_assert(VC == 4, "f32 vectors of 4");
    const float4 f = *reinterpret_cast<const float4*>(p);
    v[0] = f.x, v[1] = f.y, v[2] = f.z, v[3] = f.w;
  }
}
template <typename T, int VC>
__device__ __forceinline__ void st_vec(T* p, const float (&v)[VC]) {
  if constexpr (VC == 1) {
    *p = from_f32<T>(v[0]);
  } else if constexpr (std::is_same<T, bf16_t>::value && VC == 8) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16_t)v[e];
    *reinterpret_cast<bf16x8*>(p) = o;
  } else if constexpr (std::is_same<T, bf16_t>::value) {
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (bf16_t)v[e];
    *reinterpret_cast<bf16x4*>(p) = o;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

struct BnBranch {
  const void* z;
  int64_t ld;
  const float* mr;   // [2][c] mean, rstd
  const float* g;
  const float* b;
};

// Row kernels: a thread owns one channel (its per-channel parameters in registers) and walks
// the rows blockIdx.x + u gridDim.x (u = 0 .. RU-1), + RU gridDim.x, ...; consecutive threads take
// consecutive channels of a row. The RU rows' loads are issued together (row indices clamped,
// out-of-range rows not stored). grid = (row slices, channel blocks of blockDim.x): see rc_grid.
constexpr int RU = 4;

// y = act(bn1(z1) [+ bn2(z2)]) (+ res when res != NULL)
template <typename T, bool TWO, bool RES>
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(T* __restrict__ y, int64_t ldy, BnBranch p1, BnBranch p2,
                                                         const T* __restrict__ res, int64_t ldr, int rows, int c,
                                                         int act) {
  const int ch = blockIdx.y * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float m1 = p1.mr[ch], s1 = p1.mr[c + ch], g1 = p1.g[ch], b1 = p1.b[ch];
  const float m2 = TWO ? p2.mr[ch] : 0.f, s2 = TWO ? p2.mr[c + ch] : 0.f, g2 = TWO ? p2.g[ch] : 0.f,
              b2 = TWO ? p2.b[ch] : 0.f;
  const T* z1 = reinterpret_cast<const T*>(p1.z) + ch;
  const T* z2 = reinterpret_cast<const T*>(p2.z) + ch;
  for (int r0 = blockIdx.x; r0 < rows; r0 += RU * gridDim.x) {
    float x1[RU], x2[RU], rv[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t r = min(r0 + u * (int)gridDim.x, rows - 1);
      x1[u] = ld_(z1 + r * p1.ld);
      x2[u] = TWO ? ld_(z2 + r * p2.ld) : 0.f;
      rv[u] = RES ? ld_(res + r * ldr + ch) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = r0 + u * gridDim.x;
      float v = fmaf(g1, (x1[u] - m1) * s1, b1);
      if (TWO) v += fmaf(g2, (x2[u] - m2) * s2, b2);
      v = act_f(v, act) + rv[u];
      if (r < rows) y[(int64_t)r * ldy + ch] = from_f32<T>(v);
    }
  }
}

// dp = dy * act'(pre): per row slice y the column sums part[y] = (sum dp, sum dp xh1, sum dp xh2)
// (no float atomics: bn_act_bwd_sum_kernel adds the slices in a fixed order)
template <typename T, bool TWO>
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(const T* __restrict__ dy, int64_t ldy, BnBranch p1,
                                                                BnBranch p2, int rows, int c, int act, int per,
                                                                float* __restrict__ part) {
  __shared__ float red[3][4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  const int chc = min(ch, c - 1);
  const int r0 = blockIdx.y * per;
  const float m1 = p1.mr[chc], s1 = p1.mr[c + chc], g1 = p1.g[chc], b1 = p1.b[chc];
  const float m2 = TWO ? p2.mr[chc] : 0.f, s2 = TWO ? p2.mr[c + chc] : 0.f, g2 = TWO ? p2.g[chc] : 0.f,
              b2 = TWO ? p2.b[chc] : 0.f;
  const T* z1 = reinterpret_cast<const T*>(p1.z) + chc;
  const T* z2 = reinterpret_cast<const T*>(p2.z) + chc;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  const int r1 = min(r0 + per, rows);
  for (int r = r0 + wv; r < r1; r += 4 * RU) {
    float x1[RU], x2[RU], g[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t rr = min(r + 4 * u, r1 - 1);
      x1[u] = ld_(z1 + rr * p1.ld);
      x2[u] = TWO ? ld_(z2 + rr * p2.ld) : 0.f;
      g[u] = ld_(dy + rr * ldy + chc);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const float h1 = (x1[u] - m1) * s1, h2 = TWO ? (x2[u] - m2) * s2 : 0.f;
      float pre = fmaf(g1, h1, b1);
      if (TWO) pre += fmaf(g2, h2, b2);
      const float dp = r + 4 * u < r1 ? g[u] * act_d(pre, act) : 0.f;
      a0 += dp;
      a1 = fmaf(dp, h1, a1);
      a2 = fmaf(dp, h2, a2);
    }
  }
  red[0][wv][lane] = a0;
  red[1][wv][lane] = a1;
  red[2][wv][lane] = a2;
  __syncthreads();
  if (wv == 0 && ch < c) {
    float* pp = part + (int64_t)blockIdx.y * 3 * c;
    pp[ch] = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
    pp[c + ch] = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
    pp[2 * c + ch] = red[2][0][lane] + red[2][1][lane] + red[2][2][lane] + red[2][3][lane];
  }
}

// sums [3][c] = the slices' sums in a fixed order (wave w of 16 takes slices w, w + 16, ...), and
// the parameter gradients from them: dg1 += sums[1], db1 += sums[0], dg2 += sums[2], db2 += sums[0]
__global__ __launch_bounds__(1024) void bn_act_bwd_sum_kernel(const float* __restrict__ part, int ny, int c,
                                                              float* __restrict__ sums, float* __restrict__ dg1,
                                                              float* __restrict__ db1, float* __restrict__ dg2,
                                                              float* __restrict__ db2) {
  constexpr int NWV = 16;
  __shared__ float red[3][NWV][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  const int chc = min(ch, c - 1);
  float t[3] = {0.f, 0.f, 0.f};
#pragma unroll 4
  for (int y = wv; y < ny; y += NWV) {
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] += part[((int64_t)y * 3 + k) * c + chc];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) red[k][wv][lane] = t[k];
  __syncthreads();
  if (wv == 0 && ch < c) {
    float u[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int w = 0; w < NWV; ++w) u[k] += red[k][w][lane];
    sums[ch] = u[0];
    sums[c + ch] = u[1];
    sums[2 * c + ch] = u[2];
    if (dg1) dg1[ch] += u[1];
    if (db1) db1[ch] += u[0];
    if (dg2) dg2[ch] += u[2];
    if (db2) db2[ch] += u[0];
  }
}

// dz_k = g_k rstd_k (dp - sum dp / N - xh_k sum (dp xh_k) / N) (torch batch_norm_backward with
// the synced sums)
template <typename T, bool TWO>
__global__ __launch_bounds__(256) void bn_act_bwd_apply_kernel(T* __restrict__ dz1, int64_t ld1, T* __restrict__ dz2,
                                                               int64_t ld2, const T* __restrict__ dy, int64_t ldy,
                                                               BnBranch p1, BnBranch p2, int rows, int c, int act,
                                                               const float* __restrict__ sums, float inv_n) {
  const int ch = blockIdx.y * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float m1 = p1.mr[ch], s1 = p1.mr[c + ch], g1 = p1.g[ch], b1 = p1.b[ch];
  const float m2 = TWO ? p2.mr[ch] : 0.f, s2 = TWO ? p2.mr[c + ch] : 0.f, g2 = TWO ? p2.g[ch] : 0.f,
              b2 = TWO ? p2.b[ch] : 0.f;
  const float m0 = sums[ch] * inv_n, c1 = sums[c + ch] * inv_n, c2 = sums[2 * c + ch] * inv_n;
  const float k1 = g1 * s1, k2 = g2 * s2;
  const T* z1 = reinterpret_cast<const T*>(p1.z) + ch;
  const T* z2 = reinterpret_cast<const T*>(p2.z) + ch;
  for (int r0 = blockIdx.x; r0 < rows; r0 += RU * gridDim.x) {
    float x1[RU], x2[RU], g[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t r = min(r0 + u * (int)gridDim.x, rows - 1);
      x1[u] = ld_(z1 + r * p1.ld);
      x2[u] = TWO ? ld_(z2 + r * p2.ld) : 0.f;
      g[u] = ld_(dy + r * ldy + ch);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = r0 + u * gridDim.x;
      const float h1 = (x1[u] - m1) * s1, h2 = TWO ? (x2[u] - m2) * s2 : 0.f;
      float pre = fmaf(g1, h1, b1);
      if (TWO) pre += fmaf(g2, h2, b2);
      const float dp = g[u] * act_d(pre, act);
      if (r < rows) {
        dz1[(int64_t)r * ld1 + ch] = from_f32<T>(k1 * (dp - m0 - h1 * c1));
        if (TWO) dz2[(int64_t)r * ld2 + ch] = from_f32<T>(k2 * (dp - m0 - h2 * c2));
      }
    }
  }
}

// ---------------------------------------------------------------- conv backward pieces
// col[row][ci * kh * kw + ky * kw + kx] = x[b][oy * s - pad + ky][ox * s - pad + kx][ci] (0 outside):
// the [rows][cin][kh][kw] operand whose product with dz^T is the weight gradient in the
// reference layout [cout][cin][kh][kw]
template <typename TI, typename T>
__global__ void im2col_kernel(const TI* __restrict__ x, int64_t bs, int ps, int64_t cs, int h, int w, int cin, int kh,
                              int kw, int stride, int pad, int oh, int ow, T* __restrict__ col, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // (row, ci)
  if (e >= total) return;
  const int ci = (int)(e % cin);
  const int64_t row = e / cin;
  const int ox = (int)(row % ow);
  const int64_t t = row / ow;
  const int oy = (int)(t % oh), b = (int)(t / oh);
  T* o = col + row * ((int64_t)cin * kh * kw) + (int64_t)ci * kh * kw;
  for (int ky = 0; ky < kh; ++ky)
    for (int kx = 0; kx < kw; ++kx) {
      const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
      const bool ok = (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      o[ky * kw + kx] = ok ? from_f32<T>(to_f32(x[(int64_t)b * bs + ((int64_t)iy * w + ix) * ps + ci * cs]))
                           : from_f32<T>(0.f);
    }
}

// f32 master weights [cout][cin][kh][kw] -> the conv kernels' packed [rows][kpad] (K = ky, kx, ci):
// mode 0 forward (rows = cout), mode 1 input gradient (rows = cin, K over cout, taps flipped),
// mode 2 depthwise taps [kh*kw][c] f32 (cin = 1), mode 4 W^T of a strided conv's column GEMM
// (rows = kh*kw*cin in tap-major order (ky, kx, ci), K over cout, taps not flipped: dcol = dz W
// in the order dp_col2im reads). kc: the K dimension's channel stride (>= the real channel count:
// maps whose channels are padded to a vector multiple), zero in the pads
// elements pack_elem writes for one pack (mode 5: a plain f32 -> dtype copy of cout elements)
__host__ __device__ inline int64_t pack_total(int cout, int cin, int kh, int kw, int kpad, int mode) {
  return mode == 2 ? (int64_t)cout * kh * kw
         : mode == 3 ? (int64_t)cout * cin * kh * kw
         : mode == 4 ? (int64_t)kh * kw * cin * kpad
         : mode == 5 ? (int64_t)cout
                     : (int64_t)(mode == 0 ? cout : cin) * kpad;
}

template <typename T>
__device__ __forceinline__ void pack_elem(int64_t e, const float* __restrict__ w, int cout, int cin, int kh, int kw,
                                          void* __restrict__ out, int kpad, int kc, int mode,
                                          const float* __restrict__ scale);

template <typename T>
__global__ void conv_pack_kernel(const float* __restrict__ w, int cout, int cin, int kh, int kw, void* __restrict__ out,
                                 int kpad, int kc, int mode, const float* __restrict__ scale) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= pack_total(cout, cin, kh, kw, kpad, mode)) return;
  pack_elem<T>(e, w, cout, cin, kh, kw, out, kpad, kc, mode, scale);
}

// every pack of a training plan's pack tape in one launch: block row y = pack y of the table,
// the x blocks stride over its elements (the dtype per entry, uniform per block)
__global__ void conv_pack_batch_kernel(const dp_pack_desc* __restrict__ tab) {
  const dp_pack_desc d = tab[blockIdx.y];
  const int64_t total = pack_total(d.cout, d.cin, d.kh, d.kw, d.kpad, d.mode);
  const int kc = d.kc > 0 ? d.kc : (d.mode == 0 ? d.cin : d.cout);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    if (d.dtype == DP_BF16) pack_elem<bf16_t>(e, d.w, d.cout, d.cin, d.kh, d.kw, d.out, d.kpad, kc, d.mode, d.scale);
    else pack_elem<float>(e, d.w, d.cout, d.cin, d.kh, d.kw, d.out, d.kpad, kc, d.mode, d.scale);
  }
}

template <typename T>
__device__ __forceinline__ void pack_elem(int64_t e, const float* __restrict__ w, int cout, int cin, int kh, int kw,
                                          void* __restrict__ out, int kpad, int kc, int mode,
                                          const float* __restrict__ scale) {
  if (mode == 5) {
    reinterpret_cast<T*>(out)[e] = from_f32<T>(w[e]);
    return;
  }
  if (mode == 2) {
    const int tap = (int)(e / cout), ch = (int)(e % cout);
    reinterpret_cast<float*>(out)[e] = w[(int64_t)ch * kh * kw + tap] * (scale ? scale[ch] : 1.f);
    return;
  }
  if (mode == 3) {
    const int K = cin * kh * kw;
    reinterpret_cast<float*>(out)[e] = w[e] * (scale ? scale[e / K] : 1.f);
    return;
  }
  if (mode == 4) {
    const int r = (int)(e / kpad), j = (int)(e % kpad);
    const int tap = r / cin, ci = r - tap * cin;
    const float v = j < cout ? w[((int64_t)j * cin + ci) * kh * kw + tap] * (scale ? scale[j] : 1.f) : 0.f;
    reinterpret_cast<T*>(out)[e] = from_f32<T>(v);
    return;
  }
  const int inner = mode == 0 ? cin : cout;
  const int r = (int)(e / kpad), k = (int)(e % kpad);
  float v = 0.f;
  const int tap = k / kc, j = k - tap * kc;
  if (tap < kh * kw && j < inner) {
    const int ky = tap / kw, kx = tap - ky * kw;
    v = mode == 0 ? w[(((int64_t)r * cin + j) * kh + ky) * kw + kx] * (scale ? scale[r] : 1.f)
                  : w[(((int64_t)j * cin + r) * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)] * (scale ? scale[j] : 1.f);
  }
  reinterpret_cast<T*>(out)[e] = from_f32<T>(v);
}

// depthwise conv backward (SCDown's 3x3 s2, hybrid_encoder.py:156-170; HGNetv2's 3x3 s2
// downsample and 5x5 / 3x3 LightConvBNAct, hgnetv2.py:144-163). A lane = VC consecutive channels
// (one VC-element vector load per pixel: 8 bytes for bf16 at VC = 4), a wave = 64 such chunks of
// one row tile of DW_TW pixels; K, S compile-time so the taps, the tile and the accumulators live
// in registers. dx (+=): stride 1 slides a register window of the dz row over the tile; dw (+=):
// a thread sums its channels' K*K taps over the tiles it walks, the block's channels x K*K sums
// are transposed through LDS so the f32 atomics hit contiguous addresses of the [c][K][K]
// gradient. VC = 1 is the any-stride / any-alignment form.
constexpr int DW_TW = 8;

template <typename T, int K, int S, int VC>
__global__ __launch_bounds__(256) void dw_bwd_data_kernel(const T* __restrict__ dz, int64_t zbs, int zps,
                                                          const float* __restrict__ wt, int h, int w, int c, int pad,
                                                          int oh, int ow, T* __restrict__ dx, int64_t xbs, int xps,
                                                          int ntiles) {
  const int ch = (blockIdx.x * 64 + threadIdx.x) * VC;
  if (ch >= c) return;
  float wk[K * K][VC];
#pragma unroll
  for (int t = 0; t < K * K; ++t)
#pragma unroll
    for (int v = 0; v < VC; ++v) wk[t][v] = wt[t * c + ch + v];
  const int ntx = (w + DW_TW - 1) / DW_TW;
  for (int tt = blockIdx.y * 4 + threadIdx.y; tt < ntiles; tt += gridDim.y * 4) {
    const int x0 = (tt % ntx) * DW_TW, t2 = tt / ntx;
    const int y = t2 % h, b = t2 / h;
    const T* zb = dz + (int64_t)b * zbs + ch;
    float acc[DW_TW][VC];
#pragma unroll
    for (int i = 0; i < DW_TW; ++i)
#pragma unroll
      for (int v = 0; v < VC; ++v) acc[i][v] = 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ny = y + pad - ky;
      if (ny < 0 || ny % S) continue;
      const int oy = ny / S;
      if (oy >= oh) continue;
      const T* zr = zb + (int64_t)oy * ow * zps;
      if (S == 1) {
        // output x0 + i takes dz[ox = x0 + i + pad - kx]: window j = i + K - 1 - kx
        float zw[DW_TW + K - 1][VC];
#pragma unroll
        for (int j = 0; j < DW_TW + K - 1; ++j) {
          const int ox = x0 + pad - (K - 1) + j;
          ld_vec<T, VC>(zr + (int64_t)min(max(ox, 0), ow - 1) * zps, zw[j]);
          if (ox < 0 || ox >= ow)
#pragma unroll
            for (int v = 0; v < VC; ++v) zw[j][v] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < DW_TW; ++i)
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int v = 0; v < VC; ++v) acc[i][v] = fmaf(zw[i + K - 1 - kx][v], wk[ky * K + kx][v], acc[i][v]);
      } else {
#pragma unroll
        for (int i = 0; i < DW_TW; ++i)
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            const int nx = x0 + i + pad - kx;
            const int ox = nx / S;
            float zv[VC];
            ld_vec<T, VC>(zr + (int64_t)min(max(ox, 0), ow - 1) * zps, zv);
            const bool ok = nx >= 0 && nx % S == 0 && ox < ow;
#pragma unroll
            for (int v = 0; v < VC; ++v) acc[i][v] = fmaf(ok ? zv[v] : 0.f, wk[ky * K + kx][v], acc[i][v]);
          }
      }
    }
    T* o = dx + (int64_t)b * xbs + (int64_t)y * w * xps + ch;
    float prev[DW_TW][VC];
#pragma unroll
    for (int i = 0; i < DW_TW; ++i) ld_vec<T, VC>(o + (int64_t)min(x0 + i, w - 1) * xps, prev[i]);
#pragma unroll
    for (int i = 0; i < DW_TW; ++i)
      if (x0 + i < w) {
        float r[VC];
#pragma unroll
        for (int v = 0; v < VC; ++v) r[v] = prev[i][v] + acc[i][v];
        st_vec<T, VC>(o + (int64_t)(x0 + i) * xps, r);
      }
  }
}

template <typename T, int K, int S, int VC>
__global__ __launch_bounds__(256) void dw_bwd_weight_kernel(const T* __restrict__ x, int64_t xbs, int xps,
                                                            const T* __restrict__ dz, int64_t zbs, int zps, int h,
                                                            int w, int c, int pad, int oh, int ow, int ntiles,
                                                            float* __restrict__ dw) {
  constexpr int XW = (DW_TW - 1) * S + K;
  constexpr int CB = 64 * VC;   // the block's channels
  __shared__ float red[CB * K * K];   // the four waves' sums, added in wave order
  const int ch = (blockIdx.x * 64 + threadIdx.x) * VC;
  const bool active = ch < c;
  float acc[K * K][VC];
#pragma unroll
  for (int t = 0; t < K * K; ++t)
#pragma unroll
    for (int v = 0; v < VC; ++v) acc[t][v] = 0.f;
  const int ntx = (ow + DW_TW - 1) / DW_TW;
  if (active) {
    for (int tt = blockIdx.y * 4 + threadIdx.y; tt < ntiles; tt += gridDim.y * 4) {
      const int ox0 = (tt % ntx) * DW_TW, t2 = tt / ntx;
      const int oy = t2 % oh, b = t2 / oh;
      float g[DW_TW][VC];
      const T* zr = dz + (int64_t)b * zbs + (int64_t)oy * ow * zps + ch;
#pragma unroll
      for (int i = 0; i < DW_TW; ++i) {
        ld_vec<T, VC>(zr + (int64_t)min(ox0 + i, ow - 1) * zps, g[i]);
        if (ox0 + i >= ow)
#pragma unroll
          for (int v = 0; v < VC; ++v) g[i][v] = 0.f;
      }
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        const int iy = oy * S - pad + ky;
        if (iy < 0 || iy >= h) continue;
        const T* xr = x + (int64_t)b * xbs + (int64_t)iy * w * xps + ch;
        float xw[XW][VC];
#pragma unroll
        for (int j = 0; j < XW; ++j) {
          const int ix = ox0 * S - pad + j;
          ld_vec<T, VC>(xr + (int64_t)min(max(ix, 0), w - 1) * xps, xw[j]);
          if (ix < 0 || ix >= w)
#pragma unroll
            for (int v = 0; v < VC; ++v) xw[j][v] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < DW_TW; ++i)
#pragma unroll
          for (int kx = 0; kx < K; ++kx)
#pragma unroll
            for (int v = 0; v < VC; ++v) acc[ky * K + kx][v] = fmaf(g[i][v], xw[i * S + kx][v], acc[ky * K + kx][v]);
      }
    }
  }
  // [channel][tap] order in LDS: the block's channels ch0 .. own dw[ch0*K*K ..] contiguously
  for (int wy = 0; wy < 4; ++wy) {
    if (threadIdx.y == wy) {
#pragma unroll
      for (int t = 0; t < K * K; ++t)
#pragma unroll
        for (int v = 0; v < VC; ++v) {
          float& r = red[(threadIdx.x * VC + v) * K * K + t];
          r = wy ? r + acc[t][v] : acc[t][v];
        }
    }
    __syncthreads();
  }
  const int ch0 = blockIdx.x * CB;
  const int n = min(CB, c - ch0) * K * K;
  for (int e = threadIdx.y * 64 + threadIdx.x; e < n; e += 256) atomicAdd(dw + (int64_t)ch0 * K * K + e, red[e]);
}

template <typename T, int K, int S, int VC>
void dw_bwd_launch(const void* x, int64_t xbs, int xps, const void* dz, int64_t zbs, int zps, const float* wt,
                   int batch, int h, int w, int c, int pad, int oh, int ow, void* dx, int64_t dxbs, int dxps,
                   float* dw, hipStream_t s) {
  const unsigned gx = (unsigned)((c + 64 * VC - 1) / (64 * VC));
  if (dx) {
    const int ntiles = batch * h * ((w + DW_TW - 1) / DW_TW);
    const unsigned gy = (unsigned)std::min((ntiles + 3) / 4, 65535);
    hipLaunchKernelGGL((dw_bwd_data_kernel<T, K, S, VC>), dim3(gx, gy), dim3(64, 4), 0, s, (const T*)dz, zbs, zps, wt,
                       h, w, c, pad, oh, ow, (T*)dx, dxbs, dxps, ntiles);
  }
  if (dw) {
    const int ntiles = batch * oh * ((ow + DW_TW - 1) / DW_TW);
    // about 4 tiles per thread: enough waves to fill the chip, the atomics a small fraction
    // (capping the row blocks at 64 / 32 to shorten the atomic chains measured 1.4x / 2.1x slower)
    const unsigned gy = (unsigned)std::max(1, std::min((ntiles + 15) / 16, 65535));
    hipLaunchKernelGGL((dw_bwd_weight_kernel<T, K, S, VC>), dim3(gx, gy), dim3(64, 4), 0, s, (const T*)x, xbs, xps,
                       (const T*)dz, zbs, zps, h, w, c, pad, oh, ow, ntiles, dw);
  }
}

// ---------------------------------------------------------------- rows
// nearest x2 (F.interpolate(scale_factor=2, nearest), hybrid_encoder.py:487): forward copy and
// its backward (2x2 sum, +=)
template <typename T>
__global__ void up2_kernel(const T* __restrict__ src, int64_t sbs, int sps, int h, int w, int c, T* __restrict__ dst,
                           int64_t dbs, int dps, int bwd, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over the small map
  if (e >= total) return;
  const int ch = (int)(e % c);
  const int64_t p = e / c;
  const int x = (int)(p % w);
  const int64_t t = p / w;
  const int y = (int)(t % h), b = (int)(t / h);
  const int64_t big[4] = {((int64_t)(2 * y) * (2 * w) + 2 * x), ((int64_t)(2 * y) * (2 * w) + 2 * x + 1),
                          ((int64_t)(2 * y + 1) * (2 * w) + 2 * x), ((int64_t)(2 * y + 1) * (2 * w) + 2 * x + 1)};
  if (!bwd) {
    const T v = src[(int64_t)b * sbs + ((int64_t)y * w + x) * sps + ch];
    for (int q = 0; q < 4; ++q) dst[(int64_t)b * dbs + big[q] * dps + ch] = v;
  } else {   // src = d big map, dst = d small map (+=)
    float acc = 0.f;
    for (int q = 0; q < 4; ++q) acc += ld_(src + (int64_t)b * sbs + big[q] * sps + ch);
    T* o = dst + (int64_t)b * dbs + ((int64_t)y * w + x) * dps + ch;
    *o = from_f32<T>(ld_(o) + acc);
  }
}

// y (=|+=) alpha a [+ beta b]: residual adds and their backward (gradient fan-out)
template <typename T, bool HB, bool ACC>
__global__ __launch_bounds__(256) void axpby_kernel(T* __restrict__ y, int64_t ldy, const T* __restrict__ a, int64_t lda,
                                                    float alpha, const T* __restrict__ b, int64_t ldb, float beta,
                                                    int rows, int c) {
  const int ch = blockIdx.y * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  for (int r0 = blockIdx.x; r0 < rows; r0 += RU * gridDim.x) {
    float va[RU], vb[RU], vy[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t r = min(r0 + u * (int)gridDim.x, rows - 1);
      va[u] = ld_(a + r * lda + ch);
      vb[u] = HB ? ld_(b + r * ldb + ch) : 0.f;
      vy[u] = ACC ? ld_(y + r * ldy + ch) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = r0 + u * gridDim.x;
      float v = alpha * va[u];
      if (HB) v = fmaf(beta, vb[u], v);
      if (r < rows) y[(int64_t)r * ldy + ch] = from_f32<T>(ACC ? vy[u] + v : v);
    }
  }
}

// dx = dy * act'(pre) (the AIFI FFN's GELU, hybrid_encoder.py:292)
template <typename T>
__global__ __launch_bounds__(256) void act_bwd_kernel(const T* __restrict__ pre, int64_t ldp, const T* __restrict__ dy,
                                                      int64_t ldy, T* __restrict__ dx, int64_t ldx, int rows, int c,
                                                      int act) {
  const int ch = blockIdx.y * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  for (int r0 = blockIdx.x; r0 < rows; r0 += RU * gridDim.x) {
    float vp[RU], vg[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t r = min(r0 + u * (int)gridDim.x, rows - 1);
      vp[u] = ld_(pre + r * ldp + ch);
      vg[u] = ld_(dy + r * ldy + ch);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int r = r0 + u * gridDim.x;
      if (r < rows) dx[(int64_t)r * ldx + ch] = from_f32<T>(vg[u] * act_d(vp[u], act));
    }
  }
}

// (row slices, channel blocks) of a row kernel: blockDim.x = the channels rounded to a wave (at
// most 256), about 512 K threads per launch (8 waves per SIMD), each at least RU rows
struct RC {
  dim3 grid, block;
};
RC rc_grid(int rows, int c) {
  const int bx = c >= 256 ? 256 : (c + 63) / 64 * 64;
  const int gy = (c + bx - 1) / bx;
  int gx = (1 << 19) / (bx * gy);
  if (gx > (rows + RU - 1) / RU) gx = (rows + RU - 1) / RU;
  if (gx < 1) gx = 1;
  return {dim3((unsigned)gx, (unsigned)gy), dim3((unsigned)bx)};
}

int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace

#define DP_DT(CALL)                    \
  do {                                 \
    if (dtype == DP_BF16) {            \
      using T = bf16_t;                \
      CALL;                            \
    } else {                           \
      using T = float;                 \
      CALL;                            \
    }                                  \
  } while (0)

// row slices of dp_bn_stats: 256-row slices, or longer ones (multiples of 32 rows) when a map
// would need more than max(64, 2048 / channel blocks) of them: about 2048 blocks fill the chip,
// and the reduction stays a few rounds of loads per wave
inline int bn_slice_rows(int rows, int c) {
  const int cb = (c + 63) / 64, cap = std::max(64, 2048 / cb);
  const int per = (rows + cap - 1) / cap;
  return std::max(256, (per + 31) / 32 * 32);
}

extern "C" int64_t dp_bn_stats_ws_bytes(int32_t rows, int32_t c) {
  if (rows <= 0 || c <= 0) return -1;
  const int sl = bn_slice_rows(rows, c);
  return (int64_t)((rows + sl - 1) / sl) * 2 * c * (int64_t)sizeof(float);
}

static int bn_stats_launch(const void* x, int64_t ld, int32_t rows, int32_t c, float* out, float* ws,
                           int64_t ws_bytes, int32_t dtype, hipStream_t s, const BnFin& fin) {
  DP_REQUIRE(x && out && ws && rows > 0 && c > 0 && ld >= c, "dp_bn_stats: bad arguments");
  DP_REQUIRE(ws_bytes >= dp_bn_stats_ws_bytes(rows, c), "dp_bn_stats: workspace of %lld bytes < %lld",
             (long long)ws_bytes, (long long)dp_bn_stats_ws_bytes(rows, c));
  const int sl = bn_slice_rows(rows, c), ny = (rows + sl - 1) / sl;
  dim3 grid((c + 63) / 64, ny);
  DP_DT(hipLaunchKernelGGL(bn_stats_kernel<T>, grid, dim3(256), 0, s, (const T*)x, ld, rows, c, sl, ws));
  DP_DT(hipLaunchKernelGGL(bn_stats_reduce_kernel<T>, dim3((c + 63) / 64), dim3(1024), 0, s, (const T*)x, ws, ny, c,
                           out, fin));
  return dp_check_launch("dp_bn_stats");
}

extern "C" int dp_bn_stats(const void* x, int64_t ld, int32_t rows, int32_t c, float* out, float* ws, int64_t ws_bytes,
                           int32_t dtype, void* stream) {
  return bn_stats_launch(x, ld, rows, c, out, ws, ws_bytes, dtype, as_stream(stream), BnFin{0.f, 0.f, 0.f, nullptr,
                                                                                           nullptr, nullptr});
}

extern "C" int dp_bn_stats_finalize(const void* x, int64_t ld, int32_t rows, int32_t c, float* out, float* ws,
                                    int64_t ws_bytes, float eps, float momentum, float* running_mean,
                                    float* running_var, float* mean_rstd, int32_t dtype, void* stream) {
  DP_REQUIRE(mean_rstd && (!running_mean == !running_var), "dp_bn_stats_finalize: bad arguments");
  return bn_stats_launch(x, ld, rows, c, out, ws, ws_bytes, dtype, as_stream(stream),
                         BnFin{(float)rows, eps, momentum, running_mean, running_var, mean_rstd});
}

extern "C" int dp_bn_finalize(const float* parts, int32_t nparts, float count, int32_t c, float eps, float momentum,
                              float* running_mean, float* running_var, float* mean_rstd, void* stream) {
  DP_REQUIRE(parts && nparts > 0 && count > 0.f && c > 0 && mean_rstd && (!running_mean == !running_var),
             "dp_bn_finalize: bad arguments");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((c + 255) / 256), dim3(256), 0, as_stream(stream), parts, nparts, count,
                     c, eps, momentum, running_mean, running_var, mean_rstd);
  return dp_check_launch("dp_bn_finalize");
}

extern "C" int dp_bn_act_fwd(void* y, int64_t ld_y, const void* z1, int64_t ld1, const float* mr1, const float* g1,
                             const float* b1, const void* z2, int64_t ld2, const float* mr2, const float* g2,
                             const float* b2, const void* res, int64_t ld_res, int32_t rows, int32_t c, int32_t act,
                             int32_t dtype, void* stream) {
  DP_REQUIRE(y && z1 && mr1 && g1 && b1 && rows > 0 && c > 0 && (!z2 || (mr2 && g2 && b2)),
             "dp_bn_act_fwd: bad arguments");
  const BnBranch p1{z1, ld1, mr1, g1, b1}, p2{z2, ld2, mr2, g2, b2};
  const RC g = rc_grid(rows, c);
#define BNF(TW_, RS_)                                                                                           \
  DP_DT(hipLaunchKernelGGL((bn_act_fwd_kernel<T, TW_, RS_>), g.grid, g.block, 0, as_stream(stream), (T*)y, ld_y, p1, \
                           p2, (const T*)res, ld_res, rows, c, act))
  if (z2) {
    if (res) BNF(true, true); else BNF(true, false);
  } else {
    if (res) BNF(false, true); else BNF(false, false);
  }
#undef BNF
  return dp_check_launch("dp_bn_act_fwd");
}

extern "C" int64_t dp_bn_act_bwd_reduce_ws_bytes(int32_t rows, int32_t c) {
  if (rows <= 0 || c <= 0) return -1;
  return (int64_t)((rows + 255) / 256) * 3 * c * (int64_t)sizeof(float);
}

extern "C" int dp_bn_act_bwd_reduce(const void* dy, int64_t ld_dy, const void* z1, int64_t ld1, const float* mr1,
                                    const float* g1, const float* b1, const void* z2, int64_t ld2, const float* mr2,
                                    const float* g2, const float* b2, int32_t rows, int32_t c, int32_t act,
                                    float* sums, float* dg1, float* db1, float* dg2, float* db2, float* ws,
                                    int64_t ws_bytes, int32_t dtype, void* stream) {
  DP_REQUIRE(dy && z1 && mr1 && g1 && b1 && sums && ws && rows > 0 && c > 0 && (!z2 || (mr2 && g2 && b2)),
             "dp_bn_act_bwd_reduce: bad arguments");
  DP_REQUIRE(ws_bytes >= dp_bn_act_bwd_reduce_ws_bytes(rows, c), "dp_bn_act_bwd_reduce: workspace of %lld bytes < %lld",
             (long long)ws_bytes, (long long)dp_bn_act_bwd_reduce_ws_bytes(rows, c));
  hipStream_t s = as_stream(stream);
  const BnBranch p1{z1, ld1, mr1, g1, b1}, p2{z2, ld2, mr2, g2, b2};
  // 256-row slices into the workspace, then one fixed-order pass over them (no float atomics:
  // the same sums on every run; capping the slices instead measured slower)
  const int cb = (c + 63) / 64, per = 256, ny = (rows + per - 1) / per;
  dim3 grid(cb, ny);
  if (z2)
    DP_DT(hipLaunchKernelGGL((bn_act_bwd_reduce_kernel<T, true>), grid, dim3(256), 0, s, (const T*)dy, ld_dy, p1, p2,
                             rows, c, act, per, ws));
  else
    DP_DT(hipLaunchKernelGGL((bn_act_bwd_reduce_kernel<T, false>), grid, dim3(256), 0, s, (const T*)dy, ld_dy, p1, p2,
                             rows, c, act, per, ws));
  hipLaunchKernelGGL(bn_act_bwd_sum_kernel, dim3(cb), dim3(1024), 0, s, ws, ny, c, sums, dg1, db1, dg2, db2);
  return dp_check_launch("dp_bn_act_bwd_reduce");
}

extern "C" int dp_bn_act_bwd_apply(void* dz1, int64_t ld_dz1, void* dz2, int64_t ld_dz2, const void* dy, int64_t ld_dy,
                                   const void* z1, int64_t ld1, const float* mr1, const float* g1, const float* b1,
                                   const void* z2, int64_t ld2, const float* mr2, const float* g2, const float* b2,
                                   int32_t rows, int32_t c, int32_t act, const float* sums, float count, int32_t dtype,
                                   void* stream) {
  DP_REQUIRE(dz1 && dy && z1 && mr1 && g1 && b1 && sums && rows > 0 && c > 0 && count > 0.f &&
                 (!z2 || (mr2 && g2 && b2 && dz2)),
             "dp_bn_act_bwd_apply: bad arguments");
  const BnBranch p1{z1, ld1, mr1, g1, b1}, p2{z2, ld2, mr2, g2, b2};
  const RC g = rc_grid(rows, c);
  if (z2)
    DP_DT(hipLaunchKernelGGL((bn_act_bwd_apply_kernel<T, true>), g.grid, g.block, 0, as_stream(stream), (T*)dz1,
                             ld_dz1, (T*)dz2, ld_dz2, (const T*)dy, ld_dy, p1, p2, rows, c, act, sums, 1.f / count));
  else
    DP_DT(hipLaunchKernelGGL((bn_act_bwd_apply_kernel<T, false>), g.grid, g.block, 0, as_stream(stream), (T*)dz1,
                             ld_dz1, (T*)nullptr, ld_dz2, (const T*)dy, ld_dy, p1, p2, rows, c, act, sums,
                             1.f / count));
  return dp_check_launch("dp_bn_act_bwd_apply");
}

extern "C" int dp_im2col(const void* x, int64_t bstride, int32_t pstride, int64_t cstride, int32_t batch, int32_t h,
                         int32_t w, int32_t cin, int32_t kh, int32_t kw, int32_t stride, int32_t pad, int32_t oh,
                         int32_t ow, void* col, int32_t x_dtype, int32_t dtype, void* stream) {
  DP_REQUIRE(x && col && batch > 0 && cin > 0 && kh > 0 && kw > 0 && stride > 0 && oh > 0 && ow > 0,
             "dp_im2col: bad arguments");
  const int64_t total = (int64_t)batch * oh * ow * cin;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (x_dtype == DP_F32)
    DP_DT(hipLaunchKernelGGL((im2col_kernel<float, T>), grid, dim3(256), 0, as_stream(stream), (const float*)x,
                             bstride, pstride, cstride, h, w, cin, kh, kw, stride, pad, oh, ow, (T*)col, total));
  else
    DP_DT(hipLaunchKernelGGL((im2col_kernel<bf16_t, T>), grid, dim3(256), 0, as_stream(stream), (const bf16_t*)x,
                             bstride, pstride, cstride, h, w, cin, kh, kw, stride, pad, oh, ow, (T*)col, total));
  return dp_check_launch("dp_im2col");
}

extern "C" int dp_conv_pack(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw, void* out, int32_t kpad,
                            int32_t kc, int32_t mode, const float* scale, int32_t dtype, void* stream) {
  if (kc <= 0) kc = mode == 0 ? cin : cout;
  DP_REQUIRE(w && out && cout > 0 && cin > 0 && mode >= 0 && mode <= 4 &&
                 (mode == 2 ? cin == 1 : mode == 3 || (mode == 4 ? kpad >= cout : kc >= (mode == 0 ? cin : cout) &&
                                                                                    kpad >= kh * kw * kc)),
             "dp_conv_pack: bad arguments");
  const int64_t total = mode == 2 ? (int64_t)cout * kh * kw
                        : mode == 3 ? (int64_t)cout * cin * kh * kw
                        : mode == 4 ? (int64_t)kh * kw * cin * kpad
                                    : (int64_t)(mode == 0 ? cout : cin) * kpad;
  DP_DT(hipLaunchKernelGGL(conv_pack_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                           w, cout, cin, kh, kw, out, kpad, kc, mode, scale));
  return dp_check_launch("dp_conv_pack");
}

// the pack table's entries as dp_conv_pack would accept them one by one (mode 5: cout elements
// copied f32 -> dtype); mode 2 / 3 pack f32
extern "C" int dp_conv_pack_check(const dp_pack_desc* tab, int32_t n) {
  DP_REQUIRE(tab && n > 0 && n < 65536, "dp_conv_pack_check: bad table");
  for (int i = 0; i < n; ++i) {
    const dp_pack_desc& d = tab[i];
    const int kc = d.kc > 0 ? d.kc : (d.mode == 0 ? d.cin : d.cout);
    const bool ok = d.w && d.out && d.cout > 0 && d.cin > 0 && d.kh > 0 && d.kw > 0 && d.mode >= 0 && d.mode <= 5 &&
                    (d.dtype == DP_BF16 || d.dtype == DP_F32) && (d.mode != 2 && d.mode != 3 || d.dtype == DP_F32) &&
                    (d.mode == 2 ? d.cin == 1
                     : d.mode == 3 || d.mode == 5 ? true
                     : d.mode == 4 ? d.kpad >= d.cout
                                   : kc >= (d.mode == 0 ? d.cin : d.cout) && d.kpad >= d.kh * d.kw * kc);
    DP_REQUIRE(ok, "dp_conv_pack_check: entry %d (mode %d, cout %d, cin %d, k %dx%d, kpad %d, kc %d, dtype %d)", i, d.mode,
               d.cout, d.cin, d.kh, d.kw, d.kpad, d.kc, d.dtype);
  }
  return 0;
}

extern "C" int dp_conv_pack_batch(const dp_pack_desc* tab_dev, int32_t n, int32_t blocks_per_pack, void* stream) {
  DP_REQUIRE(tab_dev && n > 0 && n < 65536 && blocks_per_pack > 0, "dp_conv_pack_batch: bad arguments");
  hipLaunchKernelGGL(conv_pack_batch_kernel, dim3((unsigned)blocks_per_pack, (unsigned)n), dim3(256), 0,
                     as_stream(stream), tab_dev);
  return dp_check_launch("dp_conv_pack_batch");
}

extern "C" int dp_dwconv_bwd(const void* x, int64_t x_bstride, int32_t x_pstride, const void* dz, int64_t z_bstride,
                             int32_t z_pstride, const float* wt, int32_t batch, int32_t h, int32_t w, int32_t c,
                             int32_t k, int32_t stride, int32_t pad, int32_t oh, int32_t ow, void* dx,
                             int64_t dx_bstride, int32_t dx_pstride, float* dw, int32_t dtype, void* stream) {
  DP_REQUIRE(x && dz && wt && batch > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0,
             "dp_dwconv_bwd: bad arguments");
  DP_REQUIRE((k == 3 || k == 5) && (stride == 1 || stride == 2), "dp_dwconv_bwd: k %d stride %d (3 / 5, 1 / 2)", k,
             stride);
  hipStream_t s = as_stream(stream);
  // 4-channel vectors for the stride-2 convs when every row of channels is 4-aligned: L b16 tapes
  // 0.348 -> 0.314 ms for the downsamples; the 5x5 stride-1 LightConvs are faster scalar (1.13 vs
  // 1.25 ms: 220-240 VGPRs at 4 channels). DETRPOSE_DW_BWD_VEC = 0 (never) / 2 (always): A/B.
  static const int vec_env = getenv("DETRPOSE_DW_BWD_VEC") ? atoi(getenv("DETRPOSE_DW_BWD_VEC")) : 1;
  const int esz = dtype == DP_BF16 ? 2 : 4;
  auto al = [&](const void* p) { return !p || (reinterpret_cast<uintptr_t>(p) & (4 * esz - 1)) == 0; };
  const bool vec = (vec_env == 2 || (vec_env == 1 && stride == 2)) && c % 4 == 0 && x_pstride % 4 == 0 && z_pstride % 4 == 0 && dx_pstride % 4 == 0 &&
                   x_bstride % 4 == 0 && z_bstride % 4 == 0 && dx_bstride % 4 == 0 && al(x) && al(dz) && al(dx) &&
                   al(wt);
#define DW_CASE(KK, SS)                                                                                          \
  if (k == KK && stride == SS) {                                                                                 \
    if (vec)                                                                                                     \
      DP_DT((dw_bwd_launch<T, KK, SS, 4>(x, x_bstride, x_pstride, dz, z_bstride, z_pstride, wt, batch, h, w, c, pad, \
                                         oh, ow, dx, dx_bstride, dx_pstride, dw, s)));                          \
    else                                                                                                         \
      DP_DT((dw_bwd_launch<T, KK, SS, 1>(x, x_bstride, x_pstride, dz, z_bstride, z_pstride, wt, batch, h, w, c, pad, \
                                         oh, ow, dx, dx_bstride, dx_pstride, dw, s)));                          \
  }
  DW_CASE(3, 1) else DW_CASE(3, 2) else DW_CASE(5, 1) else DW_CASE(5, 2)
#undef DW_CASE
  return dp_check_launch("dp_dwconv_bwd");
}

extern "C" int dp_upsample2x(const void* src, int64_t src_bstride, int32_t src_pstride, int32_t batch, int32_t h,
                             int32_t w, int32_t c, void* dst, int64_t dst_bstride, int32_t dst_pstride,
                             int32_t backward, int32_t dtype, void* stream) {
  DP_REQUIRE(src && dst && batch > 0 && h > 0 && w > 0 && c > 0, "dp_upsample2x: bad arguments");
  const int64_t total = (int64_t)batch * h * w * c;
  DP_DT(hipLaunchKernelGGL(up2_kernel<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                           (const T*)src, src_bstride, src_pstride, h, w, c, (T*)dst, dst_bstride, dst_pstride,
                           backward, total));
  return dp_check_launch("dp_upsample2x");
}

extern "C" int dp_axpby_rows(void* y, int64_t ld_y, const void* a, int64_t ld_a, float alpha, const void* b,
                             int64_t ld_b, float beta, int32_t rows, int32_t c, int32_t accumulate, int32_t dtype,
                             void* stream) {
  DP_REQUIRE(y && a && rows > 0 && c > 0, "dp_axpby_rows: bad arguments");
  if (rows == 1 && c > 65536) {   // one long row (the EMA over the flat parameters): 1024-wide rows
    const int main = c / 1024 * 1024, es = dtype == DP_BF16 ? 2 : 4;
    int rc = dp_axpby_rows(y, 1024, a, 1024, alpha, b, 1024, beta, main / 1024, 1024, accumulate, dtype, stream);
    if (rc || main == c) return rc;
    return dp_axpby_rows((char*)y + (int64_t)main * es, c - main, (const char*)a + (int64_t)main * es, c - main, alpha,
                         b ? (const char*)b + (int64_t)main * es : nullptr, c - main, beta, 1, c - main, accumulate,
                         dtype, stream);
  }
  const RC g = rc_grid(rows, c);
#define AXP(HB_, AC_)                                                                                            \
  DP_DT(hipLaunchKernelGGL((axpby_kernel<T, HB_, AC_>), g.grid, g.block, 0, as_stream(stream), (T*)y, ld_y,          \
                           (const T*)a, ld_a, alpha, (const T*)b, ld_b, beta, rows, c))
  if (b) {
    if (accumulate) AXP(true, true); else AXP(true, false);
  } else {
    if (accumulate) AXP(false, true); else AXP(false, false);
  }
#undef AXP
  return dp_check_launch("dp_axpby_rows");
}

extern "C" int dp_act_bwd(const void* pre, int64_t ld_pre, const void* dy, int64_t ld_dy, void* dx, int64_t ld_dx,
                          int32_t rows, int32_t c, int32_t act, int32_t dtype, void* stream) {
  DP_REQUIRE(pre && dy && dx && rows > 0 && c > 0, "dp_act_bwd: bad arguments");
  const RC g = rc_grid(rows, c);
  DP_DT(hipLaunchKernelGGL(act_bwd_kernel<T>, g.grid, g.block, 0, as_stream(stream), (const T*)pre, ld_pre,
                           (const T*)dy, ld_dy, (T*)dx, ld_dx, rows, c, act));
  return dp_check_launch("dp_act_bwd");
}
