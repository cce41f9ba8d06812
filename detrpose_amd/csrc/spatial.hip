// Bandwidth-bound spatial kernels of the HGNetv2 backbone / SCDown, NHWC:
//  * depthwise k x k conv + folded BN + act (LightConvBNAct.conv2, hgnetv2.py:137-166;
//    HG_Stage downsample, hgnetv2.py:349-358; SCDown.cv2, hybrid_encoder.py:130-137)
//  * StemBlock.stem1 3x3 s2 conv straight from the f32 NCHW image (hgnetv2.py:171-177)
//  * StemBlock's F.pad(0,1,0,1) + MaxPool2d(2,1,ceil_mode) (hgnetv2.py:215,217)
// These run at arithmetic intensity 2-12 FLOP/B, far under the MFMA ridge (~312), so
// they are plain 16-byte-vector VALU kernels with consecutive threads on consecutive
// channel chunks (coalesced pixel rows).
#include "common.h"
#include "conv_lds.h"
#include <stdlib.h>

namespace {

// Depthwise k x k, stride S: one thread = PX consecutive output pixels of one row x one
// 16-byte channel chunk. Per kernel row the (PX-1)*S+KS input pixels are loaded once and
// reused by all KS taps and PX outputs (register sliding window); the per-channel
// weights of a tap are read once for all PX outputs.
template <typename T, int KS, int S, int PX>
__global__ __launch_bounds__(256) void dwconv_kernel(dp_conv_desc d, int64_t total, int nchunk, int ntx) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int NIN = (PX - 1) * S + KS;
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;   // total < 2^31 (host check)
  if (gid >= (unsigned)total) return;
  unsigned rest = gid / (unsigned)nchunk;
  const int cc = (int)(gid - rest * (unsigned)nchunk);
  unsigned r2 = rest / (unsigned)ntx;
  const int tx = (int)(rest - r2 * (unsigned)ntx);
  const unsigned b_ = r2 / (unsigned)d.out_h;
  const int oy = (int)(r2 - b_ * (unsigned)d.out_h);
  const int b = (int)b_;
  const int ox0 = tx * PX;
  const int c0 = cc * VEC;
  const T* in = reinterpret_cast<const T*>(d.in) + (int64_t)b * d.in_bstride + c0;
  const float* w = reinterpret_cast<const float*>(d.weight) + c0;
  float acc[PX][VEC];
#pragma unroll
  for (int t = 0; t < VEC; ++t) {
    const float bv = d.bias ? d.bias[c0 + t] : 0.f;
#pragma unroll
    for (int p = 0; p < PX; ++p) acc[p][t] = bv;
  }
  const int iy0 = oy * S - d.pad_t, ix0 = ox0 * S - d.pad_l;
#pragma unroll
  for (int ky = 0; ky < KS; ++ky) {
    const int iy = iy0 + ky;
    if (iy < 0 || iy >= d.in_h) continue;
    Vec16<T> xin[NIN];
#pragma unroll
    for (int j = 0; j < NIN; ++j) {
      const int ix = ix0 + j;
      if (ix >= 0 && ix < d.in_w) xin[j] = load16(in + ((int64_t)iy * d.in_w + ix) * d.in_pstride);
      else *reinterpret_cast<uint4*>(&xin[j].v) = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int kx = 0; kx < KS; ++kx) {
      const float* wk = w + (ky * KS + kx) * d.cin;
      float wv[VEC];
#pragma unroll
      for (int t = 0; t < VEC; t += 4) *reinterpret_cast<float4*>(&wv[t]) = *reinterpret_cast<const float4*>(wk + t);
#pragma unroll
      for (int p = 0; p < PX; ++p)
#pragma unroll
        for (int t = 0; t < VEC; ++t) acc[p][t] = fmaf(xin[p * S + kx].get(t), wv[t], acc[p][t]);
    }
  }
  T* out = reinterpret_cast<T*>(d.out) + (int64_t)b * d.out_bstride + c0;
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    const int ox = ox0 + p;
    if (ox >= d.out_w) break;
    Vec16<T> o;
#pragma unroll
    for (int t = 0; t < VEC; ++t) {
      float v = apply_act(acc[p][t], d.act);
      if (d.has_lab) v = d.lab_scale * v + d.lab_bias;
      o.set(t, v);
    }
    store16(out + ((int64_t)oy * d.out_w + ox) * d.out_pstride, o);
  }
}

// One thread per output pixel, all COUT channels; image f32 NCHW, 3 channels. The
// weights are wave-uniform, so they are read with scalar loads (SGPR operands of the
// FMAs) rather than staged through LDS.
template <typename T, int COUT>
__global__ __launch_bounds__(256) void stem_conv_kernel(const float* __restrict__ img, int batch, int h, int w,
                                                        const float* __restrict__ wt, const float* __restrict__ bias,
                                                        int has_lab, float ls, float lb, T* __restrict__ out,
                                                        int64_t obs, int ops) {
  const int oh = (h + 1) / 2, ow = (w + 1) / 2;
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (unsigned)(batch * oh * ow)) return;
  const int b = (int)(gid / (unsigned)(oh * ow));
  const int rem = (int)(gid - (unsigned)b * (unsigned)(oh * ow));
  const int oy = rem / ow, ox = rem - oy * ow;
  float x[27];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iy = 2 * oy - 1 + ky, ix = 2 * ox - 1 + kx;
        const bool ok = iy >= 0 && iy < h && ix >= 0 && ix < w;
        x[(c * 3 + ky) * 3 + kx] = ok ? img[(((int64_t)b * 3 + c) * h + iy) * w + ix] : 0.f;
      }
  T* o = out + (int64_t)b * obs + (int64_t)rem * ops;
#pragma unroll
  for (int n0 = 0; n0 < COUT; n0 += 8) {
    float r[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      float a = bias[n0 + t];
#pragma unroll
      for (int k = 0; k < 27; ++k) a = fmaf(x[k], wt[(n0 + t) * 27 + k], a);
      a = fmaxf(a, 0.f);
      if (has_lab) a = ls * a + lb;
      r[t] = a;
    }
    constexpr int V = Vec16<T>::N;
#pragma unroll
    for (int h0 = 0; h0 < 8; h0 += V) {
      Vec16<T> v;
#pragma unroll
      for (int t = 0; t < V; ++t) v.set(t, r[h0 + t]);
      store16(o + n0 + h0, v);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_kernel(const T* __restrict__ in, int64_t ibs, int ips, int batch, int h,
                                                      int w, int c, T* __restrict__ out, int64_t obs, int ops) {
  constexpr int VEC = Vec16<T>::N;
  const int nchunk = c / VEC;
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (unsigned)(batch * h * w * nchunk)) return;
  const unsigned pix = gid / (unsigned)nchunk;
  const int cc = (int)(gid - pix * (unsigned)nchunk);
  const int b = (int)(pix / (unsigned)(h * w));
  const int rem = (int)(pix - (unsigned)b * (unsigned)(h * w));
  const int y = rem / w, x = rem - y * w;
  const T* base = in + (int64_t)b * ibs + cc * VEC;
  float m[VEC];
#pragma unroll
  for (int t = 0; t < VEC; ++t) m[t] = -INFINITY;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int yy = y + dy, xx = x + dx;
      if (yy < h && xx < w) {
        Vec16<T> v = load16(base + ((int64_t)yy * w + xx) * ips);
#pragma unroll
        for (int t = 0; t < VEC; ++t) m[t] = fmaxf(m[t], v.get(t));
      } else {
#pragma unroll
        for (int t = 0; t < VEC; ++t) m[t] = fmaxf(m[t], 0.f);  // the F.pad zero takes part in the max
      }
    }
  Vec16<T> o;
#pragma unroll
  for (int t = 0; t < VEC; ++t) o.set(t, m[t]);
  store16(out + (int64_t)b * obs + (int64_t)rem * ops + cc * VEC, o);
}


// Depthwise k x k, bf16, LDS-tiled (production path for channels % 64 == 0): a tile is TH x
// TW output pixels x 64 channels. The ((TH-1)S+KS) x ((TW-1)S+KS) input patch is read ONCE
// with whole 128-byte pixel lines (8 lanes per pixel) into LDS by LDS-DMA (zeros outside the
// map = the conv padding), then each thread computes PX consecutive outputs of one 16-byte
// channel chunk from LDS with a register sliding window per kernel row.
// Persistent blocks, double-buffered patches: a block keeps ONE 64-channel chunk (its tap
// weights and biases stay in LDS / registers) and walks that chunk's tiles; the next tile's
// patch is DMA'd while the current one computes, so the patch latency (the whole cost of a
// one-tile block on the 40x40 5x5 convs) overlaps the FMAs. Block order is XCD-sliced
// (logical = (blockIdx % 8) * (G / 8) + blockIdx / 8): the tiles sharing halo rows run on one
// XCD at about the same time and re-read the halo from its L2.
template <int KS, int S, int TH, int TW, int PX, bool PERSIST, int ACT>
__global__ __launch_bounds__(256) void dwconv_lds_kernel(dp_conv_desc d, int tiles_x, int tiles_y, int nchk,
                                                         int ntiles) {
  constexpr int PH = (TH - 1) * S + KS, PW = (TW - 1) * S + KS;
  constexpr int NIN = (PX - 1) * S + KS;
  constexpr int GX = TW / PX;
  constexpr int PBYTES = (PH * PW * 128 + 1023) / 1024 * 1024;   // DMA groups are whole 1 KB
  // (a one-tile-per-block launch allocates one buffer: the prefetch below never fires there)
  static_assert(TW % PX == 0, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];     // [2][patch] + weights
  const int G = gridDim.x;                                        // multiple of 8 * nchk
  const int L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int ck = L % nchk;
  const int spatial = ntiles / nchk;                              // tiles of this chunk
  const int first = L / nchk, step = G / nchk;
  if (first >= spatial) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  float* wl = reinterpret_cast<float*>(smem + (PERSIST ? 2 : 1) * PBYTES);

  auto issue_patch = [&](int t, char* patch) {
    int rest = t;
    const int tx = rest % tiles_x;
    rest /= tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int iy0 = ty * TH * S - d.pad_t, ix0 = tx * TW * S - d.pad_l;
    const dpconv::i32x4 rs =
        dpconv::make_rsrc(reinterpret_cast<const bf16_t*>(d.in) + (int64_t)b * d.in_bstride + ck * 64);
    constexpr int NE = PH * PW * 8;
    for (int e0 = wave * 64; e0 < NE; e0 += 256) {
      const int e = e0 + lane;
      const int px = e >> 3, c = e & 7;
      const int py = px / PW, pxx = px - py * PW;
      const int iy = iy0 + py, ix = ix0 + pxx;
      const bool ok = e < NE && (unsigned)iy < (unsigned)d.in_h && (unsigned)ix < (unsigned)d.in_w;
      const int o = ok ? ((iy * d.in_w + ix) * d.in_pstride + c * 8) * 2 : dpconv::OOB;
      dpconv::dma16(rs, patch + e0 * 16, o);
    }
  };

  issue_patch(first, smem);
  // the chunk's 64 channels of the KS*KS tap weights (f32), and this thread's 8 biases
  for (int e = tid; e < KS * KS * 16; e += 256) {
    const int tap = e >> 4, q = e & 15;
    *reinterpret_cast<f32x4*>(wl + tap * 64 + 4 * q) =
        *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(d.weight) + tap * d.cin + ck * 64 + 4 * q);
  }
  const int c = tid & 7, c0 = c * 8;   // items it = tid + 256 k all have chunk tid & 7
  float bias[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) bias[t] = d.bias ? d.bias[ck * 64 + c0 + t] : 0.f;
  dpconv::wait_vmcnt<0>();
  __syncthreads();

  int u = 0;
  for (int t = first; t < spatial; t += step, ++u) {
    // next tile's patch into the other buffer (its previous readers passed the barrier below)
    if (PERSIST && t + step < spatial) issue_patch(t + step, smem + ((u + 1) & 1) * PBYTES);
    const char* patch = smem + (PERSIST ? (u & 1) * PBYTES : 0);
    int rest = t;
    const int tx = rest % tiles_x;
    rest /= tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int oy0 = ty * TH, ox0 = tx * TW;
    for (int it = tid; it < TH * GX * 8; it += 256) {
      const int pg = it >> 3;
      const int row = pg / GX, xg = pg - row * GX;
      const int oy = oy0 + row, oxb = ox0 + xg * PX;
      if (oy >= d.out_h || oxb >= d.out_w) continue;
      float acc[PX][8];
#pragma unroll
      for (int tt = 0; tt < 8; ++tt)
#pragma unroll
        for (int p = 0; p < PX; ++p) acc[p][tt] = bias[tt];
      // kernel rows double-buffered in registers: row ky+1's LDS reads are in flight while
      // row ky's FMAs run (a fully unrolled 5x5 needs more than 256 VGPRs)
      auto load_row = [&](int ky, bf16x8 (&x)[NIN]) __attribute__((always_inline)) {
        const char* prow = patch + ((row * S + ky) * PW + xg * PX * S) * 128 + c * 16;
#pragma unroll
        for (int j = 0; j < NIN; ++j) x[j] = *reinterpret_cast<const bf16x8*>(prow + j * 128);
      };
      auto fma_row = [&](int ky, const bf16x8 (&x)[NIN]) __attribute__((always_inline)) {
#pragma unroll
        for (int kx = 0; kx < KS; ++kx) {
          const float* wk = wl + (ky * KS + kx) * 64 + c0;
          const f32x4 w0 = *reinterpret_cast<const f32x4*>(wk), w1 = *reinterpret_cast<const f32x4*>(wk + 4);
          const float wv[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
          for (int p = 0; p < PX; ++p)
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) acc[p][tt] = fmaf((float)x[p * S + kx][tt], wv[tt], acc[p][tt]);
        }
      };
      bf16x8 xa[NIN], xb[NIN];
      load_row(0, xa);
#pragma unroll 1
      for (int ky = 0; ky < KS; ky += 2) {
        if (ky + 1 < KS) load_row(ky + 1, xb);
        fma_row(ky, xa);
        if (ky + 1 < KS) {
          if (ky + 2 < KS) load_row(ky + 2, xa);
          fma_row(ky + 1, xb);
        }
      }
      bf16_t* out = reinterpret_cast<bf16_t*>(d.out) + (int64_t)b * d.out_bstride + ck * 64 + c0;
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        const int ox = oxb + p;
        if (ox >= d.out_w) break;
        bf16x8 o;
#pragma unroll
        for (int tt = 0; tt < 8; ++tt) {
          float v = dpconv::act_t<ACT>(acc[p][tt]);
          if (d.has_lab) v = d.lab_scale * v + d.lab_bias;
          o[tt] = (bf16_t)v;
        }
        *reinterpret_cast<bf16x8*>(out + ((int64_t)oy * d.out_w + ox) * d.out_pstride) = o;
      }
    }
    // the next patch has landed (and this tile's stores are out); every wave is done with
    // this buffer before the following iteration DMAs into it
    dpconv::wait_vmcnt<0>();
    __syncthreads();
  }
}

// PERSIST: persistent blocks with double-buffered patches (the compute-heavy 5x5 / 3x3 s1
// convs); otherwise one tile per block and a single patch buffer, i.e. twice as many
// resident blocks (the HBM-bound stride-2 downsamples want the bytes in flight)
template <int KS, int S, int TH, int TW, int PX, bool PERSIST>
int launch_dw_lds(const dp_conv_desc& d, hipStream_t s) {
  constexpr int PH = (TH - 1) * S + KS, PW = (TW - 1) * S + KS;
  constexpr int lds = (PERSIST ? 2 : 1) * ((PH * PW * 128 + 1023) / 1024 * 1024) + KS * KS * 64 * 4;
  static_assert(lds <= 160 * 1024, "patch");
  const int tiles_x = (d.out_w + TW - 1) / TW, tiles_y = (d.out_h + TH - 1) / TH, nchk = d.cin / 64;
  const int64_t ntiles = (int64_t)d.batch * tiles_y * tiles_x * nchk;
  DP_REQUIRE(ntiles < (1ll << 30), "dp_dwconv2d: too many tiles");
  // whole groups of 8 * nchk blocks (one channel chunk per block); persistent: about the LDS
  // occupancy per CU, never more blocks than tiles
  const int per_cu = (160 * 1024) / lds;
  const int unit = 8 * nchk;
  const int64_t need = (ntiles + unit - 1) / unit * unit;
  int64_t grid = PERSIST ? (int64_t)per_cu * dpconv::num_cus() / unit * unit : need;
  if (grid > need) grid = need;
  if (grid < unit) grid = unit;
#define DP_DWL(A_)                                                                                          \
  hipLaunchKernelGGL((dwconv_lds_kernel<KS, S, TH, TW, PX, PERSIST, A_>), dim3((unsigned)grid), dim3(256), lds, s, d, \
                     tiles_x, tiles_y, nchk, (int)ntiles)
  switch (d.act) {
    case DP_ACT_RELU: DP_DWL(DP_ACT_RELU); break;
    case DP_ACT_SILU: DP_DWL(DP_ACT_SILU); break;
    case DP_ACT_GELU: DP_DWL(DP_ACT_GELU); break;
    default: DP_DWL(DP_ACT_NONE); break;
  }
#undef DP_DWL
  return dp_check_launch("dp_dwconv2d(lds)");
}

// One tile per block (the original form): the HBM-bound stride-2 downsamples, where many
// small resident blocks keep more bytes in flight than persistent double-buffered ones
// (A/B: s2.down 0.133 ms one-tile vs 0.148-0.170 persistent).
template <int KS, int S, int TH, int TW, int PX, int ACT>
__global__ __launch_bounds__(256) void dwconv_tile_kernel(dp_conv_desc d, int tiles_x, int tiles_y, int nchk,
                                                         int ntiles) {
  constexpr int PH = (TH - 1) * S + KS, PW = (TW - 1) * S + KS;
  constexpr int NIN = (PX - 1) * S + KS;
  constexpr int GX = TW / PX;
  static_assert(TW % PX == 0, "tile");
  extern __shared__ __attribute__((aligned(16))) char patch[];   // [PH][PW][128 B]
  const int G = gridDim.x;
  const int L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (L >= ntiles) return;
  const int ck = L % nchk;
  int rest = L / nchk;
  const int tx = rest % tiles_x;
  rest /= tiles_x;
  const int ty = rest % tiles_y, b = rest / tiles_y;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - d.pad_t, ix0 = ox0 * S - d.pad_l;
  const int tid = threadIdx.x;
  const bf16_t* in = reinterpret_cast<const bf16_t*>(d.in) + (int64_t)b * d.in_bstride + ck * 64;

  // ---- patch -> LDS by LDS-DMA: every 16-byte piece of the patch in flight at once
  // (no staging VGPRs); the buffer descriptor returns 0 for the out-of-map offsets
  {
    const int wave = tid >> 6, lane = tid & 63;
    const dpconv::i32x4 rs = dpconv::make_rsrc(in);
    constexpr int NE = PH * PW * 8;
    for (int e0 = wave * 64; e0 < NE; e0 += 256) {
      const int e = e0 + lane;
      const int px = e >> 3, c = e & 7;
      const int py = px / PW, pxx = px - py * PW;
      const int iy = iy0 + py, ix = ix0 + pxx;
      const bool ok = e < NE && (unsigned)iy < (unsigned)d.in_h && (unsigned)ix < (unsigned)d.in_w;
      const int o = ok ? ((iy * d.in_w + ix) * d.in_pstride + c * 8) * 2 : dpconv::OOB;
      dpconv::dma16(rs, patch + e0 * 16, o);
    }
  }
  // the block's 64 channels of the KS*KS tap weights (f32) behind the patch
  float* wl = reinterpret_cast<float*>(patch + (PH * PW * 128 + 1023) / 1024 * 1024);   // past the last DMA group
  for (int e = tid; e < KS * KS * 16; e += 256) {
    const int tap = e >> 4, q = e & 15;
    *reinterpret_cast<f32x4*>(wl + tap * 64 + 4 * q) =
        *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(d.weight) + tap * d.cin + ck * 64 + 4 * q);
  }
  dpconv::wait_vmcnt<0>();
  __syncthreads();

  // ---- compute: item = ((row * GX) + xg) * 8 + chunk
  const float* w = wl;
  for (int it = tid; it < TH * GX * 8; it += 256) {
    const int c = it & 7, pg = it >> 3;
    const int row = pg / GX, xg = pg - row * GX;
    const int oy = oy0 + row, oxb = ox0 + xg * PX;
    if (oy >= d.out_h || oxb >= d.out_w) continue;
    const int c0 = c * 8;
    float acc[PX][8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float bv = d.bias ? d.bias[ck * 64 + c0 + t] : 0.f;
#pragma unroll
      for (int p = 0; p < PX; ++p) acc[p][t] = bv;
    }
#pragma unroll 1
    for (int ky = 0; ky < KS; ++ky) {
      const char* prow = patch + ((row * S + ky) * PW + xg * PX * S) * 128 + c * 16;
      bf16x8 xin[NIN];
#pragma unroll
      for (int j = 0; j < NIN; ++j) xin[j] = *reinterpret_cast<const bf16x8*>(prow + j * 128);
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        const float* wk = w + (ky * KS + kx) * 64 + c0;
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wk), w1 = *reinterpret_cast<const f32x4*>(wk + 4);
        const float wv[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
        for (int p = 0; p < PX; ++p)
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[p][t] = fmaf((float)xin[p * S + kx][t], wv[t], acc[p][t]);
      }
    }
    bf16_t* out = reinterpret_cast<bf16_t*>(d.out) + (int64_t)b * d.out_bstride + ck * 64 + c0;
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      const int ox = oxb + p;
      if (ox >= d.out_w) break;
      bf16x8 o;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        float v = dpconv::act_t<ACT>(acc[p][t]);
        if (d.has_lab) v = d.lab_scale * v + d.lab_bias;
        o[t] = (bf16_t)v;
      }
      *reinterpret_cast<bf16x8*>(out + ((int64_t)oy * d.out_w + ox) * d.out_pstride) = o;
    }
  }
}

template <int KS, int S, int TH, int TW, int PX>
int launch_dw_tile(const dp_conv_desc& d, hipStream_t s) {
  constexpr int PH = (TH - 1) * S + KS, PW = (TW - 1) * S + KS;
  constexpr int lds = (PH * PW * 128 + 1023) / 1024 * 1024 + KS * KS * 64 * 4;   // DMA groups are whole 1 KB
  static_assert(lds <= 64 * 1024, "patch");
  const int tiles_x = (d.out_w + TW - 1) / TW, tiles_y = (d.out_h + TH - 1) / TH, nchk = d.cin / 64;
  const int64_t ntiles = (int64_t)d.batch * tiles_y * tiles_x * nchk;
  DP_REQUIRE(ntiles < (1ll << 30), "dp_dwconv2d: too many tiles");
  const int grid = (int)((ntiles + 7) / 8 * 8);
#define DP_DWL(A_)                                                                                          \
  hipLaunchKernelGGL((dwconv_tile_kernel<KS, S, TH, TW, PX, A_>), dim3(grid), dim3(256), lds, s, d, tiles_x, \
                     tiles_y, nchk, (int)ntiles)
  switch (d.act) {
    case DP_ACT_RELU: DP_DWL(DP_ACT_RELU); break;
    case DP_ACT_SILU: DP_DWL(DP_ACT_SILU); break;
    case DP_ACT_GELU: DP_DWL(DP_ACT_GELU); break;
    default: DP_DWL(DP_ACT_NONE); break;
  }
#undef DP_DWL
  return dp_check_launch("dp_dwconv2d(lds)");
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

#ifndef DP_DW5_TH
#define DP_DW5_TH 8    // output rows per 5x5 tile
#endif
#ifndef DP_DWS2_TH
#define DP_DWS2_TH 2   // output rows per 3x3 stride-2 tile (2: more, smaller blocks in flight; 2-3% over 4)
#endif

}  // namespace

extern "C" int dp_dwconv2d(const dp_conv_desc* dp, void* stream) {
  DP_REQUIRE(dp != nullptr, "dp_dwconv2d: null descriptor");
  const dp_conv_desc& d = *dp;
  const int VEC = d.dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE(d.cin == d.cout && d.cin % VEC == 0, "dp_dwconv2d: channels %d/%d must match and be a multiple of %d",
             d.cin, d.cout, VEC);
  DP_REQUIRE(d.in_pstride % VEC == 0 && d.out_pstride % VEC == 0 && d.in_bstride % VEC == 0 &&
                 d.out_bstride % VEC == 0 && al16(d.in) && al16(d.out) && al16(d.weight),
             "dp_dwconv2d: 16-byte alignment required");
  hipStream_t s = as_stream(stream);
  static const bool no_lds = getenv("DETRPOSE_DW_NO_LDS") != nullptr;
  if (d.dtype == DP_BF16 && d.cin % 64 == 0 && !no_lds) {
    // maps at most 20 wide (HGNetv2 stage 4's 20x20 5x5s): one 4 x 20 tile per block, 4 outputs
    // per thread (86 VGPRs, 31 KB LDS: 5 blocks per CU) measured 22.5 vs 26.6 us for the
    // persistent 8 x 20 form at L b64; the 40x40 maps keep the persistent form (35.4 vs 38.0),
    // profiles/r5_dw5_ab.txt
    if (d.kh == 5 && d.kw == 5 && d.stride == 1 && d.out_w <= 20) return launch_dw_tile<5, 1, 4, 20, 4>(d, s);
    if (d.kh == 5 && d.kw == 5 && d.stride == 1) return launch_dw_lds<5, 1, DP_DW5_TH, 20, 5, true>(d, s);
    if (d.kh == 3 && d.kw == 3 && d.stride == 1) return launch_dw_lds<3, 1, 8, 20, 5, true>(d, s);
    if (d.kh == 3 && d.kw == 3 && d.stride == 2) return launch_dw_tile<3, 2, DP_DWS2_TH, 16, 2>(d, s);
  }
  const int nchunk = d.cin / VEC;
  constexpr int PX = 4;
  const int ntx = (d.out_w + PX - 1) / PX;
  const int64_t total = (int64_t)d.batch * d.out_h * ntx * nchunk;
  DP_REQUIRE(total < (1ll << 31), "dp_dwconv2d: %lld work items exceed 2^31", (long long)total);
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
#define DP_DW(T_, KS_, S_)                                                                            \
  if (d.kh == KS_ && d.kw == KS_ && d.stride == S_) {                                                \
    hipLaunchKernelGGL((dwconv_kernel<T_, KS_, S_, PX>), grid, block, 0, s, d, total, nchunk, ntx); \
    return dp_check_launch("dp_dwconv2d");                                                           \
  }
  if (d.dtype == DP_BF16) {
    DP_DW(bf16_t, 3, 1) DP_DW(bf16_t, 3, 2) DP_DW(bf16_t, 5, 1) DP_DW(bf16_t, 5, 2)
  } else {
    DP_DW(float, 3, 1) DP_DW(float, 3, 2) DP_DW(float, 5, 1) DP_DW(float, 5, 2)
  }
#undef DP_DW
  dp_set_error("dp_dwconv2d: kernel %dx%d stride %d not supported (3/5, stride 1/2)", d.kh, d.kw, d.stride);
  return DP_EINVAL;
}

int dp_stem1_mfma(const float* image, int batch, int h, int w, const float* weight, const float* bias, int cout,
                  int has_lab, float ls, float lb, void* out, int64_t obs, int ops, hipStream_t s);

extern "C" int dp_stem_conv(const float* image, int32_t batch, int32_t h, int32_t w, const float* weight,
                            const float* bias, int32_t cout, int32_t has_lab, float lab_scale, float lab_bias,
                            void* out, int64_t out_bstride, int32_t out_pstride, int32_t dtype, void* stream) {
  DP_REQUIRE(image && weight && bias && out, "dp_stem_conv: null pointer");
  DP_REQUIRE(out_pstride % 8 == 0 && out_bstride % 8 == 0 && al16(out), "dp_stem_conv: output alignment");
  const int64_t total = (int64_t)batch * ((h + 1) / 2) * ((w + 1) / 2);
  DP_REQUIRE(total < (1ll << 31), "dp_stem_conv: batch too large");
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16) {   // bf16 storage: MFMA kernel (stem.hip), image rounded to bf16 like every activation
    const int r = dp_stem1_mfma(image, batch, h, w, weight, bias, cout, has_lab, lab_scale, lab_bias, out, out_bstride,
                                out_pstride, s);
    if (r >= 0) return r;
  }
#define DP_STEM(T_, N_)                                                                                     \
  if (cout == N_) {                                                                                        \
    hipLaunchKernelGGL((stem_conv_kernel<T_, N_>), grid, block, 0, s, image, batch, h, w, weight, bias,     \
                       has_lab, lab_scale, lab_bias, reinterpret_cast<T_*>(out), out_bstride, out_pstride); \
    return dp_check_launch("dp_stem_conv");                                                                \
  }
  if (dtype == DP_BF16) {
    DP_STEM(bf16_t, 16) DP_STEM(bf16_t, 24) DP_STEM(bf16_t, 32) DP_STEM(bf16_t, 48) DP_STEM(bf16_t, 64)
  } else {
    DP_STEM(float, 16) DP_STEM(float, 24) DP_STEM(float, 32) DP_STEM(float, 48) DP_STEM(float, 64)
  }
#undef DP_STEM
  dp_set_error("dp_stem_conv: cout=%d not instantiated (16/24/32/48/64)", cout);
  return DP_EINVAL;
}

extern "C" int dp_maxpool2x2_pad_rb(const void* in, int64_t in_bstride, int32_t in_pstride, int32_t batch, int32_t h,
                                    int32_t w, int32_t c, void* out, int64_t out_bstride, int32_t out_pstride,
                                    int32_t dtype, void* stream) {
  const int VEC = dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE(c % VEC == 0 && in_pstride % VEC == 0 && out_pstride % VEC == 0 && al16(in) && al16(out),
             "dp_maxpool2x2_pad_rb: 16-byte alignment required");
  const int64_t total = (int64_t)batch * h * w * (c / VEC);
  DP_REQUIRE(total < (1ll << 31), "dp_maxpool2x2_pad_rb: batch too large");
  dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(maxpool_kernel<bf16_t>, grid, block, 0, as_stream(stream), reinterpret_cast<const bf16_t*>(in),
                       in_bstride, in_pstride, batch, h, w, c, reinterpret_cast<bf16_t*>(out), out_bstride, out_pstride);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, grid, block, 0, as_stream(stream), reinterpret_cast<const float*>(in),
                       in_bstride, in_pstride, batch, h, w, c, reinterpret_cast<float*>(out), out_bstride, out_pstride);
  return dp_check_launch("dp_maxpool2x2_pad_rb");
}
