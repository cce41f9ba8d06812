// Shared pieces of the LDS-DMA convolution kernels (conv_stream.hip, conv_halo.hip):
// buffer descriptors, the inline-asm LDS-DMA, counted waits, activations and the
// register epilogue (bias + act + LAB + residual + nearest-x2 copy, 16-byte stores).
#pragma once
#include "common.h"

namespace dpconv {

constexpr int OOB = 0x7fffffff;

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Buffer resource words (base, no stride, 2 GB range, gfx950 raw-buffer flags) in SGPRs.
__device__ __forceinline__ i32x4 make_rsrc(const void* base) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffffu));
  r[2] = 0x7ffffff0;
  r[3] = 0x00020000;
  return r;
}

// 16 bytes per lane HBM/L2 -> LDS (M0 = wave-uniform LDS byte address; lane L lands at
// M0 + 16 L). Inline asm rather than the builtin: the compiler would otherwise treat every
// later ds_read as a possible alias of the DMA and insert s_waitcnt vmcnt(0), draining the
// ring; completion is tracked by hand (wait_vmcnt + barrier) below.
// The descriptor words go through readfirstlane: they are uniform, but a descriptor assigned
// under loop control the compiler cannot prove uniform lands in VGPRs, which the "s"
// operand would not accept (free when they already sit in SGPRs).
__device__ __forceinline__ void dma16(const i32x4& rsrc, const char* lds, int voff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds));
  i32x4 r;
#pragma unroll
  for (int w = 0; w < 4; ++w) r[w] = __builtin_amdgcn_readfirstlane(rsrc[w]);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(r)
               : "memory");
}

// s_waitcnt vmcnt(N) (expcnt/lgkmcnt untouched) as the builtin, so the compiler's own
// wait insertion sees it and does not add a second vmcnt(0) for its epilogue loads/stores.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xf << 8));
}

template <int ACT>
__device__ __forceinline__ float act_t(float x) {
  if constexpr (ACT == DP_ACT_RELU) return fmaxf(x, 0.f);
  else if constexpr (ACT == DP_ACT_SILU) return silu_f(x);
  else if constexpr (ACT == DP_ACT_GELU) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  else return x;
}

// Channel of lane-group g's accumulator element e = 4 j + r (tile j, row r) within the
// wave's 4*NPL output channels. The lane's elements are cut into 16-byte chunks of VO
// channels, and chunk c of the four lane groups is laid side by side:
//   chan(g, e) = (e / VO) * 4 VO + g VO + e % VO
// so each 16-byte store instruction of the epilogue writes 4 x 16 = 64 CONTIGUOUS bytes of
// every pixel (16 pixels per instruction) instead of four 16-byte pieces 32-64 B apart.
// The weight rows are permuted into LDS with the same map, so this costs nothing.
template <int VO>
__device__ __forceinline__ constexpr int lane_chan(int g, int e) {
  return (e / VO) * (4 * VO) + g * VO + e % VO;
}

// every row start of out / res / up is 16-byte aligned (the launchers' vec_ok, recomputed
// for the cout-edge path of epi_pixel)
__device__ __forceinline__ bool vec_aligned(const dp_conv_desc& d) {
  const int e = d.out_f32 ? 4 : 2;
  const uintptr_t bits = reinterpret_cast<uintptr_t>(d.out) | reinterpret_cast<uintptr_t>(d.res) |
                         reinterpret_cast<uintptr_t>(d.up);
  const int64_t st = (d.out_bstride | d.out_pstride | (d.res ? (d.res_bstride | d.res_pstride) : 0) |
                      (d.up ? (d.up_bstride | d.up_pstride) : 0)) * e;
  return ((bits | (uintptr_t)st) & 15) == 0;
}

// One output pixel's NPL = 4*TN channels of lane group g (lane_chan map over the wave's
// channel base nbw) from the accumulators of one MFMA row-fragment: bias/act/LAB in f32,
// residual add, 16-byte non-temporal stores (scalar tail when the chunk is not whole or not
// aligned).
template <int ACT, typename TO, int TN>
__device__ __forceinline__ void epi_pixel(const dp_conv_desc& d, const f32x4 (&acc)[TN], const float (&bias)[4 * TN],
                                          int b, int oy, int ox, int nbw, int g, bool full) {
  constexpr int NPL = 4 * TN;
  constexpr int VO = 16 / (int)sizeof(TO);
  constexpr int CPL = NPL / VO;   // 16-byte chunks per lane per pixel
  static_assert(NPL % VO == 0, "lane channel group must be whole 16-byte chunks");
  TO* __restrict__ out = reinterpret_cast<TO*>(d.out);
  const TO* __restrict__ res = reinterpret_cast<const TO*>(d.res);
  TO* __restrict__ up = reinterpret_cast<TO*>(d.up);
  const int64_t pix = (int64_t)oy * d.out_w + ox;
  const int nb = nbw + g * VO;     // channel of the lane's chunk 0; chunk c at nb + 4 VO c
  float v[NPL];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = act_t<ACT>(acc[j][r] + bias[4 * j + r]);
      if (d.has_lab) x = d.lab_scale * x + d.lab_bias;
      v[4 * j + r] = x;
    }
  const int64_t oo = (int64_t)b * d.out_bstride + pix * d.out_pstride + nb;
  if (full) {
    Vec16<TO> ch[CPL];
    if (res) {
      const TO* rp = res + (int64_t)b * d.res_bstride + pix * d.res_pstride + nb;
#pragma unroll
      for (int c = 0; c < CPL; ++c) ch[c] = load16(rp + c * 4 * VO);
#pragma unroll
      for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int t = 0; t < VO; ++t) ch[c].set(t, v[c * VO + t] + ch[c].get(t));
    } else {
#pragma unroll
      for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int t = 0; t < VO; ++t) ch[c].set(t, v[c * VO + t]);
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) store16_nt(out + oo + c * 4 * VO, ch[c]);
    if (up) {
      const int64_t ub = (int64_t)b * d.up_bstride + nb;
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          TO* upp = up + ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride;
#pragma unroll
          for (int c = 0; c < CPL; ++c) store16_nt(upp + c * 4 * VO, ch[c]);
        }
    }
  } else {
    // edge of cout (or unaligned rows): whole chunks still go out as 16-byte vectors
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int cb = nb + c * 4 * VO;
      if (cb >= d.cout) break;
      const int64_t po = (int64_t)b * d.out_bstride + pix * d.out_pstride + cb;
      const int64_t pr = (int64_t)b * d.res_bstride + pix * d.res_pstride + cb;
      const int64_t ub = (int64_t)b * d.up_bstride + cb;
      if (vec_aligned(d) && cb + VO <= d.cout) {
        Vec16<TO> ch;
        if (res) ch = load16(res + pr);
#pragma unroll
        for (int t = 0; t < VO; ++t) ch.set(t, v[c * VO + t] + (res ? ch.get(t) : 0.f));
        store16(out + po, ch);
        if (up)
          for (int dy = 0; dy < 2; ++dy)
            for (int dx = 0; dx < 2; ++dx)
              store16(up + ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride, ch);
        continue;
      }
      for (int t = 0; t < VO && cb + t < d.cout; ++t) {
        float x = v[c * VO + t];
        if (res) x += to_f32(res[pr + t]);
        const TO y = from_f32<TO>(x);
        out[po + t] = y;
        if (up)
          for (int dy = 0; dy < 2; ++dy)
            for (int dx = 0; dx < 2; ++dx)
              up[ub + t + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride] = y;
      }
    }
  }
}

// the lane's chunks are whole and inside cout (vector path of epi_pixel)
template <typename TO, int NPL>
__device__ __forceinline__ bool lane_full(const dp_conv_desc& d, int nbw, int g, int vec_ok) {
  constexpr int VO = 16 / (int)sizeof(TO);
  return vec_ok && nbw + lane_chan<VO>(g, NPL - 1) < d.cout;
}

// bias of the lane's NPL channels (lane_chan map; 0 past cout)
template <typename TO, int NPL>
__device__ __forceinline__ void load_bias(const dp_conv_desc& d, int nbw, int g, float (&bias)[NPL]) {
  constexpr int VO = 16 / (int)sizeof(TO);
#pragma unroll
  for (int e = 0; e < NPL; ++e) bias[e] = 0.f;
  if (!d.bias) return;
  if (nbw + lane_chan<VO>(g, NPL - 1) < d.cout) {
#pragma unroll
    for (int e = 0; e < NPL; e += 4) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(d.bias + nbw + lane_chan<VO>(g, e));
      bias[e] = b4[0], bias[e + 1] = b4[1], bias[e + 2] = b4[2], bias[e + 3] = b4[3];
    }
  } else {
#pragma unroll
    for (int e = 0; e < NPL; ++e) {
      const int cc = nbw + lane_chan<VO>(g, e);
      bias[e] = cc < d.cout ? d.bias[cc] : 0.f;
    }
  }
}

int num_cus();

}  // namespace dpconv
