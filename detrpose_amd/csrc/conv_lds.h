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
__device__ __forceinline__ void dma16(const i32x4& rsrc, const char* lds, int voff) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(rsrc)
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
  else if constexpr (ACT == DP_ACT_SILU) return x / (1.f + __expf(-x));
  else if constexpr (ACT == DP_ACT_GELU) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  else return x;
}

// One output pixel's NPL = 4*TN consecutive channels nb.. from the accumulators of one
// MFMA row-fragment (value acc[j][r] is channel nb + 4 j + r): bias/act/LAB in f32, residual
// add, 16-byte stores (scalar tail when the group is not whole or not aligned).
template <int ACT, typename TO, int TN>
__device__ __forceinline__ void epi_pixel(const dp_conv_desc& d, const f32x4 (&acc)[TN], const float (&bias)[4 * TN],
                                          int b, int oy, int ox, int nb, bool full) {
  constexpr int NPL = 4 * TN;
  constexpr int VO = 16 / (int)sizeof(TO);
  constexpr int CPL = NPL / VO;   // 16-byte chunks per lane per pixel
  static_assert(NPL % VO == 0, "lane channel group must be whole 16-byte chunks");
  TO* __restrict__ out = reinterpret_cast<TO*>(d.out);
  const TO* __restrict__ res = reinterpret_cast<const TO*>(d.res);
  TO* __restrict__ up = reinterpret_cast<TO*>(d.up);
  const int64_t pix = (int64_t)oy * d.out_w + ox;
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
      for (int c = 0; c < CPL; ++c) ch[c] = load16(rp + c * VO);
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
    for (int c = 0; c < CPL; ++c) store16(out + oo + c * VO, ch[c]);
    if (up) {
      const int64_t ub = (int64_t)b * d.up_bstride + nb;
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          TO* upp = up + ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride;
#pragma unroll
          for (int c = 0; c < CPL; ++c) store16(upp + c * VO, ch[c]);
        }
    }
  } else {
    const int nn = min(NPL, d.cout - nb);
#pragma unroll
    for (int c = 0; c < NPL; ++c) {
      if (c >= nn) break;
      float x = v[c];
      if (res) x += to_f32(res[(int64_t)b * d.res_bstride + pix * d.res_pstride + nb + c]);
      const TO y = from_f32<TO>(x);
      out[oo + c] = y;
      if (up) {
        const int64_t ub = (int64_t)b * d.up_bstride + nb + c;
        for (int dy = 0; dy < 2; ++dy)
          for (int dx = 0; dx < 2; ++dx)
            up[ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride] = y;
      }
    }
  }
}

// bias of the lane's NPL channels (0 past cout)
template <int NPL>
__device__ __forceinline__ void load_bias(const dp_conv_desc& d, int nb, float (&bias)[NPL]) {
#pragma unroll
  for (int c = 0; c < NPL; ++c) bias[c] = 0.f;
  if (!d.bias) return;
  if (nb + NPL <= d.cout) {
#pragma unroll
    for (int c = 0; c < NPL; c += 4) {
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(d.bias + nb + c);
      bias[c] = b4[0], bias[c + 1] = b4[1], bias[c + 2] = b4[2], bias[c + 3] = b4[3];
    }
  } else {
#pragma unroll
    for (int c = 0; c < NPL; ++c) bias[c] = nb + c < d.cout ? d.bias[nb + c] : 0.f;
  }
}

int num_cus();

}  // namespace dpconv
