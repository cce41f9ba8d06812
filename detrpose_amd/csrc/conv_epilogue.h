// Epilogue of the f32 implicit-GEMM conv kernel (conv_gemm.hip):
// bias (folded BN) + activation + LAB into an LDS tile, then 16-byte row writes with the
// residual add, the optional nearest-x2 copy (FPN upsample + concat) and bf16/f32 output.
#pragma once
#include "common.h"

template <typename TO, int BM, int BN, int WGM, int TM, int TN>
__device__ __forceinline__ void conv_epilogue(const dp_conv_desc& d, const f32x4 (&acc)[TM][TN], char* smem_raw,
                                              int M, int m0, int n0, int vec_ok) {
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int VO = 16 / sizeof(TO);
  constexpr int CP = BN + VO;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int hwo = d.out_h * d.out_w;
  TO* Cs = reinterpret_cast<TO*>(smem_raw);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WN + j * 16 + (lane & 15);
    const int n = n0 + nl;
    const float bias = (d.bias && n < d.cout) ? d.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ml = wm * WM + i * 16 + (lane >> 4) * 4 + r;
        float v = apply_act(acc[i][j][r] + bias, d.act);
        if (d.has_lab) v = d.lab_scale * v + d.lab_bias;
        Cs[ml * CP + nl] = from_f32<TO>(v);
      }
    }
  }
  __syncthreads();

  TO* __restrict__ out = reinterpret_cast<TO*>(d.out);
  const TO* __restrict__ res = reinterpret_cast<const TO*>(d.res);
  TO* __restrict__ up = reinterpret_cast<TO*>(d.up);
  constexpr int CPR = BN / VO;  // chunks per row
  for (int e = tid; e < BM * CPR; e += 256) {
    const int ml = e / CPR, cc = e - ml * CPR;
    const int m = m0 + ml;
    const int n = n0 + cc * VO;
    if (m >= M || n >= d.cout) continue;
    const int b = m / hwo, rem = m - b * hwo;
    const int oy = rem / d.out_w, ox = rem - oy * d.out_w;
    const int64_t pix = (int64_t)oy * d.out_w + ox;
    const int64_t oo = (int64_t)b * d.out_bstride + pix * d.out_pstride + n;
    Vec16<TO> v = load16(Cs + ml * CP + cc * VO);
    if (vec_ok && n + VO <= d.cout) {
      if (res) {
        Vec16<TO> rv = load16(res + (int64_t)b * d.res_bstride + pix * d.res_pstride + n);
#pragma unroll
        for (int t = 0; t < VO; ++t) v.set(t, v.get(t) + rv.get(t));
      }
      store16(out + oo, v);
      if (up) {
        const int64_t ub = (int64_t)b * d.up_bstride + n;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx)
            store16(up + ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride, v);
      }
    } else {
      const int nn = min(VO, d.cout - n);
      for (int t = 0; t < nn; ++t) {
        float x = v.get(t);
        if (res) x += to_f32(res[(int64_t)b * d.res_bstride + pix * d.res_pstride + n + t]);
        out[oo + t] = from_f32<TO>(x);
        if (up) {
          const int64_t ub = (int64_t)b * d.up_bstride + n + t;
          for (int dy = 0; dy < 2; ++dy)
            for (int dx = 0; dx < 2; ++dx)
              up[ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride] = from_f32<TO>(x);
        }
      }
    }
  }
}
