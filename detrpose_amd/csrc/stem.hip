// StemBlock 2x2 convs (stem2a / stem2b, hgnetv2.py:171-220) as register-direct MFMA kernels.
//
// Both convs are 2x2 stride 1 over F.pad(x, (0,1,0,1)) with 8..32 channels in and out:
// K = 4 * cin <= 128, so the arithmetic is a handful of MFMAs per 16 pixels and the layers
// are pure HBM streams (stem1 output read once, stem2a/stem2b outputs written once). A
// staged (LDS patch + barrier) kernel spends most of its life waiting for its patch; here
// each wave gathers its MFMA B fragments straight from global memory into registers (lane
// (q, g) of K-slab s loads the 8 channels ci of tap t = k / cin, k = 32 s + 8 g, of pixel
// x0 + q: one 16-byte load, the 2x2 neighbours come from L1/L2), keeps G pixel groups of
// loads in flight, and has no LDS and no barriers. The weights (A operand, [cout][kpad],
// k = tap * cin + ci as every conv of the path) sit in registers for the wave's life.
//
// POOL (stem2a): the B fragments already hold the four taps of the zero-padded 2x2 window,
// i.e. MaxPool2d(2, 1) of F.pad(x,(0,1,0,1)) (hgnetv2.py:215-217) is a max over registers:
// cin 32 -> lane g holds taps 0..3 of channels 8g..8g+7; cin 16 -> taps {g>>1, 2+(g>>1)} of
// channels 8(g&1)..+7, completed by one cross-half exchange (lane ^ 32).
#include "common.h"
#include "stem_k.h"

namespace {

// Output channel of MFMA C element (tile j, lane group g, row r). With two 16-row tiles the
// weight rows are permuted (A row 16j + q holds channel stem_chan(j, q>>2, q&3)) so lane g
// ends with channels 8g..8g+7 contiguous: one 16-byte store per pixel and lane instead of
// two 8-byte pieces 32 bytes apart. One tile: the natural order, 8-byte stores.
template <int NT>
__device__ __forceinline__ constexpr int stem_chan(int j, int g, int r) {
  return NT == 2 ? 8 * g + 4 * j + r : 16 * j + 4 * g + r;
}

// bias + ReLU/none + LAB of the lane's 4*NT channels: one 16-byte chunk at channel 8g
// (NT = 2, permuted rows) or NT 8-byte chunks at 16j + 4g (natural order)
template <int NT, int ACT>
__device__ __forceinline__ void stem_store(bf16_t* op, const f32x4 (&acc)[NT], const float (&bsum)[NT][4], int g,
                                           int cout, int has_lab, float ls, float lb) {
  float v[4 * NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = acc[j][r] + bsum[j][r];
      if (ACT == DP_ACT_RELU) x = fmaxf(x, 0.f);
      if (has_lab) x = ls * x + lb;
      v[4 * j + r] = x;
    }
  if constexpr (NT == 2) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16_t)v[e];
    *reinterpret_cast<bf16x8*>(op + 8 * g) = o;
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if (16 * j + 4 * g >= cout) continue;
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16_t)v[4 * j + e];
      *reinterpret_cast<bf16x4*>(op + 16 * j + 4 * g) = o;
    }
  }
}

// StemBlock.stem1 (hgnetv2.py:171-177): 3x3 stride-2 pad-1 conv over the f32 NCHW image,
// 3 -> COUT channels, folded BN + ReLU (+ LAB), NHWC bf16 out. The 27 products (c, ky, kx) are
// MFMA K slabs in the order of stem_k.h: COUT 32 (B4 / B5) two slabs in the one-launch stem's
// order, so the two kernels agree bit for bit; COUT 16 one slab, k = c * 9 + ky * 3 + kx. Lane
// (q, g) gathers its slots of output pixel x0 + q straight from the image (f32 -> bf16 in
// registers; a zero slot loads nothing: out-of-range offset), the f32 weights are converted
// into the A fragments once per wave. 864 FMAs per pixel become 2 or 4 MFMAs per 16 pixels, so
// the kernel is a stream: 12 image bytes in (L1/L2 absorb the 3x3/stride-2 overlap) and
// 2*COUT bytes out per pixel.
template <int COUT>
__global__ __launch_bounds__(256) void stem1_mfma_kernel(const float* __restrict__ img, int batch, int H, int W,
                                                         const float* __restrict__ wt, const float* __restrict__ bias,
                                                         int has_lab, float ls, float lb, bf16_t* __restrict__ out,
                                                         int64_t obs, int ops) {
  constexpr int NT = COUT / 16;
  constexpr int NS = COUT == 32 ? 2 : 1;        // K slabs (stem_k.h)
  constexpr int G = 4;                          // 16-pixel groups in flight per wave
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4;
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;
  bf16x8 wa[NS][NT];   // [slab][tile]
  int tky[NS][8], tkx[NS][8];
  bool tok[NS][8];
  int loff[NS][8];
#pragma unroll
  for (int sl = 0; sl < NS; ++sl)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int c = 0, ky = 0, kx = 0;
      const bool ok = NS == 2 ? stem1_slot(sl, g, e, c, ky, kx) : stem1_slot_c9(g, e, c, ky, kx);
      tok[sl][e] = ok, tky[sl][e] = ky, tkx[sl][e] = kx;
      // lane-constant part of the gather offset: plane c, row ky, column kx, this lane's pixel 2q;
      // the per-group part (image, row 2oy-1, column 2*ox0-1) is wave-uniform
      loff[sl][e] = (c * H + ky) * W + kx + 2 * q;
#pragma unroll
      for (int j = 0; j < NT; ++j)
        wa[sl][j][e] = (bf16_t)(ok ? wt[stem_chan<NT>(j, q >> 2, q & 3) * 27 + c * 9 + ky * 3 + kx] : 0.f);
    }
  float bsum[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bsum[j][r] = bias[stem_chan<NT>(j, g, r)];

  const int gx = (OW + 15) >> 4;
  const int ngroups = batch * OH * gx;
  const int nw = gridDim.x * 4;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int base = wid * G; base < ngroups; base += nw * G) {
    bf16x8 xb[G][NS];
    int pb[G], py[G], px0[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
      // the group (image, output row, 16-pixel column block) is wave-uniform: scalar math,
      // an SGPR image base and 32-bit lane offsets for the loads
      const int grp = __builtin_amdgcn_readfirstlane(base + i);
      const int gc = grp < ngroups ? grp : 0;
      const int bb = gc / (OH * gx), rem = gc - bb * (OH * gx);
      const int oy = rem / gx, ox0 = (rem - oy * gx) * 16;
      pb[i] = grp < ngroups ? bb : -1, py[i] = oy, px0[i] = ox0;
      // buffer loads from the image's base (SGPRs) with 32-bit byte offsets; an out-of-range
      // offset returns 0 = the conv zero padding, so the gather has no branches (loads under
      // divergent ifs would make the compiler drain vmcnt between them)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(img + (int64_t)bb * 3 * H * W), (short)0, 0x7ffffff0, 0x00020000);
      const int u = (2 * oy - 1) * W + 2 * ox0 - 1;
      const int ix0 = 2 * (ox0 + q) - 1;
#pragma unroll
      for (int sl = 0; sl < NS; ++sl)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (NS == 2 && ((e & 3) == 3 || (sl == 1 && e >= 4))) {   // zero in every lane (stem_k.h): no load
            xb[i][sl][e] = (bf16_t)0.f;
            continue;
          }
          const int iy = 2 * oy - 1 + tky[sl][e], ix = ix0 + tkx[sl][e];
          const bool ok = tok[sl][e] && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
          const unsigned bits =
              __builtin_amdgcn_raw_buffer_load_b32(rs, ok ? 4 * (u + loff[sl][e]) : 0x7ffffff0, 0, 0);
          xb[i][sl][e] = (bf16_t)__builtin_bit_cast(float, bits);   // the builtin returns the raw dword
        }
    }
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int ox = px0[i] + q;
      if (pb[i] < 0 || ox >= OW) continue;
      bf16_t* op = out + (int64_t)pb[i] * obs + ((int64_t)py[i] * OW + ox) * ops;
      f32x4 acc[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][j], xb[i][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        if constexpr (NS == 2) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][j], xb[i][1], acc[j], 0, 0, 0);
      }
      stem_store<NT, DP_ACT_RELU>(op, acc, bsum, g, COUT, has_lab, ls, lb);
    }
  }
}

// KS x KS (1 or 2) stride-1 conv, right/bottom zero padding: the stem's 2x2 convs and its
// 1x1 stem4 (cin <= 32: one or two K slabs, output of up to 4 16-channel tiles)
template <int KS, int CIN, int COUT, bool POOL, int ACT>
__global__ __launch_bounds__(256) void conv_direct_kernel(const bf16_t* __restrict__ in, int64_t ibs, int ips,
                                                             int H, int W, int batch, const bf16_t* __restrict__ wt,
                                                             int kpad, const float* __restrict__ bias, int has_lab,
                                                             float ls, float lb, bf16_t* __restrict__ out, int64_t obs,
                                                             int ops, bf16_t* __restrict__ pool, int64_t pbs, int pps) {
  constexpr int NKS = (KS * KS * CIN + 31) / 32;   // K slabs of 32
  constexpr int NT = (COUT + 15) / 16;             // 16-channel output tiles
  constexpr int G = 4;                             // pixel groups (16 px each) in flight per wave
  static_assert((KS == 1 || KS == 2) && CIN % 8 == 0 && COUT % 4 == 0 && CIN <= 32 && NT <= 4, "stem shapes");
  static_assert(!POOL || (KS == 2 && (CIN == 32 || CIN == 16)), "pool: 2x2 window, cin 16 or 32");
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4;

  bf16x8 wa[NT][NKS];
  int tap_dy[NKS], tap_dx[NKS], tap_ci[NKS];
  bool tap_ok[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int k = 32 * s + 8 * g;
    const int t = k / CIN;
    tap_ok[s] = t < KS * KS;
    tap_dy[s] = t / KS, tap_dx[s] = t % KS, tap_ci[s] = k - t * CIN;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int row = stem_chan<NT>(j, q >> 2, q & 3);
      bf16x8 w = {};
      if (row < COUT && tap_ok[s]) w = *reinterpret_cast<const bf16x8*>(wt + (int64_t)row * kpad + k);
      wa[j][s] = w;
    }
  }
  float bsum[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = stem_chan<NT>(j, g, r);
      bsum[j][r] = (bias && c < COUT) ? bias[c] : 0.f;
    }

  const int gx = (W + 15) >> 4;
  const int ngroups = batch * H * gx;
  const int nw = gridDim.x * 4;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int base = wid * G; base < ngroups; base += nw * G) {
    bf16x8 xb[G][NKS];
    int pb[G], py[G], px[G];
    bool pv[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int grp = base + i;
      const int bb = grp / (H * gx), rem = grp - bb * (H * gx);
      const int y = rem / gx, x = (rem - y * gx) * 16 + q;
      pb[i] = bb, py[i] = y, px[i] = x;
      pv[i] = grp < ngroups && x < W;
      const bf16_t* ib = in + (int64_t)(grp < ngroups ? bb : 0) * ibs;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        // branch-free: clamped (always legal) address, then select the F.pad zero
        const int iy = y + tap_dy[s], ix = x + tap_dx[s];
        const bool ok = grp < ngroups && tap_ok[s] && iy < H && ix < W;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(ib + (ok ? (int64_t)(iy * W + ix) * ips + tap_ci[s] : 0));
        const bf16x8 z = {};
        xb[i][s] = ok ? v : z;
      }
    }
#pragma unroll
    for (int i = 0; i < G; ++i) {
      f32x4 acc[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NKS; ++s) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][s], xb[i][s], acc[j], 0, 0, 0);
      }
      // C layout: lane (q, g) holds channels stem_chan(j, g, r) of pixel x0 + q
      const int64_t pix = (int64_t)py[i] * W + px[i];
      if (pv[i]) stem_store<NT, ACT>(out + (int64_t)pb[i] * obs + pix * ops, acc, bsum, g, COUT, has_lab, ls, lb);
      if constexpr (POOL) {
        bf16x8 m;
        if constexpr (CIN == 32) {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            m[e] = (bf16_t)fmaxf(fmaxf((float)xb[i][0][e], (float)xb[i][1][e]),
                                 fmaxf((float)xb[i][2][e], (float)xb[i][3][e]));
        } else {
          // cin 16: this lane has 2 of the 4 taps; lane ^ 32 (g ^ 2) has the other two
          bf16x8 h;
#pragma unroll
          for (int e = 0; e < 8; ++e) h[e] = (bf16_t)fmaxf((float)xb[i][0][e], (float)xb[i][1][e]);
          const uint4 hu = *reinterpret_cast<const uint4*>(&h);
          uint4 ou;
          ou.x = __shfl_xor(hu.x, 32, 64), ou.y = __shfl_xor(hu.y, 32, 64);
          ou.z = __shfl_xor(hu.z, 32, 64), ou.w = __shfl_xor(hu.w, 32, 64);
          const bf16x8 o = *reinterpret_cast<const bf16x8*>(&ou);
#pragma unroll
          for (int e = 0; e < 8; ++e) m[e] = (bf16_t)fmaxf((float)h[e], (float)o[e]);
        }
        // lane g stores channels 8g..8g+7 (cin 16: lanes g = 0, 1 hold the complete max)
        if (pv[i] && g < CIN / 8) *reinterpret_cast<bf16x8*>(pool + (int64_t)pb[i] * pbs + pix * pps + 8 * g) = m;
      }
    }
  }
}

template <int KS, int CIN, int COUT, bool POOL>
int launch_direct(const dp_conv_desc& d, hipStream_t s, bf16_t* pool, int64_t pbs, int pps) {
  DP_DESCRIBE("conv_direct_kernel<%d, %d, %d, %s, %d>", KS, CIN, COUT, DP_TF(POOL),
              d.act == DP_ACT_RELU ? DP_ACT_RELU : DP_ACT_NONE);
  const int gx = (d.in_w + 15) / 16;
  const int64_t ngroups = (int64_t)d.batch * d.in_h * gx;
  int blocks = (int)((ngroups + 4 * 4 - 1) / (4 * 4));   // 4 waves x G = 4 groups per block pass
  if (blocks > 256 * 8) blocks = 256 * 8;   // about one resident pass of the chip
  auto kern = d.act == DP_ACT_RELU ? conv_direct_kernel<KS, CIN, COUT, POOL, DP_ACT_RELU>
                                   : conv_direct_kernel<KS, CIN, COUT, POOL, DP_ACT_NONE>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const bf16_t*>(d.in), d.in_bstride,
                     d.in_pstride, d.in_h, d.in_w, d.batch, reinterpret_cast<const bf16_t*>(d.weight), d.kpad, d.bias,
                     d.has_lab, d.lab_scale, d.lab_bias, reinterpret_cast<bf16_t*>(d.out), d.out_bstride, d.out_pstride,
                     pool, pbs, pps);
  return dp_check_launch("dp_conv2d(stem direct)");
}

}  // namespace

// bf16 stem convs as register-direct kernels: 2x2 stride 1 with right/bottom zero padding
// (stem2a / stem2b, optionally with the fused stem max-pool) and the 1x1 stem4. Returns -1
// when the shape has no instantiation (the caller then uses the LDS halo / GEMM kernels).
int dp_conv2d_stem_direct(const dp_conv_desc& d, hipStream_t s, void* pool, int64_t pbs, int pps) {
  const int ks = d.kh;
  if (d.dtype != DP_BF16 || d.out_f32 || d.res || d.up || (ks != 1 && ks != 2) || d.kw != ks || d.stride != 1 ||
      d.pad_t || d.pad_l || d.out_h != d.in_h || d.out_w != d.in_w || (d.act != DP_ACT_RELU && d.act != DP_ACT_NONE))
    return -1;
  auto a8 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; };
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!a8(d.out) || d.out_pstride % 4 || d.out_bstride % 4 || !a16(d.in) || !a16(d.weight) || d.in_pstride % 8 ||
      d.in_bstride % 8)
    return -1;
  if ((int64_t)d.batch * d.in_h * ((d.in_w + 15) / 16) >= (1ll << 31)) return -1;
  const bool nt2 = d.cout > 16 && d.cout <= 32;   // permuted rows, 16-byte stores
  if (nt2 && (!a16(d.out) || d.out_pstride % 8 || d.out_bstride % 8)) return -1;
  bf16_t* pl = reinterpret_cast<bf16_t*>(pool);
  if (pool && (ks != 2 || !a16(pool) || pps % 8 || pbs % 8)) return -1;
  // HGNetv2 stems: B0 [3,16,16], B4 (L) [3,32,48], B5 (X) [3,32,64]
  if (ks == 2) {
#define DP_DIRECT(CI, CO)                                                          \
    if (d.cin == CI && d.cout == CO) {                                             \
      if (pool) return launch_direct<2, CI, CO, true>(d, s, pl, pbs, pps);         \
      return launch_direct<2, CI, CO, false>(d, s, nullptr, 0, 0);                 \
    }
    DP_DIRECT(32, 16)
    DP_DIRECT(16, 8)
#undef DP_DIRECT
    if (pool) return -1;
    if (d.cin == 16 && d.cout == 32) return launch_direct<2, 16, 32, false>(d, s, nullptr, 0, 0);
    if (d.cin == 8 && d.cout == 16) return launch_direct<2, 8, 16, false>(d, s, nullptr, 0, 0);
    return -1;
  }
  // stem4 (1x1)
  if (d.cin == 32 && d.cout == 48) return launch_direct<1, 32, 48, false>(d, s, nullptr, 0, 0);
  if (d.cin == 32 && d.cout == 64) return launch_direct<1, 32, 64, false>(d, s, nullptr, 0, 0);
  if (d.cin == 16 && d.cout == 16) return launch_direct<1, 16, 16, false>(d, s, nullptr, 0, 0);
  return -1;
}

// bf16 stem1 on MFMA (dp_stem_conv's bf16 path); -1 when cout has no instantiation
int dp_stem1_mfma(const float* image, int batch, int h, int w, const float* weight, const float* bias, int cout,
                  int has_lab, float ls, float lb, void* out, int64_t obs, int ops, hipStream_t s) {
  if ((cout != 16 && cout != 32) || ops % 8 || obs % 8 || (reinterpret_cast<uintptr_t>(out) & 15)) return -1;
  const int oh = (h + 1) / 2, ow = (w + 1) / 2;
  const int64_t ngroups = (int64_t)batch * oh * ((ow + 15) / 16);
  if (ngroups >= (1ll << 31) || (int64_t)batch * 3 * h * w >= (1ll << 31)) return -1;
  int blocks = (int)((ngroups + 15) / 16);
  if (blocks > 256 * 8) blocks = 256 * 8;
  auto kern = cout == 16 ? stem1_mfma_kernel<16> : stem1_mfma_kernel<32>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, image, batch, h, w, weight, bias, has_lab, ls, lb,
                     reinterpret_cast<bf16_t*>(out), obs, ops);
  return dp_check_launch("dp_stem_conv(mfma)");
}
