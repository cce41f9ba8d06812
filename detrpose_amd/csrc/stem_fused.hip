// The whole HGNetv2 StemBlock (hgnetv2.py:171-220) in one persistent kernel for the
// 32-channel stems (B4 = DETRPose-L, B5 = X): stem1 (3x3 s2 over the f32 image) -> stem2a
// (2x2 over F.pad(x,(0,1,0,1))) -> stem2b (2x2 over F.pad(x2,(0,1,0,1))) and
// MaxPool2d(2, 1) over F.pad(x) -> cat -> stem3 (3x3 s2) -> stem4 (1x1).
//
// Unfused, every intermediate map lives at half the image resolution (320x320 for a 640
// image) and crosses HBM once or twice: at L b64 the five launches move ~3 GB (stem1 out
// 0.42 GB, stem2a out, the 64-channel cat 0.84 GB written and read, ...) for ~1.07 ms. Here
// a block owns a TH x TW tile of the stem3/stem4 output (160x160), recomputes the halo it
// needs of every earlier stage into LDS and writes only stem4's output: HBM sees the image
// (read once; L2 absorbs the stride-2 overlap) and the 48/64-channel stem4 map.
//
// Regions (map coordinates of the 320x320 stage maps, origin (2 oy0 - 1, 2 ox0 - 1), the
// top-left input pixel of stem3's 3x3/s2/pad-1 window):
//   cat   (stem3 input)    RCH x RCW = (2TH+1) x (2TW+1)   pool + stem2b, 64 ch
//   s2a   (stem2b input)   (2TH+2) x (2TW+2)               16 ch
//   s1    (stem2a / pool)  (2TH+3) x (2TW+3)               32 ch
// A position outside the map holds zero in every region: that is stem3's zero padding
// (row / column -1) and the F.pad right/bottom zeros of stem2a, stem2b and the max-pool.
//
// Every stage is 16x16x32 bf16 MFMAs with the weights as the A operand and 16 pixels as the
// B operand (C^T = W X^T: lane (q, g) ends with output channels of pixel q), the K order of
// the packed weights (tap-major, k = tap * cin + ci) and f32 accumulation in the same
// sequence as the unfused kernels, bf16 rounding at the same points (each stage's output):
// the result matches the five-launch path bit for bit. 32-channel outputs use the permuted
// weight rows of stem.hip (lane g holds channels 8g .. 8g+7: one 16-byte LDS store).
// Weights: stem1/2a/2b/4 fragments in registers for the block's life, stem3's 32 x 576 in
// LDS. The image: the tile's (4TH+7) x (4TW+8) x 3 window is loaded with coalesced 16-byte
// loads (issued before this tile's stem3 for the next tile, so the HBM latency hides behind
// stem3/stem4), rounded to bf16 into an LDS patch, and stem1's B fragments are built from it.
#include "common.h"

//
// LDS layout: the stage maps are stored planar by 16-byte channel chunk ([chunk][pixel],
// 16 B per pixel per plane) so that the 16 lanes of an MFMA B-fragment read (16 consecutive
// pixels, one chunk per lane group) hit 16 distinct bank slots: plane strides are multiples of
// 256 B (cat: 16 mod 256, whose stem3 reads step 2 pixels per lane). Every address a stage
// reads or writes is a lane constant (the tile geometry is the same for every tile) plus a
// compile-time offset: the per-tile work is MFMAs, LDS traffic and the epilogues.
#ifndef DP_STEM_ABL
#define DP_STEM_ABL 0   // ablation builds only: skip stage 1 / 2 / 3 / 4 / 5 (bits 0..4), 32: no image loads
#endif

namespace {

constexpr int TH = 4, TW = 16;   // stem3 / stem4 output tile: 4 rows x 16 columns, 8 waves
constexpr int NWAVE = 8, NTHR = 64 * NWAVE;
constexpr int R1H = 2 * TH + 3, R1W = 2 * TW + 3, N1 = R1H * R1W;   // 11 x 35 stem1 region
constexpr int R2H = 2 * TH + 2, R2W = 2 * TW + 2, N2 = R2H * R2W;   // 10 x 34 stem2a region
constexpr int RCH = 2 * TH + 1, RCW = 2 * TW + 1, NC = RCH * RCW;   //  9 x 33 cat region
constexpr int G1 = (N1 + 15) / 16, G2 = (N2 + 15) / 16, GC = (NC + 15) / 16;
constexpr int PF1 = (G1 + NWAVE - 1) / NWAVE, PF2 = (G2 + NWAVE - 1) / NWAVE, PFC = (GC + NWAVE - 1) / NWAVE;
constexpr int NPOOL = NC * 4, PFP = (NPOOL + NTHR - 1) / NTHR;      // max-pool items (pixel, chunk)
constexpr int K3 = 9 * 64;
constexpr int W3ROW = K3 * 2 + 16;             // +16 B: 16 consecutive rows hit 16 distinct bank slots
constexpr int rup(int x, int m) { return (x + m - 1) / m * m; }
constexpr int P1 = rup(N1 * 16, 256), P2 = rup(N2 * 16, 256), PC = rup(NC * 16 - 16, 256) + 16, P3 = TH * TW * 16;
constexpr int OFF_S1 = 0, OFF_S2 = OFF_S1 + 4 * P1, OFF_CAT = OFF_S2 + 2 * P2, OFF_S3 = OFF_CAT + 8 * PC;
constexpr int OFF_W3 = OFF_S3 + 4 * P3;
// image patch: rows 4 oy0 - 3 .. +IPH-1, columns 4 ox0 - 4 .. +IPW-1 (16-byte aligned starts)
constexpr int IPH = 2 * R1H + 1, IPW = 2 * R1W + 2;                 // 23 x 72
constexpr int IPV = IPW / 4, NIMG = 3 * IPH * IPV;                  // float4 per row, per tile
constexpr int PFV = (NIMG + NTHR - 1) / NTHR;                        // float4 loads per thread
// 4 planes: stem1's K = 27 is padded to 32 with k = 27..31 -> plane 3, which stays zero
constexpr int IPP = IPH * IPW * 2, OFF_IMG = OFF_W3 + 32 * W3ROW;
constexpr int LDS_BYTES = OFF_IMG + 4 * IPP;
static_assert(LDS_BYTES <= 160 * 1024 && TH * TW == 16 * 4 && IPW % 4 == 0 && OFF_IMG % 16 == 0 && IPP % 16 == 0,
              "stem tile");

// output channel of C element (tile j, lane group g, row r) for the permuted 32-channel convs
__device__ __forceinline__ constexpr int chan32(int j, int g, int r) { return 8 * g + 4 * j + r; }

struct StemArgs {
  const float* w1;
  const float* b1;
  const bf16_t* w2a;
  const float* b2a;
  const bf16_t* w2b;
  const float* b2b;
  const bf16_t* w3;
  const float* b3;
  const bf16_t* w4;
  const float* b4;
  int k2a, k2b, k3, k4;
  float lab[5][2];
};

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ T lds_ld(const char* smem, int off) {
  return *reinterpret_cast<const T*>(smem + off);
}
template <typename T>
__device__ __forceinline__ void lds_st(char* smem, int off, const T& v) {
  *reinterpret_cast<T*>(smem + off) = v;
}

// folded-BN bias + ReLU (+ LAB); + 0.f turns a -0 into +0, so the non-negative bf16 maps can
// be max-pooled as unsigned 16-bit integers
template <bool LAB>
__device__ __forceinline__ float relu_lab(float x, const StemArgs& P, int s) {
  x = fmaxf(x, 0.f) + 0.f;
  if constexpr (LAB) x = P.lab[s][0] * x + P.lab[s][1];
  return x;
}

// region pixel p -> (row, column) packed as row << 8 | column
template <int RW>
__device__ __forceinline__ int rc_of(int p) {
  const int r = p / RW;
  return (r << 8) | (p - r * RW);
}

template <int COUT, bool LAB>
__global__ __launch_bounds__(NTHR) void stem_fused_kernel(const float* __restrict__ img, int H, int W, StemArgs P,
                                                          bf16_t* __restrict__ out, int64_t obs, int ops, int tiles_x,
                                                          int tiles_y, int ntiles) {
  constexpr int NT4 = COUT / 16;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, q = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;                                   // multiple of 8
  const int L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (L >= ntiles) return;
  const int OH1 = (H + 1) / 2, OW1 = (W + 1) / 2;
  const int OH3 = (OH1 + 1) / 2, OW3 = (OW1 + 1) / 2;

  // ---- stem3 weights -> LDS, rows permuted (LDS row 16j + r = channel chan32(j, r>>2, r&3))
  for (int e = tid; e < 32 * (K3 / 8); e += NTHR) {
    const int row = e / (K3 / 8), kc = e - row * (K3 / 8);
    const int ch = chan32(row >> 4, (row & 15) >> 2, row & 3);
    lds_st(smem, OFF_W3 + row * W3ROW + kc * 16, *reinterpret_cast<const bf16x8*>(P.w3 + (int64_t)ch * P.k3 + kc * 8));
  }
  for (int e = tid; e < IPP / 16; e += NTHR) lds_st(smem, OFF_IMG + 3 * IPP + 16 * e, u32x4{0u, 0u, 0u, 0u});
  // ---- register weights and biases
  bf16x8 wa1[2], wa2[4], wb2[2][2], w4f[NT4];
  int poff[8];   // stem1 K value 8g + e: patch byte offset of (c, ky, kx + 1); k >= 27 lands in plane 3
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * g + e;   // stem1 K: k = c*9 + ky*3 + kx (the OIHW flattening of the f32 weights)
    const int c = k / 9, t = k - 9 * (k / 9), ky = t / 3, kx = t - 3 * (t / 3);
    poff[e] = OFF_IMG + ((c * IPH + ky) * IPW + kx + 1) * 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) wa1[j][e] = (bf16_t)(k < 27 ? P.w1[chan32(j, q >> 2, q & 3) * 27 + k] : 0.f);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) wa2[s] = *reinterpret_cast<const bf16x8*>(P.w2a + (int64_t)q * P.k2a + 32 * s + 8 * g);
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s)
      wb2[j][s] = *reinterpret_cast<const bf16x8*>(P.w2b + (int64_t)chan32(j, q >> 2, q & 3) * P.k2b + 32 * s + 8 * g);
#pragma unroll
  for (int j = 0; j < NT4; ++j) w4f[j] = *reinterpret_cast<const bf16x8*>(P.w4 + (int64_t)(16 * j + q) * P.k4 + 8 * g);
  float bs1[2][4], bs2a[4], bs2b[2][4], bs3[2][4], bs4[NT4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    bs2a[r] = P.b2a[4 * g + r];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bs1[j][r] = P.b1[chan32(j, g, r)];
      bs2b[j][r] = P.b2b[chan32(j, g, r)];
      bs3[j][r] = P.b3[chan32(j, g, r)];
    }
#pragma unroll
    for (int j = 0; j < NT4; ++j) bs4[j][r] = P.b4[16 * j + 4 * g + r];
  }

  // ---- tile-invariant lane geometry (region pixel of each item this lane handles)
  int rc1[PF1], a1[PF1];             // stem1: (row, col), patch byte offset of the window corner
#pragma unroll
  for (int i = 0; i < PF1; ++i) {
    const int p = min((wave + NWAVE * i) * 16 + q, N1 - 1);
    rc1[i] = rc_of<R1W>(p);
    a1[i] = ((rc1[i] >> 8) * 2 * IPW + (rc1[i] & 255) * 2) * 2;
  }
  int rc2[PF2], a2[PF2];             // stem2a: (row, col), s1 read address of tap (0, 0), chunk g
#pragma unroll
  for (int i = 0; i < PF2; ++i) {
    const int p = min((wave + NWAVE * i) * 16 + q, N2 - 1);
    rc2[i] = rc_of<R2W>(p);
    a2[i] = OFF_S1 + g * P1 + ((rc2[i] >> 8) * R1W + (rc2[i] & 255)) * 16;
  }
  int rcp[PFP], ap[PFP], sp[PFP];    // pool item (chunk c = it / NC, pixel it % NC): s1 read, cat write
#pragma unroll
  for (int t = 0; t < PFP; ++t) {
    const int it = min(tid + NTHR * t, NPOOL - 1);
    const int c = it / NC, p = it - c * NC;
    rcp[t] = rc_of<RCW>(p);
    ap[t] = OFF_S1 + c * P1 + ((rcp[t] >> 8) * R1W + (rcp[t] & 255)) * 16;
    sp[t] = OFF_CAT + c * PC + p * 16;
  }
  int rcc[PFC], ac[PFC];             // stem2b: (row, col), s2a read address of k-slab 0
#pragma unroll
  for (int i = 0; i < PFC; ++i) {
    const int p = min((wave + NWAVE * i) * 16 + q, NC - 1);
    rcc[i] = rc_of<RCW>(p);
    ac[i] = OFF_S2 + (g & 1) * P2 + ((rcc[i] >> 8) * R2W + (rcc[i] & 255) + (g >> 1)) * 16;
  }
  const int i3 = wave & 3, j3 = wave >> 2;   // stem3: output row i3, N tile j3
  const int a3 = OFF_CAT + g * PC + (2 * i3 * RCW + 2 * q) * 16;
  const int w3a = OFF_W3 + (16 * j3 + q) * W3ROW + 16 * g;

  // ---- image window of a tile: float4 loads into registers (issued a tile ahead), then
  // rounded to bf16 into the LDS patch [c][row][col]. Buffer loads: an out-of-range offset
  // returns 0 (the conv's zero padding; W % 4 == 0 so a float4 is wholly in or out).
  f32x4 xr[PFV];
  auto load_img = [&](int tile) __attribute__((always_inline)) {
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int iy0 = 4 * ty * TH - 3, ix0 = 4 * tx * TW - 4;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(img + (int64_t)b * 3 * H * W), (short)0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int t = 0; t < PFV; ++t) {
      const int e = tid + NTHR * t;
      const int c = e / (IPH * IPV), rem = e - c * (IPH * IPV);
      const int r = rem / IPV, v = rem - r * IPV;
      const int iy = iy0 + r, ix = ix0 + 4 * v;
      const bool ok = e < NIMG && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      int o = ok ? 4 * ((c * H + iy) * W + ix) : 0x7ffffff0;
      asm volatile("" : "+v"(o));   // keep the select: a split into branches would drain vmcnt
      xr[t] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
    }
  };
  auto store_img = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < PFV; ++t) {
      const int e = tid + NTHR * t;
      if (e < NIMG) {
        const int c = e / (IPH * IPV), rem = e - c * (IPH * IPV);
        const int r = rem / IPV, v = rem - r * IPV;
        bf16x4 h4;
#pragma unroll
        for (int k = 0; k < 4; ++k) h4[k] = (bf16_t)xr[t][k];
        lds_st(smem, OFF_IMG + ((c * IPH + r) * IPW + 4 * v) * 2, h4);
      }
    }
  };
  load_img(L);
  store_img();
  for (int tile = L; tile < ntiles; tile += G) {
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int oy0 = ty * TH, ox0 = tx * TW;
    const int cy0 = 2 * oy0 - 1, cx0 = 2 * ox0 - 1;
    // interior tile: every region pixel inside the 320x320 map (no zeroing checks)
    const bool interior = cy0 >= 0 && cx0 >= 0 && cy0 + R1H <= OH1 && cx0 + R1W <= OW1;
    auto in_map = [&](int rc) __attribute__((always_inline)) {
      return interior || ((unsigned)(cy0 + (rc >> 8)) < (unsigned)OH1 && (unsigned)(cx0 + (rc & 255)) < (unsigned)OW1);
    };
    __syncthreads();   // the tile's image patch is in LDS

    // ---- stage 1: stem1 over the s1 region: pixel (ry, rx) reads patch rows 2ry + ky,
    // columns 2rx + kx + 1
    if (!(DP_STEM_ABL & 1)) {
#pragma unroll
      for (int i = 0; i < PF1; ++i) {
        const int grp = wave + NWAVE * i;
        if (grp >= G1) break;
        bf16x8 xb;
#pragma unroll
        for (int e = 0; e < 8; ++e) xb[e] = lds_ld<bf16_t>(smem, poff[e] + a1[i]);
        f32x4 acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa1[j], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const bool ok = in_map(rc1[i]);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[4 * j + r] = (bf16_t)(ok ? relu_lab<LAB>(acc[j][r] + bs1[j][r], P, 0) : 0.f);
        if (grp * 16 + q < N1) lds_st(smem, OFF_S1 + g * P1 + (grp * 16 + q) * 16, o);
      }
    }
    __syncthreads();

    // ---- stage 2: stem2a over the s2a region, max-pool into cat channels 0..31
    if (!(DP_STEM_ABL & 2)) {
#pragma unroll
      for (int i = 0; i < PF2; ++i) {
        const int grp = wave + NWAVE * i;
        if (grp >= G2) break;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {   // slab s = tap (dy, dx) = (s >> 1, s & 1), channels 8g..8g+7
          const bf16x8 xb = lds_ld<bf16x8>(smem, a2[i] + ((s >> 1) * R1W + (s & 1)) * 16);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa2[s], xb, acc, 0, 0, 0);
        }
        const bool ok = in_map(rc2[i]);
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16_t)(ok ? relu_lab<LAB>(acc[r] + bs2a[r], P, 1) : 0.f);
        if (grp * 16 + q < N2) lds_st(smem, OFF_S2 + (g >> 1) * P2 + (grp * 16 + q) * 16 + (g & 1) * 8, o);
      }
#pragma unroll
      for (int t = 0; t < PFP; ++t) {
        if (tid + NTHR * t >= NPOOL) break;
        const bool ok = in_map(rcp[t]);
        u16x8 m;
        if constexpr (!LAB) {   // non-negative bf16: the unsigned 16-bit order is the value order
          const u16x8 v0 = lds_ld<u16x8>(smem, ap[t]), v1 = lds_ld<u16x8>(smem, ap[t] + 16);
          const u16x8 v2 = lds_ld<u16x8>(smem, ap[t] + R1W * 16), v3 = lds_ld<u16x8>(smem, ap[t] + R1W * 16 + 16);
          m = __builtin_elementwise_max(__builtin_elementwise_max(v0, v1), __builtin_elementwise_max(v2, v3));
        } else {
          const bf16x8 v0 = lds_ld<bf16x8>(smem, ap[t]), v1 = lds_ld<bf16x8>(smem, ap[t] + 16);
          const bf16x8 v2 = lds_ld<bf16x8>(smem, ap[t] + R1W * 16), v3 = lds_ld<bf16x8>(smem, ap[t] + R1W * 16 + 16);
          bf16x8 f;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            f[e] = (bf16_t)fmaxf(fmaxf((float)v0[e], (float)v1[e]), fmaxf((float)v2[e], (float)v3[e]));
          m = __builtin_bit_cast(u16x8, f);
        }
        if (!ok) m = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        lds_st(smem, sp[t], m);
      }
    }
    __syncthreads();

    // ---- stage 3: stem2b over the cat region -> cat channels 32..63
    if (!(DP_STEM_ABL & 4)) {
#pragma unroll
      for (int i = 0; i < PFC; ++i) {
        const int grp = wave + NWAVE * i;
        if (grp >= GC) break;
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < 2; ++s) {   // k = 32s + 8g: tap 2s + (g>>1) = (dy, dx) = (s, g>>1), channels 8(g&1)..
          const bf16x8 xb = lds_ld<bf16x8>(smem, ac[i] + s * R2W * 16);
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb2[j][s], xb, acc[j], 0, 0, 0);
        }
        const bool ok = in_map(rcc[i]);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) o[4 * j + r] = (bf16_t)(ok ? relu_lab<LAB>(acc[j][r] + bs2b[j][r], P, 2) : 0.f);
        if (grp * 16 + q < NC) lds_st(smem, OFF_CAT + (4 + g) * PC + (grp * 16 + q) * 16, o);
      }
    }
    __syncthreads();

    // ---- stage 4: next tile's image loads in flight, then stem3: wave (row i3, N tile j3),
    // K-step kk = (tap, channel half): cat pixel (2 i3 + ky, 2q + kx), chunk 4 half + g
    if (tile + G < ntiles && !(DP_STEM_ABL & 32)) load_img(tile + G);
    if (!(DP_STEM_ABL & 8)) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < K3 / 32; ++kk) {
        const int tap = kk >> 1, half = kk & 1;
        const int ky = tap / 3, kx = tap % 3;
        const bf16x8 xb = lds_ld<bf16x8>(smem, a3 + 4 * half * PC + (ky * RCW + kx) * 16);
        const bf16x8 wf = lds_ld<bf16x8>(smem, w3a + kk * 64);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xb, acc, 0, 0, 0);
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16_t)relu_lab<LAB>(acc[r] + bs3[j3][r], P, 3);
      lds_st(smem, OFF_S3 + g * P3 + (16 * i3 + q) * 16 + 8 * j3, o);   // channels 8g + 4 j3 .. +3
    }
    __syncthreads();

    // ---- stage 5: stem4 (1x1, K = 32) of row i = wave, straight to HBM
    if (wave < TH && !(DP_STEM_ABL & 16)) {
      const int i = wave;
      const int oy = oy0 + i, ox = ox0 + q;
      const bf16x8 xb = lds_ld<bf16x8>(smem, OFF_S3 + g * P3 + (16 * i + q) * 16);
      f32x4 acc[NT4];
#pragma unroll
      for (int j = 0; j < NT4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w4f[j], xb, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if (oy < OH3 && ox < OW3) {
        bf16_t* op = out + (int64_t)b * obs + ((int64_t)oy * OW3 + ox) * ops;
#pragma unroll
        for (int j = 0; j < NT4; ++j) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16_t)relu_lab<LAB>(acc[j][r] + bs4[j][r], P, 4);
          *reinterpret_cast<bf16x4*>(op + 16 * j + 4 * g) = o;
        }
      }
    }
    // next tile's image window -> LDS (its last reader, stage 1, is three barriers back)
    if (tile + G < ntiles) store_img();
  }
}

}  // namespace

namespace dpconv {
int num_cus();
}

extern "C" int dp_stem_fused(const float* image, int32_t batch, int32_t h, int32_t w, const dp_stem_weights* wts,
                             void* out, int64_t out_bstride, int32_t out_pstride, void* stream) {
  DP_REQUIRE(image && wts && out, "dp_stem_fused: null pointer");
  const dp_stem_weights& s = *wts;
  DP_REQUIRE(s.w1 && s.b1 && s.w2a && s.b2a && s.w2b && s.b2b && s.w3 && s.b3 && s.w4 && s.b4,
             "dp_stem_fused: null weight pointer");
  DP_REQUIRE(s.mid == 32 && (s.cout == 48 || s.cout == 64),
             "dp_stem_fused: stem channels [3, 32, 48|64] only (HGNetv2 B4 / B5), got mid %d out %d", s.mid, s.cout);
  DP_REQUIRE(s.k2a >= 128 && s.k2b >= 64 && s.k3 >= K3 && s.k4 >= 32 && s.k2a % 8 == 0 && s.k2b % 8 == 0 &&
                 s.k3 % 8 == 0 && s.k4 % 8 == 0,
             "dp_stem_fused: packed weight rows too short");
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  DP_REQUIRE(al16(s.w2a) && al16(s.w2b) && al16(s.w3) && al16(s.w4), "dp_stem_fused: weights must be 16-byte aligned");
  DP_REQUIRE((reinterpret_cast<uintptr_t>(out) & 7) == 0 && out_pstride % 4 == 0 && out_bstride % 4 == 0,
             "dp_stem_fused: output must be 8-byte aligned per pixel");
  DP_REQUIRE(batch > 0 && h >= 4 && w >= 4 && w % 4 == 0 && (reinterpret_cast<uintptr_t>(image) & 15) == 0 && (int64_t)3 * h * w * 4 < 0x7ff00000ll,
             "dp_stem_fused: image must be 16-byte aligned with w %% 4 == 0 and under 2 GB per image");
  const int oh3 = ((h + 1) / 2 + 1) / 2, ow3 = ((w + 1) / 2 + 1) / 2;
  const int tiles_x = (ow3 + TW - 1) / TW, tiles_y = (oh3 + TH - 1) / TH;
  const int64_t nt = (int64_t)batch * tiles_x * tiles_y;
  DP_REQUIRE(nt < (1ll << 31), "dp_stem_fused: batch too large");
  StemArgs P;
  P.w1 = s.w1, P.b1 = s.b1;
  P.w2a = reinterpret_cast<const bf16_t*>(s.w2a), P.b2a = s.b2a;
  P.w2b = reinterpret_cast<const bf16_t*>(s.w2b), P.b2b = s.b2b;
  P.w3 = reinterpret_cast<const bf16_t*>(s.w3), P.b3 = s.b3;
  P.w4 = reinterpret_cast<const bf16_t*>(s.w4), P.b4 = s.b4;
  P.k2a = s.k2a, P.k2b = s.k2b, P.k3 = s.k3, P.k4 = s.k4;
  for (int i = 0; i < 5; ++i) P.lab[i][0] = s.lab[i][0], P.lab[i][1] = s.lab[i][1];
  const int ntiles = (int)nt;
  int grid = dpconv::num_cus();   // one 8-wave block per CU (115 KB of LDS)
  const int need = (ntiles + 7) / 8 * 8;
  if (grid > need) grid = need;
  grid = grid / 8 * 8;
  if (grid < 8) grid = 8;
  hipStream_t st = as_stream(stream);
  bf16_t* o = reinterpret_cast<bf16_t*>(out);
#define DP_STEM_LAUNCH(C_, L_)                                                                                    \
  hipLaunchKernelGGL((stem_fused_kernel<C_, L_>), dim3(grid), dim3(NTHR), 0, st, image, h, w, P, o, out_bstride,     \
                     out_pstride, tiles_x, tiles_y, ntiles)
  if (s.cout == 48 && !s.has_lab) DP_STEM_LAUNCH(48, false);
  else if (s.cout == 48) DP_STEM_LAUNCH(48, true);
  else if (!s.has_lab) DP_STEM_LAUNCH(64, false);
  else DP_STEM_LAUNCH(64, true);
#undef DP_STEM_LAUNCH
  return dp_check_launch("dp_stem_fused");
}
