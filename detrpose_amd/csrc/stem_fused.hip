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
// the packed weights (tap-major, k = tap * cin + ci; stem1: stem_k.h) and f32 accumulation in
// the same sequence as the unfused kernels, bf16 rounding at the same points (each stage's
// output): the result matches the five-launch path bit for bit. 32-channel outputs use the
// permuted weight rows of stem.hip (lane g holds channels 8g .. 8g+7: one 16-byte LDS store).
// Weights: stem1/2a/2b/4 fragments in registers for the block's life, stem3's 32 x 576 in
// LDS. The image: the tile's (4TH+7) x (4TW+8) x 3 window is loaded with coalesced 16-byte
// loads two tiles ahead, rounded to bf16 into a pixel-major LDS patch ([row][col][c0 c1 c2 0],
// 8 bytes a pixel), so each stem1 B fragment is two 8-byte reads of two taps' channels.
//
// Pipeline (per-stage ablation, profiles/r6h_stem_ablation.txt: every stage of the five-barrier
// form cost 70-130 us at L b64, latency rather than work at two waves per SIMD): one block per
// CU walks its tiles in three barrier phases per tile,
//   A: waves 0-3: stem3 of tile t (one output row each, both 16-channel halves) and stem4
//      straight from stem3's registers (the C layout of stem3 is stem4's B fragment), to HBM;
//      waves 4-7: stem1 of tile t+1 (image patch -> s1); every wave issues tile t+2's image loads
//   B: stem2a (s1 -> s2a) and the max-pool (s1 -> cat 0..31) of tile t+1
//   C: stem2b (s2a -> cat 32..63) of tile t+1; tile t+2's image -> LDS patch
// so stem1 overlaps stem3/stem4 and the image latency hides behind three phases. Barriers wait
// for LDS traffic only (lgkmcnt), never for the image loads in flight.
#include "common.h"
#include "stem_k.h"

//
// LDS layout: the stage maps are stored planar by 16-byte channel chunk ([chunk][pixel],
// 16 B per pixel per plane) so that the 16 lanes of an MFMA B-fragment read (16 consecutive
// pixels, one chunk per lane group) hit 16 distinct bank slots: plane strides are multiples of
// 256 B (cat: 16 mod 256, whose stem3 reads step 2 pixels per lane).

namespace {

constexpr int TH = 4, TW = 16;   // stem3 / stem4 output tile: 4 rows x 16 columns, 8 waves
constexpr int NWAVE = 8, NTHR = 64 * NWAVE;
constexpr int R1H = 2 * TH + 3, R1W = 2 * TW + 3, N1 = R1H * R1W;   // 11 x 35 stem1 region
constexpr int R2H = 2 * TH + 2, R2W = 2 * TW + 2, N2 = R2H * R2W;   // 10 x 34 stem2a region
constexpr int RCH = 2 * TH + 1, RCW = 2 * TW + 1, NC = RCH * RCW;   //  9 x 33 cat region
constexpr int G1 = (N1 + 15) / 16, G2 = (N2 + 15) / 16, GC = (NC + 15) / 16;
constexpr int PF2 = (G2 + NWAVE - 1) / NWAVE, PFC = (GC + NWAVE - 1) / NWAVE;
constexpr int K3 = 9 * 64;
constexpr int W3ROW = K3 * 2 + 16;             // +16 B: 16 consecutive rows hit 16 distinct bank slots
constexpr int rup(int x, int m) { return (x + m - 1) / m * m; }
constexpr int P1 = rup(N1 * 16, 256), P2 = rup(N2 * 16, 256), PC = rup(NC * 16 - 16, 256) + 16;
constexpr int OFF_S1 = 0, OFF_S2 = OFF_S1 + 4 * P1, OFF_CAT = OFF_S2 + 2 * P2, OFF_W3 = OFF_CAT + 8 * PC;
// image patch: rows 4 oy0 - 3 .. +IPH-1, columns 4 ox0 - 4 .. +IPW-1 (16-byte aligned starts),
// 8 bytes a pixel; the row stride is 8 mod 16 bytes (146 dwords, 18 mod 64 banks), so the two
// rows of one fragment read (and lane groups g, g+1) land on disjoint bank pairs
constexpr int IPH = 2 * R1H + 1, IPW = 2 * R1W + 2;                 // 23 x 72
constexpr int IRS = IPW * 8 + 8;
constexpr int IPV = IPW / 4, NIMG = IPH * IPV;                      // 4-column items (3 float4 loads each)
constexpr int OFF_IMG = OFF_W3 + 32 * W3ROW;
constexpr int OFF_Z = OFF_IMG + IPH * IRS;                          // 8 zero bytes (slab 1 of lanes g > 0)
constexpr int LDS_BYTES = OFF_Z + 16;
// every 16-pixel group's lanes store unconditionally: the planes hold whole groups (lanes past the
// region write padding no stage reads)
static_assert(P1 >= G1 * 16 * 16 && P2 >= G2 * 16 * 16 && PC >= GC * 16 * 16, "plane padding");
static_assert(LDS_BYTES <= 160 * 1024 && TH * TW == 16 * 4 && IPW % 4 == 0 && OFF_IMG % 16 == 0 && NIMG <= NTHR &&
                  TH == NWAVE / 2,
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

// block barrier for LDS hand-offs: LDS traffic retired, then s_barrier; the image loads in
// flight (vmcnt) are not waited for
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// folded-BN bias + ReLU (+ LAB); + 0.f turns a -0 into +0, so the non-negative bf16 maps can
// be max-pooled as unsigned 16-bit integers
template <bool LAB>
__device__ __forceinline__ float relu_lab(float x, const StemArgs& P, int s) {
  x = fmaxf(x, 0.f) + 0.f;
  if constexpr (LAB) x = P.lab[s][0] * x + P.lab[s][1];
  return x;
}

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// bf16(relu(a + ba)), bf16(relu(b + bb)) as one dword: the f32 bias adds (one packed add), round
// to bf16 (RNE), then ReLU on the bf16 bits: a negative value or -0 has the sign bit set, so
// max with 0 as int16 gives +0 — the same bits as rounding relu(x) for every finite x
__device__ __forceinline__ unsigned relu_pk(float a, float b, float ba, float bb) {
  const f32x2 v = f32x2{a, b} + f32x2{ba, bb};
  const bf16x2 h = __builtin_convertvector(v, bf16x2);   // one v_cvt_pk_bf16_f32
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2, h), s16x2{0, 0}));
}

// a stage's output of 8 channels (C tiles j = 0, 1; element 4j + r): bias + ReLU (+ LAB),
// zero outside the map (!ok)
template <bool LAB>
__device__ __forceinline__ bf16x8 epi8(const f32x4 (&acc)[2], const float (&bs)[2][4], bool ok, const StemArgs& P,
                                       int s) {
  if constexpr (LAB) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[4 * j + r] = (bf16_t)(ok ? relu_lab<LAB>(acc[j][r] + bs[j][r], P, s) : 0.f);
    return o;
  } else {
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const unsigned v = relu_pk(acc[j][2 * h], acc[j][2 * h + 1], bs[j][2 * h], bs[j][2 * h + 1]);
        w[2 * j + h] = ok ? v : 0u;
      }
    return __builtin_bit_cast(bf16x8, w);
  }
}

// 4 channels of one C tile
template <bool LAB>
__device__ __forceinline__ bf16x4 epi4(const f32x4& acc, const float (&bs)[4], bool ok, const StemArgs& P, int s) {
  if constexpr (LAB) {
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (bf16_t)(ok ? relu_lab<LAB>(acc[r] + bs[r], P, s) : 0.f);
    return o;
  } else {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    u32x2 w;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned v = relu_pk(acc[2 * h], acc[2 * h + 1], bs[2 * h], bs[2 * h + 1]);
      w[h] = ok ? v : 0u;
    }
    return __builtin_bit_cast(bf16x4, w);
  }
}

// a tile's place: image b, stem3 output origin (oy0, ox0), region origin (cy0, cx0) in the
// 320x320 stage maps, and whether every region pixel lies inside them (no zeroing checks)
struct TileGeom {
  int b, oy0, ox0, cy0, cx0;
  bool interior;
};

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
  if (tid == 0) lds_st(smem, OFF_Z, u32x4{0u, 0u, 0u, 0u});
  // ---- register weights and biases
  bf16x8 wa1[2][2], wa2[4], wb2[2][2], w4f[NT4];   // wa1: [K slab][16-channel tile]
#pragma unroll
  for (int sl = 0; sl < 2; ++sl)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int c = 0, ky = 0, kx = 0;
      const bool ok = stem1_slot(sl, g, e, c, ky, kx);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        wa1[sl][j][e] = (bf16_t)(ok ? P.w1[chan32(j, q >> 2, q & 3) * 27 + c * 9 + ky * 3 + kx] : 0.f);
    }
  // stem1 slab-0 fragment: two taps' 8-byte pixels at these offsets from the pixel's tap (0, 0)
  const int o1a = g < 3 ? g * IRS : IRS + 16, o1b = g < 3 ? g * IRS + 8 : 16;
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

  auto geom = [&](int tile) __attribute__((always_inline)) {
    TileGeom t;
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y;
    t.b = rest / tiles_y;
    t.oy0 = ty * TH, t.ox0 = tx * TW;
    t.cy0 = 2 * t.oy0 - 1, t.cx0 = 2 * t.ox0 - 1;
    t.interior = t.cy0 >= 0 && t.cx0 >= 0 && t.cy0 + R1H <= OH1 && t.cx0 + R1W <= OW1;
    return t;
  };
  auto in_map = [&](const TileGeom& t, int ry, int rx) __attribute__((always_inline)) {
    return t.interior || ((unsigned)(t.cy0 + ry) < (unsigned)OH1 && (unsigned)(t.cx0 + rx) < (unsigned)OW1);
  };

  // ---- image window of a tile: thread (row r, 4 columns v) loads the 3 channels' float4s
  // (buffer loads: an out-of-range offset returns 0 = the conv's zero padding; W % 4 == 0 so a
  // float4 is wholly in or out), then writes 4 pixels [c0 c1 c2 0] to the patch
  f32x4 xr[3];
  auto load_img = [&](int tile) __attribute__((always_inline)) {
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int iy0 = 4 * ty * TH - 3, ix0 = 4 * tx * TW - 4;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(img + (int64_t)b * 3 * H * W), (short)0, 0x7ffffff0, 0x00020000);
    const int r = tid / IPV, v = tid - r * IPV;
    const int iy = iy0 + r, ix = ix0 + 4 * v;
    const bool ok = tid < NIMG && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      int o = ok ? 4 * ((c * H + iy) * W + ix) : 0x7ffffff0;
      asm volatile("" : "+v"(o));   // keep the select: a split into branches would drain vmcnt
      xr[c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
    }
  };
  auto store_img = [&]() __attribute__((always_inline)) {
    if (tid < NIMG) {
      const int r = tid / IPV, v = tid - r * IPV;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const bf16x2 h01 = __builtin_convertvector(f32x2{xr[0][x], xr[1][x]}, bf16x2);
        const bf16x2 h2z = __builtin_convertvector(f32x2{xr[2][x], 0.f}, bf16x2);
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        lds_st(smem, OFF_IMG + r * IRS + (4 * v + x) * 8,
               u32x2{__builtin_bit_cast(unsigned, h01), __builtin_bit_cast(unsigned, h2z)});
      }
    }
  };

  // ---- stem1 over the s1 region (groups wsub, wsub + NW, ...): pixel (ry, rx) reads patch
  // rows 2ry + ky, columns 2rx + kx + 1
  auto stage1 = [&](const TileGeom& t, int wsub, auto nw_c) __attribute__((always_inline)) {
    constexpr int NW = decltype(nw_c)::value;
#pragma unroll
    for (int i = 0; i < (G1 + NW - 1) / NW; ++i) {
      const int grp = wsub + NW * i;
      if (grp >= G1) break;
      const int p = min(grp * 16 + q, N1 - 1);
      const int ry = p / R1W, rx = p - ry * R1W;
      const int base = OFF_IMG + 2 * ry * IRS + (2 * rx + 1) * 8;
      const bf16x4 lo = lds_ld<bf16x4>(smem, base + o1a), hi = lds_ld<bf16x4>(smem, base + o1b);
      const bf16x4 z = lds_ld<bf16x4>(smem, g == 0 ? base + 2 * IRS + 16 : OFF_Z);   // tap (2, 2)
      const bf16x8 xb0 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const bf16x8 xb1 = {z[0], z[1], z[2], z[3], (bf16_t)0.f, (bf16_t)0.f, (bf16_t)0.f, (bf16_t)0.f};
      f32x4 acc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa1[0][j], xb0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa1[1][j], xb1, acc[j], 0, 0, 0);
      }
      const bf16x8 o = epi8<LAB>(acc, bs1, in_map(t, ry, rx), P, 0);
      lds_st(smem, OFF_S1 + g * P1 + (grp * 16 + q) * 16, o);   // lanes past N1: plane padding
    }
  };

  // ---- stem2a over the s2a region (all waves). Its four K slabs are the 2x2 window's taps of
  // channels 8g..8g+7, the max-pool's window at the same position (the cat region is the s2a
  // region minus its last row and column): their max is the pool output, cat channels 0..31
  auto stage2 = [&](const TileGeom& t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PF2; ++i) {
      const int grp = wave + NWAVE * i;
      if (grp >= G2) break;
      const int p = min(grp * 16 + q, N2 - 1);
      const int ry = p / R2W, rx = p - ry * R2W;
      const int a2 = OFF_S1 + g * P1 + (ry * R1W + rx) * 16;
      bf16x8 xb[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) xb[s] = lds_ld<bf16x8>(smem, a2 + ((s >> 1) * R1W + (s & 1)) * 16);
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 4; ++s)   // slab s = tap (dy, dx) = (s >> 1, s & 1), channels 8g..8g+7
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa2[s], xb[s], acc, 0, 0, 0);
      const bool ok = in_map(t, ry, rx);
      const bf16x4 o = epi4<LAB>(acc, bs2a, ok, P, 1);
      lds_st(smem, OFF_S2 + (g >> 1) * P2 + (grp * 16 + q) * 16 + (g & 1) * 8, o);   // past N2: padding
      u16x8 m;
      if constexpr (!LAB) {   // non-negative bf16: the unsigned 16-bit order is the value order
        const u16x8 v0 = __builtin_bit_cast(u16x8, xb[0]), v1 = __builtin_bit_cast(u16x8, xb[1]);
        const u16x8 v2 = __builtin_bit_cast(u16x8, xb[2]), v3 = __builtin_bit_cast(u16x8, xb[3]);
        m = __builtin_elementwise_max(__builtin_elementwise_max(v0, v1), __builtin_elementwise_max(v2, v3));
      } else {
        bf16x8 f;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          f[e] = (bf16_t)fmaxf(fmaxf((float)xb[0][e], (float)xb[1][e]), fmaxf((float)xb[2][e], (float)xb[3][e]));
        m = __builtin_bit_cast(u16x8, f);
      }
      if (!ok) m = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (ry < RCH && rx < RCW) lds_st(smem, OFF_CAT + g * PC + (ry * RCW + rx) * 16, m);   // clamped lanes: ry = 9
    }
  };

  // ---- stem2b over the cat region -> cat channels 32..63 (all waves)
  auto stage3 = [&](const TileGeom& t) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PFC; ++i) {
      const int grp = wave + NWAVE * i;
      if (grp >= GC) break;
      const int p = min(grp * 16 + q, NC - 1);
      const int ry = p / RCW, rx = p - ry * RCW;
      const int ac = OFF_S2 + (g & 1) * P2 + (ry * R2W + rx + (g >> 1)) * 16;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 2; ++s) {   // k = 32s + 8g: tap 2s + (g>>1) = (dy, dx) = (s, g>>1), channels 8(g&1)..
        const bf16x8 xb = lds_ld<bf16x8>(smem, ac + s * R2W * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb2[j][s], xb, acc[j], 0, 0, 0);
      }
      const bf16x8 o = epi8<LAB>(acc, bs2b, in_map(t, ry, rx), P, 2);
      lds_st(smem, OFF_CAT + (4 + g) * PC + (grp * 16 + q) * 16, o);   // past NC: padding, never read
    }
  };

  // ---- stem3 of output row i = wave (waves 0..3), both 16-channel halves: K-step kk = (tap,
  // channel half) reads cat pixel (2i + ky, 2q + kx), chunk 4 half + g; then stem4 (1x1, K = 32)
  // on stem3's bf16 output as the B fragment (lane (q, g) holds channels 8g..8g+7), to HBM
  auto stage45 = [&](const TileGeom& t) __attribute__((always_inline)) {
    const int i = wave;
    const int a3 = OFF_CAT + g * PC + (2 * i * RCW + 2 * q) * 16;
    const int w3a = OFF_W3 + q * W3ROW + 16 * g;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < K3 / 32; ++kk) {
      const int tap = kk >> 1, half = kk & 1;
      const int ky = tap / 3, kx = tap % 3;
      const bf16x8 xb = lds_ld<bf16x8>(smem, a3 + 4 * half * PC + (ky * RCW + kx) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16x8 wf = lds_ld<bf16x8>(smem, w3a + 16 * j * W3ROW + kk * 64);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xb, acc[j], 0, 0, 0);
      }
    }
    const bf16x8 x4 = epi8<LAB>(acc, bs3, true, P, 3);
    f32x4 a4[NT4];
#pragma unroll
    for (int j = 0; j < NT4; ++j)
      a4[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w4f[j], x4, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    const int oy = t.oy0 + i, ox = t.ox0 + q;
    if (oy < OH3 && ox < OW3) {
      bf16_t* op = out + (int64_t)t.b * obs + ((int64_t)oy * OW3 + ox) * ops;
#pragma unroll
      for (int j = 0; j < NT4; ++j) *reinterpret_cast<bf16x4*>(op + 16 * j + 4 * g) = epi4<LAB>(a4[j], bs4[j], true, P, 4);
    }
  };

  // ---- prologue: tile L through stem2b
  TileGeom cur = geom(L);
  load_img(L);
  store_img();
  lds_barrier();
  stage1(cur, wave, std::integral_constant<int, NWAVE>{});
  lds_barrier();
  int nxt = L + G;
  if (nxt < ntiles) load_img(nxt);
  stage2(cur);
  lds_barrier();
  stage3(cur);
  if (nxt < ntiles) store_img();
  lds_barrier();
  // ---- steady state: phase A (stem3/stem4 of cur | stem1 of nxt), B, C (stem2a/pool, stem2b of nxt)
  for (;;) {
    const bool more = nxt < ntiles;
    const TileGeom nx = geom(more ? nxt : L);
    if (more && nxt + G < ntiles) load_img(nxt + G);
    if (wave < NWAVE / 2) stage45(cur);
    else if (more) stage1(nx, wave - NWAVE / 2, std::integral_constant<int, NWAVE / 2>{});
    if (!more) break;
    lds_barrier();
    stage2(nx);
    lds_barrier();
    stage3(nx);
    if (nxt + G < ntiles) store_img();
    lds_barrier();
    cur = nx;
    nxt += G;
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
  int grid = dpconv::num_cus();   // one 8-wave block per CU (124 KB of LDS)
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
