// Implicit-GEMM convolution / linear for gfx950 (MFMA), NHWC: the f32 (parity mode)
// kernel and the dp_conv2d entry point; bf16 dispatches to conv_halo.hip / conv_stream.hip.
//
// Replaces every dense nn.Conv2d(+BN)(+act) and nn.Linear on the DETRPose forward:
//   ConvBNAct (hgnetv2.py:82-134), ConvNormLayer(_fuse) (hybrid_encoder.py:56-128),
//   VGGBlock deploy conv (hybrid_encoder.py:139-189), the MHA in/out projections,
//   FFN / Gate / MSDA-projection / MLP-head linears (transformer.py, utils.py:75-87).
//
// GEMM view: C[M=batch*oh*ow][N=cout] = A[M][K] * W[N][K]^T, K = kh*kw*cin, A gathered
// on the fly from the NHWC input.  Both operands are K-major, the native operand
// layout of v_mfma_f32_16x16x32_bf16 (lane l holds 8 consecutive k of row l&15), so
// staging is straight 16-byte copies.
//
// Loads are buffer loads from a per-block descriptor (base = first image the block
// touches, 32-bit offsets): an out-of-range offset returns 0, which is exactly the
// conv zero padding, the K tail and the M/N tails — no branches or exec juggling around
// the loads (T8/T20 of the CDNA guide). The next PD K-steps are kept in flight in
// registers while the current one runs from LDS (double-buffered, one barrier per
// K-step). 4 waves per block arranged WGM x WGN; BN may be 16/32/48/64/128 so narrow
// layers (stem, stage-1 48-channel convs) do not pay for a 64/128-wide tile.
// Epilogue: bias (folded BN), activation, LAB, staged through LDS and written as
// 16-byte rows with the residual add (HG_Block identity, CSP x_1 + x_2), an optional
// nearest-x2 copy (FPN upsample + concat, hybrid_encoder.py:495-496), f32 or bf16 out.
// Blocks are remapped so each XCD walks a contiguous range of tiles: the N-tiles that
// share one A tile run on one XCD (L2 reuse of the gathered activations).
#include "common.h"
#include "conv_epilogue.h"
#include <stdlib.h>

namespace {

constexpr int OOB = 0x7fffffff;  // voffset beyond num_records -> load returns 0

template <typename T, typename TO, int BM, int BN, int BK>
struct Cfg {
  static constexpr int VEC = 16 / sizeof(T);          // elements per 16-byte chunk
  static constexpr int CH = BK / VEC;                 // chunks per row per K-step
  static constexpr int BKP = BK + VEC;                // LDS row pitch (+16 B pad)
  static constexpr int RPP = 256 / CH;                // rows covered per thread pass
  static constexpr int AR = (BM + RPP - 1) / RPP;     // A row-passes per thread
  static constexpr int BR = (BN + RPP - 1) / RPP;     // B row-passes per thread
  static constexpr int AB = 2 * (BM + BN) * BKP * (int)sizeof(T);
  static constexpr int VO = 16 / sizeof(TO);
  static constexpr int CP = BN + VO;
  static constexpr int CB = BM * CP * (int)sizeof(TO);
  static constexpr int BYTES = AB > CB ? AB : CB;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7ffffff0, 0x00020000);
}

template <typename T>
__device__ __forceinline__ Vec16<T> bload(__amdgpu_buffer_rsrc_t r, int byte_off) {
  Vec16<T> v;
  auto x = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  *reinterpret_cast<decltype(x)*>(&v.v) = x;
  return v;
}

template <typename T, typename TO, int BM, int BN, int BK, int WGM, int PD, bool K1X1>
__global__ __launch_bounds__(256) void conv_gemm_kernel(dp_conv_desc d, int M, int nt_n, int vec_ok) {
  using G = Cfg<T, TO, BM, BN, BK>;
  constexpr int VEC = G::VEC, CH = G::CH, BKP = G::BKP, RPP = G::RPP, AR = G::AR, BR = G::BR;
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;        // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;          // 16x16 MFMA tiles per wave
  static_assert(TM >= 1 && TN >= 1 && WM % 16 == 0 && WN % 16 == 0, "bad wave tile");
  __shared__ __attribute__((aligned(16))) char smem_raw[G::BYTES];
  T* As = reinterpret_cast<T*>(smem_raw);   // [2][BM][BKP]
  T* Bs = As + 2 * BM * BKP;                // [2][BN][BKP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  // XCD-aware bijective remap of the 1-D grid (blocks b, b+8, ... share an XCD)
  const int nwg = gridDim.x, pid = blockIdx.x;
  const int xcd = pid & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (pid >> 3);
  const int tn = logical % nt_n, tm = logical / nt_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int hwo = d.out_h * d.out_w;
  const int b_first = m0 / hwo;
  const __amdgpu_buffer_rsrc_t ra_src = make_rsrc(reinterpret_cast<const T*>(d.in) + (int64_t)b_first * d.in_bstride);
  const __amdgpu_buffer_rsrc_t rb_src = make_rsrc(d.weight);
  const int chunk = tid % CH;
  const int row0 = tid / CH;

  // per-thread A rows: element offset of the row's pixel (K1X1) or of its image (KxK)
  int a_off[AR], a_iy0[AR], a_ix0[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + row0 + i * RPP;
    const bool ok = m < M && row0 + i * RPP < BM;
    const int mm = ok ? m : m0;
    const int b = mm / hwo, rem = mm - b * hwo;
    const int oy = rem / d.out_w, ox = rem - oy * d.out_w;
    const int iy0 = oy * d.stride - d.pad_t;
    a_iy0[i] = ok ? iy0 : -0x4000000;   // masked rows fail every bounds test
    a_ix0[i] = ox * d.stride - d.pad_l;
    int off = (b - b_first) * (int)d.in_bstride;
    if (K1X1) off += (iy0 * d.in_w + a_ix0[i]) * d.in_pstride;
    a_off[i] = ok ? off : OOB;
  }
  int b_off[BR];
#pragma unroll
  for (int j = 0; j < BR; ++j) {
    const int n = n0 + row0 + j * RPP;
    b_off[j] = (n < d.cout && row0 + j * RPP < BN) ? n * d.kpad + chunk * VEC : OOB;
  }
  const int ntap = d.kh * d.kw;

  Vec16<T> ra[PD][AR], rb[PD][BR];
  auto g2r = [&](int kt, int set) {
    const int kk = kt * BK + chunk * VEC;
    if (K1X1) {
      const bool kv = kk < d.cin;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int o = (a_off[i] != OOB && kv) ? (a_off[i] + kk) * (int)sizeof(T) : OOB;
        ra[set][i] = bload<T>(ra_src, o);
      }
    } else {
      const int tap = kk / d.cin, ci = kk - tap * d.cin;
      const int ky = tap / d.kw, kx = tap - ky * d.kw;
      const bool kv = tap < ntap;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int iy = a_iy0[i] + ky, ix = a_ix0[i] + kx;
        const bool ok = kv && (unsigned)iy < (unsigned)d.in_h && (unsigned)ix < (unsigned)d.in_w;
        const int o = ok ? (a_off[i] + (iy * d.in_w + ix) * d.in_pstride + ci) * (int)sizeof(T) : OOB;
        ra[set][i] = bload<T>(ra_src, o);
      }
    }
#pragma unroll
    for (int j = 0; j < BR; ++j)
      rb[set][j] = bload<T>(rb_src, b_off[j] != OOB ? (b_off[j] + kt * BK) * (int)sizeof(T) : OOB);
  };
  auto r2s = [&](int set, int buf) {
    T* a = As + buf * BM * BKP;
    T* b = Bs + buf * BN * BKP;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      if (row0 + i * RPP < BM) store16(a + (row0 + i * RPP) * BKP + chunk * VEC, ra[set][i]);
#pragma unroll
    for (int j = 0; j < BR; ++j)
      if (row0 + j * RPP < BN) store16(b + (row0 + j * RPP) * BKP + chunk * VEC, rb[set][j]);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = d.kpad / BK;
  g2r(0, 0);
  if (PD == 2 && nk > 1) g2r(1, PD - 1);
  r2s(0, 0);
  __syncthreads();
  // K loop unrolled by PD so every register-set index is a compile-time constant
  for (int k0 = 0; k0 < nk; k0 += PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      const int kt = k0 + u;
      if (kt >= nk) break;
      const int cur = kt & 1;
      if (kt + PD < nk) g2r(kt + PD, u);   // set u (== kt % PD) was moved to LDS already
      const T* a = As + cur * BM * BKP + (wm * WM + (lane & 15)) * BKP;
      const T* b = Bs + cur * BN * BKP + (wn * WN + (lane & 15)) * BKP;
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
          bf16x8 af[TM], bfr[TN];
          const int ko = ks * 32 + (lane >> 4) * 8;
#pragma unroll
          for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(a + i * 16 * BKP + ko);
#pragma unroll
          for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * BKP + ko);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
          float af[TM], bfr[TN];
          const int ko = ks * 4 + (lane >> 4);
#pragma unroll
          for (int i = 0; i < TM; ++i) af[i] = to_f32(a[i * 16 * BKP + ko]);
#pragma unroll
          for (int j = 0; j < TN; ++j) bfr[j] = to_f32(b[j * 16 * BKP + ko]);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      }
      if (kt + 1 < nk) r2s((u + 1) % PD, cur ^ 1);
      __syncthreads();
    }
  }

  conv_epilogue<TO, BM, BN, WGM, TM, TN>(d, acc, smem_raw, M, m0, n0, vec_ok);
}

#ifndef DP_CONV_PD
#define DP_CONV_PD 1
#endif
#ifndef DP_SMALLN_BM
#define DP_SMALLN_BM 128   // row tile of narrow (cout <= 64) layers
#endif

template <typename T, typename TO, int BM, int BN, int BK, int WGM>
int launch(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  const int M = d.batch * d.out_h * d.out_w;
  const int mt = (M + BM - 1) / BM, nt = (d.cout + BN - 1) / BN;
  const bool k1 = d.kh == 1 && d.kw == 1 && d.pad_t == 0 && d.pad_l == 0;
  DP_DESCRIBE("conv_gemm_kernel<%s, %s, %d, %d, %d, %d, %d, %s>", sizeof(T) == 2 ? "bf16" : "float",
              sizeof(TO) == 2 ? "bf16" : "float", BM, BN, BK, WGM, DP_CONV_PD, DP_TF(sizeof(TO) != sizeof(T) || k1));
  dim3 grid(mt * nt), block(256);
  constexpr int PD = DP_CONV_PD;
  if constexpr (sizeof(TO) != sizeof(T)) {
    hipLaunchKernelGGL((conv_gemm_kernel<T, TO, BM, BN, BK, WGM, PD, true>), grid, block, 0, s, d, M, nt, vec_ok);
  } else {
    if (k1) hipLaunchKernelGGL((conv_gemm_kernel<T, TO, BM, BN, BK, WGM, PD, true>), grid, block, 0, s, d, M, nt, vec_ok);
    else hipLaunchKernelGGL((conv_gemm_kernel<T, TO, BM, BN, BK, WGM, PD, false>), grid, block, 0, s, d, M, nt, vec_ok);
  }
  return dp_check_launch("dp_conv2d");
}

// conv_stream.hip / conv_halo.hip
}  // namespace
int dp_conv2d_stream(const dp_conv_desc& d, hipStream_t s, int vec_ok);
int dp_conv2d_halo(const dp_conv_desc& d, hipStream_t s, int vec_ok);
int dp_conv2d_stem_direct(const dp_conv_desc& d, hipStream_t s, void* pool, int64_t pbs, int pps);
namespace {

template <typename T, typename TO>
int dispatch(const dp_conv_desc& d, hipStream_t s) {
  constexpr int VO = 16 / sizeof(TO);
  constexpr int BK = 128 / sizeof(T);   // 64 bf16 / 32 f32: 128 bytes of k per row
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  int vec_ok = (d.out_pstride % VO == 0) && (d.out_bstride % VO == 0) && al(d.out);
  if (d.res) vec_ok = vec_ok && (d.res_pstride % VO == 0) && (d.res_bstride % VO == 0) && al(d.res);
  if (d.up) vec_ok = vec_ok && (d.up_pstride % VO == 0) && (d.up_bstride % VO == 0) && al(d.up);
  const int M = d.batch * d.out_h * d.out_w;
  if constexpr (sizeof(T) == 2) {
    if (d.in_seg_ch) return dp_conv2d_stream(d, s, vec_ok);   // segmented input: the 1x1 GEMM path
    // bf16: LDS halo-tile kernel for the KxK convs it covers, persistent LDS-DMA GEMM otherwise
    if (d.kh <= 2 && d.cin <= 32) {   // the stem's 2x2 / 1x1 convs: register-direct kernels
      const int r = dp_conv2d_stem_direct(d, s, nullptr, 0, 0);
      if (r >= 0) return r;
    }
    if (d.kh * d.kw > 1) {
      const int r = dp_conv2d_halo(d, s, vec_ok);
      if (r >= 0) return r;
    }
    return dp_conv2d_stream(d, s, vec_ok);
  } else {
    constexpr int SB = DP_SMALLN_BM;
    if (d.cout <= 16) return launch<T, TO, SB, 16, BK, 4>(d, s, vec_ok);
    if (d.cout <= 32) return launch<T, TO, SB, 32, BK, 4>(d, s, vec_ok);
    if (d.cout <= 48) return launch<T, TO, SB, 48, BK, 4>(d, s, vec_ok);
    if (d.cout <= 64) return launch<T, TO, SB, 64, BK, 4>(d, s, vec_ok);
    if (M <= 8192) return launch<T, TO, 64, 128, BK, 2>(d, s, vec_ok);
    return launch<T, TO, 128, 128, BK, 2>(d, s, vec_ok);
  }
}

}  // namespace

static int conv2d_impl(const dp_conv_desc* dp, void* stream);

extern "C" int dp_conv2d(const dp_conv_desc* dp, void* stream) { return conv2d_impl(dp, stream); }

extern "C" int dp_conv2d_describe(const dp_conv_desc* dp, char* buf, int32_t buflen) {
  DP_REQUIRE(buf != nullptr && buflen > 0, "dp_conv2d_describe: no buffer");
  buf[0] = 0;
  dp_describe_set(buf, buflen);
  const int r = conv2d_impl(dp, nullptr);
  dp_describe_set(nullptr, 0);
  return r;
}

static int conv2d_impl(const dp_conv_desc* dp, void* stream) {
  DP_REQUIRE(dp != nullptr, "dp_conv2d: null descriptor");
  const dp_conv_desc& d = *dp;
  const int VEC = d.dtype == DP_BF16 ? 8 : 4;
  const int BK = d.dtype == DP_BF16 ? 64 : 32;
  const int es = d.dtype == DP_BF16 ? 2 : 4;
  DP_REQUIRE(d.dtype == DP_BF16 || d.dtype == DP_F32, "dp_conv2d: bad dtype %d", d.dtype);
  DP_REQUIRE(d.in && d.weight && d.out, "dp_conv2d: null pointer");
  DP_REQUIRE(d.batch > 0 && d.out_h > 0 && d.out_w > 0 && d.cout > 0 && d.cin > 0, "dp_conv2d: bad shape");
  DP_REQUIRE(d.cin % VEC == 0, "dp_conv2d: cin=%d must be a multiple of %d", d.cin, VEC);
  DP_REQUIRE(d.in_pstride % VEC == 0 && d.in_bstride % VEC == 0 &&
                 (reinterpret_cast<uintptr_t>(d.in) & 15) == 0,
             "dp_conv2d: input must be 16-byte aligned per pixel (pstride=%d)", d.in_pstride);
  DP_REQUIRE(d.kpad % BK == 0 && d.kpad >= d.kh * d.kw * d.cin, "dp_conv2d: kpad=%d invalid (K=%d, BK=%d)",
             d.kpad, d.kh * d.kw * d.cin, BK);
  DP_REQUIRE((reinterpret_cast<uintptr_t>(d.weight) & 15) == 0, "dp_conv2d: weight not 16-byte aligned");
  DP_REQUIRE((int64_t)d.batch * d.out_h * d.out_w < (1ll << 31), "dp_conv2d: M too large");
  // 32-bit buffer offsets: a block spans at most ceil(256 / (oh*ow)) + 1 images of the input,
  // and the weight tensor must fit as well
  const int64_t hwo = (int64_t)d.out_h * d.out_w;
  const int64_t span = ((256 + hwo - 1) / hwo + 1) * d.in_bstride * es;
  DP_REQUIRE(span < 0x7ff00000ll && (int64_t)d.cout * d.kpad * es < 0x7ff00000ll,
             "dp_conv2d: per-block input span / weight exceeds 2 GB of 32-bit buffer offsets");
  DP_REQUIRE(!d.out_f32 || (d.kh == 1 && d.kw == 1 && d.pad_t == 0 && d.pad_l == 0 && !d.up),
             "dp_conv2d: out_f32 is supported for 1x1 / linear layers without upsample");
  DP_REQUIRE(!d.in_seg_ch || (d.dtype == DP_BF16 && d.kh == 1 && d.kw == 1 && d.stride == 1 && d.pad_t == 0 &&
                              d.pad_l == 0 && d.in_seg_ch % 8 == 0 && d.cin % d.in_seg_ch == 0 &&
                              d.in_seg_stride % 8 == 0 &&
                              span + (d.cin / d.in_seg_ch - 1) * d.in_seg_stride * es < 0x7ff00000ll),
             "dp_conv2d: segmented input only for bf16 1x1 convs, in_seg_ch %% 8 == 0 dividing cin, "
             "segments within 2 GB of 32-bit offsets");
  hipStream_t s = as_stream(stream);
  if (d.dtype == DP_BF16) return d.out_f32 ? dispatch<bf16_t, float>(d, s) : dispatch<bf16_t, bf16_t>(d, s);
  return dispatch<float, float>(d, s);
}
