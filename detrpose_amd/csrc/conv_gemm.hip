// Implicit-GEMM convolution / linear for gfx950 (MFMA), NHWC.
//
// Replaces every dense nn.Conv2d(+BN)(+act) and nn.Linear on the DETRPose forward:
//   ConvBNAct (hgnetv2.py:82-134), ConvNormLayer(_fuse) (hybrid_encoder.py:56-128),
//   VGGBlock deploy conv (hybrid_encoder.py:139-189), the MHA in/out projections,
//   FFN / Gate / MSDA-projection / MLP-head linears (transformer.py, utils.py:75-87).
//
// GEMM view: C[M=batch*oh*ow][N=cout] = A[M][K] * W[N][K]^T, K = kh*kw*cin, A gathered
// on the fly from the NHWC input (zero for padding taps).  Both operands are K-major,
// which is the native operand layout of v_mfma_f32_16x16x32_bf16 (lane l holds 8
// consecutive k of row l&15), so global->LDS staging is straight 16-byte copies.
//
// Block: 256 threads = 4 waves in 2x2, tile BM x BN, K-step BK = 128 bytes of k per
// row (64 bf16 / 32 f32). Register-staged, double-buffered LDS (one barrier per
// K-step). Epilogue: bias (folded BN), activation, LAB, staged through LDS and written
// as 16-byte rows with the residual add (HG_Block identity, CSP x_1 + x_2) and an
// optional nearest-x2 copy (FPN upsample + concat, hybrid_encoder.py:495-496).
// Blocks are remapped so each XCD walks a contiguous range of tiles and the BN-tiles
// that share one A tile run on one XCD (L2 reuse of the gathered activations).
#include "common.h"

namespace {

template <typename T>
struct Geo {
  static constexpr int VEC = 16 / sizeof(T);    // elements per 16-byte chunk
  static constexpr int BK = 128 / sizeof(T);    // 8 chunks per row per K-step
  static constexpr int BKP = BK + VEC;          // LDS row pitch (+16 B pad)
};

template <typename T, typename TO, int BM, int BN>
struct Smem {
  static constexpr int AB = 2 * (BM + BN) * Geo<T>::BKP * (int)sizeof(T);   // double-buffered A|B
  static constexpr int CP = BN + Geo<TO>::VEC;                               // epilogue tile pitch
  static constexpr int C = BM * CP * (int)sizeof(TO);
  static constexpr int BYTES = AB > C ? AB : C;
};

template <typename T, typename TO, int BM, int BN, bool K1X1>
__global__ __launch_bounds__(256) void conv_gemm_kernel(dp_conv_desc d, int M, int nt_n, int vec_ok) {
  using G = Geo<T>;
  constexpr int VEC = G::VEC, BK = G::BK, BKP = G::BKP;
  constexpr int AR = BM / 32, BR = BN / 32;          // rows per thread per K-step
  constexpr int WM = BM / 2, WN = BN / 2;            // wave tile
  constexpr int TM = WM / 16, TN = WN / 16;          // 16x16 MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) char smem_raw[Smem<T, TO, BM, BN>::BYTES];
  T* As = reinterpret_cast<T*>(smem_raw);   // [2][BM][BKP]
  T* Bs = As + 2 * BM * BKP;                // [2][BN][BKP]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap of the 1-D grid (blocks b, b+8, ... share an XCD)
  const int nwg = gridDim.x, pid = blockIdx.x;
  const int xcd = pid & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (pid >> 3);
  const int tn = logical % nt_n, tm = logical / nt_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const T* __restrict__ in = reinterpret_cast<const T*>(d.in);
  const T* __restrict__ wt = reinterpret_cast<const T*>(d.weight);
  const int hwo = d.out_h * d.out_w;
  const int chunk = tid & 7;

  // per-thread A rows
  int64_t a_base[AR];
  int a_iy0[AR], a_ix0[AR];
  bool a_ok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    int m = m0 + (tid >> 3) + i * 32;
    a_ok[i] = m < M;
    int mm = a_ok[i] ? m : 0;
    int b = mm / hwo, rem = mm - b * hwo;
    int oy = rem / d.out_w, ox = rem - oy * d.out_w;
    a_iy0[i] = oy * d.stride - d.pad_t;
    a_ix0[i] = ox * d.stride - d.pad_l;
    a_base[i] = (int64_t)b * d.in_bstride;
    if (K1X1) a_base[i] += ((int64_t)a_iy0[i] * d.in_w + a_ix0[i]) * d.in_pstride;
  }
  const int ntap = d.kh * d.kw;

  Vec16<T> ra[AR], rb[BR];
  auto g2r = [&](int kt) {
    const int kk = kt * BK + chunk * VEC;
    if (K1X1) {
      const bool kv = kk < d.cin;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        if (a_ok[i] && kv) ra[i] = load16(in + a_base[i] + kk);
        else *reinterpret_cast<uint4*>(&ra[i].v) = make_uint4(0, 0, 0, 0);
      }
    } else {
      const int tap = kk / d.cin, ci = kk - tap * d.cin;
      const int ky = tap / d.kw, kx = tap - ky * d.kw;
      const bool kv = tap < ntap;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int iy = a_iy0[i] + ky, ix = a_ix0[i] + kx;
        const bool ok = a_ok[i] && kv && iy >= 0 && iy < d.in_h && ix >= 0 && ix < d.in_w;
        if (ok) ra[i] = load16(in + a_base[i] + ((int64_t)iy * d.in_w + ix) * d.in_pstride + ci);
        else *reinterpret_cast<uint4*>(&ra[i].v) = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < BR; ++j) {
      const int n = n0 + (tid >> 3) + j * 32;
      if (n < d.cout) rb[j] = load16(wt + (int64_t)n * d.kpad + kt * BK + chunk * VEC);
      else *reinterpret_cast<uint4*>(&rb[j].v) = make_uint4(0, 0, 0, 0);
    }
  };
  auto r2s = [&](int buf) {
    T* a = As + buf * BM * BKP;
    T* b = Bs + buf * BN * BKP;
#pragma unroll
    for (int i = 0; i < AR; ++i) store16(a + ((tid >> 3) + i * 32) * BKP + chunk * VEC, ra[i]);
#pragma unroll
    for (int j = 0; j < BR; ++j) store16(b + ((tid >> 3) + j * 32) * BKP + chunk * VEC, rb[j]);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = d.kpad / BK;
  g2r(0);
  r2s(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) g2r(kt + 1);
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
    if (kt + 1 < nk) r2s(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bias + act + LAB into an LDS tile, then 16-byte row writes
  constexpr int CP = Smem<T, TO, BM, BN>::CP;
  constexpr int VO = Geo<TO>::VEC;
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

template <typename T, typename TO, int BM, int BN>
int launch(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  const int M = d.batch * d.out_h * d.out_w;
  const int mt = (M + BM - 1) / BM, nt = (d.cout + BN - 1) / BN;
  const bool k1 = d.kh == 1 && d.kw == 1 && d.pad_t == 0 && d.pad_l == 0;
  dim3 grid(mt * nt), block(256);
  if constexpr (sizeof(TO) != sizeof(T)) {
    hipLaunchKernelGGL((conv_gemm_kernel<T, TO, BM, BN, true>), grid, block, 0, s, d, M, nt, vec_ok);
  } else {
    if (k1) hipLaunchKernelGGL((conv_gemm_kernel<T, TO, BM, BN, true>), grid, block, 0, s, d, M, nt, vec_ok);
    else hipLaunchKernelGGL((conv_gemm_kernel<T, TO, BM, BN, false>), grid, block, 0, s, d, M, nt, vec_ok);
  }
  return dp_check_launch("dp_conv2d");
}

template <typename T, typename TO>
int dispatch(const dp_conv_desc& d, hipStream_t s) {
  constexpr int VEC = Geo<TO>::VEC;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  int vec_ok = (d.out_pstride % VEC == 0) && (d.out_bstride % VEC == 0) && al(d.out);
  if (d.res) vec_ok = vec_ok && (d.res_pstride % VEC == 0) && (d.res_bstride % VEC == 0) && al(d.res);
  if (d.up) vec_ok = vec_ok && (d.up_pstride % VEC == 0) && (d.up_bstride % VEC == 0) && al(d.up);
  const int M = d.batch * d.out_h * d.out_w;
  if constexpr (sizeof(TO) != sizeof(T)) {  // f32-output heads: few shapes
    if (M <= 8192) return launch<T, TO, 64, 128>(d, s, vec_ok);
    return launch<T, TO, 128, 128>(d, s, vec_ok);
  } else {
    if (d.cout <= 32) return launch<T, TO, 128, 32>(d, s, vec_ok);
    if (d.cout <= 64) return launch<T, TO, 128, 64>(d, s, vec_ok);
    if (M <= 8192) return launch<T, TO, 64, 128>(d, s, vec_ok);
    return launch<T, TO, 128, 128>(d, s, vec_ok);
  }
}

}  // namespace

extern "C" int dp_conv2d(const dp_conv_desc* dp, void* stream) {
  DP_REQUIRE(dp != nullptr, "dp_conv2d: null descriptor");
  const dp_conv_desc& d = *dp;
  const int VEC = d.dtype == DP_BF16 ? 8 : 4;
  const int BK = d.dtype == DP_BF16 ? 64 : 32;
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
  DP_REQUIRE(!d.out_f32 || (d.kh == 1 && d.kw == 1 && d.pad_t == 0 && d.pad_l == 0 && !d.up),
             "dp_conv2d: out_f32 is supported for 1x1 / linear layers without upsample");
  hipStream_t s = as_stream(stream);
  if (d.dtype == DP_BF16) return d.out_f32 ? dispatch<bf16_t, float>(d, s) : dispatch<bf16_t, bf16_t>(d, s);
  return dispatch<float, float>(d, s);
}
