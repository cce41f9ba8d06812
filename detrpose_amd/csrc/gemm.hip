// General strided (batched) GEMM on MFMA for the training step: every nn.Linear forward,
// its input gradient (dgrad) and its weight gradient (wgrad) is one dp_gemm call with the
// right strides, so no operand is ever transposed in memory.
//
//   C(b, m, n) = epilogue( alpha * sum_k A(b, m, k) * B(b, k, n) )
//   A(b, m, k) = a[b*a_bs + m*a_rs + k*a_ks],  B(b, k, n) = b[b*b_bs + k*b_ks + n*b_ns],
//   C(b, m, n) = c[b*c_bs + m*c_rs + n].
//   Linear y = x W^T:  A = x (a_rs = ld, a_ks = 1), B(k, n) = W[n][k] (b_ks = 1, b_ns = K)
//   dgrad dx = dy W:   A = dy,                       B(k, n) = W[k][n] (b_ks = K, b_ns = 1)
//   wgrad dW = dy^T x: A(m, k) = dy[k][m] (a_rs = 1, a_ks = ld), B(k, n) = x[k][n]
//
// Tile: 64x64 outputs per 256-thread block (4 waves, 32x32 each = 2x2 MFMA 16x16 tiles), K step
// of 128 bytes per row (64 bf16 / 32 f32). A and B tiles are staged in LDS k-contiguous
// ([row][k], 16-byte padded rows) whatever their global layout: a k-contiguous operand loads
// 16-byte row chunks, an m/n-contiguous one loads 16-byte column chunks and scatters them,
// anything else loads elements. The next K step's global loads are issued into registers
// before the MFMAs of the current one (register double buffer, one LDS buffer per operand).
// bf16 inputs: mfma_f32_16x16x32_bf16; f32 inputs: mfma_f32_16x16x4f32 (exact f32 products).
// Split-K (when the M x N grid cannot fill the chip, e.g. wgrad over 10^5 rows): each block
// adds alpha * its partial product into f32 C with atomics (C pre-initialised by the caller).
#include "common.h"
#include <cmath>
#include "conv_lds.h"

extern "C" int dp_colsum(const void* x, int64_t ld, int32_t rows, int32_t n, float* out, int32_t accumulate,
                         int32_t dtype, void* stream);

namespace {

constexpr int TM = 64, TN = 64;

template <typename TI>
struct GemmTraits;
template <>
struct GemmTraits<bf16_t> {
  static constexpr int BK = 64, VEC = 8, PITCH = 72;   // 144-byte LDS rows
};
template <>
struct GemmTraits<float> {
  static constexpr int BK = 32, VEC = 4, PITCH = 36;   // 144-byte LDS rows
};

struct Operand {
  const void* p;
  int64_t bs, rs, ks;   // batch, row (m or n), k strides (elements)
  int rows;             // M or N
};

// global -> registers for one 64 x BK tile of an operand (row r, k), zero outside.
// mode 0: k contiguous (ks == 1): 2 x 16-byte chunks per thread of (row, k-chunk)
// mode 1: rows contiguous (rs == 1): 2 x 16-byte chunks per thread of (k, row-chunk)
// mode 2: generic: per-element loads
template <typename TI>
struct TileRegs {
  static constexpr int BK = GemmTraits<TI>::BK, VEC = GemmTraits<TI>::VEC;
  static constexpr int NE = TM * BK / 256;   // elements per thread (16 bf16 / 8 f32)
  TI v[NE];
};

template <typename TI>
__device__ __forceinline__ void load_tile(TileRegs<TI>& t, const Operand& op, int mode, int64_t base, int r0, int k0,
                                          int K) {
  constexpr int BK = GemmTraits<TI>::BK, VEC = GemmTraits<TI>::VEC;
  const TI* p = reinterpret_cast<const TI*>(op.p) + base;
  const int tid = threadIdx.x;
  // a tile wholly inside the operand (block-uniform test): both chunks load unguarded, back to
  // back (a per-lane guard makes a branch around each load, and the loads issue one at a time)
  const bool interior = mode < 2 && r0 + TM <= op.rows && k0 + BK <= K;
  if (interior && mode == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int r = c / (BK / VEC), kc = (c % (BK / VEC)) * VEC;
      *reinterpret_cast<uint4*>(&t.v[i * VEC]) = *reinterpret_cast<const uint4*>(p + (int64_t)(r0 + r) * op.rs + k0 + kc);
    }
  } else if (interior) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int kk = c / (TM / VEC), rc = (c % (TM / VEC)) * VEC;
      *reinterpret_cast<uint4*>(&t.v[i * VEC]) = *reinterpret_cast<const uint4*>(p + (int64_t)(k0 + kk) * op.ks + r0 + rc);
    }
  } else if (mode == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int r = c / (BK / VEC), kc = (c % (BK / VEC)) * VEC;
      const int gr = r0 + r, gk = k0 + kc;
      if (gr < op.rows && gk + VEC <= K) {
        *reinterpret_cast<uint4*>(&t.v[i * VEC]) = *reinterpret_cast<const uint4*>(p + (int64_t)gr * op.rs + gk);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          t.v[i * VEC + e] = (gr < op.rows && gk + e < K) ? p[(int64_t)gr * op.rs + gk + e] : (TI)0.f;
      }
    }
  } else if (mode == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int kk = c / (TM / VEC), rc = (c % (TM / VEC)) * VEC;
      const int gr = r0 + rc, gk = k0 + kk;
      if (gk < K && gr + VEC <= op.rows) {
        *reinterpret_cast<uint4*>(&t.v[i * VEC]) = *reinterpret_cast<const uint4*>(p + (int64_t)gk * op.ks + gr);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e)
          t.v[i * VEC + e] = (gk < K && gr + e < op.rows) ? p[(int64_t)gk * op.ks + gr + e] : (TI)0.f;
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < TileRegs<TI>::NE; ++e) {
      const int idx = tid + 256 * e;
      const int r = idx / BK, kk = idx % BK;
      const int gr = r0 + r, gk = k0 + kk;
      t.v[e] = (gr < op.rows && gk < K) ? p[(int64_t)gr * op.rs + (int64_t)gk * op.ks] : (TI)0.f;
    }
  }
}

template <typename TI>
__device__ __forceinline__ void store_tile(const TileRegs<TI>& t, TI* lds, int mode) {
  constexpr int BK = GemmTraits<TI>::BK, VEC = GemmTraits<TI>::VEC, PITCH = GemmTraits<TI>::PITCH;
  const int tid = threadIdx.x;
  if (mode == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int r = c / (BK / VEC), kc = (c % (BK / VEC)) * VEC;
      *reinterpret_cast<uint4*>(lds + r * PITCH + kc) = *reinterpret_cast<const uint4*>(&t.v[i * VEC]);
    }
  } else if (mode == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      const int kk = c / (TM / VEC), rc = (c % (TM / VEC)) * VEC;
#pragma unroll
      for (int e = 0; e < VEC; ++e) lds[(rc + e) * PITCH + kk] = t.v[i * VEC + e];
    }
  } else {
#pragma unroll
    for (int e = 0; e < TileRegs<TI>::NE; ++e) {
      const int idx = tid + 256 * e;
      lds[(idx / BK) * PITCH + idx % BK] = t.v[e];
    }
  }
}

struct GemmArgs {
  Operand A, B;
  float* cf;
  bf16_t* cb;
  int64_t c_bs, c_rs;
  int M, N, K, batch, splits, kchunk;
  const float* bias;
  float alpha, beta;
  int act;
  const void* gate;
  int64_t g_bs, g_rs;
  int gate_bf16;
  int modeA, modeB;
  int tiles_n;
  float* colsum;   // wgrad_tt_kernel: colsum[m] += alpha * sum_k A(m, k) (bias gradient), or NULL
  // B operand mode 3 (dp_conv_wgrad): B(k = output pixel p, n = tap * cin + ci) = x at the
  // tap's input pixel of p (zero outside the map) -- im2col on the fly
  const bf16_t* ix;
  int64_t ix_bs;
  int ix_ps, ih, iw, icin, ioh, iow, ikw, istride, ipad;
};

template <typename TI>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs g) {
  constexpr int BK = GemmTraits<TI>::BK, PITCH = GemmTraits<TI>::PITCH;
  __shared__ __attribute__((aligned(16))) TI As[TM * PITCH];
  __shared__ __attribute__((aligned(16))) TI Bs[TN * PITCH];
  const int tile = blockIdx.x;
  const int tm = tile / g.tiles_n, tn = tile - tm * g.tiles_n;
  const int zb = blockIdx.y;
  const int bidx = zb / g.splits, split = zb - bidx * g.splits;
  const int m0 = tm * TM, n0 = tn * TN;
  const int kb = split * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  const int64_t abase = (int64_t)bidx * g.A.bs, bbase = (int64_t)bidx * g.B.bs;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  TileRegs<TI> ra, rb;
  // k is measured from kb inside the chunk (the operand base absorbs kb)
  Operand A = g.A, B = g.B;
  const int64_t aoff = abase + (int64_t)kb * A.ks, boff = bbase + (int64_t)kb * B.ks;
  const int KC = ke - kb;
  if (KC > 0) {
    load_tile<TI>(ra, A, g.modeA, aoff, m0, 0, KC);
    load_tile<TI>(rb, B, g.modeB, boff, n0, 0, KC);
  }
  for (int k0 = 0; k0 < KC; k0 += BK) {
    __syncthreads();
    store_tile<TI>(ra, As, g.modeA);
    store_tile<TI>(rb, Bs, g.modeB);
    __syncthreads();
    if (k0 + BK < KC) {
      load_tile<TI>(ra, A, g.modeA, aoff, m0, k0 + BK, KC);
      load_tile<TI>(rb, B, g.modeB, boff, n0, k0 + BK, KC);
    }
    if constexpr (sizeof(TI) == 2) {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        const int ko = ks * 32 + (lane >> 4) * 8;
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As + (wm + 16 * i + (lane & 15)) * PITCH + ko);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn + 16 * j + (lane & 15)) * PITCH + ko);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        const int ko = ks * 4 + (lane >> 4);
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = As[(wm + 16 * i + (lane & 15)) * PITCH + ko];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = Bs[(wn + 16 * j + (lane & 15)) * PITCH + ko];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  // epilogue: lane holds C[row = 4 (lane >> 4) + r][col = lane & 15] of each 16x16 tile
  const int64_t cb = (int64_t)bidx * g.c_bs;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 16 * j + (lane & 15);
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        if (m >= g.M) continue;
        const int64_t o = cb + (int64_t)m * g.c_rs + n;
        float v = g.alpha * acc[i][j][r];
        if (g.splits > 1) {
          unsafeAtomicAdd(g.cf + o, v);
          continue;
        }
        if (g.bias) v += g.bias[n];
        if (g.beta != 0.f) v += g.beta * (g.cf ? g.cf[o] : (float)g.cb[o]);
        if (g.act == DP_ACT_RELU) v = fmaxf(v, 0.f);
        else if (g.act == DP_ACT_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        if (g.gate) {
          const int64_t go = (int64_t)bidx * g.g_bs + (int64_t)m * g.g_rs + n;
          const float gv = g.gate_bf16 ? (float)reinterpret_cast<const bf16_t*>(g.gate)[go]
                                       : reinterpret_cast<const float*>(g.gate)[go];
          if (!(gv > 0.f)) v = 0.f;
        }
        if (g.cf) g.cf[o] = v;
        else g.cb[o] = (bf16_t)v;
      }
    }
}

// ---------------------------------------------------------------- 128x128 bf16 tiles
// The large-shape bf16 path (every decoder / AIFI Linear of the training step at batch 16:
// M = rows of 10^4-10^5, N and K of 256-1024, and their split-K weight gradients): 128 x 128
// outputs per 256-thread block, 4 waves of 64 x 64 (4 x 4 MFMA 16x16x32 tiles), K steps of 64,
// LDS double-buffered (one barrier per K step; the next step's global loads are in registers
// while the current step's 32 MFMAs run). Operand images in LDS:
//   k-contiguous operand (mode 0): [128 rows][72] (144-byte rows, 16-byte stores, b128
//     fragment reads), as the 64 x 64 kernel;
//   row-contiguous operand (mode 1: the transposed operand of dgrad / wgrad): [64 k][128 rows]
//     in 256-byte rows with the 16-byte chunk XOR swizzle of cdna_hip_programming.md T10 (b),
//     written with 16-byte stores and read back with ds_read_b64_tr_b16 (two 4-k reads per
//     fragment: lane group g takes k = 8g .. 8g+7, the same k slots as the b128 reads).
constexpr int BT = 128, BKB = 64, P0 = 72;
// Two waves per SIMD (the LDS allows two blocks per CU): holds every instantiation at <= 256
// VGPRs (the both-transposed <1, 1> had 272, i.e. one block per CU). DP_GEMM128_WPE=0: no bound (A/B)
#ifndef DP_GEMM128_WPE
#define DP_GEMM128_WPE 2
#endif
#if DP_GEMM128_WPE
#define DP_G128_ATTR __attribute__((amdgpu_waves_per_eu(DP_GEMM128_WPE)))
#else
#define DP_G128_ATTR
#endif
constexpr int IMG = BT * P0 > BKB * BT ? BT * P0 : BKB * BT;   // elements per operand image

__device__ __forceinline__ int swz_off(int r, int ch) {   // bytes of chunk ch of k-row r
  return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

struct Tile2Regs {
  uint4 v[4];
};

__device__ __forceinline__ void load_tile2(Tile2Regs& t, const Operand& op, int mode, int64_t base, int r0, int k0,
                                           int K) {
  const bf16_t* p = reinterpret_cast<const bf16_t*>(op.p) + base;
  const int tid = threadIdx.x;
  if (r0 + BT <= op.rows && k0 + BKB <= K) {   // interior tile (block-uniform): unguarded loads
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      t.v[i] = mode == 0 ? *reinterpret_cast<const uint4*>(p + (int64_t)(r0 + (c >> 3)) * op.rs + k0 + (c & 7) * 8)
                         : *reinterpret_cast<const uint4*>(p + (int64_t)(k0 + (c >> 4)) * op.ks + r0 + (c & 15) * 8);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    int gr, gk;
    if (mode == 0) {
      gr = r0 + (c >> 3);
      gk = k0 + (c & 7) * 8;
      if (gr < op.rows && gk + 8 <= K) {
        t.v[i] = *reinterpret_cast<const uint4*>(p + (int64_t)gr * op.rs + gk);
      } else {
        bf16_t e8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) e8[e] = (gr < op.rows && gk + e < K) ? p[(int64_t)gr * op.rs + gk + e] : (bf16_t)0.f;
        t.v[i] = *reinterpret_cast<const uint4*>(e8);
      }
    } else {
      gk = k0 + (c >> 4);
      gr = r0 + (c & 15) * 8;
      if (gk < K && gr + 8 <= op.rows) {
        t.v[i] = *reinterpret_cast<const uint4*>(p + (int64_t)gk * op.ks + gr);
      } else if (gk >= K || gr >= op.rows) {   // wholly outside (e.g. rows past a 48-channel cout)
        t.v[i] = uint4{0u, 0u, 0u, 0u};
      } else {
        bf16_t e8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) e8[e] = (gk < K && gr + e < op.rows) ? p[(int64_t)gk * op.ks + gr + e] : (bf16_t)0.f;
        t.v[i] = *reinterpret_cast<const uint4*>(e8);
      }
    }
  }
}

// B tile of mode 3: k rows kabs .. kabs+63 (output pixels), n columns n0 .. n0+127 (tap-major:
// n = tap * cin + ci; cin % 8 == 0 so a 16-byte chunk is 8 channels of one tap). Every load is
// issued (address clamped into the map), the chunk zeroed where the tap falls outside it.
// A thread's four chunks share one column n (c & 15 == tid & 15), so its tap / channel split is
// computed once per block (ImLane); the pixel index is split by float reciprocals with a
// one-step correction (exact for K < 2^24, host check) instead of runtime integer divisions,
// which had made the gather VALU-bound (six divisions per chunk against 32 MFMAs per wave).
struct ImLane {
  int dy, dx, cic;   // tap offsets (ky - pad, kx - pad) and channel of this thread's column
  bool nok;          // column inside N
  float inv_w, inv_h;
};

__device__ __forceinline__ int fdivi(int a, int d, float inv) {   // a / d for 0 <= a < 2^24
  int q = (int)((float)a * inv);
  const int r = a - q * d;
  q += r >= d ? 1 : 0;
  q -= r < 0 ? 1 : 0;
  return q;
}

__device__ __forceinline__ ImLane im_lane(const GemmArgs& g, int n0) {
  ImLane L;
  const int n = n0 + (threadIdx.x & 15) * 8;
  L.nok = n < g.N;
  const int nn = L.nok ? n : 0;
  const int tap = nn / g.icin, ky = tap / g.ikw;
  L.cic = nn - tap * g.icin;
  L.dy = ky - g.ipad;
  L.dx = tap - ky * g.ikw - g.ipad;
  L.inv_w = 1.f / (float)g.iow;
  L.inv_h = 1.f / (float)g.ioh;
  return L;
}

__device__ __forceinline__ void load_tile_im(Tile2Regs& t, const GemmArgs& g, int kabs, int kend, const ImLane& L) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = kabs + (tid >> 4) + 16 * i;
    const int pc = min(p, kend - 1);
    const int t2 = fdivi(pc, g.iow, L.inv_w), ox = pc - t2 * g.iow;
    const int b = fdivi(t2, g.ioh, L.inv_h), oy = t2 - b * g.ioh;
    const int y = oy * g.istride + L.dy, x = ox * g.istride + L.dx;
    const bool ok = p < kend && L.nok && (unsigned)y < (unsigned)g.ih && (unsigned)x < (unsigned)g.iw;
    const int yc = min(max(y, 0), g.ih - 1), xc = min(max(x, 0), g.iw - 1);
    const uint4 v = *reinterpret_cast<const uint4*>(g.ix + (int64_t)b * g.ix_bs + ((int64_t)yc * g.iw + xc) * g.ix_ps + L.cic);
    t.v[i] = ok ? v : uint4{0u, 0u, 0u, 0u};
  }
}

__device__ __forceinline__ void store_tile2(const Tile2Regs& t, bf16_t* img, int mode) {
  const int tid = threadIdx.x;
  char* b = reinterpret_cast<char*>(img);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if (mode == 0) *reinterpret_cast<uint4*>(img + (c >> 3) * P0 + (c & 7) * 8) = t.v[i];
    else *reinterpret_cast<uint4*>(b + swz_off(c >> 4, c & 15)) = t.v[i];
  }
}

// the 16x16x32 operand fragment of rows r0 .. r0+15 at k = kb + 8 (lane >> 4) .. +7
__device__ __forceinline__ bf16x8 frag2(const bf16_t* img, int mode, int r0, int kb) {
  const int lane = threadIdx.x & 63;
  if (mode == 0) return *reinterpret_cast<const bf16x8*>(img + (r0 + (lane & 15)) * P0 + kb + 8 * (lane >> 4));
  typedef short s4 __attribute__((ext_vector_type(4)));
  const int q = (lane & 15) >> 2, pp = lane & 3, g = lane >> 4;
  const char* b = reinterpret_cast<const char*>(img);
  const int ch = (r0 >> 3) + (pp >> 1);
  const int k0 = kb + 8 * g + q;
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(b + swz_off(k0, ch) + 8 * (pp & 1)));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(b + swz_off(k0 + 4, ch) + 8 * (pp & 1)));
  short t8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return *reinterpret_cast<const bf16x8*>(t8);
}

// MA / MB: the operands' modes as compile-time constants (no branch in the fragment reads)
template <int MA, int MB>
__global__ __launch_bounds__(256) DP_G128_ATTR void gemm128_kernel(const GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem128[];   // [buffer][A | B][IMG]
  bf16_t(*sm)[2][IMG] = reinterpret_cast<bf16_t(*)[2][IMG]>(smem128);
  const int tile = blockIdx.x;
  const int tm = tile / g.tiles_n, tn = tile - tm * g.tiles_n;
  const int zb = blockIdx.y;
  const int bidx = zb / g.splits, split = zb - bidx * g.splits;
  const int m0 = tm * BT, n0 = tn * BT;
  const int kb = split * g.kchunk;
  const int ke = min(g.K, kb + g.kchunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const Operand A = g.A, B = g.B;
  const int64_t aoff = (int64_t)bidx * A.bs + (int64_t)kb * A.ks, boff = (int64_t)bidx * B.bs + (int64_t)kb * B.ks;
  const int KC = ke - kb;
  ImLane il{};
  if constexpr (MB == 3) il = im_lane(g, n0);
  auto load_step = [&](Tile2Regs& ra, Tile2Regs& rb, int k0) __attribute__((always_inline)) {
    load_tile2(ra, A, MA, aoff, m0, k0, KC);
    if constexpr (MB == 3) load_tile_im(rb, g, kb + k0, ke, il);
    else load_tile2(rb, B, MB, boff, n0, k0, KC);
  };
  auto store_step = [&](const Tile2Regs& ra, const Tile2Regs& rb, int buf) __attribute__((always_inline)) {
    store_tile2(ra, sm[buf][0], MA);
    store_tile2(rb, sm[buf][1], MB == 3 ? 1 : MB);
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    const bf16_t* Ai = sm[buf][0];
    const bf16_t* Bi = sm[buf][1];
#pragma unroll
    for (int ks = 0; ks < BKB / 32; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag2(Ai, MA, wm + 16 * i, 32 * ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag2(Bi, MB == 3 ? 1 : MB, wn + 16 * j, 32 * ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nst = (KC + BKB - 1) / BKB;   // K steps of this split
  Tile2Regs ra, rb;
  if (nst > 0) {
    load_step(ra, rb, 0);
    store_step(ra, rb, 0);
  }
  __syncthreads();
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    const bool more = st + 1 < nst;
    if (more) load_step(ra, rb, (st + 1) * BKB);
    compute(cur);
    if (more) store_step(ra, rb, cur ^ 1);   // the other buffer's readers passed the last barrier
    __syncthreads();
    cur ^= 1;
  }
  const int64_t cbo = (int64_t)bidx * g.c_bs;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + 16 * j + (lane & 15);
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        if (m >= g.M) continue;
        const int64_t o = cbo + (int64_t)m * g.c_rs + n;
        float v = g.alpha * acc[i][j][r];
        if (g.splits > 1) {
          unsafeAtomicAdd(g.cf + o, v);
          continue;
        }
        if (g.bias) v += g.bias[n];
        if (g.beta != 0.f) v += g.beta * (g.cf ? g.cf[o] : (float)g.cb[o]);
        if (g.act == DP_ACT_RELU) v = fmaxf(v, 0.f);
        else if (g.act == DP_ACT_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        if (g.gate) {
          const int64_t go = (int64_t)bidx * g.g_bs + (int64_t)m * g.g_rs + n;
          const float gv = g.gate_bf16 ? (float)reinterpret_cast<const bf16_t*>(g.gate)[go]
                                       : reinterpret_cast<const float*>(g.gate)[go];
          if (!(gv > 0.f)) v = 0.f;
        }
        if (g.cf) g.cf[o] = v;
        else g.cb[o] = (bf16_t)v;
      }
    }
}

int operand_mode(const Operand& op, int vec, int64_t align_bytes_ok) {
  if (op.ks == 1 && op.rs % vec == 0 && align_bytes_ok) return 0;
  if (op.rs == 1 && op.ks % vec == 0 && align_bytes_ok) return 1;
  return 2;
}


// ---------------------------------------------------------------- weight-gradient GEMM on an LDS-DMA ring
// C[m][n] += alpha * sum_k A[k][m] B[k][n] with both operands row-contiguous in k-major rows
// (mode 1 / 1: dW = dy^T x of every 1x1 conv and Linear, dy [P][M], x [P][N], P = pixels or
// tokens of 10^4 - 10^6), bf16 in, f32 C accumulated with float atomics over K splits. The
// register-staged 128 x 128 kernel above reaches 6-20 % of MFMA peak here: its one K-step of
// register prefetch cannot cover the HBM latency of a K-major stream. Here 128 x 256 tiles of
// 8 waves (64 x 64 each) stream through a 3-deep LDS ring filled by buffer_load ... lds (no
// staging registers; conv_lds.h): each 16-byte DMA lane fetches the global chunk that belongs
// at its LDS slot under the [64 k][128 col] XOR swizzle of swz_off, so the ds_read_b64_tr_b16
// fragment reads of frag2 apply unchanged. One block per CU (144 KB of LDS); the block order
// is XCD-sliced so the tiles of one K split (which read the same rows of A and B) share an L2.
constexpr int WT_BM = 128, WT_BN = 256, WT_NS = 3;
constexpr int WT_SUB = 64 * 256;               // bytes of one [64 k][128 col] sub-image
constexpr int WT_STAGE = 3 * WT_SUB;           // A | B cols 0-127 | B cols 128-255
constexpr int WT_DMA = 6;                      // DMA instructions per wave per K-step (2 A + 4 B)

// IM: B is dp_conv_wgrad's implicit im2col (mode 3: B(k = output pixel p, n = tap * cin + ci) =
// x at the tap's input pixel of p, zero outside the map): each B DMA lane gathers the 16-byte
// chunk of 8 channels of its column's tap at its row's pixel (an out-of-map pixel is an OOB
// offset: zeros).
template <bool IM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
void wgrad_tt_kernel(const GemmArgs g, int ntiles, int tiles_n) {
  using namespace dpconv;
  extern __shared__ __attribute__((aligned(1024))) char smw[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;                       // multiple of 8
  const int Lb = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int tile = Lb % ntiles, split = Lb / ntiles;
  if (split >= g.splits) return;
  const int kb = split * g.kchunk;
  const int nst = (min(g.K, kb + g.kchunk) - kb + 63) / 64;
  if (nst <= 0) return;
  const int krem = min(g.K, kb + g.kchunk) - kb;   // rows of this split
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * WT_BM, n0 = tn * WT_BN;
  const bf16_t* pa = reinterpret_cast<const bf16_t*>(g.A.p) + (int64_t)kb * g.A.ks;
  const bf16_t* pb = IM ? g.ix : reinterpret_cast<const bf16_t*>(g.B.p) + (int64_t)kb * g.B.ks;
  const i32x4 ra = make_rsrc(pa), rb = make_rsrc(pb);
  // this wave's DMA instructions: t = 0, 1 -> A k-row groups 4 (2 wave + t); t = 2 .. 5 -> B
  // instruction q = 4 wave + t - 2: sub-image q / 16, k-row group 4 (q % 16). Lane: row kr + rr,
  // LDS slot s = lane % 16 holding logical chunk s ^ swizzle(row).
  const int rr = lane >> 4, sl = lane & 15;
  int row[WT_DMA], colb[WT_DMA], ldso[WT_DMA];
  bool cok[WT_DMA];
  int tdy[WT_DMA], tdx[WT_DMA];   // IM: the B column's tap offsets (colb: its channel, bytes)
#pragma unroll
  for (int t = 0; t < WT_DMA; ++t) {
    int sub, kr;
    if (t < 2) {
      sub = 0, kr = 4 * (2 * wave + t);
    } else {
      const int q = 4 * wave + t - 2;
      sub = 1 + q / 16, kr = 4 * (q % 16);
    }
    const int r = kr + rr;
    const int ch = sl ^ (((r & 3) << 2) | ((r >> 2) & 3));
    const int col = (sub == 0 ? m0 : n0 + 128 * (sub - 1)) + 8 * ch;
    row[t] = r;
    colb[t] = col * 2;
    cok[t] = col < (sub == 0 ? g.M : g.N);
    ldso[t] = sub * WT_SUB + kr * 256;
    tdy[t] = tdx[t] = 0;
    if (IM && sub > 0) {
      const int nn = cok[t] ? col : 0;
      const int tap = nn / g.icin, ky = tap / g.ikw;
      colb[t] = (nn - tap * g.icin) * 2;
      tdy[t] = ky - g.ipad;
      tdx[t] = tap - ky * g.ikw - g.ipad;
    }
  }
  const float inv_w = 1.f / (float)g.iow, inv_h = 1.f / (float)g.ioh;
  const int64_t a_step = (int64_t)g.A.ks * 2, b_step = (int64_t)g.B.ks * 2;   // bytes per k row
  auto issue = [&](int st) {
    char* base = smw + (st % WT_NS) * WT_STAGE;
#pragma unroll
    for (int t = 0; t < WT_DMA; ++t) {
      const int k = st * 64 + row[t];
      bool ok = cok[t] && k < krem;
      int o;
      if (IM && t >= 2) {
        // output pixel p -> (image, oy, ox) -> the tap's input pixel (p < 2^24: fdivi exact)
        const int pp = min(kb + k, g.K - 1);
        const int t2 = fdivi(pp, g.iow, inv_w), ox = pp - t2 * g.iow;
        const int b = fdivi(t2, g.ioh, inv_h), oy = t2 - b * g.ioh;
        const int y = oy * g.istride + tdy[t], x = ox * g.istride + tdx[t];
        ok = ok && (unsigned)y < (unsigned)g.ih && (unsigned)x < (unsigned)g.iw;
        o = ok ? (int)((b * g.ix_bs + (int64_t)(y * g.iw + x) * g.ix_ps) * 2) + colb[t] : OOB;
      } else {
        o = ok ? (int)(k * (t < 2 ? a_step : b_step)) + colb[t] : OOB;
      }
      dma16(t < 2 ? ra : rb, base + ldso[t], o);
    }
  };
  const int wm = (wave >> 2) * 64, wn = (wave & 3) * 64;
  const int bsub = 1 + (wn >> 7), bcol = wn & 127;
  // the bias gradient (A's column sums over k) from the A fragments this wave reads anyway: the
  // waves of the first N-tile column (wn == 0) of the tiles at n0 == 0, each over its 64 rows
  const bool csum = !IM && g.colsum != nullptr && tn == 0 && (wave & 3) == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < WT_NS - 1; ++p)
    if (p < nst) issue(p);
  for (int st = 0; st < nst; ++st) {
    // stage st landed: the younger stages in flight are st+1 .. st+NS-2 (each WT_DMA per wave)
    if (st + WT_NS - 2 < nst) wait_vmcnt<(WT_NS - 2) * WT_DMA>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // the slot of st + NS - 1 held st - 1, which every wave is past (barrier)
    if (st + WT_NS - 1 < nst) issue(st + WT_NS - 1);
    const char* base = smw + (st % WT_NS) * WT_STAGE;
    const bf16_t* Ai = reinterpret_cast<const bf16_t*>(base);
    const bf16_t* Bi = reinterpret_cast<const bf16_t*>(base + bsub * WT_SUB);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag2(Ai, 1, wm + 16 * i, 32 * ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag2(Bi, 1, bcol + 16 * j, 32 * ks);
      if (csum) {   // lane: row m = wm + 16 i + lane % 16, k = 32 ks + 8 (lane / 16) .. + 7
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[i] += (float)af[i][e];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + 16 * j + (lane & 15);
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        if (m < g.M) unsafeAtomicAdd(g.cf + (int64_t)m * g.c_rs + n, g.alpha * acc[i][j][r]);
      }
    }
  if (csum) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = cs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int m = m0 + wm + 16 * i + (lane & 15);
      if (lane < 16 && m < g.M) unsafeAtomicAdd(g.colsum + m, g.alpha * v);
    }
  }
}

// K splits of the weight-gradient kernel: each split adds a 128 x 256 f32 tile with float atomics
// (131 KB, ~0.1 us of the chip's ~1.3 TB/s atomic rate per split and tile), each K-step costs a
// block ~0.9 us, so a launch takes about ks64 / sp * 0.9 + ntl * sp * 0.1 us: sp ~ sqrt(8.6 ks64 /
// ntl), at most one round of blocks (one per CU) and at least 4 K-steps per split. (One block per
// CU regardless measured 27 us a call on the decoder's 256 x 256 weight gradients over 13824 rows,
// 2 K-steps a block behind 33 MB of atomics.)
inline int wgrad_tt_splits(int ntl, int ks64) {
  int sp = (int)std::lround(std::sqrt(8.6 * ks64 / (double)ntl));
  const int cap = (dpconv::num_cus() + ntl - 1) / ntl;
  if (sp > cap) sp = cap;
  if (sp > ks64 / 4) sp = ks64 / 4;
  return sp < 1 ? 1 : sp;
}

// dw[co][ci][tap] += s[co][tap][ci] (the reference's [cout][cin][kh][kw] from the tap-major sums);
// CLEAR: each scratch element (read exactly once) is set back to zero, so the next call on this
// scratch needs no zero-fill launch (dp_conv_wgrad_zs)
template <bool CLEAR>
__global__ void wgrad_permute_kernel(float* __restrict__ s, float* __restrict__ dw, int cout, int cin, int taps) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over dw
  const int64_t total = (int64_t)cout * cin * taps;
  if (e >= total) return;
  const int tap = (int)(e % taps);
  const int64_t r = e / taps;
  const int ci = (int)(r % cin), co = (int)(r / cin);
  float* sp = s + ((int64_t)co * taps + tap) * cin + ci;
  dw[e] += *sp;
  if (CLEAR) *sp = 0.f;
}

// C[m][n] = beta C[m][n] + bias[n] (beta 0: C is not read) over an M x N f32 block of row
// stride c_rs: the start value of a split-K GEMM whose partial products then add with atomics
__global__ void gemm_init_c_kernel(float* __restrict__ c, int64_t c_rs, int m, int n, float beta,
                                   const float* __restrict__ bias) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)m * n) return;
  const int r = (int)(e / n), col = (int)(e - (int64_t)r * n);
  float* p = c + (int64_t)r * c_rs + col;
  const float b = bias ? bias[col] : 0.f;
  *p = beta != 0.f ? beta * *p + b : b;
}

}  // namespace

extern "C" int dp_gemm(const dp_gemm_desc* dp, void* stream) {
  DP_REQUIRE(dp != nullptr, "dp_gemm: null descriptor");
  const dp_gemm_desc& d = *dp;
  DP_REQUIRE(d.a && d.b && d.c, "dp_gemm: null operand");
  DP_REQUIRE(d.m > 0 && d.n > 0 && d.k > 0 && d.batch > 0, "dp_gemm: bad sizes m=%d n=%d k=%d batch=%d", d.m, d.n,
             d.k, d.batch);
  DP_REQUIRE(d.in_dtype == DP_BF16 || d.in_dtype == DP_F32, "dp_gemm: bad input dtype %d", d.in_dtype);
  DP_REQUIRE(d.out_dtype == DP_BF16 || d.out_dtype == DP_F32, "dp_gemm: bad output dtype %d", d.out_dtype);
  DP_REQUIRE(d.act == DP_ACT_NONE || d.act == DP_ACT_RELU || d.act == DP_ACT_GELU, "dp_gemm: act %d (none / relu / gelu)",
             d.act);
  DP_REQUIRE(d.split_k >= 0, "dp_gemm: split_k %d", d.split_k);
  DP_REQUIRE(!d.colsum || (d.batch == 1 && d.alpha == 1.f && d.a_rs == 1 && d.a_ks >= d.m),
             "dp_gemm: colsum needs batch 1, alpha 1 and A(m, k) = a[k * a_ks + m]");
  const int es = d.in_dtype == DP_BF16 ? 2 : 4;
  const int vec = 16 / es;
  const int BK = d.in_dtype == DP_BF16 ? 64 : 32;
  GemmArgs g{};
  g.A = Operand{d.a, d.a_bs, d.a_rs, d.a_ks, d.m};
  g.B = Operand{d.b, d.b_bs, d.b_ns, d.b_ks, d.n};
  const bool aal = (reinterpret_cast<uintptr_t>(d.a) & 15) == 0 && d.a_bs % vec == 0;
  const bool bal = (reinterpret_cast<uintptr_t>(d.b) & 15) == 0 && d.b_bs % vec == 0;
  g.modeA = operand_mode(g.A, vec, aal);
  g.modeB = operand_mode(g.B, vec, bal);
  g.cf = d.out_dtype == DP_F32 ? reinterpret_cast<float*>(d.c) : nullptr;
  g.cb = d.out_dtype == DP_BF16 ? reinterpret_cast<bf16_t*>(d.c) : nullptr;
  g.c_bs = d.c_bs;
  g.c_rs = d.c_rs;
  g.M = d.m, g.N = d.n, g.K = d.k, g.batch = d.batch;
  g.bias = d.bias;
  g.alpha = d.alpha;
  g.beta = d.beta;
  g.act = d.act;
  g.gate = d.gate;
  g.g_bs = d.gate_bs;
  g.g_rs = d.gate_rs;
  g.gate_bf16 = d.gate_dtype == DP_BF16;
  // 128 x 128 tiles for large bf16 shapes whose operands load as 16-byte rows or columns
  // (DETRPOSE_GEMM64=1: the 64 x 64 kernel everywhere, for A/B)
  static const bool force64 = getenv("DETRPOSE_GEMM64") != nullptr;
  const bool splittable = d.out_dtype == DP_F32 && !d.bias && d.act == DP_ACT_NONE && !d.gate && d.beta == 1.f &&
                          d.k >= 8 * 64;
  const bool big = !force64 && d.in_dtype == DP_BF16 && g.modeA < 2 && g.modeB < 2 && d.m >= 128 && d.n >= 96 &&
                   ((int64_t)d.m * d.n >= (int64_t)128 * 128 * 64 || (splittable && d.split_k == 0));
  // weight gradients (both operands k-major rows, f32 C accumulated): the LDS-DMA ring kernel
  // (DETRPOSE_WGRAD_TT=0 keeps the 128 x 128 kernel, A/B)
  static const bool tt_off = getenv("DETRPOSE_WGRAD_TT") && atoi(getenv("DETRPOSE_WGRAD_TT")) == 0;
  // (mode 1 rows are 16-byte aligned with ld % 8 == 0, so a 16-byte chunk never straddles two k
  // rows: a chunk past M / N reads the row's padding, which feeds only discarded C rows / columns)
  g.colsum = nullptr;
  if (!tt_off && !force64 && d.in_dtype == DP_BF16 && splittable && d.split_k == 0 && d.batch == 1 && g.modeA == 1 &&
      g.modeB == 1 && d.k >= 2048) {
    const int tmw = (d.m + WT_BM - 1) / WT_BM, tnw = (d.n + WT_BN - 1) / WT_BN;
    const int ntl = tmw * tnw;
    const int ksteps64 = (d.k + 63) / 64;
    const int sp = wgrad_tt_splits(ntl, ksteps64);
    const int kchunk = ((ksteps64 + sp - 1) / sp) * 64;
    // 32-bit buffer offsets from each split's first row
    if (((int64_t)kchunk * d.a_ks + d.m) * 2 < 0x7ff00000ll && ((int64_t)kchunk * d.b_ks + d.n) * 2 < 0x7ff00000ll) {
      g.splits = sp;
      g.kchunk = kchunk;
      g.colsum = d.colsum;
      static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_tt_kernel<false>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   WT_NS * WT_STAGE) == hipSuccess;
      DP_REQUIRE(attr, "dp_gemm: cannot set the weight-gradient kernel's LDS size");
      const int nb = (ntl * sp + 7) / 8 * 8;
      hipLaunchKernelGGL(wgrad_tt_kernel<false>, dim3((unsigned)nb), dim3(512), WT_NS * WT_STAGE, as_stream(stream), g,
                         ntl, tnw);
      return dp_check_launch("dp_gemm(wgrad)");
    }
  }
  const int TMs = big ? BT : TM, TNs = big ? BT : TN;
  const int tm = (d.m + TMs - 1) / TMs, tn = (d.n + TNs - 1) / TNs;
  g.tiles_n = tn;
  // split-K when the output grid cannot fill the chip and K is long (f32 C, plain epilogue)
  int splits = 1;
  const int ksteps = (d.k + BK - 1) / BK;
  const int64_t tiles = (int64_t)tm * tn * d.batch;
  if (d.split_k > 0) {
    splits = d.split_k;
  } else if (tiles < 512 && ksteps >= 8 && d.out_dtype == DP_F32 && !d.bias && d.act == DP_ACT_NONE && !d.gate &&
             d.beta == 1.f) {
    // 128 x 128 tiles: ~512 blocks (more splits only add atomics); 64 x 64 tiles (small M, the
    // stage-0/1 convs' weight gradients): ~4096 blocks, measured 535 -> 400 us (M 48, K 409600)
    // and 463 -> 312 us (M 96, K 102400) over the 512 target (scripts/gemm_bench.py)
    // A split runs at least kmin K-steps (4 on 128 x 128 tiles, 8 on 64 x 64), except for small
    // outputs (M N <= 512 x 512: the transformer heads' class / pose / LQE weight gradients), where
    // each split's float atomics are few and a block's time is its K-steps' load latency: 1 there
    // (the class-head dW, 2 x 256 over 768 rows: 45 -> 15 us; profiles/r6u_train_ops_all.json vs
    // r6x_train_ops_all.json. A 4-deep register ring of K-step loads instead measured slower on
    // the small forward GEMMs: 284 VGPRs, one wave per SIMD)
    const bool small_out = (int64_t)d.m * d.n <= 512 * 512;
    const int target = big ? 512 : 4096, kmin = big ? 4 : small_out ? 1 : 8;
    splits = (int)((target + tiles - 1) / tiles);
    if (splits > ksteps / kmin) splits = ksteps / kmin;
    // bounded float-atomic adds per output address: 512 for a one-tile output (stem1's 32 x 27
    // weight gradient over 1.6 M pixels had 3200 splits: 0.245 -> 0.177 ms; 256 measured 0.295),
    // 256 otherwise (the encoder / aggregation weight gradients: -0.14 ms per b16 sub-batch);
    // profiles/r5_gemm_split_cap_ab.txt. DETRPOSE_GEMM_SPLIT_CAP overrides (A/B, 0 = none)
    static const int cap_env = getenv("DETRPOSE_GEMM_SPLIT_CAP") ? atoi(getenv("DETRPOSE_GEMM_SPLIT_CAP")) : -1;
    const int cap = cap_env >= 0 ? cap_env : (tiles > 1 ? 256 : 512);
    if (cap > 0 && splits > cap) splits = cap;
    if (splits < 1) splits = 1;
  }
  // small f32 outputs with beta != 1 and no bias (the heads' input gradients: a few blocks of 4-8
  // K-steps, each step a full load latency): C starts as beta C in one launch, then the K splits
  // add into it as above. Not for a GEMM with a bias, i.e. a Linear's forward: float atomics
  // would make the forward differ run to run (tests/test_gpu_train_graphs.py asserts it is
  // bit-identical, as the reference's is)
  bool init_c = false;
  if (!big && splits == 1 && d.split_k == 0 && d.out_dtype == DP_F32 && d.act == DP_ACT_NONE && !d.gate &&
      d.batch == 1 && tiles < 512 && ksteps >= 4 && (int64_t)d.m * d.n <= 512 * 512 && !d.bias && d.beta != 1.f) {
    splits = (int)std::min<int64_t>((4096 + tiles - 1) / tiles, ksteps);
    if (splits > 1) {
      init_c = true;
      g.bias = nullptr;
      g.beta = 1.f;
    } else {
      splits = 1;
    }
  }
  if (splits > ksteps) splits = ksteps;
  DP_REQUIRE(splits == 1 || (d.out_dtype == DP_F32 && (init_c || (!d.bias && d.beta == 1.f)) && d.act == DP_ACT_NONE &&
                             !d.gate),
             "dp_gemm: split-K accumulates into f32 C (beta 1, no bias / act / gate)");
  g.splits = splits;
  g.kchunk = ((ksteps + splits - 1) / splits) * BK;
  DP_REQUIRE(tiles * 1 < (1ll << 31) && (int64_t)d.batch * splits < 65536, "dp_gemm: grid too large");
  dim3 grid((unsigned)(tm * tn), (unsigned)(d.batch * splits)), block(256);
  hipStream_t s = as_stream(stream);
  if (init_c) {
    const int64_t mn = (int64_t)d.m * d.n;
    hipLaunchKernelGGL(gemm_init_c_kernel, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<float*>(d.c), d.c_rs, d.m, d.n, d.beta, d.bias);
  }
  if (big) {
    constexpr size_t lds = sizeof(bf16_t) * 4 * IMG;   // 72 KB: two buffers of both operands
    static const bool attr_ok = [] {
      bool ok = true;
      for (const void* k : {reinterpret_cast<const void*>(&gemm128_kernel<0, 0>),
                            reinterpret_cast<const void*>(&gemm128_kernel<0, 1>),
                            reinterpret_cast<const void*>(&gemm128_kernel<1, 0>),
                            reinterpret_cast<const void*>(&gemm128_kernel<1, 1>)})
        ok = ok && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
      return ok;
    }();
    DP_REQUIRE(attr_ok, "dp_gemm: cannot set the 128x128 kernel's LDS size");
    if (g.modeA == 0 && g.modeB == 0) hipLaunchKernelGGL((gemm128_kernel<0, 0>), grid, block, lds, s, g);
    else if (g.modeA == 0) hipLaunchKernelGGL((gemm128_kernel<0, 1>), grid, block, lds, s, g);
    else if (g.modeB == 0) hipLaunchKernelGGL((gemm128_kernel<1, 0>), grid, block, lds, s, g);
    else hipLaunchKernelGGL((gemm128_kernel<1, 1>), grid, block, lds, s, g);
  }
  else if (d.in_dtype == DP_BF16)
    hipLaunchKernelGGL(gemm_kernel<bf16_t>, grid, block, 0, s, g);
  else
    hipLaunchKernelGGL(gemm_kernel<float>, grid, block, 0, s, g);
  if (d.colsum) {   // the kernels above do not fuse it: the bias gradient on its own kernel
    const int rc = dp_colsum(d.a, d.a_ks, d.k, d.m, d.colsum, 1, d.in_dtype, stream);
    if (rc) return rc;
  }
  return dp_check_launch("dp_gemm");
}

static int conv_wgrad(const void* x, int64_t x_bstride, int32_t x_pstride, int32_t batch, int32_t h, int32_t w,
                      int32_t cin, const void* dz, int64_t dz_ld, int32_t oh, int32_t ow, int32_t cout, int32_t kh,
                      int32_t kw, int32_t stride, int32_t pad, float* scratch, float* dw, int32_t dtype, void* stream,
                      bool scratch_zero) {
  DP_REQUIRE(x && dz && scratch && dw && batch > 0 && h > 0 && w > 0 && oh > 0 && ow > 0 && cout > 0 && kh > 0 &&
                 kw > 0 && stride > 0 && pad >= 0,
             "dp_conv_wgrad: bad arguments");
  DP_REQUIRE(dtype == DP_BF16 && cin % 8 == 0 && x_pstride % 8 == 0 && x_bstride % 8 == 0 && dz_ld % 8 == 0 &&
                 (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(dz) & 15) == 0,
             "dp_conv_wgrad: bf16, cin %% 8 == 0, 16-byte aligned pixels (cin %d, pstride %d, ld %lld)", cin,
             x_pstride, (long long)dz_ld);
  // the gather splits a pixel index with a float reciprocal, exact below 2^24: larger batches run
  // as consecutive image chunks accumulating into the same scratch (beta = 1)
  const int64_t ppi = (int64_t)oh * ow;
  DP_REQUIRE(ppi < (1ll << 24), "dp_conv_wgrad: %lld output pixels per image (needs < 2^24)", (long long)ppi);
  const int chunk = (int)std::min<int64_t>(batch, ((1ll << 24) - 1) / ppi);
  hipStream_t s = as_stream(stream);
  const int taps = kh * kw, N = taps * cin;
  // the LDS-DMA ring kernel (wgrad_tt_kernel<true>) wherever its 32-bit buffer offsets reach. Its
  // float atomics go to the tap-major scratch (contiguous columns), permuted into dw after: adding
  // straight into dw[co][ci][tap] (columns 9 floats apart) measured 3.9 -> 18.8 ms per L step.
  static const bool tt_off = getenv("DETRPOSE_WGRAD_TT") && atoi(getenv("DETRPOSE_WGRAD_TT")) == 0;
  const bool tt = !tt_off && cout % 8 == 0 && N % 8 == 0 && (int64_t)chunk * x_bstride * 2 < 0x7ff00000ll &&
                  ((int64_t)chunk * ppi * dz_ld + cout) * 2 < 0x7ff00000ll;
  if (!scratch_zero && dp_zero_async(scratch, (size_t)cout * N * sizeof(float), s)) {
    dp_set_error("dp_conv_wgrad: memset failed");
    return DP_EINVAL;
  }
  GemmArgs g{};
  g.A = Operand{dz, 0, 1, dz_ld, cout};   // A(m = co, k = p) = dz[p][co]: rows contiguous (mode 1)
  g.B = Operand{x, 0, 0, 0, N};
  g.modeA = 1;
  g.modeB = 3;
  g.cf = scratch;
  g.cb = nullptr;
  g.c_bs = 0;
  g.c_rs = N;
  g.M = cout, g.N = N, g.batch = 1;
  g.alpha = 1.f;
  g.beta = 1.f;
  g.act = DP_ACT_NONE;
  g.ix = reinterpret_cast<const bf16_t*>(x);
  g.ix_bs = x_bstride;
  g.ix_ps = x_pstride;
  g.ih = h, g.iw = w, g.icin = cin, g.ioh = oh, g.iow = ow, g.ikw = kw, g.istride = stride, g.ipad = pad;
  const int tm = (cout + BT - 1) / BT, tn = (N + BT - 1) / BT;
  g.tiles_n = tn;
  constexpr size_t lds = sizeof(bf16_t) * 4 * IMG;
  static const bool attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm128_kernel<1, 3>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  DP_REQUIRE(attr_ok, "dp_conv_wgrad: cannot set the kernel's LDS size");
  for (int b0 = 0; b0 < batch; b0 += chunk) {
    const int nb = std::min(chunk, batch - b0);
    const int64_t K = (int64_t)nb * ppi;
    g.A.p = reinterpret_cast<const bf16_t*>(dz) + (int64_t)b0 * ppi * dz_ld;
    g.ix = reinterpret_cast<const bf16_t*>(x) + (int64_t)b0 * x_bstride;
    g.B.p = g.ix;
    g.K = (int)K;
    if (tt) {
      const int tmw = (cout + WT_BM - 1) / WT_BM, tnw = (N + WT_BN - 1) / WT_BN;
      const int ntl = tmw * tnw;
      const int ks64 = (int)((K + 63) / 64);
      const int sp = wgrad_tt_splits(ntl, ks64);
      g.splits = sp;
      g.kchunk = ((ks64 + sp - 1) / sp) * 64;
      static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_tt_kernel<true>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   WT_NS * WT_STAGE) == hipSuccess;
      DP_REQUIRE(attr, "dp_conv_wgrad: cannot set the weight-gradient kernel's LDS size");
      hipLaunchKernelGGL(wgrad_tt_kernel<true>, dim3((unsigned)((ntl * sp + 7) / 8 * 8)), dim3(512),
                         WT_NS * WT_STAGE, s, g, ntl, tnw);
      continue;
    }
    const int ksteps = (int)((K + BKB - 1) / BKB);
    int splits = (512 + tm * tn - 1) / (tm * tn);
    if (splits > ksteps / 4) splits = ksteps / 4;
    if (splits < 1) splits = 1;
    g.splits = splits;
    g.kchunk = ((ksteps + splits - 1) / splits) * BKB;
    hipLaunchKernelGGL((gemm128_kernel<1, 3>), dim3((unsigned)(tm * tn), (unsigned)splits), dim3(256), lds, s, g);
  }
  const int64_t total = (int64_t)cout * N;
  if (scratch_zero)
    hipLaunchKernelGGL(wgrad_permute_kernel<true>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, scratch, dw,
                       cout, cin, taps);
  else
    hipLaunchKernelGGL(wgrad_permute_kernel<false>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, scratch,
                       dw, cout, cin, taps);
  return dp_check_launch("dp_conv_wgrad");
}

extern "C" int dp_conv_wgrad(const void* x, int64_t x_bstride, int32_t x_pstride, int32_t batch, int32_t h,
                             int32_t w, int32_t cin, const void* dz, int64_t dz_ld, int32_t oh, int32_t ow,
                             int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad, float* scratch,
                             float* dw, int32_t dtype, void* stream) {
  return conv_wgrad(x, x_bstride, x_pstride, batch, h, w, cin, dz, dz_ld, oh, ow, cout, kh, kw, stride, pad, scratch,
                    dw, dtype, stream, false);
}

extern "C" int dp_conv_wgrad_zs(const void* x, int64_t x_bstride, int32_t x_pstride, int32_t batch, int32_t h,
                                int32_t w, int32_t cin, const void* dz, int64_t dz_ld, int32_t oh, int32_t ow,
                                int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad, float* scratch,
                                float* dw, int32_t dtype, void* stream) {
  return conv_wgrad(x, x_bstride, x_pstride, batch, h, w, cin, dz, dz_ld, oh, ow, cout, kh, kw, stride, pad, scratch,
                    dw, dtype, stream, true);
}
