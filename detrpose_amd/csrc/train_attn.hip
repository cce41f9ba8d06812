// Training attention core on MFMA (bf16, sequences of at most 128 tokens, or 400 with 32-wide
// heads): the decoder's within-instance (18 tokens) and across-instance (60 + DN tokens, with the
// DN attn_mask) nn.MultiheadAttention cores of the training step (transformer.py:403-419;
// dn_component.py:155-167) and the encoder's AIFI layer (hybrid_encoder.py:276-279, the 20 x 20
// map), behind dp_attn_fwd / dp_attn_bwd (train.hip) for dtype bf16. Same interface and
// saved tensor as the scalar kernels in train.hip: P f32 [pair][key][query].
//
// All three kernels run one wave per (sequence, head, 16-row tile) on v_mfma_f32_16x16x32_bf16,
// the whole other side of the sequence (<= 16 KT rows) in registers, nothing shared across
// waves (no block barrier). Operand layouts (cdna_hip_programming.md §3): lane (lr = lane & 15,
// lg = lane >> 4) holds A[row lr][k 8lg .. 8lg+7], B[k 8lg .. 8lg+7][col lr], and C[row 4lg + r]
// [col lr] in register r.
//   forward (query tile i):  S^T = K Q^T (key rows x query columns), softmax down the columns
//     (registers + two xor-shuffles), P saved, O^T = V^T P^T: the lane's P^T values of key tiles
//     (2m, 2m+1) are its B fragment for the 32-key step m with k slot s <-> key 32m + 4lg + s
//     (s < 4) / 32m + 16 + 4lg + s - 4 (s >= 4); the A fragment V^T[d][those keys] comes from V
//     staged transposed in the wave's LDS slice (two 8-byte reads).
//   dQ (query tile i):       dP^T = V dO^T, dS^T = P^T (dP^T - D) with D_i = dO_i . O_i, then
//     dQ^T = K^T dS^T the same way (K^T in LDS).
//   dK, dV (key tile j):     dP = dO V^T (query rows x key columns), dS = P (dP - D), then
//     dV^T = dO^T P and dK^T = Q^T dS: contractions over the queries, whose P / dS tiles
//     (2m, 2m+1) are the B fragments with the same slot order; dO^T and Q^T in LDS.
// Rows past the sequence read as zero; keys past it (and masked keys) get P = 0; a query whose
// keys are all masked gets P = 0 and O = 0, as the scalar kernel.
#include "common.h"

namespace {

// waves per block: 4, or 2 for the 400-token AIFI instantiation (its per-wave LDS slices)
template <int KT>
constexpr int wpb_of() { return KT > 8 ? 2 : 4; }

// SH (sequences of more than 32 tokens: the decoder's across-instance attention with its DN
// queries, the 400-token AIFI layer): every wave of a block works on the SAME (sequence, head)
// pair, one query (or key) tile each, and the block stages the pair's transposed operands into
// LDS once (was once per wave: AIFI's 25 waves per pair re-staged the same 26 KB, the backward's
// dK/dV kernel also recomputed D over all the queries per wave). Block = nw waves (nw | tiles
// when a divisor in 4..8 exists), grid = pairs x ceil(tiles / nw); waves past the tiles only
// stage. The within-instance attention (18 tokens, 2 tiles) keeps one pair tile per wave.
template <int KT>
constexpr bool shared_of() { return KT >= 4; }
constexpr int SH_MAXW = 8;

// block width (waves) of a shared-staging launch over `tiles` tiles per pair
static inline int sh_waves(int tiles) {
  for (int w = SH_MAXW; w >= 4; --w)
    if (tiles % w == 0) return w;
  return tiles < SH_MAXW ? tiles : SH_MAXW;
}

// (pair, tile, live) of this wave: SH from the block's pair and the wave's slot, else one item
// per wave (item = pair * tiles + tile)
template <bool SH>
__device__ __forceinline__ bool wave_item(int tiles, int items, int wpb, int wave, int& pair, int& t) {
  if (SH) {
    const int nw = blockDim.x >> 6, bpp = (tiles + nw - 1) / nw;
    pair = blockIdx.x / bpp;
    t = (blockIdx.x - pair * bpp) * nw + wave;
    return t < tiles;
  }
  const int item = blockIdx.x * wpb + wave;
  pair = item / tiles;
  t = item - pair * tiles;
  return item < items;
}

__device__ __forceinline__ int64_t row_base(int pair, int nhead, int n_inner, int64_t so, int64_t si) {
  const int sq = pair / nhead;
  const int o = sq / n_inner, ii = sq - o * n_inner;
  return (int64_t)o * so + (int64_t)ii * si;
}

// one 16-byte row chunk (8 bf16) of row `row` (zero past L or past the head dim)
template <int DH>
__device__ __forceinline__ bf16x8 frag_row(const bf16_t* p, int64_t base, int64_t st, int64_t ld, int col0, int row,
                                           int L, int d0) {
  if (row < L && d0 < DH) return *reinterpret_cast<const bf16x8*>(p + (base + (int64_t)row * st) * ld + col0 + d0);
  return bf16x8{};
}

// rows 0 .. NK-1 of a head (zero past L), transposed into dst[DH][VP]
template <int DH, int NK, int VP>
__device__ __forceinline__ void stage_t(bf16_t* dst, const bf16_t* src, int64_t base, int64_t st, int64_t ld, int col0,
                                        int L, int lane, int nthreads = 64) {
  constexpr int CH = DH / 8;
  for (int c = lane; c < NK * CH; c += nthreads) {
    const int row = c / CH, dc = c - row * CH;
    bf16x8 v = bf16x8{};
    if (row < L) v = *reinterpret_cast<const bf16x8*>(src + (base + (int64_t)row * st) * ld + col0 + dc * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) dst[(dc * 8 + e) * VP + row] = v[e];
  }
}

// A fragment of a [DH][VP] transposed tile for the 32-row step m: row d, k slots as above
template <int VP>
__device__ __forceinline__ bf16x8 frag_t(const bf16_t* t, int d, int m, int lg) {
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(t + d * VP + 32 * m + 4 * lg);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(t + d * VP + 32 * m + 16 + 4 * lg);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int DH, int KT>
__global__ __launch_bounds__(256) void attn_fwd_mfma_kernel(const bf16_t* __restrict__ q, int ldq,
                                                            const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                            int ldkv, bf16_t* __restrict__ out, int ldo,
                                                            float* __restrict__ psave,
                                                            const uint8_t* __restrict__ mask, int n_inner, int64_t so,
                                                            int64_t si, int64_t st, int L, int nhead, int items,
                                                            float scale) {
  constexpr int KS = (DH + 31) / 32, ND = DH / 16, NK = 16 * KT, VP = NK + 8, NM = (KT + 1) / 2;
  static_assert(KT % 2 == 0, "tiles are read in pairs: an odd KT would read past a V^T row");
  // the forward stages V^T only: shared staging measured no faster for AIFI (65 us either way) and
  // slower for the across attention (44 -> 49 us), so each wave keeps its own slice
  constexpr bool SH = false;
  __shared__ __attribute__((aligned(16))) bf16_t lds[SH ? 1 : wpb_of<KT>()][DH * VP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nqt = (L + 15) / 16;
  int pair, it;
  const bool live = wave_item<SH>(nqt, items, wpb_of<KT>(), wave, pair, it);
  if (!SH && !live) return;   // wave-uniform
  const int h = pair % nhead;
  const int64_t base = row_base(pair, nhead, n_inner, so, si);
  const int lr = lane & 15, lg = lane >> 4;
  bf16_t* Vt = lds[SH ? 0 : wave];
  if (SH) {
    stage_t<DH, NK, VP>(Vt, v, base, st, ldkv, h * DH, L, threadIdx.x, blockDim.x);
    __syncthreads();
    if (!live) return;
  } else {
    stage_t<DH, NK, VP>(Vt, v, base, st, ldkv, h * DH, L, lane);
  }
  const int qi = 16 * it + lr;
  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qf[ks] = frag_row<DH>(q, base, st, ldq, h * DH, qi, L, 32 * ks + 8 * lg);
  f32x4 s[KT];
#pragma unroll
  for (int j = 0; j < KT; ++j) {
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 kf = frag_row<DH>(k, base, st, ldkv, h * DH, 16 * j + lr, L, 32 * ks + 8 * lg);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], a, 0, 0, 0);
    }
    s[j] = a;
  }
  const int qc = min(qi, L - 1);
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < KT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * j + 4 * lg + r;
      bool ok = key < L;
      if (mask) ok = ok && mask[(int64_t)qc * L + min(key, L - 1)] == 0;
      const float x = ok ? s[j][r] * scale : -INFINITY;
      s[j][r] = x;
      mx = fmaxf(mx, x);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float mref = mx == -INFINITY ? 0.f : mx;
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < KT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = __expf(s[j][r] - mref);
      s[j][r] = p;
      sum += p;
    }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  float* P = psave + (int64_t)pair * L * L;
#pragma unroll
  for (int j = 0; j < KT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[j][r] *= inv;
      const int key = 16 * j + 4 * lg + r;
      if (key < L && qi < L) P[(int64_t)key * L + qi] = s[j][r];
    }
  lds_sync();
  f32x4 o[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    bf16x8 pf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pf[r] = (bf16_t)s[2 * m][r];
      pf[4 + r] = 2 * m + 1 < KT ? (bf16_t)s[2 * m + 1 < KT ? 2 * m + 1 : 0][r] : (bf16_t)0.f;
    }
#pragma unroll
    for (int d = 0; d < ND; ++d) o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t<VP>(Vt, 16 * d + lr, m, lg), pf,
                                                                                 o[d], 0, 0, 0);
  }
  if (qi < L) {
    bf16_t* op = out + (base + (int64_t)qi * st) * ldo + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const bf16x4 ov = bf16x4{(bf16_t)o[d][0], (bf16_t)o[d][1], (bf16_t)o[d][2], (bf16_t)o[d][3]};
      *reinterpret_cast<bf16x4*>(op + 16 * d + 4 * lg) = ov;
    }
  }
}

template <int DH, int KT>
__global__ __launch_bounds__(shared_of<KT>() ? 64 * SH_MAXW : 256) void attn_bwd_q_mfma_kernel(const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                              int ldkv, const float* __restrict__ psave,
                                                              const bf16_t* __restrict__ dout,
                                                              const bf16_t* __restrict__ out, int ldo,
                                                              bf16_t* __restrict__ dq, int lddq, int n_inner,
                                                              int64_t so, int64_t si, int64_t st, int L, int nhead,
                                                              int items, float scale) {
  constexpr int KS = (DH + 31) / 32, ND = DH / 16, NK = 16 * KT, VP = NK + 8, NM = (KT + 1) / 2;
  static_assert(KT % 2 == 0, "tiles are read in pairs: an odd KT would read past a V^T row");
  constexpr bool SH = shared_of<KT>();
  __shared__ __attribute__((aligned(16))) bf16_t lds[SH ? 1 : wpb_of<KT>()][DH * VP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nqt = (L + 15) / 16;
  int pair, it;
  const bool live = wave_item<SH>(nqt, items, wpb_of<KT>(), wave, pair, it);
  if (!SH && !live) return;
  const int h = pair % nhead;
  const int64_t base = row_base(pair, nhead, n_inner, so, si);
  const int lr = lane & 15, lg = lane >> 4;
  bf16_t* Kt = lds[SH ? 0 : wave];
  if (SH) {
    stage_t<DH, NK, VP>(Kt, k, base, st, ldkv, h * DH, L, threadIdx.x, blockDim.x);
    __syncthreads();
    if (!live) return;
  } else {
    stage_t<DH, NK, VP>(Kt, k, base, st, ldkv, h * DH, L, lane);
  }
  const int qi = 16 * it + lr;
  bf16x8 gf[KS];
  float D = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    gf[ks] = frag_row<DH>(dout, base, st, ldo, h * DH, qi, L, 32 * ks + 8 * lg);
    const bf16x8 of = frag_row<DH>(out, base, st, ldo, h * DH, qi, L, 32 * ks + 8 * lg);
#pragma unroll
    for (int e = 0; e < 8; ++e) D = fmaf((float)gf[ks][e], (float)of[e], D);
  }
  D += __shfl_xor(D, 16, 64);
  D += __shfl_xor(D, 32, 64);
  const float* P = psave + (int64_t)pair * L * L;
  const int qc = min(qi, L - 1);
  f32x4 ds[KT];
#pragma unroll
  for (int j = 0; j < KT; ++j) {
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 vf = frag_row<DH>(v, base, st, ldkv, h * DH, 16 * j + lr, L, 32 * ks + 8 * lg);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, gf[ks], a, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * j + 4 * lg + r;
      const float p = P[(int64_t)min(key, L - 1) * L + qc];
      ds[j][r] = key < L && qi < L ? p * (a[r] - D) : 0.f;
    }
  }
  lds_sync();
  f32x4 acc[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) acc[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    bf16x8 bf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bf[r] = (bf16_t)ds[2 * m][r];
      bf[4 + r] = 2 * m + 1 < KT ? (bf16_t)ds[2 * m + 1 < KT ? 2 * m + 1 : 0][r] : (bf16_t)0.f;
    }
#pragma unroll
    for (int d = 0; d < ND; ++d)
      acc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t<VP>(Kt, 16 * d + lr, m, lg), bf, acc[d], 0, 0, 0);
  }
  if (qi < L) {
    bf16_t* op = dq + (base + (int64_t)qi * st) * lddq + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const bf16x4 ov = bf16x4{(bf16_t)(acc[d][0] * scale), (bf16_t)(acc[d][1] * scale), (bf16_t)(acc[d][2] * scale),
                               (bf16_t)(acc[d][3] * scale)};
      *reinterpret_cast<bf16x4*>(op + 16 * d + 4 * lg) = ov;
    }
  }
}

template <int DH, int KT>
__global__ __launch_bounds__(shared_of<KT>() ? 64 * SH_MAXW : 256) void attn_bwd_kv_mfma_kernel(const bf16_t* __restrict__ q, int ldq,
                                                               const bf16_t* __restrict__ v, int ldkv,
                                                               const float* __restrict__ psave,
                                                               const bf16_t* __restrict__ dout,
                                                               const bf16_t* __restrict__ out, int ldo,
                                                               bf16_t* __restrict__ dk, bf16_t* __restrict__ dv,
                                                               int lddkv, int n_inner, int64_t so, int64_t si,
                                                               int64_t st, int L, int nhead, int items, float scale) {
  constexpr int KS = (DH + 31) / 32, ND = DH / 16, NK = 16 * KT, VP = NK + 8, NM = (KT + 1) / 2;
  static_assert(KT % 2 == 0, "tiles are read in pairs: an odd KT would read past a V^T row");
  constexpr bool SH = shared_of<KT>();
  constexpr int NSL = SH ? 1 : wpb_of<KT>();
  __shared__ __attribute__((aligned(16))) bf16_t lds[NSL][2 * DH * VP];
  __shared__ float Ds[NSL][NK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nkt = (L + 15) / 16;
  int pair, jt;
  const bool live = wave_item<SH>(nkt, items, wpb_of<KT>(), wave, pair, jt);
  if (!SH && !live) return;
  const int h = pair % nhead;
  const int64_t base = row_base(pair, nhead, n_inner, so, si);
  const int lr = lane & 15, lg = lane >> 4;
  const int sl = SH ? 0 : wave;
  bf16_t* Gt = lds[sl];             // dO^T [DH][VP]
  bf16_t* Qt = lds[sl] + DH * VP;   // Q^T  [DH][VP]
  // SH: the block stages once (all its threads); otherwise each wave its own slice
  const int t0 = SH ? (int)threadIdx.x : lane, tn = SH ? (int)blockDim.x : 64;
  stage_t<DH, NK, VP>(Gt, dout, base, st, ldo, h * DH, L, t0, tn);
  stage_t<DH, NK, VP>(Qt, q, base, st, ldq, h * DH, L, t0, tn);
  for (int qq = t0; qq < NK; qq += tn) {   // D_q = dO_q . O_q
    float D = 0.f;
    if (qq < L) {
      const int64_t rb = (base + (int64_t)qq * st) * ldo + h * DH;
#pragma unroll
      for (int c = 0; c < DH / 8; ++c) {
        const bf16x8 g = *reinterpret_cast<const bf16x8*>(dout + rb + 8 * c);
        const bf16x8 o = *reinterpret_cast<const bf16x8*>(out + rb + 8 * c);
#pragma unroll
        for (int e = 0; e < 8; ++e) D = fmaf((float)g[e], (float)o[e], D);
      }
    }
    Ds[sl][qq] = D;
  }
  if (SH) {
    __syncthreads();
    if (!live) return;
  }
  const int kj = 16 * jt + lr;   // this lane's key column
  bf16x8 vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) vf[ks] = frag_row<DH>(v, base, st, ldkv, h * DH, kj, L, 32 * ks + 8 * lg);
  lds_sync();
  const float* P = psave + (int64_t)pair * L * L + (int64_t)min(kj, L - 1) * L;
  f32x4 p[KT], ds[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 gf = frag_row<DH>(dout, base, st, ldo, h * DH, 16 * i + lr, L, 32 * ks + 8 * lg);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gf, vf[ks], a, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qq = 16 * i + 4 * lg + r;
      const float pv = P[min(qq, L - 1)];
      const bool ok = qq < L && kj < L;
      p[i][r] = ok ? pv : 0.f;
      ds[i][r] = ok ? pv * (a[r] - Ds[sl][min(qq, NK - 1)]) : 0.f;
    }
  }
  f32x4 av[ND], ak[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    av[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    ak[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    bf16x8 pf, sf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i1 = 2 * m + 1 < KT ? 2 * m + 1 : 0;
      pf[r] = (bf16_t)p[2 * m][r];
      sf[r] = (bf16_t)ds[2 * m][r];
      pf[4 + r] = 2 * m + 1 < KT ? (bf16_t)p[i1][r] : (bf16_t)0.f;
      sf[4 + r] = 2 * m + 1 < KT ? (bf16_t)ds[i1][r] : (bf16_t)0.f;
    }
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      av[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t<VP>(Gt, 16 * d + lr, m, lg), pf, av[d], 0, 0, 0);
      ak[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t<VP>(Qt, 16 * d + lr, m, lg), sf, ak[d], 0, 0, 0);
    }
  }
  if (kj < L) {
    const int64_t rb = (base + (int64_t)kj * st) * lddkv + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      *reinterpret_cast<bf16x4*>(dv + rb + 16 * d + 4 * lg) =
          bf16x4{(bf16_t)av[d][0], (bf16_t)av[d][1], (bf16_t)av[d][2], (bf16_t)av[d][3]};
      *reinterpret_cast<bf16x4*>(dk + rb + 16 * d + 4 * lg) =
          bf16x4{(bf16_t)(ak[d][0] * scale), (bf16_t)(ak[d][1] * scale), (bf16_t)(ak[d][2] * scale),
                 (bf16_t)(ak[d][3] * scale)};
    }
  }
}

template <int DH, int KT>
void launch_fwd(const bf16_t* q, int ldq, const bf16_t* k, const bf16_t* v, int ldkv, bf16_t* out, int ldo, float* ps,
                const uint8_t* mask, int npairs, int n_inner, int64_t so, int64_t si, int64_t st, int L, int nhead,
                float scale, hipStream_t s) {
  const int items = npairs * ((L + 15) / 16);
  constexpr int WPB = wpb_of<KT>();
  const dim3 grid((items + WPB - 1) / WPB), block(64 * WPB);
  hipLaunchKernelGGL((attn_fwd_mfma_kernel<DH, KT>), grid, block, 0, s, q, ldq, k, v,
                     ldkv, out, ldo, ps, mask, n_inner, so, si, st, L, nhead, items, scale);
}

template <int DH, int KT>
void launch_bwd(const bf16_t* q, int ldq, const bf16_t* k, const bf16_t* v, int ldkv, const float* ps,
                const bf16_t* dout, const bf16_t* out, int ldo, bf16_t* dq, int lddq, bf16_t* dk, bf16_t* dv, int lddkv,
                int npairs, int n_inner, int64_t so, int64_t si, int64_t st, int L, int nhead, float scale,
                hipStream_t s) {
  const int tiles = (L + 15) / 16, items = npairs * tiles;
  constexpr int WPB = wpb_of<KT>();
  const int nw = shared_of<KT>() ? sh_waves(tiles) : WPB;
  const dim3 grid(shared_of<KT>() ? npairs * ((tiles + nw - 1) / nw) : (items + WPB - 1) / WPB), block(64 * nw);
  hipLaunchKernelGGL((attn_bwd_q_mfma_kernel<DH, KT>), grid, block, 0, s, k, v, ldkv, ps, dout, out, ldo, dq, lddq,
                     n_inner, so, si, st, L, nhead, items, scale);
  hipLaunchKernelGGL((attn_bwd_kv_mfma_kernel<DH, KT>), grid, block, 0, s, q, ldq, v, ldkv, ps, dout, out, ldo, dk, dv,
                     lddkv, n_inner, so, si, st, L, nhead, items, scale);
}

template <int DH>
bool dispatch_kt(int L, bool bwd, const void* const* a, const int64_t* n, float scale, hipStream_t s) {
  // a / n: the pointer / integer arguments in the order of dp_attn_fwd / dp_attn_bwd
  const int kt = (L + 15) / 16;
#define DP_ATT_KT(KTV)                                                                                               \
  if (kt <= KTV) {                                                                                                   \
    if (!bwd)                                                                                                        \
      launch_fwd<DH, KTV>((const bf16_t*)a[0], (int)n[0], (const bf16_t*)a[1], (const bf16_t*)a[2], (int)n[1],       \
                          (bf16_t*)a[3], (int)n[2], (float*)a[4], (const uint8_t*)a[5], (int)n[3], (int)n[4], n[5],  \
                          n[6], n[7], L, (int)n[8], scale, s);                                                       \
    else                                                                                                             \
      launch_bwd<DH, KTV>((const bf16_t*)a[0], (int)n[0], (const bf16_t*)a[1], (const bf16_t*)a[2], (int)n[1],       \
                          (const float*)a[3], (const bf16_t*)a[4], (const bf16_t*)a[5], (int)n[2], (bf16_t*)a[6],    \
                          (int)n[3], (bf16_t*)a[7], (bf16_t*)a[8], (int)n[9], (int)n[4], (int)n[5], n[6], n[7], n[8], \
                          L, (int)n[10], scale, s);                                                                  \
    return true;                                                                                                     \
  }
  DP_ATT_KT(2)
  DP_ATT_KT(4)
  DP_ATT_KT(8)
  // AIFI (hybrid_encoder.py:276-279): the 20 x 20 = 400 tokens of the stride-32 map, 32-wide heads
  if constexpr (DH == 32) {
    DP_ATT_KT(26)   // even: the PV step reads key tiles in pairs (V^T rows of 16 KT + 8)
  }
#undef DP_ATT_KT
  return false;
}

}  // namespace

// Called by dp_attn_fwd / dp_attn_bwd (train.hip) for bf16: false when the shape is not covered
// (sequence > 128 tokens, head dim not 16 / 32 / 48 / 64) and the scalar kernels run instead.
// every row start of a bf16 operand with row pitch ld (elements) is 16-byte aligned
static bool rows16(const void* p, int64_t ld) {
  return p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 8 == 0;
}

bool dp_attn_fwd_mfma(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, void* out, int32_t ld_o,
                      float* p_save, const uint8_t* mask, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si,
                      int64_t st, int32_t seqlen, int32_t nhead, int32_t dh, float scale, hipStream_t s) {
  if (seqlen > (dh == 32 ? 400 : 128)) return false;
  // 16-byte bf16x8 / 8-byte bf16x4 rows: other layouts take the scalar kernels
  if (!rows16(q, ld_q) || !rows16(k, ld_kv) || !rows16(v, ld_kv) || !rows16(out, ld_o)) return false;
  const void* a[6] = {q, k, v, out, p_save, mask};
  const int64_t n[9] = {ld_q, ld_kv, ld_o, (int64_t)n_outer * n_inner * nhead, n_inner, so, si, st, nhead};
  switch (dh) {
    case 16: return dispatch_kt<16>(seqlen, false, a, n, scale, s);
    case 32: return dispatch_kt<32>(seqlen, false, a, n, scale, s);
    case 48: return dispatch_kt<48>(seqlen, false, a, n, scale, s);
    case 64: return dispatch_kt<64>(seqlen, false, a, n, scale, s);
    default: return false;
  }
}

bool dp_attn_bwd_mfma(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, const float* p_save,
                      const void* dout, const void* out, int32_t ld_o, void* dq, int32_t ld_dq, void* dk, void* dv,
                      int32_t ld_dkv, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si, int64_t st,
                      int32_t seqlen, int32_t nhead, int32_t dh, float scale, hipStream_t s) {
  if (seqlen > (dh == 32 ? 400 : 128)) return false;
  if (!rows16(q, ld_q) || !rows16(k, ld_kv) || !rows16(v, ld_kv) || !rows16(out, ld_o) || !rows16(dout, ld_o) ||
      !rows16(dq, ld_dq) || !rows16(dk, ld_dkv) || !rows16(dv, ld_dkv))
    return false;
  const void* a[9] = {q, k, v, p_save, dout, out, dq, dk, dv};
  const int64_t n[11] = {ld_q, ld_kv, ld_o, ld_dq, (int64_t)n_outer * n_inner * nhead, n_inner, so, si, st, ld_dkv,
                         nhead};
  switch (dh) {
    case 16: return dispatch_kt<16>(seqlen, true, a, n, scale, s);
    case 32: return dispatch_kt<32>(seqlen, true, a, n, scale, s);
    case 48: return dispatch_kt<48>(seqlen, true, a, n, scale, s);
    case 64: return dispatch_kt<64>(seqlen, true, a, n, scale, s);
    default: return false;
  }
}
