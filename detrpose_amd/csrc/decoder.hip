// Row-block fused kernels of the decoder layer (gfx950, bf16 storage, f32 accumulation).
//
// The decoder's token GEMMs have N = C (128 / 256 / 384) or a few C: one block can own
// every output channel of its rows, so whatever follows a GEMM row-wise (bias, residual,
// LayerNorm, the Gate's sigmoid mix, the in-place pos add, a second or third GEMM of an
// MLP) finishes inside the block instead of round-tripping through HBM:
//   dp_linear_layernorm       out_proj + residual + LN (+ pos re-add)   transformer.py:403-422
//   dp_gate_linear_layernorm  Gate: Linear(2C->2C), sigmoid mix, LN     transformer.py:222-235
//   dp_ffn_layernorm          Linear-ReLU-Linear + residual + LN        transformer.py:371-385
//   dp_query_pos              sine embedding -> MLP(C,C,C,2) -> pos, tgt += pos
//                                                                        transformer.py:360-370, 518-540, 588-592
//   dp_pose_mlp               pose_embed MLP(C,C,66,3) (+ previous corners)  transformer.py:705-719
//
// Block = BM token rows (64 / 96 / 128) and NW = C/32 waves; wave w owns output channels
// [32w, 32w+32) of EVERY row of the block (TM = BM/16 row tiles x 2 column tiles of
// 16x16), so each weight fragment it loads feeds TM MFMAs: the weights are re-read from
// L2 once per BM rows (flop per L2 weight byte = BM), which is what bounds these K = C
// GEMMs. The row tile is staged once into LDS (16-byte chunks XOR-swizzled by row:
// conflict-free ds_read_b128 of 16 rows x one chunk); weight fragments go straight from
// L2 into registers (no other wave needs them), prefetched D k-steps ahead; the weights
// are pre-packed in MFMA-fragment order (include/detrpose_hip.h, "fragment layout"), so
// each fragment load is one contiguous 1 KB wave access instead of 16 rows x 64 B. MFMA
// 16x16x32 with the weights as the A operand and the rows as B, so a lane ends with 8
// CONTIGUOUS channels of one row (the A-row -> channel map below): bias, LN and stores
// work on whole 16-byte chunks. Hidden activations of an MLP go back to LDS as bf16
// (they are the next GEMM's B operand). LayerNorm statistics: shuffles across the lane
// groups, then NW partial sums per row through LDS, two passes (mean, then centred
// variance) as nn.LayerNorm computes them.
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int TN = 2;          // 16-column tiles per wave: 32 channels
constexpr int NV = 4 * TN;     // channels per lane per row (contiguous)

// byte offset of 16-byte chunk c of row m in a [rows][K] bf16 LDS image (K % 128 == 0)
template <int K>
__device__ __forceinline__ int sw(int m, int c) {
  return m * (K * 2) + (((c & ~15) | ((c ^ m) & 15)) << 4);
}

__device__ __forceinline__ bf16x8 lds16(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}
__device__ __forceinline__ void sts16(char* base, int off, const bf16x8& v) {
  *reinterpret_cast<bf16x8*>(base + off) = v;
}
__device__ __forceinline__ bf16x8 gld16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// Stage rows [row0, row0+BM) of a row-mapped bf16 matrix (K columns) into LDS in two
// halves, so a kernel can issue its weight prefetch between them: stage_load issues the
// global loads, stage_store writes the LDS image (rows past `rows` are zero). With ADD,
// the element-wise sum of two row-mapped sources rounded to bf16.
template <int K, int BM, int NTH, bool ADD>
struct Stage {
  static constexpr int CH = K / 8;
  static constexpr int PER = BM * CH / NTH;   // chunks per thread
  static_assert((BM * CH) % NTH == 0, "stage");
  bf16x8 v[PER], v2[ADD ? PER : 1];

  __device__ __forceinline__ void load(const bf16_t* __restrict__ x, dp_rowmap xm, const bf16_t* __restrict__ x2,
                                       dp_rowmap x2m, int row0, int rows) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int e = threadIdx.x + NTH * t;
      const int m = e / CH, c = e - m * CH;
      const int r = min(row0 + m, rows - 1);
      v[t] = gld16(x + rowmap_off(xm, r) + c * 8);
      if constexpr (ADD) v2[t] = gld16(x2 + rowmap_off(x2m, r) + c * 8);
    }
  }
  __device__ __forceinline__ void store(char* lds, int row0, int rows) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int e = threadIdx.x + NTH * t;
      const int m = e / CH, c = e - m * CH;
      bf16x8 o = v[t];
      if constexpr (ADD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16_t)((float)v[t][j] + (float)v2[t][j]);
      }
      if (row0 + m >= rows) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16_t)0.f;
      }
      sts16(lds, sw<K>(m, c), o);
    }
  }
};

// Block barrier for LDS hand-offs only: LDS writes retired, then s_barrier. Unlike
// __syncthreads() it does not wait for outstanding global loads, so the weight-fragment
// prefetch of the next GEMM stays in flight across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// channel (within the wave's 32) of A-operand row a (0..15) of column tile j: lane group
// g of the C tile then holds channels 8g + 4j + r (r = 0..3) = 8 contiguous channels
__device__ __forceinline__ int a_chan(int j, int a) { return (a >> 2) * NV + 4 * j + (a & 3); }

// Weight-fragment ring of one wave: the fragments of k-step s of the running GEMM sit in
// f[s % D]; D k-steps are in flight.
constexpr int D = 4;
template <int DD>
struct WPipeT {
  bf16x8 f[DD][TN];
};
using WPipe = WPipeT<D>;

// Fragment-layout weights: for output-channel block nb (32 channels) and k-step s, the
// TN fragments of the 64 lanes are 1 KB each, contiguous: frag(nb, s, j) at
// ((nb * NS + s) * TN + j) * 512 elements, lane l's 8 elements at + 8 l. `wb` below is a
// lane's pointer to its fragment of (nb, s0, 0).
__device__ __forceinline__ const bf16_t* frag_base(const bf16_t* w, int nb, int ksteps, int s0 = 0) {
  const int lane = threadIdx.x & 63;
  return w + ((int64_t)(nb * ksteps + s0) * TN * 64 + lane) * 8;
}

template <int DD>
__device__ __forceinline__ void pipe_start(WPipeT<DD>& p, const bf16_t* wb) {
#pragma unroll
  for (int s = 0; s < DD; ++s)
#pragma unroll
    for (int j = 0; j < TN; ++j) p.f[s][j] = gld16(wb + (s * TN + j) * 512);
}

// acc[i][j] += sum_k X[16i + q][k] * W[chan_j][k] over K, X from the LDS image, W as
// fragments from global. The pipe holds this GEMM's first D k-steps on entry; as its own
// steps run out it loads the first D k-steps of the NEXT GEMM (fragment base nx), so the
// ring never drains between the GEMMs of a kernel. The X fragments of k-step s+1 are read
// from LDS while the MFMAs of step s run (XDB; otherwise each step's X fragments are read
// just before its MFMAs: fewer registers, the latency left to the other waves of the SIMD).
template <int K, int TM, int DD = D, bool XDB = true>
__device__ __forceinline__ void wave_gemm(f32x4 (&acc)[TM][TN], const char* xl, const bf16_t* wb, WPipeT<DD>& p,
                                          const bf16_t* nx) {
  constexpr int NS = K / 32;
  static_assert(NS % DD == 0, "k-steps must fill the ring");
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4;
  bf16x8 xf[XDB ? 2 : 1][TM];
  if constexpr (XDB) {
#pragma unroll
    for (int i = 0; i < TM; ++i) xf[0][i] = lds16(xl, sw<K>(16 * i + q, g));
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    bf16x8 w[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) w[j] = p.f[s % DD][j];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      p.f[s % DD][j] = gld16(s + DD < NS ? wb + ((s + DD) * TN + j) * 512 : nx + ((s + DD - NS) * TN + j) * 512);
    if constexpr (XDB) {
      if (s + 1 < NS) {
#pragma unroll
        for (int i = 0; i < TM; ++i) xf[(s + 1) & 1][i] = lds16(xl, sw<K>(16 * i + q, 4 * (s + 1) + g));
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) xf[0][i] = lds16(xl, sw<K>(16 * i + q, 4 * s + g));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xf[XDB ? (s & 1) : 0][i], acc[i][j], 0, 0, 0);
  }
}

template <int TM>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[TM][TN]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// the lane's 8 contiguous channel values of row tile i
template <int TM>
__device__ __forceinline__ void lane_vals(const f32x4 (&acc)[TM][TN], int i, float (&v)[NV]) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[4 * j + r] = acc[i][j][r];
}

// per-row sum over the block's channels (lane: 8 values of row 16i+q); result broadcast to
// every lane holding that row. red: NW x BM floats of LDS.
template <int TM, int NW>
__device__ __forceinline__ void row_sums(const float (&x)[TM][NV], float (&out)[TM], float* red) {
  constexpr int BM = 16 * TM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < NV; ++e) s += x[i][e];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (g == 0) red[w * BM + 16 * i + q] = s;
  }
  lds_barrier();
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = 16 * i + q;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) s += red[ww * BM + m];
    out[i] = s;
  }
  lds_barrier();
}

// in-place LayerNorm of the block's rows: x[i][e] is channel cb + e of row 16i+q; gg/bb are
// the lane's gamma/beta (fetched at kernel start with everything else)
template <int TM, int NW>
__device__ __forceinline__ void layernorm_rows(float (&x)[TM][NV], const float (&gg)[NV], const float (&bb)[NV],
                                               float eps, float* red) {
  constexpr float invc = 1.f / (32 * NW);
  float mean[TM], var[TM];
  row_sums<TM, NW>(x, mean, red);
#pragma unroll
  for (int i = 0; i < TM; ++i) mean[i] *= invc;
  float d[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      const float t = x[i][e] - mean[i];
      d[i][e] = t * t;
    }
  row_sums<TM, NW>(d, var, red);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const float rstd = rsqrtf(var[i] * invc + eps);
#pragma unroll
    for (int e = 0; e < NV; ++e) x[i][e] = (x[i][e] - mean[i]) * rstd * gg[e] + bb[e];
  }
}

// layernorm_rows in one LDS round: per lane (mean, M2) of its 8 values, merged over the lane
// groups (xor shuffles) and then the waves (LDS) by the equal-count pairwise update
// M2 = M2a + M2b + (ma - mb)^2 n / 2 (Chan et al.), in a fixed order. red: NW x BM float2.
template <int TM, int NW>
__device__ __forceinline__ void layernorm_rows_1p(float (&x)[TM][NV], const float (&gg)[NV], const float (&bb)[NV],
                                                  float eps, float* red) {
  constexpr int BM = 16 * TM;
  static_assert(NW == 8, "three merge levels over the waves");
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, w = threadIdx.x >> 6;
  float2* r2 = reinterpret_cast<float2*>(red);
  float mean[TM], rstd[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float m = 0.f;
#pragma unroll
    for (int e = 0; e < NV; ++e) m += x[i][e];
    m *= 1.f / NV;
    float m2 = 0.f;
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      const float t = x[i][e] - m;
      m2 = fmaf(t, t, m2);
    }
    float n = NV;
#pragma unroll
    for (int sh = 16; sh <= 32; sh *= 2) {
      const float mo = __shfl_xor(m, sh, 64), qo = __shfl_xor(m2, sh, 64);
      const float d = m - mo;
      // the same operand order in both lanes of a pair: lower lane first
      const bool lo = (lane & sh) == 0;
      const float ma = lo ? m : mo, mb = lo ? mo : m, qa = lo ? m2 : qo, qb = lo ? qo : m2;
      m2 = qa + qb + d * d * (0.5f * n);
      m = 0.5f * (ma + mb);
      n *= 2.f;
    }
    if (g == 0) r2[w * BM + 16 * i + q] = make_float2(m, m2);
  }
  lds_barrier();
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = 16 * i + q;
    float2 v[NW];
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v[ww] = r2[ww * BM + row];
    float n = 32.f;
#pragma unroll
    for (int span = 1; span < NW; span *= 2) {
#pragma unroll
      for (int a = 0; a < NW; a += 2 * span) {
        const float d = v[a].x - v[a + span].x;
        v[a].y = v[a].y + v[a + span].y + d * d * (0.5f * n);
        v[a].x = 0.5f * (v[a].x + v[a + span].x);
      }
      n *= 2.f;
    }
    mean[i] = v[0].x;
    rstd[i] = rsqrtf(v[0].y * (1.f / (32 * NW)) + eps);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < NV; ++e) x[i][e] = (x[i][e] - mean[i]) * rstd[i] * gg[e] + bb[e];
}

__device__ __forceinline__ void load_bias(const float* __restrict__ b, int cb, float (&v)[NV]) {
#pragma unroll
  for (int e = 0; e < NV; e += 4) {
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(b + cb + e);
#pragma unroll
    for (int t = 0; t < 4; ++t) v[e + t] = b4[t];
  }
}

__device__ __forceinline__ void load_row_vals(const bf16_t* p, float (&v)[NV]) {
  const bf16x8 c = gld16(p);
#pragma unroll
  for (int t = 0; t < 8; ++t) v[t] = (float)c[t];
}

__device__ __forceinline__ void store_row_vals(bf16_t* p, const float (&v)[NV]) {
  bf16x8 c;
#pragma unroll
  for (int t = 0; t < 8; ++t) c[t] = (bf16_t)v[t];
  *reinterpret_cast<bf16x8*>(p) = c;
}

// the lane's 8 channels (chunk cb/8) of row m as bf16 into an LDS image with KH columns
template <int KH>
__device__ __forceinline__ void put_lds_row(char* lds, int m, int cb, const float (&v)[NV]) {
  bf16x8 c;
#pragma unroll
  for (int t = 0; t < 8; ++t) c[t] = (bf16_t)v[t];
  sts16(lds, sw<KH>(m, cb >> 3), c);
}


// ------------------------------------------------------------------ out_proj + res + LN
template <int C, int BM, bool POST>
__global__ __launch_bounds__(C * 2) void linear_ln_kernel(bf16_t* out, dp_rowmap om, const bf16_t* x, dp_rowmap xm,
                                                          const bf16_t* __restrict__ w, const float* __restrict__ b,
                                                          const bf16_t* res, dp_rowmap rm,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, int rows,
                                                          const bf16_t* post, dp_rowmap pm, int post_group,
                                                          int post_skip) {
  constexpr int NW = C / 32, NTH = 64 * NW, TM = BM / 16, K = C;
  __shared__ __attribute__((aligned(16))) char smem[BM * K * 2 + NW * BM * 4];
  char* xl = smem;
  float* red = reinterpret_cast<float*>(smem + BM * K * 2);
  const int row0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int wbase = wv * 32, cb = wbase + g * NV;
  // every global load of the block goes out before the first wait: rows, weights, residual
  Stage<K, BM, NTH, false> st;
  st.load(x, xm, nullptr, xm, row0, rows);
  const bf16_t* wb = frag_base(w, wv, K / 32);
  WPipe p;
  pipe_start(p, wb);
  bf16x8 rv[TM], pv[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = min(row0 + 16 * i + q, rows - 1);
    rv[i] = gld16(res + rowmap_off(rm, r) + cb);
    if (POST) {
      const int grp = r / post_group, wi = r - grp * post_group;
      pv[i] = gld16(post + rowmap_off(pm, (int64_t)grp * (post_group - post_skip) + max(wi - post_skip, 0)) + cb);
    }
  }
  float bias[NV], gg[NV], bb[NV];
  load_bias(b, cb, bias);
  load_bias(gamma, cb, gg);
  load_bias(beta, cb, bb);
  st.store(xl, row0, rows);
  lds_barrier();
  f32x4 acc[TM][TN];
  zero_acc<TM>(acc);
  wave_gemm<K, TM>(acc, xl, wb, p, wb);
  float v[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float a[NV];
    lane_vals<TM>(acc, i, a);
#pragma unroll
    for (int e = 0; e < NV; ++e) v[i][e] = a[e] + bias[e] + (float)rv[i][e];
  }
  layernorm_rows<TM, NW>(v, gg, bb, eps, red);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = row0 + 16 * i + q;
    if (r >= rows) continue;
    if (POST) {
      const int grp = r / post_group, wi = r - grp * post_group;
      if (wi >= post_skip) {
#pragma unroll
        for (int e = 0; e < NV; ++e) v[i][e] += (float)pv[i][e];
      }
    }
    store_row_vals(out + rowmap_off(om, r) + cb, v[i]);
  }
}

// ------------------------------------------------------------------ enc_output + LN + class max
// The two-stage selection head (transformer.py:1232-1240) in one pass over memory's rows:
// output_memory = LayerNorm(enc_output(memory)) with the border/invalid rows replaced by
// masked_row (= LN(enc_output bias), the reference's masked_fill(0) then Linear), and the
// class-score max over the STORED (bf16) row, as dp_layernorm_classmax computes it. The
// enc_output GEMM runs as linear_ln_kernel's; the class dot products are reduced over the
// lane groups by shuffles and over the waves through LDS.
template <int C, int BM>
__global__ __launch_bounds__(C * 2) void linear_ln_cls_kernel(bf16_t* out, const bf16_t* x,
                                                              const bf16_t* __restrict__ w, const float* __restrict__ b,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps, int rows,
                                                              const uint8_t* __restrict__ mask, int mask_period,
                                                              const float* __restrict__ masked_row,
                                                              const float* __restrict__ cw,
                                                              const float* __restrict__ cbias, int ncls,
                                                              float* __restrict__ cls_out) {
  constexpr int NW = C / 32, NTH = 64 * NW, TM = BM / 16, K = C, MAXCLS = 4;
  __shared__ __attribute__((aligned(16))) char smem[BM * K * 2 + MAXCLS * NW * BM * 4];
  char* xl = smem;
  float* red = reinterpret_cast<float*>(smem + BM * K * 2);
  const int row0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int wbase = wv * 32, cb = wbase + g * NV;
  const dp_rowmap xm{0, 1, K, 0};   // contiguous rows
  Stage<K, BM, NTH, false> st;
  st.load(x, xm, nullptr, xm, row0, rows);
  const bf16_t* wb = frag_base(w, wv, K / 32);
  WPipe p;
  pipe_start(p, wb);
  float bias[NV], gg[NV], bb[NV];
  load_bias(b, cb, bias);
  load_bias(gamma, cb, gg);
  load_bias(beta, cb, bb);
  st.store(xl, row0, rows);
  lds_barrier();
  f32x4 acc[TM][TN];
  zero_acc<TM>(acc);
  wave_gemm<K, TM>(acc, xl, wb, p, wb);
  float v[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float a[NV];
    lane_vals<TM>(acc, i, a);
#pragma unroll
    for (int e = 0; e < NV; ++e) v[i][e] = a[e] + bias[e];
  }
  layernorm_rows<TM, NW>(v, gg, bb, eps, red);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = row0 + 16 * i + q;
    if (mask && r < rows && mask[(unsigned)r % (unsigned)mask_period]) {
#pragma unroll
      for (int e = 0; e < NV; ++e) v[i][e] = masked_row[cb + e];
    }
#pragma unroll
    for (int e = 0; e < NV; ++e) v[i][e] = (float)(bf16_t)v[i][e];   // the stored value
    if (r < rows) store_row_vals(out + (int64_t)r * K + cb, v[i]);
  }
  // class scores: per-wave partial dot products of the lane's 8 channels, lane groups by
  // shuffles, waves through LDS
  for (int j = 0; j < ncls; ++j) {
    float cwv[NV];
    load_bias(cw + j * K, cb, cwv);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float sj = 0.f;
#pragma unroll
      for (int e = 0; e < NV; ++e) sj = fmaf(v[i][e], cwv[e], sj);
      sj += __shfl_xor(sj, 16, 64);
      sj += __shfl_xor(sj, 32, 64);
      if (g == 0) red[(j * NW + wv) * BM + 16 * i + q] = sj;
    }
  }
  lds_barrier();
  for (int t = threadIdx.x; t < BM; t += NTH) {
    const int r = row0 + t;
    if (r >= rows) continue;
    float best = -INFINITY;
    for (int j = 0; j < ncls; ++j) {
      float sj = cbias[j];
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sj += red[(j * NW + ww) * BM + t];
      best = fmaxf(best, sj);
    }
    cls_out[r] = best;
  }
}

// ------------------------------------------------------------------ fused MHA + out_proj + res + LN
// nn.MultiheadAttention(q = k = v = x) + residual + LayerNorm of the decoder layer's two token
// attentions (transformer.py:403-422): within-instance (the T tokens of a query, rows
// contiguous) and across-instance (the nq queries of one token slot, rows T apart). One block
// = GB sequences of SEQ tokens, block row m = g * SEQ + t (padded to TM tiles of 16), C = 256,
// 8 heads of 32, 8 waves: wave h = head h.
//   1. X rows -> LDS; wave h runs its head's Q, K, V projections (3 x [R x 32] GEMMs off the
//      LDS image, weight fragments from L2): Q and K stay in registers as bf16 MFMA fragments
//      (the projection's C layout -- 8 contiguous channels of one row per lane -- IS the A/B
//      operand layout for K = dh = 32), V goes to the wave's own LDS slice (row-major).
//   2. per 16-query tile: S^T = K Q^T over the key tiles of its sequences (one MFMA each,
//      other sequences masked), softmax over registers + 2 xor-shuffles, O^T = V^T P^T with P
//      from registers and V^T by ds_read_b64_tr_b16 (attention.hip's attn_long scheme); O (bf16)
//      overwrites the X image in LDS (all waves are past their projections).
//   3. out_proj off the O image, + bias + residual (x rows re-read, L2) -> LayerNorm (+ the
//      across attention's pos re-add on keypoint rows) -> out.
// HBM: x read once (+ the residual re-read from L2), out written once: the qkv (3C) and
// attention-output (C) round trips of the unfused path are gone.
#ifdef DP_MHA_TIMING
// A/B builds only: wall-clock stamps of each block's wave 0 at the kernel's phase boundaries
constexpr int MHA_DBG_BLOCKS = 8192, MHA_DBG_N = 12;
__device__ long long g_mha_dbg[MHA_DBG_BLOCKS * MHA_DBG_N];
#define MHA_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < MHA_DBG_BLOCKS) g_mha_dbg[blockIdx.x * MHA_DBG_N + (k)] = (long long)wall_clock64()
#else
#define MHA_STAMP(k)
#endif

template <int SEQ, int GB, bool POST, int DHP, bool NEXT, int MODE>
__global__ __launch_bounds__(512, 2) void mha_ln_kernel(bf16_t* out, dp_rowmap om, const bf16_t* x, dp_rowmap xm,
                                                     int n_inner, int64_t so, int64_t si, int64_t st, int nseq,
                                                     const bf16_t* __restrict__ wqkv, const float* __restrict__ bqkv,
                                                     const bf16_t* __restrict__ wo, const float* __restrict__ bo,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, float scale, const bf16_t* post, dp_rowmap pm,
                                                     int post_group, int post_skip, bf16_t* __restrict__ nout,
                                                     int nout_ld, const bf16_t* __restrict__ wn,
                                                     const float* __restrict__ bn, int nn) {
  constexpr int C = 256, NW = 8, NTH = 512, DH = 32;
  constexpr int RR = SEQ * GB, TM = (RR + 15) / 16, R = 16 * TM;
  // LDS: the waves' V slices [NW][R][DHP] (DHP: row pitch in elements, 40 or 48 keep the
  // transposed reads conflict-free), the X / O image [R][C], the LayerNorm partials. The PV
  // MFMA of a last odd key tile reads 16 rows past a slice: the next wave's slice, or for
  // wave 7 the image's first rows -- finite values under zero probabilities either way.
  // R = 64 / DHP = 40 is 76 KB: two blocks per CU (WPE = 4 waves per SIMD).
  typedef short s4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) char smem[NW * R * DHP * 2 + R * C * 2 + NW * R * 8 + R * 4];
  char* xl = smem + NW * R * DHP * 2;
  int* rows_l = reinterpret_cast<int*>(xl + R * C * 2 + NW * R * 8);   // row_of(m), for the epilogue
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  bf16_t* V = reinterpret_cast<bf16_t*>(smem) + wv * R * DHP;
  float* red = reinterpret_cast<float*>(xl + R * C * 2);
  MHA_STAMP(11);
  const int sq0 = blockIdx.x * GB;
  // block row m -> token row (o * so + ii * si + t * st < 2^31, checked by the launcher); -1
  // past the last sequence / padding
  auto row_of = [&](int m) -> int {
    if (m >= RR) return -1;
    const int gq = m / SEQ, t = m - gq * SEQ, sq = sq0 + gq;
    if (sq >= nseq) return -1;
    const int o = (int)((unsigned)sq / (unsigned)n_inner), ii = sq - o * n_inner;
    return o * (int)so + ii * (int)si + t * (int)st;
  };
  const bf16_t* wq = frag_base(wqkv, wv, C / 32);
  const bf16_t* wk = frag_base(wqkv, NW + wv, C / 32);
  const bf16_t* wvv = frag_base(wqkv, 2 * NW + wv, C / 32);
  const bf16_t* wob = frag_base(wo, wv, C / 32);
  // MODE 0: the V, K, Q projections as three GEMMs (32 output channels each) through one
  // weight ring; 1: one GEMM of 96 output channels (each X fragment read from LDS feeds six
  // MFMAs instead of two)
  constexpr bool FUSED = MODE == 1;
  constexpr int MD = D;
  constexpr bool XDB = true;
  constexpr int QD = 2;   // FUSED: the projection's ring depth (k-steps of 3 x TN fragments)
  WPipeT<MD> p;
  bf16x8 pf[FUSED ? QD : 1][3][TN];
  auto ring_start = [&]() __attribute__((always_inline)) {
    if constexpr (FUSED) {
#pragma unroll
      for (int s = 0; s < QD; ++s)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          pf[s][0][j] = gld16(wvv + (s * TN + j) * 512);
          pf[s][1][j] = gld16(wk + (s * TN + j) * 512);
          pf[s][2][j] = gld16(wq + (s * TN + j) * 512);
        }
    } else {
      pipe_start(p, wvv);
    }
  };
  ring_start();
  // ---- X rows -> registers -> LDS (zero rows past the block's tokens)
  constexpr int CH = C / 8, PER = R * CH / NTH;
  bf16x8 xv[PER];
  auto load_x = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int e = threadIdx.x + NTH * t;
      const int m = e / CH, c = e - m * CH;
      const int r = row_of(m);
      xv[t] = r >= 0 ? gld16(x + rowmap_off(xm, r) + c * 8) : bf16x8{};
    }
  };
  load_x();
  const int cb = g * NV;   // the lane's 8 contiguous channels within a 32-channel block
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int e = threadIdx.x + NTH * t;
    const int m = e / CH, c = e - m * CH;
    sts16(xl, sw<C>(m, c), xv[t]);
  }
  if (threadIdx.x < R) rows_l[threadIdx.x] = row_of(threadIdx.x);
  lds_barrier();
  MHA_STAMP(0);

  // ---- 1. this head's projections
  bf16x8 qf[TM], kf[TM];
  f32x4 acc[TM][TN];
  // + bias (channels 32 wv + cb .. of projection `part`), bf16: the MFMA fragment of row 16i + q
  auto frag_of = [&](int i, int part) __attribute__((always_inline)) {
    float b[NV];
    load_bias(bqkv, part * C + 32 * wv + cb, b);
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) f[4 * j + r] = (bf16_t)(acc[i][j][r] + b[4 * j + r]);
    return f;
  };
  if constexpr (FUSED) {
    f32x4 a3[3][TM][TN];
#pragma unroll
    for (int t = 0; t < 3; ++t) zero_acc<TM>(a3[t]);
    constexpr int NS = C / 32;
    const bf16_t* wp3[3] = {wvv, wk, wq};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      bf16x8 w[3][TN];
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int j = 0; j < TN; ++j) w[t][j] = pf[s % QD][t][j];
      if (s + QD < NS) {
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int j = 0; j < TN; ++j) pf[s % QD][t][j] = gld16(wp3[t] + ((s + QD) * TN + j) * 512);
      }
      bf16x8 xf[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) xf[i] = lds16(xl, sw<C>(16 * i + q, 4 * s + g));
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            a3[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][j], xf[i], a3[t][i][j], 0, 0, 0);
    }
    pipe_start(p, wob);   // the out_proj's first k-steps, in flight across the attention
    MHA_STAMP(1);
    auto frag3 = [&](int t, int i, int part) __attribute__((always_inline)) {
      float b[NV];
      load_bias(bqkv, part * C + 32 * wv + cb, b);
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) f[4 * j + r] = (bf16_t)(a3[t][i][j][r] + b[4 * j + r]);
      return f;
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      *reinterpret_cast<bf16x8*>(V + (16 * i + q) * DHP + cb) = frag3(0, i, 2);
      kf[i] = frag3(1, i, 1);
      qf[i] = frag3(2, i, 0);
    }
    MHA_STAMP(2);
    MHA_STAMP(3);
  } else {
    // V first (to LDS), then K, then Q: the fewest fragments live across a GEMM
    zero_acc<TM>(acc);
    wave_gemm<C, TM, MD, XDB>(acc, xl, wvv, p, wk);
    MHA_STAMP(1);
#pragma unroll
    for (int i = 0; i < TM; ++i) *reinterpret_cast<bf16x8*>(V + (16 * i + q) * DHP + cb) = frag_of(i, 2);
    zero_acc<TM>(acc);
    wave_gemm<C, TM, MD, XDB>(acc, xl, wk, p, wq);
    MHA_STAMP(2);
#pragma unroll
    for (int i = 0; i < TM; ++i) kf[i] = frag_of(i, 1);
    zero_acc<TM>(acc);
    wave_gemm<C, TM, MD, XDB>(acc, xl, wq, p, wob);
    MHA_STAMP(3);
#pragma unroll
    for (int i = 0; i < TM; ++i) qf[i] = frag_of(i, 0);
  }
  lds_barrier();   // every wave is past its projections: the X image may be overwritten by O
  MHA_STAMP(4);

  // ---- 2. attention, one 16-query tile at a time
  const int q4 = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    // key tiles of the sequences this query tile touches (compile time)
    const int glo = (16 * i) / SEQ, ghi = min((16 * i + 15) / SEQ, GB - 1);
    const int klo = (glo * SEQ) / 16, khi = ((ghi + 1) * SEQ - 1) / 16;
    constexpr int NKMAX = (SEQ + 15) / 16 + 2;
    f32x4 sv[NKMAX];
    const int qm = 16 * i + q;          // this lane's query row
    const int qg = qm / SEQ;
    float mx = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < NKMAX; ++kk) {
      const int kt = klo + kk;
      if (kt > khi) break;
      sv[kk] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt], qf[i], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int km = 16 * kt + 4 * g + r;   // key row of S^T element r
        const float v = (km < RR && km / SEQ == qg) ? sv[kk][r] * scale : -INFINITY;
        sv[kk][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int kk = 0; kk < NKMAX; ++kk) {
      if (klo + kk > khi) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(sv[kk][r] - mx);
        sv[kk][r] = e;
        sum += e;
      }
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    f32x4 oacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < NKMAX; kk += 2) {
      const int kt = klo + kk;
      if (kt > khi) break;
      const bool two = kt + 1 <= khi;
      bf16x8 pf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = (bf16_t)sv[kk][r];
        pf[4 + r] = (bf16_t)(two ? sv[kk + 1][r] : 0.f);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const bf16_t* a0 = V + (16 * kt + 4 * g + q4) * DHP + 16 * d + 4 * p4;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0 + 16 * DHP));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 vfr = *reinterpret_cast<const bf16x8*>(tmp);
        oacc[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfr, pf, oacc[d], 0, 0, 0);
      }
    }
    // O^T[16d + 4g + r][query q] -> O image row qm, channels 32 wv + 16 d + 4 g .. +3
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16_t)(oacc[d][r] * inv);
      const int ch = 32 * wv + 16 * d + 4 * g;
      *reinterpret_cast<bf16x4*>(xl + sw<C>(qm, ch >> 3) + (ch & 7) * 2) = w;
    }
  }
  MHA_STAMP(5);
  // residual rows for the epilogue: in flight across the barrier and the out_proj GEMM (one
  // block per CU), or fetched after the GEMM (two blocks per CU: registers)
  bf16x8 rv[TM], pv[TM];
  float bias[NV], gg[NV], bb[NV];
  auto load_res = [&]() __attribute__((always_inline)) {
    const int ocb = 32 * wv + cb;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = max(rows_l[16 * i + q], 0);
      rv[i] = gld16(x + rowmap_off(xm, r) + ocb);
      if (POST) {
        const int grp = (int)((unsigned)r / (unsigned)post_group), wi = r - grp * post_group;
        pv[i] = gld16(post + rowmap_off(pm, grp * (post_group - post_skip) + max(wi - post_skip, 0)) + ocb);
      }
    }
  };
  if constexpr (XDB) load_res();
  lds_barrier();   // the O image is complete
  MHA_STAMP(6);

  // ---- 3. out_proj + bias + residual -> LayerNorm -> out
  zero_acc<TM>(acc);
  wave_gemm<C, TM, MD, XDB>(acc, xl, wob, p, wob);
  MHA_STAMP(7);
  if constexpr (!XDB) load_res();
  load_bias(bo, 32 * wv + cb, bias);
  load_bias(gamma, 32 * wv + cb, gg);
  load_bias(beta, 32 * wv + cb, bb);
  float v[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float a[NV];
    lane_vals<TM>(acc, i, a);
#pragma unroll
    for (int e = 0; e < NV; ++e) v[i][e] = a[e] + bias[e] + (float)rv[i][e];
  }
  layernorm_rows_1p<TM, NW>(v, gg, bb, eps, red);
  MHA_STAMP(8);
  const int ocb = 32 * wv + cb;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = rows_l[16 * i + q];
    if (r < 0) continue;
    if (POST) {
      const int wi = (int)((unsigned)r % (unsigned)post_group);
      if (wi >= post_skip) {
#pragma unroll
        for (int e = 0; e < NV; ++e) v[i][e] += (float)pv[i][e];
      }
    }
    store_row_vals(out + rowmap_off(om, r) + ocb, v[i]);
  }
  MHA_STAMP(9);
  if constexpr (NEXT) {
    // 4. the next Linear on the rows just stored (the across attention's output + pos is the
    //    MSDA query: its sampling-offset / attention-logit projection, ms_deform_attn.py:
    //    428-432), straight from registers: the stored bf16 rows -> the LDS image (every wave
    //    is past the out_proj GEMM: layernorm_rows' barriers), nn / 32 channel blocks over the
    //    waves, + bias, 16-byte stores.
#pragma unroll
    for (int i = 0; i < TM; ++i) put_lds_row<C>(xl, 16 * i + q, ocb, v[i]);
    lds_barrier();
    for (int nb = wv; nb < nn / 32; nb += NW) {
      const bf16_t* wnb = frag_base(wn, nb, C / 32);
      pipe_start(p, wnb);
      zero_acc<TM>(acc);
      wave_gemm<C, TM, MD, XDB>(acc, xl, wnb, p, wnb);
      float nbias[NV];
      load_bias(bn, 32 * nb + cb, nbias);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = rows_l[16 * i + q];
        if (r < 0) continue;
        float a[NV];
        lane_vals<TM>(acc, i, a);
#pragma unroll
        for (int e = 0; e < NV; ++e) a[e] += nbias[e];
        store_row_vals(nout + (int64_t)r * nout_ld + 32 * nb + cb, a);
      }
    }
  }
  MHA_STAMP(10);
}

// ------------------------------------------------------------------ Gate: Linear + sigmoid mix + LN
// xcat = [x1 | x2] (K = 2C); gate rows n < C -> g1, n >= C -> g2. Wave w computes g1 AND
// g2 of its 32 channels, so the mix sigmoid(g1) x1 + sigmoid(g2) x2 is lane-local.
template <int C, int BM>
__global__ __launch_bounds__(C * 2) void gate_ln_kernel(bf16_t* out, dp_rowmap om, const bf16_t* x, dp_rowmap xm,
                                                        const bf16_t* __restrict__ w, const float* __restrict__ b,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, int rows) {
  constexpr int NW = C / 32, NTH = 64 * NW, TM = BM / 16, K = 2 * C;
  __shared__ __attribute__((aligned(16))) char smem[BM * K * 2 + NW * BM * 4];
  char* xl = smem;
  float* red = reinterpret_cast<float*>(smem + BM * K * 2);
  const int row0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int wbase = wv * 32, cb = wbase + g * NV;
  Stage<K, BM, NTH, false> st;
  st.load(x, xm, nullptr, xm, row0, rows);
  const bf16_t* wb1 = frag_base(w, wv, K / 32);        // gate rows [32w, 32w+32): g1
  const bf16_t* wb2 = frag_base(w, NW + wv, K / 32);   // gate rows C + [32w, 32w+32): g2
  WPipe p;
  pipe_start(p, wb1);
  float b1[NV], b2[NV], gg[NV], bb[NV];
  load_bias(b, cb, b1);
  load_bias(b + C, cb, b2);
  load_bias(gamma, cb, gg);
  load_bias(beta, cb, bb);
  st.store(xl, row0, rows);
  lds_barrier();
  f32x4 a1[TM][TN], a2[TM][TN];
  zero_acc<TM>(a1);
  zero_acc<TM>(a2);
  wave_gemm<K, TM>(a1, xl, wb1, p, wb2);
  wave_gemm<K, TM>(a2, xl, wb2, p, wb2);
  float v[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = 16 * i + q;
    float g1[NV], g2[NV];
    lane_vals<TM>(a1, i, g1);
    lane_vals<TM>(a2, i, g2);
    const bf16x8 x1 = lds16(xl, sw<K>(m, cb >> 3));
    const bf16x8 x2 = lds16(xl, sw<K>(m, (C + cb) >> 3));
#pragma unroll
    for (int t = 0; t < NV; ++t)
      v[i][t] = sigmoidf_(g1[t] + b1[t]) * (float)x1[t] + sigmoidf_(g2[t] + b2[t]) * (float)x2[t];
  }
  layernorm_rows<TM, NW>(v, gg, bb, eps, red);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = row0 + 16 * i + q;
    if (r < rows) store_row_vals(out + rowmap_off(om, r) + cb, v[i]);
  }
}

// ------------------------------------------------------------------ FFN + residual + LN
// hidden in chunks of HC = min(256, C) columns, computed by the first HC/32 waves:
// H = relu(X W1[chunk]^T + b1) -> LDS (bf16); then every wave Y += H W2[:, chunk]^T.
// One weight ring runs through the whole chain W1[0] -> W2[0] -> W1[1] -> ... The block's
// own staged rows are the residual.
template <int C, int BM, int F>
__global__ __launch_bounds__(C * 2) void ffn_ln_kernel(bf16_t* out, dp_rowmap om, const bf16_t* x, dp_rowmap xm,
                                                       const bf16_t* __restrict__ w1, const float* __restrict__ b1,
                                                       const bf16_t* __restrict__ w2, const float* __restrict__ b2,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps, int rows) {
  constexpr int NW = C / 32, NTH = 64 * NW, TM = BM / 16;
  constexpr int HC = C < 256 ? C : 256, HW = HC / 32, NCH = F / HC;
  static_assert(F % HC == 0, "ffn hidden");
  __shared__ __attribute__((aligned(16))) char smem[BM * C * 2 + BM * HC * 2 + NW * BM * 4];
  char* xl = smem;
  char* hl = smem + BM * C * 2;
  float* red = reinterpret_cast<float*>(smem + BM * C * 2 + BM * HC * 2);
  const int row0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int wbase = wv * 32, cb = wbase + g * NV;
  const bool g1w = wv < HW;   // wave-uniform: this wave computes hidden columns
  Stage<C, BM, NTH, false> st;
  st.load(x, xm, nullptr, xm, row0, rows);
  // W1 [F][C]: this wave's hidden block of chunk h is nb = h*HW + wv (C/32 k-steps);
  // W2 [C][F]: output block nb = wv, chunk h covers k-steps [h*HC/32, (h+1)*HC/32)
  auto w1b = [&](int h) { return frag_base(w1, h * HW + (g1w ? wv : 0), C / 32); };
  auto w2b = [&](int h) { return frag_base(w2, wv, F / 32, h * (HC / 32)); };
  WPipe p;
  pipe_start(p, g1w ? w1b(0) : w2b(0));
  float bias[NV], gg[NV], bb[NV], bh[NV];
  load_bias(b2, cb, bias);
  load_bias(gamma, cb, gg);
  load_bias(beta, cb, bb);
  load_bias(b1, g1w ? cb : 0, bh);
  st.store(xl, row0, rows);
  lds_barrier();
  f32x4 acc[TM][TN];
  zero_acc<TM>(acc);
#pragma unroll 1
  for (int h = 0; h < NCH; ++h) {
    const int h0 = h * HC;
    float bn[NV];   // next chunk's hidden bias, in flight during this chunk
    load_bias(b1 + (h + 1 < NCH ? h0 + HC : 0), g1w ? cb : 0, bn);
    const bf16_t* c1 = w1b(h);
    const bf16_t* c2 = w2b(h);
    const bf16_t* n1 = h + 1 < NCH ? (g1w ? w1b(h + 1) : w2b(h + 1)) : c2;
    if (g1w) {
      f32x4 ah[TM][TN];
      zero_acc<TM>(ah);
      wave_gemm<C, TM>(ah, xl, c1, p, c2);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float hv[NV];
        lane_vals<TM>(ah, i, hv);
#pragma unroll
        for (int e = 0; e < NV; ++e) hv[e] = fmaxf(hv[e] + bh[e], 0.f);
        put_lds_row<HC>(hl, 16 * i + q, cb, hv);
      }
    }
    lds_barrier();
    wave_gemm<HC, TM>(acc, hl, c2, p, n1);
    lds_barrier();   // every wave done reading this chunk's H before the next one lands
#pragma unroll
    for (int e = 0; e < NV; ++e) bh[e] = bn[e];
  }
  float v[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = 16 * i + q;
    float a[NV];
    lane_vals<TM>(acc, i, a);
    const bf16x8 xr = lds16(xl, sw<C>(m, cb >> 3));
#pragma unroll
    for (int t = 0; t < NV; ++t) v[i][t] = a[t] + bias[t] + (float)xr[t];
  }
  layernorm_rows<TM, NW>(v, gg, bb, eps, red);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = row0 + 16 * i + q;
    if (r < rows) store_row_vals(out + rowmap_off(om, r) + cb, v[i]);
  }
}

// ------------------------------------------------------------------ query pos of the keypoint tokens
// row r = (query row qr = r / nkp, keypoint kp = r % nkp): sine embedding of ref[qr][1+kp]
// (cat(pos_y, pos_x), sin on even / cos on odd dims), MLP(C, C, C, 2) -> pos[r] (bf16) and
// tgt keypoint row r += pos (in place, the reference's with_pos_embed).
template <int C, int BM>
__global__ __launch_bounds__(C * 2) void query_pos_kernel(const float* __restrict__ ref, int rows, int nkp,
                                                          const float* __restrict__ dim_t,
                                                          const bf16_t* __restrict__ w0, const float* __restrict__ b0,
                                                          const bf16_t* __restrict__ w1, const float* __restrict__ b1,
                                                          bf16_t* pos, bf16_t* tgt, dp_rowmap tm) {
  constexpr int NW = C / 32, NTH = 64 * NW, TM = BM / 16, CH = C / 8, PER = BM * CH / NTH;
  __shared__ __attribute__((aligned(16))) char smem[2 * BM * C * 2];
  char* xl = smem;
  char* hl = smem + BM * C * 2;
  const int row0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int wbase = wv * 32, cb = wbase + g * NV;
  const bf16_t* wb0 = frag_base(w0, wv, C / 32);
  const bf16_t* wb1 = frag_base(w1, wv, C / 32);
  WPipe p;
  pipe_start(p, wb0);
  bf16x8 tv[TM];   // the tgt keypoint rows this lane updates at the end
#pragma unroll
  for (int i = 0; i < TM; ++i) tv[i] = gld16(tgt + rowmap_off(tm, min(row0 + 16 * i + q, rows - 1)) + cb);
  float bias0[NV], bias1[NV];
  load_bias(b0, cb, bias0);
  load_bias(b1, cb, bias1);
  constexpr int half = C / 2;
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int e = threadIdx.x + NTH * t;
    const int m = e / CH, c0 = (e - m * CH) * 8;
    const int r = min(row0 + m, rows - 1);
    const int qr = r / nkp, kp = r - qr * nkp;
    const float* pp = ref + ((int64_t)qr * (nkp + 1) + 1 + kp) * 2;
    const bool ylow = c0 < half;
    const int i0 = ylow ? c0 : c0 - half;
    const float coord = (ylow ? pp[1] : pp[0]) * 6.283185307179586f;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = coord * __builtin_amdgcn_rcpf(dim_t[i0 + j]);   // 1 ulp; bf16 output
      o[j] = (bf16_t)(((i0 + j) & 1) ? __cosf(a) : __sinf(a));
    }
    sts16(xl, sw<C>(m, c0 >> 3), o);
  }
  lds_barrier();
  f32x4 acc[TM][TN];
  zero_acc<TM>(acc);
  wave_gemm<C, TM>(acc, xl, wb0, p, wb1);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float hv[NV];
    lane_vals<TM>(acc, i, hv);
#pragma unroll
    for (int e = 0; e < NV; ++e) hv[e] = fmaxf(hv[e] + bias0[e], 0.f);
    put_lds_row<C>(hl, 16 * i + q, cb, hv);
  }
  lds_barrier();
  zero_acc<TM>(acc);
  wave_gemm<C, TM>(acc, hl, wb1, p, wb1);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = row0 + 16 * i + q;
    if (r >= rows) continue;
    float pv[NV], t2[NV];
    lane_vals<TM>(acc, i, pv);
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      pv[e] = (float)(bf16_t)(pv[e] + bias1[e]);   // pos as stored
      t2[e] = (float)tv[i][e] + pv[e];
    }
    store_row_vals(pos + (int64_t)r * C + cb, pv);
    store_row_vals(tgt + rowmap_off(tm, r) + cb, t2);
  }
}

// ------------------------------------------------------------------ pose head MLP(C, C, nout, 3)
// x (+ x2) -> relu(W0) -> relu(W1) -> W2 (+ b2) (+ prev) -> out f32 [rows][nout]. The last
// layer's nout (66) columns are computed by the first ceil(nout/32) waves; columns past
// nout use clamped weight rows and are never stored.
template <int C, int BM, bool ADD, bool PREV>
__global__ __launch_bounds__(C * 2) void pose_mlp_kernel(const bf16_t* x, dp_rowmap xm, const bf16_t* x2,
                                                         dp_rowmap x2m, int rows, const bf16_t* __restrict__ w0,
                                                         const float* __restrict__ b0, const bf16_t* __restrict__ w1,
                                                         const float* __restrict__ b1, const bf16_t* __restrict__ w2,
                                                         const float* __restrict__ b2, int nout,
                                                         const float* __restrict__ prev, float* __restrict__ out) {
  constexpr int NW = C / 32, NTH = 64 * NW, TM = BM / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * BM * C * 2];
  char* xl = smem;
  char* hl = smem + BM * C * 2;
  const int row0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int wbase = wv * 32, cb = wbase + g * NV;
  Stage<C, BM, NTH, ADD> st;
  st.load(x, xm, x2, x2m, row0, rows);
  const bf16_t* wb0 = frag_base(w0, wv, C / 32);
  const bf16_t* wb1 = frag_base(w1, wv, C / 32);
  // w2 is packed with its rows padded to a multiple of 32: waves past nout read block 0
  const bf16_t* wb2 = frag_base(w2, wbase < nout ? wv : 0, C / 32);
  WPipe p;
  pipe_start(p, wb0);
  float bias0[NV], bias1[NV], bias2[NV];
  load_bias(b0, cb, bias0);
  load_bias(b1, cb, bias1);
#pragma unroll
  for (int e = 0; e < NV; ++e) bias2[e] = b2[min(cb + e, nout - 1)];
  st.store(xl, row0, rows);
  lds_barrier();
  f32x4 acc[TM][TN];
  zero_acc<TM>(acc);
  wave_gemm<C, TM>(acc, xl, wb0, p, wb1);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float hv[NV];
    lane_vals<TM>(acc, i, hv);
#pragma unroll
    for (int e = 0; e < NV; ++e) hv[e] = fmaxf(hv[e] + bias0[e], 0.f);
    put_lds_row<C>(hl, 16 * i + q, cb, hv);
  }
  lds_barrier();
  zero_acc<TM>(acc);
  wave_gemm<C, TM>(acc, hl, wb1, p, wb2);
  lds_barrier();   // every wave done reading xl (GEMM 0) before H2 overwrites it
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float hv[NV];
    lane_vals<TM>(acc, i, hv);
#pragma unroll
    for (int e = 0; e < NV; ++e) hv[e] = fmaxf(hv[e] + bias1[e], 0.f);
    put_lds_row<C>(xl, 16 * i + q, cb, hv);
  }
  lds_barrier();
  if (wbase >= nout) return;   // wave-uniform: no barrier after this point
  // the previous corners of the lane's rows, in flight during the last GEMM
  float pr[TM][NV];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < NV; ++e)
      pr[i][e] = PREV ? prev[(int64_t)min(row0 + 16 * i + q, rows - 1) * nout + min(cb + e, nout - 1)] : 0.f;
  zero_acc<TM>(acc);
  wave_gemm<C, TM>(acc, xl, wb2, p, wb2);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = row0 + 16 * i + q;
    if (r >= rows) continue;
    float v[NV];
    lane_vals<TM>(acc, i, v);
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      const int n = cb + e;
      if (n < nout) out[(int64_t)r * nout + n] = v[e] + bias2[e] + pr[i][e];
    }
  }
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
bool map16(const dp_rowmap& m) { return m.base % 8 == 0 && m.stride_g % 8 == 0 && m.stride_r % 8 == 0 && m.group > 0; }

// Rows per block: every kernel here runs one block per CU (LDS / registers), so a launch
// takes ceil(blocks / CUs) rounds of equal length; pick the row tile with the least total
// rows x rounds (ties: the larger tile, fewer weight re-reads). DETRPOSE_DEC_BM overrides.
template <typename K>
int blocks_per_cu(K kern, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kern), threads, 0) !=
          hipSuccess ||
      n < 1)
    n = 1;
  return n;
}

// Rows per block: the candidate whose launch runs the fewest row-rounds, a round being one
// block per resident slot (occ = blocks per CU of that instantiation, by registers and LDS:
// a 64-row block that fits twice per CU overlaps its load / GEMM / epilogue phases with the
// other's).
int pick_bm(int rows, int c, int max_bm = 128, int occ128 = 1, int occ96 = 1, int occ64 = 1) {
  static const int forced = [] {
    const char* e = getenv("DETRPOSE_DEC_BM");
    return e ? atoi(e) : 0;
  }();
  if (c != 256) return 64;
  if ((forced == 64 || forced == 96 || forced == 128) && forced <= max_bm) return forced;
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess)
    cus = 256;
  int best = 64;
  int64_t best_cost = INT64_MAX;
  for (int bm : {128, 96, 64}) {
    if (bm > max_bm) continue;
    const int64_t blocks = (rows + bm - 1) / bm;
    const int64_t slots = (int64_t)cus * (bm == 128 ? occ128 : bm == 96 ? occ96 : occ64);
    const int64_t cost = (blocks + slots - 1) / slots * bm;
    if (cost < best_cost) best_cost = cost, best = bm;
  }
  return best;
}

}  // namespace

// Instantiation table: C in {128, 256, 384}; BM in {64, 96, 128} for C = 256, 64 otherwise.
#define DP_FOR_BM64(C_, X) \
  if (c == C_ && bm == 64) X(C_, 64);
#define DP_FOR_BM256(X)                \
  if (c == 256 && bm == 64) X(256, 64);  \
  if (c == 256 && bm == 96) X(256, 96);  \
  if (c == 256 && bm == 128) X(256, 128);
#define DP_FOR_BM(X) DP_FOR_BM64(128, X) DP_FOR_BM256(X) DP_FOR_BM64(384, X)

extern "C" int dp_linear_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, int32_t k, const void* w,
                                   const float* b, const void* res, dp_rowmap rm, const float* gamma,
                                   const float* beta, float eps, int32_t rows, int32_t c, const void* post,
                                   dp_rowmap pm, int32_t post_group, int32_t post_skip, void* stream) {
  DP_REQUIRE(out && x && w && b && res && gamma && beta && rows > 0, "dp_linear_layernorm: bad args");
  DP_REQUIRE(al16(out) && al16(x) && al16(w) && al16(res) && map16(om) && map16(xm) && map16(rm) &&
                 (!post || (al16(post) && map16(pm) && post_group > post_skip)),
             "dp_linear_layernorm: rows must be 16-byte aligned");
  DP_REQUIRE(k == c, "dp_linear_layernorm: k=%d != c=%d (out_proj only)", k, c);
  hipStream_t s = as_stream(stream);
  static const int ol1[3] = {blocks_per_cu(linear_ln_kernel<256, 128, true>, 512),
                             blocks_per_cu(linear_ln_kernel<256, 96, true>, 512),
                             blocks_per_cu(linear_ln_kernel<256, 64, true>, 512)};
  static const int ol0[3] = {blocks_per_cu(linear_ln_kernel<256, 128, false>, 512),
                             blocks_per_cu(linear_ln_kernel<256, 96, false>, 512),
                             blocks_per_cu(linear_ln_kernel<256, 64, false>, 512)};
  const int* ol = post ? ol1 : ol0;
  const int bm = pick_bm(rows, c, 128, ol[0], ol[1], ol[2]);
  dim3 grid((rows + bm - 1) / bm);
#define DP_LLN(C_, BM_)                                                                                            \
  do {                                                                                                             \
    if (post)                                                                                                      \
      hipLaunchKernelGGL((linear_ln_kernel<C_, BM_, true>), grid, dim3(2 * C_), 0, s, (bf16_t*)out, om,              \
                         (const bf16_t*)x, xm, (const bf16_t*)w, b, (const bf16_t*)res, rm, gamma, beta, eps, rows,    \
                         (const bf16_t*)post, pm, post_group, post_skip);                                           \
    else                                                                                                           \
      hipLaunchKernelGGL((linear_ln_kernel<C_, BM_, false>), grid, dim3(2 * C_), 0, s, (bf16_t*)out, om,             \
                         (const bf16_t*)x, xm, (const bf16_t*)w, b, (const bf16_t*)res, rm, gamma, beta, eps, rows,    \
                         (const bf16_t*)nullptr, pm, 1, 0);                                                         \
    return dp_check_launch("dp_linear_layernorm");                                                                 \
  } while (0)
  DP_FOR_BM(DP_LLN)
#undef DP_LLN
  dp_set_error("dp_linear_layernorm: c=%d unsupported (128/256/384)", c);
  return DP_EINVAL;
}

extern "C" int dp_gate_linear_layernorm(void* out, dp_rowmap om, const void* xcat, dp_rowmap xm, const void* w,
                                        const float* b, const float* gamma, const float* beta, float eps,
                                        int32_t rows, int32_t c, void* stream) {
  DP_REQUIRE(out && xcat && w && b && gamma && beta && rows > 0, "dp_gate_linear_layernorm: bad args");
  DP_REQUIRE(al16(out) && al16(xcat) && al16(w) && map16(om) && map16(xm),
             "dp_gate_linear_layernorm: rows must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int bm = pick_bm(rows, c, 64);   // two accumulator sets: larger row tiles spill
  dim3 grid((rows + bm - 1) / bm);
#define DP_GLN(C_, BM_)                                                                                           \
  do {                                                                                                            \
    hipLaunchKernelGGL((gate_ln_kernel<C_, BM_>), grid, dim3(2 * C_), 0, s, (bf16_t*)out, om, (const bf16_t*)xcat, \
                       xm, (const bf16_t*)w, b, gamma, beta, eps, rows);                                           \
    return dp_check_launch("dp_gate_linear_layernorm");                                                           \
  } while (0)
  DP_FOR_BM64(128, DP_GLN) DP_FOR_BM64(256, DP_GLN) DP_FOR_BM64(384, DP_GLN)
#undef DP_GLN
  dp_set_error("dp_gate_linear_layernorm: c=%d unsupported (128/256/384)", c);
  return DP_EINVAL;
}

extern "C" int dp_ffn_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, const void* w1, const float* b1,
                                int32_t f, const void* w2, const float* b2, const float* gamma, const float* beta,
                                float eps, int32_t rows, int32_t c, void* stream) {
  DP_REQUIRE(out && x && w1 && b1 && w2 && b2 && gamma && beta && rows > 0, "dp_ffn_layernorm: bad args");
  DP_REQUIRE(al16(out) && al16(x) && al16(w1) && al16(w2) && map16(om) && map16(xm),
             "dp_ffn_layernorm: rows must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int bm = pick_bm(rows, c, 64);   // larger row tiles spill
  dim3 grid((rows + bm - 1) / bm);
#define DP_FLN(C_, BM_, F_)                                                                                        \
  do {                                                                                                             \
    hipLaunchKernelGGL((ffn_ln_kernel<C_, BM_, F_>), grid, dim3(2 * C_), 0, s, (bf16_t*)out, om, (const bf16_t*)x,   \
                       xm, (const bf16_t*)w1, b1, (const bf16_t*)w2, b2, gamma, beta, eps, rows);                  \
    return dp_check_launch("dp_ffn_layernorm");                                                                    \
  } while (0)
#define DP_FLN_N(C_, BM_) if (f == 512) DP_FLN(C_, BM_, 512)
#define DP_FLN_X(C_, BM_)                   \
  if (f == 1024) DP_FLN(C_, BM_, 1024);     \
  if (f == 2048) DP_FLN(C_, BM_, 2048)
  DP_FOR_BM64(128, DP_FLN_N)
  if (c == 256 && f == 1024 && bm == 64) DP_FLN(256, 64, 1024);
  if (c == 256 && f == 1024 && bm == 96) DP_FLN(256, 96, 1024);
  DP_FOR_BM64(384, DP_FLN_X)
#undef DP_FLN_N
#undef DP_FLN_X
#undef DP_FLN
  dp_set_error("dp_ffn_layernorm: c=%d, f=%d unsupported (128/512, 256/1024, 384/1024 or 2048)", c, f);
  return DP_EINVAL;
}

extern "C" int dp_query_pos(const float* ref, int32_t rows, int32_t nkp, const float* dim_t, const void* w0,
                            const float* b0, const void* w1, const float* b1, void* pos, void* tgt, dp_rowmap tm,
                            int32_t c, void* stream) {
  DP_REQUIRE(ref && dim_t && w0 && b0 && w1 && b1 && pos && tgt && rows > 0 && nkp > 0, "dp_query_pos: bad args");
  DP_REQUIRE(al16(pos) && al16(tgt) && al16(w0) && al16(w1) && map16(tm), "dp_query_pos: rows must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  static const int oq[3] = {blocks_per_cu(query_pos_kernel<256, 128>, 512), blocks_per_cu(query_pos_kernel<256, 96>, 512),
                            blocks_per_cu(query_pos_kernel<256, 64>, 512)};
  const int bm = pick_bm(rows, c, 128, oq[0], oq[1], oq[2]);
  dim3 grid((rows + bm - 1) / bm);
#define DP_QP(C_, BM_)                                                                                           \
  do {                                                                                                           \
    hipLaunchKernelGGL((query_pos_kernel<C_, BM_>), grid, dim3(2 * C_), 0, s, ref, rows, nkp, dim_t,              \
                       (const bf16_t*)w0, b0, (const bf16_t*)w1, b1, (bf16_t*)pos, (bf16_t*)tgt, tm);            \
    return dp_check_launch("dp_query_pos");                                                                      \
  } while (0)
  DP_FOR_BM(DP_QP)
#undef DP_QP
  dp_set_error("dp_query_pos: c=%d unsupported (128/256/384)", c);
  return DP_EINVAL;
}

extern "C" int dp_pose_mlp(const void* x, dp_rowmap xm, const void* x2, dp_rowmap x2m, int32_t rows, const void* w0,
                           const float* b0, const void* w1, const float* b1, const void* w2, const float* b2,
                           int32_t nout, const float* prev, float* out, int32_t c, void* stream) {
  DP_REQUIRE(x && w0 && b0 && w1 && b1 && w2 && b2 && out && rows > 0 && nout > 0 && nout <= c,
             "dp_pose_mlp: bad args (nout 1..c)");
  DP_REQUIRE((x2 != nullptr) == (prev != nullptr), "dp_pose_mlp: x2 and prev come together (layers > 0)");
  DP_REQUIRE(al16(x) && al16(w0) && al16(w1) && al16(w2) && map16(xm) && (!x2 || (al16(x2) && map16(x2m))),
             "dp_pose_mlp: rows must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  static const int op1[3] = {blocks_per_cu(pose_mlp_kernel<256, 128, true, true>, 512),
                             blocks_per_cu(pose_mlp_kernel<256, 96, true, true>, 512),
                             blocks_per_cu(pose_mlp_kernel<256, 64, true, true>, 512)};
  static const int op0[3] = {blocks_per_cu(pose_mlp_kernel<256, 128, false, false>, 512),
                             blocks_per_cu(pose_mlp_kernel<256, 96, false, false>, 512),
                             blocks_per_cu(pose_mlp_kernel<256, 64, false, false>, 512)};
  const int* op = x2 ? op1 : op0;
  const int bm = pick_bm(rows, c, 128, op[0], op[1], op[2]);
  dim3 grid((rows + bm - 1) / bm);
#define DP_PM(C_, BM_)                                                                                            \
  do {                                                                                                            \
    if (x2)                                                                                                       \
      hipLaunchKernelGGL((pose_mlp_kernel<C_, BM_, true, true>), grid, dim3(2 * C_), 0, s, (const bf16_t*)x, xm,    \
                         (const bf16_t*)x2, x2m, rows, (const bf16_t*)w0, b0, (const bf16_t*)w1, b1,                \
                         (const bf16_t*)w2, b2, nout, prev, out);                                                  \
    else                                                                                                          \
      hipLaunchKernelGGL((pose_mlp_kernel<C_, BM_, false, false>), grid, dim3(2 * C_), 0, s, (const bf16_t*)x, xm,  \
                         (const bf16_t*)x2, x2m, rows, (const bf16_t*)w0, b0, (const bf16_t*)w1, b1,                \
                         (const bf16_t*)w2, b2, nout, prev, out);                                                  \
    return dp_check_launch("dp_pose_mlp");                                                                        \
  } while (0)
  DP_FOR_BM(DP_PM)
#undef DP_PM
  dp_set_error("dp_pose_mlp: c=%d unsupported (128/256/384)", c);
  return DP_EINVAL;
}

#ifdef DP_MHA_TIMING
extern "C" int dp_debug_mha_stamps(long long* host, int32_t n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_mha_dbg), sizeof(long long) * std::min(n, MHA_DBG_BLOCKS * MHA_DBG_N)) ==
                 hipSuccess ? 0 : DP_EINVAL;
}
#endif

extern "C" int dp_mha_layernorm(void* out, dp_rowmap om, const void* x, dp_rowmap xm, int32_t n_outer,
                                int32_t n_inner, int64_t so, int64_t si, int64_t st, int32_t seqlen, const void* wqkv,
                                const float* bqkv, const void* wo, const float* bo, const float* gamma,
                                const float* beta, float eps, int32_t c, int32_t nhead, const void* post, dp_rowmap pm,
                                int32_t post_group, int32_t post_skip, void* next_out, int32_t next_ld,
                                const void* next_w, const float* next_b, int32_t next_n, void* stream) {
  DP_REQUIRE(out && x && wqkv && bqkv && wo && bo && gamma && beta && n_outer > 0 && n_inner > 0,
             "dp_mha_layernorm: bad args");
  DP_REQUIRE(al16(out) && al16(x) && al16(wqkv) && al16(wo) && map16(om) && map16(xm) &&
                 (!post || (al16(post) && map16(pm) && post_group > post_skip)),
             "dp_mha_layernorm: rows must be 16-byte aligned");
  DP_REQUIRE(c == 256 && nhead == 8, "dp_mha_layernorm: C = 256 with 8 heads only (got %d / %d)", c, nhead);
  DP_REQUIRE(!next_out || (next_w && next_b && next_n > 0 && next_n % 32 == 0 && next_ld % 8 == 0 && next_ld >= next_n &&
                           al16(next_out) && al16(next_w)),
             "dp_mha_layernorm: next linear needs n %% 32 == 0, 16-byte aligned rows");
  const int64_t nseq = (int64_t)n_outer * n_inner;
  DP_REQUIRE((int64_t)(n_outer - 1) * so + (int64_t)(n_inner - 1) * si + (int64_t)(seqlen - 1) * st < (1ll << 31),
             "dp_mha_layernorm: token rows exceed 2^31");
  hipStream_t s = as_stream(stream);
  const float scale = 1.f / sqrtf(32.f);
  // DETRPOSE_MHA_MODE: 1 (default) the fused V/K/Q projection; 0: three projection GEMMs
  static const int mode = [] {
    const char* e = getenv("DETRPOSE_MHA_MODE");
    return e ? atoi(e) : 1;
  }();
#define DP_MHA_L(SEQ_, GB_, POST_, NEXT_, DHP_, WPE_)                                                              \
  hipLaunchKernelGGL((mha_ln_kernel<SEQ_, GB_, POST_, DHP_, NEXT_, WPE_>), grid, dim3(512), 0, s, (bf16_t*)out, om, \
                     (const bf16_t*)x, xm, n_inner, so, si, st, (int)nseq, (const bf16_t*)wqkv, bqkv,              \
                     (const bf16_t*)wo, bo, gamma, beta, eps, scale, (const bf16_t*)post, pm, POST_ ? post_group : 1, \
                     POST_ ? post_skip : 0, (bf16_t*)next_out, next_ld, (const bf16_t*)next_w, next_b, next_n)
#define DP_MHA(SEQ_, GB_, DHP_, WPE_)                                                                              \
  do {                                                                                                             \
    const int64_t tiles_ = (nseq + GB_ - 1) / GB_;                                                                 \
    dim3 grid((unsigned)tiles_);                                                                                   \
    if (post && next_out) DP_MHA_L(SEQ_, GB_, true, true, DHP_, WPE_);                                             \
    else if (post) DP_MHA_L(SEQ_, GB_, true, false, DHP_, WPE_);                                                   \
    else if (next_out) DP_MHA_L(SEQ_, GB_, false, true, DHP_, WPE_);                                               \
    else DP_MHA_L(SEQ_, GB_, false, false, DHP_, WPE_);                                                            \
    return dp_check_launch("dp_mha_layernorm");                                                                    \
  } while (0)
  // within-instance: the 1 + 17 tokens of a query; across-instance: the 60 queries of a slot
  if (mode == 0) {
    if (seqlen == 18) DP_MHA(18, 4, 48, 0);
    if (seqlen == 60) DP_MHA(60, 1, 48, 0);
  } else {
    if (seqlen == 18) DP_MHA(18, 4, 48, 1);
    if (seqlen == 60) DP_MHA(60, 1, 48, 1);
  }
#undef DP_MHA
#undef DP_MHA_L
  dp_set_error("dp_mha_layernorm: seqlen %d not instantiated (18 / 60)", seqlen);
  return DP_EINVAL;
}

extern "C" int dp_linear_layernorm_classmax(void* out, const void* x, int32_t rows, int32_t c, const void* w,
                                            const float* b, const float* gamma, const float* beta, float eps,
                                            const uint8_t* row_mask, int32_t mask_period, const float* masked_row,
                                            const float* cls_w, const float* cls_b, int32_t nclass, float* cls_out,
                                            void* stream) {
  DP_REQUIRE(out && x && w && b && gamma && beta && cls_w && cls_b && cls_out && rows > 0,
             "dp_linear_layernorm_classmax: bad args");
  DP_REQUIRE(al16(out) && al16(x) && al16(w), "dp_linear_layernorm_classmax: rows must be 16-byte aligned");
  DP_REQUIRE(c == 256 && nclass >= 1 && nclass <= 4, "dp_linear_layernorm_classmax: c=%d (256), nclass=%d (1..4)", c,
             nclass);
  DP_REQUIRE(!row_mask || (mask_period > 0 && masked_row), "dp_linear_layernorm_classmax: bad mask");
  DP_REQUIRE((int64_t)rows * c < (1ll << 40), "dp_linear_layernorm_classmax: too many rows");
  hipStream_t s = as_stream(stream);
#ifndef DP_ENC_BM
#define DP_ENC_BM 64   // 64 rows: 40 KB LDS and <= 128 VGPRs, two blocks per CU overlap their phases
#endif
  constexpr int BM = DP_ENC_BM;
  dim3 grid((rows + BM - 1) / BM);
  hipLaunchKernelGGL((linear_ln_cls_kernel<256, BM>), grid, dim3(512), 0, s, (bf16_t*)out, (const bf16_t*)x,
                     (const bf16_t*)w, b, gamma, beta, eps, rows, row_mask, mask_period, masked_row, cls_w, cls_b,
                     nclass, cls_out);
  return dp_check_launch("dp_linear_layernorm_classmax");
}
