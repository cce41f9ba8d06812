// Row ops of the training step: forward versions that save what the
// backward needs, and the backward kernels, for the transformer's training forward with
// OKS-denoising queries. The Linear layers are dp_gemm (gemm.hip); the MSDA module is
// dp_msda / dp_msda_bwd (msda.hip, msda_train.hip). Reference lines on each entry point in
// include/detrpose_hip.h. f32 math everywhere; activations / activation gradients of dtype.
#include <algorithm>
#include <stdlib.h>
#include <initializer_list>

#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ T* tp(void* p) {
  return reinterpret_cast<T*>(p);
}
template <typename T>
__device__ __forceinline__ const T* tp(const void* p) {
  return reinterpret_cast<const T*>(p);
}

constexpr int LN_E = 8;   // c <= 512: up to 8 elements per lane

// ---------------------------------------------------------------- LayerNorm
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(T* __restrict__ y, int ld_y, const T* __restrict__ x,
                                                     const T* __restrict__ res, T* __restrict__ s,
                                                     float* __restrict__ stats, const float* __restrict__ g,
                                                     const float* __restrict__ bt, float eps, int rows, int c,
                                                     const T* __restrict__ post, int pgroup, int pskip) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float v[LN_E];
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < LN_E; ++t) {
    const int j = lane + 64 * t;
    v[t] = 0.f;
    if (j < c) {
      v[t] = to_f32(x[(int64_t)r * c + j]) + (res ? to_f32(res[(int64_t)r * c + j]) : 0.f);
      if (s) s[(int64_t)r * c + j] = from_f32<T>(v[t]);
      sum += v[t];
    }
  }
  const float mean = wave_sum(sum) / c;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < LN_E; ++t)
    if (lane + 64 * t < c) q += (v[t] - mean) * (v[t] - mean);
  const float rstd = rsqrtf(wave_sum(q) / c + eps);
  if (lane == 0) {
    stats[2 * (int64_t)r] = mean;
    stats[2 * (int64_t)r + 1] = rstd;
  }
  int64_t prow = -1;
  if (post) {
    const int gi = r % pgroup;
    if (gi >= pskip) prow = (int64_t)(r / pgroup) * (pgroup - pskip) + gi - pskip;
  }
#pragma unroll
  for (int t = 0; t < LN_E; ++t) {
    const int j = lane + 64 * t;
    if (j < c) {
      float o = (v[t] - mean) * rstd * g[j] + bt[j];
      if (prow >= 0) o += to_f32(post[prow * c + j]);
      y[(int64_t)r * ld_y + j] = from_f32<T>(o);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(T* __restrict__ dx, const T* __restrict__ dy, int ld_dy,
                                                     const T* __restrict__ s, const float* __restrict__ stats,
                                                     const float* __restrict__ g, int rows, int c,
                                                     float* __restrict__ dgamma, float* __restrict__ dbeta, int acc) {
  __shared__ float red[2][4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[LN_E], pb[LN_E];
#pragma unroll
  for (int t = 0; t < LN_E; ++t) pg[t] = pb[t] = 0.f;
  for (int r = blockIdx.x * 4 + wave; r < rows; r += gridDim.x * 4) {
    const float mean = stats[2 * (int64_t)r], rstd = stats[2 * (int64_t)r + 1];
    float xh[LN_E], gy[LN_E], d[LN_E];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_E; ++t) {
      const int j = lane + 64 * t;
      xh[t] = gy[t] = d[t] = 0.f;
      if (j < c) {
        d[t] = to_f32(dy[(int64_t)r * ld_dy + j]);
        xh[t] = (to_f32(s[(int64_t)r * c + j]) - mean) * rstd;
        gy[t] = d[t] * g[j];
        s1 += gy[t];
        s2 += gy[t] * xh[t];
        pg[t] += d[t] * xh[t];
        pb[t] += d[t];
      }
    }
    s1 = wave_sum(s1) / c;
    s2 = wave_sum(s2) / c;
#pragma unroll
    for (int t = 0; t < LN_E; ++t) {
      const int j = lane + 64 * t;
      if (j < c) {
        float o = rstd * (gy[t] - s1 - xh[t] * s2);
        T* p = dx + (int64_t)r * c + j;
        if (acc) o += to_f32(*p);
        *p = from_f32<T>(o);
      }
    }
  }
  if (!dgamma) return;
#pragma unroll
  for (int t = 0; t < LN_E; ++t) {
    const int j = lane + 64 * t;
    if (j < c) {
      red[0][wave][j] = pg[t];
      red[1][wave][j] = pb[t];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < c; j += 256) {
    unsafeAtomicAdd(dgamma + j, red[0][0][j] + red[0][1][j] + red[0][2][j] + red[0][3][j]);
    unsafeAtomicAdd(dbeta + j, red[1][0][j] + red[1][1][j] + red[1][2][j] + red[1][3][j]);
  }
}

// The same two kernels with each lane owning E = c / 64 CONTIGUOUS channels (c = 128 / 256 / 512):
// one E-element vector load per row and operand instead of E masked 2-byte loads (the strided
// form above runs its LN_E = 8 slots for every c, half of them masked at c = 256).
template <typename T, int E>
__device__ __forceinline__ void ldE(const T* p, float (&v)[E]) {
  typedef T VT __attribute__((ext_vector_type(E)));
  const VT u = *reinterpret_cast<const VT*>(p);
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = to_f32(u[e]);
}
template <typename T, int E>
__device__ __forceinline__ void stE(T* p, const float (&v)[E]) {
  typedef T VT __attribute__((ext_vector_type(E)));
  VT u;
#pragma unroll
  for (int e = 0; e < E; ++e) u[e] = from_f32<T>(v[e]);
  *reinterpret_cast<VT*>(p) = u;
}

template <typename T, int E>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(T* __restrict__ y, int ld_y, const T* __restrict__ x,
                                                         const T* __restrict__ res, T* __restrict__ s,
                                                         float* __restrict__ stats, const float* __restrict__ g,
                                                         const float* __restrict__ bt, float eps, int rows,
                                                         const T* __restrict__ post, int pgroup, int pskip) {
  constexpr int c = 64 * E;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int j0 = E * lane;
  float v[E];
  ldE<T, E>(x + (int64_t)r * c + j0, v);
  if (res) {
    float rv[E];
    ldE<T, E>(res + (int64_t)r * c + j0, rv);
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] += rv[e];
  }
  if (s) stE<T, E>(s + (int64_t)r * c + j0, v);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) sum += v[e];
  const float mean = wave_sum(sum) / c;
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) q += (v[e] - mean) * (v[e] - mean);
  const float rstd = rsqrtf(wave_sum(q) / c + eps);
  if (lane == 0) {
    stats[2 * (int64_t)r] = mean;
    stats[2 * (int64_t)r + 1] = rstd;
  }
  float pv[E];
  bool addp = false;
  if (post) {
    const int gi = r % pgroup;
    if (gi >= pskip) {
      ldE<T, E>(post + ((int64_t)(r / pgroup) * (pgroup - pskip) + gi - pskip) * c + j0, pv);
      addp = true;
    }
  }
  float o[E];
#pragma unroll
  for (int e = 0; e < E; ++e) o[e] = (v[e] - mean) * rstd * g[j0 + e] + bt[j0 + e] + (addp ? pv[e] : 0.f);
  stE<T, E>(y + (int64_t)r * ld_y + j0, o);
}

template <typename T, int E>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(T* __restrict__ dx, const T* __restrict__ dy, int ld_dy,
                                                         const T* __restrict__ s, const float* __restrict__ stats,
                                                         const float* __restrict__ g, int rows,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta, int acc) {
  constexpr int c = 64 * E;
  __shared__ float red[2][4][c];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j0 = E * lane;
  float gw[E], pg[E], pb[E];
#pragma unroll
  for (int e = 0; e < E; ++e) gw[e] = g[j0 + e], pg[e] = pb[e] = 0.f;
  for (int r = blockIdx.x * 4 + wave; r < rows; r += gridDim.x * 4) {
    const float mean = stats[2 * (int64_t)r], rstd = stats[2 * (int64_t)r + 1];
    float d[E], xh[E], gy[E];
    ldE<T, E>(dy + (int64_t)r * ld_dy + j0, d);
    ldE<T, E>(s + (int64_t)r * c + j0, xh);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      xh[e] = (xh[e] - mean) * rstd;
      gy[e] = d[e] * gw[e];
      s1 += gy[e];
      s2 += gy[e] * xh[e];
      pg[e] += d[e] * xh[e];
      pb[e] += d[e];
    }
    s1 = wave_sum(s1) / c;
    s2 = wave_sum(s2) / c;
    float o[E];
#pragma unroll
    for (int e = 0; e < E; ++e) o[e] = rstd * (gy[e] - s1 - xh[e] * s2);
    T* p = dx + (int64_t)r * c + j0;
    if (acc) {
      float pr[E];
      ldE<T, E>(p, pr);
#pragma unroll
      for (int e = 0; e < E; ++e) o[e] += pr[e];
    }
    stE<T, E>(p, o);
  }
  if (!dgamma) return;
#pragma unroll
  for (int e = 0; e < E; ++e) red[0][wave][j0 + e] = pg[e], red[1][wave][j0 + e] = pb[e];
  __syncthreads();
  for (int j = threadIdx.x; j < c; j += 256) {
    unsafeAtomicAdd(dgamma + j, red[0][0][j] + red[0][1][j] + red[0][2][j] + red[0][3][j]);
    unsafeAtomicAdd(dbeta + j, red[1][0][j] + red[1][1][j] + red[1][2][j] + red[1][3][j]);
  }
}

// E (elements per lane) for the vector forms: c = 64 E, rows and pointers E-element aligned
inline int ln_vec_e(int c, int esz, std::initializer_list<int64_t> lds, std::initializer_list<const void*> ptrs) {
  static const bool off = getenv("DETRPOSE_LN_VEC") && atoi(getenv("DETRPOSE_LN_VEC")) == 0;   // A/B
  const int e = c / 64;
  if (off || c % 64 || (e != 2 && e != 4 && e != 8)) return 0;
  for (int64_t l : lds)
    if (l % e) return 0;
  for (const void* q : ptrs)
    if (q && (reinterpret_cast<uintptr_t>(q) % (uintptr_t)(e * esz))) return 0;
  return e;
}

// ---------------------------------------------------------------- column sums (bias grads)
// A block = (256 / cw) row phases x cw columns (cw = n rounded up to a power of two, at most 256):
// narrow outputs (the pose heads' 34 / 4 columns) keep the lanes busy; 8 rows per step with the
// loads issued together; the block's phases are summed through LDS, one atomic per column.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ x, int64_t ld, int rows, int n,
                                                     float* __restrict__ out, int rows_per, int cw_log2) {
  __shared__ float red[256];
  const int cw = 1 << cw_log2, nph = 256 >> cw_log2;
  const int jl = threadIdx.x & (cw - 1), ph = threadIdx.x >> cw_log2;
  const int j = blockIdx.x * cw + jl;
  const int jc = min(j, n - 1);
  const int r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  float acc = 0.f;
  for (int r = r0 + ph; r < r1; r += 8 * nph) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = to_f32(x[(int64_t)min(r + u * nph, r1 - 1) * ld + jc]);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += r + u * nph < r1 ? v[u] : 0.f;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (ph == 0 && j < n) {
    float t = 0.f;
    for (int q = 0; q < nph; ++q) t += red[q * cw + jl];
    unsafeAtomicAdd(out + j, t);
  }
}

// The same over 16-byte column vectors (VC = 8 bf16 / 4 f32 columns per thread): 8x / 4x fewer
// load instructions than one column per lane.
template <typename T, int VC>
__global__ __launch_bounds__(256) void colsum_vec_kernel(const T* __restrict__ x, int64_t ld, int rows, int n,
                                                         float* __restrict__ out, int rows_per, int cw_log2) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  __shared__ float red[256][VC];
  const int cw = 1 << cw_log2, nph = 256 >> cw_log2;
  const int jl = threadIdx.x & (cw - 1), ph = threadIdx.x >> cw_log2;
  const int nv = n / VC;
  const int j = blockIdx.x * cw + jl;
  const int jc = min(j, nv - 1);
  const int r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  float acc[VC];
#pragma unroll
  for (int v = 0; v < VC; ++v) acc[v] = 0.f;
  for (int r = r0 + ph; r < r1; r += 4 * nph) {
    u32x4_t u[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      u[q] = *reinterpret_cast<const u32x4_t*>(x + (int64_t)min(r + q * nph, r1 - 1) * ld + (int64_t)jc * VC);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (r + q * nph >= r1) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (VC == 8) {
          acc[2 * e] += __uint_as_float(u[q][e] << 16);
          acc[2 * e + 1] += __uint_as_float(u[q][e] & 0xffff0000u);
        } else {
          acc[e] += __uint_as_float(u[q][e]);
        }
      }
    }
  }
#pragma unroll
  for (int v = 0; v < VC; ++v) red[threadIdx.x][v] = acc[v];
  __syncthreads();
  for (int pr = threadIdx.x; pr < cw * VC; pr += 256) {   // (vector, element) pairs of the block
    const int pl = pr / VC, v = pr - pl * VC, jj = blockIdx.x * cw + pl;
    if (jj >= nv) continue;
    float t = 0.f;
    for (int q = 0; q < nph; ++q) t += red[q * cw + pl][v];
    unsafeAtomicAdd(out + jj * VC + v, t);
  }
}

// ---------------------------------------------------------------- attention core
// One wave per (sequence, head, 64-row block): lane = a query (forward, dQ) or a key (dK, dV) of
// the block, so every sequence length keeps the chip busy (the AIFI layer's 400 tokens give 7
// blocks per (image, head)). The other side's rows stream through LDS in 64-row chunks (f32, row
// pitch DH: the lanes' uniform reads are broadcasts and vectorise). P is saved as [key j][query i]
// (coalesced over the query lanes) and only read by the backward, so a backward can be replayed;
// the backward's D_i = sum_j P_ij dO_i . V_j is dO_i . O_i, from the forward's output O.
// The head dim is a template constant and every load is unconditional (row indices clamped,
// out-of-range values selected away): a guarded load compiles to a branch around it, and the
// loads then issue one at a time.
constexpr int ACH = 64, MPT = ACH + 4;

// one row's DH values (f32) of a head
template <int DH, typename T>
__device__ __forceinline__ void load_head(float (&x)[DH], const T* p, float mul) {
#pragma unroll
  for (int dd = 0; dd < DH; ++dd) x[dd] = to_f32(p[dd]) * mul;
}

// rows j0 .. j0+63 of the sequence (zero past L), head columns col0 .., into dst[ACH][DH]
template <int DH, typename T>
__device__ __forceinline__ void stage_rows(float* dst, const T* src, int64_t ld, int64_t row0, int64_t st, int j0,
                                           int L, int col0) {
#pragma unroll 8
  for (int r = 0; r < DH; ++r) {
    const int e = r * 64 + threadIdx.x;
    const int t = e / DH, dd = e % DH;
    const int j = j0 + t;
    const float v = to_f32(src[(row0 + (int64_t)min(j, L - 1) * st) * ld + col0 + dd]);
    dst[e] = j < L ? v : 0.f;
  }
}

// P[j0 .. j0+63][i0 .. i0+63] of one (sequence, head) into dst[64][65] (zero past L)
__device__ __forceinline__ void stage_p(float* dst, const float* P, int L, int j0, int i0) {
  const int c = threadIdx.x;
  const int ic = min(i0 + c, L - 1);
#pragma unroll 8
  for (int t = 0; t < ACH; ++t) {
    const float v = P[(int64_t)min(j0 + t, L - 1) * L + ic];
    dst[t * (ACH + 1) + c] = (j0 + t < L && i0 + c < L) ? v : 0.f;
  }
}

template <typename T, int DH>
__global__ __launch_bounds__(64) void attn_fwd_kernel(const T* __restrict__ q, int ldq, const T* __restrict__ k,
                                                      const T* __restrict__ v, int ldkv, T* __restrict__ out, int ldo,
                                                      float* __restrict__ psave, const uint8_t* __restrict__ mask,
                                                      int n_inner, int64_t so, int64_t si, int64_t st, int L,
                                                      int nhead, float scale) {
  __shared__ float Ks[ACH * DH], Vs[ACH * DH];
  __shared__ uint8_t Ms[ACH * MPT];   // [query a][key c], pitch 68 B: lane rows hit distinct banks
  const int lane = threadIdx.x;
  const int h = blockIdx.x % nhead;
  const int seq = blockIdx.x / nhead;
  const int o = seq / n_inner, ii = seq - o * n_inner;
  const int64_t row0 = o * so + ii * si;
  const int ib = blockIdx.y * ACH;
  const int i = ib + lane;
  const bool live = i < L;
  const int64_t ri = row0 + (int64_t)min(i, L - 1) * st;
  float qi[DH];
  load_head<DH>(qi, q + ri * ldq + h * DH, scale);
  float* P = psave + (int64_t)blockIdx.x * L * L;
  auto stage_mask = [&](int j0) {   // lane = key column
    const int kc = min(j0 + lane, L - 1);
#pragma unroll 8
    for (int qa = 0; qa < ACH; ++qa) {
      const uint8_t mv = mask[(int64_t)min(ib + qa, L - 1) * L + kc];
      Ms[qa * MPT + lane] = j0 + lane < L ? mv : (uint8_t)1;
    }
  };
  // pass 1: row max and sum (online)
  float m = -INFINITY, l = 0.f;
  for (int j0 = 0; j0 < L; j0 += ACH) {
    __syncthreads();
    stage_rows<DH>(Ks, k, ldkv, row0, st, j0, L, h * DH);
    if (mask) stage_mask(j0);
    __syncthreads();
    const int nj = min(ACH, L - j0);
    for (int t = 0; t < nj; ++t) {
      float sc = 0.f;
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) sc = fmaf(qi[dd], Ks[t * DH + dd], sc);
      if (mask && Ms[lane * MPT + t]) continue;
      const float mn = fmaxf(m, sc);
      l = l * __expf(m - mn) + __expf(sc - mn);
      m = mn;
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  float acc[DH];
#pragma unroll
  for (int dd = 0; dd < DH; ++dd) acc[dd] = 0.f;
  // pass 2: P (saved) and P V
  for (int j0 = 0; j0 < L; j0 += ACH) {
    __syncthreads();
    stage_rows<DH>(Ks, k, ldkv, row0, st, j0, L, h * DH);
    stage_rows<DH>(Vs, v, ldkv, row0, st, j0, L, h * DH);
    if (mask) stage_mask(j0);
    __syncthreads();
    const int nj = min(ACH, L - j0);
    for (int t = 0; t < nj; ++t) {
      float sc = 0.f;
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) sc = fmaf(qi[dd], Ks[t * DH + dd], sc);
      float p = __expf(sc - m) * inv;
      if (mask && Ms[lane * MPT + t]) p = 0.f;
      if (live) P[(int64_t)(j0 + t) * L + i] = p;
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) acc[dd] = fmaf(p, Vs[t * DH + dd], acc[dd]);
    }
  }
  if (live) {
#pragma unroll
    for (int dd = 0; dd < DH; ++dd) out[ri * ldo + h * DH + dd] = from_f32<T>(acc[dd]);
  }
}

// Backward, query side (lane = query i): dS_ij = P_ij (dO_i . V_j - D_i), dQ_i = scale sum_j dS_ij K_j.
template <typename T, int DH>
__global__ __launch_bounds__(64) void attn_bwd_q_kernel(const T* __restrict__ k, const T* __restrict__ v, int ldkv,
                                                        const float* __restrict__ psave, const T* __restrict__ dout,
                                                        const T* __restrict__ out, int ldo, T* __restrict__ dq,
                                                        int lddq, int n_inner, int64_t so, int64_t si, int64_t st,
                                                        int L, int nhead, float scale) {
  __shared__ float Ks[ACH * DH], Vs[ACH * DH], Ps[ACH * (ACH + 1)];
  const int lane = threadIdx.x;
  const int h = blockIdx.x % nhead;
  const int seq = blockIdx.x / nhead;
  const int o = seq / n_inner, ii = seq - o * n_inner;
  const int64_t row0 = o * so + ii * si;
  const int i = blockIdx.y * ACH + lane;
  const bool live = i < L;
  const int64_t ri = row0 + (int64_t)min(i, L - 1) * st;
  float dOi[DH], oi[DH], acc[DH];
  load_head<DH>(dOi, dout + ri * ldo + h * DH, 1.f);
  load_head<DH>(oi, out + ri * ldo + h * DH, 1.f);
  float Di = 0.f;
#pragma unroll
  for (int dd = 0; dd < DH; ++dd) {
    Di = fmaf(dOi[dd], oi[dd], Di);
    acc[dd] = 0.f;
  }
  const float* P = psave + (int64_t)blockIdx.x * L * L;
  for (int j0 = 0; j0 < L; j0 += ACH) {
    __syncthreads();
    stage_rows<DH>(Ks, k, ldkv, row0, st, j0, L, h * DH);
    stage_rows<DH>(Vs, v, ldkv, row0, st, j0, L, h * DH);
    stage_p(Ps, P, L, j0, blockIdx.y * ACH);
    __syncthreads();
    const int nj = min(ACH, L - j0);
    for (int t = 0; t < nj; ++t) {
      const float p = Ps[t * (ACH + 1) + lane];
      float dp = 0.f;
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) dp = fmaf(dOi[dd], Vs[t * DH + dd], dp);
      const float ds = p * (dp - Di);
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) acc[dd] = fmaf(ds, Ks[t * DH + dd], acc[dd]);
    }
  }
  if (live) {
#pragma unroll
    for (int dd = 0; dd < DH; ++dd) dq[ri * lddq + h * DH + dd] = from_f32<T>(acc[dd] * scale);
  }
}

// Backward, key side (lane = key j): dV_j = sum_i P_ij dO_i, dK_j = scale sum_i dS_ij Q_i. The
// 64 x 64 block of P (this block's keys x a chunk of queries) is staged through LDS with coalesced
// row reads (row j of P is contiguous in i), pitch 65.
template <typename T, int DH>
__global__ __launch_bounds__(64) void attn_bwd_k_kernel(const T* __restrict__ q, int ldq, const T* __restrict__ v,
                                                        int ldkv, const float* __restrict__ psave,
                                                        const T* __restrict__ dout, const T* __restrict__ out, int ldo,
                                                        T* __restrict__ dk, T* __restrict__ dv, int lddkv, int n_inner,
                                                        int64_t so, int64_t si, int64_t st, int L, int nhead,
                                                        float scale) {
  __shared__ float Qs[ACH * DH], Gs[ACH * DH], Ps[ACH * (ACH + 1)], Dr[ACH];
  const int lane = threadIdx.x;
  const int h = blockIdx.x % nhead;
  const int seq = blockIdx.x / nhead;
  const int o = seq / n_inner, ii = seq - o * n_inner;
  const int64_t row0 = o * so + ii * si;
  const int jb = blockIdx.y * ACH;
  const int j = jb + lane;
  const bool live = j < L;
  const int64_t rj = row0 + (int64_t)min(j, L - 1) * st;
  float Vj[DH], dvacc[DH], dkacc[DH];
  load_head<DH>(Vj, v + rj * ldkv + h * DH, 1.f);
#pragma unroll
  for (int dd = 0; dd < DH; ++dd) {
    dvacc[dd] = 0.f;
    dkacc[dd] = 0.f;
  }
  const float* P = psave + (int64_t)blockIdx.x * L * L;
  for (int i0 = 0; i0 < L; i0 += ACH) {
    __syncthreads();
    stage_rows<DH>(Qs, q, ldq, row0, st, i0, L, h * DH);
    stage_rows<DH>(Gs, dout, ldo, row0, st, i0, L, h * DH);
    stage_p(Ps, P, L, jb, i0);
    __syncthreads();
    {   // D of the chunk's queries (lane = query): its dO row is staged, its O row read here
      const int64_t ri = row0 + (int64_t)min(i0 + lane, L - 1) * st;
      float oi[DH];
      load_head<DH>(oi, out + ri * ldo + h * DH, 1.f);
      float d = 0.f;
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) d = fmaf(Gs[lane * DH + dd], oi[dd], d);
      Dr[lane] = d;
    }
    __syncthreads();
    const int ni = min(ACH, L - i0);
    for (int c = 0; c < ni; ++c) {
      const float p = Ps[lane * (ACH + 1) + c];
      float dp = 0.f;
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) dp = fmaf(Gs[c * DH + dd], Vj[dd], dp);
      const float ds = p * (dp - Dr[c]);
#pragma unroll
      for (int dd = 0; dd < DH; ++dd) {
        dvacc[dd] = fmaf(p, Gs[c * DH + dd], dvacc[dd]);
        dkacc[dd] = fmaf(ds, Qs[c * DH + dd], dkacc[dd]);
      }
    }
  }
  if (live) {
#pragma unroll
    for (int dd = 0; dd < DH; ++dd) {
      dv[rj * lddkv + h * DH + dd] = from_f32<T>(dvacc[dd]);
      dk[rj * lddkv + h * DH + dd] = from_f32<T>(dkacc[dd] * scale);
    }
  }
}

// ---------------------------------------------------------------- Gate
// (row slices x channel blocks: a thread owns channel j and walks rows, no per-element division)
template <typename T>
__global__ void gate_fwd_kernel(const T* __restrict__ G, const T* __restrict__ xcat, T* __restrict__ gs,
                                T* __restrict__ z, int rows, int c) {
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= c) return;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t e = (int64_t)r * c + j;
    const int64_t b2 = (int64_t)r * 2 * c;
    const float g1 = sigmoidf_(to_f32(G[b2 + j])), g2 = sigmoidf_(to_f32(G[b2 + c + j]));
    gs[b2 + j] = from_f32<T>(g1);
    gs[b2 + c + j] = from_f32<T>(g2);
    z[e] = from_f32<T>(g1 * to_f32(xcat[b2 + j]) + g2 * to_f32(xcat[b2 + c + j]));
  }
}

template <typename T>
__global__ void gate_bwd_kernel(const T* __restrict__ dz, const T* __restrict__ gs, const T* __restrict__ xcat,
                                T* __restrict__ dG, T* __restrict__ dx, int rows, int c) {
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= c) return;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    const int64_t e = (int64_t)r * c + j;
    const int64_t b2 = (int64_t)r * 2 * c;
    const float d = to_f32(dz[e]);
    const float g1 = to_f32(gs[b2 + j]), g2 = to_f32(gs[b2 + c + j]);
    const float x1 = to_f32(xcat[b2 + j]), x2 = to_f32(xcat[b2 + c + j]);
    dG[b2 + j] = from_f32<T>(d * x1 * g1 * (1.f - g1));
    dG[b2 + c + j] = from_f32<T>(d * x2 * g2 * (1.f - g2));
    dx[b2 + j] = from_f32<T>(d * g1);
    dx[b2 + c + j] = from_f32<T>(d * g2);
  }
}

// (row slices, channel blocks): about 512 K threads (8 waves per SIMD), so the per-thread row walk
// stays short
dim3 rows_grid(int rows, int c, dim3* block) {
  const int bx = c >= 256 ? 256 : (c + 63) / 64 * 64, gy = (c + bx - 1) / bx;
  int gx = (1 << 19) / (bx * gy);
  if (gx > rows) gx = rows;
  if (gx < 1) gx = 1;
  *block = dim3((unsigned)bx);
  return dim3((unsigned)gx, (unsigned)gy);
}

// ---------------------------------------------------------------- query construction
template <typename T>
__global__ void query_build_kernel(const float* __restrict__ te, const float* __restrict__ ke,
                                   const float* __restrict__ ie, const float* __restrict__ le,
                                   const float* __restrict__ pe, const int* __restrict__ lab, int pad, int nq, int nkp,
                                   int c, int64_t total, T* __restrict__ tgt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int T_ = nkp + 1, Qt = pad + nq;
  const int ch = (int)(e % c);
  int64_t r = e / c;
  const int t = (int)(r % T_);
  r /= T_;
  const int qq = (int)(r % Qt);
  const int b = (int)(r / Qt);
  float v;
  if (qq < pad) {
    const int l = lab[(int64_t)b * pad + qq];
    v = l < 0 ? 0.f : (t == 0 ? le[(int64_t)l * c + ch] : pe[(int64_t)(t - 1) * c + ch]);
  } else {
    const int q = qq - pad;
    v = t == 0 ? ie[ch] : te[(int64_t)q * c + ch] + ke[(int64_t)(t - 1) * c + ch];
  }
  tgt[e] = from_f32<T>(v);
}

// Column sums over row sets (the embedding gradients of the query build): block (x, task) owns 64
// consecutive output elements (lane = channel, coalesced rows) and its QB_W waves split the task's
// rows, partials summed in wave order through LDS (deterministic; was one thread per output element
// walking all of its rows: the instance embedding's 256 threads each summed B * nq = 480 rows).
// task 0 tgt_embed [nq][c] over (b, t >= 1); 1 keypoint_embedding [nkp][c] over (b, q); 2
// instance_embedding [c] over (b, q); 3 pose_enc [nkp][c] over the labelled DN slots (b, i);
// 4 label_enc rows (float atomics per DN slot, element-wise).
constexpr int QB_W = 16;
template <typename T>
__global__ __launch_bounds__(64 * QB_W) void query_build_bwd_kernel(const T* __restrict__ d, const int* __restrict__ lab,
                                                                   int B, int pad, int nq, int nkp, int c,
                                                                   float* __restrict__ gte, float* __restrict__ gke,
                                                                   float* __restrict__ gie, float* __restrict__ gle,
                                                                   float* __restrict__ gpe) {
  const int T_ = nkp + 1, Qt = pad + nq;
  const int task = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  auto at = [&](int b, int qq, int t, int ch) { return to_f32(d[(((int64_t)b * Qt + qq) * T_ + t) * c + ch]); };
  if (task == 4) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= B * pad * c || !gle) return;
    const int slot = e / c, ch = e % c;
    const int b = slot / pad, i = slot % pad;
    const int l = lab[slot];
    if (l >= 0) unsafeAtomicAdd(gle + (int64_t)l * c + ch, at(b, i, 0, ch));
    return;
  }
  __shared__ float part[QB_W][64];
  const int n_out = task == 0 ? nq * c : task == 2 ? c : nkp * c;
  float* g = task == 0 ? gte : task == 1 ? gke : task == 2 ? gie : gpe;
  if (!g || blockIdx.x * 64 >= n_out) return;   // block-uniform
  const int e = blockIdx.x * 64 + lane;
  const bool live = e < n_out;
  const int row = live ? e / c : 0, ch = live ? e % c : 0;
  const int nrows = task == 0 ? B * (T_ - 1) : task == 3 ? B * pad : B * nq;
  float s = 0.f;
  if (live) {
    for (int r = w; r < nrows; r += QB_W) {
      if (task == 0) {
        const int b = r / (T_ - 1), t = 1 + r % (T_ - 1);
        s += at(b, pad + row, t, ch);
      } else if (task == 3) {
        const int b = r / pad, i = r % pad;
        if (lab[(int64_t)b * pad + i] >= 0) s += at(b, i, row + 1, ch);
      } else {
        const int b = r / nq, q = r % nq;
        s += at(b, pad + q, task == 1 ? row + 1 : 0, ch);
      }
    }
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && live) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < QB_W; ++i) t += part[i][lane];
    g[e] += t;
  }
}

// ---------------------------------------------------------------- heads
__global__ void pose_refine_bwd_kernel(const float* __restrict__ corners, const float* __restrict__ proj, int nb,
                                       float inv_s, const float* __restrict__ dk, int n, float* __restrict__ dc,
                                       int acc) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;   // (row, kp, coordinate)
  if (e >= n) return;
  const float* cr = corners + (int64_t)e * nb;
  float mx = -INFINITY;
  for (int i = 0; i < nb; ++i) mx = fmaxf(mx, cr[i]);
  float den = 0.f, num = 0.f;
  for (int i = 0; i < nb; ++i) {
    const float p = __expf(cr[i] - mx);
    den += p;
    num += p * proj[i];
  }
  const float mean_w = num / den;
  const float g = dk[e] * inv_s;
  float* o = dc + (int64_t)e * nb;
  for (int i = 0; i < nb; ++i) {
    const float p = __expf(cr[i] - mx) / den;
    const float v = g * p * (proj[i] - mean_w);
    o[i] = acc ? o[i] + v : v;
  }
}

__global__ void sigmoid_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy, float* __restrict__ dx,
                                   int rows, int n, int64_t ldy, int64_t lddy, int64_t lddx) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)rows * n) return;
  const int64_t r = e / n;
  const int j = (int)(e - r * n);
  const float s = y[r * ldy + j];
  dx[r * lddx + j] = dy[r * lddy + j] * s * (1.f - s);
}

// one wave per keypoint: the forward's sample + top-4 (lqe_kernel in heads.hip: channels
// lane*E .. lane*E + E - 1, ties to the lowest lane / element) recomputed, then
// d stat / d(x, y) through the bilinear weights (feat detached).
template <typename T, int E>
__global__ __launch_bounds__(256) void lqe_bwd_kernel(const T* __restrict__ feat, int64_t fbs, int h, int w, int c,
                                                      const float* __restrict__ kps, const float* __restrict__ dst,
                                                      int nq, int nkp, int total, float* __restrict__ dkps,
                                                      float* __restrict__ dfeat, int64_t dfbs) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= total) return;
  const int b = (unsigned)g / (unsigned)(nq * nkp);
  const float x = kps[2 * (int64_t)g] * w - 0.5f, y = kps[2 * (int64_t)g + 1] * h - 0.5f;
  const float fx = floorf(x), fy = floorf(y);
  const int x0 = (int)fx, y0 = (int)fy;
  const float ax = x - fx, ay = y - fy;
  const float wt[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
  // d wt / d ax, d wt / d ay
  const float wx[4] = {-(1.f - ay), (1.f - ay), -ay, ay};
  const float wy[4] = {-(1.f - ax), -ax, (1.f - ax), ax};
  float v[E], gx[E], gy[E];
#pragma unroll
  for (int t = 0; t < E; ++t) v[t] = gx[t] = gy[t] = 0.f;
  const T* fb = feat + (int64_t)b * fbs + lane * E;
#pragma unroll
  for (int cn = 0; cn < 4; ++cn) {
    const int xi = x0 + (cn & 1), yi = y0 + (cn >> 1);
    if (xi < 0 || xi >= w || yi < 0 || yi >= h) continue;
    const T* p = fb + ((int64_t)yi * w + xi) * c;
#pragma unroll
    for (int t = 0; t < E; ++t) {
      const float f = to_f32(p[t]);
      v[t] = fmaf(wt[cn], f, v[t]);
      gx[t] = fmaf(wx[cn], f, gx[t]);
      gy[t] = fmaf(wy[cn], f, gy[t]);
    }
  }
  const float* ds = dst + (int64_t)g * 5;
  const float dmean = ds[4] * 0.25f;
  float ax_acc = 0.f, ay_acc = 0.f;
  unsigned used = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    float lm = -INFINITY;
    int li = -1;
#pragma unroll
    for (int t = 0; t < E; ++t)
      if (!(used & (1u << t)) && v[t] > lm) {
        lm = v[t];
        li = t;
      }
    const float wm = wave_max(lm);
    const unsigned long long ball = __ballot(lm == wm && li >= 0);
    const int winner = __ffsll((long long)ball) - 1;
    if (lane == winner) {
      used |= 1u << li;
      const float coef = ds[s] + dmean;
      if (dfeat) {   // d feat: the bilinear weights of the selected channel's four corners
        float* df = dfeat + (int64_t)b * dfbs + lane * E + li;
#pragma unroll
        for (int cn = 0; cn < 4; ++cn) {
          const int xi = x0 + (cn & 1), yi = y0 + (cn >> 1);
          if (xi >= 0 && xi < w && yi >= 0 && yi < h) atomicAdd(df + ((int64_t)yi * w + xi) * c, coef * wt[cn]);
        }
      }
#pragma unroll
      for (int t = 0; t < E; ++t)
        if (t == li) {
          ax_acc += coef * gx[t];
          ay_acc += coef * gy[t];
        }
    }
  }
  ax_acc = wave_sum(ax_acc);
  ay_acc = wave_sum(ay_acc);
  if (lane == 0) {
    dkps[2 * (int64_t)g] += ax_acc * w;
    dkps[2 * (int64_t)g + 1] += ay_acc * h;
  }
}

// ---------------------------------------------------------------- row moves
template <typename T>
__global__ void scatter_rows_kernel(const T* __restrict__ src, int lds, const int64_t* __restrict__ idx,
                                    const uint8_t* __restrict__ mask, int period, int k, int c, T* __restrict__ dst,
                                    int64_t dbs, int ldd, int acc, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int ch = (int)(e % c);
  const int64_t rj = e / c;   // b * k + j
  const int b = (int)(rj / k);
  const int64_t dr = idx[rj];
  if (mask && mask[dr % period]) return;   // masked_fill'ed row: no gradient reaches it
  T* p = dst + (int64_t)b * dbs + dr * ldd + ch;
  float v = to_f32(src[rj * lds + ch]);
  if (acc) v += to_f32(*p);
  *p = from_f32<T>(v);
}

template <typename T>
__global__ void gather_masked_kernel(const T* __restrict__ src, int64_t sbs, const int64_t* __restrict__ idx,
                                     const uint8_t* __restrict__ mask, int period, int k, int c, T* __restrict__ dst,
                                     int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int ch = (int)(e % c);
  const int64_t rj = e / c;
  const int b = (int)(rj / k);
  const int64_t sr = idx[rj];
  const bool m = mask && mask[sr % period];
  dst[e] = m ? from_f32<T>(0.f) : src[(int64_t)b * sbs + sr * c + ch];
}

template <typename TS, typename TD>
__global__ void convert_kernel(const TS* __restrict__ src, int64_t lds, TD* __restrict__ dst, int64_t ldd, int rows,
                               int n, float scale, int acc) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)rows * n) return;
  // 32-bit division when the index fits (every launch of the step), 64-bit otherwise
  int64_t r;
  int j;
  if (e < 0x7fffffff) {
    const unsigned ue = (unsigned)e, un = (unsigned)n;
    const unsigned ur = ue / un;
    r = ur;
    j = (int)(ue - ur * un);
  } else {
    r = e / n;
    j = (int)(e - r * n);
  }
  float v = to_f32(src[r * lds + j]) * scale;
  TD* p = dst + r * ldd + j;
  if (acc) v += to_f32(*p);
  *p = from_f32<TD>(v);
}

// ---------------------------------------------------------------- OKS-denoising draws
// counter-based uniform [0, 1): splitmix64 finaliser of (seed, stream, index)
__device__ __forceinline__ float urand(uint64_t seed, uint32_t stream, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1) + ((uint64_t)stream << 40);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// one thread per (image, DN slot, point): prepare_for_cdn's noised labels and keypoints
// (dn_component.py:51-153) for slot = group * single_pad + t, t < targets of the image
// (even groups positive, odd negative); padding slots get label -1 and ref 0.5.
__global__ void cdn_build_kernel(const int* __restrict__ off, const int* __restrict__ labels,
                                 const float* __restrict__ kps, const float* __restrict__ area,
                                 const float* __restrict__ boxes, const float* __restrict__ sig, int B, int pad,
                                 int single, int nkp, float label_noise, int num_classes, float img_h, float img_w,
                                 uint64_t seed, int* __restrict__ dn_label, float* __restrict__ dn_ref) {
  const int T = nkp + 1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * pad * T) return;
  const int pt = (int)(e % T);
  const int64_t bs = e / T;
  const int slot = (int)(bs % pad), b = (int)(bs / pad);
  const int g = slot / single, t = slot - g * single;
  const int n = off[b + 1] - off[b];
  float* rf = dn_ref + e * 2;
  if (t >= n) {
    if (pt == 0) dn_label[bs] = -1;
    rf[0] = rf[1] = 0.5f;   // sigmoid(0): the zero padding of input_query_pose
    return;
  }
  const int tg = off[b] + t;
  const uint64_t key = ((uint64_t)g * 1048576ull + (uint64_t)tg) * 64ull;   // (group, target) draw stream
  if (pt == 0) {
    int lab = labels[tg];
    if (urand(seed, 1, key) < label_noise * 0.5f) lab = min((int)(urand(seed, 2, key) * num_classes), num_classes - 1);
    dn_label[bs] = lab;
  }
  // point pt: 0 = centre of the xyxy box (dn_component.py:95), 1..K the keypoints
  float x, y;
  bool viz;
  if (pt == 0) {
    const float* bx = boxes + (int64_t)tg * 4;
    x = (bx[0] + bx[2]) * 0.5f;
    y = (bx[1] + bx[3]) * 0.5f;
    viz = false;   // the centre is never noised (dn_component.py:104)
  } else {
    const float* kp = kps + (int64_t)tg * 3 * nkp;
    x = kp[2 * (pt - 1)];
    y = kp[2 * (pt - 1) + 1];
    viz = kp[2 * nkp + pt - 1] != 0.f;
  }
  if (viz) {
    // direction: normalize(rand_like) (first quadrant, dn_component.py:121-122); distance:
    // alpha ~ U(0, ln 2) positive / U(ln 2, ln 10) negative, * 2 (area*h*w + eps) var, sqrt, / max(h, w)
    const float u1 = urand(seed, 3, key + pt), u2 = urand(seed, 4, key + pt);
    const float nrm = fmaxf(sqrtf(u1 * u1 + u2 * u2), 1e-12f);
    const float ua = urand(seed, 5, key + pt);
    const bool neg = g & 1;
    const float lo = neg ? 0.69314718f : 0.f, hi = neg ? 2.30258509f : 0.69314718f;
    float alpha = lo + (hi - lo) * ua;
    const float s2 = 2.f * sig[pt];
    alpha *= 2.f * (area[tg] * img_h * img_w + 1.1920929e-07f) * s2 * s2;
    alpha = sqrtf(alpha) / fmaxf(img_h, img_w);
    x += alpha * u1 / nrm;
    y += alpha * u2 / nrm;
  }
  // inverse_sigmoid (utils.py:133-137) then the sigmoid of transformer.py:1279
  auto isig = [](float v) {
    v = fminf(fmaxf(v, 0.f), 1.f);
    return logf(fmaxf(v, 1e-3f) / fmaxf(1.f - v, 1e-3f));
  };
  rf[0] = 1.f / (1.f + expf(-isig(x)));
  rf[1] = 1.f / (1.f + expf(-isig(y)));
}

// ---------------------------------------------------------------- optimizer
// Squared norm in two fixed-shape passes (no float atomics): DP_SQNORM_PARTS block partials, then
// one block sums them in a fixed order. The result is bit-identical for identical gradients, so
// DDP ranks holding the all-reduced gradient clip by the same factor and their parameters stay
// identical (the replica invariant DDP relies on after its initial broadcast).
__global__ void sqnorm_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc = fmaf(g[i], g[i], acc);
  acc = wave_sum(acc);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void sqnorm_final_kernel(const float* __restrict__ part, int nparts, float* __restrict__ out) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  acc = wave_sum(acc);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

// torch.optim.AdamW step (decoupled weight decay, bias corrections) after
// clip_grad_norm_(max_norm): g *= min(max_norm / (||g|| + 1e-6), 1) with ||g||^2 from sqnorm
// skip (device flag, NULL = never): a non-zero value leaves parameters and moments unchanged
// (dp_finite_guard set it: a non-finite loss or gradient norm). A non-finite norm skips too:
// fminf(max_norm / NaN, 1) would otherwise be 1, silently turning the clipping off.
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2, float max_norm, const float* __restrict__ sq,
                             const float* __restrict__ skip) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (skip && *skip != 0.f) return;
  float scale = 1.f;
  if (max_norm > 0.f) {
    const float nrm = sqrtf(*sq);
    if (!isfinite(nrm)) return;
    scale = fminf(max_norm / (nrm + 1e-6f), 1.f);
  }
  const float gi = g[i] * scale;
  float pi = p[i] * (1.f - lr * wd);
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  pi -= (lr / bc1) * mi / (sqrtf(vi) / sqrtf(bc2) + eps);
  p[i] = pi;
}

// bad[0] = 1 when any of v[0..n) is not finite (left unchanged otherwise): one block
__global__ void finite_guard_kernel(const float* __restrict__ v, int64_t n, float* __restrict__ bad) {
  int nonfinite = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) nonfinite |= !isfinite(v[i]);
  if (__syncthreads_or(nonfinite) && threadIdx.x == 0) bad[0] = 1.f;
}

// ModelEMA: e = d e + (1 - d) p, unless *skip != 0
__global__ void ema_kernel(float* __restrict__ e, const float* __restrict__ p, int64_t n, float d,
                           const float* __restrict__ skip) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (skip && *skip != 0.f)) return;
  e[i] = d * e[i] + (1.f - d) * p[i];
}

inline unsigned nblk(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// ================================================================== C ABI
extern "C" int dp_ln_fwd(void* y, int32_t ld_y, const void* x, const void* res, void* s, float* stats,
                         const float* gamma, const float* beta, float eps, int32_t rows, int32_t c, const void* post,
                         int32_t post_group, int32_t post_skip, int32_t dtype, void* stream) {
  DP_REQUIRE(y && x && stats && gamma && beta, "dp_ln_fwd: null pointer");
  DP_REQUIRE(c > 0 && c <= 64 * LN_E && rows > 0 && ld_y >= c, "dp_ln_fwd: c=%d rows=%d ld_y=%d", c, rows, ld_y);
  DP_REQUIRE(!post || (post_group > post_skip && post_skip >= 0), "dp_ln_fwd: bad post map");
  hipStream_t st = as_stream(stream);
  const int esz = dtype == DP_BF16 ? 2 : 4;
  if (const int e = ln_vec_e(c, esz, {ld_y}, {y, x, res, s, post})) {
#define LNF(T_, E_)                                                                                              \
  hipLaunchKernelGGL((ln_fwd_vec_kernel<T_, E_>), dim3(nblk(rows, 4)), dim3(256), 0, st, (T_*)y, ld_y, (const T_*)x, \
                     (const T_*)res, (T_*)s, stats, gamma, beta, eps, rows, (const T_*)post, post_group, post_skip)
    if (dtype == DP_BF16) {
      if (e == 2) LNF(bf16_t, 2); else if (e == 4) LNF(bf16_t, 4); else LNF(bf16_t, 8);
    } else {
      if (e == 2) LNF(float, 2); else if (e == 4) LNF(float, 4); else LNF(float, 8);
    }
#undef LNF
    return dp_check_launch("dp_ln_fwd");
  }
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, dim3(nblk(rows, 4)), dim3(256), 0, st, (bf16_t*)y, ld_y,
                       (const bf16_t*)x, (const bf16_t*)res, (bf16_t*)s, stats, gamma, beta, eps, rows, c,
                       (const bf16_t*)post, post_group, post_skip);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3(nblk(rows, 4)), dim3(256), 0, st, (float*)y, ld_y, (const float*)x,
                       (const float*)res, (float*)s, stats, gamma, beta, eps, rows, c, (const float*)post, post_group,
                       post_skip);
  return dp_check_launch("dp_ln_fwd");
}

extern "C" int dp_ln_bwd(void* dx, const void* dy, int32_t ld_dy, const void* s, const float* stats,
                         const float* gamma, int32_t rows, int32_t c, float* dgamma, float* dbeta, int32_t accumulate,
                         int32_t dtype, void* stream) {
  DP_REQUIRE(dx && dy && s && stats && gamma, "dp_ln_bwd: null pointer");
  DP_REQUIRE(c > 0 && c <= 64 * LN_E && rows > 0 && ld_dy >= c, "dp_ln_bwd: c=%d rows=%d", c, rows);
  DP_REQUIRE((dgamma == nullptr) == (dbeta == nullptr), "dp_ln_bwd: dgamma / dbeta both or neither");
  // every block adds its dgamma / dbeta partials with one atomic per column: 256 blocks (one per
  // CU) keep the same-address atomic chains short (2048 blocks cost ~2x the kernel)
  int grid = (rows + 3) / 4;
  if (grid > 256) grid = 256;
  hipStream_t st = as_stream(stream);
  const int esz = dtype == DP_BF16 ? 2 : 4;
  if (const int e = ln_vec_e(c, esz, {ld_dy}, {dx, dy, s})) {
#define LNB(T_, E_)                                                                                               \
  hipLaunchKernelGGL((ln_bwd_vec_kernel<T_, E_>), dim3(grid), dim3(256), 0, st, (T_*)dx, (const T_*)dy, ld_dy,      \
                     (const T_*)s, stats, gamma, rows, dgamma, dbeta, accumulate)
    if (dtype == DP_BF16) {
      if (e == 2) LNB(bf16_t, 2); else if (e == 4) LNB(bf16_t, 4); else LNB(bf16_t, 8);
    } else {
      if (e == 2) LNB(float, 2); else if (e == 4) LNB(float, 4); else LNB(float, 8);
    }
#undef LNB
    return dp_check_launch("dp_ln_bwd");
  }
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, st, (bf16_t*)dx, (const bf16_t*)dy, ld_dy,
                       (const bf16_t*)s, stats, gamma, rows, c, dgamma, dbeta, accumulate);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(grid), dim3(256), 0, st, (float*)dx, (const float*)dy, ld_dy,
                       (const float*)s, stats, gamma, rows, c, dgamma, dbeta, accumulate);
  return dp_check_launch("dp_ln_bwd");
}

extern "C" int dp_colsum(const void* x, int64_t ld, int32_t rows, int32_t n, float* out, int32_t accumulate,
                         int32_t dtype, void* stream) {
  DP_REQUIRE(x && out && rows > 0 && n > 0 && ld >= n, "dp_colsum: bad arguments");
  hipStream_t st = as_stream(stream);
  if (!accumulate && dp_zero_async(out, (size_t)n * 4, st)) return dp_check_launch("dp_colsum");
  const int vc = dtype == DP_BF16 ? 8 : 4;
  if (n % vc == 0 && ld % vc == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int nv = n / vc;
    int lg = 0;
    while ((1 << lg) < nv && lg < 8) ++lg;
    const int cw = 1 << lg, gx = (nv + cw - 1) / cw, nph = 256 / cw;
    int chunks = std::max(1, std::min((rows + 4 * nph - 1) / (4 * nph), std::max(1, 256 / gx)));   // one block per CU: each column takes <= 256 atomics
    const int per = (rows + chunks - 1) / chunks;
    chunks = (rows + per - 1) / per;
    dim3 grid((unsigned)gx, (unsigned)chunks);
    if (dtype == DP_BF16)
      hipLaunchKernelGGL((colsum_vec_kernel<bf16_t, 8>), grid, dim3(256), 0, st, (const bf16_t*)x, ld, rows, n, out,
                         per, lg);
    else
      hipLaunchKernelGGL((colsum_vec_kernel<float, 4>), grid, dim3(256), 0, st, (const float*)x, ld, rows, n, out,
                         per, lg);
    return dp_check_launch("dp_colsum");
  }
  int lg = 0;
  while ((1 << lg) < n && lg < 8) ++lg;
  const int cw = 1 << lg, gx = (n + cw - 1) / cw;
  // about 1024 blocks, each at least 8 row steps of its phases
  const int nph = 256 / cw;
  int chunks = std::max(1, std::min((rows + 8 * nph - 1) / (8 * nph), std::max(1, 256 / gx)));   // <= 256 atomics per column
  const int per = (rows + chunks - 1) / chunks;
  chunks = (rows + per - 1) / per;
  dim3 grid((unsigned)gx, (unsigned)chunks);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, ld, rows, n, out, per, lg);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, (const float*)x, ld, rows, n, out, per, lg);
  return dp_check_launch("dp_colsum");
}

// the head dim picks the instantiation (the decoder's and the AIFI layer's heads are 32 wide)
#define ATT_LAUNCH(KERN, T, GRID, BLOCK, LDS, STREAM, ...)                                                \
  do {                                                                                                    \
    switch (dh) {                                                                                         \
      case 16: hipLaunchKernelGGL((KERN<T, 16>), GRID, BLOCK, LDS, STREAM, __VA_ARGS__); break;           \
      case 32: hipLaunchKernelGGL((KERN<T, 32>), GRID, BLOCK, LDS, STREAM, __VA_ARGS__); break;           \
      case 48: hipLaunchKernelGGL((KERN<T, 48>), GRID, BLOCK, LDS, STREAM, __VA_ARGS__); break;           \
      default: hipLaunchKernelGGL((KERN<T, 64>), GRID, BLOCK, LDS, STREAM, __VA_ARGS__); break;           \
    }                                                                                                     \
  } while (0)

// bf16 MFMA kernels for sequences of <= 128 tokens (train_attn.hip); false = not covered
bool dp_attn_fwd_mfma(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, void* out, int32_t ld_o,
                      float* p_save, const uint8_t* mask, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si,
                      int64_t st, int32_t seqlen, int32_t nhead, int32_t dh, float scale, hipStream_t s);
bool dp_attn_bwd_mfma(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, const float* p_save,
                      const void* dout, const void* out, int32_t ld_o, void* dq, int32_t ld_dq, void* dk, void* dv,
                      int32_t ld_dkv, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si, int64_t st,
                      int32_t seqlen, int32_t nhead, int32_t dh, float scale, hipStream_t s);
static bool attn_scalar_forced() {   // A/B switch: DETRPOSE_ATTN_SCALAR=1 keeps the scalar bf16 kernels
  static const bool f = getenv("DETRPOSE_ATTN_SCALAR") != nullptr;
  return f;
}

extern "C" int dp_attn_fwd(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, void* out,
                           int32_t ld_o, float* p_save, const uint8_t* mask, int32_t n_outer, int32_t n_inner,
                           int64_t so, int64_t si, int64_t st, int32_t seqlen, int32_t nhead, int32_t dh, int32_t dtype,
                           void* stream) {
  DP_REQUIRE(q && k && v && out && p_save, "dp_attn_fwd: null pointer");
  DP_REQUIRE(seqlen > 0 && (dh == 16 || dh == 32 || dh == 48 || dh == 64),
             "dp_attn_fwd: seqlen %d x dh %d (dh 16 / 32 / 48 / 64)", seqlen, dh);
  DP_REQUIRE((int64_t)n_outer * n_inner * nhead < (1ll << 31), "dp_attn_fwd: too many sequences");
  const float scale = 1.f / sqrtf((float)dh);
  dim3 grid((unsigned)(n_outer * n_inner * nhead), (unsigned)((seqlen + ACH - 1) / ACH));
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16 && !attn_scalar_forced() &&
      dp_attn_fwd_mfma(q, ld_q, k, v, ld_kv, out, ld_o, p_save, mask, n_outer, n_inner, so, si, st, seqlen, nhead, dh,
                       scale, s))
    return dp_check_launch("dp_attn_fwd");
  if (dtype == DP_BF16)
    ATT_LAUNCH(attn_fwd_kernel, bf16_t, grid, dim3(64), 0, s, (const bf16_t*)q, ld_q, (const bf16_t*)k,
                       (const bf16_t*)v, ld_kv, (bf16_t*)out, ld_o, p_save, mask, n_inner, so, si, st, seqlen, nhead,
                       scale);
  else
    ATT_LAUNCH(attn_fwd_kernel, float, grid, dim3(64), 0, s, (const float*)q, ld_q, (const float*)k,
                       (const float*)v, ld_kv, (float*)out, ld_o, p_save, mask, n_inner, so, si, st, seqlen, nhead,
                       scale);
  return dp_check_launch("dp_attn_fwd");
}

extern "C" int dp_attn_bwd(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv,
                           const float* p_save, const void* dout, const void* out, int32_t ld_o, void* dq,
                           int32_t ld_dq, void* dk, void* dv, int32_t ld_dkv, int32_t n_outer, int32_t n_inner,
                           int64_t so, int64_t si, int64_t st, int32_t seqlen, int32_t nhead, int32_t dh, int32_t dtype,
                           void* stream) {
  DP_REQUIRE(q && k && v && p_save && dout && out && dq && dk && dv, "dp_attn_bwd: null pointer");
  DP_REQUIRE(seqlen > 0 && (dh == 16 || dh == 32 || dh == 48 || dh == 64),
             "dp_attn_bwd: seqlen %d x dh %d (dh 16 / 32 / 48 / 64)", seqlen, dh);
  const float scale = 1.f / sqrtf((float)dh);
  dim3 grid((unsigned)(n_outer * n_inner * nhead), (unsigned)((seqlen + ACH - 1) / ACH));
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16 && !attn_scalar_forced() &&
      dp_attn_bwd_mfma(q, ld_q, k, v, ld_kv, p_save, dout, out, ld_o, dq, ld_dq, dk, dv, ld_dkv, n_outer, n_inner, so,
                       si, st, seqlen, nhead, dh, scale, s))
    return dp_check_launch("dp_attn_bwd");
  if (dtype == DP_BF16) {
    ATT_LAUNCH(attn_bwd_q_kernel, bf16_t, grid, dim3(64), 0, s, (const bf16_t*)k, (const bf16_t*)v, ld_kv,
                       p_save, (const bf16_t*)dout, (const bf16_t*)out, ld_o, (bf16_t*)dq, ld_dq, n_inner, so, si, st,
                       seqlen, nhead, scale);
    ATT_LAUNCH(attn_bwd_k_kernel, bf16_t, grid, dim3(64), 0, s, (const bf16_t*)q, ld_q, (const bf16_t*)v,
                       ld_kv, p_save, (const bf16_t*)dout, (const bf16_t*)out, ld_o, (bf16_t*)dk, (bf16_t*)dv, ld_dkv,
                       n_inner, so, si, st, seqlen, nhead, scale);
  } else {
    ATT_LAUNCH(attn_bwd_q_kernel, float, grid, dim3(64), 0, s, (const float*)k, (const float*)v, ld_kv, p_save,
                       (const float*)dout, (const float*)out, ld_o, (float*)dq, ld_dq, n_inner, so, si, st, seqlen,
                       nhead, scale);
    ATT_LAUNCH(attn_bwd_k_kernel, float, grid, dim3(64), 0, s, (const float*)q, ld_q, (const float*)v, ld_kv,
                       p_save, (const float*)dout, (const float*)out, ld_o, (float*)dk, (float*)dv, ld_dkv, n_inner,
                       so, si, st, seqlen, nhead, scale);
  }
  return dp_check_launch("dp_attn_bwd");
}

extern "C" int dp_gate_fwd(const void* G, const void* xcat, void* g, void* z, int32_t rows, int32_t c, int32_t dtype,
                           void* stream) {
  DP_REQUIRE(G && xcat && g && z && rows > 0 && c > 0, "dp_gate_fwd: bad arguments");
  hipStream_t s = as_stream(stream);
  dim3 block;
  const dim3 grid = rows_grid(rows, c, &block);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(gate_fwd_kernel<bf16_t>, grid, block, 0, s, (const bf16_t*)G, (const bf16_t*)xcat, (bf16_t*)g,
                       (bf16_t*)z, rows, c);
  else
    hipLaunchKernelGGL(gate_fwd_kernel<float>, grid, block, 0, s, (const float*)G, (const float*)xcat, (float*)g,
                       (float*)z, rows, c);
  return dp_check_launch("dp_gate_fwd");
}

extern "C" int dp_gate_bwd(const void* dz, const void* g, const void* xcat, void* dG, void* dxcat, int32_t rows,
                           int32_t c, int32_t dtype, void* stream) {
  DP_REQUIRE(dz && g && xcat && dG && dxcat && rows > 0 && c > 0, "dp_gate_bwd: bad arguments");
  hipStream_t s = as_stream(stream);
  dim3 block;
  const dim3 grid = rows_grid(rows, c, &block);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(gate_bwd_kernel<bf16_t>, grid, block, 0, s, (const bf16_t*)dz, (const bf16_t*)g,
                       (const bf16_t*)xcat, (bf16_t*)dG, (bf16_t*)dxcat, rows, c);
  else
    hipLaunchKernelGGL(gate_bwd_kernel<float>, grid, block, 0, s, (const float*)dz, (const float*)g, (const float*)xcat,
                       (float*)dG, (float*)dxcat, rows, c);
  return dp_check_launch("dp_gate_bwd");
}

extern "C" int dp_query_build(const float* tgt_embed, const float* kp_embed, const float* inst_embed,
                              const float* label_enc, const float* pose_enc, const int32_t* dn_label, int32_t batch,
                              int32_t pad, int32_t nq, int32_t nkp, int32_t c, void* tgt, int32_t dtype, void* stream) {
  DP_REQUIRE(tgt_embed && kp_embed && inst_embed && tgt && batch > 0 && nq > 0 && nkp > 0 && c > 0,
             "dp_query_build: bad arguments");
  DP_REQUIRE(pad == 0 || (label_enc && pose_enc && dn_label), "dp_query_build: DN slots need label_enc / pose_enc");
  const int64_t total = (int64_t)batch * (pad + nq) * (nkp + 1) * c;
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(query_build_kernel<bf16_t>, dim3(nblk(total, 256)), dim3(256), 0, s, tgt_embed, kp_embed,
                       inst_embed, label_enc, pose_enc, dn_label, pad, nq, nkp, c, total, (bf16_t*)tgt);
  else
    hipLaunchKernelGGL(query_build_kernel<float>, dim3(nblk(total, 256)), dim3(256), 0, s, tgt_embed, kp_embed,
                       inst_embed, label_enc, pose_enc, dn_label, pad, nq, nkp, c, total, (float*)tgt);
  return dp_check_launch("dp_query_build");
}

extern "C" int dp_query_build_bwd(const void* dtgt, const int32_t* dn_label, int32_t batch, int32_t pad, int32_t nq,
                                  int32_t nkp, int32_t c, float* g_tgt_embed, float* g_kp_embed, float* g_inst_embed,
                                  float* g_label_enc, int32_t n_label, float* g_pose_enc, int32_t dtype, void* stream) {
  DP_REQUIRE(dtgt && g_tgt_embed && g_kp_embed && g_inst_embed, "dp_query_build_bwd: null pointer");
  DP_REQUIRE(pad == 0 || dn_label, "dp_query_build_bwd: DN slots need dn_label");
  (void)n_label;
  // x blocks: 64 output elements each (tasks 0-3), or 64 * QB_W label_enc elements (task 4)
  int most = (nq * c + 63) / 64;
  if ((nkp * c + 63) / 64 > most) most = (nkp * c + 63) / 64;
  if (pad > 0 && (batch * pad * c + 64 * QB_W - 1) / (64 * QB_W) > most)
    most = (batch * pad * c + 64 * QB_W - 1) / (64 * QB_W);
  dim3 grid(most, pad > 0 ? 5 : 3);
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(query_build_bwd_kernel<bf16_t>, grid, dim3(64 * QB_W), 0, s, (const bf16_t*)dtgt, dn_label, batch,
                       pad, nq, nkp, c, g_tgt_embed, g_kp_embed, g_inst_embed, g_label_enc, g_pose_enc);
  else
    hipLaunchKernelGGL(query_build_bwd_kernel<float>, grid, dim3(64 * QB_W), 0, s, (const float*)dtgt, dn_label, batch,
                       pad, nq, nkp, c, g_tgt_embed, g_kp_embed, g_inst_embed, g_label_enc, g_pose_enc);
  return dp_check_launch("dp_query_build_bwd");
}

extern "C" int dp_pose_refine_bwd(const float* corners, const float* project, int32_t reg_max, float reg_scale,
                                  const float* dkps, int32_t rows, int32_t nkp, float* dcorners, int32_t accumulate,
                                  void* stream) {
  DP_REQUIRE(corners && project && dkps && dcorners && rows > 0 && nkp > 0, "dp_pose_refine_bwd: bad arguments");
  const int n = rows * nkp * 2;
  hipLaunchKernelGGL(pose_refine_bwd_kernel, dim3(nblk(n, 256)), dim3(256), 0, as_stream(stream), corners, project,
                     reg_max + 1, 1.f / fabsf(reg_scale), dkps, n, dcorners, accumulate);
  return dp_check_launch("dp_pose_refine_bwd");
}

extern "C" int dp_sigmoid_bwd(const float* out, const float* dout, float* din, int32_t rows, int32_t n, int64_t ld_out,
                              int64_t ld_dout, int64_t ld_din, void* stream) {
  DP_REQUIRE(out && dout && din && rows > 0 && n > 0, "dp_sigmoid_bwd: bad arguments");
  const int64_t tot = (int64_t)rows * n;
  hipLaunchKernelGGL(sigmoid_bwd_kernel, dim3(nblk(tot, 256)), dim3(256), 0, as_stream(stream), out, dout, din, rows,
                     n, ld_out, ld_dout, ld_din);
  return dp_check_launch("dp_sigmoid_bwd");
}

extern "C" int dp_lqe_stats_bwd(const void* feat, int64_t feat_bstride, int32_t h, int32_t w, int32_t c,
                                const float* kps, const float* dstats, int32_t batch, int32_t nq, int32_t nkp,
                                float* dkps, float* dfeat, int64_t dfeat_bstride, int32_t dtype, void* stream) {
  DP_REQUIRE(feat && kps && dstats && dkps, "dp_lqe_stats_bwd: null pointer");
  DP_REQUIRE(c % 64 == 0 && c / 64 >= 1 && c / 64 <= 8, "dp_lqe_stats_bwd: c=%d (64..512, multiple of 64)", c);
  const int total = batch * nq * nkp;
  hipStream_t s = as_stream(stream);
#define DP_LQEB(T_, E_)                                                                                         \
  case E_:                                                                                                      \
    hipLaunchKernelGGL((lqe_bwd_kernel<T_, E_>), dim3(nblk(total, 4)), dim3(256), 0, s, (const T_*)feat,        \
                       feat_bstride, h, w, c, kps, dstats, nq, nkp, total, dkps, dfeat, dfeat_bstride);         \
    break;
  if (dtype == DP_BF16) {
    switch (c / 64) { DP_LQEB(bf16_t, 1) DP_LQEB(bf16_t, 2) DP_LQEB(bf16_t, 3) DP_LQEB(bf16_t, 4) DP_LQEB(bf16_t, 5)
                      DP_LQEB(bf16_t, 6) DP_LQEB(bf16_t, 7) DP_LQEB(bf16_t, 8) }
  } else {
    switch (c / 64) { DP_LQEB(float, 1) DP_LQEB(float, 2) DP_LQEB(float, 3) DP_LQEB(float, 4) DP_LQEB(float, 5)
                      DP_LQEB(float, 6) DP_LQEB(float, 7) DP_LQEB(float, 8) }
  }
#undef DP_LQEB
  return dp_check_launch("dp_lqe_stats_bwd");
}

extern "C" int dp_scatter_rows(const void* src, int32_t ld_src, const int64_t* idx, const uint8_t* row_mask,
                               int32_t mask_period, int32_t batch, int32_t k, int32_t c, void* dst,
                               int64_t dst_bstride, int32_t ld_dst, int32_t accumulate, int32_t dtype, void* stream) {
  DP_REQUIRE(src && idx && dst && batch > 0 && k > 0 && c > 0 && (!row_mask || mask_period > 0),
             "dp_scatter_rows: bad arguments");
  const int64_t total = (int64_t)batch * k * c;
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(scatter_rows_kernel<bf16_t>, dim3(nblk(total, 256)), dim3(256), 0, s, (const bf16_t*)src, ld_src,
                       idx, row_mask, mask_period, k, c, (bf16_t*)dst, dst_bstride, ld_dst, accumulate, total);
  else
    hipLaunchKernelGGL(scatter_rows_kernel<float>, dim3(nblk(total, 256)), dim3(256), 0, s, (const float*)src, ld_src,
                       idx, row_mask, mask_period, k, c, (float*)dst, dst_bstride, ld_dst, accumulate, total);
  return dp_check_launch("dp_scatter_rows");
}

extern "C" int dp_gather_rows_masked(const void* src, int64_t src_bstride, const int64_t* idx, const uint8_t* row_mask,
                                     int32_t mask_period, int32_t batch, int32_t k, int32_t c, void* dst, int32_t dtype,
                                     void* stream) {
  DP_REQUIRE(src && idx && dst && batch > 0 && k > 0 && c > 0 && (!row_mask || mask_period > 0),
             "dp_gather_rows_masked: bad arguments");
  const int64_t total = (int64_t)batch * k * c;
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(gather_masked_kernel<bf16_t>, dim3(nblk(total, 256)), dim3(256), 0, s, (const bf16_t*)src,
                       src_bstride, idx, row_mask, mask_period, k, c, (bf16_t*)dst, total);
  else
    hipLaunchKernelGGL(gather_masked_kernel<float>, dim3(nblk(total, 256)), dim3(256), 0, s, (const float*)src,
                       src_bstride, idx, row_mask, mask_period, k, c, (float*)dst, total);
  return dp_check_launch("dp_gather_rows_masked");
}

extern "C" int dp_convert_rows(const void* src, int32_t src_dtype, int64_t ld_src, void* dst, int32_t dst_dtype,
                               int64_t ld_dst, int32_t rows, int32_t n, float scale, int32_t accumulate, void* stream) {
  DP_REQUIRE(src && dst && rows > 0 && n > 0, "dp_convert_rows: bad arguments");
  const int64_t tot = (int64_t)rows * n;
  hipStream_t s = as_stream(stream);
  dim3 grid(nblk(tot, 256)), block(256);
  if (src_dtype == DP_BF16 && dst_dtype == DP_BF16)
    hipLaunchKernelGGL((convert_kernel<bf16_t, bf16_t>), grid, block, 0, s, (const bf16_t*)src, ld_src, (bf16_t*)dst,
                       ld_dst, rows, n, scale, accumulate);
  else if (src_dtype == DP_BF16)
    hipLaunchKernelGGL((convert_kernel<bf16_t, float>), grid, block, 0, s, (const bf16_t*)src, ld_src, (float*)dst,
                       ld_dst, rows, n, scale, accumulate);
  else if (dst_dtype == DP_BF16)
    hipLaunchKernelGGL((convert_kernel<float, bf16_t>), grid, block, 0, s, (const float*)src, ld_src, (bf16_t*)dst,
                       ld_dst, rows, n, scale, accumulate);
  else
    hipLaunchKernelGGL((convert_kernel<float, float>), grid, block, 0, s, (const float*)src, ld_src, (float*)dst,
                       ld_dst, rows, n, scale, accumulate);
  return dp_check_launch("dp_convert_rows");
}

// ---------------------------------------------------------------- batched f32 row copies
// One launch for a table of strided f32 row copies (the criterion's head packing and its
// gradient hand-off: ~70 small dp_convert_rows launches per sub-batch before). Block (x, e)
// strides over entry e's rows x n elements; dst = src0 (+ src1): the same f32 sum as a copy
// followed by an accumulating dp_convert_rows (a + b == b + a in f32).
__global__ void copy_rows_batch_kernel(const dp_rowcopy_desc* __restrict__ tab) {
  const dp_rowcopy_desc d = tab[blockIdx.y];
  const unsigned tot = (unsigned)d.rows * (unsigned)d.n, un = (unsigned)d.n;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
    const unsigned r = e / un, j = e - r * un;
    float v = d.src0[(int64_t)r * d.ld_src0 + j];
    if (d.src1) v += d.src1[(int64_t)r * d.ld_src1 + j];
    d.dst[(int64_t)r * d.ld_dst + j] = v;
  }
}

extern "C" int dp_copy_rows_check(const dp_rowcopy_desc* tab, int32_t n) {
  DP_REQUIRE(tab && n > 0 && n < 65536, "dp_copy_rows_check: bad table");
  for (int i = 0; i < n; ++i) {
    const dp_rowcopy_desc& d = tab[i];
    const bool ok = d.src0 && d.dst && d.rows > 0 && d.n > 0 && (int64_t)d.rows * d.n < (1ll << 31) &&
                    d.ld_src0 >= d.n && d.ld_dst >= d.n && (!d.src1 || d.ld_src1 >= d.n);
    DP_REQUIRE(ok, "dp_copy_rows_check: entry %d (rows %d, n %d, ld %lld / %lld / %lld)", i, d.rows, d.n,
               (long long)d.ld_src0, (long long)d.ld_src1, (long long)d.ld_dst);
  }
  return 0;
}

extern "C" int dp_copy_rows_batch(const dp_rowcopy_desc* tab_dev, int32_t n, int32_t blocks_per_entry, void* stream) {
  DP_REQUIRE(tab_dev && n > 0 && n < 65536 && blocks_per_entry > 0, "dp_copy_rows_batch: bad arguments");
  hipLaunchKernelGGL(copy_rows_batch_kernel, dim3((unsigned)blocks_per_entry, (unsigned)n), dim3(256), 0,
                     as_stream(stream), tab_dev);
  return dp_check_launch("dp_copy_rows_batch");
}

extern "C" int dp_cdn_build(const int32_t* tgt_off, const int32_t* tgt_label, const float* tgt_kps,
                            const float* tgt_area, const float* tgt_boxes, const float* sigmas, int32_t batch,
                            int32_t pad, int32_t single_pad, int32_t nkp, float label_noise_ratio, int32_t num_classes,
                            float img_h, float img_w, uint64_t seed, int32_t* dn_label, float* dn_ref, void* stream) {
  DP_REQUIRE(tgt_off && dn_label && dn_ref && sigmas && batch > 0 && pad > 0 && single_pad > 0 && pad % single_pad == 0,
             "dp_cdn_build: bad arguments");
  const int64_t total = (int64_t)batch * pad * (nkp + 1);
  hipLaunchKernelGGL(cdn_build_kernel, dim3(nblk(total, 256)), dim3(256), 0, as_stream(stream), tgt_off, tgt_label,
                     tgt_kps, tgt_area, tgt_boxes, sigmas, batch, pad, single_pad, nkp, label_noise_ratio, num_classes,
                     img_h, img_w, seed, dn_label, dn_ref);
  return dp_check_launch("dp_cdn_build");
}

extern "C" int64_t dp_grad_sqnorm_ws_floats(int64_t n) {
  return n > 0 ? std::min<int64_t>((n + 255) / 256, DP_SQNORM_PARTS) : 0;
}

extern "C" int dp_grad_sqnorm(const float* g, int64_t n, float* out, float* ws, int64_t ws_floats, void* stream) {
  DP_REQUIRE(g && out && ws && n > 0, "dp_grad_sqnorm: bad arguments");
  const int64_t grid = dp_grad_sqnorm_ws_floats(n);
  DP_REQUIRE(ws_floats >= grid, "dp_grad_sqnorm: workspace holds %lld floats, needs dp_grad_sqnorm_ws_floats(n) = %lld",
             (long long)ws_floats, (long long)grid);
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(sqnorm_kernel, dim3((int)grid), dim3(256), 0, s, g, n, ws);
  hipLaunchKernelGGL(sqnorm_final_kernel, dim3(1), dim3(256), 0, s, ws, (int)grid, out);
  return dp_check_launch("dp_grad_sqnorm");
}

extern "C" int dp_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                        float beta1, float beta2, float eps, float weight_decay, int32_t step, float max_norm,
                        const float* grad_sqnorm, const float* skip, void* stream) {
  DP_REQUIRE(param && grad && exp_avg && exp_avg_sq && n > 0 && step > 0, "dp_adamw: bad arguments");
  DP_REQUIRE(max_norm <= 0.f || grad_sqnorm, "dp_adamw: clipping needs the gradient's squared norm");
  const float bc1 = 1.f - powf(beta1, (float)step), bc2 = 1.f - powf(beta2, (float)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(nblk(n, 256)), dim3(256), 0, as_stream(stream), param, grad, exp_avg,
                     exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, bc1, bc2, max_norm, grad_sqnorm, skip);
  return dp_check_launch("dp_adamw");
}

extern "C" int dp_finite_guard(const float* v, int64_t n, float* bad, void* stream) {
  DP_REQUIRE(v && bad && n > 0, "dp_finite_guard: bad arguments");
  hipLaunchKernelGGL(finite_guard_kernel, dim3(1), dim3(256), 0, as_stream(stream), v, n, bad);
  return dp_check_launch("dp_finite_guard");
}

extern "C" int dp_ema(float* ema, const float* p, int64_t n, float decay, const float* skip, void* stream) {
  DP_REQUIRE(ema && p && n > 0, "dp_ema: bad arguments");
  hipLaunchKernelGGL(ema_kernel, dim3(nblk(n, 256)), dim3(256), 0, as_stream(stream), ema, p, n, decay, skip);
  return dp_check_launch("dp_ema");
}

// Zero fill as a kernel (16-byte stores over the aligned body): every stream-ordered clear of the
// library goes through here instead of hipMemsetAsync, whose nodes inside a captured hipGraph
// (the training tapes' replay) left the cleared buffers wrong in measured runs.
__global__ void zero_fill_kernel(char* __restrict__ p, size_t bytes) {
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15;
  const size_t h = head < bytes ? head : bytes;
  const size_t body = (bytes - h) / 16;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  if (i0 < h) p[i0] = 0;
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t* b = reinterpret_cast<u32x4_t*>(p + h);
  // streaming stores: the zeroed buffers are accumulated into much later in the tape
  for (size_t i = i0; i < body; i += st) __builtin_nontemporal_store(u32x4_t{0u, 0u, 0u, 0u}, b + i);
  const size_t tail = h + body * 16;
  if (tail + i0 < bytes) p[tail + i0] = 0;
}

int dp_zero_async(void* p, size_t bytes, hipStream_t s) {
  if (!bytes) return 0;
  const size_t body = bytes / 16 + 1;
  const unsigned grid = (unsigned)std::min<size_t>((body + 255) / 256, 16384);
  hipLaunchKernelGGL(zero_fill_kernel, dim3(grid), dim3(256), 0, s, static_cast<char*>(p), bytes);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dp_zero(void* p, int64_t bytes, void* stream) {
  DP_REQUIRE(p && bytes >= 0, "dp_zero: bad arguments");
  if (dp_zero_async(p, (size_t)bytes, as_stream(stream))) return dp_check_launch("dp_zero");
  return 0;
}
