// Short-sequence multi-head attention core: softmax(Q K^T / sqrt(dh)) V per head.
//
// The three attention shapes on the DETRPose path are tiny and many:
//   within-instance  (transformer.py:403-406): seq 18 (1 instance + 17 keypoints), B*60 seqs
//   across-instance  (transformer.py:411-419): seq 60 (queries),                  B*18 seqs
//   AIFI             (hybrid_encoder.py:276-279): seq 400 (20x20 tokens),         B seqs
// so one (sequence, head) pair is far too small for an MFMA tile. Each thread owns one
// query row (q and the output accumulator in registers); a 256-thread block packs
// P = 256/seq_tile (sequence, head) pairs and stages their K/V in LDS in key chunks,
// with a chunk-wise online softmax (chunk max first, one rescale per chunk).
// Token t of sequence (o, i) is row o*so + i*si + t*st of the projection outputs, so
// the across-instance transpose of the reference (transformer.py:409,419) is only an
// index change here.
#include "common.h"
#include <stdlib.h>

namespace {

template <typename T, int DH>
__global__ __launch_bounds__(256) void attn_kernel(const T* __restrict__ q, int ld_q, const T* __restrict__ k,
                                                   const T* __restrict__ v, int ld_kv, T* __restrict__ out, int ld_o,
                                                   int n_inner, int64_t so, int64_t si, int64_t st, int seqlen,
                                                   int nhead, int npairs, int qpb, int P, int KC, float scale) {
  extern __shared__ float sm[];
  float* Ks = sm;                 // [P][KC][DH]
  float* Vs = sm + P * KC * DH;   // [P][KC][DH]
  const int tid = threadIdx.x;
  const int p = tid / qpb;
  const int qi = blockIdx.y * qpb + (tid - p * qpb);
  const int pair = blockIdx.x * P + p;
  const bool active = p < P && pair < npairs && qi < seqlen;

  auto row_of = [&](int pr, int t) -> int64_t {
    const int h = pr % nhead, s = pr / nhead;
    const int o = s / n_inner, i = s - o * n_inner;
    return (int64_t)o * so + (int64_t)i * si + (int64_t)t * st;
  };

  float qr[DH], acc[DH];
  float m = -INFINITY, l = 0.f;
  int h = 0;
  if (active) {
    h = pair % nhead;
    const T* qp = q + row_of(pair, qi) * ld_q + h * DH;
#pragma unroll
    for (int d = 0; d < DH; ++d) qr[d] = to_f32(qp[d]) * scale;
  }
#pragma unroll
  for (int d = 0; d < DH; ++d) acc[d] = 0.f;

  for (int c0 = 0; c0 < seqlen; c0 += KC) {
    const int kl = min(KC, seqlen - c0);
    __syncthreads();
    for (int e = tid; e < P * kl * DH; e += blockDim.x) {
      const int pp = e / (kl * DH);
      const int rem = e - pp * kl * DH;
      const int t = rem / DH, d = rem - t * DH;
      const int pr = blockIdx.x * P + pp;
      float kv = 0.f, vv = 0.f;
      if (pr < npairs) {
        const int64_t off = row_of(pr, c0 + t) * ld_kv + (pr % nhead) * DH + d;
        kv = to_f32(k[off]);
        vv = to_f32(v[off]);
      }
      Ks[(pp * KC + t) * DH + d] = kv;
      Vs[(pp * KC + t) * DH + d] = vv;
    }
    __syncthreads();
    if (!active) continue;
    const float* kp = Ks + p * KC * DH;
    const float* vp = Vs + p * KC * DH;
    float cm = -INFINITY;
    for (int t = 0; t < kl; ++t) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s = fmaf(qr[d], kp[t * DH + d], s);
      cm = fmaxf(cm, s);
    }
    const float mn = fmaxf(m, cm);
    const float corr = __expf(m - mn);
    l *= corr;
#pragma unroll
    for (int d = 0; d < DH; ++d) acc[d] *= corr;
    m = mn;
    for (int t = 0; t < kl; ++t) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s = fmaf(qr[d], kp[t * DH + d], s);
      const float pw = __expf(s - m);
      l += pw;
#pragma unroll
      for (int d = 0; d < DH; ++d) acc[d] = fmaf(pw, vp[t * DH + d], acc[d]);
    }
  }
  if (!active) return;
  const float inv = 1.f / l;
  T* op = out + row_of(pair, qi) * ld_o + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) op[d] = from_f32<T>(acc[d] * inv);
}

template <typename T, int DH>
int launch(const void* q, int ld_q, const void* k, const void* v, int ld_kv, void* out, int ld_o, int n_outer,
           int n_inner, int64_t so, int64_t si, int64_t st, int seqlen, int nhead, hipStream_t s) {
  const int ntiles = (seqlen + 255) / 256;
  const int qpb = (seqlen + ntiles - 1) / ntiles;
  const int P = 256 / qpb;
  const int npairs = n_outer * n_inner * nhead;
  int KC = 65536 / (2 * P * DH * 4);
  KC = KC < seqlen ? KC : seqlen;
  const size_t lds = (size_t)2 * P * KC * DH * sizeof(float);
  dim3 grid((unsigned)((npairs + P - 1) / P), (unsigned)ntiles), block(256);
  hipLaunchKernelGGL((attn_kernel<T, DH>), grid, block, lds, s, (const T*)q, ld_q, (const T*)k, (const T*)v, ld_kv,
                     (T*)out, ld_o, n_inner, so, si, st, seqlen, nhead, npairs, qpb, P, KC, 1.f / sqrtf((float)DH));
  return dp_check_launch("dp_attention");
}

template <typename T>
int dispatch(const void* q, int ld_q, const void* k, const void* v, int ld_kv, void* out, int ld_o, int n_outer,
             int n_inner, int64_t so, int64_t si, int64_t st, int seqlen, int nhead, int dh, hipStream_t s) {
  switch (dh) {
    case 16: return launch<T, 16>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    case 32: return launch<T, 32>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    case 48: return launch<T, 48>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    default: dp_set_error("dp_attention: head dim %d not supported (16/32/48)", dh); return DP_EINVAL;
  }
}


// ---------------------------------------------------------------------------------
// bf16 MFMA path. One wave = one (sequence, head, 64-query block). S = Q K^T runs on
// v_mfma_f32_16x16x32_bf16 with Q (A operand, query rows) and K (B operand, key rows)
// loaded straight from global in fragment layout; softmax is online over 64-key blocks
// with the row max / row sum reduced across the 16 lanes that share a row; P (bf16) and
// V^T go through the wave's private LDS slice to become the A / B operands of O = P V.
// No block-level synchronisation: the 4 waves of a block are independent work items.
constexpr int AP = 72;  // LDS pitch (elements) of P [64][AP] and V^T [DH][AP]

template <int DH>
__global__ __launch_bounds__(256) void attn_mfma_kernel(const bf16_t* __restrict__ q, int ld_q,
                                                        const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                        int ld_kv, bf16_t* __restrict__ out, int ld_o, int n_inner,
                                                        int64_t so, int64_t si, int64_t st, int seqlen, int nhead,
                                                        int npairs, int nqb, float scale) {
  constexpr int KS = (DH + 31) / 32;   // 32-wide k-steps over the head dim (zero padded)
  constexpr int ND = DH / 16;          // 16-wide output column tiles
  __shared__ __attribute__((aligned(16))) bf16_t lds[4][(64 + DH) * AP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wave;
  if (item >= npairs * nqb) return;
  const int pair = item / nqb, qb = item - pair * nqb;
  const int h = pair % nhead, sq = pair / nhead;
  const int o = sq / n_inner, ii = sq - o * n_inner;
  const int64_t base = (int64_t)o * so + (int64_t)ii * si;
  bf16_t* Ps = lds[wave];            // [64][AP]  P (query rows x keys)
  bf16_t* Vt = lds[wave] + 64 * AP;  // [DH][AP]  V^T (head dims x keys)
  const int lr = lane & 15, lg = lane >> 4;

  bf16x8 qf[4][KS];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = qb * 64 + 16 * i + lr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 32 * ks + 8 * lg;
      if (qi < seqlen && d0 < DH)
        qf[i][ks] = *reinterpret_cast<const bf16x8*>(q + (base + (int64_t)qi * st) * ld_q + h * DH + d0);
      else
        qf[i][ks] = bf16x8{};
    }
  }
  f32x4 oacc[4][ND];
  float mrow[4][4], lrow[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < ND; ++j) oacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mrow[i][r] = -INFINITY;
      lrow[i][r] = 0.f;
    }
  }
  const int nkb = (seqlen + 63) / 64;
  for (int kb = 0; kb < nkb; ++kb) {
    // ---- S = Q K^T
    f32x4 sacc[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kj = kb * 64 + 16 * j + lr;
      bf16x8 kf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 32 * ks + 8 * lg;
        if (kj < seqlen && d0 < DH)
          kf[ks] = *reinterpret_cast<const bf16x8*>(k + (base + (int64_t)kj * st) * ld_kv + h * DH + d0);
        else
          kf[ks] = bf16x8{};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[i][ks], kf[ks], a, 0, 0, 0);
        sacc[i][j] = a;
      }
    }
    // ---- V block -> V^T in LDS (keys beyond seqlen are zero)
    constexpr int VCH = DH / 8;  // 16-byte chunks per key row
#pragma unroll
    for (int t = 0; t < VCH; ++t) {
      const int c = lane + 64 * t;
      const int key = c / VCH, dc = c - key * VCH;
      const int kg = kb * 64 + key;
      bf16x8 vv = bf16x8{};
      if (kg < seqlen) vv = *reinterpret_cast<const bf16x8*>(v + (base + (int64_t)kg * st) * ld_kv + h * DH + dc * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(dc * 8 + e) * AP + key] = vv[e];
    }
    // ---- online softmax over this key block
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kj = kb * 64 + 16 * j + lr;
          const float sv = kj < seqlen ? sacc[i][j][r] * scale : -INFINITY;
          sacc[i][j][r] = sv;
          mx = fmaxf(mx, sv);
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        const float mn = fmaxf(mrow[i][r], mx);
        const float corr = __expf(mrow[i][r] - mn);
        mrow[i][r] = mn;
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = __expf(sacc[i][j][r] - mn);
          sum += p;
          Ps[(16 * i + 4 * lg + r) * AP + 16 * j + lr] = (bf16_t)p;
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
        lrow[i][r] = lrow[i][r] * corr + sum;
#pragma unroll
        for (int jd = 0; jd < ND; ++jd) oacc[i][jd][r] *= corr;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // ---- O += P V
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pf[4], vf[ND];
#pragma unroll
      for (int i = 0; i < 4; ++i) pf[i] = *reinterpret_cast<const bf16x8*>(Ps + (16 * i + lr) * AP + 32 * ks + 8 * lg);
#pragma unroll
      for (int jd = 0; jd < ND; ++jd)
        vf[jd] = *reinterpret_cast<const bf16x8*>(Vt + (16 * jd + lr) * AP + 32 * ks + 8 * lg);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jd = 0; jd < ND; ++jd)
          oacc[i][jd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf[i], vf[jd], oacc[i][jd], 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // ---- normalise and store (row = query, lane column = head dim)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = qb * 64 + 16 * i + 4 * lg + r;
      if (qi >= seqlen) continue;
      const float inv = 1.f / lrow[i][r];
      bf16_t* op = out + (base + (int64_t)qi * st) * ld_o + h * DH;
#pragma unroll
      for (int jd = 0; jd < ND; ++jd) op[16 * jd + lr] = (bf16_t)(oacc[i][jd][r] * inv);
    }
  }
}


// ---------------------------------------------------------------------------------
// bf16 short-sequence path (seq <= 16*KT, the decoder's within-instance 18 and
// across-instance 60): one wave per (sequence, head), no online softmax, no LDS for P.
//  * S^T = K Q^T on v_mfma_f32_16x16x32_bf16 (K as the A operand, Q as B, both loaded in
//    fragment layout straight from the projection rows), so lane (lr, lg) of tile (j, i)
//    holds S^T[key 16j+4lg+r][query 16i+lr]: the softmax axis (keys) sits in the lane's
//    registers and across the 4 lane groups (2 xor-shuffles per reduction).
//  * O^T = V^T P^T: the lane's P values of tiles (2m, 2m+1) ARE its B fragment for the
//    32-key step m, with k-slot s <-> key 32m + (s < 4 ? 4lg+s : 16+4lg+s-4); the A fragment
//    (V^T in the same k order) comes from V staged row-major in LDS through two
//    ds_read_b64_tr_b16 per (m, 16 head-dim rows): group lg reads the 4x16 blocks at keys
//    32m+4lg and 32m+16+4lg, delivered column-major (row pitch chosen bank-conflict free).
//  * Output: lane holds O^T[dh 16d+4lg+r][query 16i+lr] -> 8-byte stores of 4 channels.
// Padded keys get S = -inf and zero V rows; padded queries are computed and not stored.
template <int DH, int KT>
__global__ __launch_bounds__(256) void attn_short_kernel(const bf16_t* __restrict__ q, int ld_q,
                                                         const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                         int ld_kv, bf16_t* __restrict__ out, int ld_o, int n_inner,
                                                         int64_t so, int64_t si, int64_t st, int seqlen, int nhead,
                                                         int npairs, float scale) {
  constexpr int KS = (DH + 31) / 32;             // 32-deep k-steps over the head dim
  constexpr int ND = DH / 16;                    // 16-row head-dim tiles of O^T
  constexpr int NK = 16 * KT;                    // padded keys (= padded queries)
  constexpr int DHP = DH == 16 ? 16 : 48;        // V row pitch (elements): conflict-free tr reads
  constexpr int VCH = DH / 8;                    // 16-byte chunks per V row
  typedef short s4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) bf16_t vl[4][NK * DHP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pair = blockIdx.x * 4 + wave;
  if (pair >= npairs) return;                    // wave-uniform: EXEC stays full below
  const int h = pair % nhead, sq = pair / nhead;
  const int o = sq / n_inner, ii = sq - o * n_inner;
  const int64_t base = (int64_t)o * so + (int64_t)ii * si;
  const int lr = lane & 15, lg = lane >> 4;
  bf16_t* V = vl[wave];

  // V rows -> LDS (row-major, zero rows past seqlen)
#pragma unroll
  for (int t = 0; t < (NK * VCH + 63) / 64; ++t) {
    const int c = lane + 64 * t;
    if (c < NK * VCH) {
      const int key = c / VCH, dc = c - key * VCH;
      bf16x8 vv = bf16x8{};
      if (key < seqlen) vv = *reinterpret_cast<const bf16x8*>(v + (base + (int64_t)key * st) * ld_kv + h * DH + dc * 8);
      *reinterpret_cast<bf16x8*>(V + key * DHP + dc * 8) = vv;
    }
  }
  // Q (B operand, query columns) and K (A operand, key rows) fragments
  bf16x8 qf[KT][KS], kf[KT][KS];
#pragma unroll
  for (int i = 0; i < KT; ++i)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int row = 16 * i + lr, d0 = 32 * ks + 8 * lg;
      const bool ok = row < seqlen && d0 < DH;
      const int64_t rb = base + (int64_t)row * st;
      qf[i][ks] = ok ? *reinterpret_cast<const bf16x8*>(q + rb * ld_q + h * DH + d0) : bf16x8{};
      kf[i][ks] = ok ? *reinterpret_cast<const bf16x8*>(k + rb * ld_kv + h * DH + d0) : bf16x8{};
    }
  // S^T tiles
  f32x4 s[KT][KT];   // [j key tile][i query tile]
#pragma unroll
  for (int j = 0; j < KT; ++j)
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[j][ks], qf[i][ks], a, 0, 0, 0);
      s[j][i] = a;
    }
  // softmax over keys for each query column (lane lr of tile i)
  float inv[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < KT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * j + 4 * lg + r;
        const float x = key < seqlen ? s[j][i][r] * scale : -INFINITY;
        s[j][i][r] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < KT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[j][i][r] - mx);
        s[j][i][r] = p;
        sum += p;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    inv[i] = 1.f / sum;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // O^T = V^T P^T over 32-key steps
  f32x4 oacc[ND][KT];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int i = 0; i < KT; ++i) oacc[d][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q4 = (lane & 15) >> 2, p4 = lane & 3;   // tr-read address roles within the 16-lane group
#pragma unroll
  for (int m = 0; m < KT / 2; ++m) {
    bf16x8 pf[KT];
#pragma unroll
    for (int i = 0; i < KT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[i][r] = (bf16_t)s[2 * m][i][r];
        pf[i][4 + r] = (bf16_t)s[2 * m + 1][i][r];
      }
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      const bf16_t* a0 = V + (32 * m + 4 * lg + q4) * DHP + 16 * d + 4 * p4;
      const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
      const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0 + 16 * DHP));
      bf16x8 vf;
      short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      vf = *reinterpret_cast<const bf16x8*>(tmp);
#pragma unroll
      for (int i = 0; i < KT; ++i) oacc[d][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[i], oacc[d][i], 0, 0, 0);
    }
  }
  // store: query 16i+lr, channels 16d + 4lg .. +3 (8 bytes)
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    const int qi = 16 * i + lr;
    if (qi >= seqlen) continue;
    bf16_t* op = out + (base + (int64_t)qi * st) * ld_o + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16_t)(oacc[d][i][r] * inv[i]);
      *reinterpret_cast<bf16x4*>(op + 16 * d + 4 * lg) = w;
    }
  }
}

// ---------------------------------------------------------------------------------
// bf16 long-sequence path (AIFI's 400 tokens): attn_short_kernel's register scheme with an
// online softmax over 64-key blocks. One wave = one (sequence, head, 64-query block).
//  * S^T = K Q^T per key block (K rows as the A operand straight from the projection rows),
//    so the lane holds S^T[key 16j+4lg+r][query 16i+lr]: the running max / sum of query
//    column (i, lr) reduce over its registers and 2 xor-shuffles (16, 32); no LDS for P.
//  * O^T += V^T P^T: P (bf16) from registers is the B operand; V^T fragments come from the
//    block's V rows staged row-major in the wave's LDS slice with 16-byte stores and read
//    back transposed by ds_read_b64_tr_b16 (the previous kernel transposed V with 2-byte
//    scalar LDS stores: 24 % of its LDS cycles were bank conflicts).
//  * The 64-query block's O^T accumulators are rescaled by exp(m_old - m_new) per block.
template <int DH>
__global__ __launch_bounds__(256) void attn_long_kernel(const bf16_t* __restrict__ q, int ld_q,
                                                        const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
                                                        int ld_kv, bf16_t* __restrict__ out, int ld_o, int n_inner,
                                                        int64_t so, int64_t si, int64_t st, int seqlen, int nhead,
                                                        int npairs, int nqb, float scale) {
  constexpr int KT = 4;                          // 16-row tiles per 64 queries / 64 keys
  constexpr int KS = (DH + 31) / 32;
  constexpr int ND = DH / 16;
  constexpr int DHP = DH == 16 ? 16 : 48;        // V row pitch (elements): conflict-free tr reads
  constexpr int VCH = DH / 8;
  typedef short s4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) bf16_t vl[4][64 * DHP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + wave;
  if (item >= npairs * nqb) return;              // wave-uniform: EXEC stays full below
  const int pair = item / nqb, qb = item - pair * nqb;
  const int h = pair % nhead, sq = pair / nhead;
  const int o = sq / n_inner, ii = sq - o * n_inner;
  const int64_t base = (int64_t)o * so + (int64_t)ii * si;
  const int lr = lane & 15, lg = lane >> 4;
  bf16_t* V = vl[wave];

  bf16x8 qf[KT][KS];   // B operand: query columns
#pragma unroll
  for (int i = 0; i < KT; ++i)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int row = qb * 64 + 16 * i + lr, d0 = 32 * ks + 8 * lg;
      qf[i][ks] = (row < seqlen && d0 < DH)
                      ? *reinterpret_cast<const bf16x8*>(q + (base + (int64_t)row * st) * ld_q + h * DH + d0)
                      : bf16x8{};
    }
  f32x4 oacc[ND][KT];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int i = 0; i < KT; ++i) oacc[d][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[KT], lrow[KT];
#pragma unroll
  for (int i = 0; i < KT; ++i) mrow[i] = -INFINITY, lrow[i] = 0.f;
  const int q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int nkb = (seqlen + 63) / 64;
  constexpr int VT = (64 * VCH + 63) / 64;       // V chunks per lane per key block
  // K fragments and V chunks of one key block
  struct Blk {
    bf16x8 kf[KT][KS];
    bf16x8 vv[VT];
  };
  auto load_blk = [&](int kb, Blk& bk) __attribute__((always_inline)) {
    const int k0 = kb * 64;
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int row = k0 + 16 * j + lr;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int d0 = 32 * ks + 8 * lg;
        bk.kf[j][ks] = (row < seqlen && d0 < DH)
                           ? *reinterpret_cast<const bf16x8*>(k + (base + (int64_t)row * st) * ld_kv + h * DH + d0)
                           : bf16x8{};
      }
    }
#pragma unroll
    for (int t = 0; t < VT; ++t) {
      const int c = lane + 64 * t;
      const int key = c / VCH, dc = c - key * VCH;
      bk.vv[t] = (c < 64 * VCH && k0 + key < seqlen)
                     ? *reinterpret_cast<const bf16x8*>(v + (base + (int64_t)(k0 + key) * st) * ld_kv + h * DH + dc * 8)
                     : bf16x8{};
    }
  };
  auto run_blk = [&](int kb, const Blk& bk) __attribute__((always_inline)) {
    const int k0 = kb * 64;
    // V rows -> LDS (the previous block's tr reads are done: wave barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int t = 0; t < VT; ++t) {
      const int c = lane + 64 * t;
      const int key = c / VCH, dc = c - key * VCH;
      if (c < 64 * VCH) *reinterpret_cast<bf16x8*>(V + key * DHP + dc * 8) = bk.vv[t];
    }
    f32x4 sv[KT][KT];   // S^T: [j key tile][i query tile]
#pragma unroll
    for (int j = 0; j < KT; ++j)
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bk.kf[j][ks], qf[i][ks], a, 0, 0, 0);
        sv[j][i] = a;
      }
    // online softmax per query column
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < KT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 16 * j + 4 * lg + r;
          const float x = key < seqlen ? sv[j][i][r] * scale : -INFINITY;
          sv[j][i][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(mrow[i], mx);
      const float corr = __expf(mrow[i] - mn);
      mrow[i] = mn;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < KT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __expf(sv[j][i][r] - mn);
          sv[j][i][r] = pv;
          sum += pv;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      lrow[i] = lrow[i] * corr + sum;
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) oacc[d][i][r] *= corr;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // O^T += V^T P^T over the block's two 32-key steps
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      bf16x8 pf[KT];
#pragma unroll
      for (int i = 0; i < KT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pf[i][r] = (bf16_t)sv[2 * m][i][r];
          pf[i][4 + r] = (bf16_t)sv[2 * m + 1][i][r];
        }
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const bf16_t* a0 = V + (32 * m + 4 * lg + q4) * DHP + 16 * d + 4 * p4;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0));
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(a0 + 16 * DHP));
        short tmp[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(tmp);
#pragma unroll
        for (int i = 0; i < KT; ++i) oacc[d][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[i], oacc[d][i], 0, 0, 0);
      }
    }
  };
  // one key block at a time: prefetching the next block's K/V into registers (two Blk
  // buffers, kb loop unrolled by two) pushed the kernel to 255 VGPRs and measured slower
  // (74 -> 82 us at L b64); the 3-4 waves per SIMD hide the load latency instead
  Blk bk;
  for (int kb = 0; kb < nkb; ++kb) {
    load_blk(kb, bk);
    run_blk(kb, bk);
  }
  // store: query 16i+lr of the block, channels 16d + 4lg .. +3 (8 bytes)
#pragma unroll
  for (int i = 0; i < KT; ++i) {
    const int qi = qb * 64 + 16 * i + lr;
    if (qi >= seqlen) continue;
    const float inv = 1.f / lrow[i];
    bf16_t* op = out + (base + (int64_t)qi * st) * ld_o + h * DH;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      bf16x4 w;
#pragma unroll
      for (int r = 0; r < 4; ++r) w[r] = (bf16_t)(oacc[d][i][r] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * d + 4 * lg) = w;
    }
  }
}

template <int DH>
int launch_long(const void* q, int ld_q, const void* k, const void* v, int ld_kv, void* out, int ld_o, int n_outer,
                int n_inner, int64_t so, int64_t si, int64_t st, int seqlen, int nhead, hipStream_t s) {
  const int npairs = n_outer * n_inner * nhead;
  const int nqb = (seqlen + 63) / 64;
  const int64_t items = (int64_t)npairs * nqb;
  hipLaunchKernelGGL((attn_long_kernel<DH>), dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, (const bf16_t*)q,
                     ld_q, (const bf16_t*)k, (const bf16_t*)v, ld_kv, (bf16_t*)out, ld_o, n_inner, so, si, st, seqlen,
                     nhead, npairs, nqb, 1.f / sqrtf((float)DH));
  return dp_check_launch("dp_attention(long)");
}

template <int DH, int KT>
int launch_short(const void* q, int ld_q, const void* k, const void* v, int ld_kv, void* out, int ld_o, int n_outer,
                 int n_inner, int64_t so, int64_t si, int64_t st, int seqlen, int nhead, hipStream_t s) {
  const int npairs = n_outer * n_inner * nhead;
  dim3 grid((unsigned)((npairs + 3) / 4)), block(256);
  hipLaunchKernelGGL((attn_short_kernel<DH, KT>), grid, block, 0, s, (const bf16_t*)q, ld_q, (const bf16_t*)k,
                     (const bf16_t*)v, ld_kv, (bf16_t*)out, ld_o, n_inner, so, si, st, seqlen, nhead, npairs,
                     1.f / sqrtf((float)DH));
  return dp_check_launch("dp_attention(short)");
}

template <int DH>
int launch_short_any(const void* q, int ld_q, const void* k, const void* v, int ld_kv, void* out, int ld_o,
                     int n_outer, int n_inner, int64_t so, int64_t si, int64_t st, int seqlen, int nhead,
                     hipStream_t s) {
  if (seqlen <= 32)
    return launch_short<DH, 2>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
  return launch_short<DH, 4>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
}

template <int DH>
int launch_mfma(const void* q, int ld_q, const void* k, const void* v, int ld_kv, void* out, int ld_o, int n_outer,
                int n_inner, int64_t so, int64_t si, int64_t st, int seqlen, int nhead, hipStream_t s) {
  const int npairs = n_outer * n_inner * nhead;
  const int nqb = (seqlen + 63) / 64;
  const int64_t items = (int64_t)npairs * nqb;
  dim3 grid((unsigned)((items + 3) / 4)), block(256);
  hipLaunchKernelGGL((attn_mfma_kernel<DH>), grid, block, 0, s, (const bf16_t*)q, ld_q, (const bf16_t*)k,
                     (const bf16_t*)v, ld_kv, (bf16_t*)out, ld_o, n_inner, so, si, st, seqlen, nhead, npairs, nqb,
                     1.f / sqrtf((float)DH));
  return dp_check_launch("dp_attention");
}

}  // namespace

extern "C" int dp_attention(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, void* out,
                            int32_t ld_o, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si, int64_t st,
                            int32_t seqlen, int32_t nhead, int32_t dh, int32_t dtype, void* stream) {
  DP_REQUIRE(q && k && v && out, "dp_attention: null pointer");
  DP_REQUIRE(seqlen > 0 && n_outer > 0 && n_inner > 0 && nhead > 0, "dp_attention: bad shape");
  hipStream_t s = as_stream(stream);
  const bool al = ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) | reinterpret_cast<uintptr_t>(v)) &
                   15) == 0 && ld_q % 8 == 0 && ld_kv % 8 == 0;
  const bool al8 = ((reinterpret_cast<uintptr_t>(out) & 7) == 0) && ld_o % 4 == 0;
  static const bool no_short = getenv("DETRPOSE_ATTN_NO_SHORT") != nullptr;
  if (dtype == DP_BF16 && al && al8 && seqlen <= 64 && !no_short) {
    if (dh == 16) return launch_short_any<16>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    if (dh == 32) return launch_short_any<32>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    if (dh == 48) return launch_short_any<48>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
  }
  static const bool no_long = getenv("DETRPOSE_ATTN_NO_LONG") != nullptr;   // A/B: the LDS-P kernel
  if (dtype == DP_BF16 && al && al8 && !no_long) {
    if (dh == 16) return launch_long<16>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    if (dh == 32) return launch_long<32>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    if (dh == 48) return launch_long<48>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
  }
  if (dtype == DP_BF16 && al) {
    if (dh == 16) return launch_mfma<16>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    if (dh == 32) return launch_mfma<32>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
    if (dh == 48) return launch_mfma<48>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, s);
  }
  if (dtype == DP_BF16)
    return dispatch<bf16_t>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, dh, s);
  return dispatch<float>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, dh, s);
}
