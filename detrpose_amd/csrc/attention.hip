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

}  // namespace

extern "C" int dp_attention(const void* q, int32_t ld_q, const void* k, const void* v, int32_t ld_kv, void* out,
                            int32_t ld_o, int32_t n_outer, int32_t n_inner, int64_t so, int64_t si, int64_t st,
                            int32_t seqlen, int32_t nhead, int32_t dh, int32_t dtype, void* stream) {
  DP_REQUIRE(q && k && v && out, "dp_attention: null pointer");
  DP_REQUIRE(seqlen > 0 && n_outer > 0 && n_inner > 0 && nhead > 0, "dp_attention: bad shape");
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    return dispatch<bf16_t>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, dh, s);
  return dispatch<float>(q, ld_q, k, v, ld_kv, out, ld_o, n_outer, n_inner, so, si, st, seqlen, nhead, dh, s);
}
