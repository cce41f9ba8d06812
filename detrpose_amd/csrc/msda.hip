// Multi-scale deformable attention, the decoder's cross-attention sampling/aggregation.
//
// Reference: MSDeformAttn.forward default branch (ms_deform_attn.py:384-444) and
// ms_deform_attn_core_pytorch (145-193), which runs one F.grid_sample per level over a
// (B*nH, Dh, H, W) re-layout of the memory. Here the memory stays in its encoder
// layout [B][S][nH*Dh] (channels-last, head-major, levels concatenated along S), so the
// 4 bilinear corners of one (token, head, point) are 4 contiguous Dh-channel segments.
//
// Block = 256 threads over TB tokens. Phase 1 (one thread per (token, head)): softmax
// of the L*P attention logits, loc = ref + off/(W_l, H_l), bilinear setup
// (align_corners=False: pixel = loc*size - 0.5, zero outside) -> per point 4 corner row
// indices + 4 weights (attention weight folded in), staged in LDS.
// Phase 2 (one thread per (token, head, 16-byte channel chunk)): 4*L*P 16-byte gathers
// and FMAs from LDS weights; one 16-byte store. No value_proj / output_proj exist on
// this path.
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int MAXL = 4, MAXLP = 32;

struct Levels {
  int h[MAXL], w[MAXL], start[MAXL];
};

template <typename T, typename OA>
__global__ __launch_bounds__(256) void msda_kernel(const T* __restrict__ value, int S, Levels lv, int L,
                                                   const OA* __restrict__ offattn, const float* __restrict__ ref,
                                                   T* __restrict__ out, int ld_out, int lq, int rows, int nhead, int dh,
                                                   int P, int TB) {
  constexpr int VEC = Vec16<T>::N;
  extern __shared__ int smem_i[];
  const int LP = L * P;
  const int per_tok = nhead * LP;             // entries per token
  int* cidx = smem_i;                         // [TB][nhead][LP][4]
  float* cw = reinterpret_cast<float*>(smem_i + TB * per_tok * 4);  // [TB][nhead][LP][4]
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * TB;
  const int C = nhead * dh;
  const int ncol = nhead * LP * 3;

  // ---- phase 1
  for (int th = tid; th < TB * nhead; th += blockDim.x) {
    const int tl = th / nhead, h = th - tl * nhead;
    const int r = r0 + tl;
    if (r >= rows) continue;
    const OA* oa = offattn + (int64_t)r * ncol;
    const float rx = ref[2 * r], ry = ref[2 * r + 1];
    float lg[MAXLP];
    float mx = -INFINITY;
    for (int j = 0; j < LP; ++j) {
      lg[j] = to_f32(oa[nhead * LP * 2 + h * LP + j]);
      mx = fmaxf(mx, lg[j]);
    }
    float sum = 0.f;
    for (int j = 0; j < LP; ++j) {
      lg[j] = __expf(lg[j] - mx);
      sum += lg[j];
    }
    const float inv = 1.f / sum;
    for (int j = 0; j < LP; ++j) {
      const int l = j / P;
      const int H = lv.h[l], W = lv.w[l];
      const float ox = to_f32(oa[(h * LP + j) * 2]), oy = to_f32(oa[(h * LP + j) * 2 + 1]);
      const float x = (rx + ox / W) * W - 0.5f;
      const float y = (ry + oy / H) * H - 0.5f;
      const float fx0 = floorf(x), fy0 = floorf(y);
      const int x0 = (int)fx0, y0 = (int)fy0;
      const float ax = x - fx0, ay = y - fy0;
      const float a = lg[j] * inv;
      const int e = ((tl * nhead + h) * LP + j) * 4;
      const float wts[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
#pragma unroll
      for (int cnr = 0; cnr < 4; ++cnr) {
        const int xi = x0 + (cnr & 1), yi = y0 + (cnr >> 1);
        const bool ok = xi >= 0 && xi < W && yi >= 0 && yi < H;
        cidx[e + cnr] = ok ? lv.start[l] + yi * W + xi : -1;
        cw[e + cnr] = ok ? wts[cnr] * a : 0.f;
      }
    }
  }
  __syncthreads();

  // ---- phase 2
  const int cpt = dh / VEC;  // chunks per head
  const int work = TB * nhead * cpt;
  for (int wi = tid; wi < work; wi += blockDim.x) {
    const int tl = wi / (nhead * cpt);
    const int rem = wi - tl * nhead * cpt;
    const int h = rem / cpt, cc = rem - h * cpt;
    const int r = r0 + tl;
    if (r >= rows) continue;
    const int b = r / lq;
    const T* vb = value + (int64_t)b * S * C + h * dh + cc * VEC;
    float acc[VEC];
#pragma unroll
    for (int t = 0; t < VEC; ++t) acc[t] = 0.f;
    const int e0 = (tl * nhead + h) * LP * 4;
    for (int j = 0; j < LP * 4; ++j) {
      const int id = cidx[e0 + j];
      if (id < 0) continue;
      const float w = cw[e0 + j];
      Vec16<T> v = load16(vb + (int64_t)id * C);
#pragma unroll
      for (int t = 0; t < VEC; ++t) acc[t] = fmaf(w, v.get(t), acc[t]);
    }
    Vec16<T> o;
#pragma unroll
    for (int t = 0; t < VEC; ++t) o.set(t, acc[t]);
    store16(out + (int64_t)r * ld_out + h * dh + cc * VEC, o);
  }
}

// ---------------------------------------------------------------------------------
// bf16 wave-per-token kernel (the production path). Lane (t, h, c) of a wave owns token
// t (TPW tokens per wave), head h and the 16-byte channel chunk c of that head (CPT chunks
// per head, TPL = NH*CPT lanes per token).
//  * Point setup is spread over the head's CPT lanes: lane c takes points c, c+CPT, ...
//    (no idle lanes, unlike one thread per (token, head)); the softmax max/sum over the
//    head's L*P logits is reduced across those lanes with shuffles.
//  * Each point's 4 corner rows and 4 weights (attention weight and bilinear weight folded,
//    0 for a corner outside the map, row clamped to 0 so the load is always legal) go to a
//    per-wave LDS slice; the head's CPT lanes then read them back as broadcasts (the
//    (token, head) stride is padded by 16 B so 4 heads of a 16-lane group never share a bank).
//  * Gather: 4*L*P independent 16-byte loads per lane, fp32 FMAs, one 16-byte store.
//  * XCD-aware order: logical block = (blockIdx % 8) * (G / 8) + blockIdx / 8 gives each
//    of the 8 XCDs a contiguous token range, i.e. whole images: an image's 4.3 MB value
//    slab (L) is pulled into ONE XCD's L2 instead of all eight.
template <int NH, int CPT, int L, int P, typename OA>
__global__ __launch_bounds__(256) void msda_wave_kernel(const bf16_t* __restrict__ value, int S, Levels lv,
                                                        const OA* __restrict__ offattn,
                                                        const float* __restrict__ ref, bf16_t* __restrict__ out,
                                                        int ld_out, int lq, int rows, int nblk) {
  constexpr int LP = L * P;
  constexpr int TPL = NH * CPT;               // lanes per token
  constexpr int TPW = 64 / TPL;               // tokens per wave
  constexpr int NPP = (LP + CPT - 1) / CPT;   // points per lane in the setup
  constexpr int C = NH * CPT * 8;             // channels per token row
  constexpr int ESTR = LP * 32 + 16;          // bytes per (token, head) entry block
  static_assert(TPW >= 1 && LP <= MAXLP, "shape");
  __shared__ __attribute__((aligned(16))) char lds[4][TPW * NH * ESTR];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = gridDim.x;
  const int blk = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (blk >= nblk) return;
  const int t = lane / TPL, li = lane - t * TPL;
  const int h = li / CPT, c = li - h * CPT;
  const int r = (blk * 4 + wave) * TPW + t;
  const bool act = t < TPW && r < rows;
  const int rr = act ? r : 0;
  char* ent = lds[wave] + (t < TPW ? (t * NH + h) * ESTR : 0);

  // ---- setup: lane c takes points j = c + CPT*k
  const OA* oa = offattn + (int64_t)rr * (NH * LP * 3);
  float lg[NPP];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < NPP; ++k) {
    const int j = c + CPT * k;
    lg[k] = j < LP ? (float)oa[NH * LP * 2 + h * LP + j] : -INFINITY;
    mx = fmaxf(mx, lg[k]);
  }
  const int g0 = lane - c;                    // first lane of the head group
#pragma unroll
  for (int s = 0; s < CPT; ++s) mx = fmaxf(mx, __shfl(mx, g0 + s, 64));
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < NPP; ++k) {
    lg[k] = (c + CPT * k) < LP ? __expf(lg[k] - mx) : 0.f;
    sum += lg[k];
  }
  float tot = 0.f;
#pragma unroll
  for (int s = 0; s < CPT; ++s) tot += __shfl(sum, g0 + s, 64);
  const float inv = 1.f / tot;
  const float rx = ref[2 * rr], ry = ref[2 * rr + 1];
#pragma unroll
  for (int k = 0; k < NPP; ++k) {
    const int j = c + CPT * k;
    if (j >= LP || t >= TPW) continue;
    const int l = j / P;
    const int H = lv.h[l], W = lv.w[l];
    const float ox = (float)oa[(h * LP + j) * 2], oy = (float)oa[(h * LP + j) * 2 + 1];
    const float x = (rx + ox / W) * W - 0.5f;
    const float y = (ry + oy / H) * H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float ax = x - fx0, ay = y - fy0;
    const float a = lg[k] * inv;
    const float wts[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
    int4 id;
    float4 wv;
#pragma unroll
    for (int cnr = 0; cnr < 4; ++cnr) {
      const int xi = x0 + (cnr & 1), yi = y0 + (cnr >> 1);
      const bool ok = xi >= 0 && xi < W && yi >= 0 && yi < H;
      (&id.x)[cnr] = ok ? lv.start[l] + yi * W + xi : 0;
      (&wv.x)[cnr] = ok ? wts[cnr] * a : 0.f;
    }
    *reinterpret_cast<int4*>(ent + j * 32) = id;
    *reinterpret_cast<float4*>(ent + j * 32 + 16) = wv;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- gather
  if (!act) return;
  const int b = r / lq;
  const bf16_t* vb = value + (int64_t)b * S * C + h * (CPT * 8) + c * 8;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
  for (int j = 0; j < LP; ++j) {
    const int4 id = *reinterpret_cast<const int4*>(ent + j * 32);
    const float4 wv = *reinterpret_cast<const float4*>(ent + j * 32 + 16);
    bf16x8 v[4];
#pragma unroll
    for (int cnr = 0; cnr < 4; ++cnr) v[cnr] = *reinterpret_cast<const bf16x8*>(vb + (int64_t)(&id.x)[cnr] * C);
#pragma unroll
    for (int cnr = 0; cnr < 4; ++cnr)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf((&wv.x)[cnr], (float)v[cnr][e], acc[e]);
  }
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (bf16_t)acc[e];
  *reinterpret_cast<bf16x8*>(out + (int64_t)r * ld_out + h * (CPT * 8) + c * 8) = o;
}

template <int NH, int CPT, int L, int P, typename OA>
int launch_wave(const bf16_t* value, int S, const Levels& lv, const OA* offattn, const float* ref, bf16_t* out,
                int ld_out, int lq, int rows, hipStream_t s) {
  constexpr int TPW = 64 / (NH * CPT);
  const int nblk = (rows + 4 * TPW - 1) / (4 * TPW);
  const int grid = (nblk + 7) / 8 * 8;
  hipLaunchKernelGGL((msda_wave_kernel<NH, CPT, L, P, OA>), dim3(grid), dim3(256), 0, s, value, S, lv, offattn, ref,
                     out, ld_out, lq, rows, nblk);
  return dp_check_launch("dp_msda(wave)");
}

// the (nhead, dh, L, P) shapes of the DETRPose configs (N: 8x16, 2 levels x 6 points;
// L: 8x32, 3x4; X: 8x48, 3x4); -1 = no instantiation (generic kernel)
template <typename OA>
int dispatch_wave(const bf16_t* value, int S, const Levels& lv, int L, int P, int nhead, int dh,
                  const OA* offattn, const float* ref, bf16_t* out, int ld_out, int lq, int rows, hipStream_t s) {
  if (nhead != 8) return -1;
  if (dh == 32 && L == 3 && P == 4) return launch_wave<8, 4, 3, 4>(value, S, lv, offattn, ref, out, ld_out, lq, rows, s);
  if (dh == 16 && L == 2 && P == 6) return launch_wave<8, 2, 2, 6>(value, S, lv, offattn, ref, out, ld_out, lq, rows, s);
  if (dh == 48 && L == 3 && P == 4) return launch_wave<8, 6, 3, 4>(value, S, lv, offattn, ref, out, ld_out, lq, rows, s);
  if (dh == 32 && L == 4 && P == 4) return launch_wave<8, 4, 4, 4>(value, S, lv, offattn, ref, out, ld_out, lq, rows, s);
  return -1;
}

}  // namespace

extern "C" int dp_msda(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                       const void* offattn, const float* ref, void* out, int32_t ld_out, int32_t lq, int32_t nhead,
                       int32_t dh, int32_t npoints, int32_t dtype, void* stream) {
  // DP_MSDA_OFFATTN_F32 in dtype: offattn is f32 whatever the value dtype (the training step's
  // offsets Linear output, which the backward differentiates at)
  const bool oa32 = (dtype & DP_MSDA_OFFATTN_F32) != 0;
  dtype &= ~DP_MSDA_OFFATTN_F32;
  DP_REQUIRE(dtype == DP_BF16 || dtype == DP_F32, "dp_msda: bad dtype %d", dtype);
  const int VEC = dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE(value && offattn && ref && out && lvl_hw, "dp_msda: null pointer");
  DP_REQUIRE(nlevels >= 1 && nlevels <= MAXL, "dp_msda: nlevels=%d (max %d)", nlevels, MAXL);
  DP_REQUIRE(nlevels * npoints <= MAXLP, "dp_msda: L*P=%d (max %d)", nlevels * npoints, MAXLP);
  DP_REQUIRE(dh % VEC == 0 && ld_out % VEC == 0, "dp_msda: dh=%d / ld_out=%d must be multiples of %d", dh, ld_out, VEC);
  Levels lv;
  int start = 0;
  for (int l = 0; l < nlevels; ++l) {
    lv.h[l] = lvl_hw[2 * l];
    lv.w[l] = lvl_hw[2 * l + 1];
    lv.start[l] = start;
    start += lv.h[l] * lv.w[l];
  }
  DP_REQUIRE(start == S, "dp_msda: level sizes sum to %d, S=%d", start, S);
  const int rows = batch * lq;
  static const bool generic = getenv("DETRPOSE_MSDA_GENERIC") != nullptr;
  if (dtype == DP_BF16 && !generic && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(value) & 15) == 0) {
    const int rc = oa32 ? dispatch_wave((const bf16_t*)value, S, lv, nlevels, npoints, nhead, dh,
                                        (const float*)offattn, ref, (bf16_t*)out, ld_out, lq, rows, as_stream(stream))
                        : dispatch_wave((const bf16_t*)value, S, lv, nlevels, npoints, nhead, dh,
                                        (const bf16_t*)offattn, ref, (bf16_t*)out, ld_out, lq, rows, as_stream(stream));
    if (rc != -1) return rc;
  }
  const int cpt = dh / VEC;
  int TB = 256 / (nhead * cpt);
  if (TB < 1) TB = 1;
  const size_t lds = (size_t)TB * nhead * nlevels * npoints * 4 * 8;
  dim3 grid((unsigned)((rows + TB - 1) / TB)), block(256);
  if (dtype == DP_BF16 && oa32)
    hipLaunchKernelGGL((msda_kernel<bf16_t, float>), grid, block, lds, as_stream(stream), (const bf16_t*)value, S, lv,
                       nlevels, (const float*)offattn, ref, (bf16_t*)out, ld_out, lq, rows, nhead, dh, npoints, TB);
  else if (dtype == DP_BF16)
    hipLaunchKernelGGL((msda_kernel<bf16_t, bf16_t>), grid, block, lds, as_stream(stream), (const bf16_t*)value, S, lv,
                       nlevels, (const bf16_t*)offattn, ref, (bf16_t*)out, ld_out, lq, rows, nhead, dh, npoints, TB);
  else
    hipLaunchKernelGGL((msda_kernel<float, float>), grid, block, lds, as_stream(stream), (const float*)value, S, lv,
                       nlevels, (const float*)offattn, ref, (float*)out, ld_out, lq, rows, nhead, dh, npoints, TB);
  return dp_check_launch("dp_msda");
}
