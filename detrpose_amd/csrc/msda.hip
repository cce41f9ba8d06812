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

namespace {

constexpr int MAXL = 4, MAXLP = 32;

struct Levels {
  int h[MAXL], w[MAXL], start[MAXL];
};

template <typename T>
__global__ __launch_bounds__(256) void msda_kernel(const T* __restrict__ value, int S, Levels lv, int L,
                                                   const T* __restrict__ offattn, const float* __restrict__ ref,
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
    const T* oa = offattn + (int64_t)r * ncol;
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

}  // namespace

extern "C" int dp_msda(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                       const void* offattn, const float* ref, void* out, int32_t ld_out, int32_t lq, int32_t nhead,
                       int32_t dh, int32_t npoints, int32_t dtype, void* stream) {
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
  const int cpt = dh / VEC;
  int TB = 256 / (nhead * cpt);
  if (TB < 1) TB = 1;
  const size_t lds = (size_t)TB * nhead * nlevels * npoints * 4 * 8;
  dim3 grid((unsigned)((rows + TB - 1) / TB)), block(256);
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(msda_kernel<bf16_t>, grid, block, lds, as_stream(stream), (const bf16_t*)value, S, lv, nlevels,
                       (const bf16_t*)offattn, ref, (bf16_t*)out, ld_out, lq, rows, nhead, dh, npoints, TB);
  else
    hipLaunchKernelGGL(msda_kernel<float>, grid, block, lds, as_stream(stream), (const float*)value, S, lv, nlevels,
                       (const float*)offattn, ref, (float*)out, ld_out, lq, rows, nhead, dh, npoints, TB);
  return dp_check_launch("dp_msda");
}
