// MSDA core at the training interface: explicit sampling locations and (softmaxed) attention
// weights, forward and backward. The first native piece of the training step.
//
// Reference: ms_deform_attn_core_pytorch (ms_deform_attn.py:145-193) = per level
// F.grid_sample(value_l, 2*loc-1, bilinear, zeros, align_corners=False), then the
// attention-weighted sum over (level, point). Its autograd is what these kernels compute:
//   pixel coords  x = loc_x * W - 0.5, y = loc_y * H - 0.5, corners (x0 + dx, y0 + dy),
//   weights w00 = (1-fx)(1-fy), w01 = fx(1-fy), w10 = (1-fx)fy, w11 = fx fy (0 outside);
//   s = sum_k w_k v_k,  out += a * s
//   d attn    = <go, s>
//   d loc_x   = a * <go, (v01 - v00)(1-fy) + (v11 - v10) fy> * W   (floor is flat)
//   d loc_y   = a * <go, (v10 - v00)(1-fx) + (v11 - v01) fx> * H
//   d value_k += a * w_k * go    (f32 atomics: many (token, point) pairs hit one row)
// Layouts: value [N][S][nH*Dh] (levels concatenated along S, the encoder memory layout of
// the inference path), loc [N][Lq][nH][L][P][2], attn [N][Lq][nH][L][P], out / grad_out
// [N][Lq][nH*Dh]. Lanes: CPT consecutive lanes own one (token, head), 16 bytes of channels
// each; the three per-point dot products are reduced over those lanes with shuffles.
#include "common.h"

namespace {

constexpr int MAXL = 4;

struct TLevels {
  int h[MAXL], w[MAXL], start[MAXL];
};

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float (&v)[16 / sizeof(T)]) {
  const Vec16<T> x = load16(p);
#pragma unroll
  for (int e = 0; e < Vec16<T>::N; ++e) v[e] = x.get(e);
}

// sum of v over the cpt lanes [g0, g0 + cpt) of the lane's (token, head) group
__device__ __forceinline__ float group_sum(float v, int g0, int cpt) {
  float t = 0.f;
  for (int s = 0; s < cpt; ++s) t += __shfl(v, g0 + s, 64);
  return t;
}

template <typename T, bool BWD>
__global__ __launch_bounds__(256) void msda_core_kernel(const T* __restrict__ value, int S, TLevels lv, int L, int P,
                                                        const float* __restrict__ loc, const float* __restrict__ attn,
                                                        const T* __restrict__ gout, T* __restrict__ out,
                                                        float* __restrict__ gvalue, float* __restrict__ gloc,
                                                        float* __restrict__ gattn, int lq, int pairs, int nh, int dh) {
  constexpr int VEC = Vec16<T>::N;
  const int cpt = dh / VEC;
  const int ppw = 64 / cpt;                       // (token, head) pairs per wave
  const int lane = threadIdx.x & 63;
  const int slot = lane / cpt, c = lane - slot * cpt;
  const int pair = (blockIdx.x * 4 + (threadIdx.x >> 6)) * ppw + slot;
  if (slot >= ppw || pair >= pairs) return;   // whole (token, head) groups leave together
  const int g0 = lane - c;
  const int r = pair / nh, h = pair - r * nh;
  const int b = r / lq;
  const int C = nh * dh;
  const int LP = L * P;
  const int ch = h * dh + c * VEC;
  const T* vb = value + (int64_t)b * S * C + ch;
  float go[VEC], acc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
  if (BWD) load_vec(gout + (int64_t)r * C + ch, go);
  const float* lp = loc + (int64_t)pair * LP * 2;
  const float* ap = attn + (int64_t)pair * LP;
  for (int j = 0; j < LP; ++j) {
    const int l = j / P;
    const int H = lv.h[l], W = lv.w[l];
    const float x = lp[2 * j] * W - 0.5f, y = lp[2 * j + 1] * H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float fx = x - fx0, fy = y - fy0;
    const float a = ap[j];
    const float wk[4] = {(1.f - fx) * (1.f - fy), fx * (1.f - fy), (1.f - fx) * fy, fx * fy};
    float v[4][VEC];
    int row[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xi = x0 + (k & 1), yi = y0 + (k >> 1);
      const bool ok = xi >= 0 && xi < W && yi >= 0 && yi < H;
      row[k] = ok ? lv.start[l] + yi * W + xi : -1;
      if (ok) load_vec(vb + (int64_t)row[k] * C, v[k]);
      else
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[k][e] = 0.f;
    }
    if (!BWD) {
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        acc[e] += a * (wk[0] * v[0][e] + wk[1] * v[1][e] + wk[2] * v[2][e] + wk[3] * v[3][e]);
      continue;
    }
    float ga = 0.f, gx = 0.f, gy = 0.f;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float s = wk[0] * v[0][e] + wk[1] * v[1][e] + wk[2] * v[2][e] + wk[3] * v[3][e];
      ga += go[e] * s;
      gx += go[e] * ((v[1][e] - v[0][e]) * (1.f - fy) + (v[3][e] - v[2][e]) * fy);
      gy += go[e] * ((v[2][e] - v[0][e]) * (1.f - fx) + (v[3][e] - v[1][e]) * fx);
    }
    ga = group_sum(ga, g0, cpt);
    gx = group_sum(gx, g0, cpt);
    gy = group_sum(gy, g0, cpt);
    if (c == 0) {
      gattn[(int64_t)pair * LP + j] = ga;
      gloc[((int64_t)pair * LP + j) * 2] = a * gx * W;
      gloc[((int64_t)pair * LP + j) * 2 + 1] = a * gy * H;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (row[k] < 0) continue;
      float* gp = gvalue + ((int64_t)b * S + row[k]) * C + ch;
      const float s = a * wk[k];
#pragma unroll
      for (int e = 0; e < VEC; ++e) unsafeAtomicAdd(gp + e, s * go[e]);
    }
  }
  if (!BWD) {
    Vec16<T> o;
#pragma unroll
    for (int e = 0; e < VEC; ++e) o.set(e, acc[e]);
    store16(out + (int64_t)r * C + ch, o);
  }
}

// Backward of the fused inference op dp_msda (MSDeformAttn.forward's default branch,
// ms_deform_attn.py:384-441): from the raw sampling offsets | attention logits row of each
// token (the two Linear outputs) and its reference point. Per (token, head): softmax over the
// L*P logits and loc = ref + off / (W, H) recomputed in registers, then the core backward
// above, then the chain rule through them in the same pass:
//   d off_x = d loc_x / W,  d off_y = d loc_y / H,  d ref += d loc (atomics over heads),
//   d logit_j = a_j (d a_j - sum_k a_k d a_k).
// grad_oa has the offattn layout [rows][nH*L*P*2 | nH*L*P]; grad_ref [rows][2] or NULL.
template <typename T>
__global__ __launch_bounds__(256) void msda_fused_bwd_kernel(const T* __restrict__ value, int S, TLevels lv, int L,
                                                             int P, const float* __restrict__ oa,
                                                             const float* __restrict__ ref, const T* __restrict__ gout,
                                                             int ldg, float* __restrict__ gvalue,
                                                             float* __restrict__ goa, float* __restrict__ gref, int lq,
                                                             int pairs, int nh, int dh) {
  constexpr int VEC = Vec16<T>::N;
  const int cpt = dh / VEC;
  const int ppw = 64 / cpt;
  const int lane = threadIdx.x & 63;
  const int slot = lane / cpt, c = lane - slot * cpt;
  const int pair = (blockIdx.x * 4 + (threadIdx.x >> 6)) * ppw + slot;
  if (slot >= ppw || pair >= pairs) return;
  const int g0 = lane - c;
  const int r = pair / nh, h = pair - r * nh;
  const int b = r / lq;
  const int C = nh * dh;
  const int LP = L * P;
  const int ncol = nh * LP * 3;
  const int ch = h * dh + c * VEC;
  const T* vb = value + (int64_t)b * S * C + ch;
  const float* orow = oa + (int64_t)r * ncol;
  float* grow = goa + (int64_t)r * ncol;
  const float* lg = orow + nh * LP * 2 + h * LP;
  float go[VEC];
  load_vec(gout + (int64_t)r * ldg + ch, go);
  float mx = -INFINITY;
  for (int j = 0; j < LP; ++j) mx = fmaxf(mx, lg[j]);
  float den = 0.f;
  for (int j = 0; j < LP; ++j) den += expf(lg[j] - mx);
  const float inv = 1.f / den;
  const float rx = ref[2 * r], ry = ref[2 * r + 1];
  float dot = 0.f, grx = 0.f, gry = 0.f;
  for (int j = 0; j < LP; ++j) {
    const int l = j / P;
    const int H = lv.h[l], W = lv.w[l];
    const float ox = orow[(h * LP + j) * 2], oy = orow[(h * LP + j) * 2 + 1];
    const float x = (rx + ox / W) * W - 0.5f, y = (ry + oy / H) * H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float fx = x - fx0, fy = y - fy0;
    const float a = expf(lg[j] - mx) * inv;
    const float wk[4] = {(1.f - fx) * (1.f - fy), fx * (1.f - fy), (1.f - fx) * fy, fx * fy};
    float v[4][VEC];
    int row[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xi = x0 + (k & 1), yi = y0 + (k >> 1);
      const bool ok = xi >= 0 && xi < W && yi >= 0 && yi < H;
      row[k] = ok ? lv.start[l] + yi * W + xi : -1;
      if (ok) load_vec(vb + (int64_t)row[k] * C, v[k]);
      else
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[k][e] = 0.f;
    }
    float ga = 0.f, gx = 0.f, gy = 0.f;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float s = wk[0] * v[0][e] + wk[1] * v[1][e] + wk[2] * v[2][e] + wk[3] * v[3][e];
      ga += go[e] * s;
      gx += go[e] * ((v[1][e] - v[0][e]) * (1.f - fy) + (v[3][e] - v[2][e]) * fy);
      gy += go[e] * ((v[2][e] - v[0][e]) * (1.f - fx) + (v[3][e] - v[1][e]) * fx);
    }
    ga = group_sum(ga, g0, cpt);
    gx = group_sum(gx, g0, cpt);
    gy = group_sum(gy, g0, cpt);
    dot += a * ga;
    if (c == 0) {
      // d loc = a * g * (W, H); d off = d loc / (W, H)
      grow[(h * LP + j) * 2] = a * gx;
      grow[(h * LP + j) * 2 + 1] = a * gy;
      grow[nh * LP * 2 + h * LP + j] = ga;   // d attn for now; the softmax pass below finishes it
      grx += a * gx * W;
      gry += a * gy * H;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (row[k] < 0 || !gvalue) continue;
      float* gp = gvalue + ((int64_t)b * S + row[k]) * C + ch;
      const float sc = a * wk[k];
#pragma unroll
      for (int e = 0; e < VEC; ++e) unsafeAtomicAdd(gp + e, sc * go[e]);
    }
  }
  if (c == 0) {
    float* gl = grow + nh * LP * 2 + h * LP;
    for (int j = 0; j < LP; ++j) {
      const float a = expf(lg[j] - mx) * inv;
      gl[j] = a * (gl[j] - dot);
    }
    if (gref) {
      unsafeAtomicAdd(gref + 2 * r, grx);
      unsafeAtomicAdd(gref + 2 * r + 1, gry);
    }
  }
}

// The same backward with one channel per lane (dh lanes per (token, head), dh a power of two
// <= 64), used when the value gradient is wanted: each of its float-atomic wave instructions
// then adds 64/dh contiguous dh*4-byte row segments (two 128-byte rows at dh 32), the shape
// the memory-side atomic units take at full rate (MI355X_MICROARCH.md § Global float atomics),
// where the 16-byte-per-lane mapping above issued 16 scattered 4-byte adds per instruction
// (9.3 -> see DESIGN.md per L b16 layer). The per-point dot products are xor-shuffle sums over
// the pair's dh lanes.
template <typename T>
__global__ __launch_bounds__(256) void msda_fused_bwd_cl_kernel(const T* __restrict__ value, int S, TLevels lv, int L,
                                                                int P, const float* __restrict__ oa,
                                                                const float* __restrict__ ref,
                                                                const T* __restrict__ gout, int ldg,
                                                                float* __restrict__ gvalue, float* __restrict__ goa,
                                                                float* __restrict__ gref, int lq, int pairs, int nh,
                                                                int dh) {
  const int ppw = 64 / dh;
  const int lane = threadIdx.x & 63;
  const int slot = lane / dh, c = lane - slot * dh;
  const int pair0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * ppw;
  if (pair0 >= pairs) return;                    // whole waves leave together
  const int pair = min(pair0 + slot, pairs - 1);  // a ragged last wave repeats its last pair...
  const bool live = pair0 + slot < pairs;         // ...without storing or adding anything
  const int r = pair / nh, h = pair - r * nh;
  const int b = r / lq;
  const int C = nh * dh;
  const int LP = L * P;
  const int ncol = nh * LP * 3;
  const int ch = h * dh + c;
  const T* vb = value + (int64_t)b * S * C + ch;
  const float* orow = oa + (int64_t)r * ncol;
  float* grow = goa + (int64_t)r * ncol;
  const float* lg = orow + nh * LP * 2 + h * LP;
  const float go = to_f32(gout[(int64_t)r * ldg + ch]);
  float mx = -INFINITY;
  for (int j = 0; j < LP; ++j) mx = fmaxf(mx, lg[j]);
  float den = 0.f;
  for (int j = 0; j < LP; ++j) den += expf(lg[j] - mx);
  const float inv = 1.f / den;
  const float rx = ref[2 * r], ry = ref[2 * r + 1];
  float dot = 0.f, grx = 0.f, gry = 0.f;
  float* gvb = gvalue + (int64_t)b * S * C + ch;
  // unrolled, with every corner load unconditional (index clamped into the map, value selected
  // away outside it): a guarded load compiles to a branch around it, and the points' loads then
  // issue one at a time
#pragma unroll 4
  for (int j = 0; j < LP; ++j) {
    const int l = j / P;
    const int H = lv.h[l], W = lv.w[l];
    const float ox = orow[(h * LP + j) * 2], oy = orow[(h * LP + j) * 2 + 1];
    const float x = (rx + ox / W) * W - 0.5f, y = (ry + oy / H) * H - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float fx = x - fx0, fy = y - fy0;
    const float a = expf(lg[j] - mx) * inv;
    const float wk[4] = {(1.f - fx) * (1.f - fy), fx * (1.f - fy), (1.f - fx) * fy, fx * fy};
    float v[4];
    int row[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int xi = x0 + (k & 1), yi = y0 + (k >> 1);
      const bool ok = xi >= 0 && xi < W && yi >= 0 && yi < H;
      const int rc = lv.start[l] + min(max(yi, 0), H - 1) * W + min(max(xi, 0), W - 1);
      const float vv = to_f32(vb[(int64_t)rc * C]);
      row[k] = ok ? rc : -1;
      v[k] = ok ? vv : 0.f;
    }
    const float sv = wk[0] * v[0] + wk[1] * v[1] + wk[2] * v[2] + wk[3] * v[3];
    float ga = go * sv;
    float gx = go * ((v[1] - v[0]) * (1.f - fy) + (v[3] - v[2]) * fy);
    float gy = go * ((v[2] - v[0]) * (1.f - fx) + (v[3] - v[1]) * fx);
    for (int o = dh >> 1; o > 0; o >>= 1) {
      ga += __shfl_xor(ga, o, 64);
      gx += __shfl_xor(gx, o, 64);
      gy += __shfl_xor(gy, o, 64);
    }
    dot += a * ga;
    if (c == 0 && live) {
      grow[(h * LP + j) * 2] = a * gx;
      grow[(h * LP + j) * 2 + 1] = a * gy;
      grow[nh * LP * 2 + h * LP + j] = ga;
      grx += a * gx * W;
      gry += a * gy * H;
    }
    if (live) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (row[k] >= 0) unsafeAtomicAdd(gvb + (int64_t)row[k] * C, a * wk[k] * go);
    }
  }
  if (c == 0 && live) {
    float* gl = grow + nh * LP * 2 + h * LP;
    for (int j = 0; j < LP; ++j) {
      const float a = expf(lg[j] - mx) * inv;
      gl[j] = a * (gl[j] - dot);
    }
    if (gref) {
      unsafeAtomicAdd(gref + 2 * r, grx);
      unsafeAtomicAdd(gref + 2 * r + 1, gry);
    }
  }
}

template <typename T, bool BWD>
int launch_core(const void* value, int batch, int S, const TLevels& lv, int L, int P, const float* loc,
                const float* attn, const void* gout, void* out, float* gvalue, float* gloc, float* gattn, int lq, int nh,
                int dh, hipStream_t s) {
  const int cpt = dh / Vec16<T>::N;
  const int ppw = 64 / cpt;
  const int pairs = batch * lq * nh;
  const int waves = (pairs + ppw - 1) / ppw;
  const int grid = (waves + 3) / 4;
  hipLaunchKernelGGL((msda_core_kernel<T, BWD>), dim3(grid), dim3(256), 0, s, reinterpret_cast<const T*>(value), S, lv,
                     L, P, loc, attn, reinterpret_cast<const T*>(gout), reinterpret_cast<T*>(out), gvalue, gloc, gattn,
                     lq, pairs, nh, dh);
  return dp_check_launch(BWD ? "dp_msda_core_bwd" : "dp_msda_core_fwd");
}

int check_core(const void* value, int batch, int S, const int32_t* lvl_hw, int nlevels, const float* loc,
               const float* attn, int lq, int nhead, int dh, int npoints, int dtype, TLevels* lv) {
  const int VEC = dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE(value && loc && attn && lvl_hw, "dp_msda_core: null pointer");
  DP_REQUIRE(dtype == DP_BF16 || dtype == DP_F32, "dp_msda_core: bad dtype %d", dtype);
  DP_REQUIRE(nlevels >= 1 && nlevels <= MAXL, "dp_msda_core: nlevels=%d (max %d)", nlevels, MAXL);
  DP_REQUIRE(batch > 0 && lq > 0 && nhead > 0 && npoints > 0, "dp_msda_core: bad shape");
  DP_REQUIRE(dh % VEC == 0 && dh / VEC <= 64, "dp_msda_core: dh=%d must be a multiple of %d (at most %d)", dh, VEC,
             64 * VEC);
  DP_REQUIRE((reinterpret_cast<uintptr_t>(value) & 15) == 0, "dp_msda_core: value must be 16-byte aligned");
  DP_REQUIRE((int64_t)batch * lq * nhead < (1ll << 31), "dp_msda_core: too many (token, head) pairs");
  int start = 0;
  for (int l = 0; l < nlevels; ++l) {
    lv->h[l] = lvl_hw[2 * l];
    lv->w[l] = lvl_hw[2 * l + 1];
    lv->start[l] = start;
    DP_REQUIRE(lv->h[l] > 0 && lv->w[l] > 0, "dp_msda_core: empty level %d", l);
    start += lv->h[l] * lv->w[l];
  }
  DP_REQUIRE(start == S, "dp_msda_core: level sizes sum to %d, S=%d", start, S);
  return 0;
}

}  // namespace

extern "C" int dp_msda_core_fwd(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                                const float* loc, const float* attn, void* out, int32_t lq, int32_t nhead, int32_t dh,
                                int32_t npoints, int32_t dtype, void* stream) {
  TLevels lv;
  const int rc = check_core(value, batch, S, lvl_hw, nlevels, loc, attn, lq, nhead, dh, npoints, dtype, &lv);
  if (rc) return rc;
  DP_REQUIRE(out && (reinterpret_cast<uintptr_t>(out) & 15) == 0, "dp_msda_core_fwd: out must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  if (dtype == DP_BF16)
    return launch_core<bf16_t, false>(value, batch, S, lv, nlevels, npoints, loc, attn, nullptr, out, nullptr, nullptr,
                                      nullptr, lq, nhead, dh, s);
  return launch_core<float, false>(value, batch, S, lv, nlevels, npoints, loc, attn, nullptr, out, nullptr, nullptr,
                                   nullptr, lq, nhead, dh, s);
}

extern "C" int dp_msda_core_bwd(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                                const float* loc, const float* attn, const void* grad_out, int32_t lq, int32_t nhead,
                                int32_t dh, int32_t npoints, float* grad_value, float* grad_loc, float* grad_attn,
                                int32_t dtype, void* stream) {
  TLevels lv;
  const int rc = check_core(value, batch, S, lvl_hw, nlevels, loc, attn, lq, nhead, dh, npoints, dtype, &lv);
  if (rc) return rc;
  DP_REQUIRE(grad_out && grad_value && grad_loc && grad_attn, "dp_msda_core_bwd: null gradient pointer");
  DP_REQUIRE((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0, "dp_msda_core_bwd: grad_out must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  // grad_value is accumulated by atomics: clear it on the same stream first (graph-capturable)
  if (hipMemsetAsync(grad_value, 0, (size_t)batch * S * nhead * dh * sizeof(float), s) != hipSuccess)
    return dp_check_launch("dp_msda_core_bwd(memset)");
  if (dtype == DP_BF16)
    return launch_core<bf16_t, true>(value, batch, S, lv, nlevels, npoints, loc, attn, grad_out, nullptr, grad_value,
                                     grad_loc, grad_attn, lq, nhead, dh, s);
  return launch_core<float, true>(value, batch, S, lv, nlevels, npoints, loc, attn, grad_out, nullptr, grad_value,
                                  grad_loc, grad_attn, lq, nhead, dh, s);
}

extern "C" int dp_msda_bwd(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                           const float* offattn, const float* ref, const void* grad_out, int32_t ld_grad_out,
                           int32_t lq, int32_t nhead, int32_t dh, int32_t npoints, float* grad_value,
                           int32_t accumulate_value, float* grad_offattn, float* grad_ref, int32_t dtype,
                           void* stream) {
  TLevels lv;
  const int rc = check_core(value, batch, S, lvl_hw, nlevels, offattn, ref, lq, nhead, dh, npoints, dtype, &lv);
  if (rc) return rc;
  DP_REQUIRE(grad_out && grad_offattn, "dp_msda_bwd: null gradient pointer");
  const int VEC = dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0 && ld_grad_out % VEC == 0 && ld_grad_out >= nhead * dh,
             "dp_msda_bwd: grad_out must be 16-byte aligned per row (ld %d)", ld_grad_out);
  hipStream_t s = as_stream(stream);
  // grad_value (and grad_ref) are accumulated by atomics: clear them on the stream first
  if ((grad_value && !accumulate_value &&
       hipMemsetAsync(grad_value, 0, (size_t)batch * S * nhead * dh * sizeof(float), s) != hipSuccess) ||
      (grad_ref && hipMemsetAsync(grad_ref, 0, (size_t)batch * lq * 2 * sizeof(float), s) != hipSuccess))
    return dp_check_launch("dp_msda_bwd(memset)");
  const int pairs = batch * lq * nhead;
  if (grad_value && dh <= 64 && (dh & (dh - 1)) == 0 && !getenv("DETRPOSE_MSDA_BWD_VEC")) {
    const int ppw = 64 / dh;
    const int grid = ((pairs + ppw - 1) / ppw + 3) / 4;
    if (dtype == DP_BF16)
      hipLaunchKernelGGL(msda_fused_bwd_cl_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)value, S, lv,
                         nlevels, npoints, offattn, ref, (const bf16_t*)grad_out, ld_grad_out, grad_value,
                         grad_offattn, grad_ref, lq, pairs, nhead, dh);
    else
      hipLaunchKernelGGL(msda_fused_bwd_cl_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)value, S, lv,
                         nlevels, npoints, offattn, ref, (const float*)grad_out, ld_grad_out, grad_value, grad_offattn,
                         grad_ref, lq, pairs, nhead, dh);
    return dp_check_launch("dp_msda_bwd");
  }
  const int ppw = 64 / (dh / VEC);
  const int grid = ((pairs + ppw - 1) / ppw + 3) / 4;
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(msda_fused_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)value, S, lv,
                       nlevels, npoints, offattn, ref, (const bf16_t*)grad_out, ld_grad_out, grad_value, grad_offattn, grad_ref, lq,
                       pairs, nhead, dh);
  else
    hipLaunchKernelGGL(msda_fused_bwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)value, S, lv, nlevels,
                       npoints, offattn, ref, (const float*)grad_out, ld_grad_out, grad_value, grad_offattn, grad_ref, lq, pairs,
                       nhead, dh);
  return dp_check_launch("dp_msda_bwd");
}
