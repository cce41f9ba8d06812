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
#include <algorithm>

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

// ---------------------------------------------------------------------------------------------
// The same backward with the value gradient summed WITHOUT float atomics (dp_msda_bwd_sorted).
// The atomic kernel above is bound by the chip's global float-atomic rate: every (token, head,
// point, corner) adds a dh-float row segment (340 M f32 adds per DETRPose-L b16 layer, ~1 ms).
// Here each sampling point is filed under its CELL, the top-left corner (x0, y0) of its bilinear
// footprint (x0 in [-1, W-1], y0 in [-1, H-1]: a (W+1) x (H+1) grid per level), and a value pixel
// (x, y) sums the lists of the four cells whose footprint covers it, as corner k of each:
// (x - (k & 1), y - (k >> 1)) for k = 00, 01, 10, 11. Per segment (image, head):
//   KS msda_sort_kernel        one block per (segment, level), all in LDS: the softmax statistics
//                              of the segment's tokens; count the level's points per cell (LDS
//                              int atomics), scan, place (token, a, fx, fy) entries in cell order
//                              (a second atomic pass on the scanned cursors), copy the cell-ordered
//                              list out coalesced; offsets / counts per cell; the work items
//                              (pixel, chunk of <= SORT_CHUNK entries of its four lists)
//   K2 msda_sorted_bwd_kernel  the gather backward for d offsets, d logits, d ref (16-byte lanes;
//                              each lane keeps the results of every cpt-th point and stores them
//                              at the end, so a wave's stores are contiguous runs)
//   K3 msda_value_sum_kernel   per item: sum over the pixel's four lists of
//                              a * w_k(fx, fy) * grad_out[token row, head] in registers, then ONE
//                              read-add-write of the pixel's dh-float segment (float atomics only
//                              for the rare pixels whose lists span several items)
// No global counters and no scattered list writes: the sort lives in LDS. Work is mapped
// segment-major with every segment's blocks on one XCD (workgroup i runs on XCD i % 8), so a
// segment's value rows, lists and grad_out slice stay in one L2. K2 is independent of KS / K3.
constexpr int SORT_CHUNK = 32;   // list entries per K3 round (one per lane slot)
constexpr int SORT_ITEM = 256;   // list entries per K3 work item (a hot pixel's lists split in items
                                 // of this size meet in float atomics)

struct SortWs {
  float4* list;        // [NS][L * lq * P] (token as int bits, a, fx, fy) in cell order (level-major)
  float* pa;           // [NS][lq][L * P] each point's softmaxed attention weight (K2 writes it)
  int4* item;          // [NS][isz][2] (pixel | chunk, list prefixes, entries, list bases), level-major:
                       // slot p = pixel p's first chunk, its further chunks past H * W
  int32_t* nitem;      // [NS][L]
  int isz;
#ifdef DP_KS_TIMING
  long long* dbg;      // A/B builds only: per sort block, wall-clock stamps at its phase boundaries
#endif
  int spx, segmap;     // segments per XCD; 1 (default): XCD x serves segments [x * spx, (x + 1) * spx)
                       // (whole images per XCD), 0: segments s = x mod 8 (one head per XCD)
  int ibase[MAXL];     // first item slot of each level
  int bps[MAXL];       // K3 blocks per (segment, level)
};

// <a, b> over one 16-byte lane slice: bf16 pairs on v_dot2 (f32 accumulate), f32 on FMA
__device__ __forceinline__ float corner_dot(const Vec16<bf16_t>& a, const Vec16<bf16_t>& b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const uint4 x = *reinterpret_cast<const uint4*>(&a.v), y = *reinterpret_cast<const uint4*>(&b.v);
  float acc = 0.f;
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, x.x), __builtin_bit_cast(bf2, y.x), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, x.y), __builtin_bit_cast(bf2, y.y), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, x.z), __builtin_bit_cast(bf2, y.z), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, x.w), __builtin_bit_cast(bf2, y.w), acc, false);
  return acc;
}
__device__ __forceinline__ float corner_dot(const Vec16<float>& a, const Vec16<float>& b) {
  return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2] + a.v[3] * b.v[3];
}

// lane g0 + s of the lane's G-lane group (G <= 4: one DPP quad permute; else ds_bpermute)
template <int G>
__device__ __forceinline__ int group_bcast(int v, int s, int g0) {
  if constexpr (G == 4) {
    switch (s) {
      case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xf, 0xf, false);
      case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xf, 0xf, false);
      case 2: return __builtin_amdgcn_mov_dpp(v, 0xaa, 0xf, 0xf, false);
      default: return __builtin_amdgcn_mov_dpp(v, 0xff, 0xf, 0xf, false);
    }
  } else if constexpr (G == 2) {
    return s == 0 ? __builtin_amdgcn_mov_dpp(v, 0xa0, 0xf, 0xf, false)    // [0, 0, 2, 2]
                  : __builtin_amdgcn_mov_dpp(v, 0xf5, 0xf, 0xf, false);   // [1, 1, 3, 3]
  } else if constexpr (G == 1) {
    return v;
  } else {
    return __shfl(v, g0 + s, 64);
  }
}

__device__ __forceinline__ int seg_of(int xcd, int k, int spx, int segmap) {
  return segmap ? xcd * spx + k : k * 8 + xcd;
}

__device__ __forceinline__ void msda_xy(float rx, float ry, float ox, float oy, int H, int W, float& x, float& y) {
#pragma clang fp contract(off)
  x = (rx + ox / W) * W - 0.5f;
  y = (ry + oy / H) * H - 0.5f;
}

// exclusive prefix of v over a 1024-thread block; the block total to `total`
__device__ __forceinline__ int block_excl_scan(int v, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int s = wsum[i];
    pre += i < w ? s : 0;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return pre + x - v;
}

#ifdef DP_KS_TIMING
#define DP_KS_STAMP(k) \
  if (threadIdx.x == 0) ws.dbg[(int64_t)(seg * L + l) * 8 + (k)] = (long long)wall_clock64()
#else
#define DP_KS_STAMP(k)
#endif

// LDS: cell offsets [ncell + 1] int (counts, then offsets, then cursors). Each thread owns the
// points tid + u * 1024 (u < PPT) of the level and keeps their cells in registers between the two
// passes; pass 2 reloads the points' inputs (L2) and the attention weight K2 stored (ws.pa).
constexpr int SORT_PPT = 8;   // points per thread: lq * P <= 8192

__global__ __launch_bounds__(1024) void msda_sort_kernel(TLevels lv, int L, int P, const float* __restrict__ oa,
                                                         const float* __restrict__ ref, int lq, int nh, int nseg,
                                                         SortWs ws) {
  extern __shared__ int cnt[];
  __shared__ int wsum[16];
  __shared__ int novf;
  const int xcd = blockIdx.x & 7, i = blockIdx.x >> 3;
  const int seg = seg_of(xcd, i / L, ws.spx, ws.segmap), l = i - (i / L) * L;
  if (seg >= nseg) return;
  DP_KS_STAMP(0);
  const int b = seg / nh, h = seg - b * nh;
  const int H = lv.h[l], W = lv.w[l], W1 = W + 1, ncell = (H + 1) * W1;
  const int LP = L * P, npt = lq * P, tid = threadIdx.x;
  const int ncol = nh * LP * 3;
  const float* oab = oa + (int64_t)b * lq * ncol;
  for (int c = tid; c <= ncell; c += 1024) cnt[c] = 0;
  if (tid == 0) novf = 0;
  // pass 1: the cells of this thread's points (half the points' loads in flight at a time)
  int key[SORT_PPT];
  auto point_xy = [&](int u, float& x, float& y) {
    const int pt = min(tid + u * 1024, npt - 1);
    const int t = pt / P, j = l * P + pt - t * P;
    const float* orow = oab + (int64_t)t * ncol;
    msda_xy(ref[2 * (b * lq + t)], ref[2 * (b * lq + t) + 1], orow[(h * LP + j) * 2], orow[(h * LP + j) * 2 + 1], H,
            W, x, y);
  };
#pragma unroll
  for (int u0 = 0; u0 < SORT_PPT; u0 += SORT_PPT / 2) {
    __builtin_amdgcn_sched_barrier(0);
    float x[SORT_PPT / 2], y[SORT_PPT / 2];
#pragma unroll
    for (int u = 0; u < SORT_PPT / 2; ++u) point_xy(u0 + u, x[u], y[u]);
#pragma unroll
    for (int u = 0; u < SORT_PPT / 2; ++u) {
      const int x0 = (int)floorf(x[u]), y0 = (int)floorf(y[u]);
      key[u0 + u] = tid + (u0 + u) * 1024 < npt && x0 >= -1 && x0 < W && y0 >= -1 && y0 < H ? (y0 + 1) * W1 + x0 + 1
                                                                                          : -1;
    }
  }
  __syncthreads();   // counters zeroed
  DP_KS_STAMP(1);
#pragma unroll
  for (int u = 0; u < SORT_PPT; ++u)
    if (key[u] >= 0) atomicAdd(cnt + key[u], 1);
  __syncthreads();
  DP_KS_STAMP(2);
  // counts -> exclusive offsets (a contiguous range per thread), cnt[ncell] = the total
  const int per = (ncell + 1023) / 1024, c0 = min(ncell, tid * per), c1 = min(ncell, c0 + per);
  int s = 0;
  for (int c = c0; c < c1; ++c) s += cnt[c];
  int tot;
  int o = block_excl_scan(s, wsum, tot);
  for (int c = c0; c < c1; ++c) {
    const int n = cnt[c];
    cnt[c] = o;
    o += n;
  }
  if (tid == 0) cnt[ncell] = tot;
  __syncthreads();
  DP_KS_STAMP(3);
  // work items: pixel p's entries = its four cells' lists (the pixel is corner k of cell
  // (x - (k & 1), y - (k >> 1))), in chunks of SORT_ITEM; each item carries its lists' bounds.
  // Item slot p holds pixel p's first chunk (consecutive threads, consecutive 32-byte records;
  // an empty pixel's item has no entries), further chunks go past npix.
  const int lbase = l * npt;
  const int npix = H * W;
  int4* item = ws.item + ((int64_t)seg * ws.isz + ws.ibase[l]) * 2;
  for (int p = tid; p < npix; p += 1024) {
    const int py = p / W, c = (py + 1) * W1 + p - py * W + 1;
    const int cell[4] = {c, c - 1, c - W1, c - W1 - 1};
    int pr[4], base[4], n = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pr[k] = n;
      base[k] = lbase + cnt[cell[k]] - n;
      n += cnt[cell[k] + 1] - cnt[cell[k]];
    }
    const int4 i1 = make_int4(base[1], base[2], base[3], 0);
    item[2 * p] = make_int4(p, pr[1] | (pr[2] << 16), pr[3] | (n << 16), base[0]);
    item[2 * p + 1] = i1;
    for (int k = 1; k * SORT_ITEM < n; ++k) {   // rare: a hot pixel
      const int q = npix + atomicAdd(&novf, 1);
      item[2 * q] = make_int4(p | (k << 16), pr[1] | (pr[2] << 16), pr[3] | (n << 16), base[0]);
      item[2 * q + 1] = i1;
    }
  }
  __syncthreads();   // novf complete; the offsets become cursors below
  if (tid == 0) ws.nitem[seg * L + l] = npix + novf;
  DP_KS_STAMP(4);
  // pass 2: (token, a, fx, fy) at the point's slot of its cell's list (16-byte stores into this
  // block's own lq * P * 16-byte slab: its lines fill in L2)
  float4* gl = ws.list + (int64_t)seg * L * npt + lbase;
  const float* pa = ws.pa + (int64_t)seg * lq * LP;
#pragma unroll
  for (int u0 = 0; u0 < SORT_PPT; u0 += SORT_PPT / 2) {
    __builtin_amdgcn_sched_barrier(0);
    float x[SORT_PPT / 2], y[SORT_PPT / 2], aj[SORT_PPT / 2];
    int slot[SORT_PPT / 2];
#pragma unroll
    for (int u = 0; u < SORT_PPT / 2; ++u) {
      point_xy(u0 + u, x[u], y[u]);
      const int pt = min(tid + (u0 + u) * 1024, npt - 1);
      const int t = pt / P;
      aj[u] = pa[t * LP + l * P + pt - t * P];
      slot[u] = key[u0 + u] >= 0 ? atomicAdd(cnt + key[u0 + u], 1) : 0;
    }
#pragma unroll
    for (int u = 0; u < SORT_PPT / 2; ++u) {
      if (key[u0 + u] < 0) continue;
      const int t = (tid + (u0 + u) * 1024) / P;
      gl[slot[u]] = make_float4(__int_as_float(t), aj[u], x[u] - floorf(x[u]), y[u] - floorf(y[u]));
    }
  }
#ifdef DP_KS_TIMING
  __syncthreads();
#endif
  DP_KS_STAMP(5);
}

// msda_fused_bwd_kernel's gather backward for d offsets / d logits / d ref (16-byte lanes,
// CPT = dh / VEC lanes per (token, head)), segment-major (a wave's ppw pairs are consecutive tokens
// of one (image, head)). The points go CPT at a time; after the butterfly sums every lane of a
// pair holds each point's results and lane u keeps point u of the group, so the pair's results
// leave as contiguous runs at the end (no per-point scattered stores, no read-back for the
// softmax backward).
template <typename T, int CPT, int LPM>
__global__ __launch_bounds__(256) void msda_sorted_bwd_kernel(const T* __restrict__ value, int S, TLevels lv, int L,
                                                              int P, const float* __restrict__ oa,
                                                              const float* __restrict__ ref,
                                                              const T* __restrict__ gout, int ldg,
                                                              float* __restrict__ goa, float* __restrict__ gref,
                                                              int lq, int nh, int nseg, int bps, int spx, int segmap,
                                                              float* __restrict__ pa) {
  constexpr int VEC = Vec16<T>::N;
  constexpr int PPW = 64 / CPT;
  constexpr int KMAX = (LPM + CPT - 1) / CPT;   // kept points per lane, L * P <= LPM
  const int xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int seg = seg_of(xcd, bi / bps, spx, segmap), tb = bi - (bi / bps) * bps;
  if (seg >= nseg) return;
  const int lane = threadIdx.x & 63;
  const int slot = lane / CPT, c = lane - slot * CPT;
  const int t0 = (tb * 4 + (threadIdx.x >> 6)) * PPW;
  if (t0 >= lq) return;                           // whole waves leave together
  const int t = min(t0 + slot, lq - 1);           // a ragged last wave repeats its last token...
  const bool live = t0 + slot < lq;               // ...without storing anything
  const int b = seg / nh, h = seg - b * nh;
  const int r = b * lq + t;
  const int dh = CPT * VEC;
  const int C = nh * dh;
  const int LP = L * P;
  const int ncol = nh * LP * 3;
  const int ch = h * dh + c * VEC;
  const T* vb = value + (int64_t)b * S * C + ch;
  const float* orow = oa + (int64_t)r * ncol;
  const float* lg = orow + nh * LP * 2 + h * LP;
  const Vec16<T> gor = load16(gout + (int64_t)r * ldg + ch);
  // every point's logit and offsets up front (clamped indices: unconditional loads), so the loop
  // below waits only on the value rows
  constexpr int LPMAX = KMAX * CPT;
  float lgv[LPMAX], oxy[2 * LPMAX];
  if (LP == LPMAX && LPMAX % 4 == 0) {   // 16-byte loads (the head's offsets and logits are 16-byte aligned runs)
#pragma unroll
    for (int j = 0; j < 2 * LPMAX; j += 4) {
      const float4 x = *reinterpret_cast<const float4*>(orow + h * LPMAX * 2 + j);
      oxy[j] = x.x; oxy[j + 1] = x.y; oxy[j + 2] = x.z; oxy[j + 3] = x.w;
    }
#pragma unroll
    for (int j = 0; j < LPMAX; j += 4) {
      const float4 x = *reinterpret_cast<const float4*>(lg + j);
      lgv[j] = x.x; lgv[j + 1] = x.y; lgv[j + 2] = x.z; lgv[j + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < LPMAX; ++j) {
      const int jc = min(j, LP - 1);
      lgv[j] = lg[jc];
      oxy[2 * j] = orow[(h * LP + jc) * 2];
      oxy[2 * j + 1] = orow[(h * LP + jc) * 2 + 1];
    }
  }
  const float rx = ref[2 * r], ry = ref[2 * r + 1];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < LPMAX; ++j) mx = j < LP ? fmaxf(mx, lgv[j]) : mx;
  float den = 0.f;
#pragma unroll
  for (int j = 0; j < LPMAX; ++j) den += j < LP ? expf(lgv[j] - mx) : 0.f;
  const float inv = 1.f / den;
  float dot = 0.f, grx = 0.f, gry = 0.f;
  float ka[KMAX], kga[KMAX], kgx[KMAX], kgy[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i) ka[i] = kga[i] = kgx[i] = kgy[i] = 0.f;
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    if (i * CPT >= LP) break;   // (uniform; between groups only)
    // the group's CPT points: corners and weights, then all 4 * CPT row loads, then the math
    float fxu[CPT], fyu[CPT], au[CPT], Wu[CPT], Hu[CPT];
    int rcu[CPT][4];
    bool oku[CPT][4];
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const int j = i * CPT + u;
      const int l = min(j, LP - 1) / P;
      const int H = lv.h[l], W = lv.w[l];
      float x, y;
      msda_xy(rx, ry, oxy[2 * j], oxy[2 * j + 1], H, W, x, y);
      const float fx0 = floorf(x), fy0 = floorf(y);
      const int x0 = (int)fx0, y0 = (int)fy0;
      fxu[u] = x - fx0;
      fyu[u] = y - fy0;
      au[u] = j < LP ? expf(lgv[j] - mx) * inv : 0.f;   // a point past L*P contributes nothing
      Wu[u] = W;
      Hu[u] = H;
#pragma unroll
      for (int k = 0; k < 4; ++k) {   // unconditional loads at a clamped row, zeroed outside the map
        const int xi = x0 + (k & 1), yi = y0 + (k >> 1);
        oku[u][k] = xi >= 0 && xi < W && yi >= 0 && yi < H;
        rcu[u][k] = lv.start[l] + min(max(yi, 0), H - 1) * W + min(max(xi, 0), W - 1);
      }
    }
    Vec16<T> v[CPT][4];
#pragma unroll
    for (int u = 0; u < CPT; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[u][k] = load16(vb + (int64_t)rcu[u][k] * C);
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
      const float fx = fxu[u], fy = fyu[u], a = au[u];
      // d_k = <grad_out, corner k's channels> (the lane's VEC channels), 0 outside the map; then
      // the three point sums are bilinear forms in d: ga = sum w_k d_k, gx / gy its fx / fy slopes
      float d[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k] = oku[u][k] ? corner_dot(gor, v[u][k]) : 0.f;
      const float ga0 = (1.f - fx) * (1.f - fy) * d[0] + fx * (1.f - fy) * d[1] + (1.f - fx) * fy * d[2] + fx * fy * d[3];
      float ga = ga0;
      float gx = (d[1] - d[0]) * (1.f - fy) + (d[3] - d[2]) * fy;
      float gy = (d[2] - d[0]) * (1.f - fx) + (d[3] - d[1]) * fx;
#pragma unroll
      for (int o = CPT >> 1; o > 0; o >>= 1) {
        ga += __shfl_xor(ga, o, 64);
        gx += __shfl_xor(gx, o, 64);
        gy += __shfl_xor(gy, o, 64);
      }
      dot += a * ga;
      grx += a * gx * Wu[u];
      gry += a * gy * Hu[u];
      if (c == u) {
        ka[i] = a;
        kga[i] = ga;
        kgx[i] = a * gx;
        kgy[i] = a * gy;
      }
    }
  }
  if (!live) return;
  float* grow = goa + (int64_t)r * ncol;
  float* pat = pa + ((int64_t)seg * lq + t) * LP;
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const int j = i * CPT + c;
    if (j < LP) {
      *reinterpret_cast<float2*>(grow + (h * LP + j) * 2) = make_float2(kgx[i], kgy[i]);
      grow[nh * LP * 2 + h * LP + j] = ka[i] * (kga[i] - dot);   // softmax backward
      pat[j] = ka[i];                                            // the sort's value-gradient weights
    }
  }
  if (gref && c == 0) {
    unsafeAtomicAdd(gref + 2 * r, grx);
    unsafeAtomicAdd(gref + 2 * r + 1, gry);
  }
}

// K3: a group of G = dh / CPL lanes per work item (pixel, chunk), CPL channels per lane (16
// items per wave at dh 32 bf16: CPL 8, one 16-byte load per entry). The chunk's <= SORT_CHUNK entries of the pixel's four cell
// lists are loaded up front (G per step, one per lane) and turned into (token row, a * w_k), then
// broadcast one at a time from their lane while the grad_out row loads of consecutive entries are
// in flight (unconditional: a dead entry has weight 0 and row 0).
template <typename T, int G, int CPL>
__global__ __launch_bounds__(256) void msda_value_sum_kernel(const T* __restrict__ gout, int ldg,
                                                             float* __restrict__ gvalue, TLevels lv, int S, int L,
                                                             int P, int lq, int nh, int nseg, int bps_seg,
                                                             SortWs ws) {
  constexpr int VEC = Vec16<T>::N;
  static_assert(CPL % VEC == 0 && CPL % 4 == 0, "whole 16-byte loads per lane");
  constexpr int IPW = 64 / G;             // items per wave
  constexpr int EPL = SORT_CHUNK / G;     // entries per lane
  const int xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int seg = seg_of(xcd, bi / bps_seg, ws.spx, ws.segmap);
  if (seg >= nseg) return;
  int tb = bi - (bi / bps_seg) * bps_seg, l = 0;
  while (l + 1 < L && tb >= ws.bps[l]) tb -= ws.bps[l++];
  const int lane = threadIdx.x & 63;
  const int gi = lane / G, q = lane - gi * G, g0 = lane - q;
  const int wbase = (tb * 4 + (threadIdx.x >> 6)) * IPW;
  const int nitem = ws.nitem[seg * L + l];
  if (wbase >= nitem) return;              // whole waves past the item list leave
  const int it = min(wbase + gi, nitem - 1);
  const bool live = wbase + gi < nitem;
  const int4* ip = ws.item + ((int64_t)seg * ws.isz + ws.ibase[l] + it) * 2;
  const int4 ia = ip[0], ib = ip[1];
  const int p = ia.x & 0xffff, chunk = ia.x >> 16, total = ia.z >> 16;
  const int pr1 = ia.y & 0xffff, pr2 = ia.y >> 16, pr3 = ia.z & 0xffff;
  const int n = live ? min(SORT_ITEM, total - chunk * SORT_ITEM) : 0;
  const int b = seg / nh, h = seg - b * nh;
  const int dh = G * CPL;
  float* gp = gvalue + ((int64_t)b * S + lv.start[l] + p) * (nh * dh) + h * dh + CPL * q;
  float gold[CPL];   // the pixel's current gradient, loaded with the list entries
#pragma unroll
  for (int e = 0; e < CPL; e += 4) {
    const float4 x = *reinterpret_cast<const float4*>(gp + e);
    gold[e] = x.x; gold[e + 1] = x.y; gold[e + 2] = x.z; gold[e + 3] = x.w;
  }
  int nmax = n;   // the wave's longest chunk bounds the list and broadcast loops
#pragma unroll
  for (int s = G; s < 64; s <<= 1) nmax = max(nmax, __shfl_xor(nmax, s, 64));
  const T* gcol = gout + h * dh + CPL * q;
  float acc[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) acc[c] = 0.f;
  const float4* lst = ws.list + (int64_t)seg * L * lq * P;
  for (int r0 = 0; r0 < nmax; r0 += SORT_CHUNK) {   // rounds of SORT_CHUNK entries (uniform)
    int er[EPL];
    float ew[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      er[e] = 0;
      ew[e] = 0.f;
      if (r0 + e * G >= nmax) continue;   // (uniform)
      const int ie = e * G + q;
      const int ii = chunk * SORT_ITEM + r0 + ie;
      const int k = (ii >= pr1) + (ii >= pr2) + (ii >= pr3);
      const int sl = (k == 0 ? ia.w : k == 1 ? ib.x : k == 2 ? ib.y : ib.z) + ii;
      const bool ok = r0 + ie < n;
      const float4 en = lst[ok ? sl : 0];   // unconditional load (slot 0 for a dead entry), value dropped
      const float wx = (k & 1) ? en.z : 1.f - en.z, wy = (k & 2) ? en.w : 1.f - en.w;
      er[e] = b * lq + (ok ? __float_as_int(en.x) : 0);
      ew[e] = ok ? en.y * (wx * wy) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      if (r0 + e * G >= nmax) break;
      float gv[G][CPL];
#pragma unroll
      for (int s = 0; s < G; ++s) {
        const int rr = group_bcast<G>(er[e], s, g0);
#pragma unroll
        for (int c = 0; c < CPL; c += VEC) load_vec(gcol + (int64_t)rr * ldg + c, *reinterpret_cast<float(*)[VEC]>(&gv[s][c]));
      }
#pragma unroll
      for (int s = 0; s < G; ++s) {
        const float w = __int_as_float(group_bcast<G>(__float_as_int(ew[e]), s, g0));
#pragma unroll
        for (int c = 0; c < CPL; ++c) acc[c] += w * gv[s][c];
      }
    }
  }
  if (n <= 0) return;
  if (total > SORT_ITEM) {   // the pixel's lists span several items: they meet in float atomics
#pragma unroll
    for (int c = 0; c < CPL; ++c) unsafeAtomicAdd(gp + c, acc[c]);
  } else {                    // the only writer of this segment of the pixel's row
#pragma unroll
    for (int e = 0; e < CPL; e += 4)
      *reinterpret_cast<float4*>(gp + e) =
          make_float4(gold[e] + acc[e], gold[e + 1] + acc[e + 1], gold[e + 2] + acc[e + 2], gold[e + 3] + acc[e + 3]);
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

// dp_msda_bwd_sorted's workspace carved from base (NULL: sizes only); returns the bytes needed.
// Also fills the per-level cell / item bases and the LDS the KS block needs.
int64_t sort_ws_layout(int batch, int S, int lq, int nh, const TLevels& lv, int L, int P, char* base, SortWs* ws,
                       int* ks_lds = nullptr) {
  const int64_t nseg = (int64_t)batch * nh;
  const int npt = lq * P;
  int isz = 0, lds = 0;
  for (int l = 0; l < L; ++l) {
    const int cells = (lv.h[l] + 1) * (lv.w[l] + 1);
    const int items = lv.h[l] * lv.w[l] + (4 * npt + SORT_ITEM - 1) / SORT_ITEM;
    ws->ibase[l] = isz;
    isz += items;
    lds = std::max(lds, (cells + 1) * 4);
  }
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = o;
    o += (bytes + 255) / 256 * 256;
    return base ? base + at : nullptr;
  };
  ws->list = reinterpret_cast<float4*>(take(nseg * L * npt * 16));
  ws->pa = reinterpret_cast<float*>(take(nseg * npt * L * 4));
  ws->item = reinterpret_cast<int4*>(take(nseg * isz * 32));
  ws->nitem = reinterpret_cast<int32_t*>(take(nseg * L * 4));
#ifdef DP_KS_TIMING
  ws->dbg = reinterpret_cast<long long*>(take(nseg * L * 8 * 8));   // the workspace's last region
#endif
  ws->isz = isz;
  if (ks_lds) *ks_lds = lds;
  return o;
}

// a shape the sort handles: item fields are 16-bit (pixels per level, a pixel's entries), kept
// points per lane in K2 bounded (L * P <= 16)
bool sort_shape_ok(const TLevels& lv, int L, int P, int lq) {
  if (L * P > 16 || 4 * lq * P >= 65536 || lq * P > 1024 * SORT_PPT) return false;
  for (int l = 0; l < L; ++l)
    if (lv.h[l] * lv.w[l] >= 65536) return false;
  return true;
}

// LDS the sort block may declare (64 KiB: several blocks per CU)
constexpr int SORT_LDS_MAX = 64 * 1024 - 256;

}  // namespace

extern "C" int64_t dp_msda_bwd_ws_bytes(int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                                        int32_t lq, int32_t nhead, int32_t npoints) {
  if (batch <= 0 || S <= 0 || lq <= 0 || nhead <= 0 || nlevels <= 0 || nlevels > MAXL || npoints <= 0 || !lvl_hw ||
      nlevels * npoints > 16)
    return -1;
  TLevels lv;
  for (int l = 0; l < nlevels; ++l) {
    lv.h[l] = lvl_hw[2 * l];
    lv.w[l] = lvl_hw[2 * l + 1];
  }
  SortWs ws;
  int lds = 0;
  const int64_t bytes = sort_ws_layout(batch, S, lq, nhead, lv, nlevels, npoints, nullptr, &ws, &lds);
  return lds <= SORT_LDS_MAX && sort_shape_ok(lv, nlevels, npoints, lq) ? bytes : -1;
}

extern "C" int dp_msda_bwd_sorted(const void* value, int32_t batch, int32_t S, const int32_t* lvl_hw, int32_t nlevels,
                                  const float* offattn, const float* ref, const void* grad_out, int32_t ld_grad_out,
                                  int32_t lq, int32_t nhead, int32_t dh, int32_t npoints, float* grad_value,
                                  int32_t accumulate_value, float* grad_offattn, float* grad_ref, void* workspace,
                                  int64_t workspace_bytes, int32_t dtype, void* stream) {
  TLevels lv;
  const int rc = check_core(value, batch, S, lvl_hw, nlevels, offattn, ref, lq, nhead, dh, npoints, dtype, &lv);
  if (rc) return rc;
  DP_REQUIRE(grad_out && grad_offattn && grad_value && workspace, "dp_msda_bwd_sorted: null pointer");
  DP_REQUIRE(dh == 8 || dh == 16 || dh == 32 || dh == 64, "dp_msda_bwd_sorted: dh=%d (8, 16, 32 or 64)", dh);
  const int VEC = dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE((reinterpret_cast<uintptr_t>(grad_out) & 15) == 0 && ld_grad_out % VEC == 0 && ld_grad_out >= nhead * dh,
             "dp_msda_bwd_sorted: grad_out must be 16-byte aligned per row (ld %d)", ld_grad_out);
  DP_REQUIRE((reinterpret_cast<uintptr_t>(grad_value) & 15) == 0 && (reinterpret_cast<uintptr_t>(offattn) & 15) == 0,
             "dp_msda_bwd_sorted: grad_value and offattn must be 16-byte aligned");
  DP_REQUIRE((int64_t)batch * lq * nhead * nlevels * npoints * 4 < (1ll << 31), "dp_msda_bwd_sorted: too many entries");
  DP_REQUIRE(sort_shape_ok(lv, nlevels, npoints, lq),
             "dp_msda_bwd_sorted: shape outside the sort's range (levels x points <= 16, lq points <= 8192, "
             "H W < 65536 per level)");
  SortWs ws;
  int lds = 0;
  const int64_t need = sort_ws_layout(batch, S, lq, nhead, lv, nlevels, npoints, static_cast<char*>(workspace), &ws,
                                      &lds);
  DP_REQUIRE(lds <= SORT_LDS_MAX, "dp_msda_bwd_sorted: a level's cells + tokens need %d bytes of LDS (max %d)", lds,
             SORT_LDS_MAX);
  DP_REQUIRE(workspace_bytes >= need, "dp_msda_bwd_sorted: workspace %lld bytes, need %lld",
             (long long)workspace_bytes, (long long)need);
  hipStream_t s = as_stream(stream);
  const int nseg = batch * nhead;
  const int segs_per_xcd = (nseg + 7) / 8;
  ws.spx = segs_per_xcd;
  ws.segmap = getenv("DETRPOSE_MSDA_SEGMAP") ? atoi(getenv("DETRPOSE_MSDA_SEGMAP")) : 1;
  const size_t vbytes = (size_t)batch * S * nhead * dh * sizeof(float);
  if ((!accumulate_value && dp_zero_async(grad_value, vbytes, s)) ||
      (grad_ref && dp_zero_async(grad_ref, (size_t)batch * lq * 2 * sizeof(float), s)))
    return dp_check_launch("dp_msda_bwd_sorted(memset)");
  static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&msda_sort_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 SORT_LDS_MAX) == hipSuccess;
  DP_REQUIRE(lds_ok, "dp_msda_bwd_sorted: cannot raise the sort kernel's LDS limit");
  {
    const int cpt = dh / VEC;
    const int bps = (lq + 4 * (64 / cpt) - 1) / (4 * (64 / cpt));
    const dim3 grid(8 * segs_per_xcd * bps);
#define DP_K2(T, CPT)                                                                                              \
  if (nlevels * npoints <= 12)                                                                                    \
    hipLaunchKernelGGL((msda_sorted_bwd_kernel<T, CPT, 12>), grid, dim3(256), 0, s, (const T*)value, S, lv,      \
                       nlevels, npoints, offattn, ref, (const T*)grad_out, ld_grad_out, grad_offattn, grad_ref, lq,   \
                       nhead, nseg, bps, segs_per_xcd, ws.segmap, ws.pa);                                         \
  else                                                                                                            \
    hipLaunchKernelGGL((msda_sorted_bwd_kernel<T, CPT, 16>), grid, dim3(256), 0, s, (const T*)value, S, lv,      \
                       nlevels, npoints, offattn, ref, (const T*)grad_out, ld_grad_out, grad_offattn, grad_ref, lq,   \
                       nhead, nseg, bps, segs_per_xcd, ws.segmap, ws.pa)
    if (dtype == DP_BF16) {
      if (cpt == 1) { DP_K2(bf16_t, 1); } else if (cpt == 2) { DP_K2(bf16_t, 2); } else if (cpt == 4) { DP_K2(bf16_t, 4); }
      else { DP_K2(bf16_t, 8); }
    } else {
      if (cpt == 2) { DP_K2(float, 2); } else if (cpt == 4) { DP_K2(float, 4); } else if (cpt == 8) { DP_K2(float, 8); }
      else { DP_K2(float, 16); }
    }
#undef DP_K2
  }
  // the sort after K2: it reads the attention weights K2 stored (ws.pa)
  hipLaunchKernelGGL(msda_sort_kernel, dim3(8 * segs_per_xcd * nlevels), dim3(1024), lds, s, lv, nlevels, npoints,
                     offattn, ref, lq, nhead, nseg, ws);
  {
    // channels per lane: one 16-byte load per entry (8 bf16 / 4 f32; 16 items per wave at dh 32
    // bf16). 16 bf16 channels per lane (32 items per wave) measured slower: 172 / 241 vs 141 / 142
    // us (spread / clustered, r5y). DETRPOSE_MSDA_K3_CPL overrides (A/B)
    static const int cpl_env = getenv("DETRPOSE_MSDA_K3_CPL") ? atoi(getenv("DETRPOSE_MSDA_K3_CPL")) : 0;
    int cpl = dtype == DP_BF16 ? 8 : 4;
    if (cpl_env && cpl_env % VEC == 0 && dh % cpl_env == 0 && cpl_env <= 16) cpl = cpl_env;
    const int G = dh / cpl;
    const int ipb = 4 * (64 / G);   // items per block
    int bps_seg = 0;
    for (int l = 0; l < nlevels; ++l) {
      const int items = lv.h[l] * lv.w[l] + (4 * lq * npoints + SORT_ITEM - 1) / SORT_ITEM;
      ws.bps[l] = (items + ipb - 1) / ipb;
      bps_seg += ws.bps[l];
    }
    const dim3 grid(8 * segs_per_xcd * bps_seg);
#define DP_VSUM(T, GG, CC)                                                                                          \
  hipLaunchKernelGGL((msda_value_sum_kernel<T, GG, CC>), grid, dim3(256), 0, s, (const T*)grad_out, ld_grad_out,  \
                     grad_value, lv, S, nlevels, npoints, lq, nhead, nseg, bps_seg, ws)
    if (dtype == DP_BF16) {
      if (cpl == 16) {
        if (G == 1) DP_VSUM(bf16_t, 1, 16); else if (G == 2) DP_VSUM(bf16_t, 2, 16); else DP_VSUM(bf16_t, 4, 16);
      } else {
        if (G == 1) DP_VSUM(bf16_t, 1, 8); else if (G == 2) DP_VSUM(bf16_t, 2, 8); else if (G == 4) DP_VSUM(bf16_t, 4, 8);
        else DP_VSUM(bf16_t, 8, 8);
      }
    } else {
      if (cpl == 8) {
        if (G == 1) DP_VSUM(float, 1, 8); else if (G == 2) DP_VSUM(float, 2, 8); else if (G == 4) DP_VSUM(float, 4, 8);
        else DP_VSUM(float, 8, 8);
      } else if (cpl == 16) {
        if (G == 1) DP_VSUM(float, 1, 16); else if (G == 2) DP_VSUM(float, 2, 16); else DP_VSUM(float, 4, 16);
      } else {
        if (G == 2) DP_VSUM(float, 2, 4); else if (G == 4) DP_VSUM(float, 4, 4); else if (G == 8) DP_VSUM(float, 8, 4);
        else DP_VSUM(float, 16, 4);
      }
    }
#undef DP_VSUM
  }
  return dp_check_launch("dp_msda_bwd_sorted");
}

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
  if (dp_zero_async(grad_value, (size_t)batch * S * nhead * dh * sizeof(float), s))
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
       dp_zero_async(grad_value, (size_t)batch * S * nhead * dh * sizeof(float), s)) ||
      (grad_ref && dp_zero_async(grad_ref, (size_t)batch * lq * 2 * sizeof(float), s)))
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
