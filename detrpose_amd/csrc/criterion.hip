// Training criterion of DETRPose on the GPU: Hungarian matching and the
// default losses (vfl + keypoints L1 + OKS), with no device->host synchronisation.
//
// The reference (src/models/detrpose/criterion.py:285-435, matcher.py:47-112) builds the
// matching cost with torch ops, copies every cost matrix to the host (.cpu(), one sync per
// decoder/aux head) and solves it with scipy's linear_sum_assignment; then ~20 small torch
// ops per head compute the losses. Here:
//   dp_hungarian_match  one 64-lane workgroup per (head, image): the image's cost block
//                       (class focal cost + keypoint L1 + OKS cost, matcher.py:59-87) lands
//                       in LDS, then the wave runs scipy's shortest-augmenting-path LSAP
//                       (Crouse 2016; restated in oracle/lsap_cpu.py, tie-breaks included)
//                       on it in f64, lanes owning columns, the Dijkstra argmin a wave
//                       reduction. Output: match[h][b][q] = target index or -1.
//   dp_match_union      Criterion._get_go_indices (criterion.py:247-268): per query the
//                       target matched by the most heads (ties: the smallest target index,
//                       i.e. a stable sort), and the pair count num_boxes_go.
//   dp_pose_loss        one workgroup per head: loss_vfl (criterion.py:58-93) over all
//                       logits, loss_keypoints + loss_oks (200-229) over the union matching,
//                       each already multiplied by its weight_dict entry and divided by its
//                       normaliser, plus their gradients w.r.t. the head's logits/keypoints
//                       (the losses are sums of per-element terms, so forward and backward
//                       are one pass). Sums are fixed-order block reductions: deterministic.
#include "common.h"

// costs and losses follow the reference's torch expressions op by op: no FMA contraction
#pragma clang fp contract(off)

namespace {

constexpr int KPMAX = 32;   // keypoints per instance (17 COCO, 14 CrowdPose)

// matcher.py:59-87, one (query, target) entry. Op order follows the reference's torch
// expressions (fp contraction off in this file) so the f32 costs agree to rounding.
__device__ float match_cost(const float* __restrict__ lg, const float* __restrict__ kp, int label,
                            const float* __restrict__ tk, float area, const float* __restrict__ var2, int nkp,
                            float cost_class, float cost_kp, float cost_oks, float alpha) {
  const float p = 1.f / (1.f + expf(-lg[label]));
  const float neg = (1.f - alpha) * (p * p) * (-logf(1.f - p + 1e-8f));
  const float pos = alpha * ((1.f - p) * (1.f - p)) * (-logf(p + 1e-8f));
  const float cc = pos - neg;
  float l1 = 0.f, num = 0.f, vs = 0.f;
  for (int k = 0; k < nkp; ++k) {
    const float v = tk[2 * nkp + k];
    const float dx = kp[2 * k] - tk[2 * k], dy = kp[2 * k + 1] - tk[2 * k + 1];
    l1 += fabsf(dx) * v + fabsf(dy) * v;
    const float d0 = (dx * dx + dy * dy) / (area * var2[k]);
    num += expf(-d0) * v;
    vs += v;
  }
  float oks = num / (vs + 1e-6f);
  oks = fmaxf(oks, 1e-6f);
  return cost_class * cc + cost_kp * l1 + cost_oks * (1.f - oks);
}

__device__ __forceinline__ double shfl_d(double x, int lane) {
  const int2 v = *reinterpret_cast<int2*>(&x);
  int2 r;
  r.x = __shfl(v.x, lane, 64);
  r.y = __shfl(v.y, lane, 64);
  return *reinterpret_cast<double*>(&r);
}

// LDS layout of one (head, image) problem
struct LsapSmem {
  float* cost;     // [Q][nt] (matcher orientation: rows = queries)
  double* u;       // [nr]
  double* v;       // [nc]
  double* spc;     // [nc] shortest path costs
  int* path;       // [nc]
  int* row4col;    // [nc]
  int* col4row;    // [nr]
  int* rem;        // [nc] scipy's `remaining` vector
  int* pos;        // [nc] position of column j in rem (-1 once scanned)
  unsigned char* SR;
  unsigned char* SC;
};

constexpr int DP_MATCH_INFEASIBLE = -2;

__global__ __launch_bounds__(64) void hungarian_kernel(
    const float* __restrict__ logits, int64_t lg_h, int64_t lg_b, int lg_q, int ncls,
    const float* __restrict__ kps, int64_t kp_h, int64_t kp_b, int kp_q, int nkp,
    const int* __restrict__ tgt_off, const int* __restrict__ tgt_label, const float* __restrict__ tgt_kps,
    const float* __restrict__ tgt_area, int B, int Q, int max_t, float cost_class, float cost_kp, float cost_oks,
    float alpha, const float* __restrict__ sigmas, int* __restrict__ match, float* __restrict__ cost_out) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  const int h = blockIdx.x / B, b = blockIdx.x - h * B;
  const int lane = threadIdx.x;
  const int t0 = tgt_off[b], nt = tgt_off[b + 1] - t0;
  int* mt = match + ((int64_t)h * B + b) * Q;
  for (int q = lane; q < Q; q += 64) mt[q] = -1;
  if (nt <= 0 || Q <= 0) return;

  __shared__ float var2[KPMAX];
  if (lane < nkp) {
    const float s2 = sigmas[lane] * 2.f;
    var2[lane] = s2 * s2 * 2.f;   // (sigmas * 2) ** 2, times the 2 of matcher.py:77
  }
  // LDS carve: the f64 arrays first (8-byte aligned), then f32 / i32 / u8
  const bool tr = nt < Q;           // scipy transposes when rows (queries) > cols (targets)
  const int nr = tr ? nt : Q, nc = tr ? Q : nt;
  LsapSmem s;
  char* p = dsm;
  s.u = reinterpret_cast<double*>(p); p += 8 * nr;
  s.v = reinterpret_cast<double*>(p); p += 8 * nc;
  s.spc = reinterpret_cast<double*>(p); p += 8 * nc;
  s.cost = reinterpret_cast<float*>(p); p += 4 * (size_t)Q * nt;
  s.path = reinterpret_cast<int*>(p); p += 4 * nc;
  s.row4col = reinterpret_cast<int*>(p); p += 4 * nc;
  s.col4row = reinterpret_cast<int*>(p); p += 4 * nr;
  s.rem = reinterpret_cast<int*>(p); p += 4 * nc;
  s.pos = reinterpret_cast<int*>(p); p += 4 * nc;
  s.SR = reinterpret_cast<unsigned char*>(p); p += nr;
  s.SC = reinterpret_cast<unsigned char*>(p);
  __syncthreads();

  // ---- cost block [Q][nt]
  const float* lgb = logits + h * lg_h + b * lg_b;
  const float* kpb = kps + h * kp_h + b * kp_b;
  for (int e = lane; e < Q * nt; e += 64) {
    const int q = e / nt, t = e - q * nt;
    const int tg = t0 + t;
    const float c = match_cost(lgb + (int64_t)q * lg_q, kpb + (int64_t)q * kp_q, tgt_label[tg],
                               tgt_kps + (int64_t)tg * 3 * nkp, tgt_area[tg], var2, nkp, cost_class, cost_kp,
                               cost_oks, alpha);
    s.cost[e] = c;
    if (cost_out) cost_out[(((int64_t)h * B + b) * Q + q) * max_t + t] = c;
  }
  for (int i = lane; i < nr; i += 64) s.u[i] = 0.0, s.col4row[i] = -1;
  for (int j = lane; j < nc; j += 64) s.v[j] = 0.0, s.row4col[j] = -1;
  __syncthreads();
  auto cost = [&](int i, int j) -> double { return (double)(tr ? s.cost[j * nt + i] : s.cost[i * nt + j]); };

  // ---- shortest augmenting path, one row at a time (oracle/lsap_cpu.py)
  bool feasible = true;
  for (int cur = 0; cur < nr; ++cur) {
    for (int j = lane; j < nc; j += 64) {
      s.spc[j] = INFINITY;
      s.path[j] = -1;
      s.SC[j] = 0;
      s.rem[nc - 1 - j] = j;   // remaining[it] = nc - it - 1
      s.pos[j] = nc - 1 - j;
    }
    for (int i = lane; i < nr; i += 64) s.SR[i] = 0;
    __syncthreads();
    int num_rem = nc, i = cur, sink = -1;
    double min_val = 0.0;
    bool ok = true;
    while (sink == -1) {
      if (lane == 0) s.SR[i] = 1;
      const double ui = s.u[i];
      // relax the remaining columns; the lane's best under scipy's scan rule: smallest cost,
      // then among equal costs an unassigned column scanned last, else the first scanned
      double best = INFINITY;
      int bkey = 0x7fffffff;
      for (int j = lane; j < nc; j += 64) {
        const int it = s.pos[j];
        if (it < 0) continue;
        const double r = min_val + cost(i, j) - ui - s.v[j];
        double sj = s.spc[j];
        if (r < sj) {
          s.path[j] = i;
          s.spc[j] = sj = r;
        }
        const int key = s.row4col[j] == -1 ? (nc - 1 - it) : (nc + it);
        if (sj < best || (sj == best && key < bkey)) best = sj, bkey = key;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ob = shfl_d(best, lane ^ o);
        const int ok_ = __shfl_xor(bkey, o, 64);
        if (ob < best || (ob == best && ok_ < bkey)) best = ob, bkey = ok_;
      }
      if (bkey == 0x7fffffff || best == INFINITY) {   // infeasible (NaN / inf costs)
        ok = false;
        break;
      }
      min_val = best;
      const int it = bkey < nc ? nc - 1 - bkey : bkey - nc;
      const int j = s.rem[it];
      const int r4c = s.row4col[j];
      __syncthreads();
      if (lane == 0) {
        s.SC[j] = 1;
        --num_rem;
        const int moved = s.rem[num_rem];
        s.rem[it] = moved;
        s.pos[moved] = it;
        s.pos[j] = -1;
      } else {
        --num_rem;
      }
      if (r4c == -1) sink = j;
      else i = r4c;
      __syncthreads();
    }
    if (!ok) {
      feasible = false;
      break;
    }
    // dual update (u of the scanned rows, v of the scanned columns)
    for (int ii = lane; ii < nr; ii += 64)
      if (ii == cur) s.u[ii] += min_val;
      else if (s.SR[ii]) s.u[ii] += min_val - s.spc[s.col4row[ii]];
    for (int jj = lane; jj < nc; jj += 64)
      if (s.SC[jj]) s.v[jj] -= min_val - s.spc[jj];
    __syncthreads();
    if (lane == 0) {   // augment along the path
      int j = sink;
      while (true) {
        const int ii = s.path[j];
        s.row4col[j] = ii;
        const int nxt = s.col4row[ii];
        s.col4row[ii] = j;
        j = nxt;
        if (ii == cur) break;
      }
    }
    __syncthreads();
  }
  if (!feasible) {
    // NaN / inf costs: scipy's linear_sum_assignment raises; here every query of the image
    // gets DP_MATCH_INFEASIBLE and dp_pose_loss turns that head's losses into NaN
    __syncthreads();
    for (int q = lane; q < Q; q += 64) mt[q] = DP_MATCH_INFEASIBLE;
    return;
  }
  // match[q] = target of query q
  for (int r = lane; r < nr; r += 64) {
    const int c = s.col4row[r];
    if (c < 0) continue;
    if (tr) mt[c] = r;
    else mt[r] = c;
  }
}

// Criterion._get_go_indices: per query the target chosen by the most heads, ties broken
// toward the smaller target index (the reference sorts the counts with torch.argsort,
// whose order among equal counts is unspecified; a stable sort gives this rule).
__global__ __launch_bounds__(256) void match_union_kernel(const int* __restrict__ match, int H, int B, int Q,
                                                          int* __restrict__ go, float* __restrict__ n_go) {
  __shared__ int red[4];
  int cnt = 0;
  for (int e = threadIdx.x; e < B * Q; e += 256) {
    const int b = e / Q, q = e - b * Q;
    int best = -1, bc = 0;
    for (int h = 0; h < H; ++h) {
      const int t = match[((int64_t)h * B + b) * Q + q];
      if (t < 0) continue;
      int c = 0;
      for (int h2 = 0; h2 < H; ++h2) c += match[((int64_t)h2 * B + b) * Q + q] == t;
      if (c > bc || (c == bc && t < best)) bc = c, best = t;
    }
    go[e] = best;
    cnt += best >= 0;
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) *n_go = (float)(red[0] + red[1] + red[2] + red[3]);
}

struct LossHeads {
  dp_loss_head h[DP_LOSS_MAX_HEADS];
};

__device__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// OKS of one prediction against one target (keypoint_loss.py:5-19, clamp 1e-6 of :29);
// optionally the gradient of (1 - oks) w.r.t. the predicted coordinates
__device__ float oks_of(const float* kp, const float* tk, float area, const float* var2, int nkp, float* g_one_minus) {
  float num = 0.f, vs = 0.f;
  for (int k = 0; k < nkp; ++k) {
    const float v = tk[2 * nkp + k];
    const float dx = kp[2 * k] - tk[2 * k], dy = kp[2 * k + 1] - tk[2 * k + 1];
    num += expf(-((dx * dx + dy * dy) / (area * var2[k]))) * v;
    vs += v;
  }
  const float den = vs + 1e-6f;
  const float oks = num / den;
  if (g_one_minus) {
    const bool pass = oks >= 1e-6f;   // clamp(min) passes the gradient where x >= min
    for (int k = 0; k < nkp; ++k) {
      const float v = tk[2 * nkp + k];
      const float dx = kp[2 * k] - tk[2 * k], dy = kp[2 * k + 1] - tk[2 * k + 1];
      const float a = area * var2[k];
      const float e = expf(-((dx * dx + dy * dy) / a)) * v;
      // d(1 - oks)/dpx = -(e * (-2 dx / a)) / den
      g_one_minus[2 * k] = pass ? (e * 2.f * dx / a) / den : 0.f;
      g_one_minus[2 * k + 1] = pass ? (e * 2.f * dy / a) / den : 0.f;
    }
  }
  return fmaxf(oks, 1e-6f);
}

__global__ __launch_bounds__(256) void pose_loss_kernel(
    const LossHeads heads, int B, int Q, int ncls, int nkp, const int* __restrict__ go,
    const int* __restrict__ tgt_off, const int* __restrict__ tgt_label, const float* __restrict__ tgt_kps,
    const float* __restrict__ tgt_area, const float* __restrict__ sigmas, float alpha, float gamma,
    const float* __restrict__ n_boxes, const float* __restrict__ n_boxes_go, float world, float w_vfl, float w_kp,
    float w_oks, float* __restrict__ losses, float* __restrict__ g_logits, float* __restrict__ g_kp_l1,
    float* __restrict__ g_kp_oks) {
  const int h = blockIdx.x;
  const dp_loss_head& H = heads.h[h];
  __shared__ float var2[KPMAX];
  __shared__ float red[4];
  if (threadIdx.x < nkp) {
    const float s2 = sigmas[threadIdx.x] * 2.f;
    var2[threadIdx.x] = s2 * s2 * 2.f;
  }
  __syncthreads();
  const float nb = fmaxf(*n_boxes / world, 1.f);
  const float nbg = fmaxf(*n_boxes_go / world, 1.f);
  const int K2 = 2 * nkp;
  float s_vfl = 0.f, s_l1 = 0.f, s_oks = 0.f;
  for (int e = threadIdx.x; e < B * Q; e += 256) {
    const int b = e / Q, q = e - b * Q;
    const float* lg = H.logits + b * H.lg_b + (int64_t)q * H.lg_q;
    const float* kp = H.kps + b * H.kp_b + (int64_t)q * H.kp_q;
    float* gl = g_logits + (((int64_t)h * B + b) * Q + q) * ncls;
    // ---- vfl (criterion.py:58-93): target score = detached OKS at the matched class
    const int t = H.match[e];
    int label = -1;
    float ts = 0.f;
    if (t == DP_MATCH_INFEASIBLE) s_vfl = NAN;   // the matching failed: report it in the loss
    if (t >= 0) {
      const int tg = tgt_off[b] + t;
      label = tgt_label[tg];
      ts = oks_of(kp, tgt_kps + (int64_t)tg * 3 * nkp, tgt_area[tg], var2, nkp, nullptr);
    }
    for (int c = 0; c < ncls; ++c) {
      const float x = lg[c];
      const float tgt = c == label ? 1.f : 0.f;
      const float tsc = c == label ? ts : 0.f;
      const float ps = 1.f / (1.f + expf(-x));
      const float w = alpha * powf(ps, gamma) * (1.f - tgt) + tsc;
      // binary_cross_entropy_with_logits, torch's stable form
      const float mx = fmaxf(-x, 0.f);
      const float bce = (1.f - tsc) * x + mx + logf(expf(-mx) + expf(-x - mx));
      s_vfl += w * bce;
      gl[c] = w_vfl * w * (ps - tsc) / nb;
    }
    // ---- keypoints L1 + OKS over the union matching (criterion.py:200-229)
    float* g1 = g_kp_l1 + (((int64_t)h * B + b) * Q + q) * K2;
    float* g2 = g_kp_oks + (((int64_t)h * B + b) * Q + q) * K2;
    const int tu = go[e];
    if (tu >= 0) {
      const int tg = tgt_off[b] + tu;
      const float* tk = tgt_kps + (int64_t)tg * 3 * nkp;
      float gom[2 * KPMAX];
      const float oks = oks_of(kp, tk, tgt_area[tg], var2, nkp, gom);
      s_oks += 1.f - oks;
      for (int k = 0; k < K2; ++k) {
        const float v = tk[2 * nkp + k / 2];
        const float d = kp[k] - tk[k];
        s_l1 += fabsf(d) * v;
        g1[k] = w_kp * ((d > 0.f) - (d < 0.f)) * v / nbg;
        g2[k] = w_oks * gom[k] / nbg;
      }
    } else {
      for (int k = 0; k < K2; ++k) g1[k] = 0.f, g2[k] = 0.f;
    }
  }
  s_vfl = block_sum256(s_vfl, red);
  s_l1 = block_sum256(s_l1, red);
  s_oks = block_sum256(s_oks, red);
  if (threadIdx.x == 0) {
    losses[3 * h + 0] = w_vfl * s_vfl / nb;
    losses[3 * h + 1] = w_kp * s_l1 / nbg;
    losses[3 * h + 2] = w_oks * s_oks / nbg;
  }
}

}  // namespace

extern "C" int dp_hungarian_match(const float* logits, int64_t lg_h, int64_t lg_b, int lg_q, int ncls,
                                  const float* kps, int64_t kp_h, int64_t kp_b, int kp_q, int nkp, const int* tgt_off,
                                  const int* tgt_label, const float* tgt_kps, const float* tgt_area, int H, int B,
                                  int Q, int max_t, float cost_class, float cost_kp, float cost_oks, float alpha,
                                  const float* sigmas, int* match, float* cost_out, void* stream) {
  DP_REQUIRE(H > 0 && B > 0 && Q > 0 && max_t >= 0 && ncls > 0, "dp_hungarian_match: bad sizes H=%d B=%d Q=%d T=%d", H,
             B, Q, max_t);
  DP_REQUIRE(nkp > 0 && nkp <= KPMAX, "dp_hungarian_match: %d keypoints (1..%d)", nkp, KPMAX);
  DP_REQUIRE(logits && kps && tgt_off && match && sigmas, "dp_hungarian_match: null pointer");
  const int nr = max_t < Q ? max_t : Q, nc = max_t < Q ? Q : max_t;
  const size_t smem = 8 * (size_t)(nr + 2 * nc) + 4 * (size_t)Q * max_t + 4 * (size_t)(3 * nc + nr + nc) + nr + nc + 16;
  DP_REQUIRE(smem <= 160 * 1024, "dp_hungarian_match: %d queries x %d targets need %zu B of LDS (> 160 KiB)", Q, max_t,
             smem);
  hipLaunchKernelGGL(hungarian_kernel, dim3(H * B), dim3(64), smem, as_stream(stream), logits, lg_h, lg_b, lg_q, ncls,
                     kps, kp_h, kp_b, kp_q, nkp, tgt_off, tgt_label, tgt_kps, tgt_area, B, Q, max_t, cost_class,
                     cost_kp, cost_oks, alpha, sigmas, match, cost_out);
  return dp_check_launch("dp_hungarian_match");
}

extern "C" int dp_match_union(const int* match, int H, int B, int Q, int* go, float* n_go, void* stream) {
  DP_REQUIRE(H > 0 && B > 0 && Q > 0 && match && go && n_go, "dp_match_union: bad arguments");
  hipLaunchKernelGGL(match_union_kernel, dim3(1), dim3(256), 0, as_stream(stream), match, H, B, Q, go, n_go);
  return dp_check_launch("dp_match_union");
}

extern "C" int dp_pose_loss(const dp_loss_head* heads, int H, int B, int Q, int ncls, int nkp, const int* go,
                            const int* tgt_off, const int* tgt_label, const float* tgt_kps, const float* tgt_area,
                            const float* sigmas, float alpha, float gamma, const float* n_boxes,
                            const float* n_boxes_go, float world, float w_vfl, float w_kp, float w_oks, float* losses,
                            float* g_logits, float* g_kp_l1, float* g_kp_oks, void* stream) {
  DP_REQUIRE(H > 0 && H <= DP_LOSS_MAX_HEADS && B > 0 && Q > 0 && ncls > 0 && world >= 1.f,
             "dp_pose_loss: bad sizes (H=%d, at most %d heads)", H, DP_LOSS_MAX_HEADS);
  DP_REQUIRE(nkp > 0 && nkp <= KPMAX, "dp_pose_loss: %d keypoints (1..%d)", nkp, KPMAX);
  DP_REQUIRE(heads && go && tgt_off && n_boxes && n_boxes_go && losses && g_logits && g_kp_l1 && g_kp_oks,
             "dp_pose_loss: null pointer");
  LossHeads hs{};
  for (int i = 0; i < H; ++i) hs.h[i] = heads[i];
  hipLaunchKernelGGL(pose_loss_kernel, dim3(H), dim3(256), 0, as_stream(stream), hs, B, Q, ncls, nkp, go, tgt_off, tgt_label, tgt_kps,
                     tgt_area, sigmas, alpha, gamma, n_boxes, n_boxes_go, world, w_vfl, w_kp, w_oks, losses, g_logits,
                     g_kp_l1, g_kp_oks);
  return dp_check_launch("dp_pose_loss");
}
