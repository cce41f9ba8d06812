// Decoder-side small kernels: two-stage query selection, reference-point bookkeeping,
// the f32 prediction heads, FDR integral refinement, LQE statistics and PostProcess.
// All tiny (<= a few MB) and latency-bound; kept in f32 regardless of the activation
// dtype so the keypoint arithmetic matches the reference's f32.
#include "common.h"

namespace {

// ------------------------------------------------------------------ top-k (radix select)
__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

constexpr int TOPK_THREADS = 256;
constexpr int TOPK_MAXN = 16384;

__device__ int block_excl_scan(int v, int* buf, int* total) {
  // simple Hillis-Steele in LDS over 256 threads
  const int t = threadIdx.x;
  buf[t] = v;
  __syncthreads();
  for (int o = 1; o < TOPK_THREADS; o <<= 1) {
    int x = t >= o ? buf[t - o] : 0;
    __syncthreads();
    buf[t] += x;
    __syncthreads();
  }
  const int incl = buf[t];
  *total = buf[TOPK_THREADS - 1];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(TOPK_THREADS) void topk_kernel(const float* __restrict__ x, int n, int ld, int k,
                                                            float* __restrict__ ov, int64_t* __restrict__ oi) {
  extern __shared__ uint32_t keys[];           // [n]
  // NH copies of the digit histogram, lane l adding into copy l % NH: the sigmoid scores share
  // their top key bytes, so one shared histogram serialises every wave on one or two bins
  // (70 % of the kernel's LDS cycles were bank conflicts); the copies are summed per pass
  constexpr int NH = 16, HP = 257;
  __shared__ int hcopy[NH * HP];
  __shared__ int hist[256];
  __shared__ int scan_buf[TOPK_THREADS];
  __shared__ uint32_t s_prefix;
  __shared__ int s_kk;
  __shared__ uint32_t ck[256];
  __shared__ int ci[256];
  const int t = threadIdx.x;
  const float* row = x + (int64_t)blockIdx.x * ld;
  for (int i = t; i < n; i += TOPK_THREADS) keys[i] = f2key(row[i]);
  if (t == 0) {
    s_prefix = 0;
    s_kk = k;
  }
  __syncthreads();
  uint32_t mask = 0;
  int* const hmine = hcopy + (t % NH) * HP;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int e = t; e < NH * HP; e += TOPK_THREADS) hcopy[e] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    for (int i = t; i < n; i += TOPK_THREADS) {
      const uint32_t kv = keys[i];
      if ((kv & mask) == prefix) atomicAdd(&hmine[(kv >> shift) & 255], 1);
    }
    __syncthreads();
    {
      int sum = 0;
#pragma unroll
      for (int c = 0; c < NH; ++c) sum += hcopy[c * HP + t];
      hist[t] = sum;
    }
    __syncthreads();
    if (t == 0) {
      int cum = 0, kk = s_kk, d = 255;
      for (; d > 0; --d) {
        if (cum + hist[d] >= kk) break;
        cum += hist[d];
      }
      s_kk = kk - cum;
      s_prefix = prefix | ((uint32_t)d << shift);
    }
    mask |= 255u << shift;
    __syncthreads();
  }
  const uint32_t T = s_prefix;
  const int kk = s_kk;  // how many keys == T to take (lowest indices first)
  // contiguous chunks per thread keep index order across the scan
  const int chunk = (n + TOPK_THREADS - 1) / TOPK_THREADS;
  const int b0 = t * chunk, b1 = min(n, b0 + chunk);
  int ngt = 0, neq = 0;
  for (int i = b0; i < b1; ++i) {
    ngt += keys[i] > T;
    neq += keys[i] == T;
  }
  int tot_gt, tot_eq;
  const int off_gt = block_excl_scan(ngt, scan_buf, &tot_gt);
  int off_eq = block_excl_scan(neq, scan_buf, &tot_eq);
  int pg = off_gt;
  for (int i = b0; i < b1; ++i) {
    const uint32_t kv = keys[i];
    if (kv > T) {
      ck[pg] = kv;
      ci[pg] = i;
      ++pg;
    } else if (kv == T) {
      if (off_eq < kk) {
        ck[tot_gt + off_eq] = kv;
        ci[tot_gt + off_eq] = i;
      }
      ++off_eq;
    }
  }
  __syncthreads();
  int np2 = 1;
  while (np2 < k) np2 <<= 1;
  if (t >= k && t < np2) {
    ck[t] = 0;
    ci[t] = 0x7fffffff;
  }
  __syncthreads();
  // bitonic sort: descending key, ascending index
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (t < np2) {
        const int j = t ^ stride;
        if (j > t) {
          const bool desc = (t & size) == 0;
          const uint32_t ka = ck[t], kb = ck[j];
          const int ia = ci[t], ib = ci[j];
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (a_first != desc) {
            ck[t] = kb; ck[j] = ka;
            ci[t] = ib; ci[j] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  if (t < k) {
    ov[(int64_t)blockIdx.x * k + t] = key2f(ck[t]);
    oi[(int64_t)blockIdx.x * k + t] = ci[t];
  }
}

// ------------------------------------------------------------------ two-stage
// G lanes per row (64/G rows per wave), 16-byte chunks of the row per lane, weights f32.
template <typename T, int G>
__global__ __launch_bounds__(256) void class_max_kernel(const T* __restrict__ x, int rows, int c,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        int ncls, float* __restrict__ out) {
  constexpr int VEC = Vec16<T>::N;
  const int lane = threadIdx.x & 63, sub = lane % G;
  const int r = (blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / G) + lane / G;
  const bool ok = r < rows;
  const int nch = c / VEC;
  const T* xr = x + (int64_t)(ok ? r : 0) * c;
  float best = -INFINITY;
  for (int j = 0; j < ncls; ++j) {
    float s = 0.f;
    for (int ch = sub; ch < nch; ch += G) {
      const Vec16<T> v = load16(xr + ch * VEC);
      const float* wj = w + j * c + ch * VEC;
#pragma unroll
      for (int t = 0; t < VEC; ++t) s = fmaf(v.get(t), wj[t], s);
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    best = fmaxf(best, s + b[j]);
  }
  if (ok && sub == 0) out[r] = best;
}

template <typename T>
__global__ __launch_bounds__(256) void gather_rows_kernel(const T* __restrict__ src, int64_t sbs,
                                                          const int64_t* __restrict__ idx, int batch, int k, int c,
                                                          T* __restrict__ dst) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)batch * k * c) return;
  const int64_t r = gid / c;
  const int i = (int)(gid - r * c);
  const int b = (int)(r / k);
  dst[gid] = src[(int64_t)b * sbs + idx[r] * c + i];
}

__global__ void refpoint_init_kernel(const float* __restrict__ delta, const float* __restrict__ anchors,
                                     const int64_t* __restrict__ idx, int rows, int nkp, float* __restrict__ ref) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const int64_t a = idx[r];
  const float ax = anchors[2 * a], ay = anchors[2 * a + 1];
  float* o = ref + (int64_t)r * (nkp + 1) * 2;
  float sx = 0.f, sy = 0.f;
  for (int j = 0; j < nkp; ++j) {
    const float x = 1.f / (1.f + expf(-(delta[(int64_t)r * nkp * 2 + 2 * j] + ax)));
    const float y = 1.f / (1.f + expf(-(delta[(int64_t)r * nkp * 2 + 2 * j + 1] + ay)));
    o[2 + 2 * j] = x;
    o[3 + 2 * j] = y;
    sx += x;
    sy += y;
  }
  o[0] = sx / nkp;
  o[1] = sy / nkp;
}

__global__ void broadcast_kernel(const uint8_t* __restrict__ src, int64_t bytes, uint8_t* __restrict__ dst,
                                 int64_t total, int vec) {
  int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    if (gid * 16 >= total) return;
    const int64_t off = gid * 16;
    *reinterpret_cast<uint4*>(dst + off) = *reinterpret_cast<const uint4*>(src + off % bytes);
  } else {
    if (gid >= total) return;
    dst[gid] = src[gid % bytes];
  }
}

// one thread = 8 consecutive channels of one (row, keypoint): the chunk lies in one half
// (pos_y | pos_x, c/2 % 8 == 0), so one coordinate; 16-byte (bf16) / 2x16-byte (f32) store
template <typename T>
__global__ __launch_bounds__(256) void sine_embed_kernel(const float* __restrict__ ref, int rows, int nkp, int c,
                                                         const float* __restrict__ dim_t, T* __restrict__ out) {
  const unsigned nch = (unsigned)(c >> 3);
  const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (unsigned)(rows * nkp) * nch) return;
  const unsigned rk = gid / nch;
  const int ch0 = (int)(gid - rk * nch) * 8;
  const unsigned r = rk / (unsigned)nkp;
  const int kp = (int)(rk - r * (unsigned)nkp);
  const int half = c >> 1;
  const float* p = ref + ((int64_t)r * (nkp + 1) + 1 + kp) * 2;
  const bool ylow = ch0 < half;
  const int i0 = ylow ? ch0 : ch0 - half;
  const float coord = (ylow ? p[1] : p[0]) * 6.283185307179586f;  // cat(pos_y, pos_x)
  float v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const float a = coord / dim_t[i0 + t];
    v[t] = ((i0 + t) & 1) ? __cosf(a) : __sinf(a);
  }
  T* o = out + (int64_t)rk * c + ch0;
  constexpr int V = Vec16<T>::N;
#pragma unroll
  for (int h0 = 0; h0 < 8; h0 += V) {
    Vec16<T> q;
#pragma unroll
    for (int t = 0; t < V; ++t) q.set(t, v[h0 + t]);
    store16(o + h0, q);
  }
}

// ------------------------------------------------------------------ f32 heads
template <typename T>
__global__ __launch_bounds__(256) void linear_small_kernel(const T* __restrict__ x, dp_rowmap xm, int rows, int k,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           int nw, int n, int act, const float* __restrict__ add,
                                                           float* __restrict__ out) {
  extern __shared__ float xs[];  // [4][k]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 4 + wv;
  float* xr = xs + wv * k;
  if (r < rows) {
    const T* src = x + rowmap_off(xm, r);
    for (int i = lane; i < k; i += 64) xr[i] = to_f32(src[i]);
  }
  __syncthreads();
  if (r >= rows) return;
  for (int j = lane; j < n; j += 64) {
    const int jw = j % nw;
    float s = b ? b[jw] : 0.f;
    for (int i = 0; i < k; ++i) s = fmaf(xr[i], w[(int64_t)i * nw + jw], s);
    s = apply_act(s, act);
    if (add) s += add[r * n + j];
    out[r * n + j] = s;
  }
}

// one wave per query row: lane j < 2*nkp owns (keypoint j/2, coordinate j&1)
constexpr int POSE_MAXZ = 1280;   // 2 * nkp * (reg_max + 1) floats per row staged in LDS

__global__ __launch_bounds__(256) void pose_refine_kernel(const float* __restrict__ corners,
                                                          const float* __restrict__ project, int reg_max,
                                                          const float* __restrict__ ref_init, float reg_scale,
                                                          int rows, int nkp, float* __restrict__ kps,
                                                          float* __restrict__ ref) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int nb = reg_max + 1;
  const bool act = lane < 2 * nkp;
  const int kp = lane >> 1, c = lane & 1;
  float val = 0.f;
  // the row's 2*nkp*nb distribution logits are contiguous: stage them through LDS with
  // coalesced loads (one lane per (keypoint, coordinate) walking its nb bins straight from
  // global memory was a serial chain of 2*nb scattered loads per lane)
  __shared__ float zs[4][POSE_MAXZ];
  const int nz = 2 * nkp * nb;
  const float* zrow = corners + (int64_t)r * nz;
  float* zw = zs[threadIdx.x >> 6];
  for (int i = lane; i < nz; i += 64) zw[i] = zrow[i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (act) {
    const float* z = zw + (kp * 2 + c) * nb;
    float mx = -INFINITY;
    for (int i = 0; i < nb; ++i) mx = fmaxf(mx, z[i]);
    float se = 0.f, acc = 0.f;
    for (int i = 0; i < nb; ++i) {
      const float e = expf(z[i] - mx);
      se += e;
      acc = fmaf(e, project[i], acc);
    }
    val = ref_init[((int64_t)r * nkp + kp) * 2 + c] + (acc / se) / reg_scale;
    kps[((int64_t)r * nkp + kp) * 2 + c] = val;
    ref[((int64_t)r * (nkp + 1) + 1 + kp) * 2 + c] = val;
  }
  const float sx = wave_sum(act && c == 0 ? val : 0.f);
  const float sy = wave_sum(act && c == 1 ? val : 0.f);
  if (lane == 0) {
    ref[(int64_t)r * (nkp + 1) * 2] = sx / nkp;
    ref[(int64_t)r * (nkp + 1) * 2 + 1] = sy / nkp;
  }
}

__global__ void pre_pose_kernel(const float* __restrict__ pre, const float* __restrict__ ref, int rows, int nkp,
                                float* __restrict__ out) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= rows * nkp * 2) return;
  const int c = gid & 1;
  const int rk = gid >> 1;
  const int r = rk / nkp, j = rk - r * nkp;
  float v = ref[((int64_t)r * (nkp + 1) + 1 + j) * 2 + c];
  v = fminf(fmaxf(v, 0.f), 1.f);
  const float x1 = fmaxf(v, 1e-3f), x2 = fmaxf(1.f - v, 1e-3f);
  const float z = pre[gid] + logf(x1 / x2);
  out[gid] = 1.f / (1.f + expf(-z));
}

// one wave per (b, q, kp); lane owns E = c/64 consecutive channels (static E: the
// per-lane arrays stay in registers)
template <typename T, int E>
__global__ __launch_bounds__(256) void lqe_kernel(const T* __restrict__ feat, int64_t fbs, int h, int w, int c,
                                                  const float* __restrict__ kps, int nq, int nkp, int total,
                                                  float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + (threadIdx.x >> 6);  // (b, q, kp)
  if (g >= total) return;
  const int b = (unsigned)g / (unsigned)(nq * nkp);
  const float x = kps[2 * (int64_t)g] * w - 0.5f, y = kps[2 * (int64_t)g + 1] * h - 0.5f;
  const float fx = floorf(x), fy = floorf(y);
  const int x0 = (int)fx, y0 = (int)fy;
  const float ax = x - fx, ay = y - fy;
  const float wt[4] = {(1.f - ax) * (1.f - ay), ax * (1.f - ay), (1.f - ax) * ay, ax * ay};
  float v[E];
#pragma unroll
  for (int t = 0; t < E; ++t) v[t] = 0.f;
  const T* fb = feat + (int64_t)b * fbs + lane * E;
#pragma unroll
  for (int cn = 0; cn < 4; ++cn) {
    const int xi = x0 + (cn & 1), yi = y0 + (cn >> 1);
    if (xi < 0 || xi >= w || yi < 0 || yi >= h) continue;
    const T* p = fb + ((int64_t)yi * w + xi) * c;
    T q[E];
    if constexpr (E * sizeof(T) == 8) *reinterpret_cast<uint2*>(q) = *reinterpret_cast<const uint2*>(p);
    else if constexpr (E * sizeof(T) == 16) *reinterpret_cast<uint4*>(q) = *reinterpret_cast<const uint4*>(p);
    else {
#pragma unroll
      for (int t = 0; t < E; ++t) q[t] = p[t];
    }
#pragma unroll
    for (int t = 0; t < E; ++t) v[t] = fmaf(wt[cn], to_f32(q[t]), v[t]);
  }
  // top-4 over all c channels of the wave: 4 rounds of (lane max of the unused values,
  // wave max, the lowest winning lane retires its element)
  float top[4];
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
    if (lane == winner) used |= 1u << li;
    top[s] = wm;
  }
  if (lane == 0) {
    float* o = out + (int64_t)g * 5;
    o[0] = top[0]; o[1] = top[1]; o[2] = top[2]; o[3] = top[3];
    o[4] = (top[0] + top[1] + top[2] + top[3]) / 4.f;
  }
}

__global__ void postprocess_kernel(const float* __restrict__ logits, const float* __restrict__ kps,
                                   const float* __restrict__ tsize, int nq, int ncls, int nkp, int nsel,
                                   float* __restrict__ scores, int64_t* __restrict__ labels,
                                   float* __restrict__ okps) {
  extern __shared__ float prob[];
  const int b = blockIdx.x, n = nq * ncls;
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    prob[i] = 1.f / (1.f + expf(-logits[(int64_t)b * n + i]));
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float p = prob[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += (prob[j] > p) || (prob[j] == p && j < i);
    if (rank < nsel) {
      const int q = i / ncls;
      scores[(int64_t)b * nsel + rank] = p;
      labels[(int64_t)b * nsel + rank] = i % ncls;
      for (int j = 0; j < nkp; ++j) {
        okps[(((int64_t)b * nsel + rank) * nkp + j) * 2] = kps[(((int64_t)b * nq + q) * nkp + j) * 2] * tsize[2 * b];
        okps[(((int64_t)b * nsel + rank) * nkp + j) * 2 + 1] =
            kps[(((int64_t)b * nq + q) * nkp + j) * 2 + 1] * tsize[2 * b + 1];
      }
    }
  }
}

inline unsigned nblk(int64_t n, int t = 256) { return (unsigned)((n + t - 1) / t); }

}  // namespace

extern "C" int dp_topk(const float* x, int32_t rows, int32_t n, int32_t ld, int32_t k, float* out_val,
                       int64_t* out_idx, void* stream) {
  DP_REQUIRE(x && out_val && out_idx, "dp_topk: null pointer");
  DP_REQUIRE(k >= 1 && k <= 256 && k <= n && n <= TOPK_MAXN, "dp_topk: k=%d n=%d (k<=256, n<=%d)", k, n, TOPK_MAXN);
  hipLaunchKernelGGL(topk_kernel, dim3(rows), dim3(TOPK_THREADS), (size_t)n * 4, as_stream(stream), x, n, ld, k,
                     out_val, out_idx);
  return dp_check_launch("dp_topk");
}

extern "C" int dp_class_max(const void* x, int32_t rows, int32_t c, const float* w, const float* b, int32_t nclass,
                            float* out, int32_t dtype, void* stream) {
  DP_REQUIRE(x && w && b && out && nclass > 0, "dp_class_max: bad args");
  const int vec = dtype == DP_BF16 ? 8 : 4;
  DP_REQUIRE(c % vec == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0,
             "dp_class_max: rows must be 16-byte aligned (c=%d)", c);
  const int nch = c / vec;
  const int g = nch <= 16 ? 16 : (nch <= 32 ? 32 : 64);
  const int rpb = 4 * (64 / g);   // rows per 256-thread block
  const dim3 grid((unsigned)((rows + rpb - 1) / rpb));
#define DP_CM(T_, G_) hipLaunchKernelGGL((class_max_kernel<T_, G_>), grid, dim3(256), 0, as_stream(stream), (const T_*)x, rows, c, w, b, nclass, out)
  if (dtype == DP_BF16) {
    if (g == 16) DP_CM(bf16_t, 16); else if (g == 32) DP_CM(bf16_t, 32); else DP_CM(bf16_t, 64);
  } else {
    if (g == 16) DP_CM(float, 16); else if (g == 32) DP_CM(float, 32); else DP_CM(float, 64);
  }
#undef DP_CM
  return dp_check_launch("dp_class_max");
}

extern "C" int dp_gather_rows(const void* src, int64_t src_bstride, const int64_t* idx, int32_t batch, int32_t k,
                              int32_t c, void* dst, int32_t dtype, void* stream) {
  const int64_t total = (int64_t)batch * k * c;
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(gather_rows_kernel<bf16_t>, dim3(nblk(total)), dim3(256), 0, as_stream(stream),
                       (const bf16_t*)src, src_bstride, idx, batch, k, c, (bf16_t*)dst);
  else
    hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(nblk(total)), dim3(256), 0, as_stream(stream),
                       (const float*)src, src_bstride, idx, batch, k, c, (float*)dst);
  return dp_check_launch("dp_gather_rows");
}

extern "C" int dp_refpoint_init(const float* delta, const float* anchors, const int64_t* idx, int32_t batch,
                                int32_t k, int32_t nkp, float* ref, void* stream) {
  const int rows = batch * k;
  hipLaunchKernelGGL(refpoint_init_kernel, dim3(nblk(rows, 64)), dim3(64), 0, as_stream(stream), delta, anchors, idx,
                     rows, nkp, ref);
  return dp_check_launch("dp_refpoint_init");
}

extern "C" int dp_broadcast(const void* src, int64_t bytes, void* dst, int32_t count, void* stream) {
  const int64_t total = bytes * count;
  const int vec = (bytes % 16 == 0) && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  const int64_t nthr = vec ? total / 16 : total;
  hipLaunchKernelGGL(broadcast_kernel, dim3(nblk(nthr)), dim3(256), 0, as_stream(stream), (const uint8_t*)src, bytes,
                     (uint8_t*)dst, total, vec);
  return dp_check_launch("dp_broadcast");
}

extern "C" int dp_sine_embed(const float* ref, int32_t rows, int32_t nkp, int32_t c, const float* dim_t, void* out,
                             int32_t dtype, void* stream) {
  DP_REQUIRE(c % 16 == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0,
             "dp_sine_embed: c=%d must be a multiple of 16, out 16-byte aligned", c);
  const int64_t total = (int64_t)rows * nkp * (c / 8);
  DP_REQUIRE(total < (1ll << 31), "dp_sine_embed: too many rows");
  if (dtype == DP_BF16)
    hipLaunchKernelGGL(sine_embed_kernel<bf16_t>, dim3(nblk(total)), dim3(256), 0, as_stream(stream), ref, rows, nkp,
                       c, dim_t, (bf16_t*)out);
  else
    hipLaunchKernelGGL(sine_embed_kernel<float>, dim3(nblk(total)), dim3(256), 0, as_stream(stream), ref, rows, nkp,
                       c, dim_t, (float*)out);
  return dp_check_launch("dp_sine_embed");
}

extern "C" int dp_linear_small(const void* x, dp_rowmap xm, int32_t x_dtype, int32_t rows, int32_t k, const float* w,
                               const float* b, int32_t nw, int32_t n, int32_t act, const float* add, float* out,
                               void* stream) {
  DP_REQUIRE(x && w && out && nw > 0 && n > 0 && k > 0 && xm.group > 0, "dp_linear_small: bad args");
  DP_REQUIRE(k <= 4096, "dp_linear_small: k=%d too large", k);
  const size_t lds = (size_t)4 * k * sizeof(float);
  if (x_dtype == DP_BF16)
    hipLaunchKernelGGL(linear_small_kernel<bf16_t>, dim3(nblk(rows, 4)), dim3(256), lds, as_stream(stream),
                       (const bf16_t*)x, xm, rows, k, w, b, nw, n, act, add, out);
  else
    hipLaunchKernelGGL(linear_small_kernel<float>, dim3(nblk(rows, 4)), dim3(256), lds, as_stream(stream),
                       (const float*)x, xm, rows, k, w, b, nw, n, act, add, out);
  return dp_check_launch("dp_linear_small");
}

extern "C" int dp_pose_refine(const float* corners, const float* project, int32_t reg_max, const float* ref_init,
                              float reg_scale, int32_t rows, int32_t nkp, float* kps, float* ref, void* stream) {
  DP_REQUIRE(2 * nkp <= 64 && 2 * nkp * (reg_max + 1) <= POSE_MAXZ, "dp_pose_refine: nkp=%d reg_max=%d too large",
             nkp, reg_max);
  hipLaunchKernelGGL(pose_refine_kernel, dim3(nblk(rows, 4)), dim3(256), 0, as_stream(stream), corners, project,
                     reg_max, ref_init, reg_scale, rows, nkp, kps, ref);
  return dp_check_launch("dp_pose_refine");
}

extern "C" int dp_pre_pose(const float* pre, const float* ref, int32_t rows, int32_t nkp, float* out, void* stream) {
  hipLaunchKernelGGL(pre_pose_kernel, dim3(nblk((int64_t)rows * nkp * 2)), dim3(256), 0, as_stream(stream), pre, ref,
                     rows, nkp, out);
  return dp_check_launch("dp_pre_pose");
}

extern "C" int dp_lqe_stats(const void* feat, int64_t feat_bstride, int32_t h, int32_t w, int32_t c, const float* kps,
                            int32_t batch, int32_t nq, int32_t nkp, float* out, int32_t dtype, void* stream) {
  DP_REQUIRE(c % 64 == 0 && c <= 512, "dp_lqe_stats: c=%d must be a multiple of 64, <= 512", c);
  const int total = batch * nq * nkp;
  DP_REQUIRE((reinterpret_cast<uintptr_t>(feat) & 15) == 0, "dp_lqe_stats: feat must be 16-byte aligned");
#define DP_LQE(T_, E_)                                                                                          \
  case E_:                                                                                                      \
    hipLaunchKernelGGL((lqe_kernel<T_, E_>), dim3(nblk(total, 4)), dim3(256), 0, as_stream(stream),             \
                       (const T_*)feat, feat_bstride, h, w, c, kps, nq, nkp, total, out);                       \
    break;
  if (dtype == DP_BF16) {
    switch (c / 64) { DP_LQE(bf16_t, 1) DP_LQE(bf16_t, 2) DP_LQE(bf16_t, 3) DP_LQE(bf16_t, 4) DP_LQE(bf16_t, 5)
                      DP_LQE(bf16_t, 6) DP_LQE(bf16_t, 7) DP_LQE(bf16_t, 8) }
  } else {
    switch (c / 64) { DP_LQE(float, 1) DP_LQE(float, 2) DP_LQE(float, 3) DP_LQE(float, 4) DP_LQE(float, 5)
                      DP_LQE(float, 6) DP_LQE(float, 7) DP_LQE(float, 8) }
  }
#undef DP_LQE
  return dp_check_launch("dp_lqe_stats");
}

extern "C" int dp_postprocess(const float* logits, const float* kps, const float* target_sizes, int32_t batch,
                              int32_t nq, int32_t nclass, int32_t nkp, int32_t num_select, float* scores,
                              int64_t* labels, float* out_kps, void* stream) {
  DP_REQUIRE(num_select <= nq * nclass, "dp_postprocess: num_select=%d > %d", num_select, nq * nclass);
  hipLaunchKernelGGL(postprocess_kernel, dim3(batch), dim3(256), (size_t)nq * nclass * 4, as_stream(stream), logits,
                     kps, target_sizes, nq, nclass, nkp, num_select, scores, labels, out_kps);
  return dp_check_launch("dp_postprocess");
}
