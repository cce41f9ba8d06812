// Persistent bf16 implicit-GEMM convolution (gfx950): the path of dp_conv2d for bf16
// activations (1x1 convs, linears, and the KxK convs conv_halo.hip does not cover).
//
// Why persistent: most DETRPose convs are short in K (1x1 with cin 64..512, 2x2 stem
// convs) and near the HBM ridge, so a one-tile block spends most of its life in the
// first DMA round trip and the epilogue. Here each block walks a strided list of tiles
// and its LDS-DMA ring runs straight across tile boundaries: while tile T's epilogue
// writes, tile T+1's first K-steps are already landing in LDS.
//
// Operands: the MFMA is fed weights as the A operand and gathered activations as the B
// operand (C^T = W A^T), so each lane ends with 4 consecutive output channels of one
// pixel per 16x16 tile; the weight rows are permuted on their way into LDS (the DMA
// lane->row mapping is free) so that a lane's TN tiles hold 4*TN CONTIGUOUS channels.
// The epilogue then needs no LDS: bias/act/LAB/residual in registers, 16-byte stores
// straight from the accumulators (and the nearest-x2 copy for the FPN concat).
//
// LDS-DMA: one `buffer_load_dwordx4 ... lds` moves 8 rows x
// 128 B; chunks are XOR-swizzled by row so fragment reads are conflict-free; OOB offsets
// return 0 (conv padding, K/M/N tails). Blocks are remapped so each XCD owns a
// contiguous slice of every round of tiles (the N-tiles sharing an A tile hit one L2).
#include "common.h"
#include <stdlib.h>
#include <type_traits>

#include "conv_lds.h"

#ifndef DP_ABL_NOSTORE
#define DP_ABL_NOSTORE 0   // ablation builds only (scripts/conv_bench.py): drop the epilogue stores
#endif
#ifndef DP_ABL_NODMA
#define DP_ABL_NODMA 0     // ... drop the LDS-DMA loads
#endif
#ifndef DP_STREAM_PRIO
#define DP_STREAM_PRIO 1   // s_setprio(1) around each K-step's fragment reads + MFMAs (fpn1.cv1 +3.5%, s2.sq +2.4%, others flat)
#endif
#ifndef DP_STREAM_PIPE
#define DP_STREAM_PIPE 1   // K loop pipelined across the per-step barrier (0: the unpipelined loop, A/B only)
#endif
#ifndef DP_ABL_NOMFMA
#define DP_ABL_NOMFMA 0    // ... drop the MFMAs (fragment reads kept live)
#endif

namespace {

using namespace dpconv;

// Epilogue modes (compile time, so the store path has no runtime branches or waits):
// plain, + residual (added after act/LAB), + nearest-x2 copy into the FPN concat buffer.
enum { EPI_PLAIN = 0, EPI_RES = 1, EPI_UP = 2 };

// VMEM instructions one wave issues in the epilogue of a whole tile (every pixel row
// in range, every lane's chunks whole): the count the next K-step's wait may leave in
// flight, since loads/stores/LDS-DMA retire in issue order (MI355X_MICROARCH.md: vmcnt).
template <int EPI, int TM, int CPL>
constexpr int epi_vmem() {
  const int n = TM * CPL * (EPI == EPI_PLAIN ? 1 : (EPI == EPI_RES ? 2 : 5));
  return n > 63 ? 63 : n;
}

// Cout edge / unaligned rows (f32 heads with 2/34/66 columns, 48-channel convs in 64-wide
// tiles): scalar stores. Inlined: an out-of-line call would put the descriptor in scratch
// and make the caller save its accumulators.
template <int EPI, typename TO, int NPL>
__device__ __forceinline__ void epi_edge(const dp_conv_desc& d, const float* v, int b, int rem, int nbw,
                                                   int g) {
  constexpr int VO = 16 / (int)sizeof(TO);
  const int oy = rem / d.out_w, ox = rem - oy * d.out_w;
  TO* __restrict__ out = reinterpret_cast<TO*>(d.out);
  const TO* __restrict__ res = reinterpret_cast<const TO*>(d.res);
  TO* __restrict__ up = reinterpret_cast<TO*>(d.up);
  for (int e = 0; e < NPL; ++e) {
    const int cc = nbw + lane_chan<VO>(g, e);
    if (cc >= d.cout) continue;
    float x = v[e];
    if (EPI == EPI_RES) x += to_f32(res[(int64_t)b * d.res_bstride + (int64_t)rem * d.res_pstride + cc]);
    const TO y = from_f32<TO>(x);
    out[(int64_t)b * d.out_bstride + (int64_t)rem * d.out_pstride + cc] = y;
    if (EPI == EPI_UP)
      for (int dy = 0; dy < 2; ++dy)
        for (int dx = 0; dx < 2; ++dx)
          up[(int64_t)b * d.up_bstride + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride + cc] =
              y;
  }
}

// Epilogue of one tile from registers. Lane (g = lane>>4, q = lane&15) owns pixel rows
// m = mw + 16 i + q and the wave's channels nbw + lane_chan(g, 0 .. NPL-1); the bias of
// the tile's BN channels sits in LDS (bias_w = the wave's first channel there). Pixel
// (image, offset) pairs advance incrementally: one division per tile, not per pixel.
// Returns true when the tile was whole (every wave issued epi_vmem VMEM instructions).
template <int ACT, typename TO, int TM, int TN, int EPI>
__device__ __forceinline__ bool stream_epilogue(const dp_conv_desc& d, const f32x4 (&acc)[TM][TN],
                                                const float* bias_w, int M, int mw, int nbw, int vec_ok) {
  constexpr int NPL = 4 * TN;
  constexpr int VO = 16 / (int)sizeof(TO);
  constexpr int CPL = NPL / VO;
  static_assert(NPL % VO == 0, "lane channel group must be whole 16-byte chunks");
  const int lane = threadIdx.x & 63, q = lane & 15, g = lane >> 4;
  if (nbw >= d.cout) return false;
  const bool wave_full = vec_ok && nbw + lane_chan<VO>(3, NPL - 1) < d.cout;
  const bool full = wave_full || lane_full<TO, NPL>(d, nbw, g, vec_ok);
  float bias[NPL];
#pragma unroll
  for (int e = 0; e < NPL; e += 4) {
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias_w + lane_chan<VO>(g, e));
    bias[e] = b4[0], bias[e + 1] = b4[1], bias[e + 2] = b4[2], bias[e + 3] = b4[3];
  }
  const int hwo = d.out_h * d.out_w;
  int m = mw + q;
  int b = m / hwo, rem = m - b * hwo;
  TO* __restrict__ out = reinterpret_cast<TO*>(d.out);
  const TO* __restrict__ res = reinterpret_cast<const TO*>(d.res);
  TO* __restrict__ up = reinterpret_cast<TO*>(d.up);
  const int cb = nbw + g * VO;   // the lane's chunk 0; chunk c at cb + 4 VO c
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if (m < M) {
      float v[NPL];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = act_t<ACT>(acc[i][j][r] + bias[4 * j + r]);
          if (d.has_lab) x = d.lab_scale * x + d.lab_bias;
          v[4 * j + r] = x;
        }
#if DP_ABL_NOSTORE
#pragma unroll
      for (int e = 0; e < NPL; ++e) asm volatile("" ::"v"(v[e]), "v"(b), "v"(rem));
#else
      if (full) {
        TO* op = out + (int64_t)b * d.out_bstride + (int64_t)rem * d.out_pstride + cb;
        Vec16<TO> ch[CPL];
        if constexpr (EPI == EPI_RES) {
          const TO* rp = res + (int64_t)b * d.res_bstride + (int64_t)rem * d.res_pstride + cb;
#pragma unroll
          for (int c = 0; c < CPL; ++c) ch[c] = load16(rp + c * 4 * VO);
#pragma unroll
          for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int t = 0; t < VO; ++t) ch[c].set(t, v[c * VO + t] + ch[c].get(t));
        } else {
#pragma unroll
          for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int t = 0; t < VO; ++t) ch[c].set(t, v[c * VO + t]);
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) store16(op + c * 4 * VO, ch[c]);
        if constexpr (EPI == EPI_UP) {
          const int oy = rem / d.out_w, ox = rem - oy * d.out_w;
          TO* ub = up + (int64_t)b * d.up_bstride + cb;
#pragma unroll
          for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
              TO* upp = ub + ((int64_t)(2 * oy + dy) * (2 * d.out_w) + 2 * ox + dx) * d.up_pstride;
#pragma unroll
              for (int c = 0; c < CPL; ++c) store16(upp + c * 4 * VO, ch[c]);
            }
        }
      } else {
        epi_edge<EPI, TO, NPL>(d, v, b, rem, nbw, g);
      }
#endif
    }
    m += 16;
    rem += 16;
    while (rem >= hwo) rem -= hwo, ++b;
  }
  return wave_full && mw + 16 * TM - 1 < M;
}

// target waves per SIMD = (blocks per CU the LDS allows) x (waves per block) / 4; ask the
// register allocator for the matching budget
template <int BM, int BN, int SA, int NW>
constexpr int stream_waves() {
  const int blocks = (160 * 1024) / ((SA * BM + 2 * BN) * 128);
  const int w = blocks * NW / 4;
  return w >= 3 ? 3 : (w >= 2 ? 2 : 1);
}

// NW = waves per block (4, or 8 for the 256-row tiles of the large GEMMs).
// SA = depth of the activation (A) ring; the weight (B) ring is 2 deep. Weights are a few
// hundred KB and stay in L2, activations stream from HBM: the extra A stages are the bytes
// in flight that hide HBM latency (Little's law), where a deeper B ring would only burn LDS.
template <int BM, int BN, int WGM, int NW, int SA, bool K1X1, int ACT, typename TO, int EPI>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(stream_waves<BM, BN, SA, NW>())))
void conv_stream_kernel(dp_conv_desc d, int M, int nt_n, int ntiles, int vec_ok) {
  constexpr int WGN = NW / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int NPL = 4 * TN;
  constexpr int GA = BM / (8 * NW), GB = BN / (8 * NW);   // DMA instructions (8 rows) per wave per K-step
  constexpr int SB = 2;
  constexpr int BBYTES = BN * 128, ABYTES = BM * 128;     // one K-step of B / A
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0 && WGM * WGN == NW && TM >= 1 && TN >= 1 && SA >= 2 &&
                    SA <= 4, "tile");
  // LDS: [B ring: SB x BN rows][A ring: SA x BM rows], rows of 128 B (one 64-wide K-step),
  // then 2 x 1 KB bias slots (tile parity): the tile's BN f32 biases, DMA'd by wave 0 in
  // front of the tile's first weight K-step, so the epilogue reads them from LDS and the
  // compiler never has a VMEM load of its own to wait for behind the in-flight DMAs.
  // (pipelined loop: 4 bias slots, since with one K-step per tile the bias of tile t+2 is issued
  // before tile t's epilogue)
  // Only the 192-row tile pipelines (deep-K GEMMs on 8 waves: s2 squeeze 273 -> 256 us, the
  // decoder GEMMs 1-3 %); elsewhere it measured neutral to -2 % (profiles/r6a_conv_ab.txt), and
  // the 256 x 256 tile spills with it (its 256 registers hold the accumulators and one K-step)
  constexpr bool PIPE = DP_STREAM_PIPE && BM == 192;
  constexpr int NBS = PIPE ? 4 : 2;
  __shared__ __attribute__((aligned(1024))) char smem[SB * BBYTES + SA * ABYTES + NBS * 1024];
  char* const sa_base = smem + SB * BBYTES;
  char* const bias_base = sa_base + SA * ABYTES;
  static_assert(BN * 4 <= 1024, "bias slot");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int G = gridDim.x;                                  // multiple of 8
  const int L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (L >= ntiles) return;

  const int hwo = d.out_h * d.out_w;
  const int r8 = lane >> 3;
  const int chunk = (lane & 7) ^ r8;
  const int ntap = d.kh * d.kw;
  const int nk = d.kpad / 64;
  const int total = ((ntiles - 1 - L) / G + 1) * nk;       // K-steps this block runs
  const i32x4 rb_src = make_rsrc(d.weight);

  // weight row landing in LDS row R: permuted so lane group g of wave column wn ends with
  // channels wn*WN + lane_chan(g, 0 .. NPL-1) (see conv_lds.h)
  constexpr int VO = 16 / (int)sizeof(TO);
  auto b_chan = [&](int t) {
    const int R = (wave + NW * t) * 8 + r8;
    const int wq = R / WN, p16 = R % WN, j = p16 / 16, p = p16 % 16;
    return wq * WN + lane_chan<VO>(p >> 2, 4 * j + (p & 3));
  };

  // ---- A issue cursor (activations) and B issue cursor (weights) run SA-1 and 1 K-steps
  // ahead of the consumer, each across tile boundaries
  int a_tile = L, a_kt = 0, a_n = 0;
  int b_tile = L, b_kt = 0, b_n = 0, b_t = 0;   // b_t: tiles whose weights were issued
  i32x4 ra_src;
  int a_off[GA], a_yx[GA], b_off[GB];   // a_yx: (iy0 << 16) | (ix0 & 0xffff)
  auto setup_a = [&](int tile) {
    const int tm = tile / nt_n;
    const int m0 = tm * BM;
    const int b_first = m0 / hwo;
    ra_src = make_rsrc(reinterpret_cast<const bf16_t*>(d.in) + (int64_t)b_first * d.in_bstride);
#pragma unroll
    for (int t = 0; t < GA; ++t) {
      const int m = m0 + (wave + NW * t) * 8 + r8;
      const bool ok = m < M;
      const int mm = ok ? m : m0;
      const int b = mm / hwo, rem = mm - b * hwo;
      const int oy = rem / d.out_w, ox = rem - oy * d.out_w;
      const int iy0 = oy * d.stride - d.pad_t, ix0 = ox * d.stride - d.pad_l;
      a_yx[t] = (iy0 << 16) | (ix0 & 0xffff);
      int off = (b - b_first) * (int)d.in_bstride;
      if (K1X1) off += (iy0 * d.in_w + ix0) * d.in_pstride;
      a_off[t] = ok ? off : OOB;
    }
  };
  auto setup_b = [&](int tile) {
    const int tm = tile / nt_n, tn = tile - tm * nt_n;
    const int n0 = tn * BN;
#pragma unroll
    for (int t = 0; t < GB; ++t) {
      const int n = n0 + b_chan(t);
      b_off[t] = n < d.cout ? n * d.kpad + chunk * 8 : OOB;
    }
  };
  auto issue_a = [&]() {
    char* sb = sa_base + (a_n % SA) * ABYTES;
    const int kk = a_kt * 64 + chunk * 8;
    if (K1X1) {
      const bool kv = kk < d.cin;
      int kofs = kk;
      if (d.in_seg_ch) {   // segmented input: channel kk lives in segment kk / in_seg_ch
        const int sg = (int)((unsigned)kk / (unsigned)d.in_seg_ch);
        kofs = sg * (int)d.in_seg_stride + (kk - sg * d.in_seg_ch);
      }
#pragma unroll
      for (int t = 0; t < GA; ++t) {
        const int o = (a_off[t] != OOB && kv) ? (a_off[t] + kofs) * 2 : OOB;
        if (!DP_ABL_NODMA) dma16(ra_src, sb + (wave + NW * t) * 1024, o);
      }
    } else {
      const int tap = kk / d.cin, ci = kk - tap * d.cin;
      const int ky = tap / d.kw, kx = tap - ky * d.kw;
      const bool kv = tap < ntap;
#pragma unroll
      for (int t = 0; t < GA; ++t) {
        const int iy = (a_yx[t] >> 16) + ky, ix = (int)(short)(a_yx[t] & 0xffff) + kx;
        const bool ok = kv && a_off[t] != OOB && (unsigned)iy < (unsigned)d.in_h && (unsigned)ix < (unsigned)d.in_w;
        const int o = ok ? (a_off[t] + (iy * d.in_w + ix) * d.in_pstride + ci) * 2 : OOB;
        if (!DP_ABL_NODMA) dma16(ra_src, sb + (wave + NW * t) * 1024, o);
      }
    }
    ++a_n;
    if (++a_kt == nk) {
      a_kt = 0;
      a_tile += G;
      if (a_tile < ntiles) setup_a(a_tile);
    }
  };
  auto issue_b = [&]() {
    char* sb = smem + (b_n % SB) * BBYTES;
    if (b_kt == 0 && wave == 0) {
      // the tile's biases (older than its first weight K-step: covered by the same wait)
      const int n0 = (b_tile - (b_tile / nt_n) * nt_n) * BN;
      const int o = (d.bias && n0 + 4 * lane < d.cout && 4 * lane < BN) ? (n0 + 4 * lane) * 4 : OOB;
      if (!DP_ABL_NODMA) dma16(make_rsrc(d.bias), bias_base + (b_t % NBS) * 1024, o);
    }
#pragma unroll
    for (int t = 0; t < GB; ++t) {
      const int o = b_off[t] != OOB ? (b_off[t] + b_kt * 64) * 2 : OOB;
      if (!DP_ABL_NODMA) dma16(rb_src, sb + (wave + NW * t) * 1024, o);
    }
    ++b_n;
    if (++b_kt == nk) {
      b_kt = 0;
      ++b_t;
      b_tile += G;
      if (b_tile < ntiles) setup_b(b_tile);
    }
  };

  // prologue: B(0), then A(0 .. SA-2). Steady state, per consumed K-step c: B(c+1), A(c+SA-1).
  setup_a(a_tile);
  setup_b(b_tile);
  issue_b();
#pragma unroll
  for (int p = 0; p < SA - 1; ++p)
    if (a_n < total) issue_a();

  const int lr = lane & 15, lg = lane >> 4;
  const int wrow = wn * WN + lr;   // weight fragment rows (MFMA A operand)
  const int prow = wm * WM + lr;   // pixel fragment rows (MFMA B operand)
  int c = 0;                       // K-steps consumed
  // after an epilogue: 0 none, 1 whole tile (its epi_vmem stores/loads are the youngest VMEM
  // ops and may stay in flight), 2 partial tile (unknown count: drain)
  int dirty = 0;
  constexpr int EPIV = epi_vmem<EPI, TM, (4 * TN) / (16 / (int)sizeof(TO))>();
  f32x4 acc[TM][TN];
  // one K-step: wait for A(c) and B(c), publish them, refill both rings, 2 x TMxTN MFMAs.
  // Waits: the loads complete in order, so it suffices to count the A groups issued after
  // both A(c) and B(c): at c = 0 the prologue's A(1 .. SA-2), later the single A(c+SA-2)
  // issued right after B(c) (for SA = 2 A(c) itself is the youngest: wait for all).
  // The first K-step of a tile starts from a zero C operand instead of re-zeroing acc (a
  // zeroing loop makes the register allocator pin a second set of zero AGPRs).
  auto step = [&](auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    const int younger = SA == 2 ? 0 : (c == 0 ? min(SA - 2, a_n - 1) : (a_n > c + SA - 2 ? 1 : 0));
    if (dirty == 2) wait_vmcnt<0>();
    else if (dirty == 1) {
      // the epilogue's stores are younger than everything this step needs
      if (younger <= 0) wait_vmcnt<EPIV>();
      else if (younger == 1) wait_vmcnt<(EPIV + GA > 63 ? 63 : EPIV + GA)>();
      else wait_vmcnt<(EPIV + 2 * GA > 63 ? 63 : EPIV + 2 * GA)>();
    } else if (younger <= 0) wait_vmcnt<0>();
    else if (younger == 1) wait_vmcnt<GA>();
    else wait_vmcnt<2 * GA>();
    dirty = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (b_n < total) issue_b();
    if (a_n < total) issue_a();
    const char* sbw = smem + (c % SB) * BBYTES;
    const char* sbp = sa_base + (c % SA) * ABYTES;
    if (DP_STREAM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int cc = 4 * ks + lg;
      bf16x8 wf[TN], pf[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wrow + 16 * j;
        wf[j] = *reinterpret_cast<const bf16x8*>(sbw + r * 128 + ((cc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = prow + 16 * i;
        pf[i] = *reinterpret_cast<const bf16x8*>(sbp + r * 128 + ((cc ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#if DP_ABL_NOMFMA
        {
          asm volatile("" ::"v"(wf[j]), "v"(pf[i]));
          if (FIRST && ks == 0) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              wf[j], pf[i], (FIRST && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
#endif
    }
    if (DP_STREAM_PRIO) __builtin_amdgcn_s_setprio(0);
    ++c;
  };
  int t_n = 0;
  if constexpr (!PIPE) {
    for (int ctile = L; ctile < ntiles; ctile += G, ++t_n) {
      step(std::true_type{});
      for (int kt = 1; kt < nk; ++kt) step(std::false_type{});
      const int tm = ctile / nt_n, tn = ctile - tm * nt_n;
      const int mw = tm * BM + wm * WM;
      const float* bias_w = reinterpret_cast<const float*>(bias_base + (t_n % NBS) * 1024) + wn * WN;
      dirty = stream_epilogue<ACT, TO, TM, TN, EPI>(d, acc, bias_w, M, mw, tn * BN + wn * WN, vec_ok) ? 1 : 2;
    }
    wait_vmcnt<0>();
    return;
  }
  // Pipelined K loop: the per-step barrier sits between the two MFMA halves of a K-step. The
  // barrier in step c publishes A(c+1) / B(c+1) (the waits of the unpipelined step c+1, same
  // counts) and frees step c's ring slots; half 0 of step c+1's fragments is then read under
  // the half-1 MFMAs of step c, half 1 of a step under its own half-0 MFMAs. No MFMA waits for
  // an LDS read issued after a barrier (the unpipelined step read both halves there, every
  // wave at once, before its first MFMA). A tile's epilogue follows its last half-1 MFMAs, after
  // the barrier that issued the next tile's first DMAs, so those stay older than its stores.
  bf16x8 wf0[TN], pf0[TM], wf1[TN], pf1[TM];
  auto read_half = [&](int cs, int ks, bf16x8 (&wf)[TN], bf16x8 (&pf)[TM]) {
    const char* sbw = smem + (cs % SB) * BBYTES;
    const char* sbp = sa_base + (cs % SA) * ABYTES;
    const int cc = 4 * ks + lg;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int r = wrow + 16 * j;
      wf[j] = *reinterpret_cast<const bf16x8*>(sbw + r * 128 + ((cc ^ (r & 7)) << 4));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = prow + 16 * i;
      pf[i] = *reinterpret_cast<const bf16x8*>(sbp + r * 128 + ((cc ^ (r & 7)) << 4));
    }
  };
  auto mfma_half = [&](const bf16x8 (&wf)[TN], const bf16x8 (&pf)[TM], bool zero) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#if DP_ABL_NOMFMA
      {
        asm volatile("" ::"v"(wf[j]), "v"(pf[i]));
        if (zero) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#else
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], pf[i], zero ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j],
                                                            0, 0, 0);
#endif
  };
  // wait for A(cn) and B(cn) (cn = the step the next fragment reads belong to), publish them,
  // refill both rings: the unpipelined step's head with c = cn
  auto publish = [&](int cn) {
    const int younger = SA == 2 ? 0 : (cn == 0 ? min(SA - 2, a_n - 1) : (a_n > cn + SA - 2 ? 1 : 0));
    if (dirty == 2) wait_vmcnt<0>();
    else if (dirty == 1) {
      if (younger <= 0) wait_vmcnt<EPIV>();
      else if (younger == 1) wait_vmcnt<(EPIV + GA > 63 ? 63 : EPIV + GA)>();
      else wait_vmcnt<(EPIV + 2 * GA > 63 ? 63 : EPIV + 2 * GA)>();
    } else if (younger <= 0) wait_vmcnt<0>();
    else if (younger == 1) wait_vmcnt<GA>();
    else wait_vmcnt<2 * GA>();
    dirty = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (b_n < total) issue_b();
    if (a_n < total) issue_a();
  };
  publish(0);
  read_half(0, 0, wf0, pf0);
  for (int ctile = L; ctile < ntiles; ctile += G, ++t_n) {
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      if (DP_STREAM_PRIO) __builtin_amdgcn_s_setprio(1);
      read_half(c, 1, wf1, pf1);
      mfma_half(wf0, pf0, kt == 0);
      if (DP_STREAM_PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      // unconditional on the block's last step (its reads of step c+1's slots are harmless: every
      // DMA has landed): a branch around the reads would merge wait states before the MFMAs below
      publish(c + 1);
      if (DP_STREAM_PRIO) __builtin_amdgcn_s_setprio(1);
      read_half(c + 1, 0, wf0, pf0);
      mfma_half(wf1, pf1, false);
      if (DP_STREAM_PRIO) __builtin_amdgcn_s_setprio(0);
      ++c;
    }
    const int tm = ctile / nt_n, tn = ctile - tm * nt_n;
    const int mw = tm * BM + wm * WM;
    const float* bias_w = reinterpret_cast<const float*>(bias_base + (t_n % NBS) * 1024) + wn * WN;
    dirty = stream_epilogue<ACT, TO, TM, TN, EPI>(d, acc, bias_w, M, mw, tn * BN + wn * WN, vec_ok) ? 1 : 2;
  }
  wait_vmcnt<0>();
}

#ifndef DP_STREAM_SA
#define DP_STREAM_SA 2
#endif

template <typename K>
int occupancy(K kern, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, 0) != hipSuccess || n <= 0) n = 1;
  return n;
}

// the activation is a template parameter: a runtime switch in the epilogue costs ~20 VGPRs
// and with them the second wave per SIMD of the 128x128 kernel
// A-ring depth: DP_STREAM_SA where it keeps the blocks per CU of a 2-deep ring (the narrow
// tiles get their bytes in flight from more resident blocks instead)
#ifndef DP_NARROW_SA
#define DP_NARROW_SA 4   // A-ring depth of the narrow-cout (BN <= 64) streaming tiles: more bytes in flight
                         // beat a third resident block (s0 squeeze 285 -> 265 us); 0: the rule below
#endif

template <int BM, int BN, int NW>
constexpr int ring_a() {
  if (DP_NARROW_SA && BN <= 64) return DP_NARROW_SA;
  constexpr int want = BM == 192 ? 3 : DP_STREAM_SA;   // the 192-row tile has LDS for a 3rd A stage
  constexpr int bias = (DP_STREAM_PIPE && BM == 192) ? 4096 : 2048;   // + the bias slots
  constexpr int blocks2 = (160 * 1024) / ((2 * BM + 2 * BN) * 128 + bias);
  constexpr int blocksw = (160 * 1024) / ((want * BM + 2 * BN) * 128 + bias);
  return (blocksw >= 1 && blocksw >= blocks2) ? want : 2;
}

template <int BM, int BN, int WGM, int NW, bool K1, int ACT, typename TO, int EPI>
int launch_one(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  constexpr int SA = ring_a<BM, BN, NW>();
  DP_DESCRIBE("conv_stream_kernel<%d, %d, %d, %d, %d, %s, %d, %s, %d>", BM, BN, WGM, NW, SA, DP_TF(K1), ACT,
              sizeof(TO) == 2 ? "bf16" : "float", EPI);
  auto kern = conv_stream_kernel<BM, BN, WGM, NW, SA, K1, ACT, TO, EPI>;
  static const int occ = [&] {
    const int o = occupancy(kern, NW * 64);
    if (getenv("DETRPOSE_CONV_DEBUG")) {
      hipFuncAttributes fa{};
      (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern));
      fprintf(stderr, "conv_stream BM=%d BN=%d NW=%d SA=%d K1=%d act=%d: occupancy %d blocks/CU, regs %d, lds %zu\n", BM,
              BN, NW, SA, (int)K1, ACT, o, fa.numRegs, fa.sharedSizeBytes);
    }
    return o;
  }();
  const int M = d.batch * d.out_h * d.out_w;
  const int mt = (M + BM - 1) / BM, nt = (d.cout + BN - 1) / BN;
  const int ntiles = mt * nt;
  int grid = occ * num_cus();
  const int need = (ntiles + 7) / 8 * 8;
  if (grid > need) grid = need;
  grid = grid / 8 * 8;
  if (grid < 8) grid = 8;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), 0, s, d, M, nt, ntiles, vec_ok);
  return dp_check_launch("dp_conv2d(stream)");
}

template <int BM, int BN, int WGM, int NW, bool K1, typename TO, int EPI>
int launch_act(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  switch (d.act) {
    case DP_ACT_RELU: return launch_one<BM, BN, WGM, NW, K1, DP_ACT_RELU, TO, EPI>(d, s, vec_ok);
    case DP_ACT_SILU: return launch_one<BM, BN, WGM, NW, K1, DP_ACT_SILU, TO, EPI>(d, s, vec_ok);
    case DP_ACT_GELU: return launch_one<BM, BN, WGM, NW, K1, DP_ACT_GELU, TO, EPI>(d, s, vec_ok);
    default: return launch_one<BM, BN, WGM, NW, K1, DP_ACT_NONE, TO, EPI>(d, s, vec_ok);
  }
}

// epilogue mode (residual and upsample never come together on this path: the launcher
// refuses that descriptor; f32 outputs have no upsample, dp_conv2d checks)
template <int BM, int BN, int WGM, int NW, bool K1, typename TO>
int launch_epi(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  if (d.res) return launch_act<BM, BN, WGM, NW, K1, TO, EPI_RES>(d, s, vec_ok);
  if constexpr (sizeof(TO) == 2)
    if (d.up) return launch_act<BM, BN, WGM, NW, K1, TO, EPI_UP>(d, s, vec_ok);
  return launch_act<BM, BN, WGM, NW, K1, TO, EPI_PLAIN>(d, s, vec_ok);
}

template <int BM, int BN, int WGM, typename TO, int NW = 4>
int launch(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  const bool k1 = d.kh == 1 && d.kw == 1 && d.pad_t == 0 && d.pad_l == 0;
  return k1 ? launch_epi<BM, BN, WGM, NW, true, TO>(d, s, vec_ok) : launch_epi<BM, BN, WGM, NW, false, TO>(d, s, vec_ok);
}

#ifndef DP_BIG_TILES
#define DP_BIG_TILES 1
#endif



}  // namespace

namespace dpconv {
int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace dpconv

// bf16 entry used by dp_conv2d (conv_gemm.hip); vec_ok computed by the caller.
int dp_conv2d_stream(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  DP_REQUIRE(!(d.res && d.up), "dp_conv2d: residual together with the x2 upsample copy is not supported");
  const int M = d.batch * d.out_h * d.out_w;
  const bool f32o = d.out_f32 != 0;
  if (d.cout <= 32) return f32o ? launch<128, 32, 4, float>(d, s, vec_ok) : launch<128, 32, 4, bf16_t>(d, s, vec_ok);
  if (d.cout <= 64) return f32o ? launch<128, 64, 4, float>(d, s, vec_ok) : launch<128, 64, 4, bf16_t>(d, s, vec_ok);
  if (M <= 8192) return f32o ? launch<64, 128, 2, float>(d, s, vec_ok) : launch<64, 128, 2, bf16_t>(d, s, vec_ok);
  if (f32o) return launch<128, 128, 2, float>(d, s, vec_ok);
  static const int forced = [] {   // A/B experiments only (scripts/conv_bench.py)
    const char* e = getenv("DETRPOSE_CONV_TILE");
    return e ? atoi(e) : 0;
  }();
  if (forced && M >= 32768) {
    if (forced == 1) return launch<256, 256, 2, bf16_t, 8>(d, s, vec_ok);
    if (forced == 2) return launch<192, 256, 2, bf16_t, 8>(d, s, vec_ok);
    if (forced == 3) return launch<256, 128, 4, bf16_t, 8>(d, s, vec_ok);
    if (forced == 4) return launch<128, 128, 2, bf16_t>(d, s, vec_ok);
  }
  // large GEMMs: 256-row tiles with 8 waves halve the LDS-DMA bytes per MFMA flop
  if (DP_BIG_TILES && M >= 32768 && d.kpad >= 256) {
    if (d.cout > 128) {
      // one block per CU: a launch runs ceil(tiles / CUs) rounds, each about as long as the
      // tile has rows. Pick 256 or 192 rows by that quantization (the 192-row tile does ~4%
      // less per row, measured): e.g. the decoder's M = 64*1080 GEMMs and enc_output gain
      // 7-15%, the M = 409600 FPN/stage-1 GEMMs keep 256.
      const int nt = (d.cout + 255) / 256, cus = num_cus();
      auto rounds = [&](int bm) { return ((int64_t)((M + bm - 1) / bm) * nt + cus - 1) / cus; };
      if (rounds(192) * 192 * 104 < rounds(256) * 256 * 100) return launch<192, 256, 2, bf16_t, 8>(d, s, vec_ok);
      return launch<256, 256, 2, bf16_t, 8>(d, s, vec_ok);
    }
    if (d.kpad >= 512) return launch<256, 128, 4, bf16_t, 8>(d, s, vec_ok);
  }
  return launch<128, 128, 2, bf16_t>(d, s, vec_ok);
}
