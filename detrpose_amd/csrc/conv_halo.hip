// Spatial convolutions (3x3 s1/s2, the stem's 2x2) with an LDS halo tile (gfx950, bf16):
// dp_conv2d's path for KxK convs with cout <= 128.
//
// The implicit-GEMM kernels gather every output pixel's K = kh*kw*cin operand straight
// from L2, i.e. each input pixel is DMA'd into LDS kh*kw times per N-tile; for the 48-128
// channel 3x3 convs of HGNetv2 stages 0/1 and the encoder's VGG blocks that gather runs at
// the chip's LDS-fill rate. Here a block owns a TH x 16 tile of output pixels and all
// output channels, DMAs the ((TH-1)S+KH) x (15S+KW) input patch ONCE per tile (all input
// channels, 128-byte rows per 64 channels, XOR-swizzled), and builds the MFMA pixel
// fragments for every tap from the patch in LDS: lane (q, g) of K-step k reads patch pixel
// (row(q)*S + ky, col(q)*S + kx) of tap k / cin, channel k % cin — the same K order as the
// packed weights [cout][kpad] of the GEMM path, so the weights need no repacking.
// Weights: resident in LDS for the whole persistent block when they fit (stem, stage 0),
// otherwise streamed per K-step through a 2-deep ring. MFMA and register epilogue as in
// conv_stream.hip (weights are the A operand, pixels the B operand, permuted weight rows so
// a lane holds 4*TN contiguous output channels of one pixel).
// POOL (the stem's 2x2 conv, stem2a): the patch in LDS is exactly the zero-padded 2x2 window
// of F.pad(x,(0,1,0,1)) + MaxPool2d(2, 1), so the same kernel also writes the stem max-pool
// (hgnetv2.py:213-220) from LDS: one pass over stem1's output instead of two.
#include "conv_lds.h"
#include <stdlib.h>
#include <type_traits>

#ifndef DP_HALO_ABL
#define DP_HALO_ABL 0   // ablation builds only: 1 no K-step vmcnt wait, 2 no K-step barrier, 4 no epilogue
#endif
#ifndef DP_HALO_TAB
#define DP_HALO_TAB 1   // per-K-step tap table in LDS (0: recompute tap / channel per step, A/B only)
#endif

namespace {

using namespace dpconv;

// LDS bytes in front of the weights: the K-step -> (tap offset, channel chunk, plane) table
// (TAB_ENTRY_BYTES), then the conv's f32 biases (cout <= 128), loaded once per block
constexpr int TAB_BYTES = 2048;
constexpr int TAB_ENTRY_BYTES = 1536;

template <int TH, int KH, int KW, int S>
struct HaloGeom {
  static constexpr int TW = 16;
  static constexpr int PH = (TH - 1) * S + KH, PW = (TW - 1) * S + KW;
  static constexpr int PPX = PH * PW;
  static constexpr int PPX8 = (PPX + 7) / 8 * 8;      // patch rows rounded to whole DMA groups
  static constexpr int PLANE = PPX8 * 128;           // bytes per 64-channel plane of the patch
};

// RESW (weights resident): the patch is double-buffered and the next tile's patch is
// DMA'd while the current tile computes (only patch DMAs are in flight, so the per-tile
// vmcnt(0) retires exactly the prefetched patch). !RESW: one patch buffer, weights through a
// 2-deep ring per K-step; the second resident block on the CU overlaps the patch loads.
// 2x2 max-pool output written by the POOL instantiation (NHWC bf16, cin channels)
struct HaloPool {
  bf16_t* out;
  int64_t bstride;
  int pstride;
};

// NKC > 0 (resident weights only): the K-step count is a compile-time constant, the K loop is
// unrolled and every pixel-fragment address is a lane constant computed once per block (the
// tile geometry is the same for every tile): no tap-table reads or address arithmetic
// between the fragment reads of the MFMA loop.
// NR (streamed weights): depth of the weight ring; the K-step loop keeps NR - 1 steps of weight
// DMA in flight (a counted vmcnt wait per step instead of a full drain when NR > 2).
template <int TH, int NW, int KH, int KW, int S, int BN, bool RESW, bool DBUF, int ACT, bool POOL = false,
          int NKC = 0, int NR = 2>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 8 ? 2 : 2)))
void conv_halo_kernel(dp_conv_desc d, int tiles_x, int tiles_y, int ntiles, int vec_ok, HaloPool pool) {
  static_assert(!POOL || (KH == 2 && KW == 2 && S == 1 && !DBUF), "pool: 2x2 s1 window, single patch buffer");
  using Gm = HaloGeom<TH, KH, KW, S>;
  constexpr int TW = Gm::TW;
  constexpr int BM = TH * TW, WM = BM / NW, TM = WM / 16, TN = BN / 16, NPL = 4 * TN;
  constexpr int GB = BN / (8 * NW);                 // weight DMA instructions per wave per K-step (ring)
  // NAT (BN = 48, the 48-channel stage-0 convs): natural weight-row order, lane g holds channels
  // 16j + 4g .. +3 of tile j, 8-byte stores; otherwise the lane_chan permutation (16-byte stores)
  constexpr bool NAT = NPL % 8 != 0;
  static_assert(TM >= 1 && WM % 16 == 0 && BN % 16 == 0 && (RESW || (GB >= 1 && BN % 32 == 0)) && (RESW || !DBUF),
                "tile");
  static_assert(!NAT || (RESW && !POOL), "natural-order tiles: resident weights, plain epilogue");
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  if (L >= ntiles) return;

  const int nk = d.kpad / 64;
  const int nkc = (d.cin + 63) / 64;                 // 64-channel planes of the patch
  const int pbytes = nkc * Gm::PLANE;                // one patch buffer
  const int ktaps = KH * KW;
  int* const tab = reinterpret_cast<int*>(smem);
  float* const bias_l = reinterpret_cast<float*>(smem + TAB_ENTRY_BYTES);
  char* const wbase = smem + TAB_BYTES;
  char* const pbase0 = wbase + (RESW ? nk : NR) * BN * 128;
  const int r8 = lane >> 3;
  const i32x4 rb_src = make_rsrc(d.weight);

  // weight row -> LDS row R permuted for the register epilogue (single wave column)
  auto w_off = [&](int R) {
    const int j = R / 16, p = R % 16;
    const int n = NAT ? R : lane_chan<8>(p >> 2, 4 * j + (p & 3));
    return n < d.cout ? n * d.kpad + ((lane & 7) ^ (R & 7)) * 8 : OOB;
  };
  if (RESW) {
    // all K-steps once: (kt, 8-row group) pairs spread over the waves
    for (int t = wave; t < nk * (BN / 8); t += NW) {
      const int kt = t / (BN / 8), grp = t - kt * (BN / 8);
      const int ob = w_off(grp * 8 + r8);
      dma16(rb_src, wbase + kt * BN * 128 + grp * 1024, ob != OOB ? (ob + kt * 64) * 2 : OOB);
    }
  }
  int b_off[RESW ? 1 : GB];
  if (!RESW) {
#pragma unroll
    for (int t = 0; t < GB; ++t) b_off[t] = w_off((wave + NW * t) * 8 + r8);
  }
  auto issue_w = [&](int kt, char* dst) {
#pragma unroll
    for (int t = 0; t < GB; ++t) {
      const int o = b_off[t] != OOB ? (b_off[t] + kt * 64) * 2 : OOB;
      dma16(rb_src, dst + (wave + NW * t) * 1024, o);
    }
  };
  // the first NR - 1 weight K-steps of a tile (ring slots 0 .. NR-2)
  auto issue_w_pro = [&]() {
#pragma unroll
    for (int i = 0; i < NR - 1; ++i)
      if (i < nk) issue_w(i, wbase + i * BN * 128);
  };
  auto issue_patch = [&](int tile, char* pb) {
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int iy0 = ty * TH * S - d.pad_t, ix0 = tx * TW * S - d.pad_l;
    const i32x4 ra = make_rsrc(reinterpret_cast<const bf16_t*>(d.in) + (int64_t)b * d.in_bstride);
    constexpr int GP = Gm::PPX8 / 8;                 // DMA groups per plane
    for (int t = wave; t < GP * nkc; t += NW) {
      const int pl = t / GP, grp = t - pl * GP;
      const int p = grp * 8 + r8;
      const int py = p / Gm::PW, px = p - py * Gm::PW;
      const int iy = iy0 + py, ix = ix0 + px;
      const int ci = pl * 64 + (((lane & 7) ^ (p & 7)) << 3);
      const bool ok = p < Gm::PPX && (unsigned)iy < (unsigned)d.in_h && (unsigned)ix < (unsigned)d.in_w && ci < d.cin;
      const int o = ok ? ((iy * d.in_w + ix) * d.in_pstride + ci) * 2 : OOB;
      dma16(ra, pb + pl * Gm::PLANE + grp * 1024, o);
    }
  };

  // biases of every output channel (0 past cout), published with the table by the first barrier
  for (int e = tid; e < 128; e += NW * 64) bias_l[e] = (d.bias && e < d.cout) ? d.bias[e] : 0.f;
#if DP_HALO_TAB
  // K-step table: entry kt*8 + cc (k = 64 kt + 8 cc -> tap = k / cin, ci = k % cin) holds the
  // tap's patch-pixel offset ky*PW + kx, the 16-byte chunk (ci/8)%8 and the 64-channel plane
  // ci/64, so the MFMA loop does no division. Published by the first tile's barrier.
  for (int e = tid; e < nk * 8; e += NW * 64) {
    int tap = (e * 8) / d.cin, ci = e * 8 - tap * d.cin;
    if (tap >= ktaps) tap = 0, ci = 0;           // kpad tail: the weights are zero there
    const int ky = tap / KW, kx = tap - ky * KW;
    tab[e] = (ky * Gm::PW + kx) | (((ci >> 3) & 7) << 7) | ((ci >> 6) << 10);
  }
#endif
  // per-lane pixel fragment geometry: q = lane & 15 is the tile column, g = lane >> 4 the
  // 8-channel group of the K-step half; rows yq_i = wave*TM + i
  const int q = lane & 15, g = lane >> 4;
  const int wm = wave;
  const int cin = d.cin;
  constexpr int NKA = NKC > 0 ? NKC : 1;
  int pfa[NKA][2][TM];   // NKC: byte offset (from the patch base) of the lane's pixel fragments
  if constexpr (NKC > 0) {
    static_assert(RESW, "compile-time K loop: resident weights only");
#pragma unroll
    for (int kt = 0; kt < NKC; ++kt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int k = kt * 64 + (4 * ks + g) * 8;
        int tap = k / cin, ci = k - tap * cin;
        if (tap >= ktaps) tap = 0, ci = 0;           // kpad tail: the weights are zero there
        const int ky = tap / KW, kx = tap - ky * KW;
        const int toff = ky * Gm::PW + kx, c8 = (ci >> 3) & 7;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int pr = (wm * TM + i) * S * Gm::PW + q * S + toff;
          pfa[kt][ks][i] = (ci >> 6) * Gm::PLANE + pr * 128 + ((c8 ^ (pr & 7)) << 4);
        }
      }
  }

  // EARLY (single patch buffer, no pool epilogue): the next tile's patch (and first weight
  // K-step) is issued as soon as every wave is done reading this tile's, so its latency
  // hides behind this tile's epilogue instead of stalling the next tile's start
  constexpr bool EARLY = !DBUF && !POOL;
  if (DBUF || EARLY) issue_patch(L, pbase0);
  if (EARLY && !RESW) issue_w_pro();
  f32x4 acc[TM][TN];
  // stores one wave issues in the epilogue of a whole tile (plain epilogue, vector path): the
  // next tile's wait may leave them in flight, since VMEM ops retire in issue order and the
  // patch / weight DMAs it waits for were issued before them
  constexpr int NSTORE = NAT ? TM * TN : TM * (NPL / 8);
  // the counted wait below assumes every wave issued exactly NSTORE stores in the previous
  // tile's epilogue: only tiles whose every output channel exists (cout == BN) qualify, NAT
  // tiles included (their epilogue skips the stores of channels >= cout)
  const bool plain_full = !d.res && !d.up && d.cout == BN && (NAT || vec_ok);
  bool prev_full = false;
  int u = 0;
  for (int tile = L; tile < ntiles; tile += G, ++u) {
    const int tx = tile % tiles_x, rest = tile / tiles_x;
    const int ty = rest % tiles_y, b = rest / tiles_y;
    const int oy0 = ty * TH, ox0 = tx * TW;
    const bool tile_full = plain_full && oy0 + TH <= d.out_h && ox0 + TW <= d.out_w;
    const char* pbase;
    if (DBUF) {
      // this tile's patch (prefetched during the previous tile) has landed; every wave is
      // past the previous tile, so the other buffer is free for the next tile's patch
      if (prev_full) wait_vmcnt<NSTORE>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (tile + G < ntiles) issue_patch(tile + G, pbase0 + ((u + 1) & 1) * pbytes);
      pbase = pbase0 + (u & 1) * pbytes;
    } else if (EARLY) {
      if (prev_full) wait_vmcnt<NSTORE>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      pbase = pbase0;
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      issue_patch(tile, pbase0);
      if (!RESW) issue_w_pro();
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      pbase = pbase0;
    }

    // pixel fragments of K-step kt from the patch (this lane's 8 channels of k = 64 kt + 32 ks
    // + 8 g -> tap, channel); the patch is complete for the whole tile, so step kt+1's are
    // read during step kt, before its barrier: after a barrier only the weight fragments wait
    auto tab_e = [&](int kt, int (&te)[2]) {
#if DP_HALO_TAB
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) te[ks] = tab[kt * 8 + 4 * ks + g];
#else
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int k = kt * 64 + (4 * ks + g) * 8;
        int tap = (unsigned)k / (unsigned)cin;
        int ci = k - tap * cin;
        if (tap >= ktaps) tap = 0, ci = 0;           // kpad tail: weights are zero there
        const int ky = tap / KW, kx = tap - ky * KW;
        te[ks] = (ky * Gm::PW + kx) | (((ci >> 3) & 7) << 7) | ((ci >> 6) << 10);
      }
#endif
    };
    auto read_pf = [&](const int (&te)[2], bf16x8 (&pf)[2][TM]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int toff = te[ks] & 127, c8 = (te[ks] >> 7) & 7;
        const char* pl = pbase + (te[ks] >> 10) * Gm::PLANE;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int yq = wm * TM + i;
          const int pr = yq * S * Gm::PW + q * S + toff;
          pf[ks][i] = *reinterpret_cast<const bf16x8*>(pl + pr * 128 + ((c8 ^ (pr & 7)) << 4));
        }
      }
    };
    if constexpr (NKC > 0) {
#pragma unroll
      for (int kt = 0; kt < NKC; ++kt) {
        const char* wsl = wbase + kt * BN * 128;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int cc = 4 * ks + g;
          bf16x8 wf[TN], pf[TM];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int r = 16 * j + (lane & 15);
            wf[j] = *reinterpret_cast<const bf16x8*>(wsl + r * 128 + ((cc ^ (r & 7)) << 4));
          }
#pragma unroll
          for (int i = 0; i < TM; ++i) pf[i] = *reinterpret_cast<const bf16x8*>(pbase + pfa[kt][ks][i]);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  wf[j], pf[i], (kt == 0 && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      // tap-table entries two K-steps ahead, pixel fragments one step ahead
      bf16x8 pfc[2][TM], pfn[2][TM];
      int te[2];
      tab_e(0, te);
      read_pf(te, pfc);
      tab_e(nk > 1 ? 1 : 0, te);
      for (int kt = 0; kt < nk; ++kt) {
        const char* wsl;
        if (RESW) {
          wsl = wbase + kt * BN * 128;
        } else {
          if (kt > 0) {
            // step kt's weights landed: NR - 2 later steps may stay in flight (all near the end)
            if (!(DP_HALO_ABL & 1)) {
              if (kt + NR - 2 < nk) wait_vmcnt<(NR - 2) * GB>();
              else wait_vmcnt<0>();
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (!(DP_HALO_ABL & 2)) __builtin_amdgcn_s_barrier();
          }
          // the slot of step kt + NR - 1 held step kt - 1, which every wave is past (barrier)
          if (kt + NR - 1 < nk) issue_w(kt + NR - 1, wbase + ((kt + NR - 1) % NR) * BN * 128);
          wsl = wbase + (kt % NR) * BN * 128;
        }
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 wf[2][TN];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int r = 16 * j + (lane & 15);
            wf[ks][j] = *reinterpret_cast<const bf16x8*>(wsl + r * 128 + (((4 * ks + g) ^ (r & 7)) << 4));
          }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0][j], pfc[0][i], acc[i][j], 0, 0, 0);
        // unconditional (the last steps re-read valid entries): a branch here would merge the
        // wait-count states and make the MFMAs below wait for these reads
        __builtin_amdgcn_sched_barrier(0);   // keep these reads between the two MFMA groups
        read_pf(te, pfn);
        tab_e(kt + 2 < nk ? kt + 2 : nk - 1, te);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[1][j], pfc[1][i], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < TM; ++i) pfc[ks][i] = pfn[ks][i];
      }
    }
    if constexpr (EARLY) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (tile + G < ntiles) {
        issue_patch(tile + G, pbase0);
        if (!RESW) issue_w_pro();
      }
    }
    // epilogue: lane owns pixel (oy0 + yq, ox0 + q), channels lane_chan(g, 0 .. NPL-1)
    if constexpr ((DP_HALO_ABL & 4) != 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else if constexpr (NAT) {
      // channels 16j + 4g + r: bias + act + LAB, one 8-byte store per tile j (no res / up:
      // the dispatcher routes only plain convs here)
      f32x4 bias[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bias[j] = *reinterpret_cast<const f32x4*>(bias_l + 16 * j + 4 * g);
      bf16_t* outp = reinterpret_cast<bf16_t*>(d.out) + (int64_t)b * d.out_bstride;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int oy = oy0 + wm * TM + i, ox = ox0 + q;
        if (oy >= d.out_h || ox >= d.out_w) continue;
        bf16_t* op = outp + (int64_t)(oy * d.out_w + ox) * d.out_pstride;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (16 * j + 4 * g >= d.cout) continue;
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = act_t<ACT>(acc[i][j][r] + bias[j][r]);
            if (d.has_lab) v = d.lab_scale * v + d.lab_bias;
            o[r] = (bf16_t)v;
          }
          *reinterpret_cast<bf16x4*>(op + 16 * j + 4 * g) = o;
        }
      }
    } else {
      float bias[NPL];
#pragma unroll
      for (int e = 0; e < NPL; e += 4) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias_l + lane_chan<8>(g, e));
        bias[e] = b4[0], bias[e + 1] = b4[1], bias[e + 2] = b4[2], bias[e + 3] = b4[3];
      }
      const bool full = lane_full<bf16_t, NPL>(d, 0, g, vec_ok);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int oy = oy0 + wm * TM + i, ox = ox0 + q;
        if (oy < d.out_h && ox < d.out_w) epi_pixel<ACT, bf16_t, TN>(d, acc[i], bias, b, oy, ox, 0, g, full);
      }
    }
    if constexpr (POOL) {
      // max over the 2x2 window (yq + dy, q + dx) of the patch, 8 channels (chunk c8) per
      // lane; zero-filled patch pixels past the right/bottom edge are the F.pad zeros
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int yq = wm * TM + i;
        const int oy = oy0 + yq, ox = ox0 + q;
        if (oy >= d.out_h || ox >= d.out_w) continue;
        bf16_t* po = pool.out + (int64_t)b * pool.bstride + (int64_t)(oy * d.out_w + ox) * pool.pstride;
        for (int c8 = g; c8 < (cin >> 3); c8 += 4) {
          float m[8];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int pr = (yq + (t >> 1)) * Gm::PW + q + (t & 1);
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(pbase + pr * 128 + ((c8 ^ (pr & 7)) << 4));
#pragma unroll
            for (int e = 0; e < 8; ++e) m[e] = t ? fmaxf(m[e], (float)v[e]) : (float)v[e];
          }
          Vec16<bf16_t> o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o.set(e, m[e]);
          store16(po + c8 * 8, o);
        }
      }
    }
    prev_full = tile_full && !POOL && !(DP_HALO_ABL & 4);
  }
  wait_vmcnt<0>();
}

template <int TH, int NW, int KH, int KW, int S, int BN, bool RESW, bool DBUF, int ACT, bool POOL = false, int NKC = 0,
          int NR = 2>
int launch_halo(const dp_conv_desc& d, hipStream_t s, int vec_ok, int lds, HaloPool pool = {}) {
  DP_DESCRIBE("conv_halo_kernel<%d, %d, %d, %d, %d, %d, %s, %s, %d, %s, %d, %d>", TH, NW, KH, KW, S, BN, DP_TF(RESW),
              DP_TF(DBUF), ACT, DP_TF(POOL), NKC, NR);
  auto kern = conv_halo_kernel<TH, NW, KH, KW, S, BN, RESW, DBUF, ACT, POOL, NKC, NR>;
  static const int occ = [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, NW * 64, lds) != hipSuccess || o <= 0) o = 1;
    if (getenv("DETRPOSE_CONV_DEBUG"))
      fprintf(stderr, "conv_halo TH=%d NW=%d K=%dx%d S=%d BN=%d resw=%d act=%d: lds %d, occupancy %d\n", TH, NW, KH,
              KW, S, BN, (int)RESW, ACT, lds, o);
    return o;
  }();
  const int tiles_x = (d.out_w + 15) / 16, tiles_y = (d.out_h + TH - 1) / TH;
  const int ntiles = d.batch * tiles_x * tiles_y;
  // occupancy at THIS layer's LDS size (the static value was queried for the first one)
  int o = occ;
  const int fit = (160 * 1024) / lds;
  if (o > fit) o = fit;
  if (o < 1) o = 1;
  int grid = o * num_cus();
  const int need = (ntiles + 7) / 8 * 8;
  if (grid > need) grid = need;
  grid = grid / 8 * 8;
  if (grid < 8) grid = 8;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NW * 64), lds, s, d, tiles_x, tiles_y, ntiles, vec_ok, pool);
  return dp_check_launch("dp_conv2d(halo)");
}

template <int TH, int NW, int KH, int KW, int S, int BN, bool RESW, bool DBUF = false, bool POOL = false, int NKC = 0,
          int NR = 2>
int launch_halo_act(const dp_conv_desc& d, hipStream_t s, int vec_ok, int lds, HaloPool pool = {}) {
  switch (d.act) {
    case DP_ACT_RELU:
      return launch_halo<TH, NW, KH, KW, S, BN, RESW, DBUF, DP_ACT_RELU, POOL, NKC, NR>(d, s, vec_ok, lds, pool);
    case DP_ACT_SILU:
      return launch_halo<TH, NW, KH, KW, S, BN, RESW, DBUF, DP_ACT_SILU, POOL, NKC, NR>(d, s, vec_ok, lds, pool);
    case DP_ACT_NONE:
      return launch_halo<TH, NW, KH, KW, S, BN, RESW, DBUF, DP_ACT_NONE, POOL, NKC, NR>(d, s, vec_ok, lds, pool);
    default: return -1;
  }
}

}  // namespace

// bf16 KxK convs with cout <= 128; returns -1 when this shape has no halo instantiation
// (the caller falls back to the implicit-GEMM path).
int dp_conv2d_halo(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  static const bool off = getenv("DETRPOSE_NO_HALO") != nullptr;
  if (off || d.out_f32 || d.cout > 128 || d.act == DP_ACT_GELU) return -1;
  const int bn = (d.cout + 31) / 32 * 32;
  const int nk = d.kpad / 64, nkc = (d.cin + 63) / 64;
  constexpr int LMAX = 160 * 1024;
  if (nk * 8 * 4 > TAB_ENTRY_BYTES) return -1;
  auto lds_res = [&](int plane, int nbuf) { return TAB_BYTES + nk * bn * 128 + nbuf * nkc * plane; };  // resident W
  auto lds_str = [&](int plane) { return TAB_BYTES + 2 * bn * 128 + nkc * plane; };                     // W ring, 1 patch
  auto lds_res48 = [&](int plane, int nbuf) { return TAB_BYTES + nk * 48 * 128 + nbuf * nkc * plane; };
  if (d.kh == 3 && d.kw == 3 && d.stride == 1) {
    constexpr int P16 = HaloGeom<16, 3, 3, 1>::PLANE, P8 = HaloGeom<8, 3, 3, 1>::PLANE;
    // 48 output channels (HG stage 0 of L/X): a 48-wide tile, 25% fewer MFMAs than 64
    if (d.cout == 48 && !d.res && !d.up && d.out_pstride % 4 == 0 && d.out_bstride % 4 == 0 &&
        (reinterpret_cast<uintptr_t>(d.out) & 7) == 0 && lds_res48(P16, 2) <= LMAX) {
      static const bool rt_k = getenv("DETRPOSE_HALO_RTK") != nullptr;   // A/B: the runtime K loop
      if (nk == 7 && !rt_k)   // cin 48: 9 x 48 = 432 -> 7 K-steps
        return launch_halo_act<16, 8, 3, 3, 1, 48, true, true, false, 7>(d, s, vec_ok, lds_res48(P16, 2));
      return launch_halo_act<16, 8, 3, 3, 1, 48, true, true>(d, s, vec_ok, lds_res48(P16, 2));
    }
    if (bn == 64 && lds_res(P16, 2) <= LMAX)
      return launch_halo_act<16, 8, 3, 3, 1, 64, true, true>(d, s, vec_ok, lds_res(P16, 2));
    if (bn == 32 && lds_res(P8, 1) <= 80 * 1024) return launch_halo_act<8, 4, 3, 3, 1, 32, true>(d, s, vec_ok, lds_res(P8, 1));
    // the 128-channel convs on maps of >= 64 x 64 (the encoder's stride-8 level): 16 x 16 tiles of
    // 8 waves, one block per CU, a 4-deep weight ring (3 K-steps of weight DMA in flight): the
    // L b64 80 x 80 shapes 148.5 -> 139.4 us, outputs bit-identical (profiles/r5z_halo_nr_ab.txt);
    // 40 x 40 is slower this way (tile quantisation: 64 vs 43 us) and keeps the 8-row tiles.
    // DETRPOSE_HALO_NR = 2 (off) / 3 / 4 overrides (A/B).
    static const int halo_nr = getenv("DETRPOSE_HALO_NR") ? atoi(getenv("DETRPOSE_HALO_NR")) : 4;
    if (bn == 128 && (halo_nr == 3 || halo_nr == 4) && d.out_h >= 64 && d.out_w >= 64) {
      auto lds_nr = [&](int nr) { return TAB_BYTES + nr * bn * 128 + nkc * P16; };
      if (halo_nr == 3 && lds_nr(3) <= LMAX)
        return launch_halo_act<16, 8, 3, 3, 1, 128, false, false, false, 0, 3>(d, s, vec_ok, lds_nr(3));
      if (halo_nr == 4 && lds_nr(4) <= LMAX)
        return launch_halo_act<16, 8, 3, 3, 1, 128, false, false, false, 0, 4>(d, s, vec_ok, lds_nr(4));
    }
    if (lds_str(P8) > 80 * 1024) return -1;
    if (bn == 64) return launch_halo_act<8, 4, 3, 3, 1, 64, false>(d, s, vec_ok, lds_str(P8));
    if (bn == 96) return launch_halo_act<8, 4, 3, 3, 1, 96, false>(d, s, vec_ok, lds_str(P8));
    if (bn == 128) return launch_halo_act<8, 4, 3, 3, 1, 128, false>(d, s, vec_ok, lds_str(P8));
    return -1;
  }
  if (d.kh == 2 && d.kw == 2 && d.stride == 1) {
    constexpr int P = HaloGeom<8, 2, 2, 1>::PLANE;
    if (bn == 32 && lds_res(P, 1) <= 80 * 1024) return launch_halo_act<8, 4, 2, 2, 1, 32, true>(d, s, vec_ok, lds_res(P, 1));
    return -1;
  }
  return -1;
}

int dp_conv2d_stem_direct(const dp_conv_desc& d, hipStream_t s, void* pool, int64_t pbs, int pps);

// dp_conv2d of a 2x2 s1 bf16 conv (pad 0, zero read past the right/bottom edge) that also
// writes MaxPool2d(2, 1) of the same zero-padded input: StemBlock's stem2a + pool
// (hgnetv2.py:213-220), i.e. dp_conv2d followed by dp_maxpool2x2_pad_rb in one pass.
extern "C" int dp_conv2d_pool(const dp_conv_desc* dp, void* pool_out, int64_t pool_bstride, int32_t pool_pstride,
                              void* stream) {
  DP_REQUIRE(dp != nullptr && pool_out != nullptr, "dp_conv2d_pool: null pointer");
  const dp_conv_desc& d = *dp;
  DP_REQUIRE(d.dtype == DP_BF16 && !d.out_f32 && !d.res && !d.up, "dp_conv2d_pool: bf16 conv without res/up only");
  DP_REQUIRE(d.kh == 2 && d.kw == 2 && d.stride == 1 && d.pad_t == 0 && d.pad_l == 0,
             "dp_conv2d_pool: 2x2 stride-1 conv with right/bottom zero padding only");
  DP_REQUIRE(d.out_h == d.in_h && d.out_w == d.in_w, "dp_conv2d_pool: output must keep the input size");
  DP_REQUIRE(d.cin % 8 == 0 && d.cin <= 64 && d.cout <= 32, "dp_conv2d_pool: cin %% 8 == 0, cin <= 64, cout <= 32");
  DP_REQUIRE(d.in && d.weight && d.out && d.batch > 0 && d.kpad % 64 == 0 && d.kpad >= 4 * d.cin,
             "dp_conv2d_pool: bad descriptor");
  DP_REQUIRE((reinterpret_cast<uintptr_t>(d.in) & 15) == 0 && (reinterpret_cast<uintptr_t>(d.weight) & 15) == 0 &&
                 d.in_pstride % 8 == 0 && d.in_bstride % 8 == 0,
             "dp_conv2d_pool: input / weight must be 16-byte aligned");
  DP_REQUIRE((reinterpret_cast<uintptr_t>(pool_out) & 15) == 0 && pool_pstride % 8 == 0 && pool_bstride % 8 == 0,
             "dp_conv2d_pool: pool output must be 16-byte aligned per pixel");
  DP_REQUIRE(d.in_bstride * 2 < 0x7ff00000ll && (int64_t)d.batch * d.out_h * d.out_w < (1ll << 31),
             "dp_conv2d_pool: image exceeds 32-bit buffer offsets");
  constexpr int P = HaloGeom<8, 2, 2, 1>::PLANE;
  const int lds = TAB_BYTES + (d.kpad / 64) * 32 * 128 + P;
  DP_REQUIRE(lds <= 80 * 1024, "dp_conv2d_pool: weights do not fit LDS");
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec_ok = (d.out_pstride % 8 == 0) && (d.out_bstride % 8 == 0) && al(d.out);
  const int r = dp_conv2d_stem_direct(d, as_stream(stream), pool_out, pool_bstride, pool_pstride);
  if (r >= 0) return r;   // stem shapes: register-direct kernel (stem.hip)
  const HaloPool pool{reinterpret_cast<bf16_t*>(pool_out), pool_bstride, pool_pstride};
  return launch_halo_act<8, 4, 2, 2, 1, 32, true, false, true>(d, as_stream(stream), vec_ok, lds, pool);
}
