// bf16 implicit-GEMM convolution with LDS-DMA staging (gfx950), the main path of
// dp_conv2d for bf16 activations (conv_gemm.hip keeps the register-staged kernel for
// f32 parity mode and odd shapes).
//
// Same GEMM view as conv_gemm.hip (C[M][N] = A[M][K] W[N][K]^T, A gathered from the NHWC
// input), but the tiles go HBM/L2 -> LDS with `buffer_load_dwordx4 ... lds` (no staging
// VGPRs), through an S-stage ring so S-1 K-steps are in flight while one is consumed.
//  * One DMA instruction moves 8 rows x 128 B (one 64-wide bf16 K-step of 8 rows).
//    Lane L always lands in row L>>3, physical 16-byte chunk L&7 of its group, so the
//    16-byte chunks are XOR-swizzled by fetching logical chunk (L&7)^(L>>3): the MFMA
//    fragment reads (16 rows x 16 B per lane group) are then bank-conflict free.
//  * Out-of-range buffer offsets return 0: conv zero padding, K/M/N tails (as in v2).
//  * Each wave waits only for its own DMAs of the stage it is about to read (counted
//    vmcnt), then a raw s_barrier publishes all waves' DMAs; the barrier also retires
//    the previous stage's ds_reads before that slot is refilled (guide §5 glds rules).
#include "conv_epilogue.h"

namespace {

constexpr int OOB = 0x7fffffff;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7ffffff0, 0x00020000);
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int WGM, int S, bool K1X1, typename TO>
__global__ __launch_bounds__(256) void conv_glds_kernel(dp_conv_desc d, int M, int nt_n, int vec_ok) {
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int GA = BM / 32, GB = BN / 32;           // DMA groups (8 rows) per wave per K-step
  constexpr int LPS = GA + GB;                        // DMA instructions per wave per K-step
  constexpr int STAGE = (BM + BN) * 128;              // bytes per stage
  constexpr int CBYTES = BM * (BN + 16 / (int)sizeof(TO)) * (int)sizeof(TO);
  constexpr int BYTES = S * STAGE > CBYTES ? S * STAGE : CBYTES;
  static_assert(BM % 32 == 0 && BN % 32 == 0 && TM >= 1 && TN >= 1, "tile");
  __shared__ __attribute__((aligned(1024))) char smem[BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  const int nwg = gridDim.x, pid = blockIdx.x;
  const int xcd = pid & 7, q = nwg >> 3, rr = nwg & 7;
  const int logical = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (pid >> 3);
  const int tn = logical % nt_n, tm = logical / nt_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int hwo = d.out_h * d.out_w;
  const int b_first = m0 / hwo;
  const __amdgpu_buffer_rsrc_t ra_src =
      make_rsrc(reinterpret_cast<const bf16_t*>(d.in) + (int64_t)b_first * d.in_bstride);
  const __amdgpu_buffer_rsrc_t rb_src = make_rsrc(d.weight);

  const int r8 = lane >> 3;
  const int chunk = (lane & 7) ^ r8;   // logical 16-byte chunk this lane fetches

  int a_off[GA], a_iy0[GA], a_ix0[GA];
#pragma unroll
  for (int t = 0; t < GA; ++t) {
    const int row = (wave + 4 * t) * 8 + r8;
    const int m = m0 + row;
    const bool ok = m < M;
    const int mm = ok ? m : m0;
    const int b = mm / hwo, rem = mm - b * hwo;
    const int oy = rem / d.out_w, ox = rem - oy * d.out_w;
    const int iy0 = oy * d.stride - d.pad_t;
    a_iy0[t] = ok ? iy0 : -0x4000000;
    a_ix0[t] = ox * d.stride - d.pad_l;
    int off = (b - b_first) * (int)d.in_bstride;
    if (K1X1) off += (iy0 * d.in_w + a_ix0[t]) * d.in_pstride;
    a_off[t] = ok ? off : OOB;
  }
  int b_off[GB];
#pragma unroll
  for (int t = 0; t < GB; ++t) {
    const int n = n0 + (wave + 4 * t) * 8 + r8;
    b_off[t] = n < d.cout ? n * d.kpad + chunk * 8 : OOB;
  }
  const int ntap = d.kh * d.kw;
  const int nk = d.kpad / 64;

  auto issue = [&](int kt, int stage) {
    char* sb = smem + stage * STAGE;
    const int kk = kt * 64 + chunk * 8;
    if (K1X1) {
      const bool kv = kk < d.cin;
#pragma unroll
      for (int t = 0; t < GA; ++t) {
        const int o = (a_off[t] != OOB && kv) ? (a_off[t] + kk) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_src, (lds_ptr_t)(sb + (wave + 4 * t) * 1024), 16, o, 0, 0, 0);
      }
    } else {
      const int tap = kk / d.cin, ci = kk - tap * d.cin;
      const int ky = tap / d.kw, kx = tap - ky * d.kw;
      const bool kv = tap < ntap;
#pragma unroll
      for (int t = 0; t < GA; ++t) {
        const int iy = a_iy0[t] + ky, ix = a_ix0[t] + kx;
        const bool ok = kv && (unsigned)iy < (unsigned)d.in_h && (unsigned)ix < (unsigned)d.in_w;
        const int o = ok ? (a_off[t] + (iy * d.in_w + ix) * d.in_pstride + ci) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_src, (lds_ptr_t)(sb + (wave + 4 * t) * 1024), 16, o, 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < GB; ++t) {
      const int o = b_off[t] != OOB ? (b_off[t] + kt * 64) * 2 : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb_src, (lds_ptr_t)(sb + BM * 128 + (wave + 4 * t) * 1024), 16, o, 0,
                                               0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lg = lane >> 4;
  // fragment byte offsets within a stage: row r, logical chunk c -> r*128 + ((c ^ (r&7)) * 16)
  const int arow = wm * WM + lr;
  const int brow = wn * WN + lr;

#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    // own DMAs of stage kt done; the S-2 younger stages may stay in flight
    const int ahead = min(S - 2, nk - 1 - kt);
    if (ahead >= 2) wait_vmcnt<2 * LPS>();
    else if (ahead == 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
    const char* sb = smem + (kt % S) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 4 * ks + lg;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = arow + 16 * i;
        af[i] = *reinterpret_cast<const bf16x8*>(sb + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = brow + 16 * j;
        bfr[j] = *reinterpret_cast<const bf16x8*>(sb + BM * 128 + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  conv_epilogue<TO, BM, BN, WGM, TM, TN>(d, acc, smem, M, m0, n0, vec_ok);
}

#ifndef DP_GLDS_S
#define DP_GLDS_S 2
#endif

template <int BM, int BN, int WGM, typename TO>
int launch(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  const int M = d.batch * d.out_h * d.out_w;
  const int mt = (M + BM - 1) / BM, nt = (d.cout + BN - 1) / BN;
  const bool k1 = d.kh == 1 && d.kw == 1 && d.pad_t == 0 && d.pad_l == 0;
  dim3 grid(mt * nt), block(256);
  constexpr int S = DP_GLDS_S;
  if (k1) hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WGM, S, true, TO>), grid, block, 0, s, d, M, nt, vec_ok);
  else hipLaunchKernelGGL((conv_glds_kernel<BM, BN, WGM, S, false, TO>), grid, block, 0, s, d, M, nt, vec_ok);
  return dp_check_launch("dp_conv2d(glds)");
}

}  // namespace

// bf16 entry used by dp_conv2d (conv_gemm.hip); vec_ok computed by the caller.
int dp_conv2d_glds(const dp_conv_desc& d, hipStream_t s, int vec_ok) {
  const int M = d.batch * d.out_h * d.out_w;
  const bool f32o = d.out_f32 != 0;
  if (d.cout <= 32) return f32o ? launch<128, 32, 4, float>(d, s, vec_ok) : launch<128, 32, 4, bf16_t>(d, s, vec_ok);
  if (d.cout <= 64) return f32o ? launch<128, 64, 4, float>(d, s, vec_ok) : launch<128, 64, 4, bf16_t>(d, s, vec_ok);
  if (M <= 8192) return f32o ? launch<64, 128, 2, float>(d, s, vec_ok) : launch<64, 128, 2, bf16_t>(d, s, vec_ok);
  return f32o ? launch<128, 128, 2, float>(d, s, vec_ok) : launch<128, 128, 2, bf16_t>(d, s, vec_ok);
}
