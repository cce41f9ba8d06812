// StemBlock.stem1's K order (hgnetv2.py:171-177: 3x3 s2 conv, 3 input channels), shared by the
// one-launch stem (stem_fused.hip) and the stand-alone stem1 kernel (stem.hip) for the
// 32-channel stems (B4 / B5) so the two stay bit-identical. (The 16-channel stems, which have no
// fused kernel, keep the one-slab order k = c * 9 + ky * 3 + kx: stem1_slot_c9.)
//
// The 27 products (c, ky, kx) are laid out as two 32-wide MFMA K slabs of (tap, channel slot)
// pairs with 4 channel slots per tap (slot 3 is zero): lane group g of slab 0 holds the slots
// of two taps, 8 bf16 = 2 x 8 bytes, which in the fused kernel's pixel-major image patch
// ([row][col][4 channels]) are two 8-byte LDS reads instead of eight 2-byte ones:
//   slab 0, g = 0 / 1 / 2: taps (ky = g, kx = 0), (ky = g, kx = 1)
//   slab 0, g = 3:         taps (1, 2), (0, 2)
//   slab 1, g = 0:         tap (2, 2) in the low 4 slots; every other slab-1 slot is zero.
// The MFMAs run slab 0 then slab 1 into the same accumulator.
#pragma once

// slot e (0..7) of lane group g in slab s -> (c, ky, kx); false for a zero slot
__device__ __forceinline__ constexpr bool stem1_slot(int s, int g, int e, int& c, int& ky, int& kx) {
  c = e & 3;
  const int h = e >> 2;
  if (s == 0) {
    ky = g < 3 ? g : 1 - h;
    kx = g < 3 ? h : 2;
  } else {
    ky = 2, kx = 2;
    if (g != 0 || h != 0) return false;
  }
  return c < 3;
}

// the one-slab order: slot e of lane group g is k = 8g + e = c * 9 + ky * 3 + kx (k < 27)
__device__ __forceinline__ constexpr bool stem1_slot_c9(int g, int e, int& c, int& ky, int& kx) {
  const int k = 8 * g + e;
  c = k < 27 ? k / 9 : 0;
  const int t = k - 9 * (k / 9);
  ky = t / 3, kx = t - 3 * (t / 3);
  return k < 27;
}
