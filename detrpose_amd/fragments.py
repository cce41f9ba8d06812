"""MFMA-fragment weight layout of the row-block decoder kernels (include/detrpose_hip.h,
"fragment layout"; csrc/decoder.hip).

A weight W [N][K] (nn.Linear layout) is stored as blocks of 32 output channels x 32 input
channels; block (nb, s) holds 2 fragments of 64 lanes x 8 bf16, fragment j lane l =
(g = l // 16, q = l % 16) holding W[32 nb + chan(j, q)][32 s + 8 g : 32 s + 8 g + 8] with
chan(j, q) = (q // 4) * 8 + 4 j + q % 4: exactly the A operand a lane of a wave feeds to
v_mfma_f32_16x16x32_bf16 for its 32 channels, so one wave reads a fragment as one
contiguous 1 KB access. N is zero-padded to a multiple of 32, K must be a multiple of 32.
"""
from __future__ import annotations

import torch


def frag_pack(w: torch.Tensor) -> torch.Tensor:
    """W [N][K] -> bf16 [ceil(N/32)][K/32][2][64][8] (contiguous)."""
    n, k = w.shape
    assert k % 32 == 0, f"K={k} must be a multiple of 32"
    npad = (n + 31) // 32 * 32
    wp = torch.zeros(npad, k, dtype=torch.float32, device=w.device)
    wp[:n] = w.float()
    q = torch.arange(16)
    chan = torch.stack([(q // 4) * 8 + 4 * j + q % 4 for j in range(2)])            # [2][16]
    w5 = wp.reshape(npad // 32, 32, k // 32, 4, 8)                                    # [nb][c][s][g][8]
    f = w5[:, chan.reshape(-1).to(w.device)].reshape(npad // 32, 2, 16, k // 32, 4, 8)  # [nb][j][q][s][g][8]
    f = f.permute(0, 3, 1, 4, 2, 5)                                                   # [nb][s][j][g][q][8]
    return f.reshape(npad // 32, k // 32, 2, 64, 8).to(torch.bfloat16).contiguous()


def frag_unpack(f: torch.Tensor, n: int) -> torch.Tensor:
    """Inverse of frag_pack (tests): -> float [n][K]."""
    nb, ns = f.shape[:2]
    q = torch.arange(16)
    chan = torch.stack([(q // 4) * 8 + 4 * j + q % 4 for j in range(2)]).reshape(-1)
    g = f.float().reshape(nb, ns, 2, 4, 16, 8).permute(0, 2, 4, 1, 3, 5).reshape(nb, 32, ns, 4, 8)
    out = torch.empty_like(g)
    out[:, chan] = g
    return out.reshape(nb * 32, ns * 32)[:n]
