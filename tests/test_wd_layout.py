"""Host-side checks of the W-direct GEMM's weight layout (gemm_bf16_w4.hip, WD): the library's
packer (`w4_pack_frag`, used by vp_finalize) against a NumPy restatement, and the kernel's
fragment addressing restated on the host -- every MFMA operand element the kernel loads from the
packed copy must be the W element the LDS-staged kernel reads for the same (tile, wave, k-half,
fragment, lane) slot.  No GPU needed (the packer is host code)."""

import numpy as np
import pytest
import torch

from videoprism import _native as nat


def _np_pack(w):
    N, K = w.shape
    return w.reshape(N // 128, 8, 16, K // 32, 4, 8).transpose(0, 3, 1, 4, 2, 5).reshape(N, K)


@pytest.mark.parametrize("N,K", [(256, 64), (768, 768), (3072, 768), (768, 3072), (384, 96)])
def test_pack_frag_matches_restatement(N, K):
    rng = np.random.default_rng(N * 7 + K)
    bits = rng.integers(0, 1 << 16, size=(N, K), dtype=np.uint16)
    w = torch.from_numpy(bits.view(np.int16).copy()).view(torch.bfloat16)
    got = nat.pack_frag(w).view(torch.int16).numpy().view(np.uint16)
    np.testing.assert_array_equal(got, _np_pack(bits))


def test_pack_frag_rejects_bad_shapes():
    with pytest.raises(Exception):
        nat.pack_frag(torch.zeros(192, 64, dtype=torch.bfloat16))  # N % 128
    with pytest.raises(Exception):
        nat.pack_frag(torch.zeros(256, 48, dtype=torch.bfloat16))  # K % 32


@pytest.mark.parametrize("N,K", [(512, 128), (768, 192)])
def test_kernel_fragment_addressing(N, K):
    """Restates wload(): wave wn of tile column tn, K-tile kt, k-half kh, fragment nt, lane l,
    element e reads packed byte ((((tn*2+wn)*(K/32) + 2kt+kh) << 13) + nt*1024 + 16 l + 2 e); the
    LDS path's operand for that slot is W[tn*256 + wn*128 + nt*16 + (l & 15)][64 kt + 32 kh + 8 (l >> 4) + e]."""
    w = np.arange(N * K, dtype=np.int64).reshape(N, K)  # element ids
    packed = _np_pack(w).reshape(-1)
    for tn in range(N // 256):
        for wn in range(2):
            for kt in range(K // 64):
                for kh in range(2):
                    base = (((tn * 2 + wn) * (K // 32) + 2 * kt + kh) << 13) // 2  # in elements
                    for nt in range(8):
                        for lane in range(64):
                            off = base + nt * 512 + lane * 8
                            n = tn * 256 + wn * 128 + nt * 16 + (lane & 15)
                            k = 64 * kt + 32 * kh + 8 * (lane >> 4)
                            np.testing.assert_array_equal(packed[off:off + 8], w[n, k:k + 8])
