"""Host restatement of the 4-wave GEMM's persistent tile schedule (videoprism-mlx_amd/csrc/
gemm_bf16_w4.hip: the XCD-contiguous first/stride/count split, `coords` and `w4_ngrp`), checked
for what the kernel relies on: every output tile is computed exactly once, by one workgroup, for
every shape class the forward launches (Base / Large, B = 1..48 clips) and for odd grids.  CPU only;
the GPU side of the same property is the bitwise w4 == w8 test (tests/test_gpu_kernels.py)."""

import pytest

BM = BN = 256


def w4_ngrp(M, N, K, grid):
    """gemm_bf16_w4.hip w4_ngrp: N-tile group size of the grouped tile order."""
    tiles_n = N // BN
    w_tile = BN * K * 2
    w_all = tiles_n * w_tile
    if w_all <= (2 << 20) or K >= 2048 or (M // BM) % 8 or grid % 8:
        return tiles_n
    budget = (5 << 19) if w_all > (4 << 20) else w_all // 2
    for d in range(tiles_n, 0, -1):
        if tiles_n % d == 0 and d * w_tile <= budget:
            return d
    return tiles_n


def coords(t, M, tiles_n, ngrp):
    """gemm_bf16_w4.hip coords: tile index -> (M-block, N-tile)."""
    if ngrp == tiles_n:
        return divmod(t, tiles_n)
    mbx = (M // BM) >> 3
    x, u = divmod(t, mbx * tiles_n)
    gi, r = divmod(u, mbx * ngrp)
    rm, rn = divmod(r, ngrp)
    return x * mbx + rm, gi * ngrp + rn


def schedule(M, N, K, cus=256):
    """Tiles of every workgroup, in the order the workgroup computes them."""
    tiles_n = N // BN
    T = (M // BM) * tiles_n
    G = min(T, cus)
    ngrp = w4_ngrp(M, N, K, G)
    out = []
    for b in range(G):
        if G % 8 == 0:
            xcd, li, nx = b & 7, b >> 3, G >> 3
            lo, hi = (xcd * T) >> 3, ((xcd + 1) * T) >> 3
            first, stride = lo + li, nx
            count = (hi - first + nx - 1) // nx if first < hi else 0
        else:
            first, stride = b, G
            count = (T - b + G - 1) // G if b < T else 0
        out.append([coords(first + j * stride, M, tiles_n, ngrp) for j in range(count)])
    return out, ngrp


# (N, K) of the forward's GEMMs: Base qkv / post / ffn1 / ffn2 / patch embed, Large the same
SHAPES = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (768, 1024),
          (3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)]


@pytest.mark.parametrize("clips", [1, 2, 3, 8, 16, 32, 48])
@pytest.mark.parametrize("N,K", SHAPES)
def test_every_tile_once(clips, N, K):
    M = clips * 16 * 256
    sched, ngrp = schedule(M, N, K)
    seen = [t for wg in sched for t in wg]
    assert len(seen) == len(set(seen)) == (M // BM) * (N // BN)
    assert all(0 <= tm < M // BM and 0 <= tn < N // BN for tm, tn in seen)
    if ngrp < N // BN:  # grouped: the group's W rows fit the 2.5 MB budget, A is not HBM-streamed
        assert ngrp * BN * K * 2 <= (5 << 19) and K < 2048 and (N // BN) * BN * K * 2 > (2 << 20)


def test_grouping_applies_where_intended():
    # Base ffn_layer1 at B = 32: W = 4.7 MB > an XCD's L2 -> groups of 6 N-tiles; Base qkv (3.5 MB)
    # groups of 3; ffn_layer2 (K = 3072, A from HBM) and post (1.2 MB) stay ungrouped; Large ffn1 / qkv: 4
    M = 32 * 16 * 256
    assert schedule(M, 3072, 768)[1] == 6
    assert schedule(M, 2304, 768)[1] == 3
    assert schedule(M, 768, 768)[1] == 3
    assert schedule(M, 768, 3072)[1] == 3
    assert schedule(16 * 16 * 256, 4096, 1024)[1] == 4
    assert schedule(16 * 16 * 256, 3072, 1024)[1] == 4


def test_grouped_xcd_sweeps_m_blocks_per_group():
    """With grouping, an XCD's workgroups finish group 0's N-tiles over all the XCD's M-blocks
    before any tile of group 1 starts (in schedule order), which keeps a group's W L2-resident."""
    M, N, K = 32 * 16 * 256, 3072, 768
    sched, ngrp = schedule(M, N, K)
    G = len(sched)
    for xcd in range(8):
        wgs = [sched[b] for b in range(xcd, G, 8)]
        rounds = max(len(w) for w in wgs)
        groups = [sorted({tn // ngrp for w in wgs if j < len(w) for tn in [w[j][1]]}) for j in range(rounds)]
        flat = [g for r in groups for g in r]
        assert flat == sorted(flat)  # group index never decreases from one round to the next
