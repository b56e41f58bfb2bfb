"""Host restatement of the lane bookkeeping of the fused temporal attention (gemm_bf16_w4.hip,
EPI_QK_TATTN_LN / EPI_V_TATTN_LN), CPU only.

The QK launch feeds the 16x16x32 MFMA straight from the GEMM accumulators: a lane holds one row
and 4 consecutive columns of each 16x16 block, so the bf16 operand of 32 columns is built from two
blocks and its k-slot 8*g + i stands for column 16*(2kk + (i >= 4)) + 4*g + (i & 3).  The same
map on both operands leaves every dot product unchanged; this test restates the MFMA lane layouts
(MI355X_MICROARCH / cdna_hip_programming: A[i][k] at lane i + 16*(k // 8), B[k][j] at lane
j + 16*(k // 8), D[i][j] at lane j + 16*(i // 4)) and checks that the logits come out as
q . k^T for every (query, key), and that the P^T fragment a lane stores is the one the V launch's
lane of the same index loads as its 16x16x16 B operand (B[k][j] at lane j + 16*(k // 4)).
"""

import numpy as np


def acc_block_lane_values(M16, lane):
    """The 4 values lane `lane` holds of a 16x16 accumulator block M16[row][col]: row lane % 16,
    columns 4*(lane // 16) .. +3."""
    r, g = lane % 16, lane // 16
    return M16[r, 4 * g:4 * g + 4]


def operand_from_blocks(blkA, blkB, lane):
    """bf16x8 operand of a lane from two accumulator blocks (k-slots 0..3 from blkA, 4..7 from blkB)."""
    return np.concatenate([acc_block_lane_values(blkA, lane), acc_block_lane_values(blkB, lane)])


def mfma_16x16x32(a_lanes, b_lanes):
    """D = A . B with A [16][32] given per lane (lane l: A[l % 16][8*(l//16) .. +7]) and
    B [32][16] per lane (lane l: B[8*(l//16) .. +7][l % 16]); returns D per lane
    (lane l: D[4*(l//16) + r][l % 16], r = 0..3)."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for l in range(64):
        A[l % 16, 8 * (l // 16):8 * (l // 16) + 8] = a_lanes[l]
        B[8 * (l // 16):8 * (l // 16) + 8, l % 16] = b_lanes[l]
    D = A @ B
    return [D[4 * (l // 16):4 * (l // 16) + 4, l % 16] for l in range(64)]


def test_logits_from_accumulator_layout_operands():
    rng = np.random.default_rng(0)
    q = rng.normal(size=(16, 64))   # one sequence: 16 queries x dh 64 (columns 0..63 of the wave)
    k = rng.normal(size=(16, 64))   # its keys (columns 64..127)
    qb = [q[:, 16 * nt:16 * nt + 16] for nt in range(4)]   # accumulator blocks nt = 0..3
    kb = [k[:, 16 * nt:16 * nt + 16] for nt in range(4)]   # nt = 4..7
    x = [np.zeros(4) for _ in range(64)]
    for kk in range(2):
        kop = [operand_from_blocks(kb[2 * kk], kb[2 * kk + 1], l) for l in range(64)]
        qop = [operand_from_blocks(qb[2 * kk], qb[2 * kk + 1], l) for l in range(64)]
        d = mfma_16x16x32(kop, qop)
        x = [x[l] + d[l] for l in range(64)]
    logits = q @ k.T   # [query][key]
    for l in range(64):
        for r in range(4):
            # x[r] = logit[query l % 16][key 4*(l // 16) + r]
            assert np.isclose(x[l][r], logits[l % 16, 4 * (l // 16) + r])


def test_probability_fragment_handoff():
    """The QK launch's lane l stores P[query l%16][keys 4*(l//16)+r] at offset l*4 + r of the
    (sequence, head) record; the V launch's lane l loads offset l*4 .. +3 as its B operand
    B[k = 4*(l//16) + r][j = l % 16] = P^T[key][query], so O^T = V^T . P^T needs no shuffle."""
    rng = np.random.default_rng(1)
    P = rng.random((16, 16))
    rec = np.zeros(256)
    for l in range(64):
        for r in range(4):
            rec[l * 4 + r] = P[l % 16, 4 * (l // 16) + r]
    B = np.zeros((16, 16))
    for l in range(64):
        B[4 * (l // 16):4 * (l // 16) + 4, l % 16] = rec[l * 4:l * 4 + 4]
    assert np.array_equal(B, P.T)
    # and the 16x16x16 result D[i][j] at lane j + 16*(i // 4) is O^T[d][query]: the accumulator
    # layout of O (row = query = lane % 16, columns 16*dt + 4*(lane // 16) + r)
    V = rng.normal(size=(16, 64))
    O = P @ V
    for dt in range(4):
        D = V[:, 16 * dt:16 * dt + 16].T @ B   # O^T block [d][query]
        for l in range(64):
            got = D[4 * (l // 16):4 * (l // 16) + 4, l % 16]
            assert np.allclose(got, acc_block_lane_values(O[:, 16 * dt:16 * dt + 16], l))


def test_qk_row_permutation_of_the_projection():
    """pack_stack(qk_perm): rows [q_h | k_h] per head from the fused [q | k | v] layout, so a
    256-column tile is two heads and each wave's 128 columns one head."""
    D, H = 768, 12
    fused = np.arange(3 * D)          # row ids of [q(D) | k(D) | v(D)], head-major inside each
    perm = []
    for h in range(H):
        for which in range(2):
            perm.extend(which * D + h * 64 + np.arange(64))
    perm = np.array(perm)
    assert sorted(perm) == list(range(2 * D))
    for h in range(H):
        cols = perm[h * 128:(h + 1) * 128]
        assert np.array_equal(cols[:64], fused[h * 64:(h + 1) * 64])            # q_h
        assert np.array_equal(cols[64:], fused[D + h * 64:D + (h + 1) * 64])    # k_h
        assert (h * 128) // 128 == h   # head of the wave whose columns start at n0 = 128 h
