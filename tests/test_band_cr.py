"""The elimination schedule of k_bcr_band (ba_band.hip), restated in numpy and checked against a dense solve.

k_bcr_band solves the reduced camera system of a narrow-band window, S = [A B; B^T C] with A block-tridiagonal
(nb blocks of G dofs, the last one padded with identity rows), by odd-even cyclic reduction: level m eliminates
the blocks i with i + 1 = odd * 2^m, each survivor j pulls the Schur terms of i1 = j - 2^m and i2 = j + 2^m,
the border is carried as four right-hand sides and closed by the 4x4 system of the summed Grams. This file
restates exactly that schedule (the same neighbour arithmetic, the same in-place roles of CL / XR / BB / BV) so
that the index logic is pinned on the CPU; the GPU kernel itself is checked against the oracle in
tests/test_gpu_parity.py::test_band_one_workgroup_solve."""
import numpy as np
import pytest


def _window(nac, bc, seed):
    """A random SPD arrowhead system with camera band bc (in cameras): 6 nac camera dofs + 4 border dofs."""
    rng = np.random.default_rng(seed)
    n = 6 * nac
    J = np.zeros((8 * nac, n + 4))
    for a in range(nac):  # each 'observation' couples a camera with its successors within the band and the border
        for r in range(8):
            row = 8 * a + r
            hi = min(nac, a + bc + 1)
            J[row, 6 * a:6 * hi] = rng.normal(size=6 * (hi - a))
            J[row, n:] = rng.normal(size=4)
    S = J.T @ J + 0.1 * np.eye(n + 4)
    b = rng.normal(size=n + 4)
    return S, b


def band_cr_solve(S, b, nac, bc):
    n = 6 * nac
    G = 6 * bc
    nb = (nac + bc - 1) // bc
    D = np.zeros((nb, G, G))
    CL = np.zeros((nb, G, G))
    XR = np.zeros((nb, G, G))
    BB = np.zeros((nb, G, 4))
    BV = np.zeros((nb, G))
    for j in range(nb):  # the load phase: identity past the last camera dof
        for r in range(G):
            for c in range(G):
                dr, dc = j * G + r, j * G + c
                D[j, r, c] = S[dr, dc] if dr < n and dc < n else float(r == c)
                if j >= 1 and dr < n:
                    CL[j, r, c] = S[dr, (j - 1) * G + c]
            if j * G + r < n:
                BB[j, r] = S[n:, j * G + r]
                BV[j, r] = b[j * G + r]
    L = np.zeros_like(D)
    GR = np.zeros((nb, 4, 5))
    K = 0
    while (2 << K) <= nb:
        K += 1
    for m in range(K + 1):
        s = 1 << m
        ne = ((nb >> m) + 1) >> 1
        elim = [((2 * t + 1) << m) - 1 for t in range(ne)]
        for i in elim:
            L[i] = np.linalg.cholesky(D[i])
            rb = i + s
            CR = CL[rb].T if rb < nb else np.zeros((G, G))
            CL[i] = np.linalg.solve(L[i], CL[i])   # XL
            XR[i] = np.linalg.solve(L[i], CR)
            BV[i] = np.linalg.solve(L[i], BV[i])   # x
            BB[i] = np.linalg.solve(L[i], BB[i])   # XB
        ns = nb >> (m + 1) if m < K else 0
        for t in range(ns):
            j = ((t + 1) << (m + 1)) - 1
            i1, i2 = j - s, j + s
            D[j] -= XR[i1].T @ XR[i1]
            BV[j] -= XR[i1].T @ BV[i1]
            BB[j] -= XR[i1].T @ BB[i1]
            if i2 < nb:
                D[j] -= CL[i2].T @ CL[i2]
                BV[j] -= CL[i2].T @ BV[i2]
                BB[j] -= CL[i2].T @ BB[i2]
            CL[j] = -XR[i1].T @ CL[i1]
        for i in elim:
            GR[i, :, 0] = BB[i].T @ BV[i]
            GR[i, :, 1:] = BB[i].T @ BB[i]
    red = GR.sum(axis=0)
    C = S[n:, n:] - red[:, 1:]
    yk = np.linalg.solve(C, b[n:] - red[:, 0])
    Y = np.zeros((nb, G))
    for m in range(K, -1, -1):
        s = 1 << m
        ne = ((nb >> m) + 1) >> 1
        for t in range(ne):
            i = ((2 * t + 1) << m) - 1
            w = BV[i] - BB[i] @ yk
            if i - s >= 0:
                w -= CL[i] @ Y[i - s]
            if i + s < nb:
                w -= XR[i] @ Y[i + s]
            Y[i] = np.linalg.solve(L[i].T, w)
    return np.concatenate([Y.reshape(-1)[:n], yk])


@pytest.mark.parametrize("nac,bc", [(2, 1), (9, 1), (10, 1), (37, 2), (49, 1), (49, 3), (64, 1), (99, 1), (50, 2),
                                    (17, 3)])
def test_band_cr_schedule_solves_the_arrowhead_system(nac, bc):
    S, b = _window(nac, bc, seed=nac * 10 + bc)
    y = band_cr_solve(S, b, nac, bc)
    ref = np.linalg.solve(S, b)
    np.testing.assert_allclose(y, ref, rtol=1e-9, atol=1e-11 * np.abs(ref).max())


def test_band_blocks_are_block_tridiagonal():
    """Blocks of max(camera band, 1) cameras leave no coupling beyond the neighbouring block (what the kernel's
    load phase assumes when it reads only A(j, j - 1))."""
    nac, bc = 31, 3
    S, _ = _window(nac, bc, seed=5)
    G = 6 * bc
    n = 6 * nac
    for j in range(n // G):
        for k in range(j + 2, n // G):
            assert not np.any(S[k * G:(k + 1) * G, j * G:(j + 1) * G])
