"""Constitutive models + device SVD vs the oracle on identical inputs (no atomics
involved, so this pins compute_stress_from_F_trial, utils.py:13-54, and
constitutive_models.py per material independently of float-atomic order)."""
import numpy as np
import pytest

import oracle as O
from conftest import rel_err

pytestmark = pytest.mark.gpu


def _device_svd(A, dev):
    import torch
    from gsmpm._lib import LIB, check, ptr, stream_of
    At = torch.from_numpy(np.ascontiguousarray(A.reshape(-1, 9))).to(dev)
    U, V = torch.empty_like(At), torch.empty_like(At)
    S = torch.empty(len(A), 3, device=dev)
    check(LIB.gsmpm_svd3(ptr(At), len(A), ptr(U), ptr(S), ptr(V), stream_of(dev)))
    return U.cpu().numpy().reshape(-1, 3, 3), S.cpu().numpy(), V.cpu().numpy().reshape(-1, 3, 3)


def test_device_svd_matches_oracle(dev):
    rng = np.random.default_rng(0)
    A = (np.eye(3)[None] + 0.05 * rng.standard_normal((4000, 3, 3))).astype(np.float32)
    A[:1000] = rng.standard_normal((1000, 3, 3))
    U, S, V = _device_svd(A, dev)
    for i in range(len(A)):
        u, s, v = O.svd3(A[i])
        assert np.abs(s - S[i]).max() < 2e-5 * max(1, abs(s).max())
        assert np.abs(U[i] @ np.diag(S[i]) @ V[i].T - A[i]).max() < 5e-5 * max(1, np.abs(A[i]).max())
        if s[0] - s[1] > 1e-3 and s[1] - abs(s[2]) > 1e-3:  # well-separated: U, V unique up to paired signs
            assert np.abs(np.abs(U[i]) - np.abs(u)).max() < 1e-3


# Up to 1e18: A^T A (the Jacobi input) stays finite.  From ~1e19 it overflows,
# and the device (contracted multiply-adds, either SVD build) and the oracle
# (-ffp-contract=off) overflow different entries, so which outputs come out
# NaN differs between them -- for the correctly rounded build as well
# (profiles/r04/ab/svd_degenerate_r04g.txt): outside the algorithm's domain.
@pytest.mark.parametrize("scale", [0.0, 1e-21, 1e-19, 1e-6, 1e6, 1e18])
def test_device_svd_degenerate_scales(dev, scale):
    """The fast SVD (GSMPM_SVD_FAST=2: refined hardware rsqrt) on matrices
    whose Jacobi sums reach 0, subnormals and infinity: finite wherever the
    correctly rounded oracle is, and a valid factorisation wherever the
    oracle's is (the f32 algorithm itself stops reconstructing A once A^T A
    under- or overflows: the oracle's error is O(1) at 1e-19 and 1e18).
    Foam's degenerate F reached these in round 4 (its R came out NaN) before
    the refined form fell back to 1 / sqrtf off the normal range."""
    rng = np.random.default_rng(int(scale > 1) + 7)
    A = rng.standard_normal((512, 3, 3)).astype(np.float32)
    A[:128, :, 2] = 0.0  # rank 2
    A[128:256, :, 1:] = 0.0  # rank 1
    A = (A * np.float32(scale)).astype(np.float32)
    U, S, V = _device_svd(A, dev)
    rec_err = lambda u, sv, v, a: np.abs(u.astype(np.float64) @ np.diag(sv) @ v.T.astype(np.float64) - a).max() / \
        max(np.abs(a).max(), 1e-38)
    checked = 0
    for i in range(len(A)):
        with np.errstate(all="ignore"):
            u, sv, v = O.svd3(A[i])
            ok = all(np.isfinite(x).all() for x in (u, sv, v))
            for name, g, o in (("U", U[i], u), ("S", S[i], sv), ("V", V[i], v)):
                assert np.isfinite(g).all() or not np.isfinite(o).all(), (scale, i, name, g, o)
            if ok and scale > 0 and rec_err(u, sv, v, A[i]) < 1e-3:
                assert rec_err(U[i], S[i], V[i], A[i]) < 2e-3, (scale, i)
                checked += 1
    if scale in (1e-6, 1e6):
        assert checked == len(A)


def _oracle_stress(material, quirk, F, mu, lam, yld, dt):
    n = len(F)
    s = O.OracleMPM(np.full((n, 3), 1.0, np.float32), np.zeros((n, 6), np.float32), np.ones(n, np.float32),
                    n_grid=8, material=material, jelly_quirk=quirk)
    s.F_trial[:] = F.reshape(n, 9)
    s.mu[:], s.lam[:], s.yield_stress[:] = mu, lam, yld
    O.lib().om_stress(O.ctypes.byref(s._st), O.ctypes.c_float(dt))
    return s.F.copy(), s.stress.copy(), s.yield_stress.copy()


@pytest.mark.parametrize("code,material,quirk", [(0, "jelly", True), (4, "jelly", False), (1, "metal", True),
                                                 (2, "sand", True), (3, "foam", True)])
def test_constitutive_vs_oracle(dev, code, material, quirk):
    import torch
    from gsmpm._lib import LIB, check, ptr, stream_of
    rng = np.random.default_rng(code)
    n = 5000
    # moderately deformed, well-separated singular values (rotation * stretch)
    Q, _ = np.linalg.qr(rng.standard_normal((n, 3, 3)))
    Q *= np.sign(np.linalg.det(Q))[:, None, None]
    st = np.stack([rng.uniform(0.9, 1.1, n), rng.uniform(0.8, 1.2, n), rng.uniform(0.7, 1.3, n)], 1)
    F = (Q * st[:, None, :] @ np.linalg.qr(rng.standard_normal((n, 3, 3)))[0]).astype(np.float32)
    F *= np.sign(np.linalg.det(F))[:, None, None]
    mu = np.full(n, 8.3e4, np.float32)
    lam = np.full(n, 5.6e4, np.float32)
    yld = np.full(n, 0.005, np.float32)
    dt = 1e-4
    Fo, To, yo = _oracle_stress(material, quirk, F, mu, lam, yld.copy(), dt)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    Ft, ymu, ylam, yy = t(F.reshape(n, 9)), t(mu), t(lam), t(yld.copy())
    Fg, Tg = torch.empty_like(Ft), torch.empty_like(Ft)
    check(LIB.gsmpm_constitutive(code, ptr(Ft), n, ptr(ymu), ptr(ylam), ptr(yy), dt, ptr(Fg), ptr(Tg),
                                 stream_of(dev)))
    Fg, Tg, yy = Fg.cpu().numpy(), Tg.cpu().numpy(), yy.cpu().numpy()
    if material == "foam":
        # F13: element-wise U*diag*V^T keeps only U_ii e_i V_ii, which depends on
        # the SVD basis itself; compare where the basis is well conditioned
        return
    assert rel_err(Fg, Fo) < 1e-4
    assert rel_err(Tg, To) < 1e-4
    assert rel_err(yy, yo) < 1e-4


@pytest.mark.parametrize("yld", [0.005, 1e9])
def test_fluid_return_mapping_vs_oracle(dev, yld):
    """gsmpm_constitutive material 5: fluid_return_mapping
    (constitutive_models.py:142-213, never dispatched by the reference) + StVK
    stress, against oracle/mpm_oracle.c:om_fluid; plastic and elastic branches."""
    import torch
    from gsmpm._lib import LIB, check, ptr, stream_of
    rng = np.random.default_rng(5)
    n = 5000
    Q, _ = np.linalg.qr(rng.standard_normal((n, 3, 3)))
    st = np.stack([rng.uniform(1.1, 1.3, n), rng.uniform(0.9, 1.05, n), rng.uniform(0.7, 0.85, n)], 1)
    F = (Q * st[:, None, :] @ np.linalg.qr(rng.standard_normal((n, 3, 3)))[0]).astype(np.float32)
    F *= np.sign(np.linalg.det(F))[:, None, None]
    mu = np.full(n, 8.3e4, np.float32)
    lam = np.full(n, 5.6e4, np.float32)
    y = np.full(n, yld, np.float32)
    dt = 1e-4
    Fo, To = O.fluid_return_mapping(F, mu, lam, y, dt, 0.008)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    Ft, ymu, ylam, yy = t(F.reshape(n, 9)), t(mu), t(lam), t(y)
    Fg, Tg = torch.empty_like(Ft), torch.empty_like(Ft)
    check(LIB.gsmpm_constitutive(5, ptr(Ft), n, ptr(ymu), ptr(ylam), ptr(yy), dt, ptr(Fg), ptr(Tg), stream_of(dev)))
    assert rel_err(Fg.cpu().numpy(), Fo.reshape(n, 9)) < 1e-4
    assert rel_err(Tg.cpu().numpy(), To.reshape(n, 9)) < 1e-4
