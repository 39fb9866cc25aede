"""The opt-in tridiagonal Poisson mode (HF_POISSON_TRIDIAG) on the CPU: the
kernels' cyclic-reduction algorithm, modelled in numpy operation for
operation (csrc/hf_device.h tridiag_psi_wave / tri_E), against the oracle's
dense float64 solve of the same discrete periodic system and against its
exact Fourier-symbol form; the plan helpers of the ABI.

This mode is NOT the reference's operator (src/baseline_solver.py:59-68 is
spectral) and claims no parity with the reference; the reference has no
tridiagonal solve, so there is nothing of it to pin to ("parity unpinned"):
the dense solve of the stated system is the checker.
"""
import ctypes

import numpy as np
import pytest

from oracle import hybrid_oracle as O


def cr_model(rho, h):
    """tridiag_psi_wave + tri_E in numpy, per row (the same level order and
    expressions; float64; float32 out)."""
    x = np.asarray(rho, np.float64).copy()
    n = x.shape[-1]
    x -= x.sum(-1, keepdims=True) * (1.0 / n)
    s = 1
    while n % (2 * s) == 0:                                  # forward reduction
        i = np.arange(0, n, 2 * s)
        x[..., i] = (x[..., (i - s) % n] + x[..., i + s]) + x[..., i] * 2.0
        s *= 2
    R = n // s                                               # odd survivors: Thomas, psi[0] = 0
    dp = np.zeros(x.shape[:-1])
    for j in range(1, R):
        dp = (x[..., j * s] - dp) * (-j / (j + 1))
        x[..., j * s] = dp
    p = np.zeros(x.shape[:-1])
    for j in range(R - 1, 0, -1):
        p = x[..., j * s] + p * (j / (j + 1))
        x[..., j * s] = p
    x[..., 0] = 0.0
    s //= 2
    while s >= 1:                                            # back-substitution
        i = np.arange(s, n, 2 * s)
        x[..., i] = ((x[..., i - s] + x[..., (i + s) % n]) - x[..., i]) * 0.5
        s //= 2
    return (h * (np.roll(x, 1, -1) - np.roll(x, -1, -1))).astype(np.float32)


def densities(nx, B=4, seed=0):
    g = np.random.default_rng(seed)
    x = np.arange(nx) * 2 * np.pi / nx
    return (1 + 0.3 * np.sin(3 * x + 1) + 0.05 * g.standard_normal((B, nx))).astype(np.float32)


@pytest.mark.parametrize("nx", [1, 2, 3, 5, 13, 16, 32, 48, 64, 100, 256, 1000, 1024, 2048])
def test_cyclic_reduction_matches_dense_solve(nx):
    """Power-of-two nx (pure cyclic reduction), nx = 48 / 100 / 1000 (reduction
    levels, then the Thomas step on 3 / 25 / 125 survivors) and odd nx (Thomas
    only): the kernels' algorithm equals the dense solve to float32 rounding."""
    G = O.Grid(nx, poisson="tridiagonal")
    n = densities(nx)
    got = cr_model(n - 1.0, 0.5 * G.dx)
    want = O.solve_poisson_tridiag(G, n)
    assert np.abs(got - want).max() <= 1e-7


@pytest.mark.parametrize("nx", [16, 64, 1024, 2048])
def test_dense_and_symbol_forms_agree(nx):
    G = O.Grid(nx, poisson="tridiagonal")
    n = densities(nx, seed=1)
    assert np.abs(O.tridiag_symbol_solve(G, n) - O.solve_poisson_tridiag(G, n)).max() <= 1e-7


def test_discrete_equation_holds():
    """The oracle's E is the stated system's: a least-squares potential of the
    singular Laplacian satisfies the stencil, and its central difference is E."""
    nx = 64
    G = O.Grid(nx, poisson="tridiagonal")
    n = densities(nx, B=1)[0].astype(np.float64)
    rho = n - 1.0
    L = -2.0 * np.eye(nx) + np.roll(np.eye(nx), 1, 1) + np.roll(np.eye(nx), -1, 1)
    phi = np.linalg.lstsq(L, (rho - rho.mean()) * G.dx ** 2, rcond=None)[0]
    assert np.abs(L @ phi / G.dx ** 2 - (rho - rho.mean())).max() < 1e-10
    E = -(np.roll(phi, -1) - np.roll(phi, 1)) / (2 * G.dx)
    assert np.abs(O.solve_poisson_tridiag(G, n[None].astype(np.float32))[0] - E).max() < 1e-7


@pytest.mark.parametrize("nx,lo,hi", [(16, 5e-3, 5e-2), (64, 5e-4, 5e-3), (1024, 1e-6, 5e-5)])
def test_deviation_from_spectral_is_second_order(nx, lo, hi):
    """On the reference's ICs (seeds 1000..1015) the mode differs from the
    spectral E by O(dx^2): 1.85e-3 at nx = 64 (SURVEY.md §0 measured 1.1e-3 for a
    2nd-order solve), shrinking 16x per 4x refinement."""
    G, Gt = O.Grid(nx), O.Grid(nx, poisson="tridiagonal")
    n = np.stack([O.initial_condition(G, s)[0] for s in range(1000, 1016)])
    dev = np.abs(O.solve_poisson(Gt, n) - O.solve_poisson(G, n)).max()
    assert lo < dev < hi, dev


def test_plan_abi():
    from hybridflux import _lib
    lib = _lib.lib()
    assert lib.hf_poisson_plan_size(_lib.HF_POISSON_TRIDIAG, 64) == 1
    assert lib.hf_poisson_plan_size(_lib.HF_POISSON_SPECTRAL, 1024) == lib.hf_poisson_plan_len(1024)
    assert lib.hf_poisson_plan_size(_lib.HF_POISSON_TRIDIAG, 16385) == -1
    assert lib.hf_poisson_plan_size(7, 64) == -1
    plan = np.zeros(1)
    _lib.check(lib.hf_poisson_plan(_lib.HF_POISSON_TRIDIAG, 64, 2 * np.pi, plan.ctypes.data_as(ctypes.c_void_p)))
    assert plan[0] == 0.5 * (2 * np.pi / 64)
    spec = np.zeros(lib.hf_poisson_plan_len(64))
    ref = np.zeros_like(spec)
    _lib.check(lib.hf_poisson_plan(_lib.HF_POISSON_SPECTRAL, 64, 2 * np.pi, spec.ctypes.data_as(ctypes.c_void_p)))
    _lib.check(lib.hf_poisson_coeffs(64, 2 * np.pi, ref.ctypes.data_as(ctypes.c_void_p)))
    assert np.array_equal(spec, ref)
    assert lib.hf_poisson_plan(5, 64, 1.0, plan.ctypes.data_as(ctypes.c_void_p)) == _lib.HF_EINVAL
    assert lib.hf_poisson_plan(_lib.HF_POISSON_TRIDIAG, 20000, 1.0,
                               plan.ctypes.data_as(ctypes.c_void_p)) == _lib.HF_EUNSUPPORTED


def test_mode_arguments_checked_before_any_device_work():
    """An unknown mode, or the tridiagonal mode past its LDS limit, fails with
    the ABI's codes (B = 0: no device needed)."""
    from hybridflux import _lib
    lib = _lib.lib()
    assert lib.hf_run_ex(None, None, None, None, None, 9, 0, 64, 1, 0.1, 0.1, 0.0, 1.0, None, None, None, None, 0,
                         None) == _lib.HF_EINVAL
    assert lib.hf_step_ex(None, None, None, None, None, _lib.HF_POISSON_TRIDIAG, 0, 20000, 0.1, 0.1, 0.0, 1.0,
                          None, None, None, 0, None) == _lib.HF_EUNSUPPORTED
    assert lib.hf_poisson_ex(None, 64, None, 64, None, 3, 0, 64, None) == _lib.HF_EINVAL


def test_grid_modes():
    from hybridflux import engine
    with pytest.raises(ValueError):
        engine.Grid(64, poisson="chebyshev")
    g = engine.Grid(64, poisson="tridiagonal")
    assert g.plan.shape == (1,) and g.poisson_c.shape == (64,)   # the loss keeps the spectral plan
    s = engine.Grid(64)
    assert s.plan is s.poisson_c and s.pmode == 0 and g.pmode == 1
