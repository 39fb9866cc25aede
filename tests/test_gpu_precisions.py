"""GPU parity of the K=32 matrix-core chain kernels.

f16x3 (fp16 hi+lo split, 3 products, f32 accumulate) is held to the SAME
float32 tolerances as the exact-f32 kernels (tests/test_gpu_parity.py):
edge flux atol 2e-6; 30-step rollouts atol 1e-5 + rtol 1e-5.

bf16 (BASELINE config 4: bf16 weights AND activations, f32 accumulate) is
compared with the float32 oracle run on bf16-rounded weights; activations are
additionally rounded to bf16 at every GEMM input, so the stated tolerance is
measured, not derived: edge flux atol 2e-2, 10-step rollout atol 2e-2.
"""
import numpy as np
import pytest
import torch

from conftest import golden, rand_sd
from oracle import hybrid_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def hf():
    import hybridflux
    return hybridflux


def close(a, b, atol, rtol=0.0):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a.astype(np.float64) - b)
    assert np.isfinite(a).all()
    assert (err <= atol + rtol * np.abs(b)).all(), f"max err {err.max():.3e}"
    return float(err.max())


def weights(name):
    return dict(golden(f"weights_{name}.npz"))


@pytest.mark.parametrize("w", ["W0", "W1_r1", "W1_r2", "W1_r3"])
def test_f16x3_flux_every_step(hf, w):
    h = golden(f"hybrid_{w}_nx64.npz")
    m = hf.FluxGNN(4, 128, 4, precision="f16x3")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in weights(w).items()})
    m = m.to(DEV)
    x = hf.BaselineSolver(64, device=DEV).x
    nf, ei = hf.build_chain_graph_batch(h["states"][:, :30].reshape(-1, 3, 64), x, DEV)
    with torch.no_grad():
        fe = m(nf, ei).cpu().numpy().reshape(16, 30, 128)
    close(fe, h["flux_edge"], 2e-6)


@pytest.mark.parametrize("w", ["W1_r1", "W1_r3"])
def test_f16x3_rollout_vs_reference(hf, w):
    h = golden(f"hybrid_{w}_nx64.npz")
    solver = hf.HybridSolver(weights(w), radius=int(w[-1]), device=DEV, precision="f16x3")
    out = solver.run_batch(h["states"][:, 0], 30)
    close(out["traj"].cpu().numpy(), h["states"], 1e-5, 1e-5)


def test_f16x3_nx1024_windowed(hf):
    h = golden("hybrid_W1_r2_nx1024.npz")
    solver = hf.HybridSolver(weights("W1_r2"), radius=2, nx=1024, dt=3.125e-4, device=DEV, precision="f16x3")
    out = solver.run_batch(h["states"][:, 0], 30)
    close(out["traj"].cpu().numpy(), h["states"], 1e-5, 1e-5)


@pytest.mark.parametrize("nx", [7, 16, 32, 48, 100])
def test_f16x3_any_nx(hf, nx):
    w = weights("W1_r3")
    G = O.Grid(nx, dt=5e-3 * min(1.0, nx / 64.0))
    ics = np.stack([O.initial_condition(G, s) for s in (5, 6, 7)])
    want, _ = O.hybrid_run(O.params_from(w), G, ics, 4)
    solver = hf.HybridSolver(w, radius=3, nx=nx, dt=G.dt, device=DEV, precision="f16x3")
    close(solver.run_batch(ics, 4)["traj"].cpu().numpy(), want, 1e-5, 1e-5)


def test_f16x3_step_matches_run_and_is_deterministic(hf):
    h = golden("hybrid_W1_r2_nx64.npz")
    solver = hf.HybridSolver(weights("W1_r2"), radius=2, device=DEV, precision="f16x3")
    st = torch.as_tensor(h["states"][:, 0], device=DEV)
    cur = st
    for _ in range(3):
        cur = solver.step_batch(cur)
    a = solver.run_batch(st, 3, traj=False)["final"]
    b = solver.run_batch(st, 3, traj=False)["final"]
    assert torch.equal(cur, a) and torch.equal(a, b)


@pytest.mark.parametrize("nx", [64, 1024])
def test_bf16_vs_bf16_weight_oracle(hf, nx):
    w = weights("W1_r2")
    wb = O.bf16_weights(w)
    dt = 5e-3 if nx == 64 else 3.125e-4
    G = O.Grid(nx, dt=dt)
    ics = np.stack([O.initial_condition(G, s) for s in (1000, 1001, 1002, 1003)])
    want, fe_want = O.hybrid_run(O.params_from(wb), G, ics, 10)
    solver = hf.HybridSolver(w, radius=2, nx=nx, dt=dt, device=DEV, precision="bf16")
    nf, ei = hf.build_chain_graph_batch(ics, G.x, DEV)
    with torch.no_grad():
        fe = solver.model(nf, ei).cpu().numpy().reshape(4, 2 * nx)
    err_f = close(fe, fe_want[:, 0], 2e-2)
    err_s = close(solver.run_batch(ics, 10)["traj"].cpu().numpy(), want, 2e-2)
    print(f"bf16 nx={nx}: max flux err {err_f:.2e}, 10-step state err {err_s:.2e}")


@pytest.mark.parametrize("layers", [0, 1, 3])
@pytest.mark.parametrize("nx", [16, 48, 64, 100])
def test_bf16_flux_layers_and_nx(hf, layers, nx):
    """The pair-pipelined bf16 core at every layer count it special-cases
    (none, one, several) and every chain-kernel shape: MT = 1, 3, 4 exact and
    the windowed kernel (nx=100); vs the float32 oracle on bf16-rounded weights."""
    sd = rand_sd(layers, 40 + layers)
    G = O.Grid(nx, dt=5e-3)
    ics = np.stack([O.initial_condition(G, s) for s in (11, 12, 13, 14, 15)])
    want = O.hybrid_flux_edge(O.params_from(O.bf16_weights(sd)), G, ics)
    m = hf.FluxGNN(4, 128, layers, precision="bf16")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(DEV)
    nf, ei = hf.build_chain_graph_batch(ics, G.x, DEV)
    with torch.no_grad():
        fe = m(nf, ei).cpu().numpy().reshape(5, 2 * nx)
    err = close(fe, want, 2e-2)
    print(f"bf16 L={layers} nx={nx}: max flux err {err:.2e}")
