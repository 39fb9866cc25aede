"""Pins the CPU oracle (oracle/hybrid_oracle.py) to the golden vectors that
tests/golden/make_golden.py produced by running the reference itself.
Every comparison here is bit-exact."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hybrid_oracle as O

WEIGHTS = ["W0", "W1_r1", "W1_r2", "W1_r3"]


def test_initial_conditions_bitwise():
    g = golden("ics.npz")
    G = O.Grid(64)
    got = np.stack([O.initial_condition(G, int(s)) for s in g["seeds_nx64"]])
    assert np.array_equal(got, g["ics_nx64"])
    G1k = O.Grid(1024, dt=3.125e-4)
    got = np.stack([O.initial_condition(G1k, int(s)) for s in g["seeds_nx1024"]])
    assert np.array_equal(got, g["ics_nx1024"])
    assert np.array_equal(G.x, g["x_nx64"]) and np.array_equal(G1k.x, g["x_nx1024"])


@pytest.mark.parametrize("nx", [16, 32, 48, 64, 1024])
def test_poisson_bitwise(nx):
    g = golden("poisson.npz")
    assert np.array_equal(O.solve_poisson(O.Grid(nx), g[f"n_nx{nx}"]), g[f"E_nx{nx}"])


def test_classical_bitwise():
    g = golden("classical.npz")
    S, F = O.classical_run(O.Grid(64), g["seed0_states"][0], 30)
    assert np.array_equal(S, g["seed0_states"]) and np.array_equal(F, g["seed0_fluxes"])
    S, F = O.classical_run(O.Grid(64), g["b16_states"][:, 0], 30)
    assert np.array_equal(S, g["b16_states"]) and np.array_equal(F, g["b16_fluxes"])
    S, F = O.classical_run(O.Grid(1024, dt=3.125e-4), g["nx1024_states"][:, 0], 30)
    assert np.array_equal(S, g["nx1024_states"]) and np.array_equal(F, g["nx1024_fluxes"])


@pytest.mark.parametrize("w", WEIGHTS)
def test_hybrid_rollout_bitwise(w):
    p = O.params_from(dict(golden(f"weights_{w}.npz")))
    h = golden(f"hybrid_{w}_nx64.npz")
    S, FE = O.hybrid_run(p, O.Grid(64), h["states"][:, 0], 30)
    assert np.array_equal(S, h["states"])
    assert np.array_equal(FE, h["flux_edge"])


def test_hybrid_per_ic_bitwise():
    p = O.params_from(dict(golden("weights_W1_r1.npz")))
    h = golden("hybrid_W1_r1_nx64.npz")
    S = O.hybrid_run_per_ic(p, O.Grid(64), h["states"][:3, 0], 30)
    assert np.array_equal(S, h["states"][:3])


def test_hybrid_nx1024_first_steps():
    p = O.params_from(dict(golden("weights_W1_r2.npz")))
    h = golden("hybrid_W1_r2_nx1024.npz")
    S, FE = O.hybrid_run(p, O.Grid(1024, dt=3.125e-4), h["states"][:2, 0], 4)
    assert np.array_equal(S, h["states"][:2, :5])
    assert np.array_equal(FE, h["flux_edge"][:2])


def test_random_graph_forward():
    g = golden("fluxgnn_random.npz")
    small = O.params_from({k[len("small."):]: g[k] for k in g.files if k.startswith("small.")})
    import torch
    got = O.flux_gnn_forward(small, torch.from_numpy(g["small_nf"]), torch.from_numpy(g["small_ei"]))
    assert np.array_equal(got.detach().numpy(), g["small_flux"])
    big = O.params_from(dict(golden("weights_W0.npz")))
    got = O.flux_gnn_forward(big, torch.from_numpy(g["big_nf"]), torch.from_numpy(g["big_ei"]))
    assert np.array_equal(got.detach().numpy(), g["big_flux"])


# ------------------------------------------------------------------ gradients
def _grads_close(got, want, rel=1e-5):
    scale = float(np.abs(want).max()) or 1.0
    assert np.abs(got - want).max() <= rel * scale + 1e-12, (np.abs(got - want).max(), scale)


@pytest.mark.parametrize("tag", ["small", "big"])
def test_oracle_backward_random_graph_vs_reference(tag):
    """Autograd through the oracle forward == the reference FluxGNN's autograd."""
    g = golden("grads.npz")
    rnd = golden("fluxgnn_random.npz")
    if tag == "small":
        sd = {k[6:]: rnd[k] for k in rnd.files if k.startswith("small.")}
    else:
        w0 = golden("weights_W0.npz")
        sd = {k: w0[k] for k in w0.files}
    p = {k: v.clone().requires_grad_(True) for k, v in O.params_from(sd).items()}
    nf = torch.from_numpy(rnd[f"{tag}_nf"]).clone().requires_grad_(True)
    flux = O.flux_gnn_forward(p, nf, torch.from_numpy(rnd[f"{tag}_ei"]))
    (flux * torch.from_numpy(g[f"{tag}_g"])).sum().backward()
    _grads_close(nf.grad.numpy(), g[f"{tag}_grad_nf"])
    for k, v in p.items():
        _grads_close(v.grad.numpy(), g[f"{tag}_grad.{k}"])


def test_oracle_ablation_loss_vs_reference():
    """oracle.ablation_loss == scripts/training/train_ablation.py's loss ('full'
    config) and its parameter gradients, on the three golden samples."""
    from hybridflux.config import ABLATION_CONFIGS
    g = golden("grads.npz")
    cl = golden("classical.npz")
    w1 = golden("weights_W1_r1.npz")
    grid = O.Grid(64)
    for j, (ic, t) in enumerate(g["loss_picks"]):
        p = {k: v.clone().requires_grad_(True) for k, v in O.params_from({k: w1[k] for k in w1.files}).items()}
        S, F = cl["b16_states"], cl["b16_fluxes"]
        loss, fl = O.ablation_loss(p, grid, S[ic, t], F[ic, t], S[ic, t + 1], ABLATION_CONFIGS["full"])
        loss.backward()
        assert abs(loss.item() - float(g[f"loss{j}_value"])) <= 1e-6 * abs(float(g[f"loss{j}_value"]))
        assert abs(fl.item() - float(g[f"loss{j}_flux"])) <= 1e-6 * abs(float(g[f"loss{j}_flux"]))
        for k, v in p.items():
            _grads_close(v.grad.numpy(), g[f"loss{j}_grad.{k}"])


# ------------------------------------------------------------ PureGNN / PINN
def _sub(d, prefix):
    return O.params_from({k[len(prefix):]: d[k] for k in d.files if k.startswith(prefix)})


def test_oracle_pure_gnn_and_pinn_vs_reference():
    """Oracle restatements of PureGNN / PINN == the reference classes' outputs
    (rollouts of evaluate_multi_ic.py:45-83, a random graph, a batched PINN call)."""
    b = golden("baselines.npz")
    grid = O.Grid(64)
    pg, pn = _sub(b, "pure_gnn."), _sub(b, "pinn.")
    with torch.no_grad():
        d = O.pure_gnn_forward(pg, torch.from_numpy(b["pure_gnn_graph_nf"]), torch.from_numpy(b["pure_gnn_graph_ei"]))
        np.testing.assert_allclose(d.numpy(), b["pure_gnn_graph_delta"], atol=2e-6, rtol=1e-5)
        out = O.pinn_forward(pn, torch.from_numpy(b["ics"][:3]))
        np.testing.assert_allclose(out.numpy(), b["pinn_batch_out"], atol=2e-6, rtol=1e-5)
        for j, ic in enumerate(b["ics"]):
            np.testing.assert_allclose(O.pure_gnn_rollout(pg, grid, ic, 10), b["pure_gnn_traj"][j], atol=1e-5, rtol=1e-5)
            s = torch.from_numpy(ic)
            traj = [ic]
            for _ in range(10):
                s = O.pinn_forward(pn, s[None])[0]
                traj.append(s.numpy())
            np.testing.assert_allclose(np.array(traj), b["pinn_traj"][j], atol=1e-5, rtol=1e-5)


# ------------------------------------------------------------ rollout scoring (8f rank 1)
def test_oracle_compute_metrics_vs_reference():
    """oracle.compute_metrics == the reference's evaluate_all.compute_metrics
    (scripts/evaluation/evaluate_all.py:118-159) on its own hybrid-vs-classical
    rollouts, key by key, bit for bit (same float32 numpy arithmetic)."""
    m = golden("metrics.npz")
    hyb, cla = golden("hybrid_W1_r1_nx64.npz"), golden("classical.npz")
    got = O.compute_metrics(hyb["states"], cla["b16_states"])
    for k, v in got.items():
        np.testing.assert_array_equal(np.asarray(v, np.float64), m[f"cm_{k}"], err_msg=k)


def test_oracle_multi_ic_mse_vs_reference():
    """mean over t of mse_total (scripts/evaluation/evaluate_multi_ic.py:88-94) from
    the oracle's hybrid and classical rollouts == evaluate_model_on_ic('hybrid', ...)."""
    m = golden("metrics.npz")
    w = golden("weights_W1_r1.npz")
    grid = O.Grid(64)
    ics = np.stack([O.initial_condition(grid, int(s)) for s in m["multi_ic_seeds"]])
    S, _ = O.hybrid_run(O.params_from({k: w[k] for k in w.files}), grid, ics, 30)
    C = np.stack([O.classical_run(grid, ic, 30)[0] for ic in ics])
    got = O.compute_metrics(S, C)["mean_mse"]
    np.testing.assert_allclose(got, m["multi_ic_mse"], rtol=1e-6, atol=0)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_oracle_long_rollout_explosion_vs_reference(i):
    """Explosion tracking of scripts/evaluation/evaluate_long_rollout.py:18-81 (seed
    2000; W1_r1 and W1_r1 with edge_mlp.2.weight scaled): the oracle finds the same
    first non-finite step and the same energy-drift series."""
    m = golden("metrics.npz")
    w = {k: v for k, v in golden("weights_W1_r1.npz").items()}
    w["edge_mlp.2.weight"] = w["edge_mlp.2.weight"] * m[f"long{i}_scale"]
    grid = O.Grid(64)
    ex, actual, drift = O.long_rollout(O.params_from(w), grid, O.initial_condition(grid, 2000),
                                       int(m[f"long{i}_steps"]))
    assert (-1 if ex is None else ex) == int(m[f"long{i}_exploded_at"])
    assert actual == int(m[f"long{i}_actual_steps"])
    want = m[f"long{i}_energy_drift_pred"][: actual + 1]
    np.testing.assert_array_equal(drift, want)


def test_bf16_emulation_structure():
    """oracle.hybrid_flux_edge_bf16 without its activation rounding is the float32
    forward on bf16-rounded weights (same edge order, P/Q split, halved W_b,
    aggregation): pins the emulation the bf16 kernels are held to."""
    w = dict(golden("weights_W1_r2.npz"))
    grid = O.Grid(64)
    ics = np.stack([O.initial_condition(grid, s) for s in (1000, 1001, 1002)])
    pb = O.params_from(O.bf16_weights(w))
    want = O.hybrid_flux_edge(pb, grid, ics)
    got = O.hybrid_flux_edge_bf16(O.params_from(w), grid, ics, act_round=lambda a: a)
    np.testing.assert_allclose(got, want, atol=2e-6, rtol=0)
    full = O.hybrid_flux_edge_bf16(O.params_from(w), grid, ics)
    assert 1e-4 < np.abs(full - want).max() < 1e-2   # the activation rounding is what differs


def test_bf16_fixture_reproducible():
    """tests/golden/bf16_nx1024.npz (made by make_oracle_vectors.py) is the
    oracle's current output (first-step fluxes and one step)."""
    g = golden("bf16_nx1024.npz")
    w = dict(golden("weights_W1_r2.npz"))
    G = O.Grid(1024, dt=3.125e-4)
    ics = g["states_emul"][:, 0]
    fe = O.hybrid_flux_edge_bf16(O.params_from(w), G, ics)
    np.testing.assert_array_equal(fe, g["flux_edge0_emul"])
    s1, _ = O.hybrid_step(O.params_from(w), G, ics, O.hybrid_flux_edge_bf16)
    np.testing.assert_array_equal(s1, g["states_emul"][:, 1])
