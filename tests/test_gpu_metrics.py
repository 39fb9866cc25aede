"""GPU parity of the rollout scoring against the
reference's own evaluation functions, run on the reference's own rollouts
(tests/golden/metrics.npz, made by tests/golden/make_golden.py metrics):

  evaluate_all.compute_metrics (scripts/evaluation/evaluate_all.py:118-159)
  evaluate_multi_ic.evaluate_model_on_ic (evaluate_multi_ic.py:21-94)
  evaluate_long_rollout.evaluate_long_rollout (evaluate_long_rollout.py:18-81)

Tolerances (about 2x the errors measured on MI355X, profiles/r02_*_parity_errors.json):
on the SAME trajectories the device sums in float64 and rounds once where
numpy sums float32 pairwise, so series agree to a few float32 ulps: rtol 2e-6
on MSEs, and on drifts (differences of O(0.05) energies and O(1) charges) 2 ulp
of the underlying value: atol 1.5e-8 (energy), 2.4e-7 (charge).  On the
device's OWN rollouts the f32 state error (<= 1e-5, test_gpu_parity) moves the
per-step MSEs by up to 4e-5 relative (measured), so rtol 1e-4 there, and the
per-IC mean/final MSE (sums over many steps/channels) by 6e-7: rtol 2e-6.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hybrid_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def hf():
    import hybridflux
    from hybridflux import _lib
    assert _lib.lib().hf_device_count() > 0, "GPU tests need a visible HIP device"
    return hybridflux


def _close(name, got, want, atol, rtol, record=None, test=None):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    assert got.shape == want.shape, (name, got.shape, want.shape)
    err = np.abs(got - want)
    rel = err / np.maximum(np.abs(want), 1e-30)
    if record:
        record(test, f"{name}_max_abs", err.max())
        record(test, f"{name}_max_rel", rel[np.abs(want) > 0].max() if (np.abs(want) > 0).any() else 0.0)
    assert (err <= atol + rtol * np.abs(want)).all(), f"{name}: max abs {err.max():.3e}, max rel {rel.max():.3e}"


def test_compute_metrics_on_reference_trajectories(hf, record):
    """evaluation.compute_metrics on the reference's hybrid and classical rollouts
    == the reference's compute_metrics on the same rollouts, key by key."""
    from hybridflux.evaluation import compute_metrics
    m = golden("metrics.npz")
    hyb = torch.as_tensor(golden("hybrid_W1_r1_nx64.npz")["states"], device=DEV)
    cla = torch.as_tensor(golden("classical.npz")["b16_states"], device=DEV)
    got = compute_metrics(hyb, cla)
    assert set(got) == {k[3:] for k in m.files if k.startswith("cm_")}
    for k, v in got.items():
        atol = 2.4e-7 if "charge_drift" in k else 1.5e-8 if "energy_drift" in k else 0.0
        _close(k, v.cpu().numpy(), m[f"cm_{k}"], atol, 2e-6, record, "compute_metrics_on_reference_trajectories")


@pytest.mark.parametrize("precision", ["f32", "f16x3"])
def test_multi_ic_mse_vs_reference(hf, record, precision):
    """The fused hybrid-vs-classical compare (hf_run_compare + hf_rollout_summary)
    on seeds 1000..1015 == evaluate_model_on_ic('hybrid', W1_r1, 1, seed, 30)."""
    from hybridflux.evaluation import multi_ic_mse
    m = golden("metrics.npz")
    solver = hf.HybridSolver(dict(golden("weights_W1_r1.npz")), radius=1, device=DEV, precision=precision)
    ics = solver.baseline.initial_conditions([int(s) for s in m["multi_ic_seeds"]], as_tensor=True)
    mean_mse, r, summ = multi_ic_mse(solver, ics, 30)
    test = f"multi_ic_mse_{precision}"
    _close("mean_mse", mean_mse.cpu().numpy(), m["multi_ic_mse"], 0.0, 2e-6, record, test)
    mse = r["mse"].cpu().numpy()
    for c, k in enumerate(("mse_n", "mse_u", "mse_E")):
        _close(k, mse[..., c], m[f"cm_{k}"], 1e-12, 1e-4, record, test)
    _close("final_mse", summ["final_mse"].cpu().numpy(), m["cm_final_mse"], 0.0, 2e-6, record, test)
    assert (summ["exploded_at"].cpu().numpy() == -1).all()
    assert (summ["actual_steps"].cpu().numpy() == 30).all()
    _close("final_energy_drift", summ["final_energy_drift"].cpu().numpy(), m["cm_final_energy_drift"],
           1.5e-8, 2e-5, record, test)
    _close("final_energy_drift_true", summ["final_energy_drift_true"].cpu().numpy(),
           m["cm_energy_drift_true"][:, -1], 1.5e-8, 2e-5, record, test)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_long_rollout_explosion_vs_reference(hf, record, i):
    """Explosion tracking (evaluate_long_rollout.py:53-66) on the device: the same
    first non-finite step as the reference's step-by-step loop, seed 2000, for
    W1_r1 (300 steps) and W1_r1 with edge_mlp.2.weight scaled x30 / x100."""
    from hybridflux.evaluation import long_rollout
    m = golden("metrics.npz")
    w = dict(golden("weights_W1_r1.npz"))
    w["edge_mlp.2.weight"] = w["edge_mlp.2.weight"] * m[f"long{i}_scale"]
    solver = hf.HybridSolver(w, radius=1, device=DEV)
    T = int(m[f"long{i}_steps"])
    d = long_rollout(solver, solver.baseline.initial_conditions([2000], as_tensor=True), T)
    ex, actual = int(d["exploded_at"].item()), int(d["actual_steps"].item())
    record(f"long_rollout_{i}", "exploded_at", ex)
    record(f"long_rollout_{i}", "exploded_at_reference", int(m[f"long{i}_exploded_at"]))
    assert ex == int(m[f"long{i}_exploded_at"]) and actual == int(m[f"long{i}_actual_steps"])
    assert bool(d["exploded"].item())
    want = m[f"long{i}_energy_drift_pred"][: actual + 1]
    got = d["energy_drift_pred"][0, : actual + 1].cpu().numpy()
    # the state error grows with the instability: compare the first half tightly
    half = actual // 2
    _close("energy_drift_first_half", got[:half], want[:half], 1e-6, 1e-3, record, f"long_rollout_{i}")


def test_summary_fields_exact(hf):
    """hf_rollout_summary field by field on hand-made series (numpy recomputation)."""
    from hybridflux import engine
    rng = np.random.default_rng(3)
    B, T = 5, 9
    met = rng.uniform(0.5, 1.5, (B, T + 1, 4)).astype(np.float32)
    met[..., 2] = 1.0
    met[1, 4:, 2] = 0.0           # explodes at t = 4
    met[2, T, 2] = 0.0            # explodes at the last step
    met[3, 1:, 2] = 0.0           # explodes at t = 1
    mse = rng.uniform(0, 1e-3, (B, T + 1, 3)).astype(np.float32)
    ref = rng.uniform(0.5, 1.5, (B, T + 1, 4)).astype(np.float32)
    t = lambda a: torch.as_tensor(a, device=DEV)  # noqa: E731
    s, dr = engine.rollout_summary(t(met), t(mse), t(ref), drift=True)
    s, dr = s.cpu().numpy(), dr.cpu().numpy()
    ex = np.array([-1, 4, T, 1, -1])
    act = np.where(ex < 0, T, ex - 1)
    assert np.array_equal(s[:, 0], ex) and np.array_equal(s[:, 1], act)
    b = np.arange(B)
    assert np.array_equal(s[:, 2], np.abs(met[b, act, 0] - met[:, 0, 0]))
    assert np.array_equal(s[:, 3], np.abs(met[b, act, 1] - met[:, 0, 1]))
    tot = (mse[..., 0] + mse[..., 1]) + mse[..., 2]
    assert np.array_equal(s[:, 4], tot[:, -1])
    np.testing.assert_allclose(s[:, 5], tot.astype(np.float64).mean(-1), rtol=1e-7)
    assert np.array_equal(s[:, 6], np.abs(ref[:, T, 0] - ref[:, 0, 0]))
    assert np.array_equal(dr[..., 0], np.abs(met[..., 0] - met[:, :1, 0]))
    assert np.array_equal(dr[..., 3], np.abs(ref[..., 1] - ref[:, :1, 1]))
    s2, _ = engine.rollout_summary(t(met[:, :1]))          # T = 0, no MSE, no reference
    s2 = s2.cpu().numpy()
    assert (s2[:, 0] == -1).all() and (s2[:, 1] == 0).all() and (s2[:, 2] == 0).all()
    assert np.isnan(s2[:, 4:]).all()


def test_traj_metrics_vs_oracle(hf):
    """hf_traj_metrics on recorded trajectories == the oracle's float64 series."""
    from hybridflux import engine
    S = golden("hybrid_W1_r2_nx1024.npz")["states"]
    got = engine.traj_metrics(torch.as_tensor(S, device=DEV)).cpu().numpy()
    e, q, f = O.rollout_metrics(S)
    np.testing.assert_allclose(got[..., 0], e, rtol=1e-7)
    np.testing.assert_allclose(got[..., 1], q, rtol=1e-7)
    assert (got[..., 2] == 1).all()


def test_metric_finite_flag_edge_values(hf):
    """The metric series' finite flag and max|n - 1| (hf_traj_metrics; the
    flag is settled from the float64 energy / charge sums, hf_device.h
    MetricAcc) on states holding NaN, +Inf, -Inf, +Inf beside -Inf in one
    channel (charge NaN), and the largest finite floats (sums that must stay
    finite), against np.isfinite(state).all() and the float32 max|n - 1|
    (NaN where the state is not finite), as evaluate_long_rollout.py:53-66
    tests finiteness."""
    from hybridflux import engine
    B, nx = 8, 64
    rng = np.random.default_rng(7)
    st = (1 + 0.1 * rng.standard_normal((B, 2, 3, nx))).astype(np.float32)
    big = np.float32(3.4e38)
    st[0, 1, 0, 5] = np.nan
    st[1, 1, 1, 7] = np.inf
    st[2, 1, 2, 9] = -np.inf
    st[3, 1, 0, 3], st[3, 1, 0, 40] = np.inf, -np.inf
    st[4, 1, 1, :], st[4, 1, 2, :] = big, -big
    st[5, 1, 0, :] = big
    st[6, 1, 1, 11], st[6, 1, 0, 12] = np.nan, np.inf
    got = engine.traj_metrics(torch.as_tensor(st, device=DEV)).cpu().numpy()
    fin = np.isfinite(st).all(axis=(2, 3))
    assert (got[:, :, 2] == fin.astype(np.float32)).all(), (got[:, :, 2], fin)
    dev = np.abs(st[:, :, 0, :] - np.float32(1)).max(axis=2)
    for b in range(B):
        for t in range(2):
            if fin[b, t]:
                assert got[b, t, 3] == dev[b, t], (b, t, got[b, t, 3], dev[b, t])
            else:
                assert np.isnan(got[b, t, 3]), (b, t, got[b, t, 3])
