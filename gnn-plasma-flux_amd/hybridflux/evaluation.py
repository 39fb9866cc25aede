"""Batched, device-side counterparts of the reference's rollout scoring
(SURVEY.md 8f rank 1).  The reference scores one IC at a time on host numpy
trajectories; here B rollouts are scored on the MI355X from the metric
series the rollout kernels write (hf_traj_metrics / hf_traj_mse /
hf_rollout_summary), so a sharded multi-GPU job can gather them.

  compute_metrics(states_pred, states_true)   scripts/evaluation/evaluate_all.py:118-159
  multi_ic_mse(solver, states0, n_steps)      scripts/evaluation/evaluate_multi_ic.py:21-94
  long_rollout(solver, states0, n_steps)      scripts/evaluation/evaluate_long_rollout.py:18-81
"""
import torch

from . import engine

SUMMARY_FIELDS = ("exploded_at", "actual_steps", "final_energy_drift", "final_charge_drift", "final_mse",
                  "mean_mse", "final_energy_drift_true", "final_charge_drift_true")


def summary_dict(summary):
    """[B, HF_NUM_SUMMARY] -> {field: [B] tensor}; exploded_at is -1 where nothing exploded."""
    return {k: summary[:, i] for i, k in enumerate(SUMMARY_FIELDS)}


def compute_metrics(states_pred, states_true):
    """evaluate_all.compute_metrics for B rollouts at once: states_* [B,T+1,3,nx]
    device tensors -> dict of device tensors with the reference's keys, each
    with a leading IC axis ([B,T+1] series, [B] scalars)."""
    mp = engine.traj_metrics(states_pred)
    mt = engine.traj_metrics(states_true)
    mse = engine.traj_mse(states_pred, states_true)
    summ, drift = engine.rollout_summary(mp, mse, mt, drift=True)
    return {
        "mse_n": mse[..., 0], "mse_u": mse[..., 1], "mse_E": mse[..., 2],
        "mse_total": (mse[..., 0] + mse[..., 1]) + mse[..., 2],
        "energy_drift_pred": drift[..., 0], "energy_drift_true": drift[..., 2],
        "charge_drift_pred": drift[..., 1], "charge_drift_true": drift[..., 3],
        "final_mse": summ[:, 4], "mean_mse": summ[:, 5],
        # evaluate_all.py:157-158 read index -1 (= T); the summary's fields 2, 3 stop
        # at the last finite step, which is T unless the rollout exploded
        "final_energy_drift": drift[:, -1, 0], "final_charge_drift": drift[:, -1, 1],
    }


def multi_ic_mse(solver, states0, n_steps):
    """evaluate_model_on_ic('hybrid', ...) for B ICs in one launch: the hybrid
    rollout and the classical BaselineSolver twin from the same states, scored
    per step.  Returns (mean MSE per IC [B] (the reference's return value),
    the compare_batch result, summary dict)."""
    r = solver.compare_batch(states0, n_steps, metrics=True)
    summ, _ = engine.rollout_summary(r["metrics"], r["mse"], r["metrics_classical"])
    d = summary_dict(summ)
    return d["mean_mse"], r, d


def long_rollout(solver, states0, n_steps, drift=True):
    """evaluate_long_rollout for B ICs: one rollout, explosion tracking and the
    energy drift series on the device.  Returns the summary dict plus
    'energy_drift_pred' [B,T+1] (valid up to actual_steps, as the reference
    stops recording there)."""
    r = solver.run_batch(states0, n_steps, traj=False, metrics=True)
    summ, dr = engine.rollout_summary(r["metrics"], drift=drift)
    d = summary_dict(summ)
    d["exploded"] = d["exploded_at"] >= 0
    if dr is not None:
        d["energy_drift_pred"] = dr[..., 0]
    d["metrics"] = r["metrics"]
    return d
