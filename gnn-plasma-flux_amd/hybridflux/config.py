"""Configuration dictionaries of the reference (src/config.py:9-79), kept with
identical keys and values so code written against the reference reads the
same settings.  Only MODEL_CONFIG is consumed on the hot path
(src/hybrid_solver.py:21-26); STENCIL_RADII is a checkpoint label only — the
graph is always the +-1 chain (src/graph_constructor.py:34-38), so every radius
runs the same kernels with different weights.
"""

DATASET_CONFIG = dict(nx=64, num_initial_conditions=50, steps_per_ic=40, dt=5e-3, t_end=1.0, nu=1e-3)

MODEL_CONFIG = dict(input_dim=4, hidden_dim=128, num_layers=4)

TRAIN_CONFIG = dict(epochs=50, lr=1e-3, device="cuda")

STENCIL_RADII = [1, 2, 3]


def _ablation(name, state, poisson, charge, e_one, e_multi, rollout):
    return dict(name=name, lambda_state=state, lambda_poisson=poisson, lambda_charge=charge,
                lambda_energy_one=e_one, lambda_energy_multi=e_multi, rollout_steps=rollout)


ABLATION_CONFIGS = {
    "baseline": _ablation("Baseline (Flux MSE only)", 0.0, 0.0, 0.0, 0.0, 0.0, 0),
    "physics": _ablation("+Physics (no rollout)", 1.0, 0.1, 0.1, 0.05, 0.0, 0),
    "full": _ablation("+Rollout (full physics + rollout)", 1.0, 0.1, 0.1, 0.05, 0.05, 3),
    "rollout_only": _ablation("Rollout only (no physics losses)", 0.0, 0.0, 0.0, 0.0, 0.05, 3),
}

EVAL_CONFIG = dict(n_steps=100, test_seed=123)
