"""Training-data generation on the MI355X.

Replaces scripts/training/generate_data.py:12-54, which runs
BaselineSolver.run one IC at a time on the CPU, with ONE batched classical
rollout (hf_run, model=NULL) over every IC.  The output file has the
reference's keys, dtypes and ordering:

  state_t    [N*steps, 3, nx] f32   states 0..steps-1 of IC 0, then IC 1, ...
  flux_t     [N*steps, nx]    f32   F_n = n*u of each of those steps
  state_next [N*steps, 3, nx] f32   states 1..steps
  x          [nx]             f32   cell centres
  dt, dx, nu                        scalars (float64, as np.savez stores Python floats)

ICs are BaselineSolver.initial_condition(seed=ic) for ic = 0..N-1, exactly as
the reference seeds them (generate_data.py:24).
"""
import os

import numpy as np

from .baseline_solver import BaselineSolver


def generate_dataset(nx=64, num_initial_conditions=20, steps_per_ic=30, dt=5e-3, t_end=1.0, nu=1e-3,
                     out_path="data/dataset.npz", device="cuda", seeds=None):
    """Returns (state_t, flux_t, state_next, x, dt, dx, nu) like the reference and
    writes them to `out_path` (skipped when out_path is None)."""
    solver = BaselineSolver(nx=nx, dt=dt, t_end=t_end, nu=nu, device=device)
    seeds = list(range(num_initial_conditions)) if seeds is None else list(seeds)
    ics = solver.initial_conditions(seeds, as_tensor=True)
    r = solver.run_batch(ics, steps_per_ic, traj=True, flux=True)
    traj = r["traj"].cpu().numpy()                     # [N, steps+1, 3, nx]
    N = traj.shape[0]
    state_t = traj[:, :-1].reshape(N * steps_per_ic, 3, nx)
    state_next = traj[:, 1:].reshape(N * steps_per_ic, 3, nx)
    flux_t = r["flux"].cpu().numpy().reshape(N * steps_per_ic, nx)
    x = solver.x.astype(np.float32)
    if out_path is not None:
        d = os.path.dirname(out_path)
        if d:
            os.makedirs(d, exist_ok=True)
        np.savez(out_path, state_t=state_t, flux_t=flux_t, state_next=state_next, x=x, dt=dt, dx=solver.dx, nu=nu)
    return state_t, flux_t, state_next, x, dt, solver.dx, nu
