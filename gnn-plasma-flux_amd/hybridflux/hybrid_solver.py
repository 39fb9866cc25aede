"""HybridSolver with the reference's API (src/hybrid_solver.py:11-73).

One step = FluxGNN edge fluxes on the periodic chain -> F = (F_fwd + F_bwd)/2
-> continuity n' = n - dt/dx (F - F_left) -> Burgers u' (no viscosity) + dt E
-> spectral Poisson E'.  On the MI355X the whole step is ONE kernel per IC
wave (chain_rollout_kernel, chain_common.h), and `run` is ONE persistent
kernel for the whole rollout when nx is 16/32/48/64; other nx use the
windowed / super-window chain kernel + the FV/Poisson kernel per step
(fv_poisson.hip).  Nothing crosses PCIe inside a rollout.

`step`/`run` keep the reference's numpy [3,nx] shapes; `step_batch`/`run_batch`
take [B,3,nx] device tensors (batched independent ICs) and return device
tensors.  `radius` is stored and unused, exactly as in the reference
(src/hybrid_solver.py:32): the stencil radius only names the checkpoint.
"""
import math
import os

import numpy as np
import torch

from . import engine
from .baseline_solver import BaselineSolver
from .config import MODEL_CONFIG
from .flux_gnn import FluxGNN


def load_state_dict(model_path):
    """Checkpoint -> state dict without executing anything from the file:
    .pt/.pth via torch.load(weights_only=True), .npz via numpy (no pickle), or
    an in-memory mapping."""
    if isinstance(model_path, dict):
        return {k: torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v
                for k, v in model_path.items()}
    path = os.fspath(model_path)
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as d:
            return {k: torch.from_numpy(d[k].copy()) for k in d.files}
    return torch.load(path, map_location="cpu", weights_only=True)


class HybridSolver:
    def __init__(self, model_path, radius, nx=64, length=2 * math.pi, dt=5e-3, t_end=1.0, device="cuda",
                 precision="f32", poisson="spectral"):
        """precision: chain-kernel arithmetic, "f32" (default, exact float32
        MFMA), "f16x3" (float32-accurate split-fp16 MFMA, ~5x the matrix rate)
        or "bf16" (bf16 weights/activations, BASELINE config 4).
        poisson: "spectral" (default, the reference's operator) or
        "tridiagonal" (opt-in, NOT the reference's: the north star's
        cyclic-reduction solve fused into the same step kernels; engine.Grid)."""
        self.device = torch.device(device)
        self.baseline = BaselineSolver(nx=nx, length=length, dt=dt, t_end=t_end, device=self.device,
                                       poisson=poisson)
        model = FluxGNN(input_dim=MODEL_CONFIG["input_dim"], hidden_dim=MODEL_CONFIG["hidden_dim"],
                        num_layers=MODEL_CONFIG["num_layers"], precision=precision)
        model.load_state_dict(load_state_dict(model_path))
        self.model = model.to(self.device)
        self.model.eval()
        self.radius = radius

    @property
    def grid(self):
        return self.baseline.grid

    def _dm(self):
        return self.model.device_model(self.device)

    def _upload(self, states):
        return self.baseline._upload(states)

    # reference-shaped API --------------------------------------------------------
    def step(self, state):
        out, _, _ = engine.step(self._dm(), self.grid, self._upload(state)[None])
        return out[0].cpu().numpy()

    def run(self, state0, n_steps=40):
        r = engine.run(self._dm(), self.grid, self._upload(state0)[None], n_steps, traj=True)
        return r["traj"][0].cpu().numpy()

    # batched device API ------------------------------------------------------------
    def step_batch(self, states, return_flux=False, metrics=False):
        """states [B,3,nx] -> next states (device).  With return_flux/metrics returns
        (states, F [B,nx], metrics [B,4])."""
        out, F, M = engine.step(self._dm(), self.grid, self._upload(states), flux_face=return_flux,
                                metrics=metrics)
        return (out, F, M) if (return_flux or metrics) else out

    def compare_batch(self, states0, n_steps, metrics=True, out=None, ws=None):
        """Roll B ICs out with this solver AND with the classical BaselineSolver
        (same dt, nu = 1e-3 as BaselineSolver's default) in one launch and score
        them per step.  Returns dict(final, mse [B,T+1,3] for (n,u,E),
        metrics, metrics_classical).  mse.sum(-1).mean(-1) is the per-IC number
        of scripts/evaluation/evaluate_multi_ic.py:88-94."""
        return engine.run_compare(self._dm(), self.grid, self._upload(states0), n_steps, metrics=metrics, out=out,
                                  ws=ws)

    def run_batch(self, states0, n_steps, traj=True, flux=False, metrics=False, out=None, ws=None):
        """Rollout of B ICs: dict(final [B,3,nx], traj [B,T+1,3,nx] | None,
        flux [B,T,nx] | None, metrics [B,T+1,4] | None), all on the device.
        out (may be states0 itself) and ws (engine.workspace) are optional
        preallocated buffers, so a timed loop allocates nothing."""
        return engine.run(self._dm(), self.grid, self._upload(states0), n_steps, traj=traj, flux=flux,
                          metrics=metrics, out=out, ws=ws)
