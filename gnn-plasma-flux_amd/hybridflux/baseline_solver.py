"""BaselineSolver with the reference's API (src/baseline_solver.py:6-118); the
classical step, rollout and Poisson solve run on the MI355X.

1-D fluid–Poisson model:
    dn/dt + d(nu)/dx = 0
    du/dt + d(u^2/2)/dx = E + nu d^2u/dx^2
    E from the spectral solve of the reference (src/baseline_solver.py:59-68),
    which satisfies dE/dx = -(n - 1 - mean(n - 1)); poisson="tridiagonal"
    selects the opt-in cyclic-reduction solve of the same equation's
    second-order potential form instead (NOT the reference's operator; see
    engine.Grid).

Single-IC methods keep the reference's numpy-in / numpy-out shape; the
`*_batch` methods take [B,3,nx] torch tensors already on the device (or numpy,
which is uploaded) and return device tensors.
"""
import math

import numpy as np
import torch

from . import engine


class BaselineSolver:
    def __init__(self, nx=64, length=2 * math.pi, dt=5e-3, t_end=1.0, nu=1e-3, device="cuda", poisson="spectral"):
        self.nx = nx
        self.length = length
        self.dx = length / nx
        self.dt = dt
        self.t_end = t_end
        self.n0 = 1.0
        self.nu = nu
        self.device = torch.device(device)
        self.grid = engine.Grid(nx, length, dt, nu, poisson=poisson)
        self.poisson = poisson
        self.x = self.grid.x
        self.k = 2.0 * np.pi * np.fft.fftfreq(nx, d=self.dx)
        if self.dt / self.dx > 0.5:  # src/baseline_solver.py:23-24
            print("Warning: dt/dx may be large; consider reducing dt for stability.")

    # -- initial conditions (host RNG, device Poisson) ---------------------------
    def _modes(self, seed):
        """n, u of src/baseline_solver.py:35-51 — MT19937 RandomState, same draws."""
        rs = np.random.RandomState(seed)
        n = np.full(self.nx, self.n0, dtype=np.float32)
        for _ in range(rs.randint(3, 6)):
            km = rs.randint(1, 6)
            amp = 0.15 + 0.15 * rs.rand()
            ph = 2 * np.pi * rs.rand()
            n += amp * np.sin(km * self.x + ph).astype(np.float32)
        u = np.zeros(self.nx, dtype=np.float32)
        for _ in range(2):
            km = rs.randint(1, 6)
            amp = 0.1 + 0.1 * rs.rand()
            ph = 2 * np.pi * rs.rand()
            u += amp * np.cos(km * self.x + ph).astype(np.float32)
        u += 0.05 * rs.randn(self.nx).astype(np.float32)
        return n, u

    def initial_condition(self, seed=None):
        return self.initial_conditions([seed])[0]

    def initial_conditions(self, seeds, as_tensor=False):
        """Batched ICs for a list of seeds -> [B,3,nx] (numpy, or a device tensor)."""
        nu = [self._modes(s) for s in seeds]
        if not nu:  # an empty shard (an IC-sharded job with more ranks than ICs)
            st = torch.zeros(0, 3, self.nx, dtype=torch.float32, device=self.device)
            return st if as_tensor else st.cpu().numpy()
        n = torch.as_tensor(np.stack([a for a, _ in nu]), device=self.device)
        u = torch.as_tensor(np.stack([b for _, b in nu]), device=self.device)
        st = torch.stack([n, u, engine.poisson(self.grid, n)], dim=1).contiguous()
        return st if as_tensor else st.cpu().numpy()

    # -- Poisson -------------------------------------------------------------------
    def solve_poisson(self, n):
        if isinstance(n, torch.Tensor):
            return engine.poisson(self.grid, n.reshape(-1, self.nx)).reshape(n.shape)
        n = np.asarray(n, dtype=np.float32)
        E = engine.poisson(self.grid, torch.as_tensor(n.reshape(-1, self.nx), device=self.device))
        return E.cpu().numpy().reshape(n.shape)

    # -- host helpers kept for API parity (not on the hot path) ---------------------
    def compute_flux_n(self, n, u):
        return (n * u).astype(np.float32)

    def compute_flux_u(self, u):
        return (0.5 * u * u).astype(np.float32)

    def laplacian_u(self, u):
        return (np.roll(u, -1) - 2 * u + np.roll(u, 1)) / (self.dx ** 2)

    # -- stepping --------------------------------------------------------------------
    def _upload(self, states):
        if isinstance(states, torch.Tensor):
            return states.to(self.device, torch.float32)
        return torch.as_tensor(np.ascontiguousarray(states, dtype=np.float32), device=self.device)

    def step(self, state, return_flux=False):
        out, F, _ = engine.step(None, self.grid, self._upload(state)[None], flux_face=return_flux)
        if return_flux:
            return out[0].cpu().numpy(), F[0].cpu().numpy()
        return out[0].cpu().numpy()

    def run(self, state0, n_steps=10, record_flux=True):
        r = engine.run(None, self.grid, self._upload(state0)[None], n_steps, traj=True, flux=record_flux)
        states = r["traj"][0].cpu().numpy()
        return states, (r["flux"][0].cpu().numpy() if record_flux else None)

    def step_batch(self, states, return_flux=False, metrics=False):
        out, F, M = engine.step(None, self.grid, self._upload(states), flux_face=return_flux, metrics=metrics)
        return (out, F, M) if (return_flux or metrics) else out

    def run_batch(self, states0, n_steps, traj=True, flux=False, metrics=False):
        return engine.run(None, self.grid, self._upload(states0), n_steps, traj=traj, flux=flux, metrics=metrics)
