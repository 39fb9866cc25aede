"""FluxGNN training on the MI355X (differentiable hybrid step).

Mirrors scripts/training/train_ablation.py (FluxDataset, train_model and the
per-sample ablation loss of :107-200).  FluxGNN's forward and backward run in
the HIP training kernels through FluxGNN's autograd Function (on tagged
chains the chain-layout MFMA GEMMs of train_chain.hip / tgemm.h, on other
graphs the generic kernels of graph.hip); the
loss assembly, the finite-volume update it differentiates through and Adam are
the reference trainer's own torch expressions, executed on the device.

Batching: the reference trains with batch size 1 (DataLoader(batch_size=1),
:85).  `batch_size=1` reproduces that loop step for step; `batch_size=B`
evaluates B samples as one batched graph (B disjoint chains) and averages the
per-sample losses, which for every term equals the mean of the B
single-sample losses — the batched training the survey asks for.

As in the reference, the Poisson / energy terms go through a detached
Poisson solve (there numpy, :138-145; here hf_poisson), so they contribute to
the loss value but not to the gradient; the multi-step rollout energies depend
only on u, which the model does not touch (:174-196).
"""
import json
import os
import time

import numpy as np
import torch

from . import engine
from .baseline_solver import BaselineSolver
from .config import ABLATION_CONFIGS, MODEL_CONFIG
from .flux_gnn import FluxGNN
from .graph_constructor import build_chain_graph_batch, shared_chain_edge_index


def _mse(a, b):
    return torch.mean((a - b) ** 2)


def _poisson_detached(grid, n):
    """E of densities n [B,nx] without gradient (train_ablation.py:47-57 solve_poisson_np)."""
    return engine.poisson(grid, n.detach())


class _StepLoss(torch.autograd.Function):
    """The loss terms as one HIP pass (hf_ablation_loss_ex): forward returns
    (loss, flux_loss) and keeps d loss / d flux_edge, which backward scales by
    the incoming gradient.  flux_loss is for reporting only.  roll = (K,
    lambda_energy_multi, dt) adds the rollout energy term (K <= 3), which
    carries no gradient."""

    @staticmethod
    def forward(ctx, flux_edge, st, ft, sn, grid, lam, roll):
        K, lam_m, dt = roll
        loss, fl, dfe = engine.ablation_loss_terms(grid, flux_edge, st, ft, sn, tuple(lam) + (lam_m,), K, dt)
        ctx.save_for_backward(dfe)
        ctx.mark_non_differentiable(fl)
        return loss, fl

    @staticmethod
    def backward(ctx, g_loss, g_fl):
        (dfe,) = ctx.saved_tensors
        return dfe * g_loss, None, None, None, None, None, None


def _has_rollout(cfg):
    return cfg["rollout_steps"] > 0 and cfg["lambda_energy_multi"] > 0  # train_ablation.py:172


def ablation_loss(model, st, ft, st_next, x, dt, dx, cfg, grid, n0=1.0, fused=True, nf=None, rollout="reuse"):
    """Loss of train_ablation.py:107-206 for a batch: st, st_next [B,3,nx], ft [B,nx]
    on the device.  Returns (loss, flux_loss); B=1 is the reference formula.
    fused: the terms (:124-170, and the rollout energy term for rollout_steps
    <= 3) in one HIP pass (hf_ablation_loss_ex) instead of the torch
    expressions below (kept as the readable statement of the same arithmetic,
    and for the comparison tests).  nf: the batch's chain node features when
    the caller has them (FluxDataset.batch with x).  rollout (torch form only):
    "reuse" runs no model forward whose result cannot reach the loss
    (_rollout_energies), "literal" the reference's loop of rollout_steps
    forwards (_rollout_energies_literal); the two give the same loss bit for bit."""
    B, _, nx = st.shape
    n_t, u_t = st[:, 0], st[:, 1]
    n_next_true, u_next_true, E_next_true = st_next[:, 0], st_next[:, 1], st_next[:, 2]
    if nf is None:
        nf, ei = build_chain_graph_batch(st, x)
    else:
        ei = shared_chain_edge_index(nx, B, st.device)
    flux_edge = model(nf, ei).reshape(B, 2 * nx)
    if fused and n0 == 1.0 and abs(dt / dx - grid.dt / grid.dx) <= 1e-12 * abs(dt / dx):
        lam = (cfg["lambda_state"], cfg["lambda_poisson"], cfg["lambda_charge"], cfg["lambda_energy_one"])
        K = cfg["rollout_steps"] if _has_rollout(cfg) else 0
        in_kernel = K <= engine.LOSS_MAX_ROLLOUT
        roll = (K, cfg["lambda_energy_multi"], dt) if in_kernel else (0, 0.0, dt)
        loss, flux_loss = _StepLoss.apply(flux_edge, st, ft, st_next, grid, lam, roll)
        if not in_kernel:  # later energies need forwards on later states
            loss = _add_rollout_term(loss, cfg, _rollout_energies(model, st, flux_edge, x, dt, dx, cfg, grid))
        return loss, flux_loss
    F_pred = 0.5 * (flux_edge[:, :nx] + flux_edge[:, nx:])                        # :124-126
    flux_loss = _mse(F_pred, ft)                                                   # :129
    loss = flux_loss
    n_next_pred = n_t - (dt / dx) * (F_pred - torch.roll(F_pred, 1, dims=-1))     # :134-135
    if cfg["lambda_state"] > 0:
        loss = loss + cfg["lambda_state"] * _mse(n_next_pred, n_next_true)
    E_next_pred = None
    if cfg["lambda_poisson"] > 0 or cfg["lambda_energy_one"] > 0:
        E_next_pred = _poisson_detached(grid, n_next_pred)
    if cfg["lambda_poisson"] > 0:                                                  # :140-147
        loss = loss + cfg["lambda_poisson"] * _mse(E_next_pred, E_next_true)
    if cfg["lambda_charge"] > 0:                                                   # :150-156
        charge_t = torch.sum(n_t - n0, dim=-1) * dx
        charge_next = torch.sum(n_next_pred - n0, dim=-1) * dx
        loss = loss + cfg["lambda_charge"] * _mse(charge_next, charge_t)
    if cfg["lambda_energy_one"] > 0:                                               # :159-170
        e_p = 0.5 * torch.mean(u_next_true ** 2 + E_next_pred ** 2, dim=-1)
        e_t = 0.5 * torch.mean(u_next_true ** 2 + E_next_true ** 2, dim=-1)
        loss = loss + cfg["lambda_energy_one"] * _mse(e_p, e_t)
    if _has_rollout(cfg):
        if rollout == "literal":
            energies = _rollout_energies_literal(model, st, x, dt, dx, cfg, grid)
        else:
            energies = _rollout_energies(model, st, flux_edge, x, dt, dx, cfg, grid)
        loss = _add_rollout_term(loss, cfg, energies)
    return loss, flux_loss


def _add_rollout_term(loss, cfg, energies):
    """+ lambda_energy_multi * mean((energies - energies[0])^2) (:204-206)."""
    return loss + cfg["lambda_energy_multi"] * torch.mean((energies - energies[0]) ** 2)


def _rollout_energies_literal(model, st, x, dt, dx, cfg, grid):
    """The rollout energies [K, B] as the reference's loop computes them
    (:173-204): K model forwards, one per rolled state."""
    B, _, nx = st.shape
    state = st.clone()
    energies = []
    for _ in range(cfg["rollout_steps"]):
        n_r, u_r, E_r = state[:, 0], state[:, 1], state[:, 2]
        energies.append(0.5 * torch.mean(u_r ** 2, dim=-1))                         # :181-182
        nf_r, ei_r = build_chain_graph_batch(state, x)
        fe_r = model(nf_r, ei_r).reshape(B, 2 * nx)
        F_r = 0.5 * (fe_r[:, :nx] + fe_r[:, nx:])
        n_next_r = n_r - (dt / dx) * (F_r - torch.roll(F_r, 1, dims=-1))
        F_u = 0.5 * u_r * u_r
        u_next_r = u_r - (dt / dx) * (F_u - torch.roll(F_u, 1, dims=-1)) + dt * E_r
        state = torch.stack([n_next_r, u_next_r, _poisson_detached(grid, n_next_r)], dim=1)
    return torch.stack(energies)                                                   # [K, B]


def _rollout_energies(model, st, flux_edge, x, dt, dx, cfg, grid):
    """The same energies [K, B] as _rollout_energies_literal, bit for bit, with
    only the forwards whose results reach them.  The energy of step k is
    0.5 mean(u_k^2) (:181) and u_{k+1} needs E_k (:196), which for k >= 1 is
    the detached Poisson E of the n_k that forward k-1 produced (:191, :198-
    200).  So the energies reach forwards 0 .. K-3 only, forward 0 is the main
    forward (the same model on the same state: its flux_edge is reused), and
    the others run untaped (no_grad: nothing differentiates through them — u
    never depends on the parameters).  For the reference's K = 3: no forward."""
    B, _, nx = st.shape
    K = cfg["rollout_steps"]
    n_r, u_r, E_r = st[:, 0], st[:, 1], st[:, 2]
    fe_r = flux_edge.detach()
    energies = []
    for k in range(K):
        energies.append(0.5 * torch.mean(u_r ** 2, dim=-1))
        if k == K - 1:
            break
        F_u = 0.5 * u_r * u_r
        u_next = u_r - (dt / dx) * (F_u - torch.roll(F_u, 1, dims=-1)) + dt * E_r
        n_next = E_next = None
        if k + 2 <= K - 1:  # E_{k+1} feeds u_{k+2}, the last energy's u at k + 2 = K - 1
            if fe_r is None:
                with torch.no_grad():
                    nf_r, ei_r = build_chain_graph_batch(torch.stack([n_r, u_r, E_r], dim=1), x)
                    fe_r = model(nf_r, ei_r).reshape(B, 2 * nx)
            F_r = 0.5 * (fe_r[:, :nx] + fe_r[:, nx:])
            n_next = n_r - (dt / dx) * (F_r - torch.roll(F_r, 1, dims=-1))
            E_next = _poisson_detached(grid, n_next)
        fe_r = None
        n_r, u_r, E_r = n_next, u_next, E_next
    return torch.stack(energies)


def train_flop_per_sample(cfg, nx=64, H=128, L=4, F=4):
    """Algorithmic FLOPs of one sample of the training step with the ablation
    config `cfg` (a dict of ABLATION_CONFIGS or its name): FluxGNN forward +
    backward (P/Q-split readout, as the inference count of SURVEY.md 8d):
    forward 329,216 per cell (input 2FH, layers L*2*2H*H, readout 2*H*2H +
    2 edges * 2H), backward = data gradients (layers L*2*2H*H, readout 2*2H*H)
    + weight gradients (the same GEMM sizes, plus the input layer's 2FH).  The
    rollout energy term ('full', 'rollout_only') adds only the forwards whose
    results reach the loss, none for the reference's rollout_steps = 3
    (_rollout_energies; the reference's own loop runs 3 forwards there, of
    which none is needed), and no backward (the term has no gradient).  The
    loss terms' elementwise FV updates and detached Poisson solves are not counted."""
    if isinstance(cfg, str):
        cfg = ABLATION_CONFIGS[cfg]
    fwd = 2 * F * H + L * 2 * 2 * H * H + 2 * H * 2 * H + 2 * 2 * H
    bwd = (L * 2 * 2 * H * H + 2 * 2 * H * H) * 2 + 2 * F * H
    extra = max(0, cfg["rollout_steps"] - 3) if _has_rollout(cfg) else 0
    return ((fwd + bwd) + extra * fwd) * nx


class FluxDataset:
    """Device-resident (state_t, flux_t, state_next) triples (train_ablation.py:27-44)."""

    def __init__(self, state_t, flux_t, state_next, device="cuda"):
        assert state_t.shape == state_next.shape and state_t.shape[0] == flux_t.shape[0]
        as_t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32), device=device)  # noqa: E731
        self.state_t, self.flux_t, self.state_next = as_t(state_t), as_t(flux_t), as_t(state_next)
        self.N, self.C, self.nx = self.state_t.shape

    def __len__(self):
        return self.N

    def check_indices(self, idx):
        """IndexError unless every index lies in [-N, N) (torch indexing's
        range; one host sync)."""
        idx = torch.as_tensor(idx)
        if idx.numel() and (int(idx.min()) < -self.N or int(idx.max()) >= self.N):
            raise IndexError(f"sample index out of range for a dataset of {self.N} samples")

    def batch(self, idx, x=None, check=True):
        """(state_t, flux_t, state_next)[idx]; with x (the grid positions [nx])
        also the batch's chain node features, all four from one HIP pass
        (engine.chain_batch): (st, ft, sn, node_features).  Indices outside
        [-N, N) raise IndexError as the reference's dataset indexing does
        (check_indices: a host sync); check=False skips that for indices the
        caller has already checked (train_steps checks a pass's order once),
        and then the device gather clamps an out-of-range index to [0, N)
        instead of raising (include/hybridflux.h hf_chain_batch_gather)."""
        if check:
            self.check_indices(idx)
        if x is None:
            return self.state_t[idx], self.flux_t[idx], self.state_next[idx]
        return engine.chain_batch(idx, self.state_t, self.flux_t, self.state_next, x)


class FlatAdam(torch.optim.Optimizer):
    """torch.optim.Adam (weight decay 0, no amsgrad: the reference trainer's
    optimizer, train_ablation.py:82, :208-209) for a model whose parameters
    share one buffer (FluxGNN.flatten_parameters_): the update of every
    parameter in one HIP launch (hf_adam_flat) with the step count on the
    device, so it is capturable (GraphedStep) and needs no host sync.  The
    gradients are read as one buffer when they are (the chain training
    backward returns them as pieces of one), otherwise concatenated first."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        from .flux_gnn import _flat_view
        self._flat_view = _flat_view
        for group in self.param_groups:
            ps = group["params"]
            flat = _flat_view(ps, ps[0].device)
            if flat is None:
                raise ValueError("FlatAdam: the parameters must share one float32 buffer in order "
                                 "(call model.flatten_parameters_() first)")
            st = self.state[ps[0]]  # (the buffer itself is found again each step: state_dict() stays plain)
            st["exp_avg"] = torch.zeros_like(flat)
            st["exp_avg_sq"] = torch.zeros_like(flat)
            st["step"] = torch.zeros(1, dtype=torch.float32, device=flat.device)
            # the kernel's done-counter: 4 zero bytes (float32 so that load_state_dict's cast keeps them 0)
            st["done"] = torch.zeros(1, dtype=torch.float32, device=flat.device)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = group["params"]
            st = self.state[ps[0]]
            flat = self._flat_view(ps, ps[0].device)
            if flat is None:
                raise RuntimeError("FlatAdam: the parameters no longer share one buffer (moved or re-created?)")
            if any(p.grad is None for p in ps):
                raise RuntimeError("FlatAdam: every parameter needs a gradient")
            for k in ("exp_avg", "exp_avg_sq", "step", "done"):  # (a state_dict loaded elsewhere)
                if st[k].device != flat.device or st[k].dtype != torch.float32 or not st[k].is_contiguous():
                    st[k] = st[k].to(device=flat.device, dtype=torch.float32).contiguous()
            g = self._flat_view([p.grad for p in ps], ps[0].device)
            if g is None:
                g = torch.cat([p.grad.reshape(-1) for p in ps])
            b1, b2 = group["betas"]
            engine.adam_flat(flat, g, st["exp_avg"], st["exp_avg_sq"], st["step"], st["done"], group["lr"],
                             b1, b2, group["eps"])
            # the kernel wrote the parameters behind autograd's back: bump their
            # version counters as an in-place torch update would, so that a packed
            # inference copy (FluxGNN.device_model keys on _version) is rebuilt
            torch.autograd.graph.increment_version(ps)
        return loss


def direct_step(model, opt, st, ft, sn, nf, x, dt, dx, cfg, grid):
    """One step of the reference trainer's loop (ablation_loss ->
    loss.backward() -> optimizer.step(), train_ablation.py:107-210) without
    autograd where it reduces to three HIP passes and the optimizer launch:
    FluxGNN with flat parameters (flatten_parameters_), FlatAdam over exactly
    those parameters, the one-pass loss (rollout_steps <= 3), and the batch's
    chain node features nf (FluxDataset.batch with x).  The forward
    (hf_graph_forward_train), the loss and its flux gradient
    (hf_ablation_loss_ex), the backward (hf_graph_backward) with that gradient
    as the incoming one -- autograd's seed is 1 and _StepLoss.backward's
    product dfe * 1 is dfe exactly -- and FlatAdam on the gradient buffer: the
    same parameters bit for bit as the autograd step, without its seed fill,
    gradient product and bookkeeping launches.  Parameter hooks are not run.
    Returns (loss, flux_loss) detached, or None when the case does not apply
    (the caller then takes the autograd step)."""
    from .flux_gnn import _flat_view
    if type(model) is not FluxGNN or not isinstance(opt, FlatAdam) or nf is None or not torch.is_grad_enabled():
        return None
    params = list(model.parameters())
    if len(opt.param_groups) != 1 or [id(q) for q in opt.param_groups[0]["params"]] != [id(q) for q in params] \
            or not all(q.requires_grad for q in params):
        return None
    dev = st.device
    flat = _flat_view(params, dev)
    K = cfg["rollout_steps"] if _has_rollout(cfg) else 0
    if flat is None or K > engine.LOSS_MAX_ROLLOUT or abs(dt / dx - grid.dt / grid.dx) > 1e-12 * abs(dt / dx):
        return None
    B, _, nx = st.shape
    dims = (model.input_dim, model.hidden_dim, model.num_layers)
    flux, tape, nf_d, ei_d, chain_nx = engine.graph_forward_train(flat, dims, nf.detach(),
                                                                  shared_chain_edge_index(nx, B, dev))
    lam = (cfg["lambda_state"], cfg["lambda_poisson"], cfg["lambda_charge"], cfg["lambda_energy_one"],
           cfg["lambda_energy_multi"])
    loss, flux_loss, dfe = engine.ablation_loss_terms(grid, flux.reshape(B, 2 * nx), st, ft, sn, lam, K, dt)
    gp, _ = engine.graph_backward(flat, dims, nf_d, ei_d, chain_nx, tape, dfe.reshape(-1), False)
    o = 0
    for q in params:
        q.grad = gp[o:o + q.numel()].view_as(q)
        o += q.numel()
    opt.step()
    return loss.detach(), flux_loss.detach()


class GraphedStep:
    """One optimizer step of the reference trainer's loop (ablation_loss ->
    backward -> optimizer step, train_ablation.py:107-210) on a fixed batch
    size, captured once as a HIP graph (torch.cuda.graph) and replayed per
    batch: the step's ~100 small launches (loss terms, FV updates, Poisson,
    FluxGNN forward/backward kernels, Adam) become one graph launch.  The
    batch indices are a static device tensor gathered inside the graph.  The
    optimizer must be capturable (torch.optim.Adam(..., capturable=True)).
    The warmup steps that precede the capture are ordinary eager steps on the
    first batches, so a pass makes exactly the eager loop's updates."""

    def __init__(self, model, opt, data, batch_size, x, dt, dx, cfg, grid, direct=True):
        self.args = (model, opt, data, x, dt, dx, cfg, grid)
        self.direct = direct  # direct_step where it applies
        dev = data.state_t.device
        self.idx = torch.zeros(batch_size, dtype=torch.long, device=dev)
        self.graph = None
        self.out = None

    def _body(self):
        model, opt, data, x, dt, dx, cfg, grid = self.args
        st, ft, sn, nf = data.batch(self.idx, x, check=False)  # (train_steps checked the order)
        if self.direct:
            r = direct_step(model, opt, st, ft, sn, nf, x, dt, dx, cfg, grid)
            if r is not None:
                return r
        loss, flux_loss = ablation_loss(model, st, ft, sn, x, dt, dx, cfg, grid, nf=nf)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss.detach(), flux_loss.detach()

    def capture(self):
        self.args[1].zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._body()

    def __call__(self, idx):
        """Step on batch idx (a device index tensor of the captured size):
        (loss, flux_loss) as fresh device scalars."""
        self.idx.copy_(idx)
        if self.graph is None:
            return self._body()
        self.graph.replay()
        # the replayed optimizer step changed the parameters without a host-side
        # in-place op: bump their versions (FluxGNN.device_model keys on them)
        torch.autograd.graph.increment_version(list(self.args[0].parameters()))
        return self.out[0].clone(), self.out[1].clone()


def train_steps(model, opt, data, order, batch_size, x, dt, dx, cfg, grid, graphed=None, warmup=3, direct=True):
    """One pass over `order` (sample indices) in batches; returns (sum of
    losses, sum of flux losses) weighted by batch size, and the step count.
    graphed: a GraphedStep of this batch size (created by the caller and kept
    across passes); its first `warmup` steps run eagerly on a side stream, then
    it is captured and every further full batch replays the graph.  direct:
    eager steps take direct_step where it applies (the same parameters bit for
    bit as the autograd step)."""
    tot, tot_flux, steps = 0.0, 0.0, 0
    losses = []
    data.check_indices(order)  # once per pass; the steps gather with check=False
    for b0 in range(0, len(order), batch_size):
        idx = order[b0:b0 + batch_size]
        if graphed is not None and len(idx) == batch_size:
            if graphed.graph is None and getattr(graphed, "_warm", 0) >= warmup:
                torch.cuda.synchronize()
                graphed.capture()
            if graphed.graph is None:
                graphed._warm = getattr(graphed, "_warm", 0) + 1
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    loss, flux_loss = graphed(idx)
                torch.cuda.current_stream().wait_stream(side)
            else:
                loss, flux_loss = graphed(idx)
        else:
            st, ft, sn, nf = data.batch(idx, x, check=False)
            r = direct_step(model, opt, st, ft, sn, nf, x, dt, dx, cfg, grid) if direct else None
            if r is not None:
                loss, flux_loss = r
            else:
                loss, flux_loss = ablation_loss(model, st, ft, sn, x, dt, dx, cfg, grid, nf=nf)
                opt.zero_grad()
                loss.backward()
                opt.step()
                loss, flux_loss = loss.detach(), flux_loss.detach()
        losses.append((loss, flux_loss, len(idx)))
        steps += 1
    for l, f, n in losses:  # one host sync per pass, not per step
        tot += float(l) * n
        tot_flux += float(f) * n
    return tot, tot_flux, steps


def train_model(state_t, flux_t, state_next, x, dt, dx, nu, config_name, stencil_radius, epochs=20, lr=1e-3,
                device="cuda", batch_size=1, seed=None, save_dir="checkpoints", log=print):
    """scripts/training/train_ablation.py:64-237 on the MI355X.  Returns
    (model, history) and writes checkpoints/hybrid_<config>_r<radius>.pt and
    history_<config>_r<radius>.json like the reference (save_dir=None skips)."""
    cfg = ABLATION_CONFIGS[config_name]
    engine.require_device(torch.empty(0, device=device), "device")
    if seed is not None:
        torch.manual_seed(seed)
    data = FluxDataset(state_t, flux_t, state_next, device)
    grid = BaselineSolver(nx=data.nx, dt=dt, nu=nu, device=device).grid
    x_dev = torch.as_tensor(np.asarray(x, dtype=np.float32), device=device)
    model = FluxGNN(MODEL_CONFIG["input_dim"], MODEL_CONFIG["hidden_dim"], MODEL_CONFIG["num_layers"]).to(device)
    model.flatten_parameters_()  # one parameter buffer: no per-step concat in the training forward
    opt = FlatAdam(model.parameters(), lr=lr)  # torch.optim.Adam's update (:82), one launch per step
    gen = torch.Generator().manual_seed(0 if seed is None else seed)
    history = {"epoch": [], "loss": [], "flux_loss": [], "seconds": []}
    model.train()
    for epoch in range(1, epochs + 1):
        order = torch.randperm(len(data), generator=gen).to(device)
        t0 = time.perf_counter()
        tot, tot_flux, _ = train_steps(model, opt, data, order, batch_size, x_dev, dt, dx, cfg, grid)
        torch.cuda.synchronize(device)
        history["epoch"].append(epoch)
        history["loss"].append(tot / len(data))
        history["flux_loss"].append(tot_flux / len(data))
        history["seconds"].append(time.perf_counter() - t0)
        if log:
            log(f"[Epoch {epoch}/{epochs}] Loss: {history['loss'][-1]:.6e}, Flux: {history['flux_loss'][-1]:.6e}")
    if save_dir is not None:
        os.makedirs(save_dir, exist_ok=True)
        # (cloned: one storage per tensor, as the reference's checkpoints, not views of the flat buffer)
        torch.save({k: v.clone() for k, v in model.state_dict().items()}, os.path.join(save_dir, f"hybrid_{config_name}_r{stencil_radius}.pt"))
        with open(os.path.join(save_dir, f"history_{config_name}_r{stencil_radius}.json"), "w") as f:
            json.dump(history, f, indent=2)
    return model, history
