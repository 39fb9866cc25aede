"""Device-side engine: owns the libhybridflux model handles and per-grid
device constants, and launches the hot path on torch's current HIP stream.

Everything here takes and returns torch tensors that already live on a HIP
device; the reference-shaped numpy API (HybridSolver / BaselineSolver) sits
on top of it.  Scalars follow the reference's rounding: the Python floats
dt/dx, dt, nu and dx**2 are rounded to float32 once on the host, exactly as
numpy does when it mixes them with float32 arrays (src/hybrid_solver.py:52,
56-57; src/baseline_solver.py:86,91,94).
"""
import math
from ctypes import c_void_p

import numpy as np
import torch

from . import _lib
from ._lib import HF_NUM_METRICS, HF_OP_COMPARE, HF_OP_RUN, HF_OP_STEP, check, lib, ptr

LOSS_MAX_ROLLOUT = 3  # hf_ablation_loss_ex forms the rollout energy term for rollout_steps <= 3

PARAM_ORDER_DOC = "input_mlp.0.{weight,bias}, update_mlps.<l>.0.{weight,bias}, edge_mlp.0.*, edge_mlp.2.*"


def require_device(t, what="tensor"):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError(
            f"hybridflux: {what} must be a torch tensor on a HIP (cuda) device; this engine has no CPU "
            f"path (got {type(t).__name__}{'' if not isinstance(t, torch.Tensor) else ' on ' + str(t.device)})")
    return t


def compute_device(t, what="tensor"):
    """The HIP device a drop-in call computes on: t's own device when t is a
    device tensor; for a host tensor (the reference's CPU call pattern,
    examples/smoke_test.py:50-56) the current HIP device, to which the
    caller's inputs are staged and from which results are copied back.  No HIP
    device visible: raises (the kernels are the only implementation)."""
    if isinstance(t, torch.Tensor) and t.is_cuda:
        return t.device
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"hybridflux: {what} must be a torch tensor, got {type(t).__name__}")
    if not torch.cuda.is_available():
        raise RuntimeError(f"hybridflux: {what} is a host tensor and no HIP device is visible; this engine has "
                           "no CPU path (host tensors are staged to the current HIP device, and there is none)")
    return torch.device("cuda", torch.cuda.current_device())


def stream_of(device):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def flatten_params(sd, layers):
    """Reference state dict (src/flux_gnn.py:17-38 keys) -> flat float32 array in
    the order include/hybridflux.h documents for hf_model_create."""
    def arr(k):
        v = sd[k]
        if isinstance(v, torch.Tensor):
            v = v.detach().to("cpu", torch.float32).numpy()
        return np.ascontiguousarray(np.asarray(v, dtype=np.float32)).reshape(-1)

    parts = [arr("input_mlp.0.weight"), arr("input_mlp.0.bias")]
    for l in range(layers):
        parts += [arr(f"update_mlps.{l}.0.weight"), arr(f"update_mlps.{l}.0.bias")]
    parts += [arr("edge_mlp.0.weight"), arr("edge_mlp.0.bias"), arr("edge_mlp.2.weight"), arr("edge_mlp.2.bias")]
    return np.ascontiguousarray(np.concatenate(parts))


def dims_of(sd):
    w_in = sd["input_mlp.0.weight"]
    hidden, in_dim = int(w_in.shape[0]), int(w_in.shape[1])
    layers = sum(1 for k in sd if k.startswith("update_mlps.") and k.endswith(".0.weight"))
    return in_dim, hidden, layers


PRECISIONS = {"f32": _lib.HF_WDTYPE_F32, "bf16": _lib.HF_WDTYPE_BF16, "f16x3": _lib.HF_WDTYPE_F16X3}


class DeviceModel:
    """A packed, read-only copy of FluxGNN weights on one device (hf_model_t).

    precision selects the chain kernels' matrix-core arithmetic:
      "f32"   v_mfma_f32_16x16x4_f32, exact float32 (parity reference)
      "f16x3" fp16 hi+lo split of weights and activations, 3 products on
              v_mfma_f32_16x16x32_f16, f32 accumulate: float32-level accuracy
              while every GEMM input stays within the fp16 range (|value| <
              65504; the physical states of this model are O(1), ~1e3x inside
              it); past it the split overflows and the flux is reported
              non-finite where f32 would still be finite (tests: test_f16x3_range)
      "bf16"  bf16 weights and activations, f32 accumulate (BASELINE config 4)
    The generic-graph path always computes in float32."""

    def __init__(self, state_dict, device, precision="f32"):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
        self.precision = precision
        self.in_dim, self.hidden, self.layers = dims_of(state_dict)
        self.device = torch.device(device)
        flat = flatten_params(state_dict, self.layers)
        want = lib().hf_model_param_count(self.in_dim, self.hidden, self.layers)
        if flat.size != want:
            raise ValueError(f"state dict has {flat.size} parameters, expected {want}")
        self.handle = c_void_p()
        with torch.cuda.device(self.device):
            check(lib().hf_model_create(flat.ctypes.data_as(c_void_p), self.in_dim, self.hidden,
                                        self.layers, PRECISIONS[precision], self.handle))

    @property
    def chain_ok(self):
        return self.in_dim == 4 and self.hidden == 128

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            lib().hf_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass


POISSON_MODES = {"spectral": _lib.HF_POISSON_SPECTRAL, "tridiagonal": _lib.HF_POISSON_TRIDIAG}


class Grid:
    """Geometry + time-step constants (src/baseline_solver.py:7-27) and their
    device copies: cell centres x (float32) and the Poisson plan.

    poisson selects the operator every step / rollout / solve of this grid
    applies: "spectral" (default) is the reference's (src/baseline_solver.py:
    59-68, the parity mode); "tridiagonal" is the OPT-IN cyclic-reduction solve
    of the second-order potential form of the same equation, which is NOT the
    reference's operator (~1e-3 from it at nx = 64; include/hybridflux.h
    HF_POISSON_TRIDIAG).  The training loss always uses the spectral plan."""

    def __init__(self, nx=64, length=2 * math.pi, dt=5e-3, nu=1e-3, poisson="spectral"):
        if poisson not in POISSON_MODES:
            raise ValueError(f"poisson must be one of {sorted(POISSON_MODES)}, got {poisson!r}")
        self.nx, self.length, self.dt, self.nu = int(nx), float(length), float(dt), float(nu)
        self.poisson, self.pmode = poisson, POISSON_MODES[poisson]
        self.dx = self.length / self.nx
        self.x = np.linspace(0.5 * self.dx, self.length - 0.5 * self.dx, self.nx)
        self.c32 = float(np.float32(self.dt / self.dx))
        self.dt32 = float(np.float32(self.dt))
        self.nu32 = float(np.float32(self.nu))
        self.dx2_32 = float(np.float32(self.dx ** 2))
        pc = np.empty(lib().hf_poisson_plan_len(self.nx), dtype=np.float64)
        check(lib().hf_poisson_coeffs(self.nx, self.length, pc.ctypes.data_as(c_void_p)))
        self.poisson_c = pc  # the spectral plan (also the training loss's)
        if self.pmode == _lib.HF_POISSON_SPECTRAL:
            self.plan = pc
        else:
            n = int(lib().hf_poisson_plan_size(self.pmode, self.nx))
            if n < 1:  # (-1: unsupported; checked before allocating)
                raise ValueError(f"{poisson} Poisson does not support nx = {self.nx}")
            self.plan = np.empty(n, dtype=np.float64)
            check(lib().hf_poisson_plan(self.pmode, self.nx, self.length, self.plan.ctypes.data_as(c_void_p)))
        self._dev = {}

    def _consts(self, device):
        device = torch.device(device)
        key = str(device)
        if key not in self._dev:
            x = torch.as_tensor(self.x.astype(np.float32), device=device)
            pc = torch.as_tensor(self.poisson_c, device=device)
            plan = pc if self.plan is self.poisson_c else torch.as_tensor(self.plan, device=device)
            self._dev[key] = (x, plan, pc)
        return self._dev[key]

    def on(self, device):
        """(x, Poisson plan of this grid's mode) on device."""
        x, plan, _ = self._consts(device)
        return x, plan

    def spectral_plan(self, device):
        """The spectral plan on device (hf_ablation_loss: the reference trainer's solve)."""
        return self._consts(device)[2]


def _state(t, nx):
    require_device(t, "state")
    if t.dtype != torch.float32 or t.dim() != 3 or t.shape[1] != 3 or t.shape[2] != nx:
        raise ValueError(f"state must be float32 [B,3,{nx}], got {tuple(t.shape)} {t.dtype}")
    return t.contiguous()


def workspace(op, B, nx, T, dev, given=None, model=None, traj=False, flux_face=False):
    """Scratch for the generic (non-fused) sequencing of hf_step / hf_run /
    hf_run_compare: the caller's uint8 device tensor (checked), or one from
    torch's stream-ordered caching allocator, so no hipMalloc runs inside a
    rollout.  Sized by hf_workspace_need for this path: `model` is the
    DeviceModel (None = classical), `traj` / `flux_face` whether the call gets
    a trajectory / face-flux buffer.  Paths that need no scratch (the fused
    rollouts, the one-launch classical rollouts) get None.  Returns (tensor or
    None, bytes)."""
    flags = (_lib.HF_WS_TRAJ if traj is not False and traj is not None else 0) | \
            (_lib.HF_WS_FLUX_FACE if flux_face is not False and flux_face is not None else 0)
    handle = model.handle if model is not None else None
    nbytes = int(lib().hf_workspace_need(handle, op, B, nx, T, flags))
    if nbytes < 0:
        raise ValueError(f"bad workspace query (op={op}, B={B}, nx={nx}, T={T})")
    if given is not None:
        if not (given.is_cuda and given.device == dev and given.numel() * given.element_size() >= nbytes):
            raise ValueError(f"workspace must be a device tensor of >= {nbytes} bytes on {dev}")
        return given, given.numel() * given.element_size()
    if nbytes == 0:
        return None, 0
    return torch.empty(nbytes, dtype=torch.uint8, device=dev), nbytes


def step(model, grid, state, flux_face=False, metrics=False, ws=None):
    """One hybrid (model) or classical (model=None) step for state [B,3,nx]."""
    state = _state(state, grid.nx)
    B, dev = state.shape[0], state.device
    out = torch.empty_like(state)
    F = torch.empty(B, grid.nx, device=dev) if flux_face else None
    M = torch.empty(B, HF_NUM_METRICS, device=dev) if metrics else None
    x, pc = grid.on(dev)
    w, wb = workspace(HF_OP_STEP, B, grid.nx, 1, dev, ws, model=model, flux_face=flux_face)
    with torch.cuda.device(dev):
        check(lib().hf_step_ex(model.handle if model else None, ptr(state), ptr(out), ptr(x), ptr(pc),
                               grid.pmode, B, grid.nx, grid.c32, grid.dt32, grid.nu32, grid.dx2_32, ptr(F), ptr(M), ptr(w), wb,
                            stream_of(dev)))
    return out, F, M


def _buf(want, given, shape, dev):
    """An output buffer: the caller's preallocated tensor (checked), a new one, or None."""
    if isinstance(given, torch.Tensor):
        if tuple(given.shape) != tuple(shape) or given.dtype != torch.float32 or given.device != dev \
                or not given.is_contiguous():
            raise ValueError(f"preallocated output must be contiguous float32 {tuple(shape)} on {dev}")
        return given
    return torch.empty(shape, device=dev) if want else None


def run(model, grid, state0, T, traj=True, flux=False, metrics=False, out=None, ws=None):
    """T-step rollout; returns dict(final, traj [B,T+1,3,nx], flux [B,T,nx], metrics [B,T+1,4]).
    traj/flux/metrics may be bools or preallocated tensors, and ws a preallocated
    workspace (kept out of timed regions).  out may be state0 itself."""
    state0 = _state(state0, grid.nx)
    B, dev = state0.shape[0], state0.device
    T = int(T)
    final = torch.empty_like(state0) if out is None else out
    tr = _buf(traj, traj, (B, T + 1, 3, grid.nx), dev)
    fl = _buf(flux, flux, (B, T, grid.nx), dev)
    me = _buf(metrics, metrics, (B, T + 1, HF_NUM_METRICS), dev)
    x, pc = grid.on(dev)
    w, wb = workspace(HF_OP_RUN, B, grid.nx, T, dev, ws, model=model, traj=tr)
    with torch.cuda.device(dev):
        check(lib().hf_run_ex(model.handle if model else None, ptr(state0), ptr(final), ptr(x), ptr(pc),
                              grid.pmode, B, grid.nx, T, grid.c32, grid.dt32, grid.nu32, grid.dx2_32, ptr(tr), ptr(fl),
                           ptr(me), ptr(w), wb, stream_of(dev)))
    return {"final": final, "traj": tr, "flux": fl, "metrics": me}


def run_compare(model, grid, state0, T, metrics=True, out=None, ws=None):
    """Hybrid rollout and its classical twin from the same ICs, scored per step
    (scripts/evaluation/evaluate_multi_ic.py:21-94).  Returns dict(final,
    mse [B,T+1,3] (n,u,E), metrics [B,T+1,4], metrics_classical [B,T+1,4])."""
    state0 = _state(state0, grid.nx)
    B, dev = state0.shape[0], state0.device
    T = int(T)
    final = torch.empty_like(state0) if out is None else out
    mse = torch.empty(B, T + 1, 3, device=dev)
    me = torch.empty(B, T + 1, HF_NUM_METRICS, device=dev) if metrics else None
    mc = torch.empty(B, T + 1, HF_NUM_METRICS, device=dev) if metrics else None
    x, pc = grid.on(dev)
    w, wb = workspace(HF_OP_COMPARE, B, grid.nx, T, dev, ws, model=model)
    with torch.cuda.device(dev):
        check(lib().hf_run_compare_ex(model.handle, ptr(state0), ptr(final), ptr(x), ptr(pc), grid.pmode, B,
                                      grid.nx, T,
                                   grid.c32, grid.dt32, grid.nu32, grid.dx2_32, ptr(mse), ptr(me), ptr(mc),
                                   ptr(w), wb, stream_of(dev)))
    return {"final": final, "mse": mse, "metrics": me, "metrics_classical": mc}


def chain_flux(model, node_features, B, nx):
    """FluxGNN.forward on B disjoint periodic chains of nx cells -> [B*2nx]."""
    require_device(node_features, "node_features")
    nf = node_features.contiguous()
    if nf.dtype != torch.float32 or nf.shape != (B * nx, 4):
        raise ValueError(f"node_features must be float32 [{B * nx},4], got {tuple(nf.shape)} {nf.dtype}")
    fe = torch.empty(B * 2 * nx, device=nf.device)
    with torch.cuda.device(nf.device):
        check(lib().hf_chain_flux(model.handle, ptr(nf), B, nx, ptr(fe), None, stream_of(nf.device)))
    return fe


def graph_flux(model, node_features, edge_index):
    """FluxGNN.forward on an arbitrary graph (generic path) -> [E]."""
    require_device(node_features, "node_features")
    nf = node_features.to(torch.float32).contiguous()
    ei = edge_index.to(device=nf.device, dtype=torch.int64).contiguous()
    N, E = nf.shape[0], ei.shape[1]
    if nf.dim() != 2 or nf.shape[1] != model.in_dim:
        raise ValueError(f"node_features must be [N,{model.in_dim}], got {tuple(nf.shape)}")
    flux = torch.empty(E, device=nf.device)
    if E == 0:
        return flux
    lo, hi = int(ei.min()), int(ei.max())  # reference raises IndexError on these too
    if lo < 0 or hi >= N:
        raise IndexError(f"edge_index entries must lie in [0, {N}), got [{lo}, {hi}]")
    ws = torch.empty(int(lib().hf_graph_workspace_bytes(model.handle, N, E)), dtype=torch.uint8,
                     device=nf.device)
    with torch.cuda.device(nf.device):
        check(lib().hf_graph_flux(model.handle, ptr(nf), N, ptr(ei), E, ptr(flux), ptr(ws),
                                  stream_of(nf.device)))
    return flux


def _graph_inputs(node_features, edge_index, in_dim):
    require_device(node_features, "node_features")
    nf = node_features.detach().to(torch.float32).contiguous()
    ei = edge_index.to(device=nf.device, dtype=torch.int64).contiguous()
    if nf.dim() != 2 or nf.shape[1] != in_dim:
        raise ValueError(f"node_features must be [N,{in_dim}], got {tuple(nf.shape)}")
    if ei.dim() != 2 or ei.shape[0] != 2:
        raise ValueError(f"edge_index must be [2,E], got {tuple(ei.shape)}")
    N, E = nf.shape[0], ei.shape[1]
    from .graph_constructor import chain_tag
    tag = chain_tag(edge_index)
    chain_nx = tag[1] if tag is not None and tag[0] * tag[1] == N and E == 2 * N else 0
    if E and not chain_nx:  # an unmodified tagged chain is in range by construction
        lo, hi = int(ei.min()), int(ei.max())  # the reference raises IndexError on these too
        if lo < 0 or hi >= N:
            raise IndexError(f"edge_index entries must lie in [0, {N}), got [{lo}, {hi}]")
    return nf, ei, N, E, chain_nx


def graph_forward_train(params, dims, node_features, edge_index):
    """Training forward (hf_graph_forward_train): params is the flat float32
    device buffer in state-dict order.  Returns (flux [E], tape, nf, ei)."""
    in_dim, hidden, layers = dims
    nf, ei, N, E, chain_nx = _graph_inputs(node_features, edge_index, in_dim)
    if params.device != nf.device:
        raise RuntimeError(f"FluxGNN parameters on {params.device} but node_features on {nf.device}")
    flux = torch.empty(E, device=nf.device)
    tape = torch.empty(int(lib().hf_graph_tape_bytes(in_dim, hidden, layers, N, E)), dtype=torch.uint8,
                       device=nf.device)
    with torch.cuda.device(nf.device):
        check(lib().hf_graph_forward_train(ptr(params), in_dim, hidden, layers, ptr(nf), N, ptr(ei), E, chain_nx,
                                           ptr(flux), ptr(tape), stream_of(nf.device)))
    return flux, tape, nf, ei, chain_nx


def graph_backward(params, dims, nf, ei, chain_nx, tape, grad_flux, want_nf_grad):
    """hf_graph_backward: (d params flat [P], d node_features [N,in] or None)."""
    in_dim, hidden, layers = dims
    N, E = nf.shape[0], ei.shape[1]
    g = grad_flux.detach().to(device=nf.device, dtype=torch.float32).contiguous()
    gp = torch.empty_like(params)
    gnf = torch.empty_like(nf) if want_nf_grad else None
    ws = torch.empty(int(lib().hf_graph_backward_workspace_bytes(in_dim, hidden, layers, N, E)),
                     dtype=torch.uint8, device=nf.device)
    with torch.cuda.device(nf.device):
        check(lib().hf_graph_backward(ptr(params), in_dim, hidden, layers, ptr(nf), N, ptr(ei), E, chain_nx, ptr(tape),
                                      ptr(g), ptr(gp), ptr(gnf) if gnf is not None else None, ptr(ws),
                                      stream_of(nf.device)))
    return gp, gnf


def poisson(grid, n):
    """Poisson E for densities n [B,nx]: the grid's mode (spectral: src/baseline_solver.py:59-68)."""
    require_device(n, "n")
    n = n.to(torch.float32).contiguous()
    B = n.shape[0]
    E = torch.empty_like(n)
    _, pc = grid.on(n.device)
    with torch.cuda.device(n.device):
        check(lib().hf_poisson_ex(ptr(n), grid.nx, ptr(E), grid.nx, ptr(pc), grid.pmode, B, grid.nx,
                                  stream_of(n.device)))
    return E


def _series(t, shape_tail, what):
    require_device(t, what)
    if t.dtype != torch.float32 or tuple(t.shape[2:]) != shape_tail or not t.is_contiguous():
        raise ValueError(f"{what} must be contiguous float32 [B,T+1,{','.join(map(str, shape_tail))}], "
                         f"got {tuple(t.shape)} {t.dtype}")
    return t


def traj_metrics(traj):
    """Metric series [B,T1,4] of trajectories [B,T1,3,nx] (hf_traj_metrics)."""
    require_device(traj, "traj")
    traj = traj.to(torch.float32).contiguous()
    B, T1, _, nx = traj.shape
    out = torch.empty(B, T1, HF_NUM_METRICS, device=traj.device)
    with torch.cuda.device(traj.device):
        check(lib().hf_traj_metrics(ptr(traj), B, T1, nx, ptr(out), stream_of(traj.device)))
    return out


def traj_mse(a, b):
    """Per-step channel MSE [B,T1,3] of two trajectories [B,T1,3,nx] (hf_traj_mse)."""
    require_device(a, "traj a")
    require_device(b, "traj b")
    a, b = a.to(torch.float32).contiguous(), b.to(device=a.device, dtype=torch.float32).contiguous()
    if a.shape != b.shape or a.dim() != 4 or a.shape[2] != 3:
        raise ValueError(f"trajectories must both be [B,T1,3,nx], got {tuple(a.shape)} and {tuple(b.shape)}")
    B, T1, _, nx = a.shape
    out = torch.empty(B, T1, 3, device=a.device)
    with torch.cuda.device(a.device):
        check(lib().hf_traj_mse(ptr(a), ptr(b), B, T1, nx, ptr(out), stream_of(a.device)))
    return out


def rollout_summary(metrics, mse=None, metrics_ref=None, drift=False):
    """hf_rollout_summary: (summary [B,8], drift [B,T+1,4] or None); fields in
    include/hybridflux.h (HF_NUM_SUMMARY)."""
    metrics = _series(metrics, (HF_NUM_METRICS,), "metrics")
    B, T1 = metrics.shape[:2]
    dev = metrics.device
    if mse is not None:
        mse = _series(mse, (3,), "mse")
    if metrics_ref is not None:
        metrics_ref = _series(metrics_ref, (HF_NUM_METRICS,), "metrics_ref")
    for o in (mse, metrics_ref):
        if o is not None and (o.shape[:2] != (B, T1) or o.device != dev):
            raise ValueError("metric series must share [B,T+1] and the device")
    summ = torch.empty(B, _lib.HF_NUM_SUMMARY, device=dev)
    dr = torch.empty(B, T1, 4, device=dev) if drift else None
    with torch.cuda.device(dev):
        check(lib().hf_rollout_summary(ptr(metrics), ptr(mse), ptr(metrics_ref), B, T1 - 1, ptr(summ), ptr(dr),
                                       stream_of(dev)))
    return summ, dr


def chain_batch(idx, state_t, flux_t, state_next, x):
    """hf_chain_batch_gather: a training batch of a device dataset
    (train_ablation.py:27-44, indexed by the batch) and its chain node
    features [n, u, E, x] (src/graph_constructor.py:6-39, batched) in one pass.
    idx [B] sample indices; state_t / state_next [N,3,nx], flux_t [N,nx]
    float32 device tensors; x [nx].  Returns (st [B,3,nx], ft [B,nx],
    sn [B,3,nx], node_features [B*nx,4])."""
    for t, what in ((state_t, "state_t"), (flux_t, "flux_t"), (state_next, "state_next")):
        require_device(t, what)
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"chain batch: {what} must be a contiguous float32 tensor")
    N, _, nx = state_t.shape
    dev = state_t.device
    if state_next.shape != state_t.shape or flux_t.shape != (N, nx):
        raise ValueError("chain batch: dataset shapes must be state [N,3,nx], flux_t [N,nx]")
    idx = torch.as_tensor(idx, device=dev).to(torch.long).reshape(-1).contiguous()
    x = torch.as_tensor(x, dtype=torch.float32, device=dev).reshape(-1).contiguous()
    if x.numel() != nx:
        raise ValueError("chain batch: x must hold nx positions")
    B = idx.numel()
    st = torch.empty(B, 3, nx, device=dev)
    ft = torch.empty(B, nx, device=dev)
    sn = torch.empty(B, 3, nx, device=dev)
    nf = torch.empty(B * nx, 4, device=dev)
    with torch.cuda.device(dev):
        check(lib().hf_chain_batch_gather(ptr(idx), B, ptr(state_t), ptr(flux_t), ptr(state_next), N, nx, ptr(x),
                                          ptr(st), ptr(ft), ptr(sn), ptr(nf), stream_of(dev)))
    return st, ft, sn, nf


def adam_flat(params, grads, exp_avg, exp_avg_sq, step, done, lr, beta1, beta2, eps):
    """hf_adam_flat: torch.optim.Adam's update on one flat float32 parameter
    buffer (train_ablation.py:208-209), the step count `step` (float32 [1]) on
    the device and incremented by the call; `done` a uint32-sized zeroed
    buffer the kernel leaves zero."""
    for t, what in ((params, "params"), (grads, "grads"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq"),
                    (step, "step"), (done, "done")):
        require_device(t, what)
        if not t.is_contiguous():
            raise ValueError(f"adam_flat: {what} must be contiguous")
    n = params.numel()
    if any(t.numel() != n or t.dtype != torch.float32 for t in (grads, exp_avg, exp_avg_sq)) or \
            params.dtype != torch.float32 or step.dtype != torch.float32 or step.numel() < 1 or done.numel() * \
            done.element_size() < 4:
        raise ValueError("adam_flat: float32 buffers of one size, a float32 step and a 4-byte done counter")
    dev = params.device
    with torch.cuda.device(dev):
        check(lib().hf_adam_flat(ptr(params), ptr(grads), ptr(exp_avg), ptr(exp_avg_sq), n, ptr(step), ptr(done),
                                 float(lr), float(beta1), float(beta2), float(eps), stream_of(dev)))


def ablation_loss_terms(grid, flux_edge, st, ft, sn, lam, rollout_steps=0, dt=None):
    """hf_ablation_loss_ex: the reference trainer's loss (scripts/training/
    train_ablation.py:120-206) for B samples.  flux_edge [B, 2nx], st / sn
    [B,3,nx], ft [B,nx] device tensors; lam = (lambda_state, lambda_poisson,
    lambda_charge, lambda_energy_one[, lambda_energy_multi]); with
    lambda_energy_multi > 0 and 0 < rollout_steps <= 3 the rollout energy term
    (:172-206) is formed in the same pass from the main forward's flux (no
    further model forward reaches it; include/hybridflux.h), with time step dt
    (default the grid's).  Returns (loss, flux MSE, d loss / d flux_edge [B, 2nx])."""
    for t, what in ((flux_edge, "flux_edge"), (st, "state_t"), (ft, "flux_t"), (sn, "state_next")):
        require_device(t, what)
    B, _, nx = st.shape
    dev = st.device
    fe = flux_edge.detach().to(torch.float32).contiguous()
    st, ft, sn = (t.to(torch.float32).contiguous() for t in (st, ft, sn))
    if fe.numel() != B * 2 * nx or ft.shape != (B, nx) or sn.shape != st.shape or nx != grid.nx:
        raise ValueError("ablation loss: shapes must be flux_edge [B,2nx], states [B,3,nx], flux_t [B,nx]")
    loss = torch.empty((), device=dev)
    fl = torch.empty((), device=dev)
    dfe = torch.empty(B, 2 * nx, device=dev)
    ws = torch.empty(int(lib().hf_ablation_loss_workspace_bytes(B, nx)), dtype=torch.uint8, device=dev)
    lam_h = np.zeros(5, dtype=np.float32)
    lam_h[:len(lam)] = np.asarray(lam, dtype=np.float32)
    dt32 = float(np.float32(grid.dt if dt is None else dt))
    pc = grid.spectral_plan(dev)
    with torch.cuda.device(dev):
        check(lib().hf_ablation_loss_ex(ptr(fe), ptr(st), ptr(ft), ptr(sn), B, nx, grid.c32,
                                        float(np.float32(grid.dx)), ptr(lam_h), int(rollout_steps), dt32, ptr(pc),
                                        ptr(loss), ptr(fl), ptr(dfe), ptr(ws), ws.numel(), stream_of(dev)))
    return loss, fl, dfe
