"""The reference's other rollout models on the MI355X.

PureGNN (scripts/training/train_pure_gnn.py:35-76) and PINN
(scripts/training/train_pinn.py:36-61) with the reference's module trees, so
their checkpoints load with load_state_dict unchanged, and forward()
signatures; inference runs in the HIP kernels of baselines.hip
(hf_pure_gnn_* / hf_pinn_*).  `rollout` batches the per-IC loops of
scripts/evaluation/evaluate_multi_ic.py:45-83 and benchmark_timing.py:100-203
over B initial conditions in one call.  forward() takes the reference's host
(CPU) tensors too (evaluate_multi_ic.py:53-83 calls them with
torch.FloatTensor states): they are staged to the current HIP device and the
result is copied back.  Inference only: these modules have no backward
kernels (the reference trains them with its own torch loops), so a forward
under autograd raises.
"""
import torch
import torch.nn as nn

from . import engine
from ._lib import check, lib, ptr


def _flat(module):
    return torch.cat([p.detach().reshape(-1).to(torch.float32) for p in module.parameters()]).contiguous()


def _no_grad_guard(module, *inputs):
    if torch.is_grad_enabled() and (any(p.requires_grad for p in module.parameters()) or
                                    any(getattr(t, "requires_grad", False) for t in inputs)):
        raise NotImplementedError(f"{type(module).__name__}: inference kernels only; wrap calls in torch.no_grad()")


class _Flat:
    """Flat device copy of a module's parameters, rebuilt when any changes."""

    def __init__(self):
        self.sig, self.buf = None, None

    def get(self, module, device):
        sig = (str(device),) + tuple((p.data_ptr(), p._version) for p in module.parameters())
        if sig != self.sig:
            self.buf = _flat(module).to(device)
            self.sig = sig
        return self.buf


class PureGNN(nn.Module):
    """End-to-end GNN predicting the state change per node (train_pure_gnn.py:35-76)."""

    def __init__(self, input_dim=4, hidden_dim=64, num_layers=3):
        super().__init__()
        self.input_dim, self.hidden_dim, self.num_layers = input_dim, hidden_dim, num_layers
        self.input_mlp = nn.Sequential(nn.Linear(input_dim, hidden_dim), nn.Tanh())
        self.update_mlps = nn.ModuleList(
            [nn.Sequential(nn.Linear(hidden_dim * 2, hidden_dim), nn.Tanh()) for _ in range(num_layers)])
        self.output_mlp = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.Tanh(), nn.Linear(hidden_dim, 3))
        self._flat = _Flat()

    def forward(self, node_features, edge_index):
        """node_features [N, input_dim], edge_index [2, E] -> delta_state [N, 3]."""
        _no_grad_guard(self, node_features)
        home = node_features.device
        dev = engine.compute_device(node_features, "node_features")
        nf, ei, N, E, chain_nx = engine._graph_inputs(node_features.to(dev), edge_index, self.input_dim)
        delta = torch.empty(N, 3, device=nf.device)
        H = self.hidden_dim
        ws = torch.empty(int(lib().hf_pure_gnn_workspace_bytes(H, N, E)), dtype=torch.uint8, device=nf.device)
        with torch.cuda.device(nf.device):
            check(lib().hf_pure_gnn_forward(ptr(self._flat.get(self, nf.device)), self.input_dim, H,
                                            self.num_layers, ptr(nf), N, ptr(ei), E, chain_nx, ptr(delta), ptr(ws),
                                            engine.stream_of(nf.device)))
        return delta.to(home)

    def rollout(self, states0, n_steps, x, traj=True):
        """B ICs [B,3,nx] (device) -> dict(final [B,3,nx], traj [B,T+1,3,nx] or None);
        the loop of evaluate_multi_ic.py:53-64 with node features [n,u,E,x]."""
        if self.input_dim != 4:
            raise ValueError("rollout builds [n,u,E,x] node features: input_dim must be 4")
        engine.require_device(states0, "states0")
        s0 = states0.to(torch.float32).contiguous()
        B, _, nx = s0.shape
        xd = torch.as_tensor(x, dtype=torch.float32, device=s0.device).contiguous()
        final = torch.empty_like(s0)
        tr = torch.empty(B, n_steps + 1, 3, nx, device=s0.device) if traj else None
        N = B * nx
        nb = int(lib().hf_pure_gnn_run_workspace_bytes(self.hidden_dim, B, nx, int(n_steps)))
        ws = torch.empty(nb, dtype=torch.uint8, device=s0.device) if nb > 0 else None
        with torch.no_grad(), torch.cuda.device(s0.device):
            check(lib().hf_pure_gnn_run(ptr(self._flat.get(self, s0.device)), self.hidden_dim, self.num_layers,
                                        ptr(s0), ptr(final), ptr(xd), B, nx, int(n_steps),
                                        ptr(tr) if tr is not None else None, ptr(ws) if ws is not None else None,
                                        engine.stream_of(s0.device)))
        return {"final": final, "traj": tr}


class PINN(nn.Module):
    """MLP on the flattened state predicting the next state (train_pinn.py:36-61)."""

    def __init__(self, input_dim=3 * 64, hidden_dim=256, num_layers=4):
        super().__init__()
        layers = [nn.Linear(input_dim, hidden_dim), nn.Tanh()]
        for _ in range(num_layers - 2):
            layers += [nn.Linear(hidden_dim, hidden_dim), nn.Tanh()]
        layers.append(nn.Linear(hidden_dim, input_dim))
        self.net = nn.Sequential(*layers)
        self.input_dim, self.hidden_dim, self.num_layers = input_dim, hidden_dim, num_layers
        self._flat = _Flat()

    def forward(self, state):
        """state [..., 3, nx] -> state + delta, same shape."""
        _no_grad_guard(self, state)
        dev = engine.compute_device(state, "state")
        s = state.to(device=dev, dtype=torch.float32).contiguous()
        flat = s.reshape(-1, self.input_dim)
        out = torch.empty_like(flat)
        B = flat.shape[0]
        nb = int(lib().hf_pinn_workspace_bytes(self.input_dim, self.hidden_dim, B))
        ws = torch.empty(nb, dtype=torch.uint8, device=s.device) if nb > 0 else None
        with torch.cuda.device(s.device):
            check(lib().hf_pinn_forward(ptr(self._flat.get(self, s.device)), self.input_dim, self.hidden_dim,
                                        self.num_layers, ptr(flat), ptr(out), B, ptr(ws) if ws is not None else None,
                                        engine.stream_of(s.device)))
        return out.reshape(state.shape).to(state.device)

    def rollout(self, states0, n_steps, traj=True):
        """B ICs [B,3,nx] -> dict(final, traj [B,T+1,3,nx] or None) (evaluate_multi_ic.py:75-81)."""
        engine.require_device(states0, "states0")
        s0 = states0.to(torch.float32).contiguous()
        B = s0.shape[0]
        if s0[0].numel() != self.input_dim:
            raise ValueError(f"states0 must hold {self.input_dim} values per IC")
        final = torch.empty_like(s0)
        tr = torch.empty((B, n_steps + 1) + tuple(s0.shape[1:]), device=s0.device) if traj else None
        nb = int(lib().hf_pinn_workspace_bytes(self.input_dim, self.hidden_dim, B))
        ws = torch.empty(nb, dtype=torch.uint8, device=s0.device) if nb > 0 else None
        with torch.no_grad(), torch.cuda.device(s0.device):
            check(lib().hf_pinn_run(ptr(self._flat.get(self, s0.device)), self.input_dim, self.hidden_dim,
                                    self.num_layers, ptr(s0), ptr(final), B, int(n_steps),
                                    ptr(tr) if tr is not None else None, ptr(ws) if ws is not None else None,
                                    engine.stream_of(s0.device)))
        return {"final": final, "traj": tr}
