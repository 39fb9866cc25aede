"""Generate the golden fixtures for the hybrid-rollout hot path FROM THE REFERENCE.

Runs ONLY in the build container (where /root/reference exists); the GPU box
never sees the reference, only the .npz files this script writes next to it.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it records (all float32 unless noted; versions in `meta.json`):

weights_W0.npz        torch.manual_seed(0); FluxGNN(4,128,4) default init
                      (src/flux_gnn.py:11-38 state-dict keys, verbatim).
weights_W1_r{1,2,3}   the reference's own trainer, 1 epoch, 'baseline' loss,
                      on the reference's own generated dataset
                      (scripts/training/train_ablation.py:64-237,
                      scripts/training/generate_data.py:12-54); seed = r.
ics.npz               BaselineSolver.initial_condition(seed) for
                      seeds {0,42,123,1000..1015,2000} at nx=64 and
                      seeds {1000..1003} at nx=1024 (src/baseline_solver.py:29-57).
poisson.npz           BaselineSolver.solve_poisson on seeded random densities
                      at nx in {16,32,48,64,1024} (src/baseline_solver.py:59-68).
classical.npz         BaselineSolver.run (states + F_n) : seed 0, T=30 (config 1);
                      seeds 1000..1015 T=30 at nx=64; seeds 1000,1001 T=30 at
                      nx=1024, dt=3.125e-4 (src/baseline_solver.py:80-118).
hybrid_<W>_nx64.npz   HybridSolver(.., device='cpu').step per IC, seeds
                      1000..1015, T=30, recording states and the per-step
                      FluxGNN edge fluxes (src/hybrid_solver.py:34-73).
hybrid_W1_r2_nx1024   same at nx=1024, dt=3.125e-4, seeds 1000..1003.
fluxgnn_random.npz    FluxGNN(4,64,3) (seed 7) on random node features and a
                      random edge_index, as examples/smoke_test.py:45-56 does,
                      plus FluxGNN(4,128,4)=W0 on a random graph.
"""
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.dont_write_bytecode = True
sys.path.insert(0, str(REF / "src"))          # hybrid_solver.py:21 does `from config import`
sys.path.insert(0, str(REF))
sys.path.insert(0, str(REF / "scripts" / "training"))

import torch  # noqa: E402

torch.set_num_threads(8)

from src.baseline_solver import BaselineSolver  # noqa: E402
from src.flux_gnn import FluxGNN  # noqa: E402
from src.graph_constructor import build_chain_graph  # noqa: E402
from src.hybrid_solver import HybridSolver  # noqa: E402
from src.config import DATASET_CONFIG  # noqa: E402


def sd_to_np(sd):
    return {k: v.detach().cpu().numpy().astype(np.float32) for k, v in sd.items()}


def save(name, **arrays):
    np.savez_compressed(OUT / name, **arrays)
    print("wrote", name, {k: getattr(v, "shape", None) for k, v in arrays.items()})


def make_weights(workdir):
    torch.manual_seed(0)
    w0 = FluxGNN(input_dim=4, hidden_dim=128, num_layers=4)
    save("weights_W0.npz", **sd_to_np(w0.state_dict()))

    from generate_data import generate_dataset
    import train_ablation

    cwd = os.getcwd()
    os.chdir(workdir)
    try:
        torch.manual_seed(0)
        st, ft, sn, x, dt, dx, nu = generate_dataset(**DATASET_CONFIG)
        out = {}
        for r in (1, 2, 3):
            torch.manual_seed(r)
            model, _ = train_ablation.train_model(st, ft, sn, x, dt, dx, nu,
                                                  config_name="baseline", stencil_radius=r,
                                                  epochs=1, lr=1e-3, device="cpu")
            save(f"weights_W1_r{r}.npz", **sd_to_np(model.state_dict()))
            out[r] = os.path.join(workdir, f"checkpoints/hybrid_baseline_r{r}.pt")
    finally:
        os.chdir(cwd)
    return out


def write_pt(npz_path, pt_path):
    d = np.load(npz_path)
    torch.save({k: torch.from_numpy(d[k]) for k in d.files}, pt_path)


def make_ics():
    s64 = BaselineSolver(nx=64)
    seeds64 = [0, 42, 123] + list(range(1000, 1016)) + [2000]
    ic64 = np.stack([s64.initial_condition(seed=s) for s in seeds64])
    s1k = BaselineSolver(nx=1024, dt=3.125e-4)
    seeds1k = list(range(1000, 1004))
    ic1k = np.stack([s1k.initial_condition(seed=s) for s in seeds1k])
    save("ics.npz", seeds_nx64=np.array(seeds64), ics_nx64=ic64,
         seeds_nx1024=np.array(seeds1k), ics_nx1024=ic1k,
         x_nx64=s64.x, x_nx1024=s1k.x)


def make_poisson():
    rng = np.random.RandomState(11)
    arrs = {}
    for nx in (16, 32, 48, 64, 1024):
        s = BaselineSolver(nx=nx)
        n = (1.0 + 0.3 * rng.randn(6, nx)).astype(np.float32)
        E = np.stack([s.solve_poisson(v) for v in n])
        arrs[f"n_nx{nx}"] = n
        arrs[f"E_nx{nx}"] = E
    save("poisson.npz", **arrs)


def make_classical():
    arrs = {}
    s = BaselineSolver(nx=64)
    st, fl = s.run(s.initial_condition(seed=0), n_steps=30, record_flux=True)
    arrs["seed0_states"], arrs["seed0_fluxes"] = st, fl
    S, F = [], []
    for seed in range(1000, 1016):
        st, fl = s.run(s.initial_condition(seed=seed), n_steps=30, record_flux=True)
        S.append(st)
        F.append(fl)
    arrs["b16_states"], arrs["b16_fluxes"] = np.stack(S), np.stack(F)
    s1k = BaselineSolver(nx=1024, dt=3.125e-4)
    S, F = [], []
    for seed in (1000, 1001):
        st, fl = s1k.run(s1k.initial_condition(seed=seed), n_steps=30, record_flux=True)
        S.append(st)
        F.append(fl)
    arrs["nx1024_states"], arrs["nx1024_fluxes"] = np.stack(S), np.stack(F)
    save("classical.npz", **arrs)


def hybrid_traj(pt_path, radius, nx, dt, seeds, T):
    solver = HybridSolver(pt_path, radius, nx=nx, dt=dt, device="cpu")
    S, FL = [], []
    for seed in seeds:
        state = solver.baseline.initial_condition(seed=seed)
        states, fluxes = [state.astype(np.float32)], []
        for _ in range(T):
            nf, ei = build_chain_graph(state, solver.baseline.x)
            with torch.no_grad():
                fluxes.append(solver.model(nf, ei).numpy())
            state = solver.step(state)
            states.append(state)
        S.append(np.stack(states))
        FL.append(np.stack(fluxes))
    return np.stack(S), np.stack(FL)


def make_hybrid(pts):
    seeds = list(range(1000, 1016))
    for name, (pt, r) in pts.items():
        S, FL = hybrid_traj(pt, r, 64, 5e-3, seeds, 30)
        save(f"hybrid_{name}_nx64.npz", seeds=np.array(seeds), states=S, flux_edge=FL)
    S, FL = hybrid_traj(pts["W1_r2"][0], 2, 1024, 3.125e-4, [1000, 1001, 1002, 1003], 30)
    save("hybrid_W1_r2_nx1024.npz", seeds=np.array([1000, 1001, 1002, 1003]),
         states=S, flux_edge=FL[:, :4])  # per-step edge fluxes only for the first 4 steps


def make_random_graph():
    arrs = {}
    torch.manual_seed(7)
    m = FluxGNN(input_dim=4, hidden_dim=64, num_layers=3)
    g = torch.Generator().manual_seed(8)
    nf = torch.randn(64, 4, generator=g)
    ei = torch.randint(0, 64, (2, 128), generator=g)
    with torch.no_grad():
        arrs["small_flux"] = m(nf, ei).numpy()
    arrs.update({f"small.{k}": v for k, v in sd_to_np(m.state_dict()).items()})
    arrs["small_nf"], arrs["small_ei"] = nf.numpy(), ei.numpy()
    w0 = np.load(OUT / "weights_W0.npz")
    big = FluxGNN(input_dim=4, hidden_dim=128, num_layers=4)
    big.load_state_dict({k: torch.from_numpy(w0[k]) for k in w0.files})
    nf = torch.randn(200, 4, generator=g)
    ei = torch.randint(0, 200, (2, 700), generator=g)
    with torch.no_grad():
        arrs["big_flux"] = big(nf, ei).numpy()
    arrs["big_nf"], arrs["big_ei"] = nf.numpy(), ei.numpy()
    save("fluxgnn_random.npz", **arrs)


def main():
    with tempfile.TemporaryDirectory() as wd:
        make_weights(wd)
        pts = {}
        for name in ("W0", "W1_r1", "W1_r2", "W1_r3"):
            p = os.path.join(wd, f"{name}.pt")
            write_pt(OUT / f"weights_{name}.npz", p)
            pts[name] = (p, 1 if name == "W0" else int(name[-1]))
        make_ics()
        make_poisson()
        make_classical()
        make_hybrid(pts)
        make_random_graph()
    meta = {"torch": torch.__version__, "numpy": np.__version__,
            "reference": "shanedirksen/gnn-plasma-flux @ /root/reference (2026-01-02 snapshot)",
            "generator": "tests/golden/make_golden.py"}
    (OUT / "meta.json").write_text(json.dumps(meta, indent=2) + "\n")


if __name__ == "__main__":
    main()
