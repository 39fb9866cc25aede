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
grads.npz             autograd of the reference FluxGNN (src/flux_gnn.py:40-67):
                      d(sum g*flux)/d(params, node_features) for seeded g on the
                      two random graphs above; and the ablation training loss
                      (scripts/training/train_ablation.py:107-206, 'full' config)
                      with its parameter gradients on three chain samples of the
                      classical fixture, W1_r1 weights; and a 6-step batch-size-1
                      Adam run ('physics' config, fixed sample order): per-step
                      losses and final weights.

baselines.npz         the reference's other rollout models:
                      PureGNN(4,128,4) (seed 11) and PINN(192,256,4) (seed 12)
                      from scripts/training/train_pure_gnn.py:35-76 and
                      train_pinn.py:36-61 — their weights, PureGNN on a random
                      graph, and 10-step rollouts of ICs 1000..1003 with the
                      loops of scripts/evaluation/evaluate_multi_ic.py:45-83.

smoke_test.npz        examples/smoke_test.py's own call sequence, verbatim, on the
                      CPU: test_graph_constructor (:30-42, np.random.seed(s)
                      first) and test_flux_gnn (:45-58: torch.manual_seed(s),
                      FluxGNN(4,64,3) built on the CPU, grad enabled,
                      torch.randn node features and a torch.randint
                      edge_index) for s in 0, 1, 2 — the fluxes, and the
                      gradients of sum(flux) w.r.t. the parameters; plus
                      FluxGNN(4,128,4)=W1_r1 on build_chain_graph(IC 1000, x,
                      'cpu') under grad (the trainer's call, train_ablation.py:
                      119-124) with d sum(flux)/d params.

metrics.npz           the reference's rollout scoring:
                      evaluate_all.compute_metrics (scripts/evaluation/
                      evaluate_all.py:118-159) of the hybrid W1_r1 rollouts of
                      hybrid_W1_r1_nx64.npz against the classical ones of
                      classical.npz (seeds 1000..1015, T=30);
                      evaluate_multi_ic.evaluate_model_on_ic('hybrid', W1_r1, 1,
                      seed, 30) for the same seeds (evaluate_multi_ic.py:21-94);
                      evaluate_long_rollout.evaluate_long_rollout (evaluate_long_
                      rollout.py:18-81) on seed 2000 for W1_r1 (300 steps) and for
                      W1_r1 with edge_mlp.2.weight scaled x30 (100 steps) and x100
                      (60 steps): exploded_at, actual_steps, the drift series.
                      Those scripts build HybridSolver(path, r) with the
                      reference's default device='cuda'; they are run with the
                      class bound to device='cpu' (this container has no GPU).

    python tests/golden/make_golden.py grads       # regenerate grads.npz only
    python tests/golden/make_golden.py baselines   # regenerate baselines.npz only
    python tests/golden/make_golden.py metrics     # regenerate metrics.npz only
    python tests/golden/make_golden.py smoke       # regenerate smoke_test.npz only
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


def ref_training_loss(model, st, ft, st_next, x, dt, dx, cfg):
    """The per-sample loss of scripts/training/train_ablation.py:107-200, with the
    reference's own FluxGNN / build_chain_graph / solve_poisson_np."""
    from train_ablation import solve_poisson_np
    mse = torch.nn.MSELoss()
    n0 = 1.0
    n_t, u_t = st[0], st[1]
    n_next_true, u_next_true, E_next_true = st_next[0], st_next[1], st_next[2]
    node_features, edge_index = build_chain_graph(st, x, device="cpu")
    flux_edge = model(node_features, edge_index)
    nx_loc = n_t.shape[0]
    F_pred = 0.5 * (flux_edge[:nx_loc] + flux_edge[nx_loc:])
    flux_loss = mse(F_pred, ft)
    loss = flux_loss
    n_next_pred = n_t - (dt / dx) * (F_pred - torch.roll(F_pred, 1))
    if cfg["lambda_state"] > 0:
        loss = loss + cfg["lambda_state"] * mse(n_next_pred, n_next_true)
    if cfg["lambda_poisson"] > 0:
        E_pred = torch.from_numpy(solve_poisson_np(n_next_pred.detach().numpy(), n0, dx))
        loss = loss + cfg["lambda_poisson"] * mse(E_pred, E_next_true)
    if cfg["lambda_charge"] > 0:
        charge_t = torch.sum(n_t - n0) * dx
        charge_next_pred = torch.sum(n_next_pred - n0) * dx
        loss = loss + cfg["lambda_charge"] * mse(charge_next_pred, charge_t)
    if cfg["lambda_energy_one"] > 0:
        E_pred = torch.from_numpy(solve_poisson_np(n_next_pred.detach().numpy(), n0, dx))
        e_p = 0.5 * torch.mean(u_next_true ** 2 + E_pred ** 2)
        e_t = 0.5 * torch.mean(u_next_true ** 2 + E_next_true ** 2)
        loss = loss + cfg["lambda_energy_one"] * mse(e_p, e_t)
    if cfg["rollout_steps"] > 0 and cfg["lambda_energy_multi"] > 0:
        state_roll = st.clone()
        energies = []
        for _ in range(cfg["rollout_steps"]):
            n_r, u_r, E_r = state_roll[0], state_roll[1], state_roll[2]
            energies.append(0.5 * torch.mean(u_r ** 2))
            nf_r, ei_r = build_chain_graph(state_roll, x, device="cpu")
            fe_r = model(nf_r, ei_r)
            F_r = 0.5 * (fe_r[:nx_loc] + fe_r[nx_loc:])
            n_next_r = n_r - (dt / dx) * (F_r - torch.roll(F_r, 1))
            F_u = 0.5 * u_r * u_r
            u_next_r = u_r - (dt / dx) * (F_u - torch.roll(F_u, 1)) + dt * E_r
            E_next_r = torch.from_numpy(solve_poisson_np(n_next_r.detach().numpy(), n0, dx))
            state_roll = torch.stack([n_next_r, u_next_r, E_next_r], dim=0)
        energies = torch.stack(energies)
        loss = loss + cfg["lambda_energy_multi"] * torch.mean((energies - energies[0]) ** 2)
    return loss, flux_loss


def make_grads():
    from src.config import ABLATION_CONFIGS
    arrs = {}
    rnd = np.load(OUT / "fluxgnn_random.npz")
    g = torch.Generator().manual_seed(9)
    # (1) random graphs: d(sum g*flux)
    small = FluxGNN(input_dim=4, hidden_dim=64, num_layers=3)
    small.load_state_dict({k[len("small."):]: torch.from_numpy(rnd[k]) for k in rnd.files if k.startswith("small.")})
    w0 = np.load(OUT / "weights_W0.npz")
    big = FluxGNN(input_dim=4, hidden_dim=128, num_layers=4)
    big.load_state_dict({k: torch.from_numpy(w0[k]) for k in w0.files})
    for tag, m in (("small", small), ("big", big)):
        nf = torch.from_numpy(rnd[f"{tag}_nf"]).clone().requires_grad_(True)
        ei = torch.from_numpy(rnd[f"{tag}_ei"])
        flux = m(nf, ei)
        gg = torch.randn(flux.shape[0], generator=g)
        m.zero_grad()
        (flux * gg).sum().backward()
        arrs[f"{tag}_g"] = gg.numpy()
        arrs[f"{tag}_grad_nf"] = nf.grad.numpy()
        for k, p in m.named_parameters():
            arrs[f"{tag}_grad.{k}"] = p.grad.numpy()
    # (2) ablation loss on chain samples (classical fixture seeds 1000.., steps t -> t+1)
    cl = np.load(OUT / "classical.npz")
    S, F = cl["b16_states"], cl["b16_fluxes"]
    solver = BaselineSolver(nx=64)
    x = solver.x
    w1 = np.load(OUT / "weights_W1_r1.npz")
    model = FluxGNN(input_dim=4, hidden_dim=128, num_layers=4)
    model.load_state_dict({k: torch.from_numpy(w1[k]) for k in w1.files})
    picks = [(0, 0), (3, 11), (9, 29)]
    for j, (ic, t) in enumerate(picks):
        st, ft, sn = (torch.from_numpy(S[ic, t]), torch.from_numpy(F[ic, t]), torch.from_numpy(S[ic, t + 1]))
        model.zero_grad()
        loss, fl = ref_training_loss(model, st, ft, sn, x, solver.dt, solver.dx, ABLATION_CONFIGS["full"])
        loss.backward()
        arrs[f"loss{j}_value"] = np.float32(loss.item())
        arrs[f"loss{j}_flux"] = np.float32(fl.item())
        for k, p in model.named_parameters():
            arrs[f"loss{j}_grad.{k}"] = p.grad.numpy()
    arrs["loss_picks"] = np.array(picks)
    # (3) 6 Adam steps, batch size 1, 'physics' config, fixed order          (train_ablation.py:87-210)
    model.load_state_dict({k: torch.from_numpy(w1[k]) for k in w1.files})
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    order = [(1, 4), (7, 20), (2, 2), (12, 8), (5, 27), (14, 15)]
    losses = []
    for ic, t in order:
        st, ft, sn = (torch.from_numpy(S[ic, t]), torch.from_numpy(F[ic, t]), torch.from_numpy(S[ic, t + 1]))
        loss, _ = ref_training_loss(model, st, ft, sn, x, solver.dt, solver.dx, ABLATION_CONFIGS["physics"])
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    arrs["adam_order"] = np.array(order)
    arrs["adam_losses"] = np.array(losses, dtype=np.float64)
    arrs.update({f"adam_final.{k}": v for k, v in sd_to_np(model.state_dict()).items()})
    save("grads.npz", **arrs)


def make_baselines():
    from train_pure_gnn import PureGNN
    from train_pinn import PINN
    arrs = {}
    solver = BaselineSolver(nx=64)
    x = solver.x
    seeds = [1000, 1001, 1002, 1003]
    ics = np.stack([solver.initial_condition(seed=s) for s in seeds])
    torch.manual_seed(11)
    pg = PureGNN(input_dim=4, hidden_dim=128, num_layers=4).eval()
    torch.manual_seed(12)
    pinn = PINN(input_dim=3 * 64, hidden_dim=256, num_layers=4).eval()
    arrs.update({f"pure_gnn.{k}": v for k, v in sd_to_np(pg.state_dict()).items()})
    arrs.update({f"pinn.{k}": v for k, v in sd_to_np(pinn.state_dict()).items()})
    x_torch = torch.FloatTensor(x)
    traj_g, traj_p = [], []
    with torch.no_grad():
        for ic in ics:                       # evaluate_multi_ic.py:45-66
            state = ic.copy()
            st = [state.copy()]
            for _ in range(10):
                _, edge_index = build_chain_graph(state, x, "cpu")
                nf = torch.FloatTensor(state).permute(1, 0)
                nf = torch.cat([nf, x_torch.unsqueeze(1)], dim=1)
                delta = pg(nf, edge_index)
                state = (torch.FloatTensor(state).permute(1, 0) + delta).permute(1, 0).numpy()
                st.append(state.copy())
            traj_g.append(np.array(st))
        for ic in ics:                       # evaluate_multi_ic.py:70-83
            state = ic.copy()
            st = [state.copy()]
            for _ in range(10):
                state = pinn(torch.FloatTensor(state).unsqueeze(0))[0].numpy()
                st.append(state.copy())
            traj_p.append(np.array(st))
        g = torch.Generator().manual_seed(13)
        nf = torch.randn(50, 4, generator=g)
        ei = torch.randint(0, 50, (2, 170), generator=g)
        arrs["pure_gnn_graph_nf"], arrs["pure_gnn_graph_ei"] = nf.numpy(), ei.numpy()
        arrs["pure_gnn_graph_delta"] = pg(nf, ei).numpy()
        batch = torch.from_numpy(ics[:3])
        arrs["pinn_batch_out"] = pinn(batch).numpy()   # batched forward, [3,3,64]
    arrs["seeds"] = np.array(seeds)
    arrs["ics"] = ics
    arrs["pure_gnn_traj"] = np.stack(traj_g).astype(np.float32)
    arrs["pinn_traj"] = np.stack(traj_p).astype(np.float32)
    save("baselines.npz", **arrs)


SMOKE_SEEDS = (0, 1, 2)


def make_smoke():
    arrs = {}
    for s in SMOKE_SEEDS:
        np.random.seed(s)                                   # smoke_test.py:35-38
        state = np.random.randn(3, 64)
        x = np.linspace(0, 1, 64)
        nf, ei = build_chain_graph(state, x, "cpu")
        arrs[f"graph{s}_state"], arrs[f"graph{s}_nf"], arrs[f"graph{s}_ei"] = state, nf.numpy(), ei.numpy()
        torch.manual_seed(s)                                # smoke_test.py:50-55, grad enabled
        model = FluxGNN(input_dim=4, hidden_dim=64, num_layers=3)
        node_features = torch.randn(64, 4)
        edge_index = torch.randint(0, 64, (2, 128))
        fluxes = model(node_features, edge_index)
        fluxes.sum().backward()
        arrs[f"flux{s}"] = fluxes.detach().numpy()
        arrs[f"flux{s}_nf"], arrs[f"flux{s}_ei"] = node_features.numpy(), edge_index.numpy()
        arrs.update({f"flux{s}_w.{k}": v for k, v in sd_to_np(model.state_dict()).items()})
        arrs.update({f"flux{s}_grad.{k}": p.grad.numpy() for k, p in model.named_parameters()})
    w1 = np.load(OUT / "weights_W1_r1.npz")
    model = FluxGNN(input_dim=4, hidden_dim=128, num_layers=4)
    model.load_state_dict({k: torch.from_numpy(w1[k]) for k in w1.files})
    solver = BaselineSolver(nx=64)
    st = solver.initial_condition(seed=1000)
    nf, ei = build_chain_graph(st, solver.x, device="cpu")
    fe = model(nf, ei)
    fe.sum().backward()
    arrs["chain_flux"] = fe.detach().numpy()
    arrs.update({f"chain_grad.{k}": p.grad.numpy() for k, p in model.named_parameters()})
    arrs["seeds"] = np.array(SMOKE_SEEDS)
    save("smoke_test.npz", **arrs)


LONG_ROLLOUTS = ((1.0, 300), (30.0, 100), (100.0, 60))  # (edge_mlp.2.weight scale, steps), seed 2000


def make_metrics():
    import functools

    sys.path.insert(0, str(REF / "scripts" / "evaluation"))
    import evaluate_all
    import evaluate_long_rollout
    import evaluate_multi_ic

    cpu_solver = functools.partial(HybridSolver, device="cpu")
    evaluate_long_rollout.HybridSolver = cpu_solver
    evaluate_multi_ic.HybridSolver = cpu_solver
    arrs = {}
    hyb = np.load(OUT / "hybrid_W1_r1_nx64.npz")
    cla = np.load(OUT / "classical.npz")
    assert list(hyb["seeds"]) == list(range(1000, 1016))
    per_ic = [evaluate_all.compute_metrics(hyb["states"][i], cla["b16_states"][i]) for i in range(16)]
    for k in per_ic[0]:
        arrs[f"cm_{k}"] = np.array([m[k] for m in per_ic], dtype=np.float64)
    w1 = np.load(OUT / "weights_W1_r1.npz")
    with tempfile.TemporaryDirectory() as wd:
        pt = os.path.join(wd, "W1_r1.pt")
        write_pt(OUT / "weights_W1_r1.npz", pt)
        arrs["multi_ic_seeds"] = np.arange(1000, 1016)
        arrs["multi_ic_mse"] = np.array([evaluate_multi_ic.evaluate_model_on_ic("hybrid", pt, 1, s, 30)
                                         for s in range(1000, 1016)])
        for i, (scale, steps) in enumerate(LONG_ROLLOUTS):
            p = os.path.join(wd, f"scaled{i}.pt")
            sd = {k: torch.from_numpy(w1[k].copy()) for k in w1.files}
            sd["edge_mlp.2.weight"] = sd["edge_mlp.2.weight"] * scale
            torch.save(sd, p)
            r = evaluate_long_rollout.evaluate_long_rollout(p, 1, 2000, n_steps=steps)
            drift = np.full(steps + 1, np.nan)
            drift[: len(r["energy_drift_pred"])] = r["energy_drift_pred"]
            base = np.array(r["energy_drift_baseline"])
            arrs[f"long{i}_scale"] = np.float32(scale)
            arrs[f"long{i}_steps"] = np.int64(steps)
            arrs[f"long{i}_exploded_at"] = np.int64(-1 if r["exploded_at"] is None else r["exploded_at"])
            arrs[f"long{i}_actual_steps"] = np.int64(r["actual_steps"])
            arrs[f"long{i}_energy_drift_pred"] = drift
            arrs[f"long{i}_energy_drift_baseline"] = base
    save("metrics.npz", **arrs)


def main():
    if sys.argv[1:] == ["metrics"]:
        make_metrics()
        return
    if sys.argv[1:] == ["smoke"]:
        make_smoke()
        return
    if sys.argv[1:] == ["grads"]:
        make_grads()
        return
    if sys.argv[1:] == ["baselines"]:
        make_baselines()
        return
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
        make_grads()
        make_baselines()
        make_metrics()
        make_smoke()
    meta = {"torch": torch.__version__, "numpy": np.__version__,
            "reference": "shanedirksen/gnn-plasma-flux @ /root/reference (2026-01-02 snapshot)",
            "generator": "tests/golden/make_golden.py"}
    (OUT / "meta.json").write_text(json.dumps(meta, indent=2) + "\n")


if __name__ == "__main__":
    main()
