"""GPU parity of the differentiable path: FluxGNN forward +
HIP backward kernels (hf_graph_forward_train / hf_graph_backward) against the
reference's own autograd (tests/golden/grads.npz, made by make_golden.py from
src/flux_gnn.py and scripts/training/train_ablation.py) and the CPU oracle.

Tolerances: gradients are float32 sums over ~10^4 terms in a different order
than the CPU BLAS, so each tensor is compared at
  |got - ref| <= 2e-5 * max|ref| + 1e-9
(the reference's own fp32 gradient differs from an fp64 evaluation at the
1e-6 relative level).  Loss values: rtol 1e-5.  Six Adam steps: per-step loss
rtol 1e-4; weights atol 2e-5 (Adam's first steps move each weight by ~lr
whatever the gradient's size, so ulp-level gradient noise on tiny components
can show up at lr scale on a handful of them: at most 0.1 % may exceed it, by
no more than 2*lr).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import hybrid_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
REL = 2e-5


def grads_close(got, want, rel=REL):
    got = got.detach().cpu().numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
    scale = float(np.abs(want).max())
    err = float(np.abs(got.astype(np.float64) - want).max())
    assert err <= rel * scale + 1e-9, (err, scale)


@pytest.fixture(scope="module")
def hf():
    import hybridflux
    return hybridflux


def load(hf, sd, dims):
    m = hf.FluxGNN(*dims)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    return m.to(DEV)


def random_graph_model(hf, tag):
    rnd = golden("fluxgnn_random.npz")
    if tag == "small":
        return load(hf, {k[6:]: rnd[k] for k in rnd.files if k.startswith("small.")}, (4, 64, 3)), rnd
    w0 = golden("weights_W0.npz")
    return load(hf, {k: w0[k] for k in w0.files}, (4, 128, 4)), rnd


@pytest.mark.parametrize("tag", ["small", "big"])
def test_backward_random_graph_vs_reference(hf, tag):
    """d(sum g*flux)/d(params, node_features) == the reference's autograd."""
    g = golden("grads.npz")
    m, rnd = random_graph_model(hf, tag)
    nf = torch.as_tensor(rnd[f"{tag}_nf"], device=DEV).requires_grad_(True)
    ei = torch.as_tensor(rnd[f"{tag}_ei"], device=DEV)
    flux = m(nf, ei)
    assert flux.requires_grad
    grads_close(flux, rnd[f"{tag}_flux"], 1e-5)
    (flux * torch.as_tensor(g[f"{tag}_g"], device=DEV)).sum().backward()
    grads_close(nf.grad, g[f"{tag}_grad_nf"])
    for k, p in m.named_parameters():
        grads_close(p.grad, g[f"{tag}_grad.{k}"])


def test_backward_deterministic_and_chain_batch_vs_oracle(hf):
    """Batched chains (8 ICs x 64 cells, W1_r2): gradients equal torch-CPU autograd
    of the oracle, both on the chain training path (tagged edge_index,
    train_chain.hip) and on the generic CSR path (an untagged copy); two
    backward passes of the chain path are bitwise identical."""
    w = golden("weights_W1_r2.npz")
    sd = {k: w[k] for k in w.files}
    m = load(hf, sd, (4, 128, 4))
    h = golden("hybrid_W1_r2_nx64.npz")
    states = h["states"][:8, 5]
    x = hf.BaselineSolver(64, device=DEV).x
    gup = torch.randn(8 * 128, generator=torch.Generator().manual_seed(4))
    runs = []
    for _ in range(2):
        m.zero_grad()
        nf, ei = hf.build_chain_graph_batch(states, x, DEV)
        (m(nf, ei) * gup.to(DEV)).sum().backward()
        runs.append({k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()})
    m.zero_grad()
    nf, ei = hf.build_chain_graph_batch(states, x, DEV)
    (m(nf, ei.clone()) * gup.to(DEV)).sum().backward()   # untagged copy: generic CSR build
    runs.append({k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()})
    for k in runs[0]:
        assert np.array_equal(runs[0][k], runs[1][k]), k
    p = {k: v.clone().requires_grad_(True) for k, v in O.params_from(sd).items()}
    fe = O.flux_gnn_forward(p, O.node_features(O.Grid(64), states), O.chain_edges(64, 8))
    (fe * gup).sum().backward()
    for k, v in p.items():
        grads_close(runs[0][k], v.grad.numpy())
        grads_close(runs[2][k], v.grad.numpy())


@pytest.mark.parametrize("nx,B,layers,hidden,kinkfree", [(64, 5, 4, 128, False), (1, 3, 2, 128, False),
                                                          (2, 4, 1, 64, False), (7, 6, 0, 32, False),
                                                          (100, 3, 3, 128, False), (64, 300, 4, 128, True),
                                                          (64, 4, 3, 16, False), (16, 3, 2, 8, False),
                                                          (8, 2, 1, 4, False), (64, 3, 2, 256, False),
                                                          (16, 5, 2, 128, False), (32, 9, 0, 128, False),
                                                          (48, 7, 8, 128, False), (32, 11, 3, 128, False),
                                                          (64, 301, 4, 128, True)])
def test_chain_training_path_vs_oracle(hf, nx, B, layers, hidden, kinkfree):
    """The chain training path (train_chain.hip: stencil-loader GEMMs, P/Q
    readout, split-K weight gradients) on tagged chains of any nx, layer count
    and width: flux, parameter and node-feature gradients vs torch-CPU autograd
    of the oracle (src/flux_gnn.py:40-67).

    A pre-activation within rounding of 0 (the P/Q split and the GEMM order
    round differently from the reference) would flip one ReLU derivative and
    move a gradient by O(g w) -- at 300 chains x 64 cells x 128 features per
    layer a few such kinks are expected.  The large case (several GEMM row
    tiles and weight-gradient splits) therefore uses weights whose every
    pre-activation is bounded away from 0 (positive biases of 4 against
    products below 3), so its ReLU derivatives are unambiguous and the gate
    stays the gradient gate; the small cases exercise the masks.  Widths 4, 8
    and 16 are below the GEMM's 32-wide reduction chunk: tagged chains of those
    widths take the generic CSR path and must give the same answers.
    FluxGNN(4, 128, L <= 8) on nx in {16, 32, 48, 64} runs the fused forward
    (chain_train_fwd_kernel: the flux kernel's pass storing the tape); nx = 1
    and 100 at width 128 run the GEMM forward.  The update layers' weight
    gradients of the fused path run on wgrad_stencil_kernel for nx in {32, 64}
    (32-cell stages with the chain's halo rows: nx = 32 wraps at both ends of
    every stage; 301 chains of 64 leave a last split of two stages) and on
    tgemm_batch for nx in {16, 48}."""
    rng = np.random.default_rng(nx * 100 + layers)
    if kinkfree:
        u = lambda a, shape: rng.uniform(-a, a, shape)  # noqa: E731
        sd = {"input_mlp.0.weight": u(0.1, (hidden, 4)), "input_mlp.0.bias": np.full(hidden, 4.0)}
        for l in range(layers):
            sd[f"update_mlps.{l}.0.weight"] = u(0.002, (hidden, 2 * hidden))
            sd[f"update_mlps.{l}.0.bias"] = np.full(hidden, 4.0)
        sd["edge_mlp.0.weight"] = u(0.002, (hidden, 2 * hidden))
        sd["edge_mlp.0.bias"] = np.full(hidden, 4.0)
    else:
        sd = {"input_mlp.0.weight": rng.normal(0, 0.5, (hidden, 4)), "input_mlp.0.bias": rng.normal(0, 0.1, hidden)}
        for l in range(layers):
            sd[f"update_mlps.{l}.0.weight"] = rng.normal(0, 1.5 / np.sqrt(2 * hidden), (hidden, 2 * hidden))
            sd[f"update_mlps.{l}.0.bias"] = rng.normal(0, 0.1, hidden)
        sd["edge_mlp.0.weight"] = rng.normal(0, 1.5 / np.sqrt(2 * hidden), (hidden, 2 * hidden))
        sd["edge_mlp.0.bias"] = rng.normal(0, 0.1, hidden)
    sd["edge_mlp.2.weight"] = rng.normal(0, 1 / np.sqrt(hidden), (1, hidden))
    sd["edge_mlp.2.bias"] = rng.normal(0, 0.1, 1)
    sd = {k: np.asarray(v, np.float32) for k, v in sd.items()}
    m = load(hf, sd, (4, hidden, layers))
    G = O.Grid(nx, dt=5e-3)
    states = np.stack([O.initial_condition(G, s) for s in range(40, 40 + B)])
    gup = torch.randn(B * 2 * nx, generator=torch.Generator().manual_seed(nx + B))
    nf, ei = hf.build_chain_graph_batch(states, G.x, DEV)
    nf = nf.clone().requires_grad_(True)
    flux = m(nf, ei)
    (flux * gup.to(DEV)).sum().backward()
    p = {k: v.clone().requires_grad_(True) for k, v in O.params_from(sd).items()}
    nf_o = O.node_features(G, states).clone().requires_grad_(True)
    fe = O.flux_gnn_forward(p, nf_o, O.chain_edges(nx, B))
    (fe * gup).sum().backward()
    grads_close(flux, fe.detach().numpy(), 1e-5)
    grads_close(nf.grad, nf_o.grad.numpy())
    for k, q in m.named_parameters():
        grads_close(q.grad, p[k].grad.numpy())


@pytest.mark.parametrize("nx,B", [(64, 1), (64, 9), (64, 2000), (16, 13), (48, 6)])
def test_fused_training_forward_equals_inference(hf, nx, B):
    """FluxGNN(4, 128, 4) under autograd on a tagged chain of nx in {16, 32, 48,
    64} runs chain_train_fwd_kernel (device-packed weights, tape stores) —
    the inference flux kernel's own pass, so its flux equals the no-grad
    forward (chain_flux_kernel) bit for bit; B = 2000 is the training bench's
    batch (several IC groups per workgroup)."""
    w = golden("weights_W1_r2.npz")
    m = load(hf, {k: w[k] for k in w.files}, (4, 128, 4))
    G = O.Grid(nx, dt=5e-3)
    states = np.stack([O.initial_condition(G, s) for s in range(7, 7 + min(B, 64))])
    states = np.concatenate([states] * ((B + len(states) - 1) // len(states)))[:B]
    nf, ei = hf.build_chain_graph_batch(states, G.x, DEV)
    with torch.no_grad():
        want = m(nf, ei).cpu().numpy()
    got = m(nf, ei)
    assert got.requires_grad
    assert np.array_equal(got.detach().cpu().numpy(), want)


def test_backward_edge_cases(hf):
    """No edges -> zero gradients; isolated nodes -> gradients only where reached."""
    m = hf.FluxGNN(4, 32, 2).to(DEV)
    nf = torch.randn(10, 4, device=DEV, requires_grad=True)
    out = m(nf, torch.zeros(2, 0, dtype=torch.long, device=DEV))
    assert out.shape == (0,)
    out.sum().backward()
    assert all(float(p.grad.abs().max()) == 0.0 for p in m.parameters()) and float(nf.grad.abs().max()) == 0.0
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ei = torch.tensor([[0, 0, 0, 5, 5], [1, 2, 9, 0, 0]])
    nf_c = torch.randn(10, 4, generator=torch.Generator().manual_seed(3))
    m.zero_grad()
    nf_d = nf_c.to(DEV).requires_grad_(True)
    (m(nf_d, ei.to(DEV)) ** 2).sum().backward()
    p = {k: v.clone().requires_grad_(True) for k, v in O.params_from(sd).items()}
    nf_o = nf_c.clone().requires_grad_(True)
    (O.flux_gnn_forward(p, nf_o, ei) ** 2).sum().backward()
    grads_close(nf_d.grad, nf_o.grad.numpy())
    for k, q in m.named_parameters():
        grads_close(q.grad, p[k].grad.numpy())


def _sample(ic, t):
    cl = golden("classical.npz")
    S, F = cl["b16_states"], cl["b16_fluxes"]
    return S[ic, t], F[ic, t], S[ic, t + 1]


def _w1_model(hf):
    w1 = golden("weights_W1_r1.npz")
    return load(hf, {k: w1[k] for k in w1.files}, (4, 128, 4))


def test_ablation_loss_grads_vs_reference(hf):
    """hybridflux.training.ablation_loss ('full' config) == train_ablation.py's
    loss and parameter gradients on the three golden samples (B=1 each), and the
    batched loss over all three is the mean of the three (loss and gradients)."""
    from hybridflux.training import ablation_loss
    g = golden("grads.npz")
    m = _w1_model(hf)
    solver = hf.BaselineSolver(64, device=DEV)
    cfg = hf.ABLATION_CONFIGS["full"]
    x = torch.as_tensor(solver.x, dtype=torch.float32, device=DEV)
    picks = [tuple(int(v) for v in pk) for pk in g["loss_picks"]]
    for j, (ic, t) in enumerate(picks):
        st, ft, sn = (torch.as_tensor(a[None], device=DEV) for a in _sample(ic, t))
        m.zero_grad()
        loss, fl = ablation_loss(m, st, ft, sn, x, solver.dt, solver.dx, cfg, solver.grid)
        loss.backward()
        assert abs(loss.item() - float(g[f"loss{j}_value"])) <= 1e-5 * abs(float(g[f"loss{j}_value"]))
        assert abs(fl.item() - float(g[f"loss{j}_flux"])) <= 1e-5 * abs(float(g[f"loss{j}_flux"]))
        for k, p in m.named_parameters():
            grads_close(p.grad, g[f"loss{j}_grad.{k}"])
    batch = [np.stack(a) for a in zip(*[_sample(ic, t) for ic, t in picks])]
    st, ft, sn = (torch.as_tensor(a, device=DEV) for a in batch)
    m.zero_grad()
    loss, _ = ablation_loss(m, st, ft, sn, x, solver.dt, solver.dx, cfg, solver.grid)
    loss.backward()
    want = np.mean([float(g[f"loss{j}_value"]) for j in range(3)])
    assert abs(loss.item() - want) <= 1e-5 * abs(want)
    for k, p in m.named_parameters():
        grads_close(p.grad, np.mean([g[f"loss{j}_grad.{k}"] for j in range(3)], axis=0))


def test_loss_gradient_without_state_term(hf):
    """lambda_state = 0 ('baseline' config): the loss has no state term
    (train_ablation.py:132 gates it), so neither may its gradient — a
    non-finite target density n'_t must leave loss and d loss/d params equal to
    the finite target's (no 0 * NaN in the continuity adjoint)."""
    from hybridflux.training import ablation_loss
    m = _w1_model(hf)
    solver = hf.BaselineSolver(64, device=DEV)
    x = torch.as_tensor(solver.x, dtype=torch.float32, device=DEV)
    st, ft, sn = (torch.as_tensor(np.stack(a), device=DEV) for a in zip(_sample(0, 3), _sample(5, 17)))
    out = []
    for poison in (False, True):
        sn_p = sn.clone()
        if poison:
            sn_p[:, 0, ::7] = float("nan")
        m.zero_grad()
        loss, _ = ablation_loss(m, st, ft, sn_p, x, solver.dt, solver.dx, hf.ABLATION_CONFIGS["baseline"],
                                solver.grid)
        loss.backward()
        out.append((loss.item(), {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}))
    assert np.isfinite(out[1][0]) and out[0][0] == out[1][0]
    for k in out[0][1]:
        assert np.isfinite(out[1][1][k]).all() and np.array_equal(out[0][1][k], out[1][1][k]), k


def test_adam_steps_vs_reference(hf):
    """Six batch-size-1 Adam steps of the reference trainer ('physics' config,
    fixed sample order) reproduced with hybridflux.training.train_steps."""
    from hybridflux.training import FluxDataset, train_steps
    g = golden("grads.npz")
    m = _w1_model(hf)
    solver = hf.BaselineSolver(64, device=DEV)
    order = [tuple(int(v) for v in o) for o in g["adam_order"]]
    samples = [_sample(ic, t) for ic, t in order]
    data = FluxDataset(np.stack([s[0] for s in samples]), np.stack([s[1] for s in samples]),
                       np.stack([s[2] for s in samples]), DEV)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    x = torch.as_tensor(solver.x, dtype=torch.float32, device=DEV)
    losses = []
    for i in range(len(order)):
        tot, _, _ = train_steps(m, opt, data, torch.tensor([i], device=DEV), 1, x, solver.dt, solver.dx,
                                hf.ABLATION_CONFIGS["physics"], solver.grid)
        losses.append(tot)
    np.testing.assert_allclose(losses, g["adam_losses"], rtol=1e-4)
    total, bad = 0, 0
    for k, p in m.state_dict().items():
        d = np.abs(p.cpu().numpy().astype(np.float64) - g[f"adam_final.{k}"])
        total += d.size
        bad += int((d > 2e-5).sum())
        assert d.max() <= 2.1e-3, (k, d.max())
    assert bad <= 1e-3 * total, (bad, total)


def test_train_model_smoke(hf, tmp_path):
    """train_model end to end on a GPU-generated dataset: loss decreases, the
    checkpoint loads into HybridSolver (reference file layout)."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import train_model
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=4, steps_per_ic=16, out_path=None,
                                                 device=DEV)
    m, hist = train_model(st, ft, sn, x, dt, dx, nu, "physics", 2, epochs=3, lr=1e-3, device=DEV, batch_size=8,
                          seed=1, save_dir=str(tmp_path), log=None)
    assert len(hist["loss"]) == 3 and hist["loss"][-1] < hist["loss"][0]
    solver = hf.HybridSolver(str(tmp_path / "hybrid_physics_r2.pt"), radius=2, device=DEV)
    out = solver.run(st[0], 5)
    assert out.shape == (6, 3, 64) and np.isfinite(out).all()


def test_graphed_steps_equal_eager(hf):
    """train_steps with a captured step (GraphedStep: HIP-graph replay of the
    loss + backward + Adam step) makes the eager loop's updates: same losses
    and weights after 8 batches of 16 ('full' config: the rollout loss runs
    the model on 4 states per sample).  Both arms use the capturable Adam (its
    device-side bias corrections round differently from the host-side ones of
    the default Adam, which after a few steps moves near-zero-gradient weights
    by O(lr) differently, as test_adam_steps_vs_reference notes)."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FluxDataset, GraphedStep, train_steps
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=4, steps_per_ic=32, out_path=None, device=DEV)
    data = FluxDataset(st, ft, sn, DEV)
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = hf.ABLATION_CONFIGS["full"]
    order = torch.randperm(len(data), generator=torch.Generator().manual_seed(5))[:128].to(DEV)
    res = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = hf.FluxGNN(4, 128, 4).to(DEV)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, capturable=True)  # same Adam arithmetic in both arms
        gs = GraphedStep(m, opt, data, 16, xd, solver.dt, solver.dx, cfg, solver.grid) if graphed else None
        tot, _, steps = train_steps(m, opt, data, order, 16, xd, solver.dt, solver.dx, cfg, solver.grid, graphed=gs)
        assert steps == 8 and (gs is None or gs.graph is not None)
        res.append((tot, {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}))
    assert abs(res[0][0] - res[1][0]) <= 1e-6 * abs(res[0][0])
    for k in res[0][1]:
        assert np.abs(res[0][1][k] - res[1][1][k]).max() <= 1e-6, k


@pytest.mark.parametrize("cfg_name", ["physics", "full", "full_k5"])
def test_direct_step_equals_autograd_step(hf, cfg_name):
    """train_steps' direct_step (forward, one-pass loss, backward with the
    loss's flux gradient as the incoming one, FlatAdam: no autograd) makes the
    autograd step's updates bit for bit: losses and every parameter after 8
    batches of 16, eager and graph-replayed.  'full_k5' (rollout_steps 5: the
    energies need model forwards) takes the autograd step in both arms."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FlatAdam, FluxDataset, GraphedStep, direct_step, train_steps
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=4, steps_per_ic=32, out_path=None, device=DEV)
    data = FluxDataset(st, ft, sn, DEV)
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = dict(hf.ABLATION_CONFIGS["full"], rollout_steps=5) if cfg_name == "full_k5" else hf.ABLATION_CONFIGS[cfg_name]
    order = torch.randperm(len(data), generator=torch.Generator().manual_seed(6))[:128].to(DEV)
    res = []
    arms = ((False, False), (True, False)) + (((True, True),) if cfg_name != "full_k5" else ())
    for direct, graphed in arms:  # (K = 5's energies take a host value: not capturable)
        torch.manual_seed(0)
        m = hf.FluxGNN(4, 128, 4).to(DEV).flatten_parameters_()
        opt = FlatAdam(m.parameters(), lr=1e-3)
        gs = GraphedStep(m, opt, data, 16, xd, solver.dt, solver.dx, cfg, solver.grid, direct=direct) if graphed else None
        tot, _, steps = train_steps(m, opt, data, order, 16, xd, solver.dt, solver.dx, cfg, solver.grid, graphed=gs,
                                    direct=direct)
        assert steps == 8 and (gs is None or gs.graph is not None)
        res.append((tot, {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}))
    # the direct step applies exactly where documented
    b_st, b_ft, b_sn, nf = data.batch(order[:16], xd)
    r = direct_step(m, opt, b_st, b_ft, b_sn, nf, xd, solver.dt, solver.dx, cfg, solver.grid)
    assert (r is None) == (cfg_name == "full_k5")
    for tot, sd in res[1:]:
        assert tot == res[0][0]
        for k in sd:
            assert np.array_equal(sd[k].view(np.uint32), res[0][1][k].view(np.uint32)), k


@pytest.mark.parametrize("cfg_name", ["baseline", "physics", "full"])
def test_fused_step_loss_equals_torch_terms(hf, cfg_name):
    """hf_ablation_loss (the loss's single-step terms in one HIP pass, with its
    own d loss / d flux_edge) against the same terms as torch expressions
    (ablation_loss(fused=False)) on 48 samples: loss and parameter gradients."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import ablation_loss
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=3, steps_per_ic=16, out_path=None, device=DEV)
    st, ft, sn = (torch.as_tensor(a, device=DEV) for a in (st, ft, sn))
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = hf.ABLATION_CONFIGS[cfg_name]
    m = _w1_model(hf)
    out = []
    for fused in (True, False):
        m.zero_grad()
        loss, fl = ablation_loss(m, st, ft, sn, xd, solver.dt, solver.dx, cfg, solver.grid, fused=fused)
        loss.backward()
        out.append((loss.item(), fl.item(), {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}))
    assert abs(out[0][0] - out[1][0]) <= 2e-6 * abs(out[1][0])
    assert abs(out[0][1] - out[1][1]) <= 2e-6 * abs(out[1][1])
    for k in out[0][2]:
        grads_close(out[0][2][k], out[1][2][k], 1e-5)


def test_chain_batch_gather_equals_indexing(hf):
    """hf_chain_batch_gather (FluxDataset.batch with x: the batch and its chain
    node features in one pass) equals torch indexing + build_chain_graph_batch
    bit for bit, negative indices included (train_ablation.py:27-44,
    src/graph_constructor.py:6-39)."""
    from hybridflux.training import FluxDataset
    g = torch.Generator().manual_seed(3)
    N, nx, B = 37, 64, 300
    st, sn = torch.randn(N, 3, nx, generator=g), torch.randn(N, 3, nx, generator=g)
    ft = torch.randn(N, nx, generator=g)
    data = FluxDataset(st.numpy(), ft.numpy(), sn.numpy(), DEV)
    idx = torch.randint(-N, N, (B,), generator=g).to(DEV)
    x = torch.linspace(0, 2 * np.pi, nx + 1)[:-1].to(DEV)
    st_b, ft_b, sn_b, nf = data.batch(idx, x)
    ref = data.batch(idx)
    for a, b in zip((st_b, ft_b, sn_b), ref):
        assert torch.equal(a, b)
    nf_ref, _ = hf.build_chain_graph_batch(ref[0], x)
    assert torch.equal(nf, nf_ref)
    e = data.batch(idx[:0], x)
    assert e[0].shape == (0, 3, nx) and e[3].shape == (0, 4)


def test_flattened_parameters_same_step(hf):
    """FluxGNN.flatten_parameters_ (one parameter buffer, no per-step concat)
    changes nothing: the same flux, gradients and Adam update bit for bit."""
    import copy
    torch.manual_seed(4)
    a = hf.FluxGNN(4, 128, 4).to(DEV)
    b = copy.deepcopy(a).flatten_parameters_()
    assert hf.flux_gnn._flat_view(list(b.parameters()), torch.device(DEV)) is not None
    assert hf.flux_gnn._flat_view(list(a.parameters()), torch.device(DEV)) is None
    st = torch.randn(6, 3, 64, device=DEV)
    x = torch.linspace(0, 2 * np.pi, 65, device=DEV)[:-1]
    out = []
    for m in (a, b):
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        nf, ei = hf.build_chain_graph_batch(st, x)
        fl = m(nf, ei)
        (fl ** 2).sum().backward()
        grads = [q.grad.clone() for q in m.parameters()]
        opt.step()
        out.append((fl.detach(), grads, [q.detach().clone() for q in m.parameters()]))
    assert torch.equal(out[0][0], out[1][0])
    for u, v in zip(out[0][1] + out[0][2], out[1][1] + out[1][2]):
        assert torch.equal(u, v)


def test_flat_adam_matches_torch_adam(hf):
    """FlatAdam (hf_adam_flat: torch.optim.Adam's update over the flattened
    parameter buffer, step count on the device) against torch.optim.Adam on
    the same gradients for 12 steps: equal within f32 rounding of the bias
    corrections (relative 1e-6 of the parameter scale), and the step count
    advanced on the device."""
    import copy
    from hybridflux.training import FlatAdam
    torch.manual_seed(6)
    a = hf.FluxGNN(4, 128, 2).to(DEV)
    b = hf.FluxGNN(4, 128, 2).to(DEV)
    b.load_state_dict(a.state_dict())
    b.flatten_parameters_()
    oa, ob = torch.optim.Adam(a.parameters(), lr=1e-3), FlatAdam(b.parameters(), lr=1e-3)
    for k in range(12):
        grads = [torch.randn_like(p) * 10 ** (k % 3 - 1) for p in a.parameters()]
        for m in (a, b):
            for p, gr in zip(m.parameters(), grads):
                p.grad = gr.clone()
        oa.step()
        ob.step()
    for (ka, pa), (kb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb
        assert (pa - pb).abs().max().item() <= 1e-6 * max(1.0, pa.abs().max().item()), ka
    st = ob.state[next(iter(b.parameters()))]
    assert st["step"].item() == 12.0 and st["done"].item() == 0
    with pytest.raises(ValueError):
        FlatAdam(a.parameters())  # not flattened
    # state_dict round trip (through the host): the same moments and step count
    sd = ob.state_dict()
    sd["state"] = {k: {n: t.cpu() for n, t in v.items()} for k, v in sd["state"].items()}
    oc = FlatAdam(b.parameters(), lr=1e-3)
    oc.load_state_dict(sd)
    for p in b.parameters():
        p.grad = torch.ones_like(p)
    ref = copy.deepcopy(b)
    ob.step()
    after_ob = [q.detach().clone() for q in b.parameters()]
    with torch.no_grad():
        for q, r in zip(b.parameters(), ref.parameters()):
            q.copy_(r)
    oc.step()
    for u, v in zip(after_ob, b.parameters()):
        assert torch.equal(u, v)


def test_graphed_flat_adam_equals_eager(hf):
    """GraphedStep replaying FlatAdam (its device step count advancing inside
    the graph) makes the eager loop's updates bit for bit."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FlatAdam, FluxDataset, GraphedStep, train_steps
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=4, steps_per_ic=32, out_path=None, device=DEV)
    data = FluxDataset(st, ft, sn, DEV)
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = hf.ABLATION_CONFIGS["physics"]
    order = torch.randperm(len(data), generator=torch.Generator().manual_seed(5))[:128].to(DEV)
    res = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = hf.FluxGNN(4, 128, 4).to(DEV).flatten_parameters_()
        opt = FlatAdam(m.parameters(), lr=1e-3)
        gs = GraphedStep(m, opt, data, 16, xd, solver.dt, solver.dx, cfg, solver.grid) if graphed else None
        tot, _, steps = train_steps(m, opt, data, order, 16, xd, solver.dt, solver.dx, cfg, solver.grid, graphed=gs)
        assert steps == 8 and (gs is None or gs.graph is not None)
        res.append((tot, {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}))
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


@pytest.mark.parametrize("nx", [1, 16, 100, 256])
def test_loss_terms_any_nx(hf, nx):
    """hf_ablation_loss at chain lengths other than the trainer's 64: the
    one-launch terms (circulant sizes: nx = 1, 16, 100) and the three-launch
    form around the FFT Poisson (nx = 256) against the torch expressions of
    the same loss ('physics' weights; loss, flux loss and d loss / d flux_edge)."""
    from hybridflux.training import ablation_loss
    g = torch.Generator().manual_seed(nx)
    B = 37
    st = (1.0 + 0.1 * torch.randn(B, 3, nx, generator=g)).to(DEV)
    sn = (1.0 + 0.1 * torch.randn(B, 3, nx, generator=g)).to(DEV)
    ft = (0.1 * torch.randn(B, nx, generator=g)).to(DEV)
    fe0 = (0.1 * torch.randn(B * 2 * nx, generator=g)).to(DEV)
    solver = hf.BaselineSolver(nx, device=DEV)
    x = torch.as_tensor(solver.x, dtype=torch.float32, device=DEV)
    cfg = hf.ABLATION_CONFIGS["physics"]
    out = []
    for fused in (True, False):
        fe = fe0.clone().requires_grad_(True)
        loss, fl = ablation_loss(lambda nf, ei: fe, st, ft, sn, x, solver.dt, solver.dx, cfg, solver.grid,
                                 fused=fused)
        loss.backward()
        out.append((loss.item(), fl.item(), fe.grad.detach().clone()))
    assert abs(out[0][0] - out[1][0]) <= 2e-6 * abs(out[1][0])
    assert abs(out[0][1] - out[1][1]) <= 2e-6 * abs(out[1][1])
    torch.testing.assert_close(out[0][2], out[1][2], rtol=1e-5, atol=1e-10)


def _rollout_cfgs(hf):
    full = hf.ABLATION_CONFIGS["full"]
    return {"full": full, "rollout_only": hf.ABLATION_CONFIGS["rollout_only"],
            "full_k1": dict(full, rollout_steps=1),   # energies [e_0]: the term is 0
            "full_k2": dict(full, rollout_steps=2),   # e_0, e_1 (u_1 from the sample's E)
            "full_k5": dict(full, rollout_steps=5)}   # energies reach forwards 1 and 2


@pytest.mark.parametrize("cfg_name", ["full", "rollout_only", "full_k1", "full_k2", "full_k5"])
def test_rollout_term_without_redundant_forwards_bitwise(hf, cfg_name):
    """The rollout energy term with only the forwards that reach an energy
    (ablation_loss rollout='reuse': forward 0 is the main forward, reused;
    none more for the reference's rollout_steps = 3; forwards 1..K-3 untaped
    otherwise) equals the reference's literal loop of rollout_steps taped
    forwards (train_ablation.py:172-206, rollout='literal') bit for bit: loss,
    flux loss and every parameter gradient, on 48 samples."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import ablation_loss
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=3, steps_per_ic=16, out_path=None, device=DEV)
    st, ft, sn = (torch.as_tensor(a, device=DEV) for a in (st, ft, sn))
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = _rollout_cfgs(hf)[cfg_name]
    m = _w1_model(hf)
    out = []
    for mode in ("literal", "reuse"):
        m.zero_grad()
        loss, fl = ablation_loss(m, st, ft, sn, xd, solver.dt, solver.dx, cfg, solver.grid, fused=False,
                                 rollout=mode)
        loss.backward()
        out.append((loss.item(), fl.item(), {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}))
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1]
    for k in out[0][2]:
        assert np.array_equal(out[0][2][k], out[1][2][k]), k


@pytest.mark.parametrize("cfg_name", ["full", "rollout_only", "full_k1", "full_k2", "full_k5"])
def test_fused_rollout_term_vs_literal(hf, cfg_name):
    """hf_ablation_loss_ex (the rollout energy term formed in the loss pass from
    the main forward's flux, K <= 3; for K = 5 the term from the reuse form's
    two untaped forwards) against the literal 3-forward torch loss: loss within
    2e-6 relative (the kernels' fixed-order sums vs torch's reductions), the
    gradients (the term has none) as the single-step comparison's."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import ablation_loss
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=3, steps_per_ic=16, out_path=None, device=DEV)
    st, ft, sn = (torch.as_tensor(a, device=DEV) for a in (st, ft, sn))
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = _rollout_cfgs(hf)[cfg_name]
    m = _w1_model(hf)
    out = []
    for fused in (True, False):
        m.zero_grad()
        loss, fl = ablation_loss(m, st, ft, sn, xd, solver.dt, solver.dx, cfg, solver.grid, fused=fused,
                                 rollout="literal")
        loss.backward()
        out.append((loss.item(), fl.item(), {k: p.grad.detach().cpu().numpy().copy() for k, p in m.named_parameters()}))
    assert abs(out[0][0] - out[1][0]) <= 2e-6 * abs(out[1][0])
    assert abs(out[0][1] - out[1][1]) <= 2e-6 * abs(out[1][1])
    for k in out[0][2]:
        grads_close(out[0][2][k], out[1][2][k], 1e-5)
    # the term is really there (K >= 2): the same loss without it differs; K = 1 adds exactly 0
    base = dict(cfg, lambda_energy_multi=0.0)
    with torch.no_grad():
        l0, _ = ablation_loss(m, st, ft, sn, xd, solver.dt, solver.dx, base, solver.grid)
    if cfg["rollout_steps"] >= 2:
        assert l0.item() != out[0][0]
    else:
        assert l0.item() == out[0][0]


def test_flat_adam_invalidates_packed_inference_weights(hf):
    """FlatAdam writes the parameters through a HIP kernel; it bumps their
    version counters, so a no-grad forward after an optimizer step (eager or a
    replayed HIP graph) uses the new weights, not the packed copy made before
    (ADVICE r05)."""
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FlatAdam, FluxDataset, GraphedStep, train_steps
    st, ft, sn, x, dt, dx, nu = generate_dataset(num_initial_conditions=2, steps_per_ic=16, out_path=None, device=DEV)
    data = FluxDataset(st, ft, sn, DEV)
    solver = hf.BaselineSolver(64, device=DEV)
    xd = torch.as_tensor(x, device=DEV)
    cfg = hf.ABLATION_CONFIGS["physics"]
    nf, ei = hf.build_chain_graph_batch(data.state_t[:4], xd)
    for graphed in (False, True):
        torch.manual_seed(0)
        m = hf.FluxGNN(4, 128, 4).to(DEV).flatten_parameters_()
        opt = FlatAdam(m.parameters(), lr=1e-3)
        gs = GraphedStep(m, opt, data, 8, xd, solver.dt, solver.dx, cfg, solver.grid) if graphed else None
        if graphed:  # 3 eager warmup steps, the capture and a replay
            train_steps(m, opt, data, torch.arange(32, device=DEV) % len(data), 8, xd, solver.dt, solver.dx, cfg,
                        solver.grid, graphed=gs)
            assert gs.graph is not None
        with torch.no_grad():
            before = m(nf, ei).clone()  # packs the current weights
        # one more step: eager FlatAdam, or a replay of the captured step only
        train_steps(m, opt, data, torch.arange(8, device=DEV) % len(data), 8, xd, solver.dt, solver.dx, cfg,
                    solver.grid, graphed=gs)
        with torch.no_grad():
            after = m(nf, ei)
            fresh = hf.FluxGNN(4, 128, 4).to(DEV)
            fresh.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
            want = fresh(nf, ei)
        assert not torch.equal(before, after)
        assert torch.equal(after, want)


def test_dataset_batch_rejects_out_of_range_indices(hf):
    """FluxDataset.batch raises IndexError outside [-N, N), as the reference's
    dataset indexing does (the device gather would clamp); train_steps checks
    a pass's order once."""
    from hybridflux.training import FluxDataset, train_steps
    g = torch.Generator().manual_seed(2)
    N, nx = 5, 64
    data = FluxDataset(torch.randn(N, 3, nx, generator=g).numpy(), torch.randn(N, nx, generator=g).numpy(),
                       torch.randn(N, 3, nx, generator=g).numpy(), DEV)
    x = torch.linspace(0, 1, nx, device=DEV)
    data.batch(torch.tensor([-N, N - 1], device=DEV), x)
    for bad in ([N], [-N - 1], [0, 7]):
        with pytest.raises(IndexError):
            data.batch(torch.tensor(bad, device=DEV), x)
        with pytest.raises(IndexError):
            data.batch(torch.tensor(bad, device=DEV))
    m = hf.FluxGNN(4, 128, 4).to(DEV)
    solver = hf.BaselineSolver(nx, device=DEV)
    with pytest.raises(IndexError):
        train_steps(m, torch.optim.Adam(m.parameters()), data, torch.tensor([0, 9], device=DEV), 2, x, solver.dt,
                    solver.dx, hf.ABLATION_CONFIGS["physics"], solver.grid)
