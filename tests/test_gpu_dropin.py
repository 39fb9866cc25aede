"""The reference's own host-tensor call pattern through the drop-in
(VERDICT r03 item 3): examples/smoke_test.py:30-58 verbatim — a FluxGNN built
on the CPU, grad enabled, CPU node features and a random CPU edge_index — and
the trainer's chain call (scripts/training/train_ablation.py:119-124:
build_chain_graph(state, x, 'cpu') into a CPU model under autograd).  The
inputs are staged to the HIP device, the flux and the gradients are computed
by the HIP kernels (graph.hip / train_chain.hip) and come back on the CPU.
Values are compared with tests/golden/smoke_test.npz, which make_golden.py
recorded by running the same sequence (same seeds) on the reference itself.

Tolerances: fluxes 2e-6 + 1e-5 |ref| (the generic-graph gate of
test_gpu_parity.py); gradients |got - ref| <= 2e-5 max|ref| (test_gpu_training.py).
"""
import numpy as np
import pytest
import torch

from conftest import close, golden
from test_gpu_training import grads_close

pytestmark = pytest.mark.gpu
SEEDS = (0, 1, 2)


@pytest.fixture(scope="module")
def hf():
    import hybridflux
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    return hybridflux


@pytest.mark.parametrize("seed", SEEDS)
def test_smoke_test_flux_gnn_verbatim(hf, seed):
    """examples/smoke_test.py:45-58 with torch.manual_seed(seed) in front."""
    g = golden("smoke_test.npz")
    FluxGNN = hf.FluxGNN
    torch.manual_seed(seed)
    model = FluxGNN(input_dim=4, hidden_dim=64, num_layers=3)
    node_features = torch.randn(64, 4)
    edge_index = torch.randint(0, 64, (2, 128))
    fluxes = model(node_features, edge_index)
    assert fluxes.shape == (128,), f"Wrong flux shape: {fluxes.shape}"
    assert fluxes.device.type == "cpu" and fluxes.requires_grad
    close(fluxes, g[f"flux{seed}"], 2e-6, 1e-5, what="flux")
    fluxes.sum().backward()
    for k, p in model.named_parameters():
        assert p.grad is not None and p.grad.device.type == "cpu"
        grads_close(p.grad, g[f"flux{seed}_grad.{k}"])
    with torch.no_grad():  # the inference kernels on the same host inputs
        f2 = model(node_features, edge_index)
    assert f2.device.type == "cpu" and not f2.requires_grad
    close(f2, g[f"flux{seed}"], 2e-6, 1e-5, what="flux_nograd")


@pytest.mark.parametrize("seed", SEEDS)
def test_smoke_test_graph_constructor_verbatim(hf, seed):
    """examples/smoke_test.py:30-42 with np.random.seed(seed) in front; the
    graph then feeds the HIP chain kernel from the host."""
    g = golden("smoke_test.npz")
    np.random.seed(seed)
    state = np.random.randn(3, 64)
    x = np.linspace(0, 1, 64)
    node_features, edge_index = hf.build_chain_graph(state, x, "cpu")
    assert node_features.shape == (64, 4), f"Wrong node features: {node_features.shape}"
    assert edge_index.shape[1] == 128, f"Wrong edge count: {edge_index.shape[1]}"
    assert np.array_equal(node_features.numpy(), g[f"graph{seed}_nf"])
    assert np.array_equal(edge_index.numpy(), g[f"graph{seed}_ei"])


def test_trainer_chain_call_on_host(hf):
    """train_ablation.py:119-124: build_chain_graph(state, x, 'cpu') into a CPU
    FluxGNN(4,128,4) under autograd -> the chain training kernels
    (train_chain.hip) on the device; flux and parameter gradients on the CPU."""
    g = golden("smoke_test.npz")
    w = golden("weights_W1_r1.npz")
    model = hf.FluxGNN(4, 128, 4)
    model.load_state_dict({k: torch.from_numpy(w[k]) for k in w.files})
    st = hf.BaselineSolver(nx=64).initial_condition(seed=1000)
    nf, ei = hf.build_chain_graph(st, hf.BaselineSolver(nx=64).x, device="cpu")
    fe = model(nf, ei)
    assert fe.device.type == "cpu" and fe.shape == (128,)
    close(fe, g["chain_flux"], 2e-6, 1e-5, what="chain_flux")
    fe.sum().backward()
    for k, p in model.named_parameters():
        assert p.grad.device.type == "cpu"
        grads_close(p.grad, g[f"chain_grad.{k}"])


def test_host_node_feature_gradient(hf):
    """d sum(g*flux) / d node_features for host inputs lands on the host and
    equals the reference autograd (grads.npz 'small')."""
    gr, rnd = golden("grads.npz"), golden("fluxgnn_random.npz")
    m = hf.FluxGNN(4, 64, 3)
    m.load_state_dict({k[6:]: torch.from_numpy(rnd[k]) for k in rnd.files if k.startswith("small.")})
    nf = torch.from_numpy(rnd["small_nf"]).clone().requires_grad_(True)
    flux = m(nf, torch.from_numpy(rnd["small_ei"]))
    (flux * torch.from_numpy(gr["small_g"])).sum().backward()
    assert nf.grad.device.type == "cpu"
    grads_close(nf.grad, gr["small_grad_nf"])


def test_baseline_models_on_host_tensors(hf):
    """PureGNN / PINN forward with the reference's host tensors
    (evaluate_multi_ic.py:53-83) against baselines.npz."""
    from hybridflux.baselines import PINN, PureGNN
    b = golden("baselines.npz")
    pg = PureGNN(4, 128, 4)
    pg.load_state_dict({k[9:]: torch.from_numpy(b[k]) for k in b.files if k.startswith("pure_gnn.")})
    pinn = PINN(3 * 64, 256, 4)
    pinn.load_state_dict({k[5:]: torch.from_numpy(b[k]) for k in b.files if k.startswith("pinn.")})
    with torch.no_grad():
        d = pg(torch.from_numpy(b["pure_gnn_graph_nf"]), torch.from_numpy(b["pure_gnn_graph_ei"]))
        out = pinn(torch.from_numpy(b["ics"][:3]))
    assert d.device.type == "cpu" and out.device.type == "cpu"
    close(d, b["pure_gnn_graph_delta"], 2e-6, 1e-5, what="pure_gnn")
    close(out, b["pinn_batch_out"], 2e-6, 1e-5, what="pinn")
