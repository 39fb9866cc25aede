import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "gnn-plasma-flux_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG_DIR, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) HIP device")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gold():
    return golden


def rand_sd(layers, seed):
    """Random FluxGNN(4, 128, layers) state dict (reference keys, src/flux_gnn.py:17-38)."""
    g = np.random.default_rng(seed)
    sd = {"input_mlp.0.weight": g.normal(0, 0.5, (128, 4)), "input_mlp.0.bias": g.normal(0, 0.1, 128)}
    for l in range(layers):
        sd[f"update_mlps.{l}.0.weight"] = g.normal(0, 1 / 16, (128, 256))
        sd[f"update_mlps.{l}.0.bias"] = g.normal(0, 0.1, 128)
    sd["edge_mlp.0.weight"] = g.normal(0, 1 / 16, (128, 256))
    sd["edge_mlp.0.bias"] = g.normal(0, 0.1, 128)
    sd["edge_mlp.2.weight"] = g.normal(0, 1 / 11, (1, 128))
    sd["edge_mlp.2.bias"] = g.normal(0, 0.1, 1)
    return {k: np.asarray(v, np.float32) for k, v in sd.items()}
