"""Where the cfg4 (bf16, 4096 ICs x 1024 cells) step time goes (diagnostic,
not a bench line).

Times bare rollouts (no trajectory, no metrics) of T steps on the cfg4 grid:
  * with the committed W1_r2 weights (the bench's cfg4 workload);
  * with random FluxGNN(4,128,L) weights for L = 0,1,2,4: the per-layer slope is
    the windowed flux kernel's message-passing cost, the intercept its input
    layer + readout plus the FV/Poisson kernel.
Kernel time from HIP events on the launch stream.  Run under
HYBRIDFLUX_LIB=<diag build> to compare timing-only variants.

    python tools/diag_cfg4.py [T]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from diag_rollout import FLOP_FIXED, FLOP_LAYER, rand_sd, timed  # noqa: E402
from hybridflux import HybridSolver, engine  # noqa: E402
from hybridflux._lib import HF_OP_RUN, version  # noqa: E402

PEAK = 2.5e15


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B, nx = int(os.environ.get("DIAG_B", 4096)), 1024
    dt = 5e-3 * 64.0 / nx
    dev = torch.device("cuda", 0)
    solver = HybridSolver(os.path.join(ROOT, "tests", "golden", "weights_W1_r2.npz"), radius=2, nx=nx, dt=dt,
                          device=dev, precision="bf16")
    s0 = solver.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    grid = engine.Grid(nx, dt=dt)
    ws, _ = engine.workspace(HF_OP_RUN, B, nx, T, dev, model=solver._dm())
    fin = torch.empty_like(s0)
    cells = B * nx * T
    out = {"build": version(), "T": T, "B": B}
    dm = solver.model.device_model(dev)
    ms = timed(lambda: engine.run(dm, grid, s0, T, traj=False, metrics=False, out=fin, ws=ws))
    out["W1_r2_ms_per_step"] = ms / T
    out["W1_r2_frac"] = (FLOP_FIXED + 4 * FLOP_LAYER) * cells / (ms * 1e-3) / PEAK
    per_l = {}
    for L in (0, 1, 2, 4):
        m = engine.DeviceModel(rand_sd(L), dev, "bf16")
        per_l[L] = timed(lambda: engine.run(m, grid, s0, T, traj=False, metrics=False, out=fin, ws=ws)) / T
        m.close()
    out["rand_ms_per_step_by_layers"] = per_l
    slope = (per_l[4] - per_l[0]) / 4
    out["layer_ms"] = slope
    out["layer_frac"] = FLOP_LAYER * B * nx / (slope * 1e-3) / PEAK
    out["fixed_ms"] = per_l[0]
    out["fixed_frac"] = FLOP_FIXED * B * nx / (per_l[0] * 1e-3) / PEAK
    print(json.dumps(out))


if __name__ == "__main__":
    main()
