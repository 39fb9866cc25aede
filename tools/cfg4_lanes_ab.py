"""cfg4 (4096 ICs x 1024 cells, bf16, W1_r2, T = 30) rollout time for A/B runs
of hf_run's lane cuts (HF_LANE_CUTS=even vs the default round-aware cuts,
capi.cpp lane_cuts): 0.3 s of the same rollout to reach the sustained clock,
then 3 timed rollouts; prints one JSON line.

    HF_LANE_CUTS=even python tools/cfg4_lanes_ab.py TAG
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(tag):
    from hybridflux import HybridSolver, engine
    from hybridflux._lib import HF_OP_RUN, version
    dev = torch.device("cuda", 0)
    w = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights_W1_r2.npz")))
    B, nx, T = 4096, 1024, 30
    s = HybridSolver(w, radius=2, nx=nx, dt=3.125e-4, device=dev, precision="bf16")
    ics = s.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    ws, _ = engine.workspace(HF_OP_RUN, B, nx, T, dev, model=s._dm())
    out = torch.empty_like(ics)
    met = torch.empty(B, T + 1, 4, device=dev)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        s.run_batch(ics, T, traj=False, metrics=met, out=out, ws=ws)
        torch.cuda.synchronize(dev)
    ms = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s.run_batch(ics, T, traj=False, metrics=met, out=out, ws=ws)
        e1.record()
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1) / T)
    flop = 329_216 * B * nx
    print(json.dumps({"tag": tag, "lane_cuts": os.environ.get("HF_LANE_CUTS", "rounds"), "ms_per_step": ms,
                      "mfma_frac": [round(flop / (m * 1e-3) / 2.5e15, 4) for m in ms],
                      "final_checksum": float(out.double().sum().item()), "build": version()}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "")
