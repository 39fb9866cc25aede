"""How long cfg4 (4096 ICs x 1024 cells, bf16, W1_r2) must be warmed before its
timed 30-step rollout runs at the sustained clock (diagnostic, not a bench
line).  Each trial idles 1 s (as bench.py's host-side setup before cfg4 does),
runs W warmup steps, then times one 30-step rollout with HIP events.

    python tools/cfg4_warmup_ab.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))

import torch  # noqa: E402

from hybridflux import HybridSolver, engine  # noqa: E402
from hybridflux._lib import HF_OP_RUN  # noqa: E402


def main():
    B, nx, T = 4096, 1024, 30
    dt = 5e-3 * 64.0 / nx
    dev = torch.device("cuda", 0)
    solver = HybridSolver(os.path.join(ROOT, "tests", "golden", "weights_W1_r2.npz"), radius=2, nx=nx, dt=dt,
                          device=dev, precision="bf16")
    ics = solver.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    ws, _ = engine.workspace(HF_OP_RUN, B, nx, T, dev, model=solver._dm())
    final = torch.empty_like(ics)
    met = torch.empty(B, T + 1, 4, device=dev)
    stream = torch.cuda.current_stream(dev)
    res = {}
    if os.environ.get("CFG4_SEQ"):  # one warmup, then 6 back-to-back timed rollouts, each timed
        torch.cuda.synchronize(dev)
        time.sleep(1.0)
        solver.run_batch(ics, 30, traj=False, ws=ws)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(7)]
        ev[0].record(stream)
        for i in range(6):
            solver.run_batch(ics, T, traj=False, metrics=met, out=final, ws=ws)
            ev[i + 1].record(stream)
        torch.cuda.synchronize(dev)
        print(json.dumps({"what": "cfg4: 30 warmup steps after 1 s idle, then six back-to-back 30-step rollouts (ms each)",
                          "ms": [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(6)]}))
        return
    for W in (30, 90, 30, 90, 60):
        torch.cuda.synchronize(dev)
        time.sleep(1.0)
        solver.run_batch(ics, W, traj=False, ws=ws)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        solver.run_batch(ics, T, traj=False, metrics=met, out=final, ws=ws)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        res.setdefault(f"W{W}", []).append(round(e0.elapsed_time(e1), 3))
        print(W, res[f"W{W}"][-1], flush=True)
    print(json.dumps({"what": "cfg4 timed 30-step rollout (ms) after 1 s idle + W warmup steps", "ms": res}))


if __name__ == "__main__":
    main()
