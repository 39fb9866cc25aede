"""A/B of hf_run's two-lane generic rollout (diagnostic, not a bench line).

Times the cfg4 workload (4096 ICs x 1024 cells, bf16, 30 steps, W1_r2) and the
same grid in f32 / f16x3 through HybridSolver.run_batch, with HIP events on the
launch stream, and records a hash of every final state so runs with
HF_RUN_LANES=1 and =2 (separate processes: the library reads it once) can be
checked bit-identical.

    HF_RUN_LANES=1 python tools/lanes_ab.py out.json
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))

import torch  # noqa: E402

from hybridflux import HybridSolver, engine  # noqa: E402
from hybridflux._lib import HF_OP_RUN  # noqa: E402


def main():
    out_path = sys.argv[1]
    B, nx, T = 4096, 1024, 30
    dt = 5e-3 * 64.0 / nx
    dev = torch.device("cuda", 0)
    w = os.path.join(ROOT, "tests", "golden", "weights_W1_r2.npz")
    res = {"lanes": os.environ.get("HF_RUN_LANES", "default")}
    for prec in os.environ.get("LANES_AB_PREC", "bf16,f32,f16x3").split(","):
        solver = HybridSolver(w, radius=2, nx=nx, dt=dt, device=dev, precision=prec)
        ics = solver.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
        ws, _ = engine.workspace(HF_OP_RUN, B, nx, T, dev, model=solver._dm())
        final = torch.empty_like(ics)
        met = torch.empty(B, T + 1, 4, device=dev)
        solver.run_batch(ics, T, traj=False, metrics=met, out=final, ws=ws)
        stream = torch.cuda.current_stream(dev)
        times = []
        for _ in range(3):
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            solver.run_batch(ics, T, traj=False, metrics=met, out=final, ws=ws)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            times.append(e0.elapsed_time(e1))
        h = hashlib.sha256(final.cpu().numpy().tobytes() + met.cpu().numpy().tobytes()).hexdigest()[:16]
        res[prec] = {"ms": [round(t, 3) for t in times], "ms_per_step": round(min(times) / T, 4),
                     "ic_steps_per_s": round(B * T / (min(times) * 1e-3), 1), "hash": h}
        print(prec, res[prec], flush=True)
        del solver, ws, final, met
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
