"""Cross-calibrate bench.py's CPU baseline (the oracle port, `cpu_baseline.kind
= "port"`) against the reference's own HybridSolver (SURVEY.md 8(d) CPU baseline,
(i) vs (ii)).

Runs ONLY in the build container, where /root/reference exists (the reference
never travels to the GPU box).  Both solvers run the same ICs (seeds 1000..),
the same W1_r3 weights and the same thread count, one IC at a time with the
reference's own loop (src/hybrid_solver.py:34-73): the reference through its
torch.load'ed FluxGNN on device='cpu', the port through
oracle/hybrid_oracle.py:hybrid_run_per_ic.  Prints one JSON line.

    python tools/cpu_calibrate.py [--ics 64] [--steps 30] [--threads 8,1]
"""
import argparse
import json
import os
import sys
import tempfile
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import hybrid_oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ics", type=int, default=64)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--threads", default="8,1")
    a = ap.parse_args()
    if not os.path.isdir(os.path.join(REF, "src")):
        sys.exit("needs the reference tree at /root/reference (build container only)")
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "src"))  # `from config import` (src/hybrid_solver.py:21)
    from src.hybrid_solver import HybridSolver  # noqa: E402

    sd = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights_W1_r3.npz")))
    ckpt = os.path.join(tempfile.mkdtemp(), "W1_r3.pt")
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, ckpt)
    ref = HybridSolver(ckpt, radius=3, device="cpu")
    G = O.Grid(64)
    ics = np.stack([O.initial_condition(G, 1000 + i) for i in range(a.ics)])
    p = O.params_from(sd)

    out = {"ics": a.ics, "steps": a.steps, "nx": 64, "cpu": os.cpu_count(), "runs": []}
    for th in [int(t) for t in a.threads.split(",")]:
        torch.set_num_threads(th)
        ref.run(ics[0], 2)
        O.hybrid_run_per_ic(p, G, ics[:1], 2)
        t0 = time.perf_counter()
        want = np.stack([ref.run(ics[i], a.steps) for i in range(a.ics)])
        t_ref = time.perf_counter() - t0
        t0 = time.perf_counter()
        got = O.hybrid_run_per_ic(p, G, ics, a.steps)
        t_port = time.perf_counter() - t0
        out["runs"].append({
            "threads": th,
            "reference_ic_steps_per_s": round(a.ics * a.steps / t_ref, 1),
            "port_ic_steps_per_s": round(a.ics * a.steps / t_port, 1),
            "port_over_reference": round(t_ref / t_port, 3),
            "max_abs_state_diff": float(np.abs(np.asarray(got, np.float64) - want).max()),
        })
    print(json.dumps(out))


if __name__ == "__main__":
    main()
