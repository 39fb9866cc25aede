"""Timing of the FV/Poisson kernels alone at FFT sizes (HIP events, 50 calls):
the classical step (fv_step_pair_kernel<false>) and hf_poisson at B ICs x nx,
with the algorithmic HBM bytes and the fraction of 8 TB/s.

    python tools/diag_fv.py [nx] [B]      (HYBRIDFLUX_LIB selects a diagnostic build)
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-plasma-flux_amd"))
import torch  # noqa: E402

from hybridflux import BaselineSolver, engine  # noqa: E402


def timed(fn, n=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us


def main(nx=1024, B=4096):
    dev = torch.device("cuda:0")
    s = BaselineSolver(nx=nx, dt=5e-3 * 64 / nx, device=dev)
    st = s.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    out = torch.empty_like(st)
    n = st[:, 0].contiguous()
    step_us = timed(lambda: engine.step(None, s.grid, st))
    pois_us = timed(lambda: engine.poisson(s.grid, n))
    step_bytes = 24 * B * nx
    print(json.dumps({"nx": nx, "B": B, "lib": os.environ.get("HYBRIDFLUX_LIB", "in-tree"),
                      "fv_step_us": round(step_us, 2), "fv_step_bytes": step_bytes,
                      "fv_step_hbm_frac": round(step_bytes / (step_us * 1e-6) / 8e12, 4),
                      "poisson_us": round(pois_us, 2), "poisson_bytes": 8 * B * nx,
                      "poisson_hbm_frac": round(8 * B * nx / (pois_us * 1e-6) / 8e12, 4)}))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:3]])
