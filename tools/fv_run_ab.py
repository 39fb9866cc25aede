"""Classical rollout at FFT sizes (BaselineSolver.run, src/baseline_solver.py:80-118):
T-step engine.run of B ICs, timed with HIP events on the library's stream
(torch's current stream), in the configuration the environment selects
(HF_FV_PERSIST=0: per-step fv_step_fft_kernel launches; unset: the one-launch
register-resident fv_run_fft_kernel).  Reports us per step and the HBM
fraction of the algorithmic bytes (trajectory rows 12 B/cell-step when
recorded; the per-step path moves 24 B/cell-step either way).

    python tools/fv_run_ab.py [nx] [B] [T]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-plasma-flux_amd"))
import torch  # noqa: E402

from hybridflux import BaselineSolver, engine  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us per call


def main(nx=1024, B=4096, T=30):
    dev = torch.device("cuda:0")
    s = BaselineSolver(nx=nx, dt=5e-3 * 64 / nx, device=dev)
    st = s.initial_conditions(range(1000, 1000 + B), as_tensor=True).contiguous()
    out = {"nx": nx, "B": B, "T": T, "persist": os.environ.get("HF_FV_PERSIST", "1")}
    tr = torch.empty(B, T + 1, 3, nx, device=dev)
    me = torch.empty(B, T + 1, 4, device=dev)
    fin = torch.empty_like(st)
    ws = engine.workspace(engine.HF_OP_RUN, B, nx, T, dev)[0]
    for name, kw, traj_bytes in (("traj", dict(traj=tr, metrics=me), 12), ("final_only", dict(traj=False), 0)):
        us = timed(lambda: engine.run(None, s.grid, st, T, out=fin, ws=ws, **kw)) / T
        alg = (traj_bytes * B * nx * T + 24 * B * nx) / T  # per step: rows written + state0/final amortised
        out[name] = {"us_per_step": round(us, 2), "alg_bytes_per_step": int(alg),
                     "hbm_frac": round(alg / (us * 1e-6) / 8e12, 4)}
    final = engine.run(None, s.grid, st, T, traj=False)["final"]
    out["final_sha"] = __import__("hashlib").sha256(final.cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps(out))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:4]])
