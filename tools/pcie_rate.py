"""Rates of the drop-in boundary when it hands over HOST buffers (the
reference's numpy / CPU-tensor call patterns), i.e. PCIe-inclusive: never the
bench value (bench.py times device-resident inputs), reported in DESIGN.md.

  batch: HybridSolver.run_batch on a host numpy batch (cfg3: 4096 ICs x 64
         cells, W1_r3, 50 steps), the trajectory copied back into host memory
         (pinned and pageable destinations);
  per_ic: the reference's own loop shape, HybridSolver.run(numpy state, 50)
         one IC at a time (src/hybrid_solver.py:66-73) for 64 ICs;
  step:  HybridSolver.step(numpy state) per call (src/hybrid_solver.py:34-64);
  flux:  FluxGNN(4,64,3) on host tensors, examples/smoke_test.py:50-55 shape.

    python tools/pcie_rate.py > profiles/r04_pcie_rates.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    import hybridflux as hf
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights_W1_r3.npz")))
    s = hf.HybridSolver(w, radius=3, device=dev)
    B, T = 4096, 50
    ics = s.baseline.initial_conditions(range(1000, 1000 + B))          # numpy [B,3,64]
    out = {"build": hf._lib.version()}
    traj_dev = torch.empty(B, T + 1, 3, 64, device=dev)
    host_pinned = torch.empty(B, T + 1, 3, 64, pin_memory=True)
    ws, _ = hf.engine.workspace(hf._lib.HF_OP_RUN, B, 64, T, dev, model=s._dm(), traj=True)

    def dev_only():
        s.run_batch(torch.as_tensor(ics, device=dev), T, traj=traj_dev, ws=ws)

    def host_pinned_fn():
        s.run_batch(ics, T, traj=traj_dev, ws=ws)
        host_pinned.copy_(traj_dev, non_blocking=True)

    def host_numpy():
        s.run_batch(ics, T, traj=traj_dev, ws=ws)
        traj_dev.cpu().numpy()

    bytes_h2d = ics.nbytes
    bytes_d2h = traj_dev.numel() * 4
    for name, fn in (("device_resident_ics", dev_only), ("host_ics_pinned_traj", host_pinned_fn),
                     ("host_ics_numpy_traj", host_numpy)):
        sec = timed(fn, 5)
        out[f"batch_{name}"] = {"ic_steps_per_s": round(B * T / sec, 1), "ms": round(sec * 1e3, 3)}
    out["batch_bytes"] = {"h2d_ics": bytes_h2d, "d2h_trajectory": bytes_d2h}
    n_ic = 64
    per = timed(lambda: [s.run(ics[i], T) for i in range(n_ic)], 2)
    out["per_ic_run_numpy"] = {"ics": n_ic, "steps": T, "ic_steps_per_s": round(n_ic * T / per, 1),
                               "ms_per_ic_rollout": round(per / n_ic * 1e3, 3)}
    st = ics[0]
    step_s = timed(lambda: s.step(st), 200)
    out["step_numpy"] = {"us_per_call": round(step_s * 1e6, 1)}
    torch.manual_seed(0)
    m = hf.FluxGNN(4, 64, 3)
    nf, ei = torch.randn(64, 4), torch.randint(0, 64, (2, 128))
    with torch.no_grad():
        f_s = timed(lambda: m(nf, ei), 200)
    g_s = timed(lambda: m(nf, ei).sum().backward(), 100)
    out["fluxgnn_host_tensors"] = {"forward_us": round(f_s * 1e6, 1), "forward_backward_us": round(g_s * 1e6, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
