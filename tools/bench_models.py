"""The reference's timing harness (scripts/evaluation/benchmark_timing.py) on the MI355X.

For every method the reference times — classical solver, hybrid FluxGNN
solver, PureGNN, PINN — report
  * `single_ic_s`: one 50-step rollout of the seed-42 IC, the reference's own
    methodology (N_RUNS=10 timed runs after a warmup, mean seconds per run);
  * `batched`: IC-steps/s for a 4096-IC batch, 50 steps, trajectory recorded,
    with the model's algorithmic FLOPs per IC-step (`flop_per_ic_step`, the
    matrix products of its forward) and the fraction of the fp32 MFMA peak
    (157.3 TFLOP/s) the batched rate reaches.
Weights are random-init of each architecture (no checkpoints ship with the
reference).  CPU column: the oracle restatements, one IC, 50 steps (bounded).

    python tools/bench_models.py [--batch 4096] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, ROOT)


def timed(fn, runs):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.mean(ts))


PEAK_F32 = 157.3e12  # dense fp32 MFMA, MI355X_MICROARCH.md


def flop_per_ic_step(name, nx=64, H=128, L=4, pinn_h=256, pinn_l=4):
    """Matrix-product FLOPs of one model step of one IC (2 per MAC; activations,
    FV, Poisson and the edge sums not counted)."""
    if name == "hybrid":  # FluxGNN(4,128,4): input, L update layers [h; agg] -> H, P/Q readout,
        # w2 . ReLU(z) of both edges (bench.py's 329,216 per cell)
        return nx * (2 * (4 * H + L * 2 * H * H + 2 * H * H) + 4 * H)
    if name == "pure_gnn":  # input, L layers of P = W_a h, Q = W_b h, output H -> H -> 3
        return nx * 2 * (4 * H + L * 2 * H * H + H * H + 3 * H)
    if name == "pinn":  # 3nx -> h, (L-2) x h -> h, h -> 3nx
        D = 3 * nx
        return 2 * (D * pinn_h + (pinn_l - 2) * pinn_h * pinn_h + pinn_h * D)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    import hybridflux as hf
    T, B = args.steps, args.batch
    torch.manual_seed(0)
    solver = hf.BaselineSolver(64, device="cuda")
    x = solver.x
    ic42 = torch.as_tensor(solver.initial_condition(seed=42), device="cuda")[None]
    ics = solver.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    flux = hf.FluxGNN(4, 128, 4)
    sd = {k: v.clone() for k, v in flux.state_dict().items()}
    hyb = hf.HybridSolver(sd, radius=2, device="cuda")
    pg = hf.PureGNN(4, 128, 4).to("cuda")
    pn = hf.PINN(3 * 64, 256, 4).to("cuda")
    methods = {
        "classical": (lambda s: solver.run_batch(s, T, traj=True)),
        "hybrid": (lambda s: hyb.run_batch(s, T)),
        "pure_gnn": (lambda s: pg.rollout(s, T, x)),
        "pinn": (lambda s: pn.rollout(s, T)),
    }
    res = {}
    for name, fn in methods.items():
        single = timed(lambda: fn(ic42), args.runs)
        batched = timed(lambda: fn(ics), 3)
        res[name] = {"single_ic_s": round(single, 6), "single_ic_steps_per_s": round(T / single, 1),
                     "batched_ic_steps_per_s": round(B * T / batched, 1), "batched_ms_per_step": round(batched / T * 1e3, 4)}
        fl = flop_per_ic_step(name)
        if fl:
            tf = fl * B * T / batched
            res[name].update(flop_per_ic_step=fl, batched_tflops=round(tf / 1e12, 2),
                             frac_of_f32_peak=round(tf / PEAK_F32, 4))
        print(name, res[name], file=sys.stderr, flush=True)
    cpu = None
    if not args.no_cpu:
        from oracle import hybrid_oracle as O
        torch.set_num_threads(16)
        grid = O.Grid(64)
        st0 = O.initial_condition(grid, 42)
        p = O.params_from(sd)
        pgp = O.params_from({k: v.cpu() for k, v in pg.state_dict().items()})
        pnp = O.params_from({k: v.cpu() for k, v in pn.state_dict().items()})

        def pinn_roll():
            with torch.no_grad():
                s = torch.from_numpy(st0)
                for _ in range(T):
                    s = O.pinn_forward(pnp, s[None])[0]

        cpu_fns = {"classical": lambda: O.classical_run(grid, st0[None], T),
                   "hybrid": lambda: O.hybrid_run_per_ic(p, grid, st0[None], T),
                   "pure_gnn": lambda: O.pure_gnn_rollout(pgp, grid, st0, T),
                   "pinn": pinn_roll}
        cpu = {}
        for name, fn in cpu_fns.items():
            fn()
            t0 = time.perf_counter()
            for _ in range(3):
                fn()
            cpu[name] = round((time.perf_counter() - t0) / 3, 5)
        cpu = {"single_ic_s": cpu, "cores": 16, "kind": "port",
               "sample": f"seed-42 IC, {T} steps, oracle restatements on torch-CPU/numpy, mean of 3 runs"}
    print(json.dumps({"metric": "benchmark_timing.py methods on MI355X", "steps": T, "batch": B,
                      "weights": "random init of each architecture", "gpu": res, "cpu_baseline": cpu}))


if __name__ == "__main__":
    main()
