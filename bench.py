"""Benchmark: hybrid rollout timesteps/sec (batched ICs) on MI355X.

Workload (BASELINE.json configs[2], the north star's "4096-IC batch of 64-cell
chains at 1 MI355X"): per GPU 4096 independent ICs x 64 cells, FluxGNN(4,128,4)
float32 with the r=3 ablation checkpoint's architecture (weights from the
committed 1-epoch fixture tests/golden/weights_W1_r3.npz), synthetic ICs from
the reference IC generator (seeds 1000 + global IC index).  A step is one full
hybrid timestep of the whole batch: GNN -> flux symmetrisation -> FV
continuity + Burgers -> spectral Poisson; the rollout records every state
(as HybridSolver.run does).  N GPUs: weak scaling, 4096 ICs per rank, no
communication while stepping, one RCCL all_gather of per-IC metrics inside the
timed region — at N = 1 too (a one-rank RCCL group); the line reports the
calls and bytes that exchange actually moved.  The timed rollout's first 16
ICs are checked against the reference's committed trajectories ("parity"),
and a library built with diagnostic flags is refused.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--ics-per-gpu B] [--no-cpu-baseline]
"""
import argparse
import datetime
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, ROOT)
# RCCL / CUDA-tensor sharing between processes needs dmabuf IPC on this host
# driver: set before torch is imported and before anything touches the GPU,
# whoever launched this process (bench.py's own launcher, torchrun, the
# driver; tests/test_distributed_cpu.py::test_bench_sets_ipc_mode_torchrun_style)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GNN_FLOP_PER_CELL_STEP = 329_216   # input 1,024 + layers 262,144 + P/Q readout 66,048
STATE_BYTES_PER_CELL_STEP = 24     # read (n,u,E) + write (n,u,E) float32
PEAK_F32_MFMA_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
PEAK_F16_MFMA_TFLOPS = 2500.0      # MI355X_MICROARCH.md: dense FP16/BF16 matrix peak (no sparsity)
PEAK_HBM_GBS = 8000.0
PEAK_L2_GBS = 34500.0              # MI355X_MICROARCH.md: L2 aggregate ~34.5 TB/s
METRIC = "hybrid rollout timesteps/sec (batched ICs) at 1/2/4/8 MI355X"


def cpu_baseline(weights, nx, T, n_ics, threads):
    """Reference-faithful CPU hybrid solver (oracle port: one IC at a time,
    torch-CPU FluxGNN + numpy FV/FFT, src/hybrid_solver.py:34-73) on a bounded
    sample; plus the batched torch-CPU form for context.  The process is pinned
    to `threads` host cores for the leg (as taskset would), then unpinned."""
    from oracle import hybrid_oracle as O
    torch.set_num_threads(threads)
    p = O.params_from(weights)
    G = O.Grid(nx)
    ics = np.stack([O.initial_condition(G, 1000 + i) for i in range(n_ics)])
    O.hybrid_run_per_ic(p, G, ics[:1], 2)  # warm the allocator / BLAS
    t0 = time.perf_counter()
    O.hybrid_run_per_ic(p, G, ics, T)
    alpha = n_ics * T / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    O.hybrid_run(p, G, ics, T)
    beta = n_ics * T / (time.perf_counter() - t0)
    return alpha, beta


def cpu_batched(weights, nx, T, n_ics, threads):
    """The batched torch-CPU form of the port alone, on `threads` threads (the
    (beta) context figure at the process's full CPU affinity set)."""
    from oracle import hybrid_oracle as O
    torch.set_num_threads(threads)
    p = O.params_from(weights)
    G = O.Grid(nx)
    ics = np.stack([O.initial_condition(G, 1000 + i) for i in range(n_ics)])
    O.hybrid_run(p, G, ics[:8], 2)
    t0 = time.perf_counter()
    O.hybrid_run(p, G, ics, T)
    return n_ics * T / (time.perf_counter() - t0)


def cgroup_cpus():
    """CPUs this process's cgroup may use (cpu.max quota / period), or None when
    unlimited or unreadable.  On the GPU box the affinity set is the whole host
    (256 CPUs) while the share is 16: torch threads beyond the quota only queue."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, int(q) // int(per))
    except (OSError, ValueError):
        return None


_T_START = time.perf_counter()


def progress(msg):
    """A phase marker on stderr (the GPU box's runner kills a run silent for 180 s)."""
    print(f"bench.py [{time.perf_counter() - _T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def pinned(n):
    """The first n CPUs this process may run on (taskset -c equivalent), as a set."""
    avail = sorted(os.sched_getaffinity(0))
    return set(avail[:n])


def timed(fn, dev, reps=1, warm_s=0.3):
    """Warm `fn` (one rollout / step) back to back for warm_s of wall time, so the
    timed calls run at the clock the chip sustains on this workload (after the
    host-side setup the GPU has idled and the clock ramps again,
    MI355X_MICROARCH.md DVFS), then time `reps` calls back to back: HIP events on
    the launch stream and the wall clock around them.  Returns (wall s, event ms)."""
    torch.cuda.synchronize(dev)
    t_end = time.perf_counter() + warm_s
    while time.perf_counter() < t_end:
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):  # back to back: only the first pays the launch latency
        fn()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0, e0.elapsed_time(e1)


def other_config(weights, dev, name, B, nx, precision, K, W, radius, fixture=None, also=None, reps=1, warm_s=0.3,
                 tridiag=False):
    """Time one more BASELINE.json single-GPU config the same way as the
    headline (preallocated outputs and workspace, HIP events on the launch
    stream, wall clock around the launches).  Reported next to the headline,
    never as it.  W untimed warmup steps run first as one rollout, then the
    timed workload itself back to back for warm_s seconds (timed()), so the
    timed rollouts run at the sustained clock (the headline keeps the driver's
    --warmup).  also: the same workload in another precision, reported under
    alt_<precision>; tridiag: the same workload with the opt-in tridiagonal
    Poisson (not the reference's operator), under alt_poisson_tridiagonal.
    fixture: {label: states [n, K+1, 3, nx]} of the batch's first n ICs
    (committed test vectors); the final states' max |error| against each is
    reported."""
    from hybridflux import HybridSolver, engine
    from hybridflux._lib import HF_OP_RUN
    dt = 5e-3 * 64.0 / nx
    solver = HybridSolver(weights, radius=radius, nx=nx, dt=dt, device=dev, precision=precision)
    ics = solver.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    ws, _ = engine.workspace(HF_OP_RUN, B, nx, K, dev, model=solver._dm())
    final = torch.empty_like(ics)
    met = torch.empty(B, K + 1, 4, device=dev)
    solver.run_batch(ics, max(W, 1), traj=False, ws=ws)
    wall, kms = timed(lambda: solver.run_batch(ics, K, traj=False, metrics=met, out=final, ws=ws), dev, reps, warm_s)
    flop = GNN_FLOP_PER_CELL_STEP * B * nx * K * reps
    peak = PEAK_F32_MFMA_TFLOPS if precision == "f32" else PEAK_F16_MFMA_TFLOPS
    out = {"workload": name, "ics": B, "nx": nx, "dt": dt, "precision": precision, "steps": K,
           "rollouts": reps,
           "weights": f"W1_r{radius}",
           "value": round(B * K * reps / wall, 1), "unit": "IC-steps/s", "ms_per_step": round(wall / (K * reps) * 1e3, 4),
           "kernel_ms": round(kms, 3), "mfma_frac": round(flop / (kms * 1e-3) / 1e12 / peak, 4),
           "finite_fraction": float(met[:, -1, 2].float().mean().item())}
    alts = []
    if also:  # the same workload in another precision (reported beside, not instead)
        alts.append((f"alt_{also}", "max_abs_diff_vs_f32_final_state", also,
                     HybridSolver(weights, radius=radius, nx=nx, dt=dt, device=dev, precision=also)))
    if tridiag:  # the opt-in tridiagonal Poisson, same precision (NOT the reference's operator)
        alts.append(("alt_poisson_tridiagonal", "max_abs_diff_vs_spectral_final_state", precision,
                     HybridSolver(weights, radius=radius, nx=nx, dt=dt, device=dev, precision=precision,
                                  poisson="tridiagonal")))
    for key, diff_key, prec, s2 in alts:
        final2 = torch.empty_like(ics)
        s2.run_batch(ics, max(W, 1), traj=False, ws=ws)
        wall2, kms2 = timed(lambda: s2.run_batch(ics, K, traj=False, metrics=met, out=final2, ws=ws), dev, reps,
                            warm_s)
        pk = PEAK_F32_MFMA_TFLOPS if prec == "f32" else PEAK_F16_MFMA_TFLOPS
        out[key] = {"value": round(B * K * reps / wall2, 1), "kernel_ms": round(kms2, 3),
                    "mfma_frac": round(flop / (kms2 * 1e-3) / 1e12 / pk, 4),
                    diff_key: float((final2 - final).abs().max().item())}
    for label, want in (fixture or {}).items():
        n = want.shape[0]
        if want.shape[1] == K + 1:
            got = final[:n].cpu().numpy()
            out[f"max_err_vs_{label}"] = float(np.abs(got.astype(np.float64) - want[:, -1]).max())
    return out


def other_models(dev, B, K, warm_s=0.3):
    """The reference's comparison models (scripts/training/
    train_pure_gnn.py:35-76 PureGNN(4,128,4), train_pinn.py:36-61 PINN(192,256,4))
    as one-launch batched rollouts of B ICs x 64 cells, K steps with the
    trajectory recorded (evaluate_multi_ic.py:45-83), weights from the
    committed fixture tests/golden/baselines.npz; warmed for warm_s of their
    own rollout, then one timed rollout each (HIP events + wall clock).
    Reported next to the headline, never as it."""
    from hybridflux import BaselineSolver
    from hybridflux.baselines import PINN, PureGNN
    b = np.load(os.path.join(ROOT, "tests", "golden", "baselines.npz"))
    solver = BaselineSolver(64, device=dev)
    ics = solver.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    pg = PureGNN(4, 128, 4)
    pg.load_state_dict({k[9:]: torch.from_numpy(b[k]) for k in b.files if k.startswith("pure_gnn.")})
    pn = PINN(3 * 64, 256, 4)
    pn.load_state_dict({k[5:]: torch.from_numpy(b[k]) for k in b.files if k.startswith("pinn.")})
    pg, pn = pg.to(dev), pn.to(dev)
    H, L, nx = 128, 4, 64
    flop = {"pure_gnn": nx * 2 * (4 * H + L * 2 * H * H + H * H + 3 * H),       # tools/bench_models.py
            "pinn": 2 * (3 * nx * 256 + 2 * 256 * 256 + 256 * 3 * nx)}
    fns = {"pure_gnn": lambda: pg.rollout(ics, K, solver.x), "pinn": lambda: pn.rollout(ics, K)}
    # L2 -> CU weight bytes per step of the one-launch rollouts (csrc/baselines.hip): PureGNN one IC
    # per workgroup, each reading the message layers' [W_a ; W_b] and output_mlp.0 (the packed copy);
    # PINN 16 ICs per workgroup, each reading every layer's weights
    pg_w = 4 * (L * 2 * H * H + H * H)
    pn_w = 4 * sum(int(v.numel()) for k, v in pn.state_dict().items() if k.endswith("weight"))
    l2_bytes = {"pure_gnn": B * pg_w, "pinn": -(-B // 16) * pn_w}
    l2_model = {"pure_gnn": f"{B} workgroups x {pg_w} B per step", "pinn": f"{-(-B // 16)} workgroups x {pn_w} B per step"}
    out = {}
    stream = torch.cuda.current_stream(dev)
    for name, fn in fns.items():
        t_end = time.perf_counter() + warm_s
        while time.perf_counter() < t_end:
            fn()
            torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        kms = e0.elapsed_time(e1)
        l2 = l2_bytes[name] * K
        out[name] = {"value": round(B * K / wall, 1), "unit": "IC-steps/s", "ics": B, "nx": nx, "steps": K,
                     "kernel_ms": round(kms, 3), "flop_per_ic_step": flop[name],
                     "mfma_frac": round(flop[name] * B * K / (kms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4),
                     # the other roof of these weight-streaming kernels: every workgroup reads
                     # the whole weight set from L2 each step (algorithmic L2 -> CU bytes)
                     "l2_weight_bytes": l2, "l2_GBs": round(l2 / (kms * 1e-3) / 1e9, 1),
                     "l2_frac": round(l2 / (kms * 1e-3) / (PEAK_L2_GBS * 1e9), 4),
                     "l2_model": l2_model[name]}
    return out


def train_line(dev, batch=2000, steps=20, cfg_name="physics", warm_s=0.3, more=("full", "rollout_only")):
    """SURVEY.md 8(f2), timed inside the driver's bench: one optimizer step of
    the reference trainer's loop (scripts/training/train_ablation.py:119-206:
    the cfg_name ablation loss, loss.backward(), Adam) on `batch` samples of
    the reference dataset recipe (DATASET_CONFIG: 50 ICs x 40 steps, nx = 64,
    generated on the GPU by hybridflux.datagen), FluxGNN(4,128,4) random-init
    (torch.manual_seed(0)).  Eager with torch's default (multi-tensor) Adam,
    eager with its single-kernel fused=True Adam (the same update), replaying
    the captured step (hybridflux.training.GraphedStep, fused capturable
    Adam), and eager / replayed with hybridflux's FlatAdam (the same update in
    one launch over the parameter buffer; with it train_steps takes
    hybridflux.training.direct_step, the autograd step's parameters bit for bit
    without autograd's launches); each warmed for warm_s, then `steps`
    steps timed with HIP events + the wall clock.  Then the configs of `more`
    (the rollout-loss ablations 'full' and 'rollout_only', half of the
    reference's checkpoints) in the best mode.  FLOPs per sample: FluxGNN
    forward + backward (hybridflux.training.train_flop_per_sample: algorithmic,
    no redundant rollout forwards); the loss terms, FV updates and Adam are
    inside the timed step but not counted."""
    from hybridflux import ABLATION_CONFIGS, BaselineSolver, FluxGNN
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FlatAdam, FluxDataset, GraphedStep, train_flop_per_sample, train_steps
    st, ft, sn, x, dt, dx, nu = generate_dataset(out_path=None, device=dev, num_initial_conditions=50,
                                                 steps_per_ic=40)
    data = FluxDataset(st, ft, sn, dev)
    solver = BaselineSolver(64, device=dev)
    x_dev = torch.as_tensor(x, device=dev)

    def arm(name, mode):
        cfg = ABLATION_CONFIGS[name]
        fps = train_flop_per_sample(cfg)
        graphed = mode.startswith("graphed")
        torch.manual_seed(0)
        m = FluxGNN(4, 128, 4).to(dev).flatten_parameters_()
        # graphed: the fused Adam kernel in its capturable form (the multi-tensor
        # capturable Adam costs ~60 us more per step inside the graph); *_flat_adam:
        # the same update in one HIP launch over the parameter buffer (FlatAdam)
        opt = (FlatAdam(m.parameters(), lr=1e-3) if mode.endswith("flat_adam") else
               torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=graphed) if mode != "eager" else
               torch.optim.Adam(m.parameters(), lr=1e-3))
        gs = GraphedStep(m, opt, data, batch, x_dev, solver.dt, solver.dx, cfg, solver.grid) if graphed else None
        gen = torch.Generator().manual_seed(1)
        order = torch.randint(0, len(data), (steps * batch,), generator=gen).to(dev)
        warm = torch.randint(0, len(data), (8 * batch,), generator=gen).to(dev)
        train_steps(m, opt, data, warm, batch, x_dev, solver.dt, solver.dx, cfg, solver.grid, graphed=gs)  # + capture
        wall, kms = timed(lambda: train_steps(m, opt, data, order, batch, x_dev, solver.dt, solver.dx, cfg,
                                              solver.grid, graphed=gs), dev, 1, warm_s)
        rate = steps * batch / wall
        del m, opt, gs
        return rate, {"value": round(rate, 1), "ms_per_step": round(wall / steps * 1e3, 4),
                      "kernel_ms": round(kms, 3), "flop_per_sample": fps,
                      "mfma_frac": round(fps * steps * batch / (kms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4)}

    out = {"metric": f"FluxGNN training samples/s ('{cfg_name}' ablation loss, Adam)", "unit": "samples/s",
           "batch": batch, "steps": steps, "flop_per_sample": train_flop_per_sample(cfg_name),
           "dataset": "DATASET_CONFIG recipe: 50 ICs x 40 steps, nx=64 (GPU classical rollout)"}
    best = None
    for mode in ("eager", "eager_fused_adam", "graphed", "eager_flat_adam", "graphed_flat_adam"):
        progress(f"training line: {mode}")
        rate, out[mode] = arm(cfg_name, mode)
        if best is None or rate > best[1]:
            best = (mode, rate)
    out["value"] = round(best[1], 1)
    out["best"] = best[0]
    for name in more:  # the rollout-loss configs, same step, best mode
        progress(f"training line: '{name}' ({best[0]})")
        rate, r = arm(name, best[0])
        r.update(mode=best[0], vs_physics=round(rate / best[1], 4),
                 note="rollout energy term (train_ablation.py:172-206) in the loss pass, no redundant forwards "
                      "(the reference's 3 rollout forwards reach no energy)")
        out[name] = r
    return out


def pmc_traffic(K, B, nx, traj, build):
    """HBM bytes per launch of the headline kernel from the committed PMC passes
    (tools/gpu_pmc_traffic.sh + tools/pmc_traffic.py): FETCH_SIZE / WRITE_SIZE at two
    step counts give a fixed part and a per-step part, so the figure applies to
    any --steps of the same workload.  The record names the src: hash of the
    library it was measured on; for any other build the figure is not this
    binary's, and the traffic is reported as null with the reason."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    if (t.get("ics_per_gpu"), t.get("nx"), t.get("traj")) != (B, nx, traj) or "per_step_bytes" not in t:
        return None, "profiles/pmc_traffic.json is for another workload"
    if t.get("build") != build:
        return None, f"stale: profiles/pmc_traffic.json was measured on src:{t.get('build')}, this is src:{build}"
    return {"traffic_bytes": t["fixed_bytes"] + t["per_step_bytes"] * K, "source": t["source"],
            "fixed_bytes": t["fixed_bytes"], "per_step_bytes": t["per_step_bytes"], "build": t["build"]}, None


def headline_parity(traj_buf, nx, K, weights_path, precision):
    """Self-check of the timed rollout: the first 16 ICs of rank 0 are seeds
    1000..1015, whose reference trajectories (src/hybrid_solver.py:66-73, run on
    the CPU by tests/golden/make_golden.py) are committed for the default
    weights; the recorded states 0..min(K, 30) must match them within the
    parity tests' rollout gate |gpu - ref| <= 2e-6 + 2e-6 |ref|
    (tests/test_gpu_parity.py ROLL_ATOL / ROLL_RTOL).  None when the timed run
    is not that workload (other weights / nx / precision, or no trajectory)."""
    default_w = os.path.join(ROOT, "tests", "golden", "weights_W1_r3.npz")
    if traj_buf is None or nx != 64 or precision != "f32" or traj_buf.shape[0] < 16 \
            or os.path.abspath(weights_path) != default_w:
        return None
    ref = np.load(os.path.join(ROOT, "tests", "golden", "hybrid_W1_r3_nx64.npz"))
    assert list(ref["seeds"]) == list(range(1000, 1016))
    k = min(K, ref["states"].shape[1] - 1)
    want = ref["states"][:, :k + 1].astype(np.float64)
    got = traj_buf[:16, :k + 1].cpu().numpy().astype(np.float64)
    err = np.abs(got - want)
    excess = float((err - (2e-6 + 2e-6 * np.abs(want))).max())
    return {"max_err_vs_reference_f32": float(err.max()), "ics": 16, "steps_checked": k,
            "gate": "|gpu - ref| <= 2e-6 + 2e-6*|ref| (tests/test_gpu_parity.py ROLL_ATOL/ROLL_RTOL)",
            "within_gate": bool(excess <= 0.0 and np.isfinite(got).all()),
            "reference": "tests/golden/hybrid_W1_r3_nx64.npz (seeds 1000..1015, reference CPU HybridSolver)"}


def rank_report(wall, ics, group=None):
    """The job's timing across ranks, from ONE all_gather of every rank's
    (wall seconds, ICs processed): the max (the job's time: the slowest shard
    ends it) plus, so that a multi-rank line checks itself, each rank's wall
    and IC count and their min / max.  float64 on the CPU for gloo, on the
    rank's HIP device for RCCL; without a process group, this rank alone."""
    if dist.is_initialized():
        backend = dist.get_backend(group)
        dev = torch.device("cuda", torch.cuda.current_device()) if backend != "gloo" else torch.device("cpu")
        world = dist.get_world_size(group)
        mine = torch.tensor([float(wall), float(ics)], dtype=torch.float64, device=dev)
        allr = torch.empty(world * 2, dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(allr, mine, group=group)
        rows = allr.view(world, 2).cpu().tolist()
    else:
        rows = [[float(wall), float(ics)]]
    walls = [r[0] for r in rows]
    return {"wall_s_max": max(walls), "wall_s_min": min(walls), "wall_s_per_rank": [round(w, 6) for w in walls],
            "ics_per_rank": [int(r[1]) for r in rows]}


def collective_entry(coll, world, exchange_ms):
    """The line's config.collective record of the end-of-rollout exchange
    (COLLECTIVES as counted by hybridflux.rollout: one packed all_gather)."""
    return {"op": "all_gather of the per-IC metric series [B,T+1,4] + summaries [B,8] (inside the timed region)",
            "backend": {"nccl": "nccl (RCCL)", "gloo": "gloo"}[coll["backend"]],
            "world_size": world, "calls": coll["calls"],
            "bytes_sent_per_rank": coll["bytes_sent"],
            "bytes_received_per_rank": coll["bytes_received"],
            "exchange_ms": round(exchange_ms, 4)}


class _StdoutToStderr:
    """fd-level redirect of stdout to stderr: RCCL prints its version banner to
    stdout when it sets up (RCCL version / HIP version / ... lines), and this
    script's stdout carries exactly one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import ctypes
        try:
            ctypes.CDLL(None).fflush(None)  # C stdio buffers written while redirected go to stderr too
        except (OSError, AttributeError):
            pass
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def init_group(backend, world, dev):
    """The process group of this job.  RCCL (backend nccl) gets a group at every
    world size, one rank included, so the end-of-rollout metric exchange is a
    real RCCL all_gather on the device even at N = 1 (a plain `python bench.py`
    has no launcher env: it becomes rank 0 of 1 on a free local port).  gloo is
    only for rehearsing N ranks and is not started at N = 1."""
    if world == 1 and backend != "nccl":
        return False
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", str(world))
    # a rank that dies before the first collective ends the job within this
    # bound instead of the 10-minute default (tests/test_distributed_cpu.py)
    timeout = datetime.timedelta(seconds=float(os.environ.get("HF_DIST_TIMEOUT_S", "120")))
    with _StdoutToStderr():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
        # RCCL sets up its communicator and channels on the first collective
        # (hundreds of ms with the GPU idle): do that here, in the setup, so the
        # timed rollout follows the warmup rollout with no idle gap in between
        # (the clock ramps down when the GPU idles, MI355X_MICROARCH.md DVFS)
        dist.all_reduce(torch.zeros(1, device=dev if backend == "nccl" else "cpu"))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    return True


def launch_ranks(n):
    """One child process per rank via torch.distributed.run (127.0.0.1, a free
    port), running this script with the same arguments; never exec: the parent
    stays, waits and returns the launcher's exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--ics-per-gpu", type=int, default=4096)
    ap.add_argument("--nx", type=int, default=64)
    ap.add_argument("--dt", type=float, default=None,
                    help="time step (default 5e-3 * 64/nx: the reference dt at nx=64, same dt/dx otherwise; "
                         "the reference itself NaNs by step 17-33 at nx=1024 with dt=5e-3)")
    ap.add_argument("--weights", default=os.path.join(ROOT, "tests", "golden", "weights_W1_r3.npz"))
    ap.add_argument("--no-traj", action="store_true", help="do not record the state trajectory")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-ics", type=int, default=256)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the measured path); gloo only to rehearse N ranks on fewer GPUs")
    ap.add_argument("--precision", default="f32", choices=["f32", "f16x3", "bf16"],
                    help="chain-kernel arithmetic of the headline line (f32 = exact float32 MFMA)")
    ap.add_argument("--also", default="f16x3",
                    help="comma list of other precisions to time in the same process (reported under 'alt'); '' = none")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the other single-GPU BASELINE configs (cfg2: 256 ICs f32; cfg4: 4096 ICs x 1024 "
                         "cells bf16), reported under 'other_configs' at N=1")
    ap.add_argument("--no-train", action="store_true", help="skip the training side line (SURVEY 8(f2))")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: start the N rank processes here,
        # before this process makes any GPU call, and exit with their code
        # (rank 0's JSON line reaches stdout through the launcher)
        raise SystemExit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    ndev = torch.cuda.device_count()
    if local >= ndev and args.dist_backend != "gloo":
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} visible GPU(s); RCCL needs one GPU per rank")
    dev = torch.device("cuda", local % max(ndev, 1))
    torch.cuda.set_device(dev)
    if os.environ.get("HF_BENCH_EXIT_RANK") == str(rank):
        # fault injection (tests/test_gpu_distributed.py): this rank vanishes
        # before the group forms; its peers must fail within HF_DIST_TIMEOUT_S
        print(f"bench.py: rank {rank} exiting early (HF_BENCH_EXIT_RANK)", file=sys.stderr, flush=True)
        raise SystemExit(0)
    group_error = None
    try:
        grouped = init_group(args.dist_backend, world, dev)
    except Exception as e:  # noqa: BLE001
        if world > 1:
            raise
        # one rank: the rollout needs no peer; report the failed RCCL setup
        # instead of a collective rather than losing the measurement
        grouped, group_error = False, f"{type(e).__name__}: {e}"
        print(f"bench.py: no process group at N = 1 ({group_error})", file=sys.stderr, flush=True)
        if dist.is_initialized():
            dist.destroy_process_group()

    from hybridflux import HybridSolver, engine
    from hybridflux._lib import HF_OP_RUN, build_hash, diagnostic_build, version
    from hybridflux.rollout import COLLECTIVES, gather_rollout, reset_collective_stats, shard_seeds
    if diagnostic_build():
        # HF_DIAG_* / HF_EXP_* builds time deliberately broken or experimental
        # kernels: never a headline (tools/diag_*.py measure those)
        raise SystemExit(f"bench.py: refusing to benchmark a diagnostic build ({version()}); rebuild with make")

    weights = dict(np.load(args.weights, allow_pickle=False))
    B, nx, K, W = args.ics_per_gpu, args.nx, args.steps, args.warmup
    n_total = B * world
    dt = args.dt if args.dt is not None else 5e-3 * 64.0 / nx
    solver = HybridSolver(weights, radius=3, nx=nx, dt=dt, device=dev, precision=args.precision)
    ics = solver.baseline.initial_conditions(shard_seeds(1000, n_total, world, rank), as_tensor=True)
    stream = torch.cuda.current_stream(dev)
    ws, _ = engine.workspace(HF_OP_RUN, B, nx, K, dev, model=solver._dm(), traj=not args.no_traj)

    # every buffer of the warmup and of the timed rollout is allocated first, so
    # the timed launch follows the warmup with no allocation in between
    Wr = max(W, 1)
    final = torch.empty_like(ics)
    traj_buf = None if args.no_traj else torch.empty(B, K + 1, 3, nx, device=dev)
    met_buf = torch.empty(B, K + 1, 4, device=dev)
    warm_traj = None if args.no_traj else torch.empty(B, Wr + 1, 3, nx, device=dev)
    warm_met = torch.empty(B, Wr + 1, 4, device=dev)
    warm_final = torch.empty_like(ics)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if os.environ.get("HF_BENCH_TOUCH", "0") == "1":  # A/B only: first-touch the output buffers before the warmup
        for t in (final, traj_buf, met_buf):
            if t is not None:
                t.zero_()
    torch.cuda.synchronize(dev)

    # warmup: one rollout of W steps (compiles nothing; faults the code objects
    # in) and its metric exchange
    progress(f"headline warmup ({B} ICs x {nx} cells, {Wr} steps)")
    warm = solver.run_batch(ics, Wr, traj=warm_traj if warm_traj is not None else False, metrics=warm_met,
                            out=warm_final, ws=ws)
    gather_rollout(warm, n_total)
    ev_g = torch.cuda.Event(enable_timing=True)
    if world > 1:  # a one-rank group has no one to wait for
        dist.barrier()
    torch.cuda.synchronize(dev)
    reset_collective_stats()
    t0 = time.perf_counter()
    ev0.record(stream)
    res = solver.run_batch(ics, K, traj=traj_buf if traj_buf is not None else False, metrics=met_buf, out=final,
                           ws=ws)
    ev1.record(stream)
    # per-IC summaries (first non-finite step, drifts) on the device,
    # then ONE exchange of the full metric series [B_rank, T+1, K] + summaries
    # (a real all_gather whenever a group exists: RCCL at every N by default)
    gathered = gather_rollout(res, n_total)
    ev_g.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1)
    exchange_ms = ev1.elapsed_time(ev_g)
    coll = dict(COLLECTIVES)
    # the timed rollout's own states against the reference's (before anything
    # below reuses traj_buf)
    parity = headline_parity(traj_buf, nx, K, args.weights, args.precision) if rank == 0 else None

    # diagnostic only (not the value): the same K-step rollout once more, right
    # behind the timed one, i.e. at the clock the chip holds once it is warm;
    # the gap to kernel_ms is the clock ramp after the short warmup
    ev2, ev3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev2.record(stream)
    solver.run_batch(ics, K, traj=traj_buf if traj_buf is not None else False, metrics=met_buf, out=final, ws=ws)
    ev3.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms_again = ev2.elapsed_time(ev3)

    # other precisions, same ICs / K / warmup, timed the same way (reported, not the headline)
    progress("headline timed; alternates")
    alt = {}
    for prec in [p for p in args.also.split(",") if p and p != args.precision]:
        s2 = HybridSolver(weights, radius=3, nx=nx, dt=dt, device=dev, precision=prec)
        s2.run_batch(ics, max(W, 1), traj=not args.no_traj)
        final2 = torch.empty_like(ics)
        torch.cuda.synchronize(dev)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ta = time.perf_counter()
        a0.record(stream)
        r2 = s2.run_batch(ics, K, traj=traj_buf if traj_buf is not None else False, metrics=met_buf, out=final2)
        a1.record(stream)
        torch.cuda.synchronize(dev)
        wall2 = time.perf_counter() - ta
        dev_err = float((final2 - final).abs().max().item())
        alt[prec] = {"value": round(B * K / wall2, 1), "ms_per_step": round(wall2 / K * 1e3, 4),
                     "kernel_ms": round(a0.elapsed_time(a1), 3),
                     "max_abs_diff_vs_headline_final_state": dev_err}
        del s2, r2
    # the north star's tridiagonal Poisson (opt-in, NOT the reference's operator:
    # include/hybridflux.h HF_POISSON_TRIDIAG), fused into the same persistent
    # kernel, same ICs / K / precision, timed the same way
    if not args.no_other_configs:
        s2 = HybridSolver(weights, radius=3, nx=nx, dt=dt, device=dev, precision=args.precision,
                          poisson="tridiagonal")
        s2.run_batch(ics, max(W, 1), traj=not args.no_traj)
        final2 = torch.empty_like(ics)
        torch.cuda.synchronize(dev)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ta = time.perf_counter()
        a0.record(stream)
        s2.run_batch(ics, K, traj=traj_buf if traj_buf is not None else False, metrics=met_buf, out=final2)
        a1.record(stream)
        torch.cuda.synchronize(dev)
        wall2 = time.perf_counter() - ta
        kt = a0.elapsed_time(a1)
        pk = PEAK_F32_MFMA_TFLOPS if args.precision == "f32" else PEAK_F16_MFMA_TFLOPS
        alt["poisson_tridiagonal"] = {
            "value": round(B * K / wall2, 1), "ms_per_step": round(wall2 / K * 1e3, 4), "kernel_ms": round(kt, 3),
            "mfma_frac": round(GNN_FLOP_PER_CELL_STEP * B * nx * K / (kt * 1e-3) / 1e12 / pk, 4),
            "max_abs_diff_vs_headline_final_state": float((final2 - final).abs().max().item()),
            "note": "opt-in cyclic-reduction tridiagonal Poisson (not the reference's spectral operator)"}
        del s2

    # cfg3 names "all ablation radii": the other two checkpoints (W1_r1, W1_r2)
    # on the same ICs, timed the same way (the radius only selects the weights)
    radii = None
    if world == 1 and not args.no_other_configs and nx == 64 and args.precision == "f32":
        radii = {}
        for r in (1, 2):
            wr = dict(np.load(os.path.join(ROOT, "tests", "golden", f"weights_W1_r{r}.npz"), allow_pickle=False))
            s2 = HybridSolver(wr, radius=r, nx=nx, dt=dt, device=dev, precision=args.precision)
            s2.run_batch(ics, max(W, 1), traj=not args.no_traj)
            final_r = torch.empty_like(ics)
            torch.cuda.synchronize(dev)
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ta = time.perf_counter()
            a0.record(stream)
            s2.run_batch(ics, K, traj=traj_buf if traj_buf is not None else False, metrics=met_buf, out=final_r)
            a1.record(stream)
            torch.cuda.synchronize(dev)
            wall2 = time.perf_counter() - ta
            radii[f"W1_r{r}"] = {"value": round(B * K / wall2, 1), "kernel_ms": round(a0.elapsed_time(a1), 3)}
            del s2

    others = None
    if world == 1 and not args.no_other_configs:
        progress("cfg2 / cfg4")
        # cfg4's first ICs (seeds 1000..1003) against committed vectors: the bf16
        # kernels' emulation and the f32 forward on bf16 weights (tests/golden/
        # make_oracle_vectors.py), and the reference's own f32 rollout
        g = np.load(os.path.join(ROOT, "tests", "golden", "bf16_nx1024.npz"))
        ref = np.load(os.path.join(ROOT, "tests", "golden", "hybrid_W1_r2_nx1024.npz"))
        fx = {"bf16_oracle": g["states_emul"], "bf16_weight_f32_oracle": g["states_wbf16"],
              "reference_f32": ref["states"]}
        w_r1 = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights_W1_r1.npz"), allow_pickle=False))
        w_r2 = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights_W1_r2.npz"), allow_pickle=False))
        # both at BASELINE's T = 30, warmed for as many steps as they time
        # cfg2's 30-step rollout lasts ~1.4 ms, so twenty run back to back (the
        # first launch's host latency would otherwise be ~4 % of the timed region)
        others = [other_config(w_r1, dev, "cfg2: 64-cell chain, 256-IC batch, r=1, f32", 256, 64, "f32", 30, 30, 1,
                               also="f16x3", reps=20),
                  other_config(w_r2, dev, "cfg4: 1024-cell chain, 4096-IC batch, r=2, bf16 MLP weights, dt=3.125e-4",
                               4096, 1024, "bf16", 30, 30, 2, fixture=fx, tridiag=True)]

    if world == 1 and not args.no_other_configs:
        progress("PureGNN / PINN")
    models = other_models(dev, 4096, 30) if world == 1 and not args.no_other_configs else None
    if world == 1 and not args.no_other_configs and not args.no_train:
        progress("training line")
    train = train_line(dev) if world == 1 and not args.no_other_configs and not args.no_train else None

    ranks = rank_report(wall, B)  # one all_gather: the max over ranks and each rank's wall / ICs
    wall_max = ranks["wall_s_max"]
    finite = float(gathered["metrics"][:, -1, 2].float().mean().item())
    exploded = int((gathered["summary"][:, 0] >= 0).sum().item())

    if rank == 0:
        traffic, traffic_why = pmc_traffic(K, B, nx, not args.no_traj, build_hash())
        value = n_total * K / wall_max
        flop = GNN_FLOP_PER_CELL_STEP * B * nx * K
        achieved = flop / (kernel_ms * 1e-3) / 1e12
        peak = PEAK_F32_MFMA_TFLOPS if args.precision == "f32" else PEAK_F16_MFMA_TFLOPS
        fused = nx in (16, 32, 48, 64)
        kernel = (f"chain_rollout_kernel<{args.precision},MT={nx // 16}> (one persistent launch)" if fused else
                  f"chain_flux_kernel<{args.precision},window> + fv_step_kernel<hybrid> per step")
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            # the GPU box's CPU share is 16 cores (os.cpu_count() there shows the whole host)
            cores = pinned(min(16, len(os.sched_getaffinity(0))))
            keep = os.sched_getaffinity(0)
            os.sched_setaffinity(0, cores)
            try:
                progress(f"cpu baseline on {len(cores)} pinned cores")
                alpha, beta = cpu_baseline(weights, nx, 30, args.cpu_sample_ics, len(cores))
            finally:
                os.sched_setaffinity(0, keep)
            quota = cgroup_cpus()
            n_all = min(len(keep), quota) if quota else len(keep)
            progress(f"cpu baseline: batched form on {n_all} threads (affinity {len(keep)}, cgroup {quota})")
            beta_all = cpu_batched(weights, nx, 30, args.cpu_sample_ics, n_all)
            cpu = {"value": round(alpha, 1), "unit": "IC-steps/s", "cores": len(cores), "kind": "port",
                   "sample": f"{args.cpu_sample_ics} ICs x 30 steps, one IC at a time (reference-faithful "
                             f"HybridSolver loop: torch-CPU FluxGNN + numpy FV/FFT), nx={nx}",
                   "pinned_cpus": f"{min(cores)}-{max(cores)} ({len(cores)} of host nproc {os.cpu_count()})",
                   "batched_torch_cpu_value": round(beta, 1),
                   "batched_torch_cpu_all_cores": {
                       "value": round(beta_all, 1), "threads": n_all, "affinity_cpus": len(keep),
                       "cgroup_cpus": quota,
                       "note": "the batched form on every CPU the process may use: its affinity set, capped at "
                               "its cgroup CPU quota (threads beyond the quota only queue)"}}
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "IC-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(wall_max / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"f32": "f32", "f16x3": "f16x3 (fp32-accurate split: 3 fp16 MFMA products, f32 accumulate)",
                      "bf16": "bf16 (f32 accumulate)"}[args.precision],
            "data": "synthetic: reference IC generator seeds 1000.., fixture weights W1_r3 (1-epoch reference trainer)",
            "config": {"workload": f"{'cfg3' if (nx == 64 and B == 4096) else 'cfg2' if (nx == 64 and B == 256) else 'cfg4' if nx == 1024 else 'custom'}: {nx}-cell periodic chain, {B}-IC batch per GPU, FluxGNN(4,128,4) {args.precision}, "
                                   f"{K}-step persistent rollout{'' if args.no_traj else ' recording every state'}",
                       "nx": nx, "dt": dt, "ics_per_gpu": B, "global_ics": n_total, "parallelism": f"ic-shard x{world}",
                       "collective": (collective_entry(coll, world, exchange_ms) if coll["calls"] else
                                      ({"backend": "none", "error": group_error} if group_error else None)),
                       # per-rank timing, so that an N > 1 line checks itself (the value uses the max);
                       # multi-GPU scaling of this path is unmeasured on hardware by this repo
                       "ranks": ranks if world > 1 else None},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "traffic": traffic["traffic_bytes"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else traffic_why,
                         "traffic_build": traffic["build"] if traffic else None,
                         "traffic_model": ({"fixed_bytes": traffic["fixed_bytes"],
                                            "per_step_bytes": traffic["per_step_bytes"]} if traffic else None),
                         "algorithmic_bytes": (12 * B * nx * (K + 1) if not args.no_traj else 0)
                                              + 24 * B * nx + 4 * B * (K + 1) * 4,
                         "kernel": kernel, "kernel_ms": round(kernel_ms, 3),
                         "kernel_ms_next_rollout": round(kernel_ms_again, 3),
                         "flop_per_launch": flop,
                         "hbm_state_frac": round(STATE_BYTES_PER_CELL_STEP * B * nx * K / (kernel_ms * 1e-3)
                                                 / (PEAK_HBM_GBS * 1e9), 6)},
            "cpu_baseline": cpu,
            "parity": parity,
            "finite_fraction": finite,
            "exploded_ics": exploded,
            "build": version(),
            # SURVEY.md 8(d) secondary rates: batch-steps/s = T / wall, cell-steps/s = IC-steps/s * nx
            "also": {"batch_steps_per_s": round(K / wall_max, 1), "cell_steps_per_s": round(value * nx, 1)},
            "alt": alt or None,
            "radii": radii,
            "other_configs": others,
            # the reference's PureGNN / PINN rollouts, 4096 ICs x 64 cells, T = 30
            "other_models": models,
            # the batched training step (reference trainer's loop), B = 2000
            "train": train,
        }
        print(json.dumps(line), flush=True)
    if grouped:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
