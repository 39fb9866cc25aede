"""cfg4 (bf16, 4096 ICs x 1024 cells) lane timeline.

`run`: the bench's cfg4 rollout (W1_r2, dt = 3.125e-4, T = 30, metrics, no
trajectory; hf_run's 3 lanes) three times back to back after a warm period,
then random-weight FluxGNN(4,128,L) rollouts at L = 0 and L = 4 the same way,
each group fenced by a 60 ms host sleep so that a kernel trace splits them.
Run it under `rocprofv3 --kernel-trace` (tools/gpu_cfg4_timeline.sh).

`analyze DB`: from the rocpd database, per group: every dispatch's start / end
on its stream (lane), and per rollout step the union of the flux kernels'
intervals, the FV kernels' time that no flux kernel overlaps (exposed FV), and
the gaps where nothing runs; rows sum to the wall span.  Prints one JSON line.

    python tools/cfg4_timeline.py run
    python tools/cfg4_timeline.py analyze /tmp/tl/run_results.db
"""
import json
import os
import sqlite3
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

B, NX, T = 4096, 1024, 30


def run():
    import torch
    from diag_rollout import rand_sd
    from hybridflux import HybridSolver, engine
    from hybridflux._lib import HF_OP_RUN, version
    dt = 5e-3 * 64.0 / NX
    dev = torch.device("cuda", 0)
    solver = HybridSolver(os.path.join(ROOT, "tests", "golden", "weights_W1_r2.npz"), radius=2, nx=NX, dt=dt,
                          device=dev, precision="bf16")
    ics = solver.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
    grid = engine.Grid(NX, dt=dt)
    ws, _ = engine.workspace(HF_OP_RUN, B, NX, T, dev, model=solver._dm())
    fin = torch.empty_like(ics)
    met = torch.empty(B, T + 1, 4, device=dev)
    models = {"W1_r2": solver.model.device_model(dev)}
    for L in (0, 4):
        models[f"rand_L{L}"] = engine.DeviceModel(rand_sd(L), dev, "bf16")
    out = {"build": version(), "B": B, "nx": NX, "T": T, "groups": []}
    for name, dm in models.items():
        def roll():
            engine.run(dm, grid, ics, T, traj=False, metrics=met, out=fin, ws=ws)
        t_end = time.perf_counter() + 0.5  # the sustained clock (MI355X_MICROARCH.md DVFS)
        while time.perf_counter() < t_end:
            roll()
            torch.cuda.synchronize(dev)
        time.sleep(0.06)  # fence: the trace's group boundary
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            roll()
        e1.record()
        torch.cuda.synchronize(dev)
        out["groups"].append({"name": name, "ms_per_step": e0.elapsed_time(e1) / (3 * T)})
        time.sleep(0.06)
        print(f"{name}: {out['groups'][-1]['ms_per_step']:.4f} ms/step", file=sys.stderr, flush=True)
    print(json.dumps(out))


def union(iv):
    """Total length of the union of [s, e) intervals, and the merged list."""
    m = []
    for s, e in sorted(iv):
        if m and s <= m[-1][1]:
            m[-1][1] = max(m[-1][1], e)
        else:
            m.append([s, e])
    return sum(e - s for s, e in m), m


def minus(a, b):
    """Length of merged intervals a not covered by merged intervals b."""
    tot = 0
    for s, e in a:
        cur = s
        for bs, be in b:
            if be <= cur or bs >= e:
                continue
            if bs > cur:
                tot += bs - cur
            cur = max(cur, be)
            if cur >= e:
                break
        if cur < e:
            tot += e - cur
    return tot


def analyze(db, names=("W1_r2", "rand_L0", "rand_L4")):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    # groups: split at host gaps > 30 ms (the fences); keep the groups made of cfg4 rollouts
    groups, cur = [], []
    for r in rows:
        if cur and r[1] - max(x[2] for x in cur[-50:]) > 30e6:
            groups.append(cur)
            cur = []
        cur.append(r)
    if cur:
        groups.append(cur)
    timed = [g for g in groups if sum("chain_flux_sw_kernel" in r[0] for r in g) == 3 * 3 * T]
    out = {"db": db, "groups_found": len(groups), "timed_groups": len(timed), "rows": []}
    for name, g in zip(names, timed):
        flux = [(s, e) for n, s, e, _ in g if "chain_flux_sw_kernel" in n]
        fv = [(s, e) for n, s, e, _ in g if "fv_step" in n]
        other = [(s, e) for n, s, e, _ in g if "chain_flux_sw_kernel" not in n and "fv_step" not in n]
        span = max(e for _, _, e, _ in g) - min(s for _, s, _, _ in g)
        fu, fm = union(flux)
        vu, vm = union(fv)
        au, am = union(flux + fv + other)
        exposed_fv = minus(vm, fm)
        exposed_other = au - fu - exposed_fv
        lanes = sorted({sid for n, _, _, sid in g if "chain_flux_sw_kernel" in n})
        per_lane = {}
        for sid in lanes:
            d = [e - s for n, s, e, t in g if t == sid and "chain_flux_sw_kernel" in n]
            v = [e - s for n, s, e, t in g if t == sid and "fv_step" in n]
            per_lane[str(sid)] = {"flux_us_avg": round(sum(d) / len(d) / 1e3, 2), "flux_n": len(d),
                                  "fv_us_avg": round(sum(v) / max(len(v), 1) / 1e3, 2), "fv_n": len(v)}
        steps = 3 * T
        row = {"group": name, "span_ms_per_step": round(span / steps / 1e6, 4),
               "flux_union_ms_per_step": round(fu / steps / 1e6, 4),
               "flux_sum_ms_per_step": round(sum(e - s for s, e in flux) / steps / 1e6, 4),
               "fv_sum_ms_per_step": round(sum(e - s for s, e in fv) / steps / 1e6, 4),
               "exposed_fv_ms_per_step": round(exposed_fv / steps / 1e6, 4),
               "exposed_other_ms_per_step": round(exposed_other / steps / 1e6, 4),
               "idle_ms_per_step": round((span - au) / steps / 1e6, 4),
               "lanes": per_lane,
               "other_kernels": sorted({n.split("(")[0][:60] for n, _, _, _ in g
                                        if "chain_flux_sw_kernel" not in n and "fv_step" not in n})}
        out["rows"].append(row)
        # the first rollout's dispatches (relative us), lane by lane: the timeline itself
        t0 = min(s for _, s, _, _ in g)
        first = [(n, s, e, t) for n, s, e, t in g if s - t0 < span / 3]
        row["first_rollout_dispatches_us"] = [
            ["flux" if "chain_flux_sw_kernel" in n else "fv" if "fv_step" in n else n.split("(")[0][:24], int(t),
             round((s - t0) / 1e3, 1), round((e - t0) / 1e3, 1)] for n, s, e, t in first]
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        analyze(sys.argv[2])
