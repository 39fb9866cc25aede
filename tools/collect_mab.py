"""Collect tools/gpu_models_ab.sh results (gpurun_out/mab_<TAG>_<lib>_<rep>.json)
into one JSON line per run:  python tools/collect_mab.py TAG [TAG ...] > profiles/X.jsonl"""
import glob
import json
import sys

for tag in sys.argv[1:]:
    for f in sorted(glob.glob(f"gpurun_out/mab_{tag}_*.json")):
        d = json.load(open(f))
        g = d["gpu"]
        rec = {"run": f.split("/")[-1][4:-5],
               "tool": "tools/bench_models.py --no-cpu (4096 ICs x 64 cells, 50 steps, traj)"}
        for m in ("pure_gnn", "pinn"):
            rec[m] = {k: g[m][k] for k in ("batched_ic_steps_per_s", "single_ic_s", "frac_of_f32_peak") if k in g[m]}
        print(json.dumps(rec))
