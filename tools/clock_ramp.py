"""Headline kernel time of twelve back-to-back 20-step rollouts after a 5-step
warmup (the driver's --steps 20 --warmup 5), with a 0.5 s idle after the
sixth: shows the clock ramp after idle (HIP events, ms per rollout)."""
import os, sys, time, json
sys.path.insert(0, "gnn-plasma-flux_amd")
import numpy as np, torch
from hybridflux import HybridSolver, engine
from hybridflux._lib import HF_OP_RUN
dev = torch.device("cuda", 0)
w = dict(np.load("tests/golden/weights_W1_r3.npz"))
s = HybridSolver(w, radius=3, device=dev)
ics = s.baseline.initial_conditions(range(1000, 1000 + 4096), as_tensor=True)
ws, _ = engine.workspace(HF_OP_RUN, 4096, 64, 20, dev, model=s._dm(), traj=True)
s.run_batch(ics, 5, traj=True, metrics=True, ws=ws)
torch.cuda.synchronize()
tr = torch.empty(4096, 21, 3, 64, device=dev); me = torch.empty(4096, 21, 4, device=dev); fin = torch.empty_like(ics)
out = []
for i in range(12):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); s.run_batch(ics, 20, traj=tr, metrics=me, out=fin, ws=ws); b.record(); torch.cuda.synchronize()
    out.append(round(a.elapsed_time(b), 3))
    if i == 5: time.sleep(0.5)
print(json.dumps(out))
