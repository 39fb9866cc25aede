"""hf_run's lane streams under HIP-graph capture (diagnostic): a cfg4-sized
bf16 rollout captured with torch.cuda.graph and replayed equals the eager call."""
import os, sys, torch, numpy as np
sys.path.insert(0, "gnn-plasma-flux_amd")
from hybridflux import engine
from hybridflux import HybridSolver
dev = torch.device("cuda", 0)
B, nx, T = 3075, 1024, 2
grid = engine.Grid(nx, dt=3.125e-4)
w = dict(np.load("tests/golden/weights_W1_r2.npz"))
m = engine.DeviceModel(w, dev, "bf16")
solver = HybridSolver(w, radius=2, nx=nx, dt=3.125e-4, device=dev, precision="bf16")
ics = solver.baseline.initial_conditions(range(1000, 1000 + B), as_tensor=True)
ref = engine.run(m, grid, ics, T, traj=False)["final"].clone()
out = torch.empty_like(ics)
ws, _ = engine.workspace(1, B, nx, T, dev, model=m)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    engine.run(m, grid, ics, T, traj=False, out=out, ws=ws)  # warm on the capture stream
torch.cuda.current_stream(dev).wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
out.zero_()
with torch.cuda.graph(g):
    engine.run(m, grid, ics, T, traj=False, out=out, ws=ws)
g.replay()
torch.cuda.synchronize()
print("graph replay equal:", torch.equal(out, ref))
