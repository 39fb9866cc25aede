"""Where the headline kernel's fixed HBM reads come from.

Launches the fused rollout kernel (f32, nx = 64) in this order, no
trajectory, under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (tools/
gpu_traffic_xcd.sh), and prints the launch order:
  W1_r3 (4 layers, 640 KiB weight stream): B = 4 (1 workgroup) at T = 0, 2, 8;
    B = 8, 32, 256 at T = 2; B = 4096 (1024 workgroups) at T = 0, 2, 8;
  random FluxGNN(4,128,L) for L = 0 (128 KiB stream) and 8 (1152 KiB): B = 4
    and 4096 at T = 2.
Fixed reads that follow the weight stream's size (and not T) are the
stream's first pass; reads that follow B are the states."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from diag_rollout import rand_sd  # noqa: E402


def main():
    from hybridflux import HybridSolver, engine
    dev = torch.device("cuda", 0)
    solver = HybridSolver(os.path.join(ROOT, "tests", "golden", "weights_W1_r3.npz"), radius=3, device=dev)
    ics = solver.baseline.initial_conditions(range(1000, 5096), as_tensor=True)
    grid = engine.Grid(64)
    runs = [("W1_r3", solver._dm(), B, T) for B, T in ((4, 0), (4, 2), (4, 8), (8, 2), (32, 2), (256, 2),
                                                        (4096, 0), (4096, 2), (4096, 8))]
    models = {L: engine.DeviceModel(rand_sd(L), dev, "f32") for L in (0, 8)}
    runs += [(f"rand_L{L}", models[L], B, 2) for L in (0, 8) for B in (4, 4096)]
    for i, (name, dm, B, T) in enumerate(runs):
        engine.run(dm, grid, ics[:B].contiguous(), T, traj=False)
        torch.cuda.synchronize()
        print(f"launch {i} weights={name} B={B} workgroups={(B + 3) // 4} T={T}", flush=True)


if __name__ == "__main__":
    main()
