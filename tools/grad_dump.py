"""One training step's loss and parameter gradients on the chain path, saved
to an .npz, for bitwise comparisons of library builds (HYBRIDFLUX_LIB selects
the build): the reference dataset recipe, random-init FluxGNN(4, 128, 4),
batch 2000, the ablation config's loss (train_ablation.py:107-206), backward.

    python tools/grad_dump.py OUT.npz [--config physics]
    python tools/grad_dump.py --compare A.npz B.npz
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))


def dump(out, cfg_name, batch):
    import torch
    import hybridflux as hf
    from hybridflux._lib import version
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FluxDataset, ablation_loss
    st, ft, sn, x, dt, dx, nu = generate_dataset(out_path=None, device="cuda", num_initial_conditions=50,
                                                 steps_per_ic=40)
    data = FluxDataset(st, ft, sn, "cuda")
    solver = hf.BaselineSolver(64, device="cuda")
    x_dev = torch.as_tensor(x, device="cuda")
    torch.manual_seed(0)
    m = hf.FluxGNN(4, 128, 4).to("cuda")
    m.flatten_parameters_()
    idx = torch.randint(0, len(data), (batch,), generator=torch.Generator().manual_seed(1)).to("cuda")
    b_st, b_ft, b_sn, nf = data.batch(idx, x_dev)
    loss, fl = ablation_loss(m, b_st, b_ft, b_sn, x_dev, solver.dt, solver.dx, hf.ABLATION_CONFIGS[cfg_name],
                             solver.grid, nf=nf)
    loss.backward()
    res = {"loss": loss.detach().cpu().numpy(), "flux_loss": fl.detach().cpu().numpy()}
    for n, p in m.named_parameters():
        res["grad." + n] = p.grad.detach().cpu().numpy()
    np.savez(out, **res)
    print(version(), out, float(loss))


def compare(a, b):
    A, B = np.load(a), np.load(b)
    worst = 0.0
    same = True
    for k in A.files:
        x, y = A[k], B[k]
        eq = np.array_equal(x.view(np.uint32), y.view(np.uint32))
        d = float(np.max(np.abs(x - y) / (np.abs(x) + 1e-30))) if x.size else 0.0
        worst = max(worst, d)
        same = same and eq
        print(f"{k:40s} {'bitwise' if eq else 'differs'} max rel {d:.3e}")
    print("ALL BITWISE" if same else f"NOT BITWISE (max rel {worst:.3e})")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--config", default="physics")
    ap.add_argument("--batch", type=int, default=2000)
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        compare(*args.compare)
    else:
        dump(args.out, args.config, args.batch)
