"""hf_ablation_loss on a seeded random batch (B = 2000, nx = 64, every
lambda on), saved to the .npz path given: a bitwise A/B of library builds of
the loss pass (HYBRIDFLUX_LIB selects the build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import hybridflux as hf
    from hybridflux import engine
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    out = {}
    for nx in (16, 64, 100):
        B = 2000
        solver = hf.BaselineSolver(nx, device=dev)
        st = (1.0 + 0.1 * torch.randn(B, 3, nx, generator=g)).to(dev)
        sn = (1.0 + 0.1 * torch.randn(B, 3, nx, generator=g)).to(dev)
        ft = (0.1 * torch.randn(B, nx, generator=g)).to(dev)
        fe = (0.1 * torch.randn(B, 2 * nx, generator=g)).to(dev)
        loss, fl, dfe = engine.ablation_loss_terms(solver.grid, fe, st, ft, sn, (1.0, 0.5, 0.25, 0.125))
        out[f"loss_{nx}"] = loss.cpu().numpy()
        out[f"fl_{nx}"] = fl.cpu().numpy()
        out[f"dfe_{nx}"] = dfe.cpu().numpy()
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1], {k: float(v.reshape(-1)[0]) for k, v in out.items() if k.startswith("loss")})


if __name__ == "__main__":
    main()
