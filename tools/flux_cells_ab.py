"""FluxGNN.forward on 256 chains of 64 cells (the cell-split flux kernel), 50
forwards per precision, HIP events on the launch stream (diagnostic; run
once per library build with HYBRIDFLUX_LIB=... to A/B them).

    python tools/flux_cells_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hybridflux import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    w = dict(np.load(os.path.join(ROOT, "tests", "golden", "weights_W1_r1.npz"), allow_pickle=False))
    B, nx = 256, 64
    g = torch.Generator().manual_seed(0)
    nf = (torch.rand(B * nx, 4, generator=g) * 0.2 + 0.9).to(dev)
    out = {}
    for prec in ("f32", "bf16", "f16x3"):
        m = engine.DeviceModel(w, dev, prec)
        engine.chain_flux(m, nf, B, nx)
        stream = torch.cuda.current_stream(dev)
        best = None
        for _ in range(3):
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(50):
                engine.chain_flux(m, nf, B, nx)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            t = e0.elapsed_time(e1)
            best = t if best is None else min(best, t)
        out[prec] = round(best, 4)
    print(json.dumps({"lib": os.path.basename(os.environ.get("HYBRIDFLUX_LIB", "libhybridflux.so")),
                      "ms_per_50_forwards": out}))


if __name__ == "__main__":
    main()
