"""FluxGNN(4,128,4) on B chains of 64 cells: the inference flux kernel
(no_grad, chain_flux_kernel) against the fused training forward
(chain_train_fwd_kernel: the same pass plus the activation tape), HIP events
over back-to-back launches.  Diagnostic: is the training forward's gap to
the inference rate the tape or the short kernel?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us per call


def main():
    import hybridflux as hf
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = hf.FluxGNN(4, 128, 4).to(dev)
    flop_cell = 329_216
    for B in (2000, 4096, 8192):
        nx = 64
        st = torch.randn(B, 3, nx, device=dev)
        x = torch.linspace(0, 2 * np.pi, nx + 1, device=dev)[:-1]
        nf, ei = hf.build_chain_graph_batch(st, x)
        with torch.no_grad():
            t_inf = timed(lambda: m(nf, ei))
        t_tr = timed(lambda: m(nf, ei))  # grad enabled: the training forward (tape kept by autograd)
        tf = lambda t: flop_cell * B * nx / (t * 1e-6) / 1e12  # noqa: E731
        print(f"B={B}: inference {t_inf:8.1f} us ({tf(t_inf):6.1f} TF/s), training forward {t_tr:8.1f} us "
              f"({tf(t_tr):6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
