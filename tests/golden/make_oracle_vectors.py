"""Fixtures computed by the CPU ORACLE (not the reference) where the reference
has no counterpart: the bf16 arithmetic of BASELINE config 4.

    python tests/golden/make_oracle_vectors.py

bf16_nx1024.npz  W1_r2, seeds 1000..1003 (the first ICs of bench.py's cfg4
                 batch), nx=1024, dt=3.125e-4, T=30 (the cfg4 horizon):
                   states_emul  [4,31,3,1024]  oracle.hybrid_flux_edge_bf16 (the
                                bf16 kernels' own arithmetic, emulated: bf16 weights
                                and GEMM inputs, hi+lo split input features, f32
                                accumulation; CoreBF16)
                   states_wbf16 [4,31,3,1024]  float32 reference forward on
                                bf16-rounded weights (oracle.bf16_weights)
                 and the first-step edge fluxes of both.
The reference's float32 rollout of the same ICs is hybrid_W1_r2_nx1024.npz.
Both oracles are pinned by tests/test_oracle_golden.py (the float32 forward
bit-exact to the reference; the emulation equals it on bf16-exact inputs).
"""
import os
import sys
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(OUT.parent.parent))
from oracle import hybrid_oracle as O  # noqa: E402


def main():
    w = dict(np.load(OUT / "weights_W1_r2.npz"))
    G = O.Grid(1024, dt=3.125e-4)
    seeds = [1000, 1001, 1002, 1003]
    ics = np.stack([O.initial_condition(G, s) for s in seeds])
    S_e, FE_e = O.hybrid_run(O.params_from(w), G, ics, 30, flux_fn=O.hybrid_flux_edge_bf16)
    S_w, FE_w = O.hybrid_run(O.params_from(O.bf16_weights(w)), G, ics, 30)
    np.savez_compressed(OUT / "bf16_nx1024.npz", seeds=np.array(seeds), states_emul=S_e, states_wbf16=S_w,
                        flux_edge0_emul=FE_e[:, 0], flux_edge0_wbf16=FE_w[:, 0])
    print("wrote bf16_nx1024.npz", S_e.shape, "max |emul - wbf16| =", float(np.abs(S_e - S_w).max()))


if __name__ == "__main__":
    main()
