"""Regression guard on the compiled device code (no GPU needed): the load
pipelines round 4 built by hand must survive the compiler.  tools/asm_wait_scan.py
compiles the sources for gfx950 (-S, the library's flags) and counts, per
kernel, the global loads waited with vmcnt(0) within three instructions of
their issue and the scratch (spill) operations.

- pinn_run_kernel: the weight stream is a software pipeline (baselines.hip
  pinn_layer); left to itself the compiler waited for every k-block load
  where it was issued (one L2 round trip per k-block, 129 M -> 190 M
  IC-steps/s when pinned).  Only the prologue's state / bias copies may wait.
- the training GEMM with the stencil operand (tgemm.h VStencil load2 /
  combine): the one-call form waited for both neighbour loads at the start of
  every stage (23 of 52 loads).
- chain_flux_sw_kernel (cfg4): no spill (the layer loop's trip counter was
  spilled and reloaded with a scratch load whose vmcnt(0) also waited out the
  ring's DMA every layer).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not installed")


def _scan(name, tmp_path):
    import asm_wait_scan
    return asm_wait_scan.scan(os.path.join(asm_wait_scan.CSRC, name), str(tmp_path))


def _kernel(stats, *parts):
    hits = [v for k, v in stats.items() if all(p in k for p in parts)]
    assert hits, parts
    return hits


def test_pinn_weight_stream_stays_pipelined(tmp_path):
    st = _scan("baselines.hip", tmp_path)
    for v in _kernel(st, "pinn_run_kernel"):
        assert v["mfma"] > 0 and v["scratch"] == 0
        assert v["waited_at_issue"] <= 3, v          # prologue copies only (was one per k-block)
    for v in _kernel(st, "pure_run_kernelILi128ELi4ELb1"):
        assert v["scratch"] == 0 and v["waited_at_issue"] <= 6, v


def test_training_stencil_loads_two_phase(tmp_path):
    st = _scan("train_chain.hip", tmp_path)
    for v in _kernel(st, "tgemm_kernel", "VStencil", "EpiAct"):
        assert v["scratch"] == 0 and v["waited_at_issue"] <= 2, v   # was 23 of 52


def test_bf16_super_window_kernel_does_not_spill(tmp_path):
    st = _scan("chain_bf16.hip", tmp_path)
    for v in _kernel(st, "chain_flux_sw_kernel"):
        assert v["scratch"] == 0, v
