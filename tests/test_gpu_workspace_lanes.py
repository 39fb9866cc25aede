"""The generic sequencing's scratch and lane streams (include/hybridflux.h:
hf_workspace_need, hf_run lanes).

* hf_workspace_need is exact per path: the fused and one-launch paths need
  nothing, and every call accepts a workspace of exactly the reported size and
  rejects one byte less.
* hf_run's lane streams belong to the caller's stream: two rollouts on two
  streams give the one-stream result, and an eager rollout on another stream
  while the first stream is being captured into a HIP graph neither joins nor
  breaks the capture.
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def hf():
    import hybridflux
    return hybridflux


def _setup(hf, nx, B, prec="f32"):
    from hybridflux import engine
    w = dict(golden("weights_W1_r2.npz"))
    dt = 5e-3 * 64.0 / nx
    m = engine.DeviceModel(w, DEV, prec)
    grid = engine.Grid(nx, dt=dt)
    ics = hf.BaselineSolver(nx, dt=dt, device=DEV).initial_conditions(range(1000, 1000 + B), as_tensor=True)
    return engine, m, grid, ics


@pytest.mark.parametrize("nx", [64, 100, 256])
def test_workspace_need_exact(hf, nx):
    from hybridflux._lib import HF_EINVAL, HF_OP_COMPARE, HF_OP_RUN, HF_OP_STEP, HF_WS_FLUX_FACE, HF_WS_TRAJ, lib, ptr
    engine, m, grid, ics = _setup(hf, nx, 5)
    B, T = 5, 3
    L = lib()
    need = {("run", tr): L.hf_workspace_need(m.handle, HF_OP_RUN, B, nx, T, HF_WS_TRAJ if tr else 0)
            for tr in (False, True)}
    need["step"] = L.hf_workspace_need(m.handle, HF_OP_STEP, B, nx, 1, 0)
    need["step_ff"] = L.hf_workspace_need(m.handle, HF_OP_STEP, B, nx, 1, HF_WS_FLUX_FACE)
    need["cmp"] = L.hf_workspace_need(m.handle, HF_OP_COMPARE, B, nx, T, 0)
    up = lambda v: (v + 255) // 256 * 256  # noqa: E731
    S, F, TR = up(12 * B * nx), up(4 * B * nx), up(12 * B * (T + 1) * nx)
    if nx == 64:
        assert all(v == 0 for v in need.values()), need
    else:
        assert need[("run", False)] == 2 * S + F and need[("run", True)] == F
        assert need["step"] == F and need["step_ff"] == 0
        assert need["cmp"] == (TR + F if nx == 256 else 2 * TR + S + F)
    for v in need.values():
        assert v <= max(L.hf_run_workspace_bytes(op, B, nx, T) for op in (0, 1, 2))
    ref = engine.run(m, grid, ics, T, traj=False)["final"]
    refc = engine.run_compare(m, grid, ics, T)["mse"]
    x, pc = grid.on(DEV)
    st = engine.stream_of(DEV)
    for tr in (False, True):
        n = need[("run", tr)]
        ws = torch.empty(max(n, 1), dtype=torch.uint8, device=DEV)
        traj = torch.empty(B, T + 1, 3, nx, device=DEV) if tr else None
        for size in (n, n - 1) if n else (0,):
            out = torch.empty_like(ics)
            rc = L.hf_run(m.handle, ptr(ics), ptr(out), ptr(x), ptr(pc), B, nx, T, grid.c32, grid.dt32, grid.nu32,
                          grid.dx2_32, ptr(traj), None, None, ptr(ws), size, st)
            if size == n:
                assert rc == 0 and torch.equal(out, ref), L.hf_last_error()
            else:
                assert rc == HF_EINVAL and b"hf_workspace_need" in L.hf_last_error()
    n = need["cmp"]
    ws = torch.empty(max(n, 1), dtype=torch.uint8, device=DEV)
    for size in (n, n - 1) if n else (0,):
        mse = torch.empty(B, T + 1, 3, device=DEV)
        out = torch.empty_like(ics)
        rc = L.hf_run_compare(m.handle, ptr(ics), ptr(out), ptr(x), ptr(pc), B, nx, T, grid.c32, grid.dt32,
                              grid.nu32, grid.dx2_32, ptr(mse), None, None, ptr(ws), size, st)
        if size == n:
            assert rc == 0 and torch.equal(mse, refc), L.hf_last_error()
        else:
            assert rc == HF_EINVAL and b"hf_workspace_need" in L.hf_last_error()
    torch.cuda.synchronize(DEV)


@pytest.mark.timeout(300)
def test_lanes_per_caller_stream(hf):
    """3-lane rollouts (B*nx >= 3*2^20 cells) on two caller streams at once,
    and an eager one on stream b while stream a is being captured."""
    B, nx, T = 3075, 1024, 2
    engine, m, grid, ics = _setup(hf, nx, B, "bf16")
    ref = engine.run(m, grid, ics, T, traj=False)["final"].clone()
    sa, sb = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    outa, outb = torch.empty_like(ics), torch.empty_like(ics)
    wsa, _ = engine.workspace(1, B, nx, T, DEV, model=m)
    wsb, _ = engine.workspace(1, B, nx, T, DEV, model=m)
    for s in (sa, sb):
        s.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(sa):
        engine.run(m, grid, ics, T, traj=False, out=outa, ws=wsa)
    with torch.cuda.stream(sb):
        engine.run(m, grid, ics, T, traj=False, out=outb, ws=wsb)
    torch.cuda.synchronize(DEV)
    assert torch.equal(outa, ref) and torch.equal(outb, ref)

    g = torch.cuda.CUDAGraph()
    outa.zero_()
    outb.zero_()
    torch.cuda.synchronize(DEV)
    with torch.cuda.graph(g, stream=sa):
        engine.run(m, grid, ics, T, traj=False, out=outa, ws=wsa)
        with torch.cuda.stream(sb):  # eager, on a stream that is not being captured
            engine.run(m, grid, ics, T, traj=False, out=outb, ws=wsb)
    sb.synchronize()
    assert torch.equal(outb, ref)
    assert not torch.equal(outa, ref)   # captured, not yet run
    g.replay()
    torch.cuda.synchronize(DEV)
    assert torch.equal(outa, ref)
