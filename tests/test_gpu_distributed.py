"""cfg5's data path with more than one rank, on the HIP kernels (BASELINE.json
configs[4]; reference workload scripts/evaluation/evaluate_multi_ic.py:106-138).

Two rank processes share the box's one GPU over gloo (RCCL needs a GPU per
rank; the 8-GPU RCCL run is the driver's).  Each runs its IC shard through
HybridSolver and the end-of-rollout exchange bench.py uses (gather_rollout:
device summary kernel + all_gather).  The gathered metric series, summaries,
final states and the compare path's MSE must equal a one-rank run of the same
seeds bit for bit: IC sharding changes no arithmetic.  Then bench.py itself,
launched plainly with --gpus 2, must start its two ranks and report them.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_rollout_worker.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**extra):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(extra)
    return env


def _run(cmd, timeout, **extra):
    p = subprocess.run(cmd, env=_env(**extra), capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, f"{cmd}\nrc={p.returncode}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return p


@pytest.mark.timeout(400)
def test_two_ranks_equal_one_rank_bitwise(tmp_path):
    one, two = tmp_path / "one.npz", tmp_path / "two.npz"
    _run([sys.executable, WORKER, str(one)], 200)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
          "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, str(two)], 300)
    a, b = np.load(one), np.load(two)
    assert int(a["world"]) == 1 and int(b["world"]) == 2
    assert int(a["grouped"]) == 0 and int(a["collective_calls"]) == 0 and str(b["backend"]) == "gloo"
    assert float(b["max_over_ranks"]) == 2.0
    for label in ("fused64_f32", "generic256_bf16", "one_ic"):
        for key in ("metrics", "summary", "final", "cmp_mse", "cmp_summary"):
            x, y = a[f"{label}/{key}"], b[f"{label}/{key}"]
            assert x.shape == y.shape, (label, key, x.shape, y.shape)
            assert np.isfinite(x).all() or key.endswith("summary")
            # bitwise (NaN-safe): the same ICs, the same kernels, gathered in global IC order
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (label, key)
    # the ragged shards: rank 0 holds ceil(n/2) ICs
    assert int(b["fused64_f32/local_n"]) == 19 and int(b["generic256_bf16/local_n"]) == 5
    assert int(b["one_ic/local_n"]) == 1 and a["one_ic/metrics"].shape[0] == 1  # rank 1 held 0 ICs


@pytest.mark.timeout(400)
def test_bench_self_launches_ranks():
    """`python bench.py --gpus 4` without a launcher starts 4 ranks itself (gloo,
    sharing this box's one GPU); rank 0's line checks itself: world_size 4, ONE
    packed exchange moving 4 x the per-rank payload, and every rank's wall
    time and IC count."""
    p = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dist-backend", "gloo",
              "--steps", "4", "--warmup", "2", "--ics-per-gpu", "1024", "--no-cpu-baseline", "--no-other-configs",
              "--also", ""], 300)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["config"]["global_ics"] == 4096 and d["config"]["ics_per_gpu"] == 1024
    assert d["finite_fraction"] == 1.0 and d["value"] > 0
    c = d["config"]["collective"]
    assert c["backend"] == "gloo" and c["world_size"] == 4 and c["calls"] == 1  # metrics + summaries packed
    assert c["bytes_received_per_rank"] == 4 * c["bytes_sent_per_rank"] == 4 * 1024 * (5 * 4 + 8) * 4
    r = d["config"]["ranks"]
    assert r["ics_per_rank"] == [1024] * 4 and len(r["wall_s_per_rank"]) == 4
    assert r["wall_s_min"] <= r["wall_s_max"] and abs(d["ms_per_step"] - r["wall_s_max"] / 4 * 1e3) < 1e-3
    assert abs(d["value"] - 4096 * 4 / r["wall_s_max"]) <= 1e-6 * d["value"] + 0.1


N_CASES = 3  # dist_rollout_worker.CASES


@pytest.mark.timeout(400)
def test_rccl_one_rank_equals_no_group_bitwise(tmp_path):
    """RCCL on this engine's data path: a one-rank nccl
    group (the box has one GPU; RCCL needs one per rank) runs the same
    end-of-rollout exchange as the 8-GPU job — device all_gather_into_tensor of
    the metric series, summaries, MSE series and final states, and the device
    all_reduce MAX of max_over_ranks — and must give exactly the no-group run's
    tensors (reference workload scripts/evaluation/evaluate_multi_ic.py:106-138)."""
    one, rccl = tmp_path / "one.npz", tmp_path / "rccl.npz"
    _run([sys.executable, WORKER, str(one)], 200)
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
          "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, str(rccl)], 300,
         HF_DIST_BACKEND="nccl")
    a, b = np.load(one), np.load(rccl)
    assert int(b["grouped"]) == 1 and int(b["world"]) == 1 and str(b["backend"]) == "nccl"
    assert float(b["max_over_ranks"]) == 1.0
    # per case: gather_rollout of the run and of the compare (one packed call each) and the final states
    assert int(b["collective_calls"]) == N_CASES * 3 + 1
    assert int(b["collective_bytes_received"]) > 0
    for label in ("fused64_f32", "generic256_bf16", "one_ic"):
        for key in ("metrics", "summary", "final", "cmp_mse", "cmp_summary"):
            x, y = a[f"{label}/{key}"], b[f"{label}/{key}"]
            assert x.shape == y.shape, (label, key, x.shape, y.shape)
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (label, key)


@pytest.mark.timeout(400)
def test_bench_one_gpu_runs_rccl_exchange():
    """A plain `python bench.py` (N = 1, default backend nccl) creates a
    one-rank RCCL group and reports the all_gather it actually ran inside the
    timed region, and the timed rollout's parity against the reference."""
    p = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
              "--no-cpu-baseline", "--no-other-configs", "--also", ""], 300)
    # stdout is exactly the one JSON line (RCCL's version banner goes to stderr)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]
    d = json.loads(lines[0])
    c = d["config"]["collective"]
    assert d["n_gpus"] == 1 and c["backend"] == "nccl (RCCL)" and c["world_size"] == 1
    assert c["calls"] == 1 and c["bytes_received_per_rank"] == 4096 * (5 * 4 + 8) * 4
    assert c["exchange_ms"] > 0
    assert d["parity"]["within_gate"] and d["parity"]["steps_checked"] == 4


@pytest.mark.timeout(600)
def test_cfg5_full_size_eight_ranks_equal_one_rank_bitwise(tmp_path):
    """BASELINE.json configs[4] at its full size: 32,768 ICs of 64 cells (r = 2
    weights, f32) sharded over 8 rank processes — 4,096 ICs each, as on the
    8-GPU node — sharing this box's one GPU over gloo (RCCL needs one GPU per
    rank; the RCCL exchange itself is test_rccl_one_rank_equals_no_group_bitwise).
    The gathered metric series, summaries, final states and the compare path's
    MSE equal one process running all 32,768 ICs bit for bit."""
    one, eight = tmp_path / "one.npz", tmp_path / "eight.npz"
    _run([sys.executable, WORKER, str(one)], 300, HF_DIST_CASES="cfg5")
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
          "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, str(eight)], 500,
         HF_DIST_CASES="cfg5")
    a, b = np.load(one), np.load(eight)
    assert int(a["world"]) == 1 and int(b["world"]) == 8 and str(b["backend"]) == "gloo"
    assert int(b["cfg5_32768_f32/local_n"]) == 4096
    for key in ("metrics", "summary", "final", "cmp_mse", "cmp_summary"):
        x, y = a[f"cfg5_32768_f32/{key}"], b[f"cfg5_32768_f32/{key}"]
        assert x.shape == y.shape and x.shape[0] == 32768, (key, x.shape, y.shape)
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), key
    assert np.isfinite(a["cfg5_32768_f32/final"]).all()


@pytest.mark.timeout(300)
def test_rank_exiting_early_fails_the_job_within_timeout(record):
    """8-GPU readiness: a 2-rank torchrun-style bench.py
    job (gloo on this box's one GPU) in which rank 1 vanishes before the group
    forms (HF_BENCH_EXIT_RANK=1, exit code 0, so the launcher keeps waiting on
    rank 0) must end non-zero within the group timeout (HF_DIST_TIMEOUT_S)
    instead of hanging for the 10-minute default."""
    import time
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--ics-per-gpu", "64",
           "--no-cpu-baseline", "--no-other-configs", "--also", ""]
    t0 = time.perf_counter()
    p = subprocess.run(cmd, env=_env(HF_BENCH_EXIT_RANK="1", HF_DIST_TIMEOUT_S="20"), capture_output=True,
                       text=True, timeout=240, cwd=ROOT)
    secs = time.perf_counter() - t0
    record("rank_exit_early", "job_seconds", secs)
    assert p.returncode != 0, p.stdout[-2000:]
    assert secs < 200, secs
    assert "exiting early" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]  # no bench line from a broken job
