"""IC-sharded multi-process rollout (hybridflux/rollout.py) on CPU with gloo,
world_size 2 and 4.  The device compute is replaced by the CPU oracle here (the
collective and sharding logic are what is under test); on GPUs the same
driver runs with backend "nccl" (RCCL) and the HIP kernels (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hybridflux.rollout import gather_ic_rows, shard_bounds, shard_seeds

T = 3
N_TOTAL = 5  # ragged over 2 ranks: 3 + 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,w", [(0, 1), (5, 2), (4096, 8), (32768, 8), (7, 3), (2, 4)])
def test_shard_bounds_partition(n, w):
    spans = [shard_bounds(n, w, r) for r in range(w)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1
    seeds = sum((shard_seeds(1000, n, w, r) for r in range(w)), [])
    assert seeds == list(range(1000, 1000 + n))


def _oracle_local(seeds):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import hybrid_oracle as O
    G = O.Grid(64)
    if not len(seeds):  # an empty shard (more ranks than ICs)
        return torch.zeros(0, T + 1, 4), np.zeros((0, T + 1, 3, 64), np.float32)
    w = dict(np.load(os.path.join(root, "tests", "golden", "weights_W1_r1.npz")))
    ics = np.stack([O.initial_condition(G, s) for s in seeds])
    S, _ = O.hybrid_run(O.params_from(w), G, ics, T)
    e, q, f = O.rollout_metrics(S)
    m = np.stack([e, q, f.astype(np.float64), np.zeros_like(e)], axis=-1).astype(np.float32)
    return torch.from_numpy(m), S


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hybridflux.rollout import sharded_rollout

    def make_ics(seeds):
        return seeds

    def run_local(seeds, T_):
        m, S = _oracle_local(seeds)
        return {"metrics": m, "final": torch.from_numpy(S[:, -1])}

    res, gathered = sharded_rollout(run_local, make_ics, 1000, N_TOTAL, T, summarize=False)
    # the other per-IC rows bench.py gathers: an [b, 8] summary and an [b, T+1, 3] series
    lo, hi = shard_bounds(N_TOTAL, world, rank)
    summ = torch.arange(lo * 8, hi * 8, dtype=torch.float32).reshape(-1, 8)
    ser = torch.arange(lo * (T + 1) * 3, hi * (T + 1) * 3, dtype=torch.float32).reshape(-1, T + 1, 3)
    g_summ, g_ser = gather_ic_rows(summ, N_TOTAL), gather_ic_rows(ser, N_TOTAL)
    from hybridflux.rollout import COLLECTIVES, max_over_ranks
    mx = max_over_ranks(0.25 * (rank + 1))               # bench.py's max-over-ranks timing
    torch.save({"gathered": gathered, "max": mx, "local_n": res["metrics"].shape[0], "summ": g_summ,
                "series": g_ser, "calls": COLLECTIVES["calls"], "backend": COLLECTIVES["backend"],
                "received": COLLECTIVES["bytes_received"]}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_gloo_sharded_rollout(tmp_path, world):
    """world 1: a one-rank group still runs every collective (as bench.py's
    one-rank RCCL group does); world 2: shards 3 + 2; world 4 (a rehearsal of
    more ranks than the GPU test's 2): 2 + 1 + 1 + 1; world 8: 1 x 5 then three
    EMPTY shards (more ranks than ICs), which still take part in the gather."""
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    want, _ = _oracle_local(list(range(1000, 1000 + N_TOTAL)))
    for r in range(world):
        d = torch.load(tmp_path / f"rank{r}.pt", weights_only=True)
        assert d["max"] == 0.25 * world
        lo, hi = shard_bounds(N_TOTAL, world, r)
        assert d["local_n"] == hi - lo
        assert d["gathered"].shape == (N_TOTAL, T + 1, 4)
        assert torch.equal(d["gathered"], want)   # same ICs, same order as one process
        assert torch.equal(d["summ"], torch.arange(N_TOTAL * 8, dtype=torch.float32).reshape(N_TOTAL, 8))
        assert torch.equal(d["series"], torch.arange(N_TOTAL * (T + 1) * 3, dtype=torch.float32)
                           .reshape(N_TOTAL, T + 1, 3))
        # 3 all_gathers + 1 all_reduce, each counted with what it moved
        cap = -(-N_TOTAL // world)
        assert d["calls"] == 4 and d["backend"] == "gloo"
        assert d["received"] == world * cap * ((T + 1) * 4 + 8 + (T + 1) * 3) * 4 + 8


def test_gather_single_process_passthrough():
    x = torch.arange(12.0).reshape(3, 4)
    assert gather_ic_rows(x, 3) is x


def _packed_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hybridflux.rollout import COLLECTIVES, gather_ic_rows_packed
    n = 5
    lo, hi = shard_bounds(n, world, rank)
    a = torch.arange(lo * 12, hi * 12, dtype=torch.float32).reshape(-1, 3, 4)
    b = torch.arange(lo * 8, hi * 8, dtype=torch.float32).reshape(-1, 8) + 1000
    ga, gb = gather_ic_rows_packed([a, b], n)
    assert torch.equal(ga, torch.arange(60.0).reshape(5, 3, 4))
    assert torch.equal(gb, torch.arange(40.0).reshape(5, 8) + 1000)
    assert COLLECTIVES["calls"] == 1
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 8])
def test_packed_gather_one_collective(world):
    """gather_rollout's packed exchange: a [b, 3, 4] series and [b, 8] summaries
    gathered in ONE collective, split back in global IC order (world 8: three
    empty shards)."""
    mp.spawn(_packed_worker, args=(world, _free_port()), nprocs=world, join=True)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_sets_ipc_mode_torchrun_style():
    """A bench.py process started by a launcher (WORLD_SIZE already set, as
    torchrun / the driver's 8-GPU run do) has HSA_ENABLE_IPC_MODE_LEGACY=0 in
    its environment before anything can touch the GPU (RCCL needs dmabuf IPC on
    this host driver), not only when bench.py launches its own ranks."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    env.update(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    code = ("import os, sys; sys.argv = ['bench.py']; import bench; "
            "print('IPC=' + str(os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY')))")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "IPC=0" in p.stdout.splitlines()


def test_bench_group_setup_times_out_without_peer():
    """Rank 0 of 2 whose peer never starts: bench.init_group must give up
    within HF_DIST_TIMEOUT_S instead of the 10-minute default (run in its own
    interpreter, as a rank is)."""
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="2",
               HF_DIST_TIMEOUT_S="5")
    code = ("import sys, time, torch; sys.argv = ['bench.py']; import bench; t0 = time.perf_counter()\n"
            "try:\n    bench.init_group('gloo', 2, torch.device('cpu')); print('RESULT joined')\n"
            "except Exception as e:\n    print('RESULT', type(e).__name__, round(time.perf_counter() - t0, 1))\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    res = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT")]
    assert res and "joined" not in res[0], (p.stdout[-1000:], p.stderr[-2000:])
    assert float(res[0].split()[-1]) < 60, res


BENCH_RANK_SCRIPT = r"""
import json, os, sys, time
sys.path.insert(0, {root!r}); sys.argv = ["bench.py"]
import torch, torch.distributed as dist
import bench
from hybridflux.rollout import COLLECTIVES, gather_ic_rows_packed, reset_collective_stats, shard_bounds
world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
bench.init_group("gloo", world, torch.device("cpu"))
n_total, T = {n_total}, {T}
lo, hi = shard_bounds(n_total, world, rank)
# the shapes bench.py gathers: metric series [b, T+1, 4] and summaries [b, 8]
met = torch.arange(lo * (T + 1) * 4, hi * (T + 1) * 4, dtype=torch.float32).reshape(-1, T + 1, 4)
summ = torch.arange(lo * 8, hi * 8, dtype=torch.float32).reshape(-1, 8)
reset_collective_stats()
g_met, g_summ = gather_ic_rows_packed([met, summ], n_total)
coll = dict(COLLECTIVES)
ranks = bench.rank_report(0.5 + 0.25 * rank, hi - lo)
assert torch.equal(g_met, torch.arange(n_total * (T + 1) * 4, dtype=torch.float32).reshape(n_total, T + 1, 4))
if rank == 0:
    print(json.dumps({{"collective": bench.collective_entry(coll, world, 0.0), "ranks": ranks}}), flush=True)
dist.destroy_process_group()
"""


def test_bench_four_rank_gloo_line_checks_itself(tmp_path):
    """4 gloo ranks started torchrun-style (as the driver
    starts bench.py) run bench.py's own end-of-rollout exchange and reporting
    (gather_ic_rows_packed, bench.rank_report, bench.collective_entry) on the
    shapes of a 4 x 1024-IC job: rank 0's record says world_size 4, ONE call,
    4 x the per-rank payload received, and every rank's wall and IC count.
    (The GPU twin, tests/test_gpu_distributed.py::test_bench_self_launches_ranks,
    runs the whole bench.py with 4 ranks on one GPU.)"""
    import json
    import subprocess
    import sys
    n_total, T = 4096, 4
    script = tmp_path / "rank.py"
    script.write_text(BENCH_RANK_SCRIPT.format(root=ROOT, n_total=n_total, T=T))
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "gnn-plasma-flux_amd") + os.pathsep + ROOT)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    c = d["collective"]
    payload = (n_total // 4) * ((T + 1) * 4 + 8) * 4
    assert c["backend"] == "gloo" and c["world_size"] == 4 and c["calls"] == 1
    assert c["bytes_sent_per_rank"] == payload and c["bytes_received_per_rank"] == 4 * payload
    r = d["ranks"]
    assert r["ics_per_rank"] == [1024] * 4
    assert r["wall_s_per_rank"] == [0.5, 0.75, 1.0, 1.25] and r["wall_s_max"] == 1.25 and r["wall_s_min"] == 0.5
