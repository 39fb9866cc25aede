"""Multi-GPU batched rollout: independent initial conditions sharded across
ranks (one process per GPU), zero communication while stepping, and ONE
collective at the end — an all_gather of the per-IC rollout metrics over
RCCL/xGMI (backend "nccl" on ROCm), or gloo on CPU for tests.

This is the reference's multi-IC evaluation loop
(scripts/evaluation/evaluate_multi_ic.py:106-138: seeds 1000.., one IC at a
time) turned into a data-parallel job: IC j of rank r is seed
`seed0 + start(r) + j`, so the union over ranks is the same seed range at any
world size.  A 64-cell chain never shards spatially (BASELINE.json north star).

Whenever a process group is initialised the exchange is a real collective,
world size 1 included (a one-rank RCCL group still runs the all_gather kernel
on the device); without a group the local tensors are returned as they are.
Every collective issued here is counted in `COLLECTIVES` (backend, calls, bytes
each rank received), so a benchmark line reports the transfer that happened,
not one computed from tensor shapes.
"""
import math

import torch
import torch.distributed as dist

# running tally of the collectives this module issued (reset_collective_stats)
COLLECTIVES = {"backend": None, "calls": 0, "bytes_received": 0, "bytes_sent": 0}


def reset_collective_stats():
    COLLECTIVES.update(backend=None, calls=0, bytes_received=0, bytes_sent=0)


def _count(backend, sent, received):
    COLLECTIVES["backend"] = backend
    COLLECTIVES["calls"] += 1
    COLLECTIVES["bytes_sent"] += int(sent)
    COLLECTIVES["bytes_received"] += int(received)


def shard_bounds(n_total, world, rank):
    """Contiguous [start, stop) of IC indices owned by `rank`; ragged totals
    give the first n_total % world ranks one extra IC."""
    base, rem = divmod(int(n_total), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_seeds(seed0, n_total, world, rank):
    a, b = shard_bounds(n_total, world, rank)
    return list(range(seed0 + a, seed0 + b))


def gather_ic_rows(local, n_total, group=None):
    """all_gather a per-IC tensor [b_local, ...] into [n_total, ...] on every
    rank, in global IC order (ragged shards are padded to the largest shard for
    the collective).  RCCL gathers device tensors in place into one contiguous
    [world*cap, ...] buffer (all_gather_into_tensor); gloo moves host memory, so
    device tensors are staged through the host for it.  No process group: the
    local tensor itself."""
    if not dist.is_initialized():
        return local
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [shard_bounds(n_total, world, r)[1] - shard_bounds(n_total, world, r)[0] for r in range(world)]
    assert local.shape[0] == counts[rank], (local.shape, counts)
    cap = max(counts)
    if cap == 0:
        return local
    backend = dist.get_backend(group)
    stage = local.is_cuda and backend == "gloo"
    src = local.cpu() if stage else local
    if src.shape[0] == cap:
        pad = src.contiguous()
    else:
        pad = src.new_zeros((cap,) + tuple(src.shape[1:]))
        pad[: src.shape[0]] = src
    row_bytes = pad.numel() * pad.element_size()
    if backend == "gloo":
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        out = torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)
    else:
        flat = pad.new_empty((world * cap,) + tuple(pad.shape[1:]))
        dist.all_gather_into_tensor(flat, pad, group=group)
        if all(c == cap for c in counts):
            out = flat
        else:
            out = torch.cat([flat[r * cap: r * cap + c] for r, c in enumerate(counts)], dim=0)
    _count(backend, row_bytes, row_bytes * world)
    return out.to(local.device) if stage else out


def gather_ic_rows_packed(tensors, n_total, group=None):
    """gather_ic_rows of several per-IC tensors [b_local, ...] (same leading
    size, dtype and device) in ONE collective: their rows are packed side by
    side into one [b_local, sum of row sizes] buffer, gathered, and split back
    into [n_total, ...] tensors.  One RCCL call instead of one per tensor (each
    call pays the collective's latency across the ranks)."""
    tensors = list(tensors)
    t0 = tensors[0]
    for t in tensors[1:]:  # torch.cat would silently promote a mixed dtype for every part
        if t.dtype != t0.dtype or t.device != t0.device or t.shape[0] != t0.shape[0]:
            raise ValueError(f"gather_ic_rows_packed: tensors must share dtype, device and leading size; got "
                             f"{t0.dtype}/{t0.device}/{t0.shape[0]} and {t.dtype}/{t.device}/{t.shape[0]}")
    if not dist.is_initialized():
        return tensors
    b = t0.shape[0]
    widths = [int(math.prod(t.shape[1:])) for t in tensors]
    packed = torch.cat([t.reshape(b, w) for t, w in zip(tensors, widths)], dim=1)
    flat = gather_ic_rows(packed, n_total, group)
    out, o = [], 0
    for t, w in zip(tensors, widths):
        out.append(flat[:, o:o + w].reshape((flat.shape[0],) + tuple(t.shape[1:])))
        o += w
    return out


def max_over_ranks(value, group=None, device=None):
    """The job's wall time: the MAX of each rank's value (bench.py's timing rule:
    the slowest shard ends the job).  A float64 all_reduce whenever a group is
    initialised (world 1 included), on the rank's current HIP device for RCCL
    and on the CPU for gloo unless `device` says otherwise; the value itself
    when not distributed."""
    if not dist.is_initialized():
        return float(value)
    backend = dist.get_backend(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if backend != "gloo" else "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    _count(backend, 8, 8)
    return float(t.item())


def gather_rollout(res, n_total, group=None):
    """The end-of-rollout exchange of an IC-sharded job: this rank's per-step
    metric series res['metrics'] [b, T+1, K] (and the MSE series res['mse']
    [b, T+1, 3] when the rollout was scored against the classical twin) are
    summarised on the device (hf_rollout_summary: first non-finite step, drifts,
    MSE totals), then series and summaries are all_gathered in global IC order,
    packed into ONE collective.
    Returns dict(metrics [n_total, T+1, K], summary [n_total, 8], mse or None)."""
    from . import engine
    summ, _ = engine.rollout_summary(res["metrics"], res.get("mse"), res.get("metrics_classical"))
    parts = [res["metrics"], summ] + ([res["mse"]] if res.get("mse") is not None else [])
    got = gather_ic_rows_packed(parts, n_total, group)  # one collective for all of them
    return {"metrics": got[0], "summary": got[1], "mse": got[2] if len(got) > 2 else None}


def sharded_rollout(run_local, make_ics, seed0, n_total, T, group=None, summarize=True):
    """Run this rank's shard and gather every IC's metrics.

    run_local(ics, T) -> dict with 'metrics' [b, T+1, K] (device tensor) and 'final'.
    make_ics(seeds) -> [b, 3, nx] states for those seeds.
    Returns (local_result, gathered): gathered is gather_rollout's dict when
    summarize (a HIP device is needed for the summary kernel), else the
    gathered metrics [n_total, T+1, K] alone.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    ics = make_ics(shard_seeds(seed0, n_total, world, rank))
    res = run_local(ics, T)
    if summarize:
        return res, gather_rollout(res, n_total, group)
    return res, gather_ic_rows(res["metrics"], n_total, group)
