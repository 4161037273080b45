"""Replicate sharding across ranks (one process per GPU) with one all-gather of the
per-replicate rows -- the only collective the bootstrap needs.

The reference runs every replicate in one process on a Rayon pool (builder.rs:816-839).
Here rank r computes replicate ids [r*per, (r+1)*per) of the OBRS-3 stream (results are a pure
function of (seed, replicate id), so the gathered rows equal a single-GPU run bit for bit), the
rows are all-gathered, and rank 0 aggregates (builder.rs:841-950). Two gathers exist:

* ``engine=True`` (the drop-in's own path): the engine's RCCL communicator
  (``ob_ctx_create_rank`` + ``ob_prepared_boot_sharded``), exactly what a Rust caller binds;
  torch.distributed only carries the 128-byte unique id from rank 0.
* ``engine=False``: torch.distributed's all_gather_into_tensor -- on-device over RCCL for an
  nccl group, through host tensors for gloo (the CPU tests).

Launch with torch.distributed.run; MASTER_ADDR=127.0.0.1.
"""
from __future__ import annotations

import numpy as np


def shard(n_reps: int, rank: int, world: int):
    """Replicate range of ``rank``: equal-sized shards (the last one padded)."""
    per = -(-n_reps // world) if world else n_reps
    first = min(rank * per, n_reps)
    return first, max(0, min(n_reps, first + per) - first), per


def gather_rows(prepared, n_reps: int, group=None, device=None):
    """Compute this rank's replicates and all-gather every rank's rows.

    ``prepared`` is anything with ``row_len``, ``boot(first, n) -> (rows, ok)`` and, for the
    device path, ``boot_device(first, n, rows_ptr, ok_ptr, stream)`` + ``sync()`` + ``device``
    (``api.PreparedRun`` provides all of them). Under an nccl group the rows stay on the GPU
    (``device`` defaults to the panel's GPU and must equal it). Returns (rows, ok) for all
    ``n_reps`` replicates in replicate order on every rank.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    first, count, per = shard(n_reps, rank, world)
    rl = prepared.row_len
    on_gpu = dist.is_initialized() and dist.get_backend(group) == "nccl"
    if on_gpu:
        panel_dev = getattr(prepared, "device", None)
        if device is None:
            device = panel_dev if panel_dev is not None else torch.cuda.current_device()
        device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if panel_dev is not None and device.index != panel_dev:
            raise ValueError(f"gather device {device} differs from the panel's GPU {panel_dev}")
        rows = torch.empty((per, rl), dtype=torch.float64, device=device)
        ok = torch.zeros(per, dtype=torch.uint8, device=device)
        if count:
            stream = torch.cuda.current_stream(device).cuda_stream
            prepared.boot_device(first, count, rows.data_ptr(), ok.data_ptr(), stream)
        if count < per:
            rows[count:].fill_(float("nan"))
    else:
        r, o = prepared.boot(first, count) if count else (np.zeros((0, rl)), np.zeros(0, np.uint8))
        rows = torch.full((per, rl), float("nan"), dtype=torch.float64)
        ok = torch.zeros(per, dtype=torch.uint8)
        rows[:count] = torch.from_numpy(np.ascontiguousarray(r))
        ok[:count] = torch.from_numpy(np.ascontiguousarray(o))
    if world > 1:
        all_rows = torch.empty((world * per, rl), dtype=rows.dtype, device=rows.device)
        all_ok = torch.empty(world * per, dtype=ok.dtype, device=ok.device)
        dist.all_gather_into_tensor(all_rows, rows, group=group)
        dist.all_gather_into_tensor(all_ok, ok, group=group)
    else:
        all_rows, all_ok = rows, ok
    if on_gpu and count:
        prepared.sync()
    return all_rows[:n_reps].cpu().numpy(), all_ok[:n_reps].cpu().numpy()


_engine_ctx: dict = {}


def engine_context(device: int, group=None):
    """This rank's engine context on an RCCL communicator spanning the group's ranks: rank 0's
    ncclUniqueId travels by broadcast_object_list; the engine owns the communicator. One context
    per (group, device, rank, world), reused by later fits: a communicator holds device buffers
    and proxy threads, so a fresh one per fit would accumulate them."""
    import torch.distributed as dist

    from . import _native as N

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    key = (id(group) if group is not None else None, int(device), rank, world)
    ctx = _engine_ctx.get(key)
    if ctx is None:
        uid = [N.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0, group=group)
        ctx = _engine_ctx[key] = N.rank_context(device, rank, world, uid[0])
    return ctx


def fit_sharded(builder, group=None, device=None, engine=False):
    """``OaxacaBuilder.run()`` over all ranks: every rank prepares the same panel (rank 0's seed
    is broadcast when the builder is unseeded), computes its shard, all ranks gather, rank 0
    returns the OaxacaResults (other ranks return None). ``engine=True`` gathers through the
    engine's own RCCL communicator (ob_prepared_boot_sharded) instead of torch.distributed."""
    import torch.distributed as dist

    from . import _native as N

    if dist.is_initialized() and builder._seed is None:
        seed = [int(np.random.SeedSequence().generate_state(1, np.uint64)[0])]
        dist.broadcast_object_list(seed, src=0, group=group)
        builder.seed(seed[0])
    if device is None:
        device = N.resolve_device(builder._device)
    builder.device(device)
    if engine:
        builder._ctx = engine_context(device, group)
    try:
        prep = builder.prepare()
    finally:
        builder._ctx = None
    try:
        if engine:
            rows, ok = prep.boot_sharded(0, builder._bootstrap_reps)
        else:
            rows, ok = gather_rows(prep, builder._bootstrap_reps, group=group, device=device)
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        return prep.finish(rows, ok) if rank == 0 else None
    finally:
        prep.close()
