"""Multi-GPU sharding of header batches.

Units are independent (a header's verdict depends only on its own bytes, eta0
and its slot), so a batch is split into static contiguous shards of
ceil(N/G) headers, one per rank/GPU, with no data-path exchange.  The single
collective is the all-gather of the per-header results (verdict byte, beta_eta,
beta_leader = 129 B/header) that the host-side sequential fold consumes
(first failure stops the fold, tpraos.first_invalid).  With the "nccl" backend
this is one RCCL all-gather over xGMI; the "gloo" backend runs the same code
on CPU tensors (tests/test_shard.py).
"""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np

RESULT_BYTES = 1 + 64 + 64


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) of rank `rank` among `world`, ceil(n/world) each."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = -(-n // world) if n else 0
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def pack_results(verdict, beta_eta, beta_leader):
    """One contiguous (n, 129) uint8 block per shard for the all-gather."""
    import torch

    n = verdict.shape[0]
    return torch.cat([verdict.reshape(n, 1), beta_eta.reshape(n, 64),
                      beta_leader.reshape(n, 64)], dim=1).contiguous()


def all_gather_results(local, n_total: int, world: int, group=None):
    """Gather every rank's (n_r, 129) block into the full (n_total, 129) result.

    Shards are padded to ceil(n/world) rows so one all_gather of equal-size
    tensors suffices (RCCL needs equal counts); padding rows are dropped."""
    import torch
    import torch.distributed as dist

    per = -(-n_total // world) if n_total else 0
    if local.shape[0] == per:
        pad = local.contiguous()
    else:
        pad = torch.zeros((per, RESULT_BYTES), dtype=torch.uint8, device=local.device)
        pad[: local.shape[0]] = local
    if local.device.type == "cuda":
        # one flat RCCL all-gather straight into the result (no list, no cat)
        full = torch.empty((world * per, RESULT_BYTES), dtype=torch.uint8, device=local.device)
        dist.all_gather_into_tensor(full, pad, group=group)
        return full[:n_total]
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat(bufs, dim=0)[:n_total]


def unpack_results(full) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    a = full.cpu().numpy() if hasattr(full, "cpu") else np.asarray(full)
    return a[:, 0].copy(), a[:, 1:65].copy(), a[:, 65:129].copy()


def verify_sharded(batch, verify: Callable = None, group=None):
    """Verify a host HeaderBatch across the ranks of `group`: each rank runs
    `verify` (default: the gfx950 kernel, tpraos.verify_headers) on its shard,
    then every rank receives all results.  Returns (verdict, beta_eta, beta_leader)."""
    import torch
    import torch.distributed as dist

    from .tpraos import verify_headers

    verify = verify or verify_headers
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = len(batch)
    lo, hi = shard_range(n, world, rank)
    v, be, bl = verify(batch.slice(lo, hi))
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    local = pack_results(torch.from_numpy(np.ascontiguousarray(v)).to(dev),
                         torch.from_numpy(np.ascontiguousarray(be)).to(dev),
                         torch.from_numpy(np.ascontiguousarray(bl)).to(dev))
    return unpack_results(all_gather_results(local, n, world, group))


def check_rank_devices(infos, expected_world: int, allow_shared: bool = False) -> None:
    """The multi-GPU line is only valid on a real N-GPU world (VERDICT r04 item
    6): `infos` is one dict per rank (all_gather_object of
    {"rank", "device", "bus_id", "host"}); raise RuntimeError unless the
    process group has exactly `expected_world` ranks, their ranks are
    0..N-1, and -- unless `allow_shared` (the gloo rehearsal with ranks on one
    GPU) -- every rank drives a distinct GPU.  A GPU is identified by its
    node AND its PCI bus id (or local index when torch exposes no bus id):
    every node of a multi-node world has the same bus ids, so ranks on
    different hosts never share a GPU.  `host` defaults to one
    node for callers that do not record it."""
    world = len(infos)
    if world != expected_world:
        raise RuntimeError(f"world size {world} != --gpus {expected_world}")
    ranks = sorted(int(i["rank"]) for i in infos)
    if ranks != list(range(world)):
        raise RuntimeError(f"ranks {ranks} are not 0..{world - 1}")
    if allow_shared:
        return
    ids = [(str(i.get("host") or ""), str(i.get("bus_id") or f"device{i['device']}"))
           for i in infos]
    if len(set(ids)) != world:
        dup = sorted({"/".join(x).lstrip("/") for x in ids if ids.count(x) > 1})
        raise RuntimeError(f"ranks share GPUs {dup}: a {world}-GPU line needs {world} devices")
