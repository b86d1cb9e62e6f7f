"""Process-group plumbing for data parallelism.

One process per GPU (torchrun-style env: RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT). On GPUs the backend is ``nccl`` - RCCL over xGMI on
MI355X; on CPU (CI) ``gloo``. The reference is single-process and has no
collectives; the ones this framework needs are:

* ``all_reduce`` of the flat gradient buffer every step (one 753 KB collective),
* ``broadcast`` of parameters + BN statistics at start / resume,
* ``all_reduce`` (mean) of the BN moving statistics at every epoch end,
* ``all_reduce`` of metric accumulators (loss sums, confusion counts, histograms),
* ``all_gather`` of predictions / labels for global AUC/MCC and of IG attributions,
* ``barrier`` around checkpointing.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import contextlib

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


_LOCAL = [False]


def world_size() -> int:
    """Ranks that share the current work (1 inside :func:`local`)."""
    return 1 if _LOCAL[0] else (dist.get_world_size() if is_initialized() else 1)


def rank() -> int:
    return 0 if _LOCAL[0] else (dist.get_rank() if is_initialized() else 0)


def global_world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def global_rank() -> int:
    return dist.get_rank() if is_initialized() else 0


@contextlib.contextmanager
def local():
    """Run independent per-rank work (e.g. one CV fold per GPU): inside, every collective of this
    module is a no-op and the rank sees a world of one, so a Trainer built here never all-reduces."""
    prev = _LOCAL[0]
    _LOCAL[0] = True
    try:
        yield
    finally:
        _LOCAL[0] = prev


def all_gather_object(obj):
    """Every rank's ``obj`` (a list in rank order; [obj] without a process group)."""
    if not is_initialized() or global_world_size() == 1:
        return [obj]
    out = [None] * global_world_size()
    dist.all_gather_object(out, obj)
    return out


def is_main() -> bool:
    return rank() == 0


def init_distributed(device: str = "auto", timeout_s: int = 600) -> torch.device:
    """Initialise the default process group from the environment; returns this rank's device."""
    world, rk, local = env_world()
    use_cuda = torch.cuda.is_available() if device == "auto" else device.startswith("cuda")
    if use_cuda:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1 and not is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = "nccl" if use_cuda else "gloo"
        kw = dict(backend=backend, rank=rk, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_cuda:
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return dev


def destroy():
    from .peer import close_all
    close_all()                    # (peer all-reduce mappings of this process, if any)
    if is_initialized():
        dist.destroy_process_group()


def barrier():
    if is_initialized() and not _LOCAL[0]:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def backend() -> Optional[str]:
    """The default process group's backend ("nccl" = RCCL on ROCm, "gloo"); None without one
    (or inside :func:`local`)."""
    return dist.get_backend() if is_initialized() and not _LOCAL[0] else None


def all_reduce_(t: torch.Tensor, op=None, force: bool = False) -> torch.Tensor:
    """In-place all-reduce (SUM by default). ``force``: issue the collective even on a one-rank
    process group (exercises the RCCL / graph-capture path on a single GPU)."""
    if is_initialized() and not _LOCAL[0] and (world_size() > 1 or force):
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_initialized() and world_size() > 1:
        dist.broadcast(t, src)
    return t


def broadcast_module(module: torch.nn.Module, src: int = 0):
    """Make parameters and buffers identical on every rank."""
    if not (is_initialized() and world_size() > 1):
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


def average_buffers(module: torch.nn.Module):
    """Mean of every floating-point buffer (BatchNorm moving mean / variance) over the ranks.

    Each rank updates the BN statistics from its own shard of the batch; Keras'
    MirroredStrategy mean-aggregates such variables, so they are averaged once per epoch,
    before evaluation, checkpointing or a resume snapshot read them. One collective over
    all buffers flattened together."""
    if not (is_initialized() and world_size() > 1):
        return
    bufs = [b for b in module.buffers() if b.is_floating_point()]
    if not bufs:
        return
    with torch.no_grad():
        flat = torch.cat([b.reshape(-1).to(torch.float64) for b in bufs])
        dist.all_reduce(flat)
        flat /= world_size()
        off = 0
        for b in bufs:
            n = b.numel()
            b.copy_(flat[off:off + n].view_as(b).to(b.dtype))
            off += n


def all_gather_var(t: torch.Tensor) -> torch.Tensor:
    """All-gather tensors whose first dim differs per rank; concatenated in rank order."""
    if not (is_initialized() and world_size() > 1):
        return t
    n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.long)
    sizes = [torch.zeros_like(n) for _ in range(world_size())]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
    pad[: t.shape[0]] = t
    out = [torch.zeros_like(pad) for _ in sizes]
    dist.all_gather(out, pad)
    return torch.cat([o[:s] for o, s in zip(out, sizes)], 0)


def max_over_ranks(x: float) -> float:
    if not (is_initialized() and world_size() > 1):
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


__all__ = ["init_distributed", "destroy", "barrier", "all_reduce_", "broadcast_", "broadcast_module", "average_buffers",
           "all_gather_var", "max_over_ranks", "world_size", "rank", "is_main", "is_initialized", "env_world",
           "local", "all_gather_object", "global_world_size", "global_rank", "backend"]
