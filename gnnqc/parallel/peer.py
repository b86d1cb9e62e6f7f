"""One-shot peer all-reduce over xGMI for the flat gradient buffer.

``csrc/kernels/peer_allreduce.hip``: every rank registers a region (gradients, double-buffered,
plus signal flags), exports it with a HIP IPC handle and opens every peer's; one kernel then
publishes this rank's gradients, signals all ranks and sums all N copies in rank order, read
directly over the point-to-point xGMI links - one step instead of RCCL's 2 (N-1) ring steps for a
753 KB buffer. The kernel is a plain launch (no host synchronisation), so it is captured in the
multi-step training graph like the RCCL collective it replaces.

Selected by :func:`peer_mode` (default ``auto``: with two or more ranks it is set up, validated
against RCCL / gloo (:meth:`PeerAllReduce.verify`) and timed against the process group's all-reduce,
and used only if it verified and was faster); one process per GPU of one node, at most 8 ranks. A
training step whose gradient producers all raise the non-finite flag reduces INSIDE the Adam launch
(``adam_peer``): that fused kernel is checked separately at setup against the all-reduce kernel
followed by ``adam_flagged`` on scratch buffers, timed against that pair, and used only when it agrees
(and, in ``auto`` mode, is faster) on every rank (:func:`check_fused_adam`). The handles
are exchanged with the default process group, so it works over gloo as well (tests: two ranks
sharing one GPU). Between different GPUs over xGMI it has NOT been run (no multi-GPU box was
available): treat it as unverified there until a multi-GPU run checks it against RCCL.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from . import dist as D


def peer_mode() -> str:
    """``GNNQC_PEER_ALLREDUCE``: ``0`` off, ``1`` on whenever it verifies, ``auto`` (default) on when
    it verifies AND beats the process group's all-reduce of the same buffer in a timing at setup
    (more than one rank only: a one-rank group needs no collective)."""
    v = os.environ.get("GNNQC_PEER_ALLREDUCE", "auto").strip().lower()
    return {"1": "on", "on": "on", "0": "off", "off": "off"}.get(v, "auto")


def peer_enabled() -> bool:
    return peer_mode() != "off"


# the last setup's decision: {"mode", "verified", "rccl_us", "peer_us", "selected"} (bench.py reports it)
LAST_SELECTION: dict = {}


class PeerAllReduce:
    def __init__(self, numel: int, device: torch.device):
        from ..utils.native import hip_ops
        self.ops = hip_ops()
        self.world, self.rank = D.world_size(), D.rank()
        if not 1 <= self.world <= 8:
            raise RuntimeError("peer all-reduce: 1..8 ranks of one node")
        self.device = torch.device(device)
        self.cap = (int(numel) + 3) // 4 * 4
        with torch.cuda.device(self.device):
            self.region = self.ops.peer_region_alloc(self.cap)
            handle = self.ops.peer_ipc_handle(self.region)
        handles = D.all_gather_object(bytes(handle.numpy().tobytes()))
        self._opened: List[int] = []
        bases = []
        for p, h in enumerate(handles):
            if p == self.rank:
                bases.append(int(self.region.data_ptr()))
            else:
                ptr = int(self.ops.peer_ipc_open(torch.frombuffer(bytearray(h), dtype=torch.uint8)))
                self._opened.append(ptr)
                bases.append(ptr)
        self.bases = bases
        D.barrier()

    def __call__(self, t: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        """In place: t <- scale * sum over ranks of t (fp32, contiguous, <= the registered size)."""
        self.ops.peer_allreduce(t, self.bases, self.region, self.rank, self.cap, float(scale))
        return t

    def timed_out(self) -> bool:
        ctl = self.region[2 * self.cap + 8 * 16: 2 * self.cap + 8 * 16 + 16].view(torch.int32)
        return bool(ctl[2].item())

    def inject_timeout(self):
        """Fault injection (tests): mark this rank's region as if a peer spin had timed out. The fused
        update (``adam_peer``) then rejects every later step on every rank, and the epoch end raises."""
        ctl = self.region[2 * self.cap + 8 * 16: 2 * self.cap + 8 * 16 + 16].view(torch.int32)
        ctl[2].fill_(1)

    @torch.no_grad()
    def verify(self, trials: int = 3) -> bool:
        """Compare with the process group's all-reduce on rank-dependent data (every rank takes
        the same decision: the verdict is all-reduced too)."""
        ok = True
        g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
        for _ in range(trials):
            x = torch.randn(self.cap, generator=g).to(self.device)
            ref = x.clone()
            D.all_reduce_(ref, force=True)
            self(x)
            torch.cuda.synchronize(self.device)
            ok &= not self.timed_out() and torch.allclose(x, ref, rtol=1e-5, atol=1e-5)
        flag = torch.tensor([0.0 if ok else 1.0], device=self.device if D.backend() == "nccl" else "cpu")
        D.all_reduce_(flag, force=True)
        return float(flag.item()) == 0.0

    def close(self):
        for p in self._opened:
            self.ops.peer_ipc_close(p)
        self._opened = []


_CACHE = {}


def make_peer_allreduce(numel: int, device) -> Optional[PeerAllReduce]:
    """A verified peer all-reduce (see :func:`peer_mode`; None when off, when it fails verification
    or, in ``auto`` mode, when the process group's collective was faster - the caller then uses that). One registered region per
    (device, size, group size) for the whole process: every Trainer (one per CV fold) reuses it
    instead of exporting and opening a new set of IPC regions."""
    mode = peer_mode()
    if mode == "off" or torch.device(device).type != "cuda" or not D.is_initialized():
        return None
    if mode == "auto" and D.world_size() < 2:
        return None
    key = (str(torch.device(device)), (int(numel) + 3) // 4 * 4, D.world_size(), D.rank(), mode)
    if key in _CACHE:
        return _CACHE[key]
    pa = _make_peer_allreduce(numel, device)
    LAST_SELECTION.clear()
    LAST_SELECTION.update(mode=mode, verified=pa is not None, rccl_us=None, peer_us=None,
                          selected="peer" if pa is not None else "process group")
    if pa is not None and mode == "auto":
        rccl_us, peer_us = _time_both(pa, numel, device)
        LAST_SELECTION.update(rccl_us=rccl_us, peer_us=peer_us)
        if not peer_us < rccl_us:
            LAST_SELECTION["selected"] = "process group"
            pa.close()
            pa = None
    _CACHE[key] = pa
    return pa


@torch.no_grad()
def _time_both(pa: "PeerAllReduce", numel: int, device, n: int = 30):
    """Mean us of the process group's all-reduce and of the peer kernel on a scratch buffer of the
    gradient's size (HIP events, max over ranks so every rank takes the same decision)."""
    buf = torch.zeros(int(numel), device=device)

    def timed(fn):
        for _ in range(3):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize(device)
        return 1e3 * sum(a.elapsed_time(b) for a, b in ev) / n

    r = timed(lambda: D.all_reduce_(buf, force=True))
    q = timed(lambda: pa(buf))
    t = torch.tensor([r, q], device=device if D.backend() == "nccl" else "cpu", dtype=torch.float64)
    D.all_reduce_(t, op=torch.distributed.ReduceOp.MAX, force=True)
    return float(t[0].item()), float(t[1].item())


PEER_SLICES = 1024        # peer_allreduce.hip: slice flags of the fused update (1024 floats each)


def fused_adam_fits(numel: int) -> bool:
    """Whether adam_peer can take a flat buffer of ``numel`` floats (one workgroup per 1024-float
    slice, at most PEER_SLICES of them)."""
    return max(1, (int(numel) // 4 + 255) // 256) <= PEER_SLICES


_FUSED = {}


@torch.no_grad()
def check_fused_adam(pa: "PeerAllReduce", numel: int, device, beta1: float = 0.9, beta2: float = 0.999,
                     eps: float = 1e-7, trials: int = 2, n_time: int = 20) -> bool:
    """Setup check of the reduction fused into the Adam launch (``adam_peer``) before a trainer uses
    it: on scratch p / m / v / g buffers (rank-dependent gradients), ``trials`` fused steps are
    compared with the verified peer all-reduce followed by ``adam_flagged`` (same rank-order sum,
    same update arithmetic: bitwise equal expected, tolerance 1e-6 relative), and the step counters
    must agree. The verdict is all-reduced so every rank decides alike. In ``auto`` mode the fused
    launch is also timed against the two separate launches and used only when faster (recorded in
    LAST_SELECTION). Cached per peer region. False (the trainer keeps the two kernels) when the buffer
    exceeds the fused kernel's slice table."""
    key = (id(pa), int(numel))
    if key in _FUSED:
        return _FUSED[key]
    from ..ops.lstm import chain_ctl
    ops = pa.ops
    dev = torch.device(device)
    world = pa.world
    ok = fused_adam_fits(numel)
    fused_us = sep_us = None
    if ok:
        gen = torch.Generator(device="cpu").manual_seed(4321)
        p0 = torch.randn(numel, generator=gen).to(dev)
        m0 = (0.01 * torch.randn(numel, generator=gen)).to(dev)
        v0 = (0.001 * torch.rand(numel, generator=gen)).to(dev)
        gr = torch.Generator(device="cpu").manual_seed(77 + pa.rank)
        lr = torch.tensor([1e-3], device=dev)
        ext = chain_ctl(dev)
        bufs = {}
        for name in ("fused", "sep"):
            bufs[name] = dict(p=p0.clone(), m=m0.clone(), v=v0.clone(), step=torch.zeros(1, device=dev),
                              state=torch.tensor([0, 0, 1, 0, 0, 0, 0, 0], dtype=torch.int32, device=dev))

        def fused(b, g):
            return ops.adam_peer(b["p"], g, b["m"], b["v"], lr, b["step"], beta1, beta2, eps, 1.0 / world, 0.0,
                                 b["state"], None, 1, pa.bases, pa.region, pa.rank, pa.cap)

        def sep(b, g):
            pa(g)
            ops.adam_flagged(b["p"], g, b["m"], b["v"], lr, b["step"], beta1, beta2, eps, 1.0 / world, 0.0,
                             b["state"], ext, None, 1)
            return True

        for _ in range(trials):
            g = torch.randn(numel, generator=gr).to(dev)
            g2 = g.clone()
            ok &= bool(fused(bufs["fused"], g))
            sep(bufs["sep"], g2)
            torch.cuda.synchronize(dev)
            ok &= not pa.timed_out() and bool((g == 0).all().item())
        a, b = bufs["fused"], bufs["sep"]
        for k in ("p", "m", "v"):
            ok &= bool(torch.allclose(a[k], b[k], rtol=1e-6, atol=0.0))
        ok &= float(a["step"].item()) == float(b["step"].item()) == float(trials)
    # agree on the verdict BEFORE the timing block: ``ok`` is rank-local (timeouts, the g == 0 check,
    # allclose), and the timing block issues peer launches and a collective, so every rank must take
    # the same branch or the collective sequences mismatch
    flag = torch.tensor([0.0 if ok else 1.0], device=dev if D.backend() == "nccl" else "cpu")
    D.all_reduce_(flag, force=True)
    verified = float(flag.item()) == 0.0
    if verified and peer_mode() == "auto":
        g = torch.zeros(numel, device=dev)

        def timed(fn, bb):
            for _ in range(3):
                fn(bb, g)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(n_time)]
            for e0, e1 in ev:
                e0.record()
                fn(bb, g)
                e1.record()
            torch.cuda.synchronize(dev)
            return 1e3 * sum(e0.elapsed_time(e1) for e0, e1 in ev) / n_time
        sep_us, fused_us = timed(sep, b), timed(fused, a)
        t = torch.tensor([sep_us, fused_us], device=dev if D.backend() == "nccl" else "cpu", dtype=torch.float64)
        D.all_reduce_(t, op=torch.distributed.ReduceOp.MAX, force=True)
        sep_us, fused_us = float(t[0].item()), float(t[1].item())
    use = verified and (fused_us is None or fused_us < sep_us)
    LAST_SELECTION.update(fused_adam_verified=verified, fused_adam_us=fused_us, separate_adam_us=sep_us,
                          fused_adam_selected=use)
    if not verified and fused_adam_fits(numel):
        import warnings
        warnings.warn("adam_peer (peer reduction fused into Adam) failed its setup check: using the all-reduce "
                      "kernel followed by adam_flagged")
    _FUSED[key] = use
    return use


def close_all():
    """Close every cached peer region's peer mappings (process teardown)."""
    for pa in _CACHE.values():
        if pa is not None:
            pa.close()
    _CACHE.clear()
    _FUSED.clear()


def _make_peer_allreduce(numel: int, device) -> Optional[PeerAllReduce]:
    pa, err = None, None
    try:                           # (IPC export / open can fail: every rank must learn it)
        pa = PeerAllReduce(numel, device)
    except RuntimeError as e:      # noqa: PERF203
        err = e
    bad = torch.tensor([0.0 if pa is not None else 1.0],
                       device=torch.device(device) if D.backend() == "nccl" else "cpu")
    D.all_reduce_(bad, force=True)
    if float(bad.item()) != 0.0:
        import warnings
        warnings.warn(f"peer all-reduce setup failed on some rank ({err}): using the process group's collective")
        if pa is not None:
            pa.close()
        return None
    if not pa.verify():
        import warnings
        warnings.warn("peer all-reduce failed verification against the process group: using it is disabled")
        pa.close()
        return None
    return pa


__all__ = ["PeerAllReduce", "make_peer_allreduce", "peer_enabled", "peer_mode", "close_all", "LAST_SELECTION",
           "check_fused_adam", "fused_adam_fits"]
