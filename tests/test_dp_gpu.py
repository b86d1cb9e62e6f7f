"""Data parallelism on the GPU box (one MI355X): two ranks on cuda:0 over gloo (the RCCL code
path of gnnqc.parallel.dist / Trainer with a different backend; RCCL itself needs one GPU per rank)
train the CML GCN through the HIP kernels - per-layer LSTM kernels, as two processes' cross-CU
chain kernels would share one device - and end with identical parameters; plus an RCCL (nccl)
process group of one rank doing the Trainer's collectives."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json
sys.path.insert(0, os.environ["GNNQC_ROOT"])
import numpy as np, torch
from gnnqc import config as C
from gnnqc.data.preprocessing import create_windows_dataset
from gnnqc.data.store import DeviceLoader, DeviceStore
from gnnqc.data.synthetic import make_cml_raw
from gnnqc.models import GCNClassifier
from gnnqc.ops.optim import make_optimizer
from gnnqc.parallel import dist as D
from gnnqc.train.engine import Trainer
backend = os.environ["BACKEND"]
torch.cuda.set_device(0)
torch.distributed.init_process_group(backend, init_method="env://")
rank, world = D.rank(), D.world_size()
dev = torch.device("cuda", 0)
pc = C.normalize_preproc(C.default("preprocessing_cml"))
pc.timestep_before, pc.timestep_after = 60, 30
ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=10, n_minutes=3 * 1440, seed=5))
st = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
torch.manual_seed(100 + rank)
m = GCNClassifier(C.default("model_cml"), pc).to(dev)
opt = make_optimizer("adam", m.parameters(), 1e-3)
D.broadcast_module(m)
t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, use_graph=True, batch_size=32)
x = torch.ones(4, device=dev) * (rank + 1)
D.all_reduce_(x)
nb = int(os.environ.get("NB", "4"))
loader = DeviceLoader(st, list(range(min(st.n_windows, 32 * nb * world))), 32, shuffle=True, seed=2, rank=rank,
                      world_size=world, drop_last=True)
logs = t.train_epoch(loader, 0)
torch.cuda.synchronize()
inj = os.environ.get("INJECT_PEER_TIMEOUT_RANK")
extra = {}
if inj is not None:          # fault injection: a peer spin timeout recorded on one rank
    p_before = opt.flat_p.double().sum().item()
    if rank == int(inj):
        t.peer.inject_timeout()
    torch.cuda.synchronize()
    try:
        t.train_epoch(loader, 1)
        extra["raised"] = False
    except RuntimeError as e:
        extra["raised"] = "spin timeout" in str(e)
    torch.cuda.synchronize()
    extra.update(p_before=p_before, p_after=opt.flat_p.double().sum().item(),
                 rejected=int(opt.guard_state[3].item()) if getattr(opt, "guard_state", None) is not None else -1)
bufs = torch.cat([b.reshape(-1).double() for b in m.buffers() if b.is_floating_point()])
out = {"sum": float(x[0]), "p": opt.flat_p.double().sum().item(), "p2": (opt.flat_p.double() ** 2).sum().item(),
       "b": bufs.sum().item(), "steps": t.global_step, "loss": logs["loss"], "skipped": logs["skipped_steps"],
       "dp_graph": bool(t.dp_graph), "multi": bool(t.multi_graph is not None), "ar_us": t.measure_allreduce(),
       "peer": t.peer is not None, "fused": bool(t.peer_fused()),
       "ps2": torch.nn.functional.pad(opt.flat_p.double(), (0, (-opt.flat_p.numel()) % 1024)).view(-1, 1024)
              .pow(2).sum(1).tolist(), **extra}
with open(os.path.join(os.environ["OUT"], f"r{rank}.json"), "w") as f:
    json.dump(out, f)
torch.distributed.destroy_process_group()
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, world, backend, chain=False, **extra):
    port = _port()
    tmp_path.mkdir(parents=True, exist_ok=True)
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK=str(r), BACKEND=backend, OUT=str(tmp_path), GNNQC_ROOT=ROOT,
                   HSA_ENABLE_IPC_MODE_LEGACY="0", **extra)
        if not chain:          # two processes' co-resident chain grids cannot share one device
            env.update(GNNQC_CHAIN="0", GNNQC_HEAD_CHAIN="0", GNNQC_CHAIN_BWD="0")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env))
    for p in procs:
        assert p.wait(timeout=240) == 0
    import json
    return [json.load(open(tmp_path / f"r{r}.json")) for r in range(world)]


def test_dp_two_ranks_one_gpu_identical_parameters(tmp_path):
    a, b = _run(tmp_path, 2, "gloo")
    assert a["sum"] == b["sum"] == 3.0
    assert a["steps"] == b["steps"] == 4 and a["skipped"] == b["skipped"] == 0
    assert a["p"] == b["p"] and a["p2"] == b["p2"], "ranks must apply the same all-reduced update"
    assert abs(a["b"] - b["b"]) <= 1e-9 * abs(a["b"]), "BN moving statistics averaged at epoch end"
    assert a["loss"] == b["loss"]


def test_rccl_process_group_single_rank(tmp_path):
    (a,) = _run(tmp_path, 1, "nccl")
    assert a["sum"] == 1.0 and a["steps"] == 4 and a["skipped"] == 0


def test_rccl_all_reduce_captured_in_multistep_graph(tmp_path):
    """The DP layout over RCCL with the gradient all-reduce INSIDE the multi-step HIP graph (forced
    collective on a one-rank nccl group, chain kernels on): it must capture, replay, and train like
    the same process without a collective (SUM over one rank is the identity)."""
    (a,) = _run(tmp_path / "a", 1, "nccl", chain=True, NB="16", GNNQC_DP_FORCE_COLLECTIVE="1")
    assert a["dp_graph"] and a["multi"], "the all-reduce must be captured in the multi-step graph"
    assert a["steps"] == 16 and a["skipped"] == 0 and a["ar_us"] is not None and a["ar_us"] > 0
    (b,) = _run(tmp_path / "b", 1, "nccl", chain=True, NB="16", GNNQC_DP_FORCE_COLLECTIVE="0")
    assert not b["dp_graph"] and b["multi"] and b["steps"] == 16
    for k in ("p", "p2", "loss"):
        assert abs(a[k] - b[k]) <= 1e-4 * abs(b[k]) + 1e-6, (k, a[k], b[k])


def test_peer_allreduce_two_ranks_one_gpu(tmp_path):
    """One-shot peer all-reduce (IPC-registered regions, flag signalling, rank-order sum) between two
    processes sharing the GPU: it verifies against gloo at setup, is captured in the multi-step
    graph, and both ranks end with identical parameters."""
    a, b = _run(tmp_path, 2, "gloo", NB="16", GNNQC_PEER_ALLREDUCE="1")
    assert a["peer"] and b["peer"], "peer all-reduce must pass its verification against gloo"
    assert a["dp_graph"] and a["multi"]
    assert a["steps"] == b["steps"] == 16 and a["skipped"] == b["skipped"] == 0
    assert a["p"] == b["p"] and a["p2"] == b["p2"]
    assert a["ar_us"] is not None and a["ar_us"] > 0


def test_peer_fused_adam_matches_separate_kernels_two_ranks(tmp_path):
    """The peer reduction fused into the flag-driven Adam launch (adam_peer) trains like the peer
    all-reduce kernel followed by adam_flagged, two ranks sharing the GPU."""
    a, b = _run(tmp_path / "fused", 2, "gloo", NB="16", GNNQC_PEER_ALLREDUCE="1")
    c, d = _run(tmp_path / "sep", 2, "gloo", NB="16", GNNQC_PEER_ALLREDUCE="1", GNNQC_PEER_FUSED_ADAM="0")
    assert a["fused"] and b["fused"] and not c["fused"] and a["peer"] and c["peer"]
    assert a["steps"] == c["steps"] == 16 and a["skipped"] == c["skipped"] == 0
    for k in ("p", "p2", "loss"):
        # ranks of one run agree bitwise; the two runs differ only by the float-atomic order of the
        # GCN backward (a separate process each; deterministic mode has no flag-driven update to
        # fuse), which 16 Adam steps amplify to ~2e-6 of the norm (measured)
        assert a[k] == b[k] and c[k] == d[k], (k, a[k], b[k], c[k], d[k])
        assert abs(a[k] - c[k]) <= 1e-4 * abs(c[k]) + 1e-9, (k, a[k], c[k])
    # per 1024-float slice (one adam_peer workgroup each): sum of squares of the parameters. A slice
    # whose update was skipped or stale moves its sum by ~2 dp / p (percents after 16 steps), far
    # outside the atomic-order noise
    for i, (u, v) in enumerate(zip(a["ps2"], c["ps2"])):
        assert abs(u - v) <= 1e-4 * abs(v) + 1e-9, (i, u, v)


def test_peer_auto_mode_selects_and_trains(tmp_path):
    """Default (auto) peer mode with two ranks: set up, verified, timed against gloo, selected only
    if faster; either way both ranks end identical."""
    a, b = _run(tmp_path, 2, "gloo", NB="8")
    assert a["peer"] == b["peer"]
    assert a["p"] == b["p"] and a["p2"] == b["p2"] and a["skipped"] == 0


def test_peer_allreduce_matches_rccl_single_rank(tmp_path):
    """The peer path on a one-rank nccl group with the chain kernels on trains like RCCL."""
    (a,) = _run(tmp_path / "peer", 1, "nccl", chain=True, NB="16", GNNQC_DP_FORCE_COLLECTIVE="1",
                GNNQC_PEER_ALLREDUCE="1")
    (b,) = _run(tmp_path / "rccl", 1, "nccl", chain=True, NB="16", GNNQC_DP_FORCE_COLLECTIVE="1")
    assert a["peer"] and not b["peer"] and a["dp_graph"] and a["multi"] and a["fused"]
    for k in ("p", "p2", "loss"):
        assert abs(a[k] - b[k]) <= 1e-4 * abs(b[k]) + 1e-6, (k, a[k], b[k])


def test_peer_fused_timeout_rejects_every_later_step_on_every_rank(tmp_path):
    """adam_peer fault handling: after a peer spin timeout recorded on ONE rank (injected), every
    later step is rejected on EVERY rank (the timed-out rank's flag bit carries the rejection), so
    the ranks' parameters stay identical and unchanged, and the epoch end raises on every rank."""
    a, b = _run(tmp_path, 2, "gloo", NB="16", GNNQC_PEER_ALLREDUCE="1", INJECT_PEER_TIMEOUT_RANK="1")
    assert a["fused"] and b["fused"]
    assert a["raised"] and b["raised"], "the epoch end must raise on every rank"
    assert a["p_after"] == b["p_after"] == a["p_before"] == b["p_before"], (a, b)
