"""Data-parallel correctness on CPU with gloo (world_size 2): the RCCL path by construction."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(seed=3):
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=4 * 1440, seed=seed))
    st = DeviceStore(ws, "rolling_median", pc.graph)
    mc = C.default("model_cml")
    mc.baseline_model.filter_1_size = 8
    return pc, mc, st


def _worker(rank, world, port, out_dir, ids):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.parallel import dist as D
    from gnnqc.train.engine import Trainer
    D.init_distributed(device="cpu")
    pc, mc, st = _setup()
    torch.manual_seed(rank + 100)            # different init per rank: broadcast must fix it
    m = BaselineClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 1e-3)
    D.broadcast_module(m)
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=False, batch_size=len(ids[rank]))
    t._body(torch.tensor(ids[rank]), with_opt=False)
    D.all_reduce_(opt.flat_g)
    g = (opt.flat_g / world).numpy()
    np.save(os.path.join(out_dir, f"g{rank}.npy"), g)
    np.save(os.path.join(out_dir, f"p{rank}.npy"), opt.flat_p.detach().numpy())
    D.destroy()


def test_dp_gradients_equal_single_process_large_batch(tmp_path):
    ids = [list(range(0, 16)), list(range(16, 32))]
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), ids), nprocs=2, join=True)
    g0, g1 = np.load(tmp_path / "g0.npy"), np.load(tmp_path / "g1.npy")
    p0, p1 = np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy")
    assert np.array_equal(p0, p1)            # broadcast made ranks identical
    assert np.allclose(g0, g1)
    # single process on the union batch, same weights
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, mc, st = _setup()
    m = BaselineClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 1e-3)
    opt.flat_p.copy_(torch.from_numpy(p0))
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=False, batch_size=32)
    t._body(torch.tensor(ids[0] + ids[1]), with_opt=False)
    ref = opt.flat_g.numpy()
    assert np.allclose(g0, ref, rtol=1e-4, atol=1e-6), np.abs(g0 - ref).max()


@pytest.mark.slow
def test_bench_runs_with_two_gloo_ranks():
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--sensors", "8", "--days", "3"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 256 and out["value"] > 0
