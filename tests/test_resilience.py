"""Failure handling: non-finite guard, fault injection, kill + resume."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from gnnqc import config as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _adam(n=37, guard=True, device="cpu"):
    from gnnqc.ops.optim import FlatAdam
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(n, device=device))
    return p, FlatAdam([p], lr=1e-2, guard=guard)


def test_guard_skips_nonfinite_step_cpu():
    p, opt = _adam()
    opt.flat_g.copy_(torch.randn_like(opt.flat_g))
    opt.step()
    p1, m1, v1 = p.detach().clone(), opt.m.clone(), opt.v.clone()
    assert opt.step_t.item() == 1 and opt.skipped_steps == 0
    opt.flat_g[3] = float("nan")
    opt.step()
    assert torch.equal(p.detach(), p1) and torch.equal(opt.m, m1) and torch.equal(opt.v, v1)
    assert opt.step_t.item() == 1 and opt.skipped_steps == 1 and opt.iterations == 2
    opt.flat_g.copy_(torch.randn_like(opt.flat_g))
    opt.flat_g[0] = float("inf")
    opt.step()
    assert opt.skipped_steps == 2
    opt.flat_g.copy_(torch.randn_like(opt.flat_g))
    opt.step()
    assert opt.step_t.item() == 2 and not torch.equal(p.detach(), p1)


@pytest.mark.parametrize("name", ["sgd", "rmsprop"])
def test_guard_other_optimizers(name):
    from gnnqc.ops.optim import make_optimizer
    p = torch.nn.Parameter(torch.randn(9))
    opt = make_optimizer(name, [p], 1e-2)
    before = p.detach().clone()
    opt.flat_g.fill_(float("nan"))
    opt.step()
    assert torch.equal(p.detach(), before) and opt.skipped_steps == 1


def test_guard_off_propagates_nan():
    p, opt = _adam(guard=False)
    opt.flat_g.fill_(float("nan"))
    opt.step()
    assert torch.isnan(p.detach()).all()


def _tiny_trainer(device="cpu", use_graph=False):
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=10 * 1440, seed=5))
    st = DeviceStore(ws, "rolling_median", pc.graph, device=torch.device(device))
    mc = C.default("model_cml")
    mc.baseline_model.filter_1_size = 16
    torch.manual_seed(0)
    m = BaselineClassifier(mc, pc).to(device)
    opt = make_optimizer("adam", m.parameters(), 3e-3)
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=use_graph, batch_size=64)
    return t, DeviceLoader(st, np.arange(min(st.n_windows, 384)), 64)


def test_nan_injection_is_skipped_cpu(monkeypatch):
    monkeypatch.setenv("GNNQC_FI_NAN_AT_STEP", "2,5")
    t, L = _tiny_trainer()
    logs = t.train_epoch(L, 0)
    assert logs["skipped_steps"] == 2
    assert t.opt.step_t.item() == t.global_step - 2
    assert all(torch.isfinite(p).all() for p in t.model.parameters())
    assert logs["windows_per_sec"] > 0
    logs = t.train_epoch(L, 1)
    assert logs["skipped_steps"] == 0


def _run_job(work, out, env_extra=None, resume=False):
    env = dict(os.environ)
    env.pop("GNNQC_FI_KILL_RANK_AT_STEP", None)
    env.pop("GNNQC_FI_NAN_AT_STEP", None)
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    cmd = [sys.executable, os.path.join(ROOT, "tests", "helpers", "resume_job.py"), str(work), str(out)]
    if resume:
        cmd.append("--resume")
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)


def test_kill_and_resume_matches_uninterrupted(tmp_path):
    from gnnqc.train.resilience import FI_EXIT_CODE
    ref = _run_job(tmp_path / "a", tmp_path / "a.pt")
    assert ref.returncode == 0, ref.stderr[-2000:]
    # 10 steps per epoch: die in the middle of the second epoch
    r = _run_job(tmp_path / "b", tmp_path / "b.pt", {"GNNQC_FI_KILL_RANK_AT_STEP": "0:15"})
    assert r.returncode == FI_EXIT_CODE, r.stderr[-2000:]
    assert not (tmp_path / "b.pt").exists()
    assert (tmp_path / "b" / "resume" / "resume.pt").exists()
    r = _run_job(tmp_path / "b", tmp_path / "b.pt", resume=True)
    assert r.returncode == 0, r.stderr[-2000:]
    a = torch.load(tmp_path / "a.pt", weights_only=True)
    b = torch.load(tmp_path / "b.pt", weights_only=True)
    assert a["loss"] == b["loss"]
    for k in a["state"]:
        assert torch.equal(a["state"][k], b["state"][k]), k


def test_rng_state_roundtrip():
    import random
    from gnnqc.train.resilience import rng_state, set_rng_state
    st = rng_state()
    x = (random.random(), np.random.rand(), torch.rand(1).item())
    set_rng_state(st)
    assert x == (random.random(), np.random.rand(), torch.rand(1).item())


@pytest.mark.gpu
def test_guard_inside_hip_graph(cuda_device, monkeypatch):
    monkeypatch.setenv("GNNQC_FI_NAN_AT_STEP", "3")
    t, L = _tiny_trainer("cuda", use_graph=True)
    logs = t.train_epoch(L, 0)
    assert t.graph is not None
    assert logs["skipped_steps"] == 1
    assert t.opt.step_t.item() == t.global_step - 1
    assert all(torch.isfinite(p).all() for p in t.model.parameters())


@pytest.mark.gpu
def test_guard_kernel_matches_eager(cuda_device):
    p, opt = _adam(n=1001, device="cuda")
    for bad in (False, True, False):
        opt.flat_g.copy_(torch.randn_like(opt.flat_g))
        if bad:
            opt.flat_g[777] = float("nan")
        before = p.detach().clone()
        opt.step()
        torch.cuda.synchronize()
        assert torch.equal(p.detach(), before) == bad
    assert opt.skipped_steps == 1 and opt.step_t.item() == 2
    assert opt.guard_state[0].item() == 0 and opt.guard_state[1].item() == 0


def _gcn_train_state(device, steps=6, det=True):
    from gnnqc.data.store import DeviceLoader
    from gnnqc.models import GCNClassifier
    from gnnqc.ops import set_deterministic
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    prev = set_deterministic(det)
    try:
        pc = C.normalize_preproc(C.default("preprocessing_cml"))
        ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=10, n_minutes=4 * 1440, seed=3))
        st = DeviceStore(ws, "rolling_median", pc.graph, device=torch.device(device))
        mc = C.default("model_cml")
        torch.manual_seed(0)
        m = GCNClassifier(mc, pc).to(device)
        opt = make_optimizer("adam", m.parameters(), 1e-3)
        t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, use_graph=True, batch_size=128)
        L = DeviceLoader(st, np.arange(min(st.n_windows, 128 * steps)), 128)
        t.train_epoch(L, 0)
        torch.cuda.synchronize()
        return {k: v.detach().clone() for k, v in m.state_dict().items()}
    finally:
        set_deterministic(prev)


@pytest.mark.gpu
def test_deterministic_mode_bitwise_reproducible(cuda_device):
    a = _gcn_train_state("cuda")
    b = _gcn_train_state("cuda")
    for k in a:
        assert torch.equal(a[k], b[k]), k
