"""Step-level launch fusion on the GPU: guard + Adam in one launch (rejects a non-finite or
chain-timed-out step on the device, advances the batch cursor), the cursor-driven batch gather,
and multi-step HIP graphs == the same steps replayed one by one."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_adam_guarded_rejects_nonfinite_and_advances_cursor(cuda_device):
    from gnnqc.ops.optim import FlatAdam
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(1001, 37)), torch.nn.Parameter(torch.randn(13))]   # n % 4 != 0
    ps_gpu = [torch.nn.Parameter(p.detach().clone().to(cuda_device)) for p in ps]
    a_cpu, a_gpu = FlatAdam(ps, 1e-2), FlatAdam(ps_gpu, 1e-2)
    cur = torch.zeros(1, dtype=torch.long, device=cuda_device)
    a_gpu.cursor, a_gpu.cursor_mod = cur, 3
    for k in range(7):
        g = torch.randn_like(a_cpu.flat_g)
        if k == 3:
            g[1234] = float("nan")
        a_cpu.flat_g.copy_(g)
        a_gpu.flat_g.copy_(g.to(cuda_device))
        before = a_gpu.flat_p.clone()
        a_cpu.step(0.5)
        a_gpu.step(0.5)
        torch.cuda.synchronize()
        if k == 3:
            assert torch.equal(a_gpu.flat_p, before), "a non-finite step must not change the parameters"
        assert float(a_gpu.flat_g.abs().max()) == 0.0, "the update clears the gradient buffer"
    assert a_gpu.skipped_steps == 1 and a_cpu.skipped_steps == 1
    assert float(a_gpu.step_t) == 6.0
    assert int(cur) == 7 % 3
    assert torch.allclose(a_cpu.flat_p, a_gpu.flat_p.cpu(), atol=1e-6)


def test_batch_gather_cursor_rows(cuda_device, cml_windows):
    from gnnqc.data.store import CursorIds, DeviceStore
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    n = st.n_windows
    table = torch.tensor([[0, 3, -1, n - 1], [n // 2, 1, 2, 4]], device=cuda_device)
    cur = torch.tensor([3], dtype=torch.long, device=cuda_device)          # 3 % 2 -> row 1
    got = st.gather(CursorIds(table, cur))
    ref = st.gather(table[1])
    for name in ("x", "adj", "node_mask", "anom", "anom_pos", "y", "y_mask", "wid"):
        assert torch.equal(getattr(got, name), getattr(ref, name)), name


def _multi_vs_single_run(steps, st, pc, mc, rows, dev, monkeypatch, k=16, prepare=False):
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    monkeypatch.setenv("GNNQC_GRAPH_STEPS", str(steps))
    torch.manual_seed(0)
    model = GCNClassifier(mc, pc).to(dev)
    opt = make_optimizer("adam", model.parameters(), 1e-3)
    tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=True, batch_size=32)
    if prepare:
        tr.prepare_graphs(rows)
        assert (tr.multi_graph1 is not None) == (steps > 1)
    tr.train_steps(rows, 3, k)
    torch.cuda.synchronize()
    assert (tr.multi_graph is not None) == (steps > 1)
    bufs = torch.cat([b.reshape(-1).double() for b in model.buffers() if b.is_floating_point()])
    return (opt.flat_p.clone(), opt.m.clone(), bufs, tr.train_metrics.sums.clone(), float(tr.last_loss),
            opt.iterations, tr.global_step)


def test_multi_step_graph_matches_single_steps(cuda_device, cml_windows, monkeypatch):
    """16 steps as two 8-step graph replays (device cursor) == 16 single-step replays: same
    parameters, optimiser slots, BN statistics and metric sums. Run with the bitwise-reproducible
    kernels: the default store-fused GCN backward sums its parameter gradients with float atomics,
    and Adam amplifies that run-to-run noise on near-zero gradients (two runs of the SAME layout
    differ by ~1e-3 of the parameter norm after a few steps), which no layout-discriminating
    tolerance survives."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.ops import set_deterministic
    pc, ws = cml_windows
    mc = C.default("model_cml")
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    loader = DeviceLoader(st, list(range(st.n_windows)), 32, shuffle=True, seed=1)
    rows = loader.batch_ids()
    prev = set_deterministic(True)
    try:
        a, b = [_multi_vs_single_run(steps, st, pc, mc, rows, cuda_device, monkeypatch) for steps in (8, 1)]
    finally:
        set_deterministic(prev)
    for x, y in zip(a[:4], b[:4]):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
    assert abs(a[4] - b[4]) <= 1e-4 * abs(b[4]) + 1e-6
    assert a[5:] == b[5:] == (16, 16)


def test_leftover_steps_replay_the_one_step_graph(cuda_device, cml_windows, monkeypatch):
    """11 steps with prepared graphs = one 8-step replay + three replays of the one-step graph of
    the same form (same device table and cursor, no host id copies) == 11 single-step replays."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.ops import set_deterministic
    pc, ws = cml_windows
    mc = C.default("model_cml")
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    rows = DeviceLoader(st, list(range(st.n_windows)), 32, shuffle=True, seed=1).batch_ids()
    prev = set_deterministic(True)
    try:
        a, b = [_multi_vs_single_run(steps, st, pc, mc, rows, cuda_device, monkeypatch, k=11, prepare=True)
                for steps in (8, 1)]
    finally:
        set_deterministic(prev)
    for x, y in zip(a[:4], b[:4]):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
    assert a[5:] == b[5:] == (11, 11)
