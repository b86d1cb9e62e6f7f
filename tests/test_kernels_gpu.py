"""HIP kernel numerics vs plain PyTorch fp32 references (run on the MI355X box)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lstm_params(Din, H, gen, dev):
    W = (torch.randn(Din, 4 * H, generator=gen) * 0.3).to(dev)
    U = (torch.randn(H, 4 * H, generator=gen) * 0.3).to(dev)
    b = (torch.randn(4 * H, generator=gen) * 0.1).to(dev)
    return W, U, b


@pytest.mark.parametrize("H", [16, 32, 64, 128])
@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("ret_seq", [True, False])
def test_lstm_fwd_bwd_matches_eager(cuda_device, H, bf16, ret_seq):
    from gnnqc.ops.lstm import _HipLSTM, lstm_eager
    dev = cuda_device
    gen = torch.Generator().manual_seed(H + 7 * bf16)
    M, T, Din = 40, 13, 18
    x = torch.randn(M, T, Din, generator=gen).to(dev)
    W, U, b = _lstm_params(Din, H, gen, dev)
    params = [t.clone().requires_grad_(True) for t in (x, W, U, b)]
    ref_params = [t.clone().double().requires_grad_(True) for t in (x, W, U, b)]
    out = _HipLSTM.apply(*params, bf16, ret_seq)
    ref = lstm_eager(*ref_params, return_sequences=ret_seq)
    tol = 3e-2 if bf16 else 2e-5
    assert torch.allclose(out.double(), ref, atol=tol, rtol=tol), (out.double() - ref).abs().max()
    g = torch.randn(out.shape, generator=gen).to(dev)
    out.backward(g)
    ref.backward(g.double())
    for p, r, name in zip(params, ref_params, "xWUb"):
        err = (p.grad.double() - r.grad).abs().max().item()
        scale = r.grad.abs().max().item() + 1e-6
        assert err / scale < (5e-2 if bf16 else 1e-4), f"grad {name}: rel err {err / scale}"


@pytest.mark.parametrize("Din,H", [(18, 16), (16, 16), (32, 64), (64, 128), (19, 16)])
def test_lstm_direct_grad_accumulation_and_padded_rows(cuda_device, Din, H):
    """Strided (row-padded) input + gradients accumulated straight into .grad views."""
    from gnnqc.ops.lstm import _HipLSTM, direct_grad_accumulation, lstm_eager
    dev = cuda_device
    gen = torch.Generator().manual_seed(Din * H)
    M, T = 37, 11
    buf = torch.randn(M, T, Din + 6, generator=gen).to(dev)
    x = buf[..., :Din]                                   # row stride Din + 6
    W, U, b = _lstm_params(Din, H, gen, dev)
    pW, pU, pb = (torch.nn.Parameter(t.clone()) for t in (W, U, b))
    for p in (pW, pU, pb):
        p.grad = torch.full_like(p, 0.5)                 # pre-existing buffer: must accumulate
    xg = x.clone().requires_grad_(True)
    with direct_grad_accumulation(True):
        out = _HipLSTM.apply(xg, pW, pU, pb, True, True)
        g = torch.randn(out.shape, generator=gen).to(dev)
        out.backward(g)
    ref_p = [t.clone().double().requires_grad_(True) for t in (x, W, U, b)]
    ref = lstm_eager(*ref_p)
    ref.backward(g.double())
    assert (out.double() - ref).abs().max().item() < 3e-2
    for p, r, name in zip((xg, pW, pU, pb), ref_p, "xWUb"):
        got = p.grad.double() - (0.0 if name == "x" else 0.5)
        err = (got - r.grad).abs().max().item() / (r.grad.abs().max().item() + 1e-6)
        assert err < 5e-2, f"{name}: {err}"


@pytest.mark.parametrize("H", [16, 32, 64, 128])
@pytest.mark.parametrize("Dw,lddx", [(16, 16), (18, 20), (32, 32), (40, 44), (64, 64), (100, 100)])
@pytest.mark.parametrize("zdt", [torch.float32, torch.bfloat16])
def test_lstm_dx_matches_matmul(cuda_device, H, Dw, lddx, zdt):
    """Standalone dx = dz W^T kernel (all row-tile / din-tile layouts; fp32 dz of the sequence-major
    recurrence, bf16 dz of the time-major ones) vs an fp32 matmul of the bf16-rounded operands;
    layout-padding columns come out as zeros."""
    from gnnqc.utils.native import hip_ops
    gen = torch.Generator().manual_seed(H + Dw)
    rows = 16 * 37 + 5
    dz = torch.randn(rows + 3, 4 * H, generator=gen).to(cuda_device).to(zdt)
    W = torch.randn(Dw, 4 * H, generator=gen).to(cuda_device) * 0.2
    like = torch.empty(rows, lddx, device=cuda_device)
    dx = hip_ops().lstm_dx(dz, W, like)
    ref = dz[:rows].bfloat16().float() @ W.bfloat16().float().t()
    torch.testing.assert_close(dx[:, :Dw], ref, atol=1e-3, rtol=1e-3)
    assert dx.dtype == torch.float32
    assert torch.count_nonzero(dx[:, Dw:]).item() == 0


def test_lstm_long_sequence_fp32_exact(cuda_device):
    from gnnqc.ops.lstm import _HipLSTM, lstm_eager
    gen = torch.Generator().manual_seed(3)
    dev = cuda_device
    x = torch.randn(128, 181, 18, generator=gen).to(dev)
    W, U, b = _lstm_params(18, 16, gen, dev)
    out = _HipLSTM.apply(x, W, U, b, False, True)
    ref = lstm_eager(x.double(), W.double(), U.double(), b.double())
    assert (out.double() - ref).abs().max().item() < 1e-4


def _gcn_inputs(gen, dev, B=6, T=9, N=7, Cin=2, F=16):
    x = torch.randn(B, T, N, Cin, generator=gen)
    mask = (torch.rand(B, N, generator=gen) > 0.25).float()
    mask[:, 0] = 1
    adj = (torch.rand(B, N, N, generator=gen) > 0.5).float()
    adj = ((adj + adj.transpose(1, 2)) > 0).float()
    adj = adj + torch.eye(N)
    adj = (adj > 0).float() * mask[:, :, None] * mask[:, None, :]
    x = x * mask[:, None, :, None]
    anom = torch.randn(B, T, Cin, generator=gen)
    anom_pos = torch.zeros(B, dtype=torch.long)
    W = torch.randn(Cin, F, generator=gen) * 0.5
    bb = torch.randn(F, generator=gen) * 0.1
    gamma = 1 + 0.1 * torch.randn(F, generator=gen)
    beta = 0.1 * torch.randn(F, generator=gen)
    alpha = 0.2 * torch.rand(F, generator=gen)
    return [t.to(dev) for t in (x, adj, mask, anom, anom_pos, W, bb, gamma, beta, alpha)]


@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("pooling", ["mean", "sum", "selection"])
def test_gcn_pool_matches_eager(cuda_device, training, pooling):
    from gnnqc.ops import gcn as G
    gen = torch.Generator().manual_seed(5)
    x, adj, mask, anom, ap, W, bb, gamma, beta, alpha = _gcn_inputs(gen, cuda_device)
    F = W.shape[1]
    rm_h, rv_h = torch.zeros(F, device=x.device), torch.ones(F, device=x.device)
    rm_e, rv_e = rm_h.clone(), rv_h.clone()
    if not training:
        rm_h.normal_(0, 0.1); rv_h.uniform_(0.5, 2.0)
        rm_e.copy_(rm_h); rv_e.copy_(rv_h)
    hp = [t.clone().requires_grad_(True) for t in (x, anom, W, bb, gamma, beta, alpha)]
    ep = [t.clone().double().requires_grad_(True) for t in (x, anom, W, bb, gamma, beta, alpha)]
    out = G._HipGCNPool.apply(hp[0], adj, mask, hp[1], ap.long().contiguous(), True,
                              {"mean": 0, "sum": 1, "selection": 2}[pooling], hp[2], hp[3], hp[4], hp[5], hp[6],
                              rm_h, rv_h, training, 0.99, 1e-3)
    h = G.general_conv_eager(ep[0], adj.double(), mask.double(), ep[2], ep[3], ep[4], ep[5], rm_e.double(),
                             rv_e.double(), ep[6], training, "mean")
    ref = torch.cat([ep[1], G.pool_nodes(h, mask.double(), ap, pooling)], -1)
    assert torch.allclose(out.double(), ref, atol=1e-4, rtol=1e-4), (out.double() - ref).abs().max()
    g = torch.randn(out.shape, generator=gen).to(x.device)
    out.backward(g)
    ref.backward(g.double())
    for p, r, name in zip(hp, ep, ["x", "anom", "W", "b", "gamma", "beta", "alpha"]):
        err = (p.grad.double() - r.grad).abs().max().item()
        assert err < 2e-3 * (1 + r.grad.abs().max().item()), f"{name}: {err}"
    if training:     # the fused prep's running-statistics update == the eager BatchNorm's
        z = torch.matmul(x.double(), W.double()) + bb.double()
        mm = mask.double()[:, None, :, None]
        n = mm.sum() * x.shape[1]
        mu = (z * mm).sum((0, 1, 2)) / n
        var = (((z - mu) ** 2) * mm).sum((0, 1, 2)) / n
        torch.testing.assert_close(rm_h.double(), 0.01 * mu, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(rv_h.double(), 0.99 + 0.01 * var, atol=1e-5, rtol=1e-4)


def test_gcn_prep_deterministic_and_eval_mode(cuda_device):
    """gcn_prep: bitwise-identical batch statistics on repeated launches (fixed-order record
    sums, no float atomics); eval mode preps BN from the running statistics untouched."""
    from gnnqc.utils.native import hip_ops
    gen = torch.Generator().manual_seed(9)
    x, adj, mask, anom, ap, W, bb, gamma, beta, alpha = _gcn_inputs(gen, cuda_device, B=40, T=30, N=11)
    F = W.shape[1]
    outs = []
    for _ in range(3):
        rm, rv = torch.zeros(F, device=x.device), torch.ones(F, device=x.device)
        w, S, st = hip_ops().gcn_prep(x, adj, mask, ap.long(), True, 0, W, bb, gamma, beta, rm, rv, True, 0.99, 1e-3)
        outs.append((w.clone(), S.clone(), st.clone(), rm.clone()))
    for o in outs[1:]:
        for a, b_ in zip(o, outs[0]):
            assert torch.equal(a, b_)
    rm, rv = torch.full((F,), 0.3, device=x.device), torch.full((F,), 2.0, device=x.device)
    w, S, st = hip_ops().gcn_prep(x, adj, mask, ap.long(), True, 0, W, bb, gamma, beta, rm, rv, False, 0.99, 1e-3)
    assert S.numel() == 0 and torch.all(rm == 0.3) and torch.all(rv == 2.0)
    torch.testing.assert_close(st[0], rm)
    torch.testing.assert_close(st[1], torch.rsqrt(rv + 1e-3))


def test_adam_kernel_matches_eager(cuda_device):
    from gnnqc.ops.optim import FlatAdam
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(37, 5)), torch.nn.Parameter(torch.randn(11))]
    ps_gpu = [torch.nn.Parameter(p.detach().clone().to(cuda_device)) for p in ps]
    a_cpu, a_gpu = FlatAdam(ps, 1e-2), FlatAdam(ps_gpu, 1e-2)
    for _ in range(5):
        g = torch.randn_like(a_cpu.flat_g)
        a_cpu.flat_g.copy_(g)
        a_gpu.flat_g.copy_(g.to(cuda_device))
        a_cpu.step(0.5)
        a_gpu.step(0.5)
    assert torch.allclose(a_cpu.flat_p, a_gpu.flat_p.cpu(), atol=1e-6)


def test_score_histogram_matches_eager(cuda_device):
    import gnnqc.ops.metrics as Mx
    torch.manual_seed(1)
    s = torch.rand(10000)
    y = (torch.rand(10000) > 0.8).float()
    m = (torch.rand(10000) > 0.1).float()
    ref = Mx.score_histogram(s, y, m, 1001)
    out = Mx.score_histogram(s.to(cuda_device), y.to(cuda_device), m.to(cuda_device), 1001)
    assert torch.equal(ref, out.cpu())


def test_window_gather_matches_torch(cuda_device, cml_windows):
    from gnnqc.data.store import DeviceStore
    from gnnqc.utils.native import hip_ops
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    st_cpu = DeviceStore(ws, "rolling_median", pc.graph, device="cpu")
    wids = torch.tensor([0, 5, -1, 17, st.n_windows - 1])
    ref = st_cpu.gather(wids)
    out = hip_ops().window_gather(st.series, st.shift, st.scale, st.win_group, st.win_center,
                                  st.win_valid_u8, wids.to(cuda_device), st.tb, st.seq_len, True)
    assert torch.allclose(out.cpu(), ref.x, atol=1e-5)
    b = st.gather(wids.to(cuda_device))
    assert torch.allclose(b.anom.cpu(), ref.anom, atol=1e-5)
    assert torch.equal(b.adj.cpu(), ref.adj)


def test_graph_captured_train_step_learns(cuda_device, cml_windows):
    from gnnqc import config as C
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, ws = cml_windows
    mc = C.default("model_cml")
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    torch.manual_seed(0)
    model = GCNClassifier(mc, pc).to(cuda_device)
    opt = make_optimizer("adam", model.parameters(), 1e-3)
    tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=True, batch_size=64)
    loader = DeviceLoader(st, list(range(st.n_windows)), 64, shuffle=True)
    losses = []
    for epoch in range(3):
        loader.set_epoch(epoch)
        for row in loader.batch_ids():
            losses.append(float(tr.train_step(row).item()))
    assert tr.graph is not None
    assert all(map(lambda v: v == v, losses))
    first = sum(losses[:5]) / 5
    last = sum(losses[-5:]) / 5
    assert last < first, (first, last)


@pytest.mark.gpu
@pytest.mark.parametrize("Fdim,R", [(128, 128), (64, 5), (32, 700), (128, 20000)])
def test_fused_head_loss_matches_eager(cuda_device, Fdim, R):
    """head_fwd/head_bwd vs the fp32 PyTorch head + weighted BCE + metric updates."""
    from gnnqc.models.layers import Dense
    from gnnqc.ops.head import fused_head_loss, head_eager
    from gnnqc.train.engine import HIST_BINS, MetricAccumulator
    from gnnqc.train.loss import weighted_bce_with_logits
    dev = cuda_device
    gen = torch.Generator().manual_seed(Fdim + R)
    layers = [Dense(Fdim, 64), Dense(64, 64), Dense(64, 1)]
    for d in layers:
        d.to(dev)
        with torch.no_grad():
            d.bias.normal_(0, 0.1)
    feat = (torch.randn(R, Fdim, generator=gen) * 0.7).to(dev).requires_grad_(True)
    y = (torch.rand(R, generator=gen) < 0.3).float().to(dev)
    mask = (torch.rand(R, generator=gen) < 0.9).float().to(dev)
    acc = MetricAccumulator(dev)
    loss, z = fused_head_loss(feat, *layers, 0.3, 0.3, y, mask, 1.0, 5.0, acc.sums, acc.hist)
    loss.backward()
    g_fused = [feat.grad.clone()] + [p.grad.clone() for d in layers for p in (d.kernel, d.bias)]
    feat.grad = None
    for d in layers:
        d.kernel.grad = d.bias.grad = None
    ref = MetricAccumulator(dev)
    zr = head_eager(feat, layers[0].kernel, layers[0].bias, layers[1].kernel, layers[1].bias, layers[2].kernel,
                    layers[2].bias, 0.3, 0.3)
    lr = weighted_bce_with_logits(zr, y, mask, 1.0, 5.0)
    lr.backward()
    ref.update(lr, zr, y, mask)
    g_ref = [feat.grad] + [p.grad for d in layers for p in (d.kernel, d.bias)]
    torch.testing.assert_close(z, zr.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(loss, lr.detach(), atol=1e-5, rtol=1e-4)
    for a, b in zip(g_fused, g_ref):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=2e-3)
    torch.testing.assert_close(acc.sums, ref.sums, atol=1e-3, rtol=1e-5)
    # histogram bins may differ by one where sigmoid implementations round differently
    assert float((acc.hist - ref.hist).abs().sum()) <= 0.002 * float(mask.sum()) + 2
    assert acc.hist.shape == (2, HIST_BINS)


@pytest.mark.gpu
def test_fused_head_direct_grad_accumulation(cuda_device):
    """In direct mode the head gradients land in the flat optimiser buffer (views)."""
    from gnnqc.models.layers import Dense
    from gnnqc.ops.head import fused_head_loss
    from gnnqc.ops.lstm import direct_grad_accumulation
    from gnnqc.ops.optim import FlatAdam
    dev = cuda_device
    layers = torch.nn.ModuleList([Dense(128, 64), Dense(64, 64), Dense(64, 1)]).to(dev)
    opt = FlatAdam(layers.parameters())
    feat = torch.randn(256, 128, device=dev)
    y = (torch.rand(256, device=dev) < 0.2).float()
    mask = torch.ones(256, device=dev)
    opt.zero_grad()
    loss, _ = fused_head_loss(feat, *layers, 0.3, 0.3, y, mask, 1.0, 5.0)
    with direct_grad_accumulation(True):
        loss.backward()
    direct = opt.flat_g.clone()
    opt.zero_grad()
    loss, _ = fused_head_loss(feat, *layers, 0.3, 0.3, y, mask, 1.0, 5.0)
    loss.backward()
    opt.relink_grads()
    torch.testing.assert_close(direct, opt.flat_g, atol=1e-6, rtol=1e-5)
    assert float(direct.abs().sum()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("M,T,C,p", [(50, 181, 16, 3), (7, 60, 32, 3), (3, 22, 128, 2), (5, 10, 64, 4),
                                     (1, 181, 4096, 3), (2, 37, 1100, 3), (1, 11, 2048, 1)])
def test_maxpool1d_matches_eager(cuda_device, M, T, C, p):
    from gnnqc.ops.pool import max_pool1d
    gen = torch.Generator().manual_seed(M * T + C)
    x = torch.randn(M, T, C, generator=gen).to(cuda_device).requires_grad_(True)
    y = max_pool1d(x, p)
    g = torch.randn(y.shape, generator=gen).to(cuda_device)
    (y * g).sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    To = T // p
    yr = xr[:, :To * p].reshape(M, To, p, C).max(2).values
    (yr * g).sum().backward()
    torch.testing.assert_close(y, yr, rtol=0, atol=0)
    torch.testing.assert_close(x.grad, xr.grad, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("aggregate", ["mean", "sum"])
@pytest.mark.parametrize("pooling", ["mean", "sum", "selection"])
def test_gcn_pool_weights_matches_eager(cuda_device, aggregate, pooling):
    from gnnqc.ops.gcn import node_pool_weights
    from gnnqc.utils.native import hip_ops
    gen = torch.Generator().manual_seed(7)
    B, N = 9, 23
    mask = (torch.rand(B, N, generator=gen) < 0.8).float()
    adj = (torch.rand(B, N, N, generator=gen) < 0.3).float()
    adj = ((adj + adj.transpose(1, 2) + torch.eye(N)) > 0).float() * mask[:, :, None] * mask[:, None, :]
    ap = torch.randint(0, N, (B,), generator=gen)
    adj, mask, ap = adj.to(cuda_device), mask.to(cuda_device), ap.to(cuda_device)
    ref = node_pool_weights(adj, mask, ap, aggregate, pooling)
    got = hip_ops().gcn_pool_weights(adj, mask, ap, aggregate == "mean",
                                     {"mean": 0, "sum": 1, "selection": 2}[pooling])
    torch.testing.assert_close(got, ref, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("H", [16, 32, 64])
@pytest.mark.parametrize("Din", [18, 16, 2, 32, 64])
@pytest.mark.parametrize("ret_seq", [True, False])
@pytest.mark.parametrize("wgrad", [True, False])
@pytest.mark.parametrize("in_rec", [False, True])
def test_lstm_time_major_fused_bwd_matches_eager(cuda_device, H, Din, ret_seq, wgrad, in_rec, monkeypatch):
    """lstm_tm_fwd / lstm_tm_bwd (recurrence + dx + fused dW/dU/db) vs fp64 eager. in_rec: the
    weight gradients inside the recurrence (lstm_tm_bwd_wg_kernel, H <= 32 with float4 x
    granules), else the separate weight-gradient pass."""
    from gnnqc.ops.lstm import lstm_eager, lstm_layer_tm, tm_eligible
    if in_rec and not (wgrad and H <= 32 and Din % 4 == 0):
        pytest.skip("the in-recurrence weight gradients take H <= 32, Din % 4 == 0")
    monkeypatch.setenv("GNNQC_TM_FUSED_WGRAD_MIN_TILES", "1" if in_rec else "100000")
    dev = cuda_device
    gen = torch.Generator().manual_seed(H * 100 + Din + 3 * ret_seq)
    M, T = 40, 13                     # 3 tiles (Mp = 48), T not a multiple of the ring depth
    x = torch.randn(M, T, Din, generator=gen).to(dev)
    if not tm_eligible(x, H, Din):
        pytest.skip("shape not handled by the time-major kernels")
    W, U, b = _lstm_params(Din, H, gen, dev)
    xt = torch.zeros(T, 48, Din, device=dev)
    xt[:, :M] = x.transpose(0, 1)
    xt.requires_grad_(True)
    Wp, Up, bp = (t.clone().requires_grad_(wgrad) for t in (W, U, b))
    out = lstm_layer_tm(xt, Wp, Up, bp, ret_seq)
    out_m = out[:, :M].transpose(0, 1) if ret_seq else out[:M]
    ref_params = [t.clone().double().requires_grad_(True) for t in (x, W, U, b)]
    ref = lstm_eager(*ref_params, return_sequences=ret_seq)
    assert torch.allclose(out_m.double(), ref, atol=3e-2, rtol=3e-2), (out_m.double() - ref).abs().max()
    g = torch.randn(ref.shape, generator=gen).to(dev)
    out_m.backward(g)
    ref.backward(g.double())
    got = [xt.grad[:, :M].transpose(0, 1)] + ([Wp.grad, Up.grad, bp.grad] if wgrad else [])
    for p, r, name in zip(got, ref_params, "xWUb"):
        err = (p.double() - r.grad).abs().max().item()
        scale = r.grad.abs().max().item() + 1e-6
        assert err / scale < 5e-2, f"grad {name}: rel err {err / scale}"
    assert float(xt.grad[:, M:].abs().max()) == 0.0          # padded rows get no gradient


@pytest.mark.parametrize("H", [16, 32])
@pytest.mark.parametrize("Din", [20, 32, 64])
@pytest.mark.parametrize("wgrad", [True, False])
@pytest.mark.parametrize("pair", [False, True])
def test_lstm_tm_recomputed_gates_match_saved_gates(cuda_device, monkeypatch, H, Din, wgrad, pair):
    """Recompute-gates backward (lstm_tm.hip RG: the forward saves only c, the backward recomputes
    i, f, g, o from x_t and h_{t-1}) vs the saved-gates form: identical forward output, gradients
    within bf16-gate rounding of each other, and the RG gradients against an fp64 eager oracle."""
    from gnnqc.ops import lstm as L
    from gnnqc.utils.native import hip_ops
    monkeypatch.setattr(L._Pipe, "enabled", False)      # (training layers of any size take RG)
    dev = cuda_device
    gen = torch.Generator().manual_seed(7 * H + Din + 100 * wgrad + 1000 * pair)
    M, T, Mp = 72, 37, 80
    x = torch.zeros(T, Mp, Din)
    x[:, :M] = torch.randn(T, M, Din, generator=gen)
    x = x.to(dev)
    WA, UA, bA = _lstm_params(Din, H, gen, dev)
    WB, UB, bB = _lstm_params(H, H, gen, dev)
    dout = torch.randn(T, Mp, H, generator=gen).to(dev)
    dout[:, M:] = 0
    _, g_rg, c_rg = hip_ops().lstm_tm_fwd(x, WA, UA, bA, True, False)
    assert g_rg.numel() == 0 and c_rg.numel() == (T + 1) * Mp * H

    def run(rg):
        monkeypatch.setenv("GNNQC_TM_RG", "1" if rg else "0")
        xi = x.clone().requires_grad_(True)
        ps = [t.clone().requires_grad_(wgrad) for t in ((WA, UA, bA, WB, UB, bB) if pair else (WA, UA, bA))]
        out = L._HipLSTMTMPair.apply(xi, *ps) if pair else L.lstm_layer_tm(xi, *ps, True)
        out.backward(dout)
        return out.detach(), [xi.grad] + ([p.grad for p in ps] if wgrad else [])

    o0, g0 = run(False)
    o1, g1 = run(True)
    # the forward arithmetic is unchanged (the two template instances may differ in the compiler's
    # contraction choices only: last-bit differences)
    torch.testing.assert_close(o1, o0, atol=1e-5, rtol=1e-5)
    for a, b_ in zip(g1, g0):
        assert (a - b_).norm().item() <= 2e-2 * (b_.norm().item() + 1e-6)
    # fp64 oracle of the RG gradients
    ref_in = [x[:, :M].transpose(0, 1).double().clone().requires_grad_(True)]
    ref_ps = [t.double().clone().requires_grad_(True) for t in ((WA, UA, bA, WB, UB, bB) if pair else (WA, UA, bA))]
    h = L.lstm_eager(ref_in[0], *ref_ps[:3], return_sequences=True)
    if pair:
        h = L.lstm_eager(h, *ref_ps[3:], return_sequences=True)
    h.backward(dout[:, :M].transpose(0, 1).double())
    got = [g1[0][:, :M].transpose(0, 1)] + (g1[1:] if wgrad else [])
    refs = [ref_in[0].grad] + ([p.grad for p in ref_ps] if wgrad else [])
    for a, r in zip(got, refs):
        err = (a.double() - r).abs().max().item() / (r.abs().max().item() + 1e-6)
        assert err < 5e-2, err
    assert float(g1[0][:, M:].abs().max()) == 0.0


@pytest.mark.parametrize("M,frozen", [(300, False), (700, False), (300, True)])
def test_timelayer_fused_pool_unpool_on_load_matches_separate_pool(cuda_device, monkeypatch, M, frozen):
    """MaxPooling1D fused into the preceding time-major layer (pair)'s autograd node, the backward
    recurrence un-pooling the pooled gradient on load (lstm_tm_bwd pidx / pool), vs separate
    maxpool1d kernels: same output, same input / weight gradients (identical arithmetic). ``frozen``:
    input gradients only (the integrated-gradients path)."""
    from gnnqc.models.timelayer import TimeLayer
    torch.manual_seed(0)
    tl = TimeLayer(20, 16, 2, "lstm", pool_size=3).to(cuda_device)
    for p in tl.parameters():
        p.requires_grad_(not frozen)
    x = torch.randn(M, 181, 20, device=cuda_device)
    monkeypatch.setenv("GNNQC_CHAIN", "0")

    def run(fuse):
        monkeypatch.setenv("GNNQC_TM_POOL_FUSE", "1" if fuse else "0")
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        out = tl(xi)
        out.pow(2).sum().backward()
        return out.detach(), [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters() if p.requires_grad]

    o0, g0 = run(False)
    o1, g1 = run(True)
    torch.testing.assert_close(o1, o0, atol=1e-5, rtol=1e-4)
    for a, b_ in zip(g1, g0):
        assert (a - b_).norm().item() <= 1e-3 * (b_.norm().item() + 1e-6)


@pytest.mark.parametrize("H,P,T", [(16, 3, 181), (32, 3, 60), (16, 2, 37), (32, 1, 12)])
def test_lstm_tm2_fwd_in_kernel_pool_matches_maxpool(cuda_device, H, P, T):
    """MaxPooling1D(P) of layer B's output by the pair kernel's storer lanes (lstm_tm2_fwd pool=P)
    == maxpool1d_fwd over the stored hB: pooled values and argmax bytes, bitwise; hA / hB unchanged."""
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    gen = torch.Generator().manual_seed(H * 10 + P + T)
    Mp, Din = 48, 20
    x = torch.randn(T, Mp, Din, generator=gen).to(cuda_device)
    WA, UA, bA = _lstm_params(Din, H, gen, cuda_device)
    WB, UB, bB = _lstm_params(H, H, gen, cuda_device)
    r0 = ops.lstm_tm2_fwd(x, WA, UA, bA, WB, UB, bB, True, False, 0)
    r1 = ops.lstm_tm2_fwd(x, WA, UA, bA, WB, UB, bB, True, False, P)
    assert torch.equal(r0[0], r1[0]) and torch.equal(r0[3], r1[3])
    ref, ridx = ops.maxpool1d_fwd(r0[3].contiguous().view(1, T, Mp * H), P)
    assert torch.equal(r1[6].view(1, T // P, Mp * H), ref)
    assert torch.equal(r1[7].view(1, T // P, Mp * H), ridx)


def test_timelayer_time_major_matches_sequence_major(cuda_device, monkeypatch):
    """The CML TimeLayer (LSTM 16,16 | pool | 32,32 | pool | 64,64 | pool | 128): time-major
    fused path vs the sequence-major kernels - forward and every parameter gradient."""
    from gnnqc.models.timelayer import TimeLayer
    from gnnqc.ops.lstm import direct_grad_accumulation
    from gnnqc.ops.optim import FlatAdam
    torch.manual_seed(0)
    tl = TimeLayer(18, 16, 2, "lstm", pool_size=3).to(cuda_device)
    x = torch.randn(128, 181, 18, device=cuda_device)

    def run(no_tm, direct):
        monkeypatch.setenv("GNNQC_NO_TM", "1" if no_tm else "0")
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        opt = FlatAdam(tl.parameters()) if direct else None
        out = tl(xi)
        with direct_grad_accumulation(direct):
            out.pow(2).sum().backward()
        if opt is not None:
            opt.relink_grads()
        return out.detach(), xi.grad.clone(), [p.grad.clone() for p in tl.parameters()]

    o1, dx1, g1 = run(True, False)
    o2, dx2, g2 = run(False, False)
    o3, dx3, g3 = run(False, True)
    torch.testing.assert_close(o2, o1, atol=2e-2, rtol=2e-2)
    for a, b_ in zip([dx2] + g2, [dx1] + g1):
        err = (a - b_).abs().max().item() / (b_.abs().max().item() + 1e-6)
        assert err < 6e-2, err
    for a, b_ in zip([dx3] + g3, [dx2] + g2):
        torch.testing.assert_close(a, b_, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("k,cin,cout,T,gap", [(5, 18, 16, 181, False), (3, 16, 32, 60, False), (5, 32, 64, 20, False),
                                              (5, 64, 128, 6, True), (1, 7, 16, 13, False), (4, 16, 16, 9, True),
                                              (7, 3, 24, 50, False), (3, 120, 128, 40, False), (3, 120, 100, 300, True)])
def test_conv1d_act_matches_eager(cuda_device, k, cin, cout, T, gap):
    """Fused Conv1D(same)+LeakyReLU(+GAP) HIP kernels vs fp64 eager: output, dx, dW, db."""
    from gnnqc.ops.conv import conv1d_act, conv1d_act_eager, hip_conv_supported
    assert hip_conv_supported(k, cin, cout)
    gen = torch.Generator().manual_seed(k * 1000 + cin * 10 + cout)
    M = 37
    x = torch.randn(M, T, cin, generator=gen)
    W = torch.randn(k, cin, cout, generator=gen) * (1.0 / (k * cin) ** 0.5)
    b = torch.randn(cout, generator=gen) * 0.1
    xs = [t.to(cuda_device).requires_grad_(True) for t in (x, W, b)]
    out = conv1d_act(*xs, alpha=0.3, gap=gap)
    ref_in = [t.double().requires_grad_(True) for t in (x, W, b)]
    ref = conv1d_act_eager(*ref_in, alpha=0.3, gap=gap)
    assert out.shape == ref.shape
    err = (out.double().cpu() - ref).abs().max().item()
    assert err < 3e-2 * (ref.abs().max().item() + 1e-3), err
    # backward: the reference uses the kernel's own LeakyReLU gate (sign of its bf16 z), since
    # a z within rounding of 0 may flip sign between bf16 and fp64 and change dz by (1-alpha) dy
    with torch.no_grad():
        z_gpu = conv1d_act(*(t.detach() for t in xs), alpha=1.0, gap=False)
    gate = torch.where(z_gpu.double().cpu() > 0, 1.0, 0.3)
    lin = conv1d_act_eager(*ref_in, alpha=1.0, gap=False) * gate
    ref_b = lin.mean(1) if gap else lin
    g = torch.randn(ref.shape, generator=gen)
    out.backward(g.to(cuda_device))
    ref_b.backward(g.double())
    for got, r, name in zip(xs, ref_in, ("x", "W", "b")):
        e = (got.grad.double().cpu() - r.grad).abs().max().item()
        scale = r.grad.abs().max().item() + 1e-6
        assert e / scale < 3e-2, f"grad {name}: rel err {e / scale}"


def test_timelayer_cnn_branch_hip_vs_eager(cuda_device, monkeypatch):
    """CNN TimeLayer: fused HIP conv kernels vs the eager path on the same weights."""
    from gnnqc.models.timelayer import TimeLayer
    torch.manual_seed(0)
    tl = TimeLayer(18, 16, 2, "cnn", kernel_size=5, pool_size=3).to(cuda_device)
    x = torch.randn(64, 181, 18, device=cuda_device)

    def run(eager):
        monkeypatch.setenv("GNNQC_FORCE_EAGER", "1" if eager else "0")
        for p in tl.parameters():
            p.grad = None
        out = tl(x)
        out.pow(2).sum().backward()
        return out.detach(), [p.grad.detach().clone() for p in tl.parameters()]

    o1, g1 = run(False)
    o0, g0 = run(True)
    assert o1.shape == o0.shape == (64, 128)
    # relative Frobenius errors: isolated LeakyReLU gate flips (bf16 vs fp32 z near 0) are sparse
    assert (o1 - o0).norm().item() < 2e-2 * o0.norm().item()
    for a, b in zip(g1, g0):
        assert (a - b).norm().item() < 5e-2 * (b.norm().item() + 1e-6)


@pytest.mark.parametrize("H", [16, 32])
@pytest.mark.parametrize("wgrad", [True, False])
@pytest.mark.parametrize("in_rec", [False, True])
def test_lstm_time_major_padded_channels(cuda_device, H, wgrad, in_rec, monkeypatch):
    """x with zero channels past W's rows (19 -> 20, float4 loader granules) == unpadded eager;
    in_rec: weight gradients inside the recurrence (the bias row sits inside the last x granule)."""
    from gnnqc.ops.lstm import lstm_eager, lstm_layer_tm
    if in_rec and not wgrad:
        pytest.skip("in-recurrence weight gradients need wgrad")
    monkeypatch.setenv("GNNQC_TM_FUSED_WGRAD_MIN_TILES", "1" if in_rec else "100000")
    dev = cuda_device
    gen = torch.Generator().manual_seed(H + 11)
    M, T, Din = 37, 14, 19
    x = torch.randn(M, T, Din, generator=gen).to(dev)
    W, U, b = _lstm_params(Din, H, gen, dev)
    xt = torch.zeros(T, 48, 20, device=dev)
    xt[:, :M, :Din] = x.transpose(0, 1)
    xt.requires_grad_(True)
    Wp, Up, bp = (t.clone().requires_grad_(wgrad) for t in (W, U, b))
    out = lstm_layer_tm(xt, Wp, Up, bp, True)
    out_m = out[:, :M].transpose(0, 1)
    ref_params = [t.clone().double().requires_grad_(True) for t in (x, W, U, b)]
    ref = lstm_eager(*ref_params)
    assert torch.allclose(out_m.double(), ref, atol=3e-2, rtol=3e-2), (out_m.double() - ref).abs().max()
    g = torch.randn(ref.shape, generator=gen).to(dev)
    out_m.backward(g)
    ref.backward(g.double())
    got = [xt.grad[:, :M, :Din].transpose(0, 1)] + ([Wp.grad, Up.grad, bp.grad] if wgrad else [])
    for p, r, name in zip(got, ref_params, "xWUb"):
        err = (p.double() - r.grad).abs().max().item()
        scale = r.grad.abs().max().item() + 1e-6
        assert err / scale < 5e-2, f"grad {name}: rel err {err / scale}"
    assert float(xt.grad[..., Din:].abs().max()) == 0.0        # padding channel: no gradient


def _soil_graph(B, N, gen, dev):
    """Random symmetric radius-like graphs with self loops and padded (masked) nodes."""
    n_valid = [N - 3 * b for b in range(B)]
    adj = torch.zeros(B, N, N)
    mask = torch.zeros(B, N)
    for b, nv in enumerate(n_valid):
        mask[b, :nv] = 1
        a = (torch.rand(nv, nv, generator=gen) < 0.12).float()
        a = ((a + a.t()) > 0).float()
        a.fill_diagonal_(1.0)
        adj[b, :nv, :nv] = a
    return adj.to(dev), mask.to(dev)


@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("aggregate", ["mean", "sum"])
@pytest.mark.parametrize("F", [16, 2])      # 16: 4-channel vector gather path, 2: scalar path
def test_gcn_node_tm_matches_eager(cuda_device, training, aggregate, F):
    """Per-node GeneralConv kernel (SoilNet): time-major output and every gradient vs fp64 eager."""
    from gnnqc.ops.gcn import gcn_node_tm, gcn_node_tm_eager
    dev = cuda_device
    gen = torch.Generator().manual_seed(5 + training + 2 * (aggregate == "sum"))
    B, T, N, Cin = 3, 9, 45, 3
    adj, mask = _soil_graph(B, N, gen, dev)
    x = (torch.randn(B, T, N, Cin, generator=gen).to(dev)) * mask[:, None, :, None]
    W = (torch.randn(Cin, F, generator=gen) * 0.5).to(dev)
    b = (torch.randn(F, generator=gen) * 0.1).to(dev)
    gamma = (1 + 0.1 * torch.randn(F, generator=gen)).to(dev)
    beta = (0.1 * torch.randn(F, generator=gen)).to(dev)
    alpha = (0.2 * torch.rand(F, generator=gen)).to(dev)
    rm0 = (0.1 * torch.randn(F, generator=gen)).to(dev)
    rv0 = (1 + 0.1 * torch.rand(F, generator=gen)).to(dev)
    ps = [t.clone().requires_grad_(True) for t in (x, W, b, gamma, beta, alpha)]
    rps = [t.clone().double().requires_grad_(True) for t in (x, W, b, gamma, beta, alpha)]
    rm, rv, rrm, rrv = rm0.clone(), rv0.clone(), rm0.clone().double(), rv0.clone().double()
    h, M = gcn_node_tm(ps[0], adj, mask, *ps[1:5], ps[5], rm, rv, training, aggregate)
    ref, Mr = gcn_node_tm_eager(rps[0], adj.double(), mask.double(), *rps[1:5], rps[5], rrm, rrv, training,
                                aggregate)
    assert M == Mr and h.shape == ref.shape, (h.shape, ref.shape)
    torch.testing.assert_close(h.double(), ref, atol=2e-4, rtol=2e-4)
    torch.testing.assert_close(rm.double(), rrm, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rv.double(), rrv, atol=1e-5, rtol=1e-5)
    g = torch.randn(ref.shape, generator=gen).to(dev)
    g[:, M:] = 0
    h.backward(g)
    ref.backward(g.double())
    for p, r, name in zip(ps, rps, ("x", "W", "b", "gamma", "beta", "alpha")):
        if r.grad is None:
            continue
        err = (p.grad.double() - r.grad).abs().max().item()
        scale = r.grad.abs().max().item() + 1e-6
        assert err / scale < 1e-3, f"grad {name}: rel err {err / scale}"


def test_soilnet_gcn_fused_path_matches_eager(cuda_device, monkeypatch):
    """SoilNet GCNClassifier: fused GCN + time-major LSTM kernels vs the same model in float64 on
    the CPU with the LSTM rounded where the kernels round (gnnqc/ops/lstm_ref.py): logits and
    every gradient within 8e-3 (rounding explains the rest)."""
    import copy

    from gnnqc import config as C
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.lstm_ref import kernel_rounding
    torch.manual_seed(0)
    pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
    mc = C.default("model_soilnet")
    model = GCNClassifier(mc, pc).to(cuda_device)
    gen = torch.Generator().manual_seed(1)
    B, T, N = 4, 337, 29
    adj, mask = _soil_graph(B, N, gen, cuda_device)
    x = torch.rand(B, T, N, 3, generator=gen).to(cuda_device) * mask[:, None, :, None]
    inputs = (x, adj, mask)
    assert model._soil_fused(inputs)
    ref = copy.deepcopy(model).cpu().double()
    for p in model.parameters():
        p.grad = None
    z1 = model.logits(inputs)
    (z1 * mask).pow(2).sum().backward()
    g1 = {k: p.grad.detach().double().cpu() for k, p in model.named_parameters() if p.grad is not None}
    ri = [t.double().cpu() for t in inputs]
    with kernel_rounding():
        z0 = ref.logits(ri)
        (z0 * ri[2]).pow(2).sum().backward()
    g0 = {k: p.grad.detach() for k, p in ref.named_parameters() if p.grad is not None}
    z1 = z1.detach().double().cpu()
    assert z1.shape == z0.shape == (B, N)
    assert (z1 - z0.detach()).norm().item() < 3e-3 * z0.norm().item()
    assert set(g1) == set(g0)
    for k in g0:
        err = (g1[k] - g0[k]).norm().item()
        assert err < 8e-3 * (g0[k].norm().item() + 1e-6), (k, err, g0[k].norm().item())


@pytest.mark.parametrize("H,Din", [(16, 20), (16, 16), (32, 16), (32, 32)])
@pytest.mark.parametrize("wgrad", [True, False])
def test_lstm_pair_fused_forward_matches_two_layers(cuda_device, H, Din, wgrad):
    """lstm_tm2_fwd (layer pair, pipelined kernel) + per-layer backward == two single layers, incl. gradients."""
    from gnnqc.ops.lstm import _HipLSTMTMPair, lstm_layer_tm
    dev = cuda_device
    gen = torch.Generator().manual_seed(H * 7 + Din)
    T, M = 23, 40
    x = torch.zeros(T, 48, Din, device=dev)
    x[:, :M, : Din - 1] = torch.randn(T, M, Din - 1, generator=gen).to(dev)   # last channel: zero pad
    WA, UA, bA = _lstm_params(Din - 1 if Din == 20 else Din, H, gen, dev)
    WB, UB, bB = _lstm_params(H, H, gen, dev)
    ps1 = [t.clone().requires_grad_(wgrad) for t in (WA, UA, bA, WB, UB, bB)]
    ps2 = [t.clone().requires_grad_(wgrad) for t in (WA, UA, bA, WB, UB, bB)]
    x1 = x.clone().requires_grad_(True)
    x2 = x.clone().requires_grad_(True)
    out1 = _HipLSTMTMPair.apply(x1, *ps1)
    out2 = lstm_layer_tm(lstm_layer_tm(x2, *ps2[:3], True), *ps2[3:], True)
    # same bf16 operands and accumulation order, but the compiler may contract the fp32 cell
    # update differently in the two kernels: a 1-ulp difference can flip a bf16 rounding of h
    torch.testing.assert_close(out1, out2, atol=2e-3, rtol=1e-2)
    g = torch.randn(out1.shape, generator=gen).to(dev)
    g[:, M:] = 0
    out1.backward(g)
    out2.backward(g)
    for a, b_ in zip([x1.grad] + ([p.grad for p in ps1] if wgrad else []),
                     [x2.grad] + ([p.grad for p in ps2] if wgrad else [])):
        assert (a - b_).norm().item() <= 1e-2 * (b_.norm().item() + 1e-6)


def test_timelayer_pair_fusion_matches_unfused(cuda_device, monkeypatch):
    """CML TimeLayer: pair-fused forward vs per-layer kernels (outputs and all gradients)."""
    from gnnqc.models.timelayer import TimeLayer
    torch.manual_seed(0)
    tl = TimeLayer(18, 16, 2, "lstm", pool_size=3).to(cuda_device)
    x = torch.randn(128, 181, 18, device=cuda_device)

    monkeypatch.setenv("GNNQC_CHAIN", "0")

    def run(no_pair):
        monkeypatch.setenv("GNNQC_NO_PAIR", "1" if no_pair else "0")
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        out = tl(xi)
        out.pow(2).sum().backward()
        return out.detach(), [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters()]

    o0, g0 = run(True)
    o1, g1 = run(False)
    torch.testing.assert_close(o1, o0, atol=2e-3, rtol=1e-2)
    for a, b_ in zip(g1, g0):
        assert (a - b_).norm().item() <= 2e-2 * (b_.norm().item() + 1e-6)


@pytest.mark.parametrize("bwd", ["chain", "per_layer"])
@pytest.mark.parametrize("M", [128, 40, 300])
def test_chain_forward_matches_per_layer(cuda_device, monkeypatch, M, bwd):
    """CML TimeLayer: the cross-CU pipelined stack forward (lstm_chain.hip) == the per-layer
    kernels (no pair fusion) for the output and every gradient; repeated launches (fresh
    epochs over reused stream buffers) stay identical and no consumer spin timed out."""
    from gnnqc.models.timelayer import TimeLayer
    from gnnqc.utils.native import hip_ops
    torch.manual_seed(0)
    tl = TimeLayer(18, 16, 2, "lstm", pool_size=3).to(cuda_device)
    x = torch.randn(M, 181, 18, device=cuda_device)
    monkeypatch.setenv("GNNQC_NO_PAIR", "1")
    monkeypatch.setenv("GNNQC_CHAIN_BWD", "1" if bwd == "chain" else "0")

    def run(chain):
        monkeypatch.setenv("GNNQC_CHAIN", "1" if chain else "0")
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        out = tl(xi)
        out.pow(2).sum().backward()
        return out.detach(), [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters()]

    seq = tl._sequence()
    h = torch.zeros(181, (M + 15) // 16 * 16, 20, device=cuda_device)
    plan = tl._chain_plan(seq, h)
    assert plan is not None and len(plan[0]) == 6 and plan[1] == [0, 3, 0, 3, 0, 3]
    st0 = hip_ops().lstm_chain_status(x).cpu()
    o0, g0 = run(False)
    o1, g1 = run(True)
    outs = [tl(x).detach() for _ in range(4)]
    torch.cuda.synchronize()
    st1 = hip_ops().lstm_chain_status(x).cpu()
    assert int(st1[2]) == 0, "a consumer spin timed out"
    assert int(st1[0]) - int(st0[0]) == (6 if bwd == "chain" else 5) and int(st1[1]) == 0, (st0, st1)
    torch.testing.assert_close(o1, o0, atol=1e-5, rtol=1e-5)
    for o in outs:
        assert torch.equal(o, o1)
    for a, b_ in zip(g1, g0):     # (bf16 rounding flips of near-tie values move gradients ~1e-3)
        assert (a - b_).norm().item() <= 5e-3 * (b_.norm().item() + 1e-6)


@pytest.mark.parametrize("P", [1, 2])
def test_chain_odd_pool_size_matches_per_layer(cuda_device, monkeypatch, P):
    """A chain that ends in MaxPooling1D(P != 3) (``_chain_plan`` accepts 1..255): forward and
    chain backward == the per-layer kernels. P = 1 guards the un-pooling stage's multiply-high
    division (its magic 2^32 wraps to 0, which once sent every dh to source step 0)."""
    from gnnqc.models.timelayer import TimeLayer
    from gnnqc.utils.native import hip_ops
    torch.manual_seed(0)
    tl = TimeLayer(18, 16, 2, "lstm", pool_size=P).to(cuda_device)
    x = torch.randn(64, 181, 18, device=cuda_device)
    monkeypatch.setenv("GNNQC_NO_PAIR", "1")
    monkeypatch.setenv("GNNQC_CHAIN_BWD", "1")
    h = torch.zeros(181, 64, 20, device=cuda_device)
    plan = tl._chain_plan(tl._sequence(), h)
    assert plan is not None and plan[1] == [0, P], plan

    def run(chain):
        monkeypatch.setenv("GNNQC_CHAIN", "1" if chain else "0")
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        out = tl(xi)
        out.pow(2).sum().backward()
        return out.detach(), [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters()]

    o0, g0 = run(False)
    o1, g1 = run(True)
    torch.cuda.synchronize()
    assert int(hip_ops().lstm_chain_status(x).cpu()[2]) == 0, "a consumer spin timed out"
    torch.testing.assert_close(o1, o0, atol=1e-5, rtol=1e-5)
    for a, b_ in zip(g1, g0):
        assert (a - b_).norm().item() <= 5e-3 * (b_.norm().item() + 1e-6)


def _soil_small_windows():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.synthetic import make_soilnet_raw
    pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
    raw = make_soilnet_raw(n_boxes=6, n_time=10 * 96, seed=2)
    pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    return pc, create_windows_dataset(pc, raw=raw)


@pytest.mark.parametrize("ds", ["cml", "soilnet"])
def test_batch_meta_matches_torch_gather(cuda_device, cml_windows, ds):
    """Fused batch assembly (window_gather + batch_meta) == the eager gather, every field."""
    from gnnqc.data.store import DeviceStore
    pc, ws = cml_windows if ds == "cml" else _soil_small_windows()
    norm = "rolling_median" if ds == "cml" else "scale_range"
    st = DeviceStore(ws, norm, pc.graph, device=cuda_device)
    st_cpu = DeviceStore(ws, norm, pc.graph, device="cpu")
    n = st.n_windows
    wids = torch.tensor([0, min(5, n - 1), -1, n // 2, n - 1])
    vs = torch.tensor([1.0, 0.0, 1.0, 1.0, 1.0])
    for valid_sample in (None, vs):
        ref = st_cpu.gather(wids, valid_sample)
        got = st.gather(wids.to(cuda_device), None if valid_sample is None else valid_sample.to(cuda_device))
        for name in ("x", "adj", "node_mask", "anom", "anom_pos", "y", "y_mask", "wid"):
            a, b_ = getattr(got, name), getattr(ref, name)
            if b_ is None:
                assert a is None, name
                continue
            assert a.shape == b_.shape and a.dtype == b_.dtype, (name, a.shape, b_.shape, a.dtype, b_.dtype)
            assert torch.allclose(a.cpu().double(), b_.double(), atol=1e-5), name


@pytest.mark.parametrize("use_graph", [True, False])
def test_pipe_training_steps_match_fused(cuda_device, cml_windows, monkeypatch, use_graph):
    """Training steps with the deferred, batched weight-gradient passes (the pipe) == the same
    steps with one fused backward kernel per layer."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.lstm import _Pipe
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, ws = cml_windows
    mc = C.default("model_cml")
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)

    def run(side):
        monkeypatch.setattr(_Pipe, "enabled", bool(side))
        torch.manual_seed(0)
        model = GCNClassifier(mc, pc).to(cuda_device)
        opt = make_optimizer("adam", model.parameters(), 1e-3)
        tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=use_graph, batch_size=64)
        loader = DeviceLoader(st, list(range(st.n_windows)), 64, shuffle=True)
        for row in list(loader.batch_ids())[:6]:
            tr.train_step(row)
        torch.cuda.synchronize()
        return torch.cat([p.detach().reshape(-1) for p in model.parameters()]), float(tr.last_loss.item())

    p1, l1 = run(True)
    p0, l0 = run(False)
    assert abs(l1 - l0) < 2e-2 * abs(l0) + 1e-4, (l1, l0)
    assert (p1 - p0).norm().item() < 2e-3 * p0.norm().item()


@pytest.mark.parametrize("ds", ["cml", "soilnet"])
def test_pipe_lstm_backward_gradients(cuda_device, cml_windows, monkeypatch, ds):
    """One backward with the pipelined LSTM backward (weight-gradient passes fused behind the
    next layer's recurrence, flushed at context exit) == the fused per-layer backward, for
    every parameter gradient."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.lstm import _Pipe, direct_grad_accumulation
    pc, ws = cml_windows if ds == "cml" else _soil_small_windows()
    st = DeviceStore(ws, "rolling_median" if ds == "cml" else "scale_range", pc.graph, device=cuda_device)
    torch.manual_seed(0)
    model = GCNClassifier(C.default(f"model_{ds}"), pc).to(cuda_device)
    b = st.gather(torch.arange(min(40, st.n_windows), device=cuda_device))
    inputs = b.model_inputs(ds, False)

    def run(mode):
        monkeypatch.setattr(_Pipe, "enabled", mode == "pipe")
        for p in model.parameters():
            p.grad = torch.zeros_like(p)
        with direct_grad_accumulation(True):
            model.logits(inputs).float().square().mean().backward()
        assert _Pipe.job is None and _Pipe.red is None and not _Pipe.batch
        torch.cuda.synchronize()
        return [p.grad.clone() for p in model.parameters()]

    g0, g1 = run("fused"), run("pipe")
    for (n, _), a, r in zip(model.named_parameters(), g1, g0):
        assert (a - r).norm().item() <= 1e-4 * r.norm().item() + 1e-7, n


def test_cml_time_major_gcn_output_matches_batch_major(cuda_device, cml_windows, monkeypatch):
    """CML GCN: kernel-written time-major LSTM input == batch-major kernel output + transpose/pad,
    for logits, every parameter gradient and the input gradients (integrated gradients)."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    torch.manual_seed(0)
    model = GCNClassifier(C.default("model_cml"), pc).to(cuda_device)
    b = st.gather(torch.arange(40, device=cuda_device))

    def run(tm):
        monkeypatch.setattr(GCNClassifier, "_cml_time_major",
                            (lambda self, i: GCNClassifier.__dict__["_cml_time_major_orig"](self, i)) if tm
                            else (lambda self, i: False))
        for p in model.parameters():
            p.grad = None
        x = b.x.clone().requires_grad_(True)
        anom = b.anom.clone().requires_grad_(True)
        z = model.logits((x, anom, b.adj, b.node_mask, b.anom_pos))
        z.pow(2).sum().backward()
        return [z.detach(), x.grad, anom.grad] + [p.grad.clone() for p in model.parameters()]

    monkeypatch.setattr(GCNClassifier, "_cml_time_major_orig", GCNClassifier._cml_time_major, raising=False)
    assert model._cml_time_major((b.x, b.anom, b.adj, b.node_mask, b.anom_pos))
    r1 = run(True)
    r0 = run(False)
    for a, b_ in zip(r1, r0):
        assert (a - b_).norm().item() <= 1e-4 * (b_.norm().item() + 1e-6)


@pytest.mark.parametrize("use_graph", [True, False])
def test_split_optimizer_graph_matches_fused(cuda_device, cml_windows, monkeypatch, use_graph):
    """The data-parallel step layout (forward/backward graph, then a separate optimizer graph
    replayed after the all-reduce) gives the same parameters as the one-graph step."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, ws = cml_windows
    mc = C.default("model_cml")
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)

    def run(split):
        monkeypatch.setenv("GNNQC_SPLIT_OPT_GRAPH", "1" if split else "0")
        torch.manual_seed(0)
        model = GCNClassifier(mc, pc).to(cuda_device)
        opt = make_optimizer("adam", model.parameters(), 1e-3)
        tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, use_graph=use_graph, batch_size=64)
        assert tr.split_opt == split
        loader = DeviceLoader(st, list(range(st.n_windows)), 64, shuffle=True)
        for row in list(loader.batch_ids())[:6]:
            tr.train_step(row)
        torch.cuda.synchronize()
        assert (tr.opt_graph is not None) == (split and use_graph)
        assert opt.iterations == 6 and float(opt.step_t.item()) == 6.0
        return torch.cat([p.detach().reshape(-1) for p in model.parameters()]), float(tr.last_loss.item())

    # bitwise-reproducible kernels: the default store-fused GCN backward sums with atomics, and
    # Adam amplifies that run-to-run noise on near-zero gradients (two runs of the SAME layout
    # differ by ~1e-3 of the parameter norm after 6 steps), which would hide a layout difference
    from gnnqc.ops import set_deterministic
    prev = set_deterministic(True)
    try:
        p1, l1 = run(True)
        p0, l0 = run(False)
    finally:
        set_deterministic(prev)
    assert abs(l1 - l0) < 1e-5 * abs(l0) + 1e-6, (l1, l0)
    assert (p1 - p0).norm().item() < 1e-6 * p0.norm().item()


@pytest.mark.parametrize("Din,Dw,T,wgrad", [(64, 64, 6, True), (64, 64, 6, False), (32, 28, 1, True),
                                            (64, 60, 16, False), (16, 16, 3, True)])
def test_time4_standalone_last_state_matches_fp64_oracle(cuda_device, Din, Dw, T, wgrad):
    """time4 (H = 128, last state) as a standalone time-major layer (time4_fwd / time4_bwd: compact
    saved state, workgroups looping over tiles) vs an fp64 eager LSTM: last state, input gradient
    (zero past the W rows and on padded rows) and weight gradients (dz -> lstm_tm_grads)."""
    from gnnqc.ops import lstm as L
    dev = cuda_device
    gen = torch.Generator().manual_seed(Din * 100 + Dw + T + 7 * wgrad)
    M, Mp = 72, 80
    x = torch.zeros(T, Mp, Din)
    x[:, :M] = torch.randn(T, M, Din, generator=gen)
    x = x.to(dev)
    W, U, b = _lstm_params(Dw, 128, gen, dev)
    U = U * 0.5
    dout = torch.randn(Mp, 128, generator=gen).to(dev)
    dout[M:] = 0
    xi = x.clone().requires_grad_(True)
    ps = [t.clone().requires_grad_(wgrad) for t in (W, U, b)]
    out = L._HipLSTMLast128.apply(xi, *ps)
    assert out.shape == (Mp, 128)
    out.backward(dout)
    rx = x[:, :M, :Dw].transpose(0, 1).double().clone().requires_grad_(True)
    rps = [t.double().clone().requires_grad_(True) for t in (W, U, b)]
    ref = L.lstm_eager(rx, *rps, return_sequences=False)
    ref.backward(dout[:M].double())
    err = (out[:M].double() - ref).abs().max().item()
    assert err < 3e-2, err                         # (bf16 MFMA operands, as the other bf16 LSTM tests)
    got = [xi.grad[:, :M, :Dw].transpose(0, 1)] + ([p.grad for p in ps] if wgrad else [])
    refs = [rx.grad] + ([p.grad for p in rps] if wgrad else [])
    for name, a, r in zip("xWUb", got, refs):
        rel = (a.double() - r).abs().max().item() / (r.abs().max().item() + 1e-6)
        assert rel < 5e-2, (name, rel)
    assert float(xi.grad[:, M:].abs().max()) == 0.0
    if Dw < Din:
        assert float(xi.grad[..., Dw:].abs().max()) == 0.0


def test_time4_standalone_tile_loop_matches_one_tile_per_workgroup(cuda_device):
    """time4_fwd / time4_bwd with 3 workgroups looping over 21 tiles == one workgroup per tile, bitwise."""
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    gen = torch.Generator().manual_seed(5)
    T, Mp, Din = 6, 21 * 16, 64
    x = torch.randn(T, Mp, Din, generator=gen).to(cuda_device)
    W, U, b = _lstm_params(Din, 128, gen, cuda_device)
    dh = torch.randn(Mp, 128, generator=gen).to(cuda_device)
    for all_h in (False, True):
        r0 = ops.time4_fwd(x, W, U, b, True, all_h, 0)
        r1 = ops.time4_fwd(x, W, U, b, True, all_h, 3)
        for a, c in zip(r0, r1):
            assert torch.equal(a, c)
        e0 = ops.time4_fwd(x, W, U, b, False, all_h, 3)[0]
        # inference (nothing saved): the same states up to the compiler's contraction choices
        torch.testing.assert_close(e0, r0[0], atol=1e-4, rtol=1e-4)
    b0 = ops.time4_bwd(dh, x, r0[1], r0[2], W, U, True, 0)
    b1 = ops.time4_bwd(dh, x, r0[1], r0[2], W, U, True, 3)
    assert torch.equal(b0[1], b1[1]) and torch.equal(b0[0][:T], b1[0][:T])
    n0 = ops.time4_bwd(dh, x, r0[1], r0[2], W, U, False, 3)
    assert n0[0].numel() == 0 and torch.equal(n0[1], b0[1])


@pytest.mark.parametrize("frozen", [False, True])
def test_timelayer_time_major_last128_matches_sequence_major(cuda_device, monkeypatch, frozen):
    """TimeLayer.forward_time_major with time4 on the standalone time-major kernels (GNNQC_T4_TM=1)
    vs the sequence-major lstm_fwd<128> path: outputs and gradients within bf16 rounding."""
    from gnnqc.models.timelayer import TimeLayer
    torch.manual_seed(1)
    tl = TimeLayer(20, 16, 2, "lstm", pool_size=3).to(cuda_device)
    for p in tl.parameters():
        p.requires_grad_(not frozen)
    M, T = 300, 180
    Mp = (M + 15) // 16 * 16
    x = torch.zeros(T, Mp, 20, device=cuda_device)
    x[:, :M] = torch.randn(T, M, 20, device=cuda_device)
    monkeypatch.setenv("GNNQC_CHAIN", "0")

    def run(on):
        monkeypatch.setenv("GNNQC_T4_TM", "1" if on else "0")
        xi = x.clone().requires_grad_(True)
        for p in tl.parameters():
            p.grad = None
        out = tl.forward_time_major(xi, M)
        out.pow(2).sum().backward()
        return out.detach(), [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters() if p.requires_grad]

    o0, g0 = run(False)
    o1, g1 = run(True)
    assert o1.shape == o0.shape == (M, 128)
    assert (o1 - o0).abs().max().item() < 2e-2
    for a, b_ in zip(g1, g0):
        assert (a - b_).norm().item() <= 3e-2 * (b_.norm().item() + 1e-6)
