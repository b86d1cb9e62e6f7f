"""Integrated gradients on the GPU (alpha folded into the batch, HIP chain / GCN input-gradient
kernels, ig_interp / ig_accum / ig_finalize) against the same explainer evaluated in float64 on the
CPU with the LSTM rounded where the kernels round (gnnqc/ops/lstm_ref.py)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("negative_values", ["keep", "abs"])
def test_ig_gpu_matches_fp64_cpu(cuda_device, cml_windows, negative_values):
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.xai.ig import IntegratedGradients, completeness_gap
    pc, ws = cml_windows
    torch.manual_seed(0)
    mc = C.default("model_cml")
    model = GCNClassifier(mc, pc).to(cuda_device)
    with torch.no_grad():                      # a non-trivial output range along the path
        model.dense_out.bias.fill_(0.3)
        for p in (model.dense.bias, model.dense2.bias):
            p.normal_(0, 0.2)
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    st_cpu = DeviceStore(ws, "rolling_median", pc.graph, device="cpu")
    ids = torch.tensor([0, 7, 19, 33])
    b = st.gather(ids.to(cuda_device))
    m = 24
    got = IntegratedGradients(model, "cml", m_steps=m, negative_values=negative_values).attribute(b)
    torch.cuda.synchronize()

    ref_model = copy.deepcopy(model).cpu().double()
    bc = st_cpu.gather(ids)
    for f in ("x", "anom", "adj", "node_mask"):
        setattr(bc, f, getattr(bc, f).double())
    from gnnqc.ops.lstm_ref import kernel_rounding
    with kernel_rounding():
        ref = IntegratedGradients(ref_model, "cml", m_steps=m, negative_values=negative_values).attribute(bc)

    for k in ("grad_x", "grad_anom", "pred", "path_pred"):
        a, r = got[k].double().cpu(), ref[k]
        err = (a - r).norm().item()
        scale = r.norm().item()
        assert err <= 6e-3 * scale + 1e-6, (k, err, scale)
    if negative_values == "keep":
        # completeness (sum of attributions ~ f(x) - f(0)) holds on the GPU as well as in fp64
        gap_g = completeness_gap(got).abs().cpu().double()
        gap_r = completeness_gap(ref).abs()
        span = (ref["path_pred"][-1] - ref["path_pred"][0]).abs()
        assert bool((gap_g <= gap_r + 0.05 * span + 2e-3).all()), (gap_g, gap_r, span)


def test_ig_hip_kernels_match_torch(cuda_device):
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    torch.manual_seed(1)
    v = torch.randn(5, 37, 3, device=cuda_device)            # numel % 4 != 0: scalar tail
    a = torch.linspace(0, 1, 7, device=cuda_device)
    out = ops.ig_interp(v, a)
    torch.testing.assert_close(out.view(7, 5, 37, 3), a.view(7, 1, 1, 1) * v.unsqueeze(0))
    g = torch.randn(7 * 5, 37, 3, device=cuda_device)
    w = torch.rand(7, device=cuda_device)
    acc = torch.randn(5, 37, 3, device=cuda_device)
    expect = acc + torch.tensordot(w, g.view(7, 5, 37, 3), dims=1)
    ops.ig_accum(acc, g, w)
    torch.testing.assert_close(acc, expect, rtol=1e-5, atol=1e-5)
    for mode, fn in ((0, lambda t: t), (1, lambda t: t.clamp(min=0)), (2, torch.abs)):
        torch.testing.assert_close(ops.ig_finalize(acc, v, mode), fn(acc * v))
    torch.testing.assert_close(ops.ig_finalize(acc, v.new_zeros(0), 0), acc)


def test_ig_path_folded_gcn_matches_replicated_path(cuda_device, cml_windows, monkeypatch):
    """The CML GCN's path-folded IG (alpha applied inside ig_gcn_pool_fwd, input gradients
    trapezoid-summed inside ig_gcn_pool_bwd) == the generic path over kk x B interpolated copies
    (ig_interp -> GCN kernels -> ig_accum), with several path chunks (max_rows < (m+1) B)."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.xai.ig import IntegratedGradients
    pc, ws = cml_windows
    torch.manual_seed(3)
    model = GCNClassifier(C.default("model_cml"), pc).to(cuda_device)
    with torch.no_grad():
        model.dense_out.bias.fill_(0.2)
        model.gcn_layer.bn_moving_mean.normal_(0, 0.3)
        model.gcn_layer.bn_moving_variance.uniform_(0.5, 2.0)
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    b = st.gather(torch.tensor([1, 5, 11, 23, 40], device=cuda_device))
    ig = IntegratedGradients(model, "cml", m_steps=30, max_rows=5 * 8)
    model.eval()                               # (attribute() switches to eval itself)
    assert ig._cml_path_folded_ok(b)
    model.train()
    got = ig.attribute(b)
    monkeypatch.setattr(IntegratedGradients, "_cml_path_folded_ok", lambda self, batch: False)
    ref = IntegratedGradients(model, "cml", m_steps=30, max_rows=5 * 8).attribute(b)
    torch.cuda.synchronize()
    for k in ("grad_x", "grad_anom", "pred", "path_pred"):
        err = (got[k] - ref[k]).abs().max().item()
        scale = ref[k].abs().max().item()
        assert err <= 1e-4 * scale + 1e-7, (k, err, scale)


def test_ig_graph_replay_matches_eager(cuda_device, cml_windows):
    """The path-folded IG replays one HIP graph per input shape: a second batch of the same shape
    (inputs copied into the captured buffers) gives what the eager attribution gives."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.xai.ig import IntegratedGradients
    pc, ws = cml_windows
    torch.manual_seed(5)
    model = GCNClassifier(C.default("model_cml"), pc).to(cuda_device)
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    b1 = st.gather(torch.tensor([2, 9, 17], device=cuda_device))
    b2 = st.gather(torch.tensor([4, 12, 30], device=cuda_device))
    ig = IntegratedGradients(model, "cml", m_steps=20)
    ig.attribute(b1)
    assert ig._graph is not None
    got = ig.attribute(b2)
    ref = IntegratedGradients(model, "cml", m_steps=20, use_graph=False).attribute(b2)
    torch.cuda.synchronize()
    for k in ("grad_x", "grad_anom", "pred", "path_pred"):
        err = (got[k] - ref[k]).abs().max().item()
        assert err <= 1e-5 * ref[k].abs().max().item() + 1e-7, (k, err)


def test_head_prob_kernels_match_torch(cuda_device):
    """head_prob_fwd / head_prob_bwd (head.hip PROB mode): sigmoid of the Dense-LeakyReLU head and
    the input gradient of sum(sigmoid) against autograd on a plain fp32 PyTorch head."""
    from gnnqc.ops.head import head_eager
    from gnnqc.utils.native import hip_ops
    torch.manual_seed(0)
    for R, F in ((37, 128), (300, 64)):
        feat = torch.randn(R, F, device=cuda_device)
        W1, b1 = torch.randn(F, 64, device=cuda_device) * 0.2, torch.randn(64, device=cuda_device) * 0.1
        W2, b2 = torch.randn(64, 64, device=cuda_device) * 0.2, torch.randn(64, device=cuda_device) * 0.1
        W3, b3 = torch.randn(64, 1, device=cuda_device) * 0.3, torch.randn(1, device=cuda_device) * 0.1
        z1, z2, prob = hip_ops().head_prob_fwd(feat, W1, b1, W2, b2, W3, b3, 0.3, 0.2)
        dfeat = hip_ops().head_prob_bwd(feat, W1, W2, W3, z1, z2, prob, 0.3, 0.2)
        f = feat.clone().requires_grad_(True)
        ref = torch.sigmoid(head_eager(f, W1, b1, W2, b2, W3, b3, 0.3, 0.2))
        (g,) = torch.autograd.grad(ref.sum(), f)
        torch.testing.assert_close(prob, ref.detach(), atol=2e-6, rtol=1e-5)
        torch.testing.assert_close(dfeat, g, atol=1e-6, rtol=1e-4)


def test_ig_hip_head_matches_torch_head(cuda_device, cml_windows, monkeypatch):
    """The path-folded IG with the frozen head on HIP (GNNQC_IG_HEAD_HIP=1, default) == with the
    PyTorch head (rocBLAS GEMMs + aten LeakyReLU / sigmoid)."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.xai.ig import IntegratedGradients
    pc, ws = cml_windows
    torch.manual_seed(7)
    model = GCNClassifier(C.default("model_cml"), pc).to(cuda_device)
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    b = st.gather(torch.tensor([3, 8, 21, 33], device=cuda_device))
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("GNNQC_IG_HEAD_HIP", flag)
        res[flag] = IntegratedGradients(model, "cml", m_steps=24, use_graph=False).attribute(b)
    torch.cuda.synchronize()
    for k in ("grad_x", "grad_anom", "pred", "path_pred"):
        err = (res["1"][k] - res["0"][k]).abs().max().item()
        assert err <= 1e-5 * res["0"][k].abs().max().item() + 1e-7, (k, err)


def test_ig_time4_fused_head_matches_separate_head(cuda_device, cml_windows, monkeypatch):
    """The path-folded IG with time4 + the frozen head in one launch (GNNQC_IG_T4_HEAD=1, default:
    time4_prob_fwd -> sigmoid outputs and d p / d h_{T-1}; time4_bwd seeded with them) == time4 alone
    followed by the head_prob kernels (GNNQC_IG_T4_HEAD=0); and the fused launch really ran."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops import lstm as L
    from gnnqc.xai.ig import IntegratedGradients
    pc, ws = cml_windows
    torch.manual_seed(11)
    model = GCNClassifier(C.default("model_cml"), pc).to(cuda_device)
    with torch.no_grad():
        model.dense_out.bias.fill_(0.3)
    st = DeviceStore(ws, "rolling_median", pc.graph, device=cuda_device)
    b = st.gather(torch.tensor([3, 8, 21, 33, 34], device=cuda_device))
    calls = []
    orig = L._HipLSTMLast128Prob.forward

    def spy(ctx, *a):
        calls.append(1)
        return orig(ctx, *a)

    monkeypatch.setattr(L._HipLSTMLast128Prob, "forward", staticmethod(spy))
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("GNNQC_IG_T4_HEAD", flag)
        res[flag] = IntegratedGradients(model, "cml", m_steps=24, use_graph=False).attribute(b)
    torch.cuda.synchronize()
    assert calls, "the fused time4 + head path did not run"
    for k in ("grad_x", "grad_anom", "pred", "path_pred"):
        err = (res["1"][k] - res["0"][k]).abs().max().item()
        assert err <= 1e-4 * res["0"][k].abs().max().item() + 1e-7, (k, err)
