"""Metrics vs sklearn; CPU training end-to-end; checkpoint round trip."""
import numpy as np
import pytest
import torch

from gnnqc import config as C
from gnnqc.eval import metrics as M


def test_metrics_match_sklearn():
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.default_rng(0)
    y = rng.random(2000) < 0.2
    p = np.clip(y * 0.3 + rng.random(2000) * 0.8, 0, 1)
    p = np.round(p, 4)
    yp = p > 0.5
    assert abs(M.matthews_corrcoef(y, yp) - sk.matthews_corrcoef(y, yp)) < 1e-12
    assert abs(M.precision_score(y, yp) - sk.precision_score(y, yp)) < 1e-12
    assert abs(M.recall_score(y, yp) - sk.recall_score(y, yp)) < 1e-12
    assert abs(M.accuracy_score(y, yp) - sk.accuracy_score(y, yp)) < 1e-12
    fpr, tpr, thr = M.roc_curve(y, p)
    f2, t2, th2 = sk.roc_curve(y, p)
    assert np.allclose(fpr, f2) and np.allclose(tpr, t2) and np.allclose(thr[1:], th2[1:])
    assert abs(M.auc(fpr, tpr) - sk.roc_auc_score(y, p)) < 1e-12
    assert abs(M.roc_auc_score(y, p) - sk.roc_auc_score(y, p)) < 1e-12


def test_select_threshold_matches_bruteforce():
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.default_rng(1)
    y = rng.random(3000) < 0.15
    p = np.clip(y * 0.25 + rng.random(3000) * 0.75, 0, 1)
    cands = np.unique(np.round(p, 3))
    brute = [sk.matthews_corrcoef(y, p > c) for c in cands]
    assert M.select_threshold(p, y, verbose=False) == pytest.approx(cands[int(np.argmax(brute))])


def test_histogram_metrics():
    from gnnqc.ops.metrics import score_histogram
    rng = np.random.default_rng(2)
    y = (rng.random(5000) < 0.3).astype(np.float32)
    p = np.clip(y * 0.3 + rng.random(5000) * 0.7, 0, 1).astype(np.float32)
    p = np.round(p, 3)
    h = score_histogram(torch.from_numpy(p), torch.from_numpy(y), None, 1001).numpy()
    thr, mcc = M.mcc_threshold_from_hist(h)
    t2 = M.select_threshold(p, y, verbose=False)
    assert thr == pytest.approx(t2, abs=1e-9)
    assert M.auc_from_hist(h) == pytest.approx(M.roc_auc_score(y, p), abs=1e-6)


def _small_cml(seed=4):
    from gnnqc.data.preprocessing import create_windows_dataset, load_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=10 * 1440, seed=seed))
    st = DeviceStore(ws, "rolling_median", pc.graph)
    return pc, ws, st


def test_train_model_cpu_end_to_end(tmp_path):
    from gnnqc.data.preprocessing import create_batched_dataset, load_dataset
    from gnnqc.eval import calculate_metrics, calculate_threshold
    from gnnqc.models import GCNClassifier
    from gnnqc.train import flatten_predictions, predict, train_model
    pc, ws, st = _small_cml()
    mc = C.default("model_cml")
    mc.epochs = 2
    mc.sequence_layer.filter_1_size = 8
    mc.dense.units = 16
    tr, va, te = load_dataset(pc, ws)
    pc.batch_size = 64
    lab = ws.labels_flat()
    va_mix = np.concatenate([va[lab[va] == 1][:64], va[lab[va] == 0][:192]])
    assert lab[va_mix].sum() > 0
    tl, pc, _ = create_batched_dataset(tr[:512], pc, st)
    vl, _, _ = create_batched_dataset(va_mix, pc, st, shuffle=False)
    torch.manual_seed(0)
    m = GCNClassifier(mc, pc)
    hist, m = train_model(m, mc, pc, tl, vl, store=st, checkpoint_path=str(tmp_path / "ckpt"),
                          log_path=str(tmp_path / "log.jsonl"), verbose=0)
    assert len(hist.history["loss"]) == 2 and "val_auc" in hist.history
    assert np.isfinite(hist.history["loss"]).all()
    thr, idx = calculate_threshold(mc, pc, vl, m)
    assert idx == pc.timestep_before and 0 <= thr <= 1
    r = flatten_predictions(predict(m, st, vl))
    out = calculate_metrics(r["y"], r["p"] > thr, r["p"], None, verbose=False)
    assert 0 <= out[4] <= 1
    # checkpoint round trip
    from gnnqc.ckpt import load_model
    m2 = load_model(str(tmp_path / "ckpt"))
    b = st.gather(torch.arange(4))
    m.eval()
    m2.eval()
    assert torch.allclose(m(b.model_inputs("cml")), m2(b.model_inputs("cml")), atol=1e-6)


def test_training_reduces_loss_cpu():
    from gnnqc.data.store import DeviceLoader
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, ws, st = _small_cml(seed=5)
    mc = C.default("model_cml")
    mc.baseline_model.filter_1_size = 8
    torch.manual_seed(0)
    m = BaselineClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 3e-3)
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=False, batch_size=64)
    L = DeviceLoader(st, np.arange(min(st.n_windows, 640)), 64)
    first = None
    for ep in range(4):
        res = t.train_epoch(L, ep)
        first = first or res["loss"]
    assert res["loss"] < first


def test_split_optimizer_step_matches_fused_cpu(monkeypatch):
    """The data-parallel step layout (backward, then a separate optimizer step after the
    all-reduce point) == the fused step, on CPU (eager; no graphs)."""
    from gnnqc.data.store import DeviceLoader
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, ws, st = _small_cml(seed=6)
    mc = C.default("model_cml")
    mc.baseline_model.filter_1_size = 8

    def run(split):
        monkeypatch.setenv("GNNQC_SPLIT_OPT_GRAPH", "1" if split else "0")
        torch.manual_seed(0)
        m = BaselineClassifier(mc, pc)
        opt = make_optimizer("adam", m.parameters(), 3e-3)
        t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=False, batch_size=32)
        assert t.split_opt == split
        L = DeviceLoader(st, np.arange(min(st.n_windows, 128)), 32)
        for row in L.batch_ids():
            t.train_step(row)
        assert opt.iterations == 4
        return torch.cat([p.detach().reshape(-1) for p in m.parameters()])

    assert torch.equal(run(True), run(False))
