"""SoilNet of the XAI generation: per-anomalous-sensor neighbourhoods (select_sensors, <box>_<sensor>
NetCDF files, depth-aware neighbours, the selected sensor's target), their window / batch layout
(anomalous-sensor series, one label per window), the GCN and baseline models on it, TFRecord
round trip with the *_anomalous_sensor features and integrated gradients
(xai/libs/preprocessing_functions.py:218-240, 419-624, 667-707, 791-802, 951-1025)."""
import os

import numpy as np
import pytest
import torch

from gnnqc import config as C


@pytest.fixture(scope="module")
def xai_soil():
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.synthetic import make_soilnet_raw
    raw = make_soilnet_raw(n_boxes=8, n_time=12 * 96, seed=3)
    pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
    pc["per_sensor"] = True
    pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    pc.timestep_before, pc.timestep_after = 900, 300          # T = 81 at 15 min
    ws = create_windows_dataset(pc, raw=raw)
    return raw, pc, ws


def test_select_sensors_and_neighbourhoods(xai_soil):
    from gnnqc.data.graph import compute_depth_matrix, compute_distance_matrix, get_neighbors
    from gnnqc.data.preprocessing import select_sensors
    raw, pc, ws = xai_soil
    sel = select_sensors(raw, 44)
    box = np.asarray(raw["box_id"].data)
    assert len(sel) == len(np.unique(box)) and len(set(box[sel])) == len(sel)   # one per box
    n_obs = (~np.isnan(np.asarray(raw["moisture"].data, np.float64))).sum(1)
    for s in sel:
        assert n_obs[s] == n_obs[box == box[s]].max()
    assert np.array_equal(sel, select_sensors(raw, 44))                        # seeded
    assert len(ws.groups) == len(sel) and ws.per_sensor and ws.ds_type == "soilnet"
    dist = compute_distance_matrix(raw, "soilnet", unit="m")
    dep = compute_depth_matrix(raw)
    ids = raw.sensor_ids
    for g, s in zip(ws.groups, sel):
        assert g.group_id == f"{box[s]}_{ids[s]}"
        assert g.sensor_ids[g.anomalous_pos] == ids[s] and g.target.ndim == 1
        nb = get_neighbors(dist, s, pc.graph.max_sample_distance, "soilnet", depths=dep, max_depth=pc.graph.max_depth)
        assert np.array_equal(g.sensor_ids, ids[nb])
        assert g.depths.shape == (len(nb), len(nb)) and g.features.shape[1] == 3
    labels = ws.labels_flat()
    assert labels.ndim == 1 and set(np.unique(labels)) <= {0, 1} and labels.sum() > 0


def test_batches_models_and_ig(xai_soil):
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import BaselineClassifier, GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    from gnnqc.xai.ig import IntegratedGradients, completeness_gap
    raw, pc, ws = xai_soil
    st = DeviceStore(ws, "scale_range", pc.graph)
    ids = torch.arange(min(12, st.n_windows))
    b = st.gather(ids)
    assert b.per_sensor and b.anom.shape == (len(ids), ws.seq_len, 3) and b.y.shape == (len(ids),)
    ap = b.anom_pos.clamp(min=0)
    assert torch.equal(b.anom, b.x[torch.arange(len(ids)), :, ap])              # the flagged sensor's series
    inp = b.model_inputs("soilnet")
    assert len(inp) == 5
    assert b.model_inputs("soilnet", baseline=True)[0] is b.anom
    mc = C.default("model_soilnet")
    mc.sequence_layer.filter_1_size = 4
    torch.manual_seed(0)
    for cls, base in ((GCNClassifier, False), (BaselineClassifier, True)):
        model = cls(mc, pc)
        assert model.per_sensor
        out = model(b.model_inputs("soilnet", base))
        assert out.shape == (len(ids),)
        opt = make_optimizer("adam", model.parameters(), 1e-3)
        tr = Trainer(model, st, opt, {0: 1.0, 1: 5.0}, baseline=base, use_graph=False, batch_size=len(ids))
        before = opt.flat_p.clone()
        assert torch.isfinite(tr.train_step(ids)) and not torch.equal(before, opt.flat_p)
    model = GCNClassifier(mc, pc).double()
    bd = st.gather(ids[:3])
    for f in ("x", "anom", "adj", "node_mask"):
        setattr(bd, f, getattr(bd, f).double())
    res = IntegratedGradients(model, "soilnet", m_steps=32).attribute(bd)
    assert res["grad_x"].shape == bd.x.shape and res["grad_anom"].shape == bd.anom.shape
    span = (res["path_pred"][-1] - res["path_pred"][0]).abs()
    assert bool((completeness_gap(res).abs() <= 0.05 * span + 1e-3).all())


def test_netcdf_files_and_tfrecords(xai_soil, tmp_path):
    from gnnqc.data.preprocessing import create_sensors_ncfiles, load_sensor_groups
    from gnnqc.data.tfrecord import TFRecordWindows, write_window_records
    from gnnqc.data.windows import WindowSet
    raw, pc, ws = xai_soil
    pc2 = C.Config(dict(pc))
    pc2["ncfiles_dir"] = str(tmp_path / "nc")
    pc2.dataset["ncfiles_dir"] = pc2["ncfiles_dir"]
    paths = create_sensors_ncfiles(raw, pc2)
    names = sorted(os.path.basename(p)[:-3] for p in paths)
    assert names == sorted(g.group_id for g in ws.groups)                       # <box>_<sensor>.nc
    back = {g.group_id: g for g in load_sensor_groups(pc2)}
    for g in ws.groups:
        h = back[g.group_id]
        assert h.per_sensor and h.anomalous_pos == g.anomalous_pos
        assert np.array_equal(h.sensor_ids, g.sensor_ids) and np.allclose(h.depths, g.depths)
        assert np.allclose(np.nan_to_num(h.target, nan=-1), np.nan_to_num(g.target, nan=-1))
    out = str(tmp_path / "rec")
    files = write_window_records(ws, out, max_records=40, graph_cfg=pc.graph)
    assert files
    tw = TFRecordWindows(files, "soilnet")
    assert tw.per_sensor and tw.y.ndim == 1
    bt = next(tw.batches(8))
    assert bt.anom is not None and bt.anom.shape[-1] == 3 and len(bt.model_inputs("soilnet")) == 5


@pytest.mark.gpu
def test_xai_soilnet_gpu_step_matches_fp64_eager(cuda_device, xai_soil):
    """The per-sensor SoilNet GCN (3 input channels) takes the CML fast path on the GPU - fused
    GCN + pooling kernel, headed LSTM chain, fused head + BCE - and matches float64 eager PyTorch."""
    import copy
    from gnnqc.data.store import DeviceStore
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.lstm import direct_grad_accumulation
    from gnnqc.train.loss import weighted_bce_with_logits
    raw, pc, ws = xai_soil
    st = DeviceStore(ws, "scale_range", pc.graph, device=cuda_device)
    st_cpu = DeviceStore(ws, "scale_range", pc.graph)
    torch.manual_seed(0)
    model = GCNClassifier(C.default("model_soilnet"), pc).to(cuda_device)
    ids = torch.arange(min(48, st.n_windows))
    b = st.gather(ids.to(cuda_device))
    inputs = b.model_inputs("soilnet")
    assert model._cml_time_major(inputs)
    for p in model.parameters():
        p.grad = torch.zeros_like(p)
    with direct_grad_accumulation(True):
        loss, z = model.fused_loss(inputs, b.y, b.y_mask, 1.0, 5.0)
        loss.backward(torch.ones((), device=cuda_device))
    torch.cuda.synchronize()
    ref = copy.deepcopy(model).cpu().double()
    for p in ref.parameters():
        p.grad = None
    bc = st_cpu.gather(ids)
    ri = [t.double() if torch.is_tensor(t) and t.is_floating_point() else t for t in bc.model_inputs("soilnet")]
    zr = ref.logits(ri)
    lr = weighted_bce_with_logits(zr, bc.y.double(), bc.y_mask.double(), 1.0, 5.0)
    lr.backward()
    assert abs(loss.item() - lr.item()) <= 2e-2 * abs(lr.item()) + 1e-4
    assert (z.cpu().double() - zr.detach()).abs().max().item() < 5e-2
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        if q.grad is None:
            continue
        err = (p.grad.cpu().double() - q.grad).norm().item()
        assert err <= 8e-2 * q.grad.norm().item() + 1e-5, (n, err)
