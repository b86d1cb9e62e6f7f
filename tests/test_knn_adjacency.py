"""k-NN (k = 5) adjacency - BASELINE.json configs[1]'s 'k=5' graph - as an explicit option next to
the reference's radius rule: graph properties, the store's per-sample adjacency
and a training step of the CML GCN on it."""
import numpy as np
import torch


def test_knn_adjacency_properties():
    from gnnqc.data.graph import knn_adjacency
    rng = np.random.default_rng(0)
    pts = rng.uniform(0, 10, size=(23, 2))
    d = np.sqrt(((pts[:, None] - pts[None]) ** 2).sum(-1))
    a = knn_adjacency(d, 5)
    assert a.dtype == bool and a.shape == (23, 23)
    assert np.array_equal(a, a.T), "symmetrised"
    assert a.diagonal().all(), "self loops (GeneralConv aggregates the node itself)"
    off = a & ~np.eye(23, dtype=bool)
    nearest = np.argsort(d + np.diag(np.full(23, np.inf)), axis=1)[:, :5]
    for i in range(23):
        assert off[i, nearest[i]].all(), "every node keeps its 5 nearest neighbours"
    assert off.sum(1).min() >= 5
    # invalid nodes drop out entirely
    valid = np.ones(23, dtype=bool)
    valid[[3, 7]] = False
    b = knn_adjacency(d, 5, valid)
    assert not b[[3, 7]].any() and not b[:, [3, 7]].any()
    assert (b & ~np.eye(23, dtype=bool))[valid][:, valid].sum(1).min() >= 5


def test_store_builds_knn_graph_and_trains():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=12, n_minutes=3 * 1440, seed=3))
    g_radius = dict(pc.graph)
    g_knn = dict(pc.graph, adjacency="knn", k=5)
    st_r = DeviceStore(ws, "rolling_median", g_radius)
    st_k = DeviceStore(ws, "rolling_median", g_knn)
    ids = torch.arange(min(16, st_k.n_windows))
    bk, br = st_k.gather(ids), st_r.gather(ids)
    assert torch.equal(bk.x, br.x)                     # only the graph differs
    adj = bk.adj
    assert torch.equal(adj, adj.transpose(1, 2))
    n_valid = bk.node_mask.sum(1)
    deg = (adj > 0).sum(2).float()                     # incl. the self loop
    live = bk.node_mask > 0
    assert bool((deg[live] >= torch.minimum(n_valid[:, None].expand_as(deg)[live], torch.tensor(6.0))).all())
    torch.manual_seed(0)
    mc = C.default("model_cml")
    mc.sequence_layer.filter_1_size = 4
    model = GCNClassifier(mc, pc)
    opt = make_optimizer("adam", model.parameters(), 1e-3)
    tr = Trainer(model, st_k, opt, {0: 1.0, 1: 5.0}, use_graph=False, batch_size=16)
    before = opt.flat_p.clone()
    loss = tr.train_step(ids)
    assert torch.isfinite(loss) and not torch.equal(before, opt.flat_p)
