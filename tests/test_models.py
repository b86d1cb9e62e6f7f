"""Model semantics on CPU (eager paths = the oracles of the HIP kernels)."""
import numpy as np
import pytest
import torch

from gnnqc import config as C
from gnnqc.models import BaselineClassifier, GCNClassifier, TimeLayer
from gnnqc.models.graphconv import AGNNConv, EdgeConv, GATConv, GatedGraphConv, GeneralConv
from gnnqc.ops import gcn as G
from gnnqc.ops.lstm import lstm_eager


def _cfgs(ds="cml"):
    pc = C.normalize_preproc(C.default(f"preprocessing_{ds}"))
    mc = C.default(f"model_{ds}")
    return mc, pc


def test_parameter_counts_match_decoded_checkpoints():
    # SURVEY §5.4 / BASELINE.md: 188,225 / 188,305 / 187,073 / 187,137 incl. BN moving stats
    for ds, gcn_total, base_total in (("cml", 188225, 187073), ("soilnet", 188305, 187137)):
        mc, pc = _cfgs(ds)
        m = GCNClassifier(mc, pc)
        n_train = sum(p.numel() for p in m.parameters())
        n_bn = m.gcn_layer.bn_moving_mean.numel() + m.gcn_layer.bn_moving_variance.numel()
        assert n_train + n_bn == gcn_total
        b = BaselineClassifier(mc, pc)
        assert sum(p.numel() for p in b.parameters()) == base_total


def test_lstm_eager_matches_torch_lstm():
    torch.manual_seed(0)
    M, T, Din, H = 5, 9, 3, 8
    lstm = torch.nn.LSTM(Din, H, batch_first=True)
    x = torch.randn(M, T, Din)
    ref, _ = lstm(x)
    # Keras layout: kernel [in, 4H], recurrent [H, 4H]; gate order i,f,c,o == torch i,f,g,o
    W = lstm.weight_ih_l0.detach().t()
    U = lstm.weight_hh_l0.detach().t()
    b = (lstm.bias_ih_l0 + lstm.bias_hh_l0).detach()
    out = lstm_eager(x, W, U, b, True)
    assert torch.allclose(out, ref, atol=1e-6)
    last = lstm_eager(x, W, U, b, False)
    assert torch.allclose(last, ref[:, -1], atol=1e-6)


def test_timelayer_shapes():
    tl = TimeLayer(18, 16, 2, "lstm")
    y = tl(torch.randn(3, 181, 18))
    assert y.shape == (3, 128)
    tc = TimeLayer(18, 16, 2, "cnn", kernel_size=5)
    assert tc(torch.randn(3, 181, 18)).shape == (3, 128)
    assert TimeLayer(19, 16, 2, "lstm")(torch.randn(2, 337, 19)).shape == (2, 128)


def test_keras_same_padding_conv():
    from gnnqc.models.layers import Conv1D
    conv = Conv1D(2, 3, 4)   # even kernel: keras pads 1 left, 2 right
    x = torch.randn(1, 10, 2)
    y = conv(x)
    assert y.shape == (1, 10, 3)
    xp = torch.nn.functional.pad(x.transpose(1, 2), (1, 2))
    ref = torch.nn.functional.conv1d(xp, conv.kernel.permute(2, 1, 0), conv.bias).transpose(1, 2)
    assert torch.allclose(y, ref)


def _graph_batch(B=3, T=5, N=6, Cin=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, N, Cin, generator=g)
    mask = torch.ones(B, N)
    mask[1, 4:] = 0
    adj = (torch.rand(B, N, N, generator=g) > 0.4).float()
    adj = ((adj + adj.transpose(1, 2) + torch.eye(N)) > 0).float() * mask[:, :, None] * mask[:, None, :]
    return x * mask[:, None, :, None], adj, mask


def test_fused_pool_identity_equals_aggregate_then_pool():
    """pool(Â a) == sum_j w_j a_j : the algebra behind the fused HIP GCN kernel."""
    x, adj, mask = _graph_batch()
    a = torch.randn(x.shape[:3] + (4,)) * mask[:, None, :, None]
    ap = torch.tensor([0, 2, 1])
    for agg in ("mean", "sum"):
        A = G.normalized_adjacency(adj, agg)
        h = torch.einsum("bij,btjf->btif", A, a)
        for pool in ("mean", "sum", "selection"):
            ref = G.pool_nodes(h, mask, ap, pool)
            w = G.node_pool_weights(adj, mask, ap, agg, pool)
            fused = torch.einsum("bj,btjf->btf", w, a)
            assert torch.allclose(ref, fused, atol=1e-5), (agg, pool)


def test_masked_batchnorm_ignores_padding():
    x, adj, mask = _graph_batch()
    F = 4
    z = torch.randn(x.shape[:3] + (F,))
    rm, rv = torch.zeros(F), torch.ones(F)
    out = G.masked_batchnorm(z, mask, torch.ones(F), torch.zeros(F), rm, rv, True)
    valid = out[mask[:, None, :].expand(-1, z.shape[1], -1) > 0]
    assert torch.allclose(valid.mean(0), torch.zeros(F), atol=1e-5)
    assert torch.allclose(valid.var(0, unbiased=False), torch.ones(F) * (1 / (1 + 1e-3)), atol=2e-3)
    assert not torch.allclose(rm, torch.zeros(F))


@pytest.mark.parametrize("cls,kw", [(GeneralConv, dict(channels=16, aggregate="mean")),
                                    (AGNNConv, dict(aggregate="sum")),
                                    (GATConv, dict(channels=4, attn_heads=2, dropout_rate=0.0)),
                                    (GatedGraphConv, dict(channels=8, n_layers=2)),
                                    (EdgeConv, dict(channels=8, mlp_hidden=[16]))])
def test_graph_layers_shapes_and_masking(cls, kw):
    x, adj, mask = _graph_batch()
    layer = cls(2, **kw)
    y = layer(x, adj, mask)
    assert y.shape[:3] == x.shape[:3] and y.shape[3] == layer.out_features
    # padded nodes stay zero and do not influence valid ones
    assert float(y[1, :, 4:].abs().sum()) == 0.0
    x2 = x.clone()
    x2[1, :, 4:] = 123.0
    if cls is GeneralConv:
        layer.eval()
    y2 = layer(x2 * mask[:, None, :, None], adj, mask)
    assert torch.allclose(y2[1, :, :4], layer(x, adj, mask)[1, :, :4], atol=1e-5)


def test_gcn_classifier_pooling_variants_and_grads():
    mc, pc = _cfgs("cml")
    x, adj, mask = _graph_batch(B=2, T=181, N=5)
    anom = x[:, :, 0, :]
    ap = torch.zeros(2, dtype=torch.long)
    for pool in ("mean", "sum", "max"):
        mc.pooling.aggregation_type = pool
        m = GCNClassifier(mc, pc)
        p = m((x, anom, adj, mask, ap))
        assert p.shape == (2,) and torch.all((p > 0) & (p < 1))
    mc.pooling.aggregation_type = "mean"
    mc.pooling.type = "selection"
    m = GCNClassifier(mc, pc)
    z = m.logits((x, anom, adj, mask, ap))
    z.sum().backward()
    assert all(p.grad is not None for p in m.parameters())


def test_soilnet_models_per_node_outputs():
    mc, pc = _cfgs("soilnet")
    pc.timestep_before, pc.timestep_after = 150, 30
    x, adj, mask = _graph_batch(B=2, T=13, N=4, Cin=3)
    m = GCNClassifier(mc, pc)
    assert m((x, adj, mask)).shape == (2, 4)
    b = BaselineClassifier(mc, pc)
    assert b((x, mask)).shape == (2, 4)


def test_spatial_transformer_and_sensors_time_layer():
    mc, pc = _cfgs("cml")
    mc.spatial_transformer = {"use": True, "min_scale": 0.001, "max_scale": 1.0, "scale_numb": 4, "units": 8}
    mc.nodes_sequence_layer = {"use": True, "units": 6, "layer_type": "lstm"}
    x, adj, mask = _graph_batch(B=2, T=181, N=5)
    coords = torch.rand(2, 5, 4) + 50
    m = GCNClassifier(mc, pc)
    p = m((x, x[:, :, 0], adj, mask, torch.zeros(2, dtype=torch.long), coords))
    assert p.shape == (2,)


def test_regularizers_and_baseline_regularizer_quirk():
    mc, pc = _cfgs("cml")
    mc.baseline_model.regularizer = 1e-4      # NameError in the reference; works here
    b = BaselineClassifier(mc, pc)
    r = b.regularization_loss()
    assert r is not None and float(r) > 0
