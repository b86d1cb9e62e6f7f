"""Model zoo: GCN classifier, graph-less baseline and their building blocks."""
from .baseline import BaselineClassifier
from .gcn import GCNClassifier, graph_reshape, timeseries_pooling
from .graphconv import AGNNConv, EdgeConv, GATConv, GatedGraphConv, GeneralConv, make_graph_layer
from .spatial import SensorsTimeLayer, SpatialTransformer
from .timelayer import TimeLayer


def create_model(model_config, preprocessing_config, baseline: bool = False):
    """``GCNClassifier`` or ``BaselineClassifier`` (the two classes of ``libs/create_model.py``)."""
    cls = BaselineClassifier if baseline else GCNClassifier
    return cls(model_config, preprocessing_config)


__all__ = ["GCNClassifier", "BaselineClassifier", "TimeLayer", "GeneralConv", "AGNNConv", "GATConv",
           "GatedGraphConv", "EdgeConv", "SpatialTransformer", "SensorsTimeLayer", "timeseries_pooling",
           "graph_reshape", "make_graph_layer", "create_model"]
