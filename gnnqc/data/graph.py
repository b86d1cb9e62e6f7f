"""Sensor graphs: distance/depth matrices, neighbour selection and adjacency rules.

Reference behaviour:

* CML distances use the link mid-point, in km (``libs/preprocessing_functions.py:25-47``);
  SoilNet uses sensor lat/lon in metres. The XAI snapshot is always metres
  (``xai/libs/preprocessing_functions.py:1046-1066``) - ``unit`` selects.
* CML neighbours of a flagged link: ``dist <= max_sample_distance`` (``:62-64``);
  the per-window edges use ``dist < max_sample_distance`` (``:408``) - so self
  loops come from the zero diagonal.
* SoilNet edges: ``(dist <= d & depth_diff == 0) | (dist == 0 & depth_diff <= max_depth)``
  (``:470-473``); XAI neighbour selection uses the same rule (``:1069-1077``).
* ``knn`` is an explicit option (BASELINE.json mentions k=5; the reference itself
  uses radius graphs).
"""
from __future__ import annotations

import numpy as np

from .geo import geodesic_distance_matrix
from .raw_io import SensorData


def sensor_positions(ds: SensorData, ds_type: str):
    if ds_type == "cml":
        lat = (ds["site_a_latitude"].data + ds["site_b_latitude"].data) / 2.0
        lon = (ds["site_a_longitude"].data + ds["site_b_longitude"].data) / 2.0
    else:
        lat = ds["latitude"].data
        lon = ds["longitude"].data
    return np.asarray(lat, np.float64), np.asarray(lon, np.float64)


def compute_distance_matrix(ds: SensorData, ds_type: str = "cml", unit: str | None = None) -> np.ndarray:
    if unit is None:
        unit = "km" if ds_type == "cml" else "m"
    lat, lon = sensor_positions(ds, ds_type)
    return geodesic_distance_matrix(lat, lon, unit=unit)


def compute_depth_matrix(ds: SensorData) -> np.ndarray:
    depth = np.asarray(ds["depth"].data, dtype=np.float64)
    return np.abs(depth[None, :] - depth[:, None])


def get_neighbors(distances: np.ndarray, sensor_pos: int, max_dist: float, ds_type: str = "cml",
                  depths: np.ndarray | None = None, max_depth: float | None = None) -> np.ndarray:
    """Positions of the neighbours (incl. the sensor itself) of ``sensor_pos``."""
    row = distances[sensor_pos]
    if ds_type == "cml" or depths is None:
        return np.nonzero(row <= max_dist)[0]
    drow = depths[sensor_pos]
    mask = ((row <= max_dist) & (drow == 0)) | ((row == 0) & (drow <= max_depth))
    return np.nonzero(mask)[0]


def cml_adjacency(distances: np.ndarray, max_distance: float) -> np.ndarray:
    return distances < max_distance


def soilnet_adjacency(distances: np.ndarray, depths: np.ndarray, max_distance: float,
                      max_depth: float) -> np.ndarray:
    return ((distances <= max_distance) & (depths == 0)) | ((distances == 0) & (depths <= max_depth))


def knn_adjacency(distances: np.ndarray, k: int, valid: np.ndarray | None = None) -> np.ndarray:
    """Symmetrised k-nearest-neighbour graph with self loops (explicit option)."""
    d = np.array(distances, dtype=np.float64, copy=True)
    n = d.shape[0]
    if valid is not None:
        d[~valid, :] = np.inf
        d[:, ~valid] = np.inf
    np.fill_diagonal(d, np.inf)
    kk = min(k, max(n - 1, 0))
    a = np.zeros((n, n), dtype=bool)
    if kk > 0:
        idx = np.argsort(d, axis=1)[:, :kk]
        rows = np.repeat(np.arange(n), kk)
        cols = idx.reshape(-1)
        ok = np.isfinite(d[rows, cols])
        a[rows[ok], cols[ok]] = True
    a = a | a.T
    np.fill_diagonal(a, True)
    if valid is not None:
        a &= valid[:, None] & valid[None, :]
    return a


def build_adjacency(cfg_graph, distances: np.ndarray, depths: np.ndarray | None, ds_type: str) -> np.ndarray:
    kind = cfg_graph.get("adjacency", "radius")
    if kind == "knn":
        return knn_adjacency(distances, int(cfg_graph.get("k", 5)))
    if ds_type == "cml":
        return cml_adjacency(distances, cfg_graph["max_sample_distance"])
    return soilnet_adjacency(distances, depths, cfg_graph["max_sample_distance"],
                             cfg_graph.get("max_neighbour_depth", cfg_graph.get("max_depth", 0.1)))


def edge_list(adjacency: np.ndarray):
    """(nodes, neighbours) like ``np.where(adjacency_matrix)`` (``:221``)."""
    return np.nonzero(adjacency)


__all__ = [
    "sensor_positions", "compute_distance_matrix", "compute_depth_matrix", "get_neighbors",
    "cml_adjacency", "soilnet_adjacency", "knn_adjacency", "build_adjacency", "edge_list",
]
