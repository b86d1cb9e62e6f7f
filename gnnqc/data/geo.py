"""Geodesy helpers (vectorised numpy).

* :func:`geodesic_distance_matrix` replaces the reference's O(N^2) Python loop over
  ``geopy.distance.geodesic`` (``libs/preprocessing_functions.py:25-47``) with a
  vectorised Vincenty inverse solution on the WGS84 ellipsoid (sub-millimetre
  agreement with Karney's algorithm for the non-antipodal distances of sensor
  networks). Pairs that do not converge (near-antipodal) fall back to a
  spherical great-circle estimate.
* :func:`utm_to_wgs84` / :func:`wgs84_to_utm` replace the pyproj call of
  ``libs/util/geo_spatial.py:5-19`` with the Krüger series for the transverse
  Mercator projection (nanometre-level accurate inside a UTM zone).
"""
from __future__ import annotations

import numpy as np

WGS84_A = 6378137.0
WGS84_F = 1.0 / 298.257223563
WGS84_B = WGS84_A * (1.0 - WGS84_F)


def vincenty_inverse(lat1, lon1, lat2, lon2, max_iter: int = 200, tol: float = 1e-12):
    """Ellipsoidal distance in metres between arrays of points (degrees)."""
    lat1, lon1, lat2, lon2 = (np.asarray(x, dtype=np.float64) for x in (lat1, lon1, lat2, lon2))
    lat1, lon1, lat2, lon2 = np.broadcast_arrays(lat1, lon1, lat2, lon2)
    a, b, f = WGS84_A, WGS84_B, WGS84_F
    L = np.radians(lon2 - lon1)
    U1 = np.arctan((1 - f) * np.tan(np.radians(lat1)))
    U2 = np.arctan((1 - f) * np.tan(np.radians(lat2)))
    sinU1, cosU1, sinU2, cosU2 = np.sin(U1), np.cos(U1), np.sin(U2), np.cos(U2)
    lam = L.copy()
    converged = np.zeros(L.shape, dtype=bool)
    sin_sigma = np.zeros_like(L)
    cos_sigma = np.ones_like(L)
    sigma = np.zeros_like(L)
    cos2_alpha = np.ones_like(L)
    cos_2sm = np.zeros_like(L)
    for _ in range(max_iter):
        sin_lam, cos_lam = np.sin(lam), np.cos(lam)
        sin_sigma = np.sqrt((cosU2 * sin_lam) ** 2 + (cosU1 * sinU2 - sinU1 * cosU2 * cos_lam) ** 2)
        cos_sigma = sinU1 * sinU2 + cosU1 * cosU2 * cos_lam
        sigma = np.arctan2(sin_sigma, cos_sigma)
        with np.errstate(invalid="ignore", divide="ignore"):
            sin_alpha = np.where(sin_sigma > 0, cosU1 * cosU2 * sin_lam / np.where(sin_sigma > 0, sin_sigma, 1), 0.0)
            cos2_alpha = 1 - sin_alpha ** 2
            cos_2sm = np.where(cos2_alpha != 0, cos_sigma - 2 * sinU1 * sinU2 / np.where(cos2_alpha != 0, cos2_alpha, 1), 0.0)
        C = f / 16 * cos2_alpha * (4 + f * (4 - 3 * cos2_alpha))
        lam_new = L + (1 - C) * f * sin_alpha * (
            sigma + C * sin_sigma * (cos_2sm + C * cos_sigma * (-1 + 2 * cos_2sm ** 2)))
        converged = np.abs(lam_new - lam) < tol
        lam = lam_new
        if converged.all():
            break
    u2 = cos2_alpha * (a ** 2 - b ** 2) / b ** 2
    A = 1 + u2 / 16384 * (4096 + u2 * (-768 + u2 * (320 - 175 * u2)))
    B = u2 / 1024 * (256 + u2 * (-128 + u2 * (74 - 47 * u2)))
    d_sigma = B * sin_sigma * (cos_2sm + B / 4 * (cos_sigma * (-1 + 2 * cos_2sm ** 2)
                                                  - B / 6 * cos_2sm * (-3 + 4 * sin_sigma ** 2) * (-3 + 4 * cos_2sm ** 2)))
    s = b * A * (sigma - d_sigma)
    same = (lat1 == lat2) & (lon1 == lon2)
    s = np.where(same, 0.0, s)
    if not converged.all():
        # near-antipodal fallback: mean-radius great circle
        bad = ~converged & ~same
        s = np.where(bad, haversine(lat1, lon1, lat2, lon2), s)
    return s


def haversine(lat1, lon1, lat2, lon2, radius: float = 6371008.8):
    p1, p2 = np.radians(lat1), np.radians(lat2)
    dphi = p2 - p1
    dl = np.radians(np.asarray(lon2) - np.asarray(lon1))
    h = np.sin(dphi / 2) ** 2 + np.cos(p1) * np.cos(p2) * np.sin(dl / 2) ** 2
    return 2 * radius * np.arcsin(np.sqrt(np.clip(h, 0, 1)))


def geodesic_distance_matrix(lat, lon, unit: str = "km") -> np.ndarray:
    """Symmetric [N, N] matrix of pairwise geodesic distances (zero diagonal)."""
    lat = np.asarray(lat, dtype=np.float64)
    lon = np.asarray(lon, dtype=np.float64)
    n = lat.shape[0]
    iu, ju = np.triu_indices(n, k=1)
    d = np.zeros((n, n), dtype=np.float64)
    if iu.size:
        vals = vincenty_inverse(lat[iu], lon[iu], lat[ju], lon[ju])
        d[iu, ju] = vals
        d[ju, iu] = vals
    scale = {"m": 1.0, "km": 1e-3}[unit]
    return d * scale


# ---------------------------------------------------------------------------
# UTM <-> WGS84 (Krüger n-series, 6th order)
# ---------------------------------------------------------------------------
_K0 = 0.9996
_N = WGS84_F / (2 - WGS84_F)
_A_RECT = WGS84_A / (1 + _N) * (1 + _N ** 2 / 4 + _N ** 4 / 64 + _N ** 6 / 256)
_ALPHA = (
    _N / 2 - 2 * _N ** 2 / 3 + 5 * _N ** 3 / 16 + 41 * _N ** 4 / 180 - 127 * _N ** 5 / 288 + 7891 * _N ** 6 / 37800,
    13 * _N ** 2 / 48 - 3 * _N ** 3 / 5 + 557 * _N ** 4 / 1440 + 281 * _N ** 5 / 630 - 1983433 * _N ** 6 / 1935360,
    61 * _N ** 3 / 240 - 103 * _N ** 4 / 140 + 15061 * _N ** 5 / 26880 + 167603 * _N ** 6 / 181440,
    49561 * _N ** 4 / 161280 - 179 * _N ** 5 / 168 + 6601661 * _N ** 6 / 7257600,
    34729 * _N ** 5 / 80640 - 3418889 * _N ** 6 / 1995840,
    212378941 * _N ** 6 / 319334400,
)
_BETA = (
    _N / 2 - 2 * _N ** 2 / 3 + 37 * _N ** 3 / 96 - _N ** 4 / 360 - 81 * _N ** 5 / 512 + 96199 * _N ** 6 / 604800,
    _N ** 2 / 48 + _N ** 3 / 15 - 437 * _N ** 4 / 1440 + 46 * _N ** 5 / 105 - 1118711 * _N ** 6 / 3870720,
    17 * _N ** 3 / 480 - 37 * _N ** 4 / 840 - 209 * _N ** 5 / 4480 + 5569 * _N ** 6 / 90720,
    4397 * _N ** 4 / 161280 - 11 * _N ** 5 / 504 - 830251 * _N ** 6 / 7257600,
    4583 * _N ** 5 / 161280 - 108847 * _N ** 6 / 3991680,
    20648693 * _N ** 6 / 638668800,
)
_E = np.sqrt(WGS84_F * (2 - WGS84_F))


def wgs84_to_utm(lat, lon, zone: int, northern: bool = True):
    lat = np.radians(np.asarray(lat, dtype=np.float64))
    lon = np.radians(np.asarray(lon, dtype=np.float64))
    lon0 = np.radians((zone - 1) * 6 - 180 + 3)
    t = np.sinh(np.arctanh(np.sin(lat)) - _E * np.arctanh(_E * np.sin(lat)))
    xi_p = np.arctan2(t, np.cos(lon - lon0))
    eta_p = np.arctanh(np.sin(lon - lon0) / np.sqrt(1 + t ** 2))
    xi, eta = xi_p.copy(), eta_p.copy()
    for j, a in enumerate(_ALPHA, start=1):
        xi = xi + a * np.sin(2 * j * xi_p) * np.cosh(2 * j * eta_p)
        eta = eta + a * np.cos(2 * j * xi_p) * np.sinh(2 * j * eta_p)
    easting = 500000.0 + _K0 * _A_RECT * eta
    northing = _K0 * _A_RECT * xi + (0.0 if northern else 10000000.0)
    return easting, northing


def utm_to_wgs84(easting, northing, zone: int, northern: bool = True):
    """Inverse transverse Mercator: UTM metres -> (lat, lon) degrees."""
    x = np.asarray(easting, dtype=np.float64) - 500000.0
    y = np.asarray(northing, dtype=np.float64) - (0.0 if northern else 10000000.0)
    xi = y / (_K0 * _A_RECT)
    eta = x / (_K0 * _A_RECT)
    xi_p, eta_p = xi.copy(), eta.copy()
    for j, b in enumerate(_BETA, start=1):
        xi_p = xi_p - b * np.sin(2 * j * xi) * np.cosh(2 * j * eta)
        eta_p = eta_p - b * np.cos(2 * j * xi) * np.sinh(2 * j * eta)
    chi = np.arcsin(np.sin(xi_p) / np.cosh(eta_p))
    # conformal latitude -> geodetic latitude (fixed-point iteration)
    tau_p = np.tan(chi)
    tau = tau_p.copy()
    for _ in range(8):
        sigma = np.sinh(_E * np.arctanh(_E * tau / np.sqrt(1 + tau ** 2)))
        tau_i = tau * np.sqrt(1 + sigma ** 2) - sigma * np.sqrt(1 + tau ** 2)
        dtau = (tau_p - tau_i) / np.sqrt(1 + tau_i ** 2) * (1 + (1 - _E ** 2) * tau ** 2) / (
            (1 - _E ** 2) * np.sqrt(1 + tau ** 2))
        tau = tau + dtau
    lat = np.degrees(np.arctan(tau))
    lon0 = (zone - 1) * 6 - 180 + 3
    lon = lon0 + np.degrees(np.arctan2(np.sinh(eta_p), np.cos(xi_p)))
    return lat, lon


__all__ = ["vincenty_inverse", "haversine", "geodesic_distance_matrix", "wgs84_to_utm", "utm_to_wgs84"]
