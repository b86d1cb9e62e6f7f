"""Raw sensor-network container and NetCDF3 I/O.

The reference keeps raw data in xarray Datasets read from NetCDF
(``notebooks/prepare_raw_example_cml.ipynb``, ``libs/preprocessing_functions.py:79-120``).
xarray/netCDF4 are not available, so :class:`SensorData` is a small named-array
container with the same schema:

* CML: dims ``expert, sensor_id, time``; vars ``TL_1, TL_2 (sensor_id, time)``,
  expert flags ``Jump, Dew, Fluctuation, Unknown anomaly (expert, sensor_id, time)``,
  ``flagged (sensor_id)``; coords ``length, site_{a,b}_{latitude,longitude},
  frequency_{1,2}, polarization_{1,2}``.
* SoilNet: dims ``sensor_id, time``; vars ``moisture, temp, battv`` and the boolean
  ``{moisture,temp}_flag_*`` masks; coords ``box_id, level_id, latitude, longitude, depth``.

Files are NetCDF3 (``scipy.io.netcdf_file``): time is stored as float64
"minutes since 1970-01-01", string coordinates as char arrays, booleans as int8.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional, Sequence, Tuple

import numpy as np

TIME_UNITS = "minutes since 1970-01-01 00:00:00"


class Variable:
    __slots__ = ("dims", "data", "attrs")

    def __init__(self, dims: Sequence[str], data, attrs: Optional[dict] = None):
        self.dims = tuple(dims)
        self.data = np.asarray(data)
        self.attrs = dict(attrs or {})
        if self.data.ndim != len(self.dims):
            raise ValueError(f"data ndim {self.data.ndim} != dims {self.dims}")

    @property
    def values(self):
        return self.data

    @property
    def shape(self):
        return self.data.shape

    def __repr__(self):
        return f"Variable(dims={self.dims}, shape={self.data.shape}, dtype={self.data.dtype})"


class SensorData:
    """Minimal xarray-like dataset: named variables over named dimensions."""

    def __init__(self, variables: Optional[Dict[str, Variable]] = None,
                 coords: Optional[Dict[str, Variable]] = None, attrs: Optional[dict] = None):
        self.variables: Dict[str, Variable] = {}
        self.coords: Dict[str, Variable] = {}
        self.attrs = dict(attrs or {})
        for k, v in (coords or {}).items():
            self.set_coord(k, *v) if isinstance(v, tuple) else self.set_coord(k, v.dims, v.data, v.attrs)
        for k, v in (variables or {}).items():
            self[k] = v

    # ---------------------------------------------------------------- access
    @property
    def dims(self) -> Dict[str, int]:
        out: Dict[str, int] = {}
        for v in list(self.coords.values()) + list(self.variables.values()):
            for d, n in zip(v.dims, v.data.shape):
                if d in out and out[d] != n:
                    raise ValueError(f"inconsistent size for dim {d}: {out[d]} vs {n}")
                out[d] = n
        return out

    def __contains__(self, key):
        return key in self.variables or key in self.coords

    def __getitem__(self, key) -> Variable:
        if key in self.variables:
            return self.variables[key]
        if key in self.coords:
            return self.coords[key]
        raise KeyError(key)

    def __setitem__(self, key, value):
        if isinstance(value, tuple):
            dims, data = value[0], value[1]
            attrs = value[2] if len(value) > 2 else None
            if isinstance(dims, str):
                dims = (dims,)
            value = Variable(dims, data, attrs)
        if not isinstance(value, Variable):
            raise TypeError("assign a Variable or a (dims, data) tuple")
        self.variables[key] = value

    def set_coord(self, key, dims, data, attrs=None):
        if isinstance(dims, str):
            dims = (dims,)
        self.coords[key] = Variable(dims, data, attrs)

    def __getattr__(self, key):
        if key in ("variables", "coords", "attrs"):
            raise AttributeError(key)
        if key in self.variables:
            return self.variables[key]
        if key in self.coords:
            return self.coords[key]
        raise AttributeError(key)

    def drop(self, names: Iterable[str]) -> "SensorData":
        names = set([names] if isinstance(names, str) else names)
        out = self.copy()
        for n in names:
            out.variables.pop(n, None)
            out.coords.pop(n, None)
        return out

    def keys(self):
        return list(self.variables.keys())

    def copy(self) -> "SensorData":
        out = SensorData(attrs=dict(self.attrs))
        out.coords = {k: Variable(v.dims, v.data.copy(), v.attrs) for k, v in self.coords.items()}
        out.variables = {k: Variable(v.dims, v.data.copy(), v.attrs) for k, v in self.variables.items()}
        return out

    # -------------------------------------------------------------- indexing
    def isel(self, **indexers) -> "SensorData":
        """Positional selection along named dimensions (int arrays, slices or bool masks)."""
        out = SensorData(attrs=dict(self.attrs))

        def take(var: Variable) -> Variable:
            data = var.data
            for ax, d in enumerate(var.dims):
                if d in indexers:
                    idx = indexers[d]
                    sl = [slice(None)] * data.ndim
                    sl[ax] = idx
                    data = data[tuple(sl)]
            return Variable(var.dims, np.ascontiguousarray(data), var.attrs)

        out.coords = {k: take(v) for k, v in self.coords.items()}
        out.variables = {k: take(v) for k, v in self.variables.items()}
        return out

    def sel_sensors(self, sensor_ids: Sequence) -> "SensorData":
        ids = list(self.coords["sensor_id"].data)
        pos = np.array([ids.index(s) for s in sensor_ids], dtype=np.int64)
        return self.isel(sensor_id=pos)

    def time_slice(self, start, stop) -> "SensorData":
        t = self.coords["time"].data
        m = (t >= np.datetime64(start)) & (t <= np.datetime64(stop))
        return self.isel(time=np.nonzero(m)[0])

    @property
    def sensor_ids(self) -> np.ndarray:
        return self.coords["sensor_id"].data

    @property
    def time(self) -> np.ndarray:
        return self.coords["time"].data

    def __repr__(self):
        lines = [f"SensorData(dims={self.dims})"]
        for k, v in self.coords.items():
            lines.append(f"  coord {k}: {v.dims} {v.data.dtype}")
        for k, v in self.variables.items():
            lines.append(f"  var   {k}: {v.dims} {v.data.dtype}")
        return "\n".join(lines)

    # -------------------------------------------------------------------- IO
    def to_netcdf(self, path: str) -> None:
        write_netcdf(self, path)

    @staticmethod
    def from_netcdf(path: str) -> "SensorData":
        return read_netcdf(path)


# ---------------------------------------------------------------------------
# NetCDF3 (classic/64-bit offset) via scipy
# ---------------------------------------------------------------------------

def _encode(name: str, var: Variable):
    """Map numpy dtype -> (netcdf-storable array, extra dims, attrs)."""
    data = var.data
    attrs = dict(var.attrs)
    dims = list(var.dims)
    if np.issubdtype(data.dtype, np.datetime64):
        minutes = data.astype("datetime64[m]").astype(np.int64).astype(np.float64)
        attrs["units"] = TIME_UNITS
        attrs["_gnnqc_dtype"] = "datetime64[m]"
        return minutes, dims, attrs
    if data.dtype == np.bool_:
        attrs["_gnnqc_dtype"] = "bool"
        return data.astype(np.int8), dims, attrs
    if data.dtype.kind in ("U", "S", "O"):
        strs = np.array([str(s) for s in data.reshape(-1)])
        width = max(1, max((len(s.encode()) for s in strs), default=1))
        arr = np.zeros(strs.shape + (width,), dtype="S1")
        for i, s in enumerate(strs):
            b = s.encode()
            arr[i, : len(b)] = np.frombuffer(b, dtype="S1")
        arr = arr.reshape(data.shape + (width,))
        dims = dims + [f"_strlen_{name}"]
        attrs["_gnnqc_dtype"] = "str"
        return arr, dims, attrs
    if data.dtype == np.int64:
        attrs["_gnnqc_dtype"] = "int64"
        return data.astype(np.float64), dims, attrs
    if data.dtype in (np.float16,):
        return data.astype(np.float32), dims, attrs
    return data, dims, attrs


def _decode(arr: np.ndarray, attrs: dict):
    kind = attrs.pop("_gnnqc_dtype", None)
    if isinstance(kind, bytes):
        kind = kind.decode()
    if kind == "datetime64[m]":
        attrs.pop("units", None)
        return np.asarray(arr).astype(np.int64).astype("datetime64[m]"), False
    if kind == "bool":
        return np.asarray(arr).astype(bool), False
    if kind == "str":
        a = np.asarray(arr)
        flat = a.reshape(-1, a.shape[-1])
        strs = np.array([b"".join(r).decode().rstrip("\x00") for r in flat])
        return strs.reshape(a.shape[:-1]), True
    if kind == "int64":
        return np.asarray(arr).astype(np.int64), False
    return np.array(arr), False


def write_netcdf(ds: SensorData, path: str) -> None:
    from scipy.io import netcdf_file

    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with netcdf_file(path, "w", version=2) as f:
        for k, v in ds.attrs.items():
            setattr(f, k, v if not isinstance(v, (list, tuple)) else np.asarray(v))
        created = set()
        names = {}
        for group, table in (("coord", ds.coords), ("var", ds.variables)):
            for name, var in table.items():
                data, dims, attrs = _encode(name, var)
                for dname, n in zip(dims, data.shape):
                    if dname not in created:
                        f.createDimension(dname, n)
                        created.add(dname)
                # netcdf variable names cannot contain some characters; keep a mapping
                vname = name.replace(" ", "__")
                names[vname] = name
                nv = f.createVariable(vname, data.dtype, tuple(dims))
                nv[...] = data
                nv._gnnqc_group = group
                nv._gnnqc_name = name
                for ak, av in attrs.items():
                    setattr(nv, ak, av)


def read_netcdf(path: str) -> SensorData:
    from scipy.io import netcdf_file

    out = SensorData()
    with netcdf_file(path, "r", mmap=False) as f:
        for k, v in f._attributes.items():
            out.attrs[k] = v.decode() if isinstance(v, bytes) else v
        for vname, nv in f.variables.items():
            attrs = {k: (v.decode() if isinstance(v, bytes) else v) for k, v in nv._attributes.items()}
            group = attrs.pop("_gnnqc_group", "var")
            name = attrs.pop("_gnnqc_name", vname.replace("__", " "))
            dims = list(nv.dimensions)
            data, was_str = _decode(nv.data.copy(), attrs)
            if was_str:
                dims = dims[:-1]
            var = Variable(dims, data, attrs)
            if group == "coord":
                out.coords[name] = var
            else:
                out.variables[name] = var
    return out


__all__ = ["Variable", "SensorData", "write_netcdf", "read_netcdf"]
