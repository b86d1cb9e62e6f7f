"""TensorFlow TensorBundle (``variables.index`` + ``variables.data-*``) reader/writer.

The reference saves Keras SavedModels whose weights live in a TensorBundle
(SURVEY §5.4): the ``.index`` file is a LevelDB-format SSTable mapping
checkpoint keys (``variables/0/.ATTRIBUTES/VARIABLE_VALUE`` ...) to
``BundleEntryProto`` records (dtype, shape, shard, offset, size, crc32c); the
``.data-00000-of-00001`` shard holds the raw little-endian tensor bytes.

This module implements both directions without TensorFlow:

* :func:`read_bundle` - parse the SSTable (footer, index block, data blocks with
  prefix-compressed keys and restart arrays), decode the protobuf records by hand,
  verify the masked CRC32C of every tensor and return ``{key: numpy array}``
  (strings as ``bytes``). Nothing in the files is executed or unpickled.
* :func:`write_bundle` - write a compatible pair (uncompressed blocks, restart
  interval 16, header entry under the empty key) so checkpoints of this framework
  use the same on-disk layout.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, List, Tuple

import numpy as np

from ..utils.native import crc32c, masked_crc32c

TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER_LEN = 48
BLOCK_TRAILER = 5

# tensorflow/core/framework/types.proto
DT_TO_NP = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
            10: np.bool_, 14: None, 19: np.float16, 17: np.uint16, 22: np.uint32, 23: np.uint64}
NP_TO_DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
            np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
            np.dtype(np.float16): 19}
DT_STRING = 7


# ----------------------------------------------------------------- varints / protobuf
def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    result = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _enc_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _proto_fields(buf: bytes):
    """Yield (field_number, wire_type, value) for a serialized protobuf message."""
    pos = 0
    while pos < len(buf):
        key, pos = _varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fn, wt, v


def _pb_key(fn, wt):
    return _enc_varint((fn << 3) | wt)


def _pb_bytes(fn, b: bytes):
    return _pb_key(fn, 2) + _enc_varint(len(b)) + b


def _pb_varint(fn, v):
    return _pb_key(fn, 0) + _enc_varint(v)


def decode_entry(buf: bytes) -> dict:
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None}
    for fn, wt, v in _proto_fields(buf):
        if fn == 1:
            e["dtype"] = v
        elif fn == 2:
            dims = []
            for f2, _, v2 in _proto_fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, v3 in _proto_fields(v2):
                        if f3 == 1:
                            size = v3 if v3 < (1 << 63) else v3 - (1 << 64)
                    dims.append(size)
            e["shape"] = dims
        elif fn == 3:
            e["shard_id"] = v
        elif fn == 4:
            e["offset"] = v
        elif fn == 5:
            e["size"] = v
        elif fn == 6:
            e["crc32c"] = v
    return e


def encode_entry(dtype: int, shape, offset: int, size: int, crc: int, shard: int = 0) -> bytes:
    dims = b"".join(_pb_bytes(2, _pb_varint(1, int(d))) for d in shape)
    out = _pb_varint(1, dtype) + _pb_bytes(2, dims)
    if shard:
        out += _pb_varint(3, shard)
    if offset:
        out += _pb_varint(4, offset)
    out += _pb_varint(5, size)
    out += _pb_key(6, 5) + struct.pack("<I", crc)
    return out


# ----------------------------------------------------------------- SSTable
def _read_block(data: bytes, offset: int, size: int) -> List[Tuple[bytes, bytes]]:
    block = data[offset:offset + size]
    ctype = data[offset + size]
    if ctype != 0:
        raise ValueError(f"compressed SSTable block (type {ctype}) not supported")
    n_restarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * n_restarts
    pos = 0
    key = b""
    out = []
    while pos < end:
        shared, pos = _varint(block, pos)
        non_shared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos:pos + non_shared]
        pos += non_shared
        out.append((key, block[pos:pos + vlen]))
        pos += vlen
    return out


def read_sstable(path: str) -> List[Tuple[bytes, bytes]]:
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < FOOTER_LEN:
        raise ValueError("file too small for an SSTable")
    footer = data[-FOOTER_LEN:]
    magic = struct.unpack_from("<Q", footer, FOOTER_LEN - 8)[0]
    if magic != TABLE_MAGIC:
        raise ValueError("bad SSTable magic")
    pos = 0
    _meta_off, pos = _varint(footer, pos)
    _meta_size, pos = _varint(footer, pos)
    idx_off, pos = _varint(footer, pos)
    idx_size, pos = _varint(footer, pos)
    entries = []
    for _k, handle in _read_block(data, idx_off, idx_size):
        off, p2 = _varint(handle, 0)
        size, _ = _varint(handle, p2)
        entries.extend(_read_block(data, off, size))
    return entries


class _BlockBuilder:
    def __init__(self, restart_interval: int = 16):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""
        self.interval = restart_interval

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.counter < self.interval:
            n = min(len(key), len(self.last))
            while shared < n and key[shared] == self.last[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _enc_varint(shared) + _enc_varint(len(key) - shared) + _enc_varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def finish(self) -> bytes:
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))

    def __len__(self):
        return len(self.buf)


def write_sstable(path: str, items: List[Tuple[bytes, bytes]], block_size: int = 4096):
    items = sorted(items, key=lambda kv: kv[0])
    out = bytearray()
    index = _BlockBuilder(restart_interval=1)

    def flush(bb: _BlockBuilder, last_key: bytes):
        raw = bb.finish()
        off = len(out)
        out.extend(raw)
        trailer_type = b"\x00"
        out.extend(trailer_type + struct.pack("<I", masked_crc32c(raw + trailer_type)))
        index.add(last_key, _enc_varint(off) + _enc_varint(len(raw)))

    bb = _BlockBuilder()
    last = b""
    for k, v in items:
        bb.add(k, v)
        last = k
        if len(bb) >= block_size:
            flush(bb, last)
            bb = _BlockBuilder()
    if bb.counter or not items:
        flush(bb, last)
    # empty metaindex block
    meta = _BlockBuilder().finish()
    meta_off = len(out)
    out.extend(meta + b"\x00" + struct.pack("<I", masked_crc32c(meta + b"\x00")))
    idx = index.finish()
    idx_off = len(out)
    out.extend(idx + b"\x00" + struct.pack("<I", masked_crc32c(idx + b"\x00")))
    footer = _enc_varint(meta_off) + _enc_varint(len(meta)) + _enc_varint(idx_off) + _enc_varint(len(idx))
    footer = footer + b"\x00" * (FOOTER_LEN - 8 - len(footer)) + struct.pack("<Q", TABLE_MAGIC)
    out.extend(footer)
    with open(path, "wb") as f:
        f.write(bytes(out))


# ----------------------------------------------------------------- bundle
def _decode_strings(raw: bytes, n: int):
    pos = 0
    lens = []
    for _ in range(n):
        ln, pos = _varint(raw, pos)
        lens.append(ln)
    pos += 4   # crc32c of the length varints
    out = []
    for ln in lens:
        out.append(raw[pos:pos + ln])
        pos += ln
    return out


def _string_crc(raw: bytes, n: int) -> int:
    """TF's string-tensor checksum: CRC32C over each length as little-endian uint32,
    then the 4 stored length-checksum bytes, then the string bytes; stored masked."""
    pos = 0
    lens = []
    for _ in range(n):
        ln, pos = _varint(raw, pos)
        lens.append(ln)
    c = crc32c(raw[pos:], crc32c(b"".join(struct.pack("<I", ln) for ln in lens)))
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _encode_strings(vals: List[bytes]) -> Tuple[bytes, int]:
    lens = b"".join(_enc_varint(len(v)) for v in vals)
    lcrc = masked_crc32c(b"".join(struct.pack("<I", len(v)) for v in vals))
    raw = lens + struct.pack("<I", lcrc) + b"".join(vals)
    return raw, _string_crc(raw, len(vals))


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, object]:
    """``prefix`` like ``model_cml/variables/variables`` -> {key: array | bytes | list}."""
    entries = read_sstable(prefix + ".index")
    header = None
    table = {}
    for k, v in entries:
        if k == b"":
            header = {fn: val for fn, _, val in _proto_fields(v)}
            continue
        table[k.decode()] = decode_entry(v)
    n_shards = header.get(1, 1) if header else 1
    shards = {}
    out: Dict[str, object] = {}
    for key, e in table.items():
        sid = e["shard_id"]
        if sid not in shards:
            with open(f"{prefix}.data-{sid:05d}-of-{n_shards:05d}", "rb") as f:
                shards[sid] = f.read()
        raw = shards[sid][e["offset"]:e["offset"] + e["size"]]
        shape = tuple(e["shape"])
        n = int(np.prod(shape)) if shape else 1
        if verify and e["crc32c"] is not None:
            got = _string_crc(raw, n) if e["dtype"] == DT_STRING else masked_crc32c(raw)
            if got != e["crc32c"]:
                raise ValueError(f"crc mismatch for {key}")
        if e["dtype"] == DT_STRING:
            vals = _decode_strings(raw, n)
            out[key] = vals[0] if not shape else vals
        else:
            dt = DT_TO_NP.get(e["dtype"])
            if dt is None:
                raise ValueError(f"unsupported dtype {e['dtype']} for {key}")
            out[key] = np.frombuffer(raw, dtype=np.dtype(dt).newbyteorder("<")).reshape(shape).copy()
    return out


def bundle_entries(prefix: str) -> Dict[str, dict]:
    """Raw entry metadata (dtype, shape, offset, size, crc) per key."""
    return {k.decode(): decode_entry(v) for k, v in read_sstable(prefix + ".index") if k}


def write_bundle(prefix: str, tensors: Dict[str, object]):
    """Write ``{key: ndarray | bytes | str}`` as ``prefix.index`` + ``prefix.data-00000-of-00001``."""
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    data = bytearray()
    items = []
    for key in sorted(tensors):
        val = tensors[key]
        if isinstance(val, (bytes, str)):
            b = val.encode() if isinstance(val, str) else val
            raw, crc = _encode_strings([b])
            dtype, shape = DT_STRING, ()
        else:
            arr = np.asarray(val)
            # (np.ascontiguousarray promotes a 0-d array to shape (1,): scalars such as
            # optimizer/_iterations keep the reference's shape [] instead)
            arr = np.ascontiguousarray(arr) if arr.ndim else arr.copy()
            if arr.dtype not in NP_TO_DT:
                arr = arr.astype(np.float32)
            raw = arr.astype(arr.dtype.newbyteorder("<")).tobytes()
            dtype, shape = NP_TO_DT[arr.dtype], arr.shape
            crc = masked_crc32c(raw)
        off = len(data)
        data.extend(raw)
        items.append((key.encode(), encode_entry(dtype, shape, off, len(raw), crc)))
    # header: num_shards = 1, endianness LITTLE (0), version {producer: 1}
    header = _pb_varint(1, 1) + _pb_bytes(3, _pb_varint(1, 1))
    items.append((b"", header))
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    write_sstable(prefix + ".index", items)


__all__ = ["read_bundle", "write_bundle", "bundle_entries", "read_sstable", "write_sstable"]
