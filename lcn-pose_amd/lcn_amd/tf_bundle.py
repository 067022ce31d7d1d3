"""TensorFlow tensor-bundle (checkpoint V2) files without TensorFlow.

The reference saves with ``tf.compat.v1.train.Saver`` (models_att.py:161-162,
256-260, 321-322) and restores with ``Saver.restore`` after
``tf.train.latest_checkpoint`` (:452-461).  A V2 checkpoint ``<prefix>`` is

* ``<prefix>.index`` -- a LevelDB-format table (TensorFlow's own table
  builder, tensorflow/core/lib/io/table_builder.cc, no compression) whose
  entries are sorted by key: the empty key holds a ``BundleHeaderProto``
  (num_shards, endianness, VersionDef), every other key is a tensor name whose
  value is a ``BundleEntryProto`` (dtype, shape, shard_id, offset, size,
  masked crc32c of the tensor bytes) -- tensorflow/core/protobuf/
  tensor_bundle.proto, tensorflow/core/util/tensor_bundle/tensor_bundle.cc;
* ``<prefix>.data-00000-of-00001`` -- the raw little-endian tensor bytes;
* ``<prefix>.meta`` -- the MetaGraphDef (a serialized TF graph).  It is not
  needed to restore into a graph the program builds itself (what the
  reference does) and is not produced here.

Protobuf messages are encoded / decoded by hand (a handful of varint and
length-delimited fields).  CRC-32C comes from liblcn (lcn_crc32c).  Parity
with real TensorFlow files is unpinned: TensorFlow is not installed here and
the reference ships no checkpoint; the format follows the public
specification above and is checked by round trips, known-answer CRCs and a
strict reader.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterator, List, Tuple

import numpy as np

MAGIC = 0xDB4775248B80FB57
BLOCK_RESTART_INTERVAL = 16      # table_options.h
BLOCK_SIZE = 262144              # table_options.h
MAX_ENCODED_HANDLE = 20          # 2 varint64
MASK_DELTA = 0xA282EAD8

# tensorflow/core/framework/types.proto
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_INT64, DT_BOOL = 1, 2, 3, 9, 10
_NP2DT = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.float64): DT_DOUBLE,
          np.dtype(np.int32): DT_INT32, np.dtype(np.int64): DT_INT64, np.dtype(np.bool_): DT_BOOL}
_DT2NP = {v: k for k, v in _NP2DT.items()}


class BundleError(ValueError):
    pass


# ----------------------------------------------------------------------------- crc
def crc32c(data: bytes, crc: int = 0) -> int:
    """leveldb crc32c::Extend(crc, data) (crc32c::Value for crc = 0)."""
    from .native import load_library
    data = bytes(data)
    return int(load_library().lcn_crc32c(crc, data, len(data)))


def mask_crc(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + MASK_DELTA) & 0xFFFFFFFF


def unmask_crc(masked: int) -> int:
    rot = (masked - MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------- protobuf bits
def _varint(v: int) -> bytes:
    if v < 0:
        v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        if pos >= len(buf):
            raise BundleError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise BundleError("varint too long")


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3) + _varint(v) if v else b""


def _field_bytes(num: int, payload: bytes, always: bool = False) -> bytes:
    if not payload and not always:
        return b""
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _parse_fields(buf: bytes) -> Iterator[Tuple[int, int, object]]:
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = buf[pos:pos + n]
            if len(v) != n:
                raise BundleError("truncated field")
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise BundleError(f"unsupported wire type {wt}")
        yield num, wt, v


def encode_header() -> bytes:
    """BundleHeaderProto{num_shards: 1, endianness: LITTLE, version{producer: 1}}."""
    return _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1), always=True)


def encode_entry(dtype: int, shape: Tuple[int, ...], offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_field_bytes(2, _field_varint(1, int(d)), always=True) for d in shape)
    out = _field_varint(1, dtype) + _field_bytes(2, dims, always=True)
    out += _field_varint(4, offset) + _field_varint(5, size)
    out += _varint((6 << 3) | 5) + struct.pack("<I", mask_crc(crc))
    return out


def decode_entry(buf: bytes) -> dict:
    e = {"dtype": 0, "shape": (), "shard_id": 0, "offset": 0, "size": 0, "crc32c": None}
    for num, wt, v in _parse_fields(buf):
        if num == 1:
            e["dtype"] = v
        elif num == 2:
            dims = []
            for dn, _, dv in _parse_fields(v):
                if dn == 2:
                    size = 0
                    for sn, _, sv in _parse_fields(dv):
                        if sn == 1:
                            size = sv
                    dims.append(size)
                elif dn == 3 and dv:
                    raise BundleError("unknown-rank tensor in checkpoint")
            e["shape"] = tuple(dims)
        elif num == 3:
            e["shard_id"] = v
        elif num == 4:
            e["offset"] = v
        elif num == 5:
            e["size"] = v
        elif num == 6:
            e["crc32c"] = v
        elif num == 7:
            raise BundleError("sliced (partitioned) tensors are not supported")
    return e


def decode_header(buf: bytes) -> dict:
    h = {"num_shards": 0, "endianness": 0, "producer": 0, "min_consumer": 0}
    for num, _, v in _parse_fields(buf):
        if num == 1:
            h["num_shards"] = v
        elif num == 2:
            h["endianness"] = v
        elif num == 3:
            for vn, _, vv in _parse_fields(v):
                if vn == 1:
                    h["producer"] = vv
                elif vn == 2:
                    h["min_consumer"] = vv
    return h


# ------------------------------------------------------------------ leveldb table
def _shortest_separator(start: bytes, limit: bytes) -> bytes:
    """leveldb BytewiseComparator::FindShortestSeparator."""
    n = min(len(start), len(limit))
    i = 0
    while i < n and start[i] == limit[i]:
        i += 1
    if i >= n:
        return start
    b = start[i]
    if b < 0xFF and b + 1 < limit[i]:
        return start[:i] + bytes([b + 1])
    return start


def _short_successor(key: bytes) -> bytes:
    """leveldb BytewiseComparator::FindShortSuccessor."""
    for i, b in enumerate(key):
        if b != 0xFF:
            return key[:i] + bytes([b + 1])
    return key


class _BlockBuilder:
    def __init__(self, restart_interval: int):
        self.interval = restart_interval
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last = b""

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.counter < self.interval:
            n = min(len(self.last), len(key))
            while shared < n and self.last[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value))
        self.buf += key[shared:] + value
        self.last = key
        self.counter += 1

    def size_estimate(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))

    def empty(self) -> bool:
        return not self.buf


def _write_block(f, contents: bytes) -> Tuple[int, int]:
    off = f.tell()
    f.write(contents)
    crc = crc32c(b"\x00", crc32c(contents))
    f.write(b"\x00" + struct.pack("<I", mask_crc(crc)))
    return off, len(contents)


def write_table(path: str, items: List[Tuple[bytes, bytes]]) -> None:
    """TableBuilder (no compression) over key-sorted items."""
    keys = [k for k, _ in items]
    if keys != sorted(keys) or len(set(keys)) != len(keys):
        raise BundleError("table keys must be unique and sorted")
    with open(path, "wb") as f:
        index = _BlockBuilder(1)
        data = _BlockBuilder(BLOCK_RESTART_INTERVAL)
        pending = None  # handle of the last flushed data block, awaiting its index key
        last_key = b""
        for k, v in items:
            if pending is not None:
                index.add(_shortest_separator(last_key, k), pending)
                pending = None
            data.add(k, v)
            last_key = k
            if data.size_estimate() >= BLOCK_SIZE:
                off, size = _write_block(f, data.finish())
                pending = _varint(off) + _varint(size)
                data = _BlockBuilder(BLOCK_RESTART_INTERVAL)
        if not data.empty():
            off, size = _write_block(f, data.finish())
            pending = _varint(off) + _varint(size)
        if pending is not None:
            index.add(_short_successor(last_key), pending)
        meta_off, meta_size = _write_block(f, _BlockBuilder(BLOCK_RESTART_INTERVAL).finish())
        idx_off, idx_size = _write_block(f, index.finish())
        footer = _varint(meta_off) + _varint(meta_size) + _varint(idx_off) + _varint(idx_size)
        footer += b"\x00" * (2 * MAX_ENCODED_HANDLE - len(footer))
        footer += struct.pack("<Q", MAGIC)
        f.write(footer)


def _read_block(raw: bytes, off: int, size: int) -> bytes:
    contents = raw[off:off + size]
    trailer = raw[off + size:off + size + 5]
    if len(contents) != size or len(trailer) != 5:
        raise BundleError("truncated table block")
    if trailer[0] != 0:
        raise BundleError(f"compressed table block (type {trailer[0]}) is not supported")
    want = unmask_crc(struct.unpack("<I", trailer[1:])[0])
    if crc32c(trailer[:1], crc32c(contents)) != want:
        raise BundleError("table block checksum mismatch")
    return contents


def _block_entries(block: bytes) -> Iterator[Tuple[bytes, bytes]]:
    if len(block) < 4:
        raise BundleError("bad block")
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * nrest
    if limit < 0:
        raise BundleError("bad restart array")
    pos, key = 0, b""
    while pos < limit:
        shared, pos = _read_varint(block, pos)
        nons, pos = _read_varint(block, pos)
        vlen, pos = _read_varint(block, pos)
        if shared > len(key):
            raise BundleError("bad key prefix")
        key = key[:shared] + block[pos:pos + nons]
        pos += nons
        yield key, block[pos:pos + vlen]
        pos += vlen


def read_table(path: str) -> List[Tuple[bytes, bytes]]:
    raw = open(path, "rb").read()
    if len(raw) < 48 or struct.unpack_from("<Q", raw, len(raw) - 8)[0] != MAGIC:
        raise BundleError(f"{path}: not a table (bad magic)")
    foot = raw[len(raw) - 48:len(raw) - 8]
    _, p = _read_varint(foot, 0)
    _, p = _read_varint(foot, p)
    idx_off, p = _read_varint(foot, p)
    idx_size, p = _read_varint(foot, p)
    out = []
    for _, handle in _block_entries(_read_block(raw, idx_off, idx_size)):
        off, q = _read_varint(handle, 0)
        size, _ = _read_varint(handle, q)
        out.extend(_block_entries(_read_block(raw, off, size)))
    return out


# ------------------------------------------------------------------------ bundle
def data_path(prefix: str) -> str:
    return prefix + ".data-00000-of-00001"


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> None:
    """Write <prefix>.index / .data-00000-of-00001 (one shard, little endian)."""
    entries = []
    tmp_data, tmp_index = data_path(prefix) + ".tmp", prefix + ".index.tmp"
    with open(tmp_data, "wb") as f:
        off = 0
        for name in sorted(tensors):
            a = np.asarray(tensors[name])
            if a.ndim:  # (ascontiguousarray would turn a scalar into shape (1,))
                a = np.ascontiguousarray(a)
            if a.dtype not in _NP2DT:
                raise BundleError(f"{name}: unsupported dtype {a.dtype}")
            a = a.astype(a.dtype.newbyteorder("<"), copy=False)
            b = a.tobytes()
            f.write(b)
            entries.append((name.encode(), encode_entry(_NP2DT[a.dtype], a.shape, off, len(b),
                                                        crc32c(b))))
            off += len(b)
    write_table(tmp_index, [(b"", encode_header())] + entries)
    os.replace(tmp_data, data_path(prefix))
    os.replace(tmp_index, prefix + ".index")


def list_bundle(prefix: str) -> Dict[str, dict]:
    items = read_table(prefix + ".index")
    if not items or items[0][0] != b"":
        raise BundleError("missing bundle header")
    h = decode_header(items[0][1])
    if h["num_shards"] != 1 or h["endianness"] != 0:
        raise BundleError(f"unsupported bundle header {h}")
    return {k.decode(): decode_entry(v) for k, v in items[1:]}


def read_bundle(prefix: str, names=None) -> Dict[str, np.ndarray]:
    """Tensors of the checkpoint (all, or `names`), checksums verified."""
    entries = list_bundle(prefix)
    out = {}
    with open(data_path(prefix), "rb") as f:
        for name, e in entries.items():
            if names is not None and name not in names:
                continue
            if e["dtype"] not in _DT2NP:
                raise BundleError(f"{name}: unsupported dtype {e['dtype']}")
            f.seek(e["offset"])
            b = f.read(e["size"])
            if len(b) != e["size"]:
                raise BundleError(f"{name}: truncated data")
            if e["crc32c"] is not None and crc32c(b) != unmask_crc(e["crc32c"]):
                raise BundleError(f"{name}: data checksum mismatch")
            out[name] = np.frombuffer(b, _DT2NP[e["dtype"]].newbyteorder("<")).reshape(e["shape"])
    return out


def print_tensors_in_checkpoint_file(file_name: str, tensor_name: str = "",
                                     all_tensors: bool = False) -> None:
    """tools/checkpoint_analysis.py's call (inspect_checkpoint): names, dtypes
    and shapes of every tensor, or the value of one / all of them."""
    entries = list_bundle(file_name)
    if tensor_name:
        print(tensor_name)
        print(read_bundle(file_name, {tensor_name})[tensor_name])
        return
    for name, e in entries.items():
        dt = _DT2NP.get(e["dtype"], e["dtype"])
        print(f"tensor_name:  {name} ({dt}) {list(e['shape'])}")
        if all_tensors:
            print(read_bundle(file_name, {name})[name])


if __name__ == "__main__":
    import sys
    print_tensors_in_checkpoint_file(sys.argv[1], *(sys.argv[2:3]))
