"""TensorFlow 1.x checkpoint (tensor bundle V2) reader in pure Python — no TensorFlow needed.

The reference saves and restores every model with ``tf.train.Saver`` (tacotron/train.py,
wavenet_vocoder/train.py:67-86, tacotron/synthesizer.py:93-94), which writes a tensor bundle:

* ``<prefix>.index``: an SSTable (LevelDB table format) mapping each variable name to a
  serialized ``BundleEntryProto`` {dtype, shape, shard_id, offset, size, crc32c}; the empty key
  holds the ``BundleHeaderProto``;
* ``<prefix>.data-SSSSS-of-NNNNN``: the raw little-endian tensor bytes.

This module parses both formats directly (SSTable blocks with prefix-compressed keys + the
protobuf wire format) and returns ``{variable name: numpy array}``, so converted weights can be
fed to ``tt2_load_tensor`` by their TF names.  Snappy-compressed index blocks are not supported
(TF writes bundle indexes uncompressed).
"""
import os
import struct

import numpy as np

_MAGIC = 0xdb4775248b80fb57
# tensorflow/core/framework/types.proto DataType -> numpy
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
           10: np.bool_, 14: np.uint16, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}


class CheckpointError(ValueError):
    pass


def _varint(buf, pos):
    shift = result = 0
    while True:
        if pos >= len(buf):
            raise CheckpointError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _block_handle(buf, pos):
    off, pos = _varint(buf, pos)
    size, pos = _varint(buf, pos)
    return (off, size), pos


def _read_block(data, handle):
    off, size = handle
    if off + size + 5 > len(data):
        raise CheckpointError("block handle past end of file")
    block = data[off:off + size]
    ctype = data[off + size]
    if ctype != 0:
        raise CheckpointError("compressed SSTable block (type %d) is not supported" % ctype)
    return block


def _block_entries(block):
    """Yield (key, value) of one SSTable block (prefix-compressed keys, restart array at the end)."""
    if len(block) < 4:
        raise CheckpointError("short block")
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(block, pos)
        non_shared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos:pos + non_shared]
        pos += non_shared
        yield key, block[pos:pos + vlen]
        pos += vlen


def _proto_fields(buf):
    """Protobuf wire format -> list of (field number, wire type, value)."""
    pos, out = 0, []
    while pos < len(buf):
        tag, pos = _varint(buf, pos)
        field, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise CheckpointError("unsupported protobuf wire type %d" % wt)
        out.append((field, wt, v))
    return out


def _entry(value):
    """BundleEntryProto (tensorflow/core/protobuf/tensor_bundle.proto)."""
    e = dict(dtype=0, shape=[], shard_id=0, offset=0, size=0, slices=False)
    for f, wt, v in _proto_fields(value):
        if f == 1:
            e["dtype"] = v
        elif f == 2:  # TensorShapeProto: repeated Dim dim = 2 {int64 size = 1}
            for f2, _, v2 in _proto_fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, v3 in _proto_fields(v2):
                        if f3 == 1:
                            size = v3 - (1 << 64) if v3 >= 1 << 63 else v3
                    e["shape"].append(size)
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 7:
            e["slices"] = True
    return e


def read_index(prefix):
    """{variable name: BundleEntryProto dict} of ``<prefix>.index`` (header entry excluded) and the
    number of data shards."""
    with open(prefix + ".index", "rb") as f:
        data = f.read()
    if len(data) < 48:
        raise CheckpointError("index file too short")
    footer = data[-48:]
    if struct.unpack_from("<Q", footer, 40)[0] != _MAGIC:
        raise CheckpointError("not an SSTable (bad magic)")
    _, pos = _block_handle(footer, 0)  # metaindex handle (unused)
    index_handle, _ = _block_handle(footer, pos)
    entries, num_shards = {}, 1
    for _, handle_bytes in _block_entries(_read_block(data, index_handle)):
        handle, _ = _block_handle(handle_bytes, 0)
        for key, value in _block_entries(_read_block(data, handle)):
            if key == b"":  # BundleHeaderProto {int32 num_shards = 1; ...}
                for f, _, v in _proto_fields(value):
                    if f == 1:
                        num_shards = v
                continue
            entries[key.decode("utf-8")] = _entry(value)
    return entries, num_shards


def list_variables(prefix):
    """[(name, shape)] like tf.train.list_variables."""
    entries, _ = read_index(prefix)
    return sorted((k, tuple(v["shape"])) for k, v in entries.items())


def read_checkpoint(prefix, names=None):
    """{name: np.ndarray} for every (or the selected) variable of the checkpoint ``prefix``
    (e.g. ``logs-Tacotron/taco_pretrained/tacotron_model.ckpt-100000``)."""
    entries, num_shards = read_index(prefix)
    shards = {}
    out = {}
    for name, e in entries.items():
        if names is not None and name not in names:
            continue
        if e["slices"]:
            raise CheckpointError("partitioned variable %s is not supported" % name)
        if e["dtype"] not in _DTYPES:
            raise CheckpointError("unsupported dtype %d for %s" % (e["dtype"], name))
        sid = e["shard_id"]
        if sid not in shards:
            path = "%s.data-%05d-of-%05d" % (prefix, sid, num_shards)
            if not os.path.exists(path):
                raise CheckpointError("missing data shard " + path)
            shards[sid] = np.memmap(path, dtype=np.uint8, mode="r")
        raw = np.asarray(shards[sid][e["offset"]:e["offset"] + e["size"]])
        dt = np.dtype(_DTYPES[e["dtype"]]).newbyteorder("<")
        arr = np.frombuffer(raw.tobytes(), dtype=dt)
        shape = tuple(e["shape"])
        if arr.size != int(np.prod(shape, dtype=np.int64)):
            raise CheckpointError("size mismatch for %s" % name)
        out[name] = arr.reshape(shape).astype(dt.newbyteorder("="))
    return out


def latest_checkpoint(directory):
    """Prefix named by ``<directory>/checkpoint`` (model_checkpoint_path), like
    tf.train.get_checkpoint_state(...).model_checkpoint_path."""
    with open(os.path.join(directory, "checkpoint")) as f:
        for line in f:
            if line.startswith("model_checkpoint_path:"):
                p = line.split(":", 1)[1].strip().strip('"')
                return p if os.path.isabs(p) else os.path.join(directory, os.path.basename(p))
    raise CheckpointError("no model_checkpoint_path in %s/checkpoint" % directory)
