"""The reference's weight files: tf.keras `save_weights` / `load_weights`
in TensorFlow's checkpoint format (model/tensorflow/model.py:190-212,
`ConfigPath.model_prefix` = "model", config.py:118), read and written
without TensorFlow.

TF 2.7.1 (the reference's pin) is not installed here and the reference ships
no checkpoint, so this restates the published format and is PARITY
UNPINNED against a file TensorFlow wrote (only crc32c is pinned, to the RFC
3720 vectors; tests/test_tf_checkpoint_cpu.py):

* `<prefix>.index` -- a LevelDB-format table (TF's lib/io/table): data
  blocks of prefix-compressed, sorted keys with restart points, an index
  block, a metaindex block and a 48-byte footer (two block handles padded to
  40 bytes + magic 0xdb4775248b80fb57); each block has a 5-byte trailer
  (compression type, masked crc32c).  Key "" holds a BundleHeaderProto
  (num_shards, endianness, version); every other key is a tensor's
  checkpoint key with a BundleEntryProto (dtype, shape, shard, offset,
  size, masked crc32c of the bytes).  Snappy-compressed blocks are read;
  blocks are written uncompressed (a reader accepts either).
* `<prefix>.data-00000-of-00001` -- the tensors' bytes back to back
  (little-endian; a string tensor is varint64 lengths, the masked crc32c
  of those lengths as uint32 words, then the bytes; its entry checksum runs
  on over the masked checksum and the bytes, as TF's WriteStringTensor).
* `_CHECKPOINTABLE_OBJECT_GRAPH` -- a TrackableObjectGraph proto (scalar
  string tensor): the object tree from the model, whose variables'
  checkpoint keys are their attribute paths.  For the reference's
  subclassed PolicyValueModel that is e.g.
  `residual_tower/conv_blocks/1/inner_conv_2/conv_layer/kernel/.ATTRIBUTES/VARIABLE_VALUE`
  (`keras_keys` below).  The writer emits the tree down to the network's
  variables; the optimizer's state (SGD iterations, momentum slots) is not
  held by this package and is neither read nor written.

The protos are encoded by hand (protobuf wire format), the python-protobuf
package has no TF message classes.
"""
import os
import struct

import numpy as np

MAGIC = 0xDB4775248B80FB57
DATA_SUFFIX = ".data-00000-of-00001"
OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
VAR_SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"

# TF DataType enum (types.proto) <-> numpy
DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8,
      9: np.int64, 10: np.bool_, 19: np.float16}
DT_STRING = 7
NP_DT = {np.dtype(v): k for k, v in DT.items()}


# ------------------------------------------------------------------ crc32c
def _crc_table():
    t = np.zeros(256, np.uint32)
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        t[i] = c
    return t


_T = _crc_table()
_TL = [int(x) for x in _T]
_SHIFT = {}


def _raw_bytes(r, data):
    for b in data:
        r = _TL[(r ^ b) & 0xFF] ^ (r >> 8)
    return r


def _shift_tables(n):
    """The register map `feed n zero bytes` (linear over GF(2)) as 4 byte tables."""
    if n not in _SHIFT:
        basis = [_raw_bytes(1 << k, bytes(n)) for k in range(32)]
        tabs = []
        for byte in range(4):
            tab = [0] * 256
            for v in range(1, 256):
                low = v & -v
                tab[v] = tab[v ^ low] ^ basis[8 * byte + low.bit_length() - 1]
            tabs.append(tab)
        _SHIFT[n] = tabs
    return _SHIFT[n]


def crc32c(data: bytes) -> int:
    """CRC-32C (Castagnoli, reflected 0x82F63B78, init and xor-out ~0).
    Large inputs run as 4096 chunks in lock step (numpy) whose registers are
    then folded: raw(A || B, r) = zeros_|B|(raw(A, r)) ^ raw(B, 0)."""
    data = bytes(data)
    n = len(data)
    r = 0xFFFFFFFF
    chunks = 4096
    L = n // chunks
    if L >= 16:
        a = np.frombuffer(data, np.uint8, count=L * chunks).reshape(chunks, L)
        reg = np.zeros(chunks, np.uint32)
        for j in range(L):
            reg = _T[(reg ^ a[:, j]) & 0xFF] ^ (reg >> 8)
        t0, t1, t2, t3 = _shift_tables(L)
        for c in reg.tolist():
            r = t0[r & 0xFF] ^ t1[(r >> 8) & 0xFF] ^ t2[(r >> 16) & 0xFF] ^ t3[r >> 24] ^ c
        data = data[L * chunks:]
    return _raw_bytes(r, data) ^ 0xFFFFFFFF


def mask(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask(m: int) -> int:
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------ wire format
def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = v = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7


def _fields(buf):
    """Protobuf message -> list of (field number, wire type, value)."""
    pos, out = 0, []
    while pos < len(buf):
        tag, pos = _read_varint(buf, pos)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            ln, pos = _read_varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            pos += ln
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"protobuf wire type {wt} not supported")
        out.append((f, wt, v))
    return out


def _pb_varint(f, v):
    return _varint(f << 3) + _varint(v) if v else b""


def _pb_bytes(f, b):
    return _varint((f << 3) | 2) + _varint(len(b)) + b


def _pb_fixed32(f, v):
    return _varint((f << 3) | 5) + struct.pack("<I", v)


def _entry_proto(dtype, shape, offset, size, crc):
    shape_pb = b"".join(_pb_bytes(2, _pb_varint(1, d) if d else b"") for d in shape)
    return (_pb_varint(1, dtype) + _pb_bytes(2, shape_pb) + _pb_varint(4, offset)
            + _pb_varint(5, size) + _pb_fixed32(6, mask(crc)))


def _parse_entry(buf):
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None}
    for f, _, v in _fields(buf):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            for g, _, dim in _fields(v):
                if g == 2:
                    size = [x for h, _, x in _fields(dim) if h == 1]
                    e["shape"].append(int(size[0]) if size else 0)
                elif g == 3 and dim:
                    raise ValueError("tensor of unknown rank")
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = unmask(v)
        elif f == 7:
            raise ValueError("partitioned (sliced) variables are not supported")
    return e


# ------------------------------------------------------------------ snappy
def snappy_decompress(buf: bytes) -> bytes:
    """Snappy raw format: varint length, then literals and back-copies."""
    n, pos = _read_varint(buf, 0)
    out = bytearray()
    while pos < len(buf):
        tag = buf[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += buf[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 4], "little")
            pos += 4
        if off == 0 or off > len(out):
            raise ValueError("snappy: bad copy offset")
        for _ in range(ln):  # copies may overlap their own output
            out.append(out[-off])
    if len(out) != n:
        raise ValueError("snappy: length mismatch")
    return bytes(out)


# ------------------------------------------------------------------ table
def _read_block(f, offset, size):
    f.seek(offset)
    raw = f.read(size + 5)
    data, ctype, crc = raw[:size], raw[size], struct.unpack("<I", raw[size + 1:size + 5])[0]
    if crc32c(raw[:size + 1]) != unmask(crc):
        raise ValueError("index block checksum mismatch")
    if ctype == 1:
        return snappy_decompress(data)
    if ctype != 0:
        raise ValueError(f"block compression {ctype} not supported")
    return data


def _block_entries(block):
    nrest = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    pos, key, out = 0, b"", []
    while pos < end:
        shared, pos = _read_varint(block, pos)
        nonshared, pos = _read_varint(block, pos)
        vlen, pos = _read_varint(block, pos)
        key = key[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        out.append((key, block[pos:pos + vlen]))
        pos += vlen
    return out


def _handle(buf, pos=0):
    off, pos = _read_varint(buf, pos)
    size, pos = _read_varint(buf, pos)
    return (off, size), pos


def read_table(path):
    """LevelDB-format table -> list of (key bytes, value bytes) in key order."""
    with open(path, "rb") as f:
        f.seek(0, 2)
        n = f.tell()
        if n < 48:
            raise ValueError(f"{path}: too short for a table")
        f.seek(n - 48)
        foot = f.read(48)
        if struct.unpack("<Q", foot[40:])[0] != MAGIC:
            raise ValueError(f"{path}: not a TensorFlow/LevelDB table (bad magic)")
        _meta, pos = _handle(foot)
        index, _ = _handle(foot, pos)
        out = []
        for _, h in _block_entries(_read_block(f, *index)):
            (off, size), _ = _handle(h)
            out += _block_entries(_read_block(f, off, size))
        return out


def _build_block(items, restart_interval=16):
    buf, restarts, prev = bytearray(), [], b""
    for i, (k, v) in enumerate(items):
        shared = 0
        if i % restart_interval == 0:
            restarts.append(len(buf))
        else:
            while shared < min(len(k), len(prev)) and k[shared] == prev[shared]:
                shared += 1
        buf += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += struct.pack("<I", r)
    buf += struct.pack("<I", len(restarts))
    return bytes(buf)


def write_table(path, items, block_size=262144):
    """(key, value) pairs (sorted by key) -> a LevelDB-format table, one data
    block per ~block_size bytes, uncompressed."""
    items = sorted(items)
    with open(path, "wb") as f:
        def emit(block):
            off = f.tell()
            f.write(block)
            f.write(b"\x00" + struct.pack("<I", mask(crc32c(block + b"\x00"))))
            return _varint(off) + _varint(len(block))

        index, cur, cur_bytes = [], [], 0
        for k, v in items:
            cur.append((k, v))
            cur_bytes += len(k) + len(v)
            if cur_bytes >= block_size:
                index.append((cur[-1][0], emit(_build_block(cur))))
                cur, cur_bytes = [], 0
        if cur or not index:
            index.append((cur[-1][0] if cur else b"", emit(_build_block(cur))))
        meta = emit(_build_block([]))
        idx = emit(_build_block(index, restart_interval=1))
        foot = meta + idx
        f.write(foot + bytes(40 - len(foot)) + struct.pack("<Q", MAGIC))


# ------------------------------------------------------------------ bundle
def read_checkpoint(prefix):
    """`<prefix>.index` + data shards -> {checkpoint key: ndarray or bytes}."""
    rows = read_table(prefix + ".index")
    header = dict((f, v) for f, _, v in _fields(rows[0][1])) if rows and rows[0][0] == b"" else {}
    shards = header.get(1, 1)
    if header.get(2, 0) != 0:
        raise ValueError("big-endian checkpoint")
    out = {}
    files = {}
    try:
        for key, val in rows:
            if key == b"":
                continue
            e = _parse_entry(val)
            sid = e["shard_id"]
            if sid not in files:
                files[sid] = open(f"{prefix}.data-{sid:05d}-of-{shards:05d}", "rb")
            fh = files[sid]
            fh.seek(e["offset"])
            raw = fh.read(e["size"])
            if e["dtype"] == DT_STRING:
                val, crc = _decode_strings(raw, e["shape"], key.decode())
                if e["crc32c"] is not None and crc != e["crc32c"]:
                    raise ValueError(f"{key.decode()}: data checksum mismatch")
                out[key.decode()] = val
                continue
            if e["crc32c"] is not None and crc32c(raw) != e["crc32c"]:
                raise ValueError(f"{key.decode()}: data checksum mismatch")
            if e["dtype"] in DT:
                out[key.decode()] = np.frombuffer(raw, DT[e["dtype"]]).reshape(e["shape"]).copy()
            else:
                raise ValueError(f"{key.decode()}: dtype {e['dtype']} not supported")
    finally:
        for fh in files.values():
            fh.close()
    return out


# A string tensor's bytes (TF tensor_bundle.cc WriteStringTensor /
# ReadStringTensor): the varint64 lengths, a masked crc32c, then the strings.
# The masked crc32c covers the lengths as fixed-width little-endian integers
# (uint32, or uint64 for a length past UINT32_MAX), NOT their varint bytes;
# the entry's crc32c continues that same checksum over the 4 masked-checksum
# bytes and then the string bytes.
def _length_words(lens):
    return b"".join(struct.pack("<I", n) if n <= 0xFFFFFFFF else struct.pack("<Q", n) for n in lens)


def _decode_strings(raw, shape, key="string tensor"):
    """-> (value, the entry crc32c TF computes while reading it).

    Also reads the LEGACY layout this package's round-3/4 writer produced
    (the masked crc32c over the lengths' varint bytes, the entry crc32c over
    the raw bytes), so a model saved by those builds still loads: its entry
    checksum is then crc32c(raw), which the caller compares as before."""
    n = int(np.prod(shape)) if shape else 1
    pos, lens = 0, []
    for _ in range(n):
        ln, pos = _read_varint(raw, pos)
        lens.append(ln)
    words = _length_words(lens)
    stored = bytes(raw[pos:pos + 4])
    legacy = False
    if len(stored) != 4 or struct.unpack("<I", stored)[0] != mask(crc32c(words)):
        if len(stored) == 4 and struct.unpack("<I", stored)[0] == mask(crc32c(bytes(raw[:pos]))):
            legacy = True  # the round-3/4 writer: checksum of the varint bytes
        else:
            raise ValueError(f"{key}: string lengths checksum mismatch (neither TensorFlow's layout, the "
                             f"lengths as uint32 words, nor this package's legacy varint-byte layout)")
    pos += 4
    out = []
    for ln in lens:
        out.append(bytes(raw[pos:pos + ln]))
        pos += ln
    if pos != len(raw):
        raise ValueError(f"{key}: string tensor size mismatch")
    crc = crc32c(bytes(raw)) if legacy else crc32c(words + stored + b"".join(out))
    return (out[0] if not shape else out), crc


def _encode_string(b):
    """One scalar string -> (its bytes in the data file, its entry crc32c)."""
    words = _length_words([len(b)])
    stored = struct.pack("<I", mask(crc32c(words)))
    return _varint(len(b)) + stored + b, crc32c(words + stored + b)


def write_checkpoint(prefix, tensors):
    """{checkpoint key: ndarray or bytes (scalar string)} -> `<prefix>.index`
    + `<prefix>.data-00000-of-00001` (one shard, keys in sorted order)."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    entries, off = [], 0
    with open(prefix + DATA_SUFFIX, "wb") as f:
        for key in sorted(tensors):
            t = tensors[key]
            if isinstance(t, (bytes, bytearray)):
                (raw, crc), dtype, shape = _encode_string(bytes(t)), DT_STRING, ()
            else:
                a = np.asarray(t)  # (ascontiguousarray would make a scalar 1-D)
                if a.dtype not in NP_DT:
                    raise ValueError(f"{key}: dtype {a.dtype} not supported")
                raw, dtype, shape = a.astype(a.dtype.newbyteorder("<")).tobytes(), NP_DT[a.dtype], a.shape
                crc = crc32c(raw)
            f.write(raw)
            entries.append((key.encode(), _entry_proto(dtype, shape, off, len(raw), crc)))
            off += len(raw)
    header = _pb_varint(1, 1) + _pb_bytes(3, _pb_varint(1, 1))  # num_shards 1, little endian, version 1
    write_table(prefix + ".index", [(b"", header)] + entries)


# ------------------------------------------------------------------ object graph
def object_graph_keys(graph: bytes):
    """TrackableObjectGraph -> {attribute path: checkpoint key} for every
    variable reachable from the root (node 0)."""
    nodes = []
    for f, _, v in _fields(graph):
        if f != 1:
            continue
        children, attrs = [], []
        for g, _, w in _fields(v):
            if g == 1:
                c = dict((h, x) for h, _, x in _fields(w))
                children.append((c.get(1, 0), c.get(2, b"").decode()))
            elif g == 2:
                a = dict((h, x) for h, _, x in _fields(w))
                attrs.append((a.get(1, b"").decode(), a.get(3, b"").decode()))
        nodes.append((children, attrs))
    out, seen, stack = {}, {0}, [(0, "")]
    while stack:
        nid, path = stack.pop()
        children, attrs = nodes[nid]
        for name, key in attrs:
            if name == "VARIABLE_VALUE":
                out[path] = key
        for cid, local in children:
            if cid not in seen:
                seen.add(cid)
                stack.append((cid, f"{path}/{local}" if path else local))
    return out


def build_object_graph(paths):
    """Variable attribute paths -> a TrackableObjectGraph holding the tree
    down to them (node 0 the model), each variable's key `path + VAR_SUFFIX`."""
    nodes = [{"children": [], "attr": None}]
    index = {"": 0}
    for p in paths:
        parts = p.split("/")
        for i in range(1, len(parts) + 1):
            sub = "/".join(parts[:i])
            if sub not in index:
                index[sub] = len(nodes)
                nodes.append({"children": [], "attr": None})
                parent = "/".join(parts[:i - 1])
                nodes[index[parent]]["children"].append((index[sub], parts[i - 1]))
        nodes[index[p]]["attr"] = p
    out = b""
    for n in nodes:
        body = b"".join(_pb_bytes(1, _pb_varint(1, cid) + _pb_bytes(2, name.encode()))
                        for cid, name in n["children"])
        if n["attr"] is not None:
            full = n["attr"].split("/")[-1] + ":0"
            body += _pb_bytes(2, _pb_bytes(1, b"VARIABLE_VALUE") + _pb_bytes(2, full.encode())
                              + _pb_bytes(3, (n["attr"] + VAR_SUFFIX).encode()))
        out += _pb_bytes(1, body)
    return out


# ------------------------------------------------------------------ the reference model's keys
_KERAS_FIELD = {"kernel": "conv_layer/kernel", "bias": "conv_layer/bias",
                "gamma": "batch_normalization_layer/gamma", "beta": "batch_normalization_layer/beta",
                "mean": "batch_normalization_layer/moving_mean",
                "var": "batch_normalization_layer/moving_variance"}


def keras_path(name: str) -> str:
    """This package's weight name (model/weights.py) -> the attribute path of
    the same variable in the reference's PolicyValueModel
    (model/tensorflow/model.py:21-170, base_layers.py:20-125)."""
    unit, field = name.rsplit(".", 1)
    dense = {"policy.dense": "policy_head/dense", "value.dense1": "value_head/dense_1",
             "value.dense2": "value_head/dense_2"}
    if unit in dense:
        return f"{dense[unit]}/{field}"
    if unit == "stem":
        block = "residual_tower/conv_blocks/0"
    elif unit.startswith("block"):
        d, conv = unit[5:].split(".")
        inner = {"conv1": "inner_conv_1", "conv2": "inner_conv_2", "res": "residual_connexion"}[conv]
        block = f"residual_tower/conv_blocks/{int(d) + 1}/{inner}"
    elif unit in ("policy.conv", "value.conv"):
        block = f"{unit.split('.')[0]}_head/inner_conv"
    else:
        raise KeyError(name)
    return f"{block}/{_KERAS_FIELD[field]}"


def keras_keys(spec):
    return {name: keras_path(name) + VAR_SUFFIX for name, _ in spec}


def save_keras_weights(prefix, spec, weights):
    """`Model.save_weights(prefix)` of the reference model: the network's
    variables under their Keras keys, the object graph, and the directory's
    `checkpoint` state file."""
    keys = keras_keys(spec)
    tensors = {keys[n]: np.asarray(weights[n], np.float32).reshape(s) for n, s in spec}
    tensors[OBJECT_GRAPH_KEY] = build_object_graph([keras_path(n) for n, _ in spec])
    write_checkpoint(prefix, tensors)
    base = os.path.basename(prefix)
    with open(os.path.join(os.path.dirname(prefix) or ".", "checkpoint"), "w") as f:
        f.write(f'model_checkpoint_path: "{base}"\nall_model_checkpoint_paths: "{base}"\n')


def load_keras_weights(prefix, spec):
    """`Model.load_weights(prefix)` for the reference model -> {name: array}.
    Keys come from the checkpoint's object graph when it has one (else the
    attribute-path keys); a missing variable or a shape mismatch raises."""
    tensors = read_checkpoint(prefix)
    by_path = object_graph_keys(tensors[OBJECT_GRAPH_KEY]) if OBJECT_GRAPH_KEY in tensors else {}
    out = {}
    for name, shape in spec:
        path = keras_path(name)
        key = by_path.get(path, path + VAR_SUFFIX)
        if key not in tensors:
            raise KeyError(f"{prefix}: no variable for {name} ({path})")
        a = np.asarray(tensors[key])
        if a.shape != tuple(shape):
            raise ValueError(f"{prefix}: {path} has shape {a.shape}, the model wants {tuple(shape)}")
        out[name] = a.astype(np.float32)
    return out
