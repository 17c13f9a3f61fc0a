"""The reference's weight files without TensorFlow (model/tf_checkpoint.py;
reference: Model.save_weights / load_weights, model/tensorflow/model.py:
190-212).  TF is absent and the reference holds no checkpoint, so the table /
bundle / object-graph layout is parity unpinned: these tests pin crc32c to
RFC 3720's vectors, snappy to hand-assembled streams, and check the rest by
round trips, corruption and mismatch refusals."""
import os
import struct
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "custom-alphazero_amd"))

from custom_alphazero.model import tf_checkpoint as T  # noqa: E402
from custom_alphazero.model.weights import init_weights, weight_spec  # noqa: E402


def test_crc32c_rfc3720_vectors():
    assert T.crc32c(b"123456789") == 0xE3069283
    assert T.crc32c(bytes(32)) == 0x8A9136AA
    assert T.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert T.crc32c(bytes(range(32))) == 0x46DD794E
    assert T.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    assert T.crc32c(b"") == 0


def test_crc32c_chunked_path_equals_bytewise():
    d = np.random.RandomState(1).bytes(4096 * 37 + 123)
    assert T.crc32c(d) == T._raw_bytes(0xFFFFFFFF, d) ^ 0xFFFFFFFF
    for v in (0, 1, 0xDEADBEEF, 0xFFFFFFFF):
        assert T.unmask(T.mask(v)) == v


def _crc32c_bitwise(data, crc=0):
    """CRC-32C bit by bit (an implementation independent of the module's tables);
    `crc` continues an earlier result (crc32c::Extend)."""
    crc ^= 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def _mask_hand(c):
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_string_tensor_follows_tensorflow_layout():
    """TF's WriteStringTensor (tensor_bundle.cc): varint64 lengths, then the
    masked crc32c of the lengths taken as little-endian uint32 words, then the
    bytes; the entry crc32c is that length crc extended over the 4 masked
    bytes and the string bytes.  Hand-assembled here for a 200-byte scalar
    (a 2-byte varint length, so the varint and uint32 forms differ) and a
    3-element vector."""
    s = bytes(range(200))
    lcrc = _crc32c_bitwise(struct.pack("<I", 200))
    masked = struct.pack("<I", _mask_hand(lcrc))
    raw = bytes([0xC8, 0x01]) + masked + s
    entry_crc = _crc32c_bitwise(s, _crc32c_bitwise(masked, lcrc))
    assert T._encode_string(s) == (raw, entry_crc)
    assert T._decode_strings(raw, ()) == (s, entry_crc)
    vec = [b"ab", b"", b"x" * 130]
    lw = struct.pack("<III", 2, 0, 130)
    lcrc = _crc32c_bitwise(lw)
    masked = struct.pack("<I", _mask_hand(lcrc))
    raw = bytes([2, 0, 0x82, 0x01]) + masked + b"".join(vec)
    assert T._decode_strings(raw, (3,)) == (vec, _crc32c_bitwise(b"".join(vec), _crc32c_bitwise(masked, lcrc)))
    bad = bytearray(raw)
    bad[4] ^= 1
    with pytest.raises(ValueError, match="lengths checksum"):
        T._decode_strings(bytes(bad), (3,))


def test_checkpoint_string_entry_carries_the_tensorflow_crc(tmp_path):
    prefix = str(tmp_path / "model")
    g = b"\x0a\x05hello" * 30
    T.write_checkpoint(prefix, {T.OBJECT_GRAPH_KEY: g, "v": np.arange(3, dtype=np.float32)})
    rows = dict(T.read_table(prefix + ".index"))
    e = T._parse_entry(rows[T.OBJECT_GRAPH_KEY.encode()])
    lcrc = _crc32c_bitwise(struct.pack("<I", len(g)))
    masked = struct.pack("<I", _mask_hand(lcrc))
    assert e["crc32c"] == _crc32c_bitwise(g, _crc32c_bitwise(masked, lcrc))
    assert T.read_checkpoint(prefix)[T.OBJECT_GRAPH_KEY] == g


def test_legacy_string_layout_still_loads(tmp_path):
    """A checkpoint written by this package's round-3/4 writer: the
    string tensor's masked crc32c covers the lengths' VARINT bytes and its
    entry crc32c is crc32c of the raw bytes.  Hand-assembled here (a 200-byte
    object graph: the varint and uint32 forms differ) and read back whole."""
    g = bytes(range(200))
    lens = bytes([0xC8, 0x01])
    raw = lens + struct.pack("<I", _mask_hand(_crc32c_bitwise(lens))) + g
    assert T._decode_strings(raw, ()) == (g, _crc32c_bitwise(raw))
    prefix = str(tmp_path / "model")
    v = np.arange(3, dtype=np.float32)
    with open(prefix + T.DATA_SUFFIX, "wb") as f:
        f.write(raw + v.tobytes())
    entries = [(T.OBJECT_GRAPH_KEY.encode(), T._entry_proto(T.DT_STRING, (), 0, len(raw), _crc32c_bitwise(raw))),
               (b"v", T._entry_proto(T.NP_DT[v.dtype], v.shape, len(raw), v.nbytes, _crc32c_bitwise(v.tobytes())))]
    header = T._pb_varint(1, 1) + T._pb_bytes(3, T._pb_varint(1, 1))
    T.write_table(prefix + ".index", [(b"", header)] + sorted(entries))
    out = T.read_checkpoint(prefix)
    assert out[T.OBJECT_GRAPH_KEY] == g
    np.testing.assert_array_equal(out["v"], v)
    # a corrupted legacy entry still fails, naming both layouts
    bad = bytearray(raw)
    bad[2] ^= 1
    with pytest.raises(ValueError, match="legacy"):
        T._decode_strings(bytes(bad), ())


def test_snappy_literals_and_overlapping_copies():
    # "abcd" literal, then a 1-byte-offset copy of 8 from offset 4 (overlaps
    # its own output), then a 2-byte-offset copy of 3 from offset 12
    stream = (T._varint(15) + bytes([(4 - 1) << 2]) + b"abcd"
              + bytes([1 | ((8 - 4) << 2) | (0 << 5)]) + bytes([4])
              + bytes([2 | ((3 - 1) << 2)]) + struct.pack("<H", 12))
    assert T.snappy_decompress(stream) == b"abcdabcdabcdabc"
    long = bytes(range(256)) * 2
    lit = T._varint(len(long)) + bytes([61 << 2]) + struct.pack("<H", len(long) - 1) + long
    assert T.snappy_decompress(lit) == long
    with pytest.raises(ValueError):
        T.snappy_decompress(T._varint(5) + bytes([(4 - 1) << 2]) + b"abcd")


def test_table_roundtrip_over_many_blocks(tmp_path):
    rng = np.random.RandomState(2)
    items = [(f"key/{i:05d}/{'x' * (i % 7)}".encode(), rng.bytes(int(rng.randint(0, 300))))
             for i in range(2000)]
    p = str(tmp_path / "t.index")
    T.write_table(p, items, block_size=4096)
    assert T.read_table(p) == sorted(items)
    T.write_table(p, [])
    assert T.read_table(p) == []


def test_table_reads_snappy_blocks(tmp_path):
    """A table whose blocks are snappy-compressed (type 1), as a writer with
    compression on may leave them."""
    items = [(f"k{i:03d}".encode(), bytes([i]) * 5) for i in range(40)]
    p = str(tmp_path / "s.index")
    with open(p, "wb") as f:
        def emit(block):
            comp = T._varint(len(block)) + bytes([61 << 2]) + struct.pack("<H", len(block) - 1) + block
            off = f.tell()
            f.write(comp + b"\x01" + struct.pack("<I", T.mask(T.crc32c(comp + b"\x01"))))
            return T._varint(off) + T._varint(len(comp))
        h = emit(T._build_block(items))
        meta = emit(T._build_block([]))
        idx = emit(T._build_block([(items[-1][0], h)], restart_interval=1))
        foot = meta + idx
        f.write(foot + bytes(40 - len(foot)) + struct.pack("<Q", T.MAGIC))
    assert T.read_table(p) == items


def test_bundle_roundtrip_dtypes_and_corruption(tmp_path):
    prefix = str(tmp_path / "ck" / "model")
    t = {"a/f32": np.arange(24, dtype=np.float32).reshape(2, 3, 4), "b/f64": np.array([1.5, -2.0]),
         "c/i64": np.array(7, np.int64), "d/empty": np.zeros((0, 3), np.float32),
         "e/str": b"\x00object graph\xff"}
    T.write_checkpoint(prefix, t)
    assert os.path.exists(prefix + ".index") and os.path.exists(prefix + T.DATA_SUFFIX)
    got = T.read_checkpoint(prefix)
    assert set(got) == set(t)
    for k, v in t.items():
        if isinstance(v, bytes):
            assert got[k] == v
        else:
            assert got[k].dtype == v.dtype and got[k].shape == v.shape
            np.testing.assert_array_equal(got[k], v)
    raw = bytearray(open(prefix + T.DATA_SUFFIX, "rb").read())
    raw[5] ^= 1
    open(prefix + T.DATA_SUFFIX, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="checksum"):
        T.read_checkpoint(prefix)
    idx = bytearray(open(prefix + ".index", "rb").read())
    idx[-1] ^= 1
    open(prefix + ".index", "wb").write(bytes(idx))
    with pytest.raises(ValueError, match="magic"):
        T.read_checkpoint(prefix)


def test_keras_keys_follow_the_reference_attributes():
    spec = weight_spec(6, 7, 7, depth=4)
    keys = T.keras_keys(spec)
    assert len(set(keys.values())) == len(spec)
    s = T.VAR_SUFFIX
    assert keys["stem.kernel"] == "residual_tower/conv_blocks/0/conv_layer/kernel" + s
    assert keys["stem.mean"] == "residual_tower/conv_blocks/0/batch_normalization_layer/moving_mean" + s
    assert keys["block0.conv1.gamma"] == "residual_tower/conv_blocks/1/inner_conv_1/batch_normalization_layer/gamma" + s
    assert keys["block3.conv2.bias"] == "residual_tower/conv_blocks/4/inner_conv_2/conv_layer/bias" + s
    assert keys["block2.res.var"] == ("residual_tower/conv_blocks/3/residual_connexion/"
                                      "batch_normalization_layer/moving_variance" + s)
    assert keys["policy.conv.kernel"] == "policy_head/inner_conv/conv_layer/kernel" + s
    assert keys["policy.dense.kernel"] == "policy_head/dense/kernel" + s
    assert keys["value.dense1.bias"] == "value_head/dense_1/bias" + s
    assert keys["value.dense2.kernel"] == "value_head/dense_2/kernel" + s


def test_object_graph_roundtrip():
    paths = [T.keras_path(n) for n, _ in weight_spec(6, 7, 7, depth=2)]
    g = T.build_object_graph(paths)
    assert T.object_graph_keys(g) == {p: p + T.VAR_SUFFIX for p in paths}


def test_keras_weights_roundtrip_and_refusals(tmp_path):
    spec = weight_spec(6, 7, 7, depth=4)
    w = init_weights(spec, seed=4, randomize_bn=True)
    prefix = str(tmp_path / "model")
    T.save_keras_weights(prefix, spec, w)
    assert open(tmp_path / "checkpoint").read().startswith('model_checkpoint_path: "model"')
    got = T.load_keras_weights(prefix, spec)
    for n, _ in spec:
        np.testing.assert_array_equal(got[n], w[n])
    with pytest.raises(ValueError, match="shape"):
        T.load_keras_weights(prefix, weight_spec(6, 7, 7, filters=64, depth=4))
    with pytest.raises(KeyError):
        T.load_keras_weights(prefix, weight_spec(6, 7, 7, depth=5))


def test_load_follows_the_object_graph_keys(tmp_path):
    """Variables are found through the checkpoint's object graph, not by
    guessing their key strings: a graph that stores a variable under another
    key is followed."""
    spec = weight_spec(5, 5, 5, depth=1)
    w = init_weights(spec, seed=6)
    paths = [T.keras_path(n) for n, _ in spec]
    graph = T.build_object_graph(paths)
    stem = T.keras_path("stem.kernel") + T.VAR_SUFFIX
    graph = graph.replace(stem.encode(), b"renamed" + stem.encode()[7:])
    tensors = {T.keras_path(n) + T.VAR_SUFFIX: w[n] for n, _ in spec}
    tensors["renamed" + stem[7:]] = tensors.pop(stem)
    tensors[T.OBJECT_GRAPH_KEY] = graph
    T.write_checkpoint(str(tmp_path / "model"), tensors)
    got = T.load_keras_weights(str(tmp_path / "model"), spec)
    np.testing.assert_array_equal(got["stem.kernel"], w["stem.kernel"])
