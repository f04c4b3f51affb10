"""Edgestore entry codec, CPU side.

1. The Python restatement of VariableLong (oracle/edgecodec.py) against the reference's own
   known-answer tests, janusgraph-test/.../graphdb/idmanagement/VariableLongTest.java:
   readWriteTest :42-94 (values written in sequence, read back in order — backward encodings from
   the end — with the encoded length checked for every value, then the 0 / Long.MAX_VALUE
   boundaries), at the ranges of testPosBackwardWrite{Small,Big} :129-137 and
   testPrefix{1,2,3}Write* :149-167 (sampled with a coarser jump where a full Python walk would be
   slow), and byteOrderPreservingPositiveBackward :287-300.
2. The C oracle decoder (jo_decode_edges, EdgeSerializer.parseRelation :86-122) recovers every field
   of entries the restated writer (EdgeSerializer.writeRelation :239-303) produced: every
   multiplicity, both directions, sort keys, trailing values, property and system entries.
"""
import numpy as np

from oracle import edgecodec as ec

LONG_MAX = (1 << 63) - 1


def _read_write_backward(max_value, jump):
    values = list(range(0, max_value + 1, jump))
    buf = b"".join(ec.write_positive_backward(v) for v in values)
    pos = len(buf)
    for v in reversed(values):
        got, npos = ec.read_positive_backward(buf, pos)
        assert got == v
        assert pos - npos == ec.backward_length(v)
        pos = npos
    assert pos == 0
    buf = ec.write_positive_backward(0) + ec.write_positive_backward(LONG_MAX)
    got, pos = ec.read_positive_backward(buf, len(buf))
    assert got == LONG_MAX
    assert ec.read_positive_backward(buf, pos)[0] == 0


def _read_write_prefix(max_value, jump, prefix_len, prefix):
    values = list(range(0, max_value + 1, jump))
    buf = b"".join(ec.write_positive_with_prefix(v, prefix, prefix_len) for v in values)
    pos = 0
    for v in values:
        got, p, npos = ec.read_positive_with_prefix(buf, pos, prefix_len)
        assert (got, p) == (v, prefix)
        # positiveWithPrefixLength = numVariableBlocks(bitLength(v) + prefixLen)
        assert npos - pos == (max(v.bit_length(), 1) + prefix_len - 1) // 7 + 1
        pos = npos
    buf = ec.write_positive_with_prefix(0, prefix, prefix_len) + ec.write_positive_with_prefix(LONG_MAX, prefix,
                                                                                               prefix_len)
    v0, _, pos = ec.read_positive_with_prefix(buf, 0, prefix_len)
    v1, _, _ = ec.read_positive_with_prefix(buf, pos, prefix_len)
    assert (v0, v1) == (0, LONG_MAX)


def test_pos_backward_write_small():
    _read_write_backward(1000000, 7)  # reference: jump 1


def test_pos_backward_write_big():
    _read_write_backward(10000000000000, 1000000000)  # reference: jump 1e6


def test_prefix_writes():
    _read_write_prefix(1000000000000, 100000000, 3, 4)  # testPrefix1WriteBig (jump 1e6 in the reference)
    _read_write_prefix(130, 1, 2, 1)                     # testPrefix2WriteTiny
    _read_write_prefix(100000, 1, 2, 1)                  # testPrefix2WriteSmall
    _read_write_prefix(100000, 1, 2, 0)                  # testPrefix3WriteSmall


def test_byte_order_preserving_positive_backward():
    rng = np.random.default_rng(3)
    vals = sorted(set(int(x) for x in rng.integers(0, 1 << 62, 2000)) | {0, 1, 127, 128, LONG_MAX})
    enc = [ec.write_positive_backward(v) for v in vals]
    assert enc == sorted(enc)
    for v, b in zip(vals, enc):
        assert ec.read_positive_backward(b, len(b)) == (v, 0)


def random_entries(n, seed=0):
    """n encoded entries of every kind; returns (bytes, off, vpos, type_ids, type_mult, expected)."""
    rng = np.random.default_rng(seed)
    labels = [ec.schema_id(int(c), "user_edge") for c in rng.integers(1, 1 << 20, 12)]
    mults = [ec.MULTI, ec.MULTI, ec.SIMPLE, ec.ONE2MANY, ec.MANY2ONE, ec.ONE2ONE] * 2
    keys = [ec.schema_id(int(c), "user_key") for c in rng.integers(1, 1 << 20, 4)]
    sys_label = ec.schema_id(3, "system_edge")
    data, off, vpos, exp = bytearray(), [0], [], []
    for i in range(n):
        kind = rng.integers(0, 20)
        if kind == 0:
            t = keys[int(rng.integers(0, len(keys)))]
            rel = int(rng.integers(0, 1 << 40))
            e, vp = ec.encode_property(t, rel, bytes(rng.integers(0, 256, int(rng.integers(1, 6)), dtype=np.uint8)))
            exp.append((t, 2, -1, -1))
        elif kind == 1:
            e, vp = ec.encode_edge(sys_label, ec.OUT, 5, 6)
            exp.append((sys_label, 3, -1, -1))
        else:
            li = int(rng.integers(0, len(labels)))
            t, m = labels[li], mults[li]
            d = int(rng.integers(0, 2))
            other = int(rng.integers(0, 1 << int(rng.integers(1, 62))))
            rel = int(rng.integers(0, 1 << int(rng.integers(1, 62))))
            sk = bytes(rng.integers(0, 256, int(rng.integers(0, 4)), dtype=np.uint8)) if m == ec.MULTI else b""
            val = bytes(rng.integers(0, 256, int(rng.integers(0, 8)), dtype=np.uint8))
            e, vp = ec.encode_edge(t, d, other, rel, m, sk, val, invisible=bool(rng.integers(0, 4) == 0))
            exp.append((t, d, other, rel))
        data += e
        off.append(len(data))
        vpos.append(vp)
    return (bytes(data), np.array(off, np.int64), np.array(vpos, np.int32), np.array(labels, np.int64),
            np.array(mults, np.int8), np.array(exp, dtype=object))


def check_decoded(decoded, exp):
    t, d, o, r = decoded
    assert np.array_equal(t, np.array([x[0] for x in exp], np.int64))
    assert np.array_equal(d, np.array([x[1] for x in exp], np.int8))
    assert np.array_equal(o, np.array([x[2] for x in exp], np.int64))
    assert np.array_equal(r, np.array([x[3] for x in exp], np.int64))


def test_oracle_decodes_every_entry_kind(oracle_lib):
    data, off, vpos, tids, tmult, exp = random_entries(4000, seed=1)
    check_decoded(oracle_lib.decode_edges(data, off, vpos, tids, tmult), exp)


def test_unlisted_labels_decode_as_multi(oracle_lib):
    t = ec.schema_id(77, "user_edge")
    e, vp = ec.encode_edge(t, ec.IN, 123456789, 42)
    got = oracle_lib.decode_edges(e, [0, len(e)], [vp])
    check_decoded(got, [(t, 1, 123456789, 42)])


# ---- edge properties in the value (the weight the GPU decodes, tests/test_gpu_weights.py) ----

def test_property_value_formats():
    """StandardSerializer.writeObject + the attribute serializers, pinned byte for byte: a null flag
    then IntegerSerializer's VariableLong.write (|v| << 1 | sign); StringSerializer's header
    (length << 3 | compressor: ASCII 2 << 4 with the last byte marked, UTF (chars << 4) + 8, null 0)."""
    assert ec.write_value(ec.INT, 5) == b"\x00\x8a"
    assert ec.write_value(ec.INT, -3) == b"\x00\x87"
    assert ec.write_value(ec.INT, 0) == b"\x00\x80"
    assert ec.write_value(ec.INT, None) == b"\xff"
    assert ec.write_value(ec.LONG, 1) == b"\x00" + (1).to_bytes(8, "big")
    assert ec.write_string("ab") == bytes([0xA0, ord("a"), ord("b") | 0x80])
    assert ec.write_string(None) == b"\x80" and ec.write_string("") == b"\x90"
    assert ec.write_string("é") == bytes([0x98, 0xC3, 0xA9])
    assert ec.read_signed(ec.write_signed(-(1 << 31)), 0) == (-(1 << 31), 5)


def test_edge_weight_parser_round_trip():
    """edge_weight (parseRelation's property loop restated) finds the weight among random properties of
    every type, on entries of every multiplicity and direction layout."""
    import numpy as np
    rng = np.random.default_rng(0)
    keys = {ec.schema_id(c, "user_key"): t for c, t in
            zip(range(3, 14), (ec.BYTE, ec.SHORT, ec.LONG, ec.CHAR, ec.BOOL, ec.INT, ec.DATE, ec.FLOAT, ec.DOUBLE,
                               ec.UUID, ec.STRING))}
    wkey = ec.schema_id(8, "user_key")  # the INT key
    width = {ec.BYTE: 1, ec.SHORT: 2, ec.LONG: 8, ec.CHAR: 2, ec.BOOL: 1, ec.DATE: 8, ec.FLOAT: 4, ec.DOUBLE: 8,
             ec.UUID: 16}
    for trial in range(300):
        props, want = [], ec.WEIGHT_ABSENT
        for k, t in keys.items():
            if rng.random() < 0.5:
                continue
            if t == ec.STRING:
                v = ["", "q", "hello", "ünï", None][int(rng.integers(0, 5))]
            elif t == ec.INT:
                v = None if rng.random() < 0.2 else int(rng.integers(-(1 << 31) + 1, 1 << 31))
                if k == wkey:
                    want = ec.WEIGHT_ABSENT if v is None else v
            else:
                v = None if rng.random() < 0.1 else bytes(rng.integers(0, 256, width[t], dtype=np.uint8))
            props.append((k, t, v))
        mult = int(rng.integers(0, 5))
        entry, vpos = ec.encode_edge(ec.schema_id(20, "user_edge"), ec.OUT, 12345 << 8, 777 + trial, mult,
                                     value=ec.write_properties(props))
        assert ec.edge_weight(entry, vpos, mult, ec.OUT, wkey, keys) == want, (trial, props)
