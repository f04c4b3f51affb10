"""Edge weights decoded on the GPU from the edgestore rows (jg_builder_set_weight_key) instead of per-entry
host weights (what GpuSnapshot.WeightReader parses with EdgeSerializer.parseRelation on the JVM).

Rows are written the JanusGraph way (oracle/edgecodec.py): every edge twice (OUT on its source row, IN on
its target row), its properties in the value after the ids, in ascending key-id order
(EdgeSerializer.writeRelation :294-302): a Long, a String (ASCII, UTF and null forms), a Double key
around the Integer `distance` key, edges without the weight, with a null weight, negative weights,
every multiplicity.  The oracle's parser (edgecodec.edge_weight, the property loop of parseRelation
:159-171 restated) gives the host weights; ShortestDistance from several seeds must then agree between
the two graphs and with the oracle, bit for bit, including the failure when a message crosses an edge
without a weight.  Unknown key types before the weight and a stored Integer.MIN_VALUE fail the build."""
import numpy as np
import pytest

from janusgraph_amd.idmanager import IDManager
from oracle import edgecodec as ec

pytestmark = pytest.mark.gpu

LONG_KEY = ec.schema_id(6, "user_key")
NAME_KEY = ec.schema_id(7, "user_key")
DIST_KEY = ec.schema_id(9, "user_key")   # the weight ("distance")
SCORE_KEY = ec.schema_id(12, "user_key")
KEY_TYPES = {LONG_KEY: ec.LONG, NAME_KEY: ec.STRING, DIST_KEY: ec.INT, SCORE_KEY: ec.DOUBLE}
VEXISTS = ec.schema_id(1, "system_key")


def weighted_store(n=400, m=3000, seed=0, weight_of=None, name_of=None):
    """(store arrays, labels table, per-entry host weights); weight_of(e, rng) -> weight or None (absent);
    name_of(rng) -> the String property's value (every edge gets one) or pre-encoded bytes."""
    rng = np.random.default_rng(seed)
    idm = IDManager(5)
    vids = sorted({(((int(c) << 5) + int(p)) << 3) for c, p in zip(rng.integers(1, 1 << 30, n), rng.integers(0, 32, n))})
    n = len(vids)
    labels = [ec.schema_id(c, "user_edge") for c in (11, 12, 13, 14)]
    mults = [ec.MULTI, ec.SIMPLE, ec.ONE2MANY, ec.MANY2ONE]
    rows = {v: [(ec.encode_property(VEXISTS, 10 + i, b"\x01"))] for i, v in enumerate(vids)}
    s = rng.integers(0, n, m)
    t = rng.integers(0, n, m)
    rel = 1000
    for e in range(m):
        props = []
        if rng.random() < 0.5:
            props.append((LONG_KEY, ec.LONG, int(rng.integers(0, 1 << 62))))
        if name_of is not None:
            props.append((NAME_KEY, ec.STRING, name_of(rng)))
        elif rng.random() < 0.5:
            props.append((NAME_KEY, ec.STRING, [None, "", "x", "abc" * 5, "é", "€uro"][int(rng.integers(0, 6))]))
        w = weight_of(e, rng) if weight_of else int(rng.integers(-3, 9))
        if w is not None:
            props.append((DIST_KEY, ec.INT, None if w == "null" else w))
        if rng.random() < 0.5:
            props.append((SCORE_KEY, ec.DOUBLE, bytes(rng.integers(0, 256, 8, dtype=np.uint8))))
        value = ec.write_properties(props)
        L = int(rng.integers(0, 4))
        a, b = vids[int(s[e])], vids[int(t[e])]
        rows[a].append(ec.encode_edge(labels[L], ec.OUT, b, rel, mults[L], value=value))
        rows[b].append(ec.encode_edge(labels[L], ec.IN, a, rel, mults[L], value=value))
        rel += 1
    keys = sorted(rows, key=idm.get_key)
    data, off, vpos, roff, weight = bytearray(), [0], [], [0], []
    mult_of = dict(zip(labels, mults))
    for v in keys:
        for b, vp in sorted(rows[v], key=lambda ev: ev[0][: ev[1]]):
            data += b
            off.append(len(data))
            vpos.append(vp)
            tid, direction = _header(b)
            weight.append(ec.edge_weight(b, vp, mult_of[tid], ec.OUT, DIST_KEY, KEY_TYPES)
                          if tid in mult_of and direction == ec.OUT else ec.WEIGHT_ABSENT)
        roff.append(len(vpos))
    store = (np.array([idm.get_key(v) for v in keys], np.uint64), np.array(roff, np.int64), bytes(data),
             np.array(off, np.int64), np.array(vpos, np.int32), np.array(labels[1:], np.int64),
             np.array(mults[1:], np.int8))
    return store, np.array(weight, np.int64)


def _header(b):
    """(type id, direction) of an entry header (IDHandler.readRelationType)."""
    v, prefix, _ = ec.read_positive_with_prefix(b, 0, 3)
    is_edge = prefix & 1
    system = (prefix >> 1) == 0
    suffix = (53 if system else 21) if is_edge else (37 if system else 5)
    return ((v >> 1) << 6) | suffix, (v & 1) if is_edge else ec.OUT


def build(store, host_weight=None, key_types=KEY_TYPES, weight_key=DIST_KEY):
    import janusgraph_amd as jg
    keys, roff, data, off, vpos, tids, tmult = store
    ctx = jg.Context((0,))
    b = ctx.builder()
    b.set_query_limit(jg.FULGORA_HARD_QUERY_LIMIT, jg.DIR_OUT)  # GpuSnapshot's settings for ShortestDistance
    b.set_schema(tids, tmult, 5)
    if host_weight is None:
        ids = [ec.inline_id(k) for k in key_types]
        b.set_weight_key(ec.inline_id(weight_key), ids, list(key_types.values()))
    half = len(keys) // 2
    for r0, r1 in ((0, half), (half, len(keys))):  # two chunks of whole rows
        e0, e1 = int(roff[r0]), int(roff[r1])
        b0, b1 = int(off[e0]), int(off[e1])
        w = None if host_weight is None else np.ascontiguousarray(host_weight[e0:e1], np.int32)
        b.add_rows(keys[r0:r1], roff[r0:r1 + 1] - e0, data[b0:b1], off[e0:e1 + 1] - b0, vpos[e0:e1], w)
    try:
        g = b.finish(jg.ADJ_IN | jg.ADJ_OUT)
    finally:
        b.close()
    return ctx, g


def sd_or_error(g, vid, seed, depth):
    import janusgraph_amd as jg
    try:
        return g.shortest_distance(int(vid[seed]), depth)
    except jg.JanusGpuError as e:
        return e.code


@pytest.mark.parametrize("seed", [0, 1])
def test_device_weights_equal_host_weights(oracle_lib, seed):
    store, hw = weighted_store(seed=seed, weight_of=lambda e, rng: (
        None if rng.random() < 0.03 else "null" if rng.random() < 0.02 else int(rng.integers(-3, 9))))
    ctx_d, gd = build(store)
    ctx_h, gh = build(store, host_weight=hw)
    vid = gd.vertex_ids()
    assert np.array_equal(vid, gh.vertex_ids())
    keys, roff, data, off, vpos, tids, tmult = store
    ov, os_, ot, ent = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, return_entries=True)
    index = {int(v): i for i, v in enumerate(ov)}
    ds = np.array([index[int(a)] for a in os_], np.int32)
    dd = np.array([index[int(b)] for b in ot], np.int32)
    w = hw[ent].astype(np.int32)
    failures = runs = 0
    for s in range(0, len(vid), 13):
        for depth in (1, 2):  # deeper runs almost always cross an edge without the weight
            runs += 1
            got_d, got_h = sd_or_error(gd, vid, s, depth), sd_or_error(gh, vid, s, depth)
            try:
                want = oracle_lib.shortest_distance(len(vid), ds, dd, s, depth, w)
            except ValueError:  # a message crosses an edge without the weight: Fulgora's edge function throws
                failures += 1
                assert isinstance(got_d, int) and got_d == got_h == -1, (got_d, got_h)  # JG_ERR_ARG
                continue
            np.testing.assert_array_equal(got_d, want)
            np.testing.assert_array_equal(got_h, want)
    assert 0 < failures < runs  # both outcomes exercised
    for g, c in ((gd, ctx_d), (gh, ctx_h)):
        g.close()
        c.close()


def test_device_weights_all_present_match_oracle(oracle_lib):
    store, hw = weighted_store(n=300, m=2500, seed=5)
    ctx, g = build(store)
    vid = g.vertex_ids()
    keys, roff, data, off, vpos, tids, tmult = store
    ov, os_, ot, ent = oracle_lib.edgestore_snapshot(keys, roff, data, off, vpos, tids, tmult, return_entries=True)
    index = {int(v): i for i, v in enumerate(ov)}
    ds = np.array([index[int(a)] for a in os_], np.int32)
    dd = np.array([index[int(b)] for b in ot], np.int32)
    assert (hw[ent] != ec.WEIGHT_ABSENT).all() and (hw[ent] < 0).any()
    for s in (0, 7, 99):
        np.testing.assert_array_equal(g.shortest_distance(int(vid[s]), 6),
                                      oracle_lib.shortest_distance(len(vid), ds, dd, s, 6, hw[ent].astype(np.int32)))
    g.close()
    ctx.close()


def full_utf_raw(body: bytes) -> bytes:
    """A full-UTF String of len(body) one-byte characters as StringSerializer.write would frame it, with lead
    bytes the writer never emits (nibbles 8-11 and 15): StringSerializer.read (:126-145) consumes one byte
    for each, so the property after it is still found."""
    return ec.write_positive((len(body) << 4) + (1 << 3)) + bytes(body)


def test_device_weights_after_odd_utf_lead_bytes(oracle_lib):
    """skip_string consumed two bytes for lead nibbles 8-11 and 15; the reference one."""
    odd = [full_utf_raw(bytes([0x85, 0x41])), full_utf_raw(bytes([0x9A, 0xB0, 0xF3])), full_utf_raw(bytes([0xA1]))]
    # every edge carries one of the odd strings, the weight after it
    store2, hw2 = weighted_store(n=200, m=1500, seed=11, weight_of=lambda e, rng: int(rng.integers(0, 9)),
                                 name_of=lambda rng: odd[int(rng.integers(0, len(odd)))])
    assert (hw2 != ec.WEIGHT_ABSENT).sum() > 1000  # the oracle's parser finds the weight after each
    ctx_d, gd = build(store2)
    ctx_h, gh = build(store2, host_weight=hw2)
    vid = gd.vertex_ids()
    for s in (0, 17, 101):
        np.testing.assert_array_equal(gd.shortest_distance(int(vid[s]), 2), gh.shortest_distance(int(vid[s]), 2))
    for g, c in ((gd, ctx_d), (gh, ctx_h)):
        g.close()
        c.close()


def test_weight_key_errors():
    import janusgraph_amd as jg
    store, _ = weighted_store(n=60, m=300, seed=3)
    # a key of unknown type ahead of the weight: its value length is unknown
    types = dict(KEY_TYPES)
    types[LONG_KEY] = 0
    with pytest.raises(jg.JanusGpuError) as e:
        build(store, key_types=types)
    assert e.value.code == jg._lib.JG_ERR_UNSUPPORTED
    # a stored Integer.MIN_VALUE is the absent-weight marker
    store2, _ = weighted_store(n=60, m=300, seed=4, weight_of=lambda e, rng: -(1 << 31) if e == 17 else 1)
    with pytest.raises(jg.JanusGpuError) as e:
        build(store2)
    assert e.value.code == jg._lib.JG_ERR_UNSUPPORTED
    # no Integer key of that name (a Double weight key): every weight absent, a crossing fails
    ctx, g = build(store, weight_key=SCORE_KEY)
    assert g.shortest_distance(int(g.vertex_ids()[0]), 0)[0] == 0  # maxDepth 0: no message crosses
    with pytest.raises(jg.JanusGpuError):
        g.shortest_distance(int(g.vertex_ids()[0]), 3)
    g.close()
    ctx.close()
