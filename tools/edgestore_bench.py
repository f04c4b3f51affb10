"""Snapshot straight from edgestore rows at RMAT scale (jg_graph_build_edgestore).

Writes the RMAT graph the way JanusGraph's edgestore holds it (vectorised restatement of
EdgeSerializer.writeRelation for a MULTI label, VariableLong.writePositiveBackward, IDManager.getKey
with graph.set-vertex-id ids (i+1) << 8): one row per vertex, its VertexExists property first, every
edge OUT on its source row and IN on its target row.  Then times, on the GPU:
  * jg_graph_build_edgestore: build_ms (host->device copies, decode, remap, CSR) and the two decode
    kernels (kernel_ms_total) against their algorithmic bytes;
  * jg_graph_build from the already-decoded (vid, src, dst) arrays, for the same adjacency;
  * the chunked builder (jg_builder_add_rows, as GpuSnapshot feeds it) with K chunks of whole rows:
    the wall time of the add_rows calls (host staging + whatever the two chunk streams have not
    overlapped), the summed per-chunk copy and copy+decode event times, and finish;
and checks every snapshot gives identical PageRank (the decoded one must equal the direct one).
Prints one JSON line.  Usage: python tools/edgestore_bench.py [--scale 20] [--chunks 1,8,32]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def backward_varint(v):
    """VariableLong.writeUnsignedBackward over an int64 array: (bytes[k, 5] left-aligned, lengths)."""
    v = v.astype(np.int64)
    bl = np.maximum(1, np.floor(np.log2(np.maximum(v, 1))).astype(np.int64) + 1)
    n = np.maximum(3, 1 + np.where(bl <= 4, 0, 1 + (bl - 5) // 7))
    out = np.zeros((len(v), int(n.max())), np.uint8)
    for j in range(out.shape[1]):
        i = n - 1 - j  # group index written at byte j
        grp = (v >> (7 * np.maximum(i, 0))) & 0x7F
        b = np.where(j == 0, 0x80 | ((n - 3) << 4) | grp, grp)
        out[:, j] = np.where(j < n, b, 0).astype(np.uint8)
    return out, n


def write_edgestore(scale, ef, seed):
    from oracle import oracle as o  # input generator only: the RMAT edge list
    n = 1 << scale
    s, t = o.rmat_edges(scale, ef, seed)
    vid = (np.arange(n, dtype=np.int64) + 1) << 8
    m = len(s)
    label_count = 3  # a user edge label with count 3: header = writePositiveWithPrefix((3 << 1) | dir, 3, 3)
    hdr = {0: np.uint8((3 << 5) | ((label_count << 1) | 0)), 1: np.uint8((3 << 5) | ((label_count << 1) | 1))}
    rel = np.arange(m, dtype=np.int64) + 1024
    # entries: OUT on s (other = t), IN on t (other = s)
    row = np.concatenate([s, t]).astype(np.int64)
    other = vid[np.concatenate([t, s])]
    dirs = np.concatenate([np.zeros(m, np.uint8), np.ones(m, np.uint8)])
    relr = np.concatenate([rel, rel])
    ob, on = backward_varint(other)
    rb, rn = backward_varint(relr)
    elen = 1 + on + rn
    # VertexExists entry per row: header 0x02 (SystemPropertyKey count 1), relation id 1 backward, value 0x01
    ex = np.array([0x02, 0x80, 0x00, 0x01, 0x01], np.uint8)
    order = np.argsort(row, kind="stable")
    cnt = np.bincount(row, minlength=n)
    row_off = np.zeros(n + 1, np.int64)
    row_off[1:] = np.cumsum(cnt + 1)
    ent_len = np.empty(2 * m + n, np.int64)
    pos_exists = row_off[:-1]
    slot = np.ones(2 * m + n, bool)
    slot[pos_exists] = False
    ent_len[pos_exists] = len(ex)
    ent_len[slot] = elen[order]
    off = np.zeros(2 * m + n + 1, np.int64)
    off[1:] = np.cumsum(ent_len)
    data = np.empty(int(off[-1]), np.uint8)
    for j in range(len(ex)):
        data[off[pos_exists] + j] = ex[j]
    eoff = off[:-1][slot]
    data[eoff] = np.where(dirs[order] == 0, hdr[0], hdr[1])
    for j in range(ob.shape[1]):
        w = j < on[order]
        data[(eoff + 1 + j)[w]] = ob[order][w, j]
    for j in range(rb.shape[1]):
        w = j < rn[order]
        data[(eoff + 1 + on[order] + j)[w]] = rb[order][w, j]
    vpos = ent_len.astype(np.int32)
    vpos[pos_exists] = 4
    keys = (vid >> 8) << 3  # IDManager.getKey at 32 partitions: partition 0 in the top bits, count << 3
    return vid, s, t, keys.astype(np.uint64), row_off, data, off, vpos


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunks", default="1,8,32")
    args = ap.parse_args()
    import janusgraph_amd as jg
    t0 = time.perf_counter()
    vid, s, t, keys, roff, data, off, vpos = write_edgestore(args.scale, args.edgefactor, 0x5EED + args.scale)
    gen_s = time.perf_counter() - t0
    ctx = jg.Context((0,))
    flags = jg.ADJ_IN
    best = None
    for _ in range(args.reps):
        g, v = ctx.build_edgestore(keys, roff, data, off, vpos, flags=flags)
        st = ctx.stats()
        if best is None or st["build_ms"] < best["build_ms"]:
            best = st
        g_es, v_es = g, v
        if _ < args.reps - 1:
            g.close()
    direct = None
    for _ in range(args.reps):
        g2 = ctx.build(vid, vid[s], vid[t], flags=flags)
        st2 = ctx.stats()
        if direct is None or st2["build_ms"] < direct["build_ms"]:
            direct = st2
        if _ < args.reps - 1:
            g2.close()
    assert np.array_equal(v_es, vid), "vertex order"
    n = len(vid)
    r1, _ = g_es.pagerank(0.85, n, 5)
    r2, _ = g2.pagerank(0.85, n, 5)
    assert np.array_equal(r1, r2), "PageRank differs between the decoded and the direct snapshot"
    chunked = []
    for k in [int(x) for x in args.chunks.split(",") if x]:
        bounds = np.linspace(0, len(keys), k + 1).astype(np.int64)
        pieces = []
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            e0, e1 = int(roff[lo]), int(roff[hi])
            b0, b1 = int(off[e0]), int(off[e1])
            pieces.append((keys[lo:hi], roff[lo:hi + 1] - e0, data[b0:b1], off[e0:e1 + 1] - b0, vpos[e0:e1]))
        narrow = bool(np.max(np.diff(off)) < 256)
        h2d = (2 * len(vpos) if narrow else 12 * len(vpos) + 8 * k) + 16 * len(keys) + 8 * k + len(data)
        runs = []
        for _ in range(args.reps):
            b = ctx.builder()
            b.set_schema()
            t0 = time.perf_counter()
            for p in pieces:
                b.add_rows(*p)
            t1 = time.perf_counter()
            gk = b.finish(flags)
            t2 = time.perf_counter()
            st = ctx.stats()
            b.close()
            runs.append({"chunks": k, "add_rows_wall_ms": round((t1 - t0) * 1e3, 2),
                         "finish_wall_ms": round((t2 - t1) * 1e3, 2),
                         "copy_ms_sum": round(st["exchange_ms"], 2),
                         "copy_decode_ms_sum": round(st["kernel_ms_total"], 2),
                         "decode_ms_sum": round(st["kernel_ms_total"] - st["exchange_ms"], 2),
                         "h2d_bytes": int(h2d), "narrow_staging": narrow,
                         "h2d_GBs": round(h2d / (st["exchange_ms"] * 1e-3) / 1e9, 1)})
            rk, _ = gk.pagerank(0.85, n, 5)
            assert np.array_equal(rk, r1), f"PageRank differs for {k} chunks"
            gk.close()
        chunked.append(min(runs, key=lambda x: x["add_rows_wall_ms"] + x["finish_wall_ms"]))
    info = g_es.info()
    kern_ms = best["kernel_ms_total"] - best.get("exchange_ms", 0.0)
    alg = best["algorithmic_bytes"]
    line = {
        "workload": f"edgestore_snapshot_rmat{args.scale}_ef{args.edgefactor}",
        "rows": int(len(keys)), "entries": int(len(vpos)), "entry_bytes": int(len(data)),
        "edges": int(info["num_edges"]),
        "build_edgestore_ms": round(best["build_ms"], 2), "build_direct_ms": round(direct["build_ms"], 2),
        "decode_kernels_ms": round(kern_ms, 3), "copy_ms": round(best.get("exchange_ms", 0.0), 2),
        "chunked_builder": chunked,
        "decode_roofline": {"bound": "hbm", "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(alg / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                            "bytes": alg},
        "entries_per_s_G": round(len(vpos) / (kern_ms * 1e-3) / 1e9, 2),
        "writer_s": round(gen_s, 1), "pagerank_identical": True,
    }
    print(json.dumps(line), flush=True)
    g_es.close()
    g2.close()
    ctx.close()


if __name__ == "__main__":
    main()
