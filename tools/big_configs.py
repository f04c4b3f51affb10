"""Full-size runs of the SURVEY.md §8 rows that are not the headline line (BASELINE.json configs[2..4]
at RMAT scale 26 by default), each with a full-size parity check that does not need the oracle to
replay the whole run:

  pr     PageRank fp64 (ADJ_IN): ms/superstep and GTEPS; parity = the oracle's superstep
         (jo_pagerank_superstep_csr) applied to the GPU's own ranks after K-1 supersteps must give the
         GPU's ranks after K (per-vertex rel err <= 1e-9), plus K=3 bit-for-bit rank sum sanity.
  cc     ConnectedComponentVertexProgram (ADJ_BOTH): iterations, ms; parity = scipy connected
         components + the String-order minimum id of every component (exact), and < 99 iterations
         so Fulgora's 100-iteration cap does not bind.
  bfs    single-source direction-optimising BFS (DIR_BOTH) on 8 sources: GTEPS (Graph500 edge count);
         parity = Graph500 validation (source depth 0, |depth(u)-depth(v)| <= 1 over every edge,
         every reached vertex has a parent one level up, reached set == the source's component).
  msbfs  64-source bit-parallel BFS: ms, levels; parity = the same validation on sources 0, 31, 63.

Writes one JSON object (stdout, and --out).  GPU + host heavy at scale 26 (≈30 GB host memory).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print("[big]", *a, file=sys.stderr, flush=True)


def host_edges(o, scale, ef, seed):
    """The same RMAT edges the device generator makes, as int32 (chunked: int64 temporaries stay small)."""
    m = ef << scale
    s32 = np.empty(m, np.int32)
    d32 = np.empty(m, np.int32)
    step = 1 << 26
    for e0 in range(0, m, step):
        c = min(step, m - e0)
        s, d = o.rmat_edges(scale, ef, seed, e0, c)
        s32[e0:e0 + c] = s
        d32[e0:e0 + c] = d
    return s32, d32


def lex_order_rank(n):
    """Rank of str(v) for v in 0..n-1 in String order (left-aligned 19-digit decimal, then length)."""
    x = np.arange(n, dtype=np.uint64)
    digits = np.ones(n, np.int64)
    t = x.copy()
    for _ in range(19):
        t //= np.uint64(10)
        digits += (t > 0)
    pad = x * (np.uint64(10) ** (19 - digits).astype(np.uint64))
    order = np.lexsort((digits, pad))
    rank = np.empty(n, np.int64)
    rank[order] = np.arange(n, dtype=np.int64)
    return rank, order


def validate_bfs(depth, source, s32, d32, comp_of, name):
    """Graph500-style BFS validation over the undirected edge list; returns (ok, reached, edges)."""
    n = depth.shape[0]
    ok = depth[source] == 0
    du = depth[s32]
    dv = depth[d32]
    ru, rv = du >= 0, dv >= 0
    ok &= bool(np.array_equal(ru, rv))                       # an edge never leaves the reached set
    both = ru & rv
    ok &= bool(np.all(np.abs(du[both] - dv[both]) <= 1))    # BFS levels differ by at most one
    has_parent = np.zeros(n, bool)
    m1 = both & (du == dv - 1)
    has_parent[d32[m1]] = True
    m2 = both & (dv == du - 1)
    has_parent[s32[m2]] = True
    reached = depth >= 0
    need = reached.copy()
    need[source] = False
    ok &= bool(np.all(has_parent[need]))                      # every reached vertex has a parent
    if comp_of is not None:
        ok &= bool(np.array_equal(reached, comp_of == comp_of[source]))  # reached == component
    edges = int(np.count_nonzero(ru))
    if not ok:
        log(f"{name}: BFS validation FAILED for source {source}")
    return bool(ok), int(reached.sum()), edges


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--edgefactor", type=int, default=16)
    p.add_argument("--which", default="pr,cc,bfs,msbfs")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--out", default=None)
    args = p.parse_args()
    import janusgraph_amd as jg
    from oracle import oracle as o
    o.build()
    which = set(args.which.split(","))
    scale, ef = args.scale, args.edgefactor
    seed = 0x5EED + scale
    n, m = 1 << scale, ef << scale
    res = {"scale": scale, "edgefactor": ef, "seed": seed, "n": n, "m": m}
    t = time.perf_counter()
    s32, d32 = host_edges(o, scale, ef, seed)
    log(f"host edges {time.perf_counter() - t:.1f}s")
    ctx = jg.Context((0,))

    if "pr" in which:
        g = ctx.build_rmat(scale, ef, seed, flags=jg.ADJ_IN)
        build_ms = ctx.stats()["build_ms"]
        g.pagerank_begin(0.85, n)
        g.pagerank_step(3)
        g.sync()
        t = time.perf_counter()
        g.pagerank_step(args.steps)
        g.sync()
        dt = time.perf_counter() - t
        g.pagerank_end(want=False)
        K = 8
        r_a, ec = g.pagerank(0.85, n, K - 1)
        r_b, _ = g.pagerank(0.85, n, K)
        g.close()
        t = time.perf_counter()
        ptr, col = o.build_in_csr(n, s32, d32)
        log(f"oracle in-CSR {time.perf_counter() - t:.1f}s")
        contrib = r_a / ec
        rank_out = np.empty(n, np.float64)
        o.pagerank_superstep_csr(n, ptr, col, contrib, ec, 0.85, n, rank_out)
        del ptr, col
        ok_deg = bool(np.array_equal(ec, np.bincount(s32, minlength=n).astype(np.float64)))
        rel = float(np.max(np.abs(r_b - rank_out) / np.abs(rank_out)))
        res["pr"] = {"build_ms": round(build_ms, 1), "ms_per_step": round(dt / args.steps * 1e3, 4),
                     "gteps": round(m * args.steps / dt / 1e9, 2), "superstep_max_rel_err": rel,
                     "edge_count_exact": ok_deg, "parity": bool(ok_deg and rel <= 1e-9)}
        log("pr", res["pr"])
        del r_a, r_b, ec, contrib, rank_out

    comp_of = None
    if which & {"cc", "bfs", "msbfs"}:
        import scipy.sparse as sp
        from scipy.sparse.csgraph import connected_components
        t = time.perf_counter()
        a = sp.csr_matrix((np.ones(m, np.int8), (s32, d32)), shape=(n, n))
        ncomp, comp_of = connected_components(a, directed=False)
        del a
        comp_of = comp_of.astype(np.int32)
        log(f"scipy components {ncomp} in {time.perf_counter() - t:.1f}s")
        g = ctx.build_rmat(scale, ef, seed, flags=jg.ADJ_BOTH)
        res["build_both_ms"] = round(ctx.stats()["build_ms"], 1)

    if "cc" in which:
        comp, it = g.connected_components()
        st = ctx.stats()
        lex, order = lex_order_rank(n)
        cmin = np.full(int(comp_of.max()) + 1, np.iinfo(np.int64).max, np.int64)
        np.minimum.at(cmin, comp_of, lex)
        expect = order[cmin[comp_of]].astype(np.int64)  # vid == dense id for RMAT graphs
        ok = bool(np.array_equal(comp, expect)) and it < 99
        res["cc"] = {"ms": round(st["compute_ms"], 2), "iterations": it, "components": int(len(np.unique(comp))),
                     "gteps_per_iteration": round(2 * m * it / (st["compute_ms"] * 1e-3) / 1e9, 2), "parity": ok}
        log("cc", res["cc"])
        del comp, expect, lex, order

    rng = np.random.default_rng(7)
    deg = None
    if which & {"bfs", "msbfs"}:
        deg = np.bincount(s32, minlength=n) + np.bincount(d32, minlength=n)
        cand = np.flatnonzero(deg > 0)
    if "bfs" in which:
        srcs = rng.choice(cand, 8, replace=False)
        teps, ms, oks = [], [], []
        for k, sv in enumerate(srcs):
            d = g.bfs([int(sv)], jg.DIR_BOTH)[0]
            st = ctx.stats()
            ms.append(st["compute_ms"])
            teps.append(st["edges_traversed"] / (st["compute_ms"] * 1e-3) / 1e9)
            if k < 3:
                ok, _, _ = validate_bfs(d, int(sv), s32, d32, comp_of, "bfs")
                oks.append(ok)
        res["bfs"] = {"sources": 8, "ms_median": round(float(np.median(ms)), 3),
                      "gteps_median": round(float(np.median(teps)), 2), "validated": len(oks), "parity": all(oks)}
        log("bfs", res["bfs"])
    if "msbfs" in which:
        srcs = rng.choice(cand, 64, replace=False)
        g.bfs(srcs, jg.DIR_BOTH, want=False)  # warm
        st = ctx.stats()
        t_ms = st["compute_ms"]
        depth = g.bfs(srcs, jg.DIR_BOTH, want=True)
        st = ctx.stats()
        oks = []
        for k in (0, 31, 63):
            ok, _, _ = validate_bfs(depth[k], int(srcs[k]), s32, d32, comp_of, "msbfs")
            oks.append(ok)
        csize_edges = np.bincount(comp_of[s32], minlength=int(comp_of.max()) + 1)
        traversed = float(csize_edges[comp_of[srcs]].sum())
        res["msbfs"] = {"sources": 64, "ms": round(t_ms, 2), "levels": st["levels"],
                        "gteps_source_edges": round(traversed / (t_ms * 1e-3) / 1e9, 2), "validated": 3,
                        "parity": all(oks)}
        log("msbfs", res["msbfs"])
    line = json.dumps(res)
    print(line)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
