"""Work model for the replicated-graph / partitioned-sources 8-GPU plan: entries
examined by a bit-parallel direction-optimising BFS of k sources (tools/micro/narrow_sim.c) against k
single-source DO-BFS traversals, on the bench's 64 sources (bench.pick_sources(deg, 64, 7)) split into
groups.  CPU only; no GPU result depends on it.
    python tools/narrow_sim.py --scale 22 --group 8
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "micro", "narrow_sim.c")
LIB = os.path.join(ROOT, "tools", "micro", "libnarrow_sim.so")


def lib():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O3", "-fopenmp", "-shared", "-fPIC", "-o", LIB, SRC])
    L = ctypes.CDLL(LIB)
    L.narrow_sim.restype = ctypes.c_int
    return L


def degree_csr(scale, ef):
    """Symmetric CSR relabelled by degree (descending), neighbours ascending: the GPU BOTH plan's order."""
    from oracle import oracle as o
    o.build()
    n = 1 << scale
    s, d = o.rmat_edges(scale, ef, 0x5EED + scale)
    s, d = s.astype(np.int32), d.astype(np.int32)
    deg = np.bincount(s, minlength=n) + np.bincount(d, minlength=n)
    order = np.argsort(-deg, kind="stable")
    new = np.empty(n, np.int64)
    new[order] = np.arange(n)
    rows = np.concatenate([new[s], new[d]])
    cols = np.concatenate([new[d], new[s]]).astype(np.int32)
    del s, d
    key = rows * n + cols
    del rows
    key.sort()
    r = (key // n).astype(np.int64)
    cols = (key % n).astype(np.int32)
    del key
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=ptr[1:])
    return n, ptr, cols, deg, new


def run(L, n, ptr, adj, srcs, alpha, beta, per_source, max_levels=64):
    out = np.zeros(max_levels * 4, np.int64)
    s = np.ascontiguousarray(srcs, np.int64)
    lv = L.narrow_sim(ctypes.c_int64(n), ptr.ctypes.data_as(ctypes.c_void_p), adj.ctypes.data_as(ctypes.c_void_p),
                      s.ctypes.data_as(ctypes.c_void_p), len(s), alpha, beta, per_source,
                      out.ctypes.data_as(ctypes.c_void_p), max_levels)
    return out[:lv * 4].reshape(lv, 4)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--group", type=int, default=8)
    p.add_argument("--alpha", type=int, default=14)
    p.add_argument("--beta", type=int, default=24)
    a = p.parse_args()
    import bench
    L = lib()
    n, ptr, adj, deg, new = degree_csr(a.scale, 16)
    srcs = new[bench.pick_sources(deg, 64, 7)]
    single = [run(L, n, ptr, adj, [x], a.alpha, a.beta, 1) for x in srcs]
    sing = np.array([[r[:, 0].sum(), r[:, 1].sum()] for r in single])
    print(json.dumps({"scale": a.scale, "single_td_bu_mean": sing.mean(0).tolist(),
                      "single_total_mean": float(sing.sum(1).mean())}), flush=True)
    for per_source in (1, 0):
        for g0 in range(0, 64, a.group):
            r = run(L, n, ptr, adj, srcs[g0:g0 + a.group], a.alpha, a.beta, per_source)
            tot = float(r[:, 0].sum() + r[:, 1].sum())
            print(json.dumps({"group": g0 // a.group, "per_source": per_source, "levels": int(len(r)),
                              "td": int(r[:, 0].sum()), "bu": int(r[:, 1].sum()),
                              "total_over_one_single": round(tot / float(sing.sum(1).mean()), 2),
                              "per_level": r.tolist()}), flush=True)


if __name__ == "__main__":
    main()
