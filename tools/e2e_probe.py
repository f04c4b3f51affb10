import sys, time, json, numpy as np
sys.path.insert(0, '.')
import janusgraph_amd as jg
n = 1 << 24
ctx = jg.Context((0,))
g = ctx.build_rmat(24, 16, 0x5EED + 24, flags=jg.ADJ_BOTH)
out = {}
for rep in range(2):
    for want in (False, True):
        t = time.perf_counter(); g.bfs([1], jg.DIR_BOTH, want=want); out[f"bfs_want{int(want)}"] = round(time.perf_counter() - t, 4)
    t = time.perf_counter(); g.connected_components(); out["cc"] = round(time.perf_counter() - t, 4); out["cc_compute"] = ctx.stats()["compute_ms"]
    srcs = np.arange(64) * 7 + 1
    for want in (False, True):
        t = time.perf_counter(); g.bfs(srcs, jg.DIR_BOTH, want=want); out[f"ms_want{int(want)}"] = round(time.perf_counter() - t, 4)
    out["ms_compute"] = ctx.stats()["compute_ms"]
print(json.dumps(out))
