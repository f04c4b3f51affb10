"""PageRank supersteps with one launch per degree class (JG_PULL_SPLIT=1 set in-process) for
per-class rocprofv3 times (diagnostic)."""
import argparse
import os
import sys

os.environ["JG_PULL_SPLIT"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=24)
ap.add_argument("--steps", type=int, default=5)
a = ap.parse_args()
ctx = jg.Context((0,))
g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=jg.ADJ_IN)
n = 1 << a.scale
g.pagerank_begin(0.85, n)
g.pagerank_step(a.steps)
g.sync()
g.pagerank_end(want=False)
