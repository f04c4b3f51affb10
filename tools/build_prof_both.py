"""One BOTH-adjacency CSR build of RMAT-<scale> (for rocprofv3 kernel stats of the build)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
ctx = jg.Context((0,))
g = ctx.build_rmat(scale, 16, 0x5EED + scale, flags=jg.ADJ_BOTH)
print("build_ms", ctx.stats()["build_ms"], flush=True)
g.close()
ctx.close()
