"""Builds RMAT graphs (diagnostic for rocprofv3 kernel traces of the CSR / plan build)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import janusgraph_amd as jg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=26)
ap.add_argument("--flags", type=int, default=jg.ADJ_IN)
a = ap.parse_args()
ctx = jg.Context((0,))
g = ctx.build_rmat(a.scale, 16, 0x5EED + a.scale, flags=a.flags)
print("build_ms", ctx.stats()["build_ms"], flush=True)
g.close()
ctx.close()
