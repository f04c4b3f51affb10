"""janusgraph_amd — MI355X-native OLAP graph computer for JanusGraph (GpuGraphComputer).

The compute path is libjanusgpu.so (hand-written HIP for gfx950, C-ABI in include/janusgpu.h);
this package is its host-side mirror of the TinkerPop GraphComputer API.
"""
from ._lib import (ADJ_BOTH, ADJ_IN, ADJ_OUT, DIR_BOTH, DIR_IN, DIR_OUT, Context, Graph, JanusGpuError,  # noqa: F401
                   LIB_PATH, load)

__all__ = ["Context", "Graph", "JanusGpuError", "load", "ADJ_IN", "ADJ_OUT", "ADJ_BOTH", "DIR_IN", "DIR_OUT",
           "DIR_BOTH", "LIB_PATH"]
