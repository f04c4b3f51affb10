"""JanusGraph vertex-id layout for the CSR snapshot (user vertices only).

Mirrors janusgraph-core/src/main/java/org/janusgraph/graphdb/idmanagement/IDManager.java:
  bit layout [0 | count | partition | 3-bit type suffix]          :441-454
  VertexIDType Normal 000b / Partitioned 010b / Unmodifiable 100b   :76-120
  constructId / getKey / getKeyID (row key <-> vertex id)           :444-506
  getCanonicalVertexId / getPartitionHashForId                      :523-547
  toVertexId / fromVertexId (graph.set-vertex-id user ids)          :578-595
The snapshot keys vertices by canonical id (FulgoraVertexMemory.getCanonicalId,
janusgraph-core/.../olap/computer/FulgoraVertexMemory.java:74-77) before the dense remap.
"""
from __future__ import annotations

from enum import Enum

TOTAL_BITS = 63  # Long.SIZE - 1
MAX_PARTITION_BITS = 16
USERVERTEX_PADDING_BITWIDTH = 3
PARTITIONED_VERTEX_PARTITION = 1
DEFAULT_PARTITION_BITS = 5  # cluster.max-partitions = 32
_MASK64 = (1 << 64) - 1


class VertexIDType(Enum):
    NormalVertex = (3, 0b000)
    PartitionedVertex = (3, 0b010)
    UnmodifiableVertex = (3, 0b100)

    @property
    def offset(self):
        return self.value[0]

    @property
    def suffix(self):
        return self.value[1]

    def add_padding(self, count):
        return (count << self.offset) | self.suffix

    def is_(self, vid):
        return (vid & ((1 << self.offset) - 1)) == self.suffix


USER_VERTEX_TYPES = (VertexIDType.NormalVertex, VertexIDType.PartitionedVertex, VertexIDType.UnmodifiableVertex)


def _signed64(x):
    x &= _MASK64
    return x - (1 << 64) if x >> 63 else x


class IDManager:
    def __init__(self, partition_bits: int = DEFAULT_PARTITION_BITS):
        if not 0 <= partition_bits <= MAX_PARTITION_BITS:
            raise ValueError(f"Partition bits can be at most {MAX_PARTITION_BITS} bits")
        self.partition_bits = partition_bits
        self.partition_bound = 1 << partition_bits
        self.vertex_count_bound = 1 << (TOTAL_BITS - partition_bits - USERVERTEX_PADDING_BITWIDTH)
        self.partition_offset = 64 - partition_bits

    # --- construction ---
    def _construct_id(self, count, partition, vtype):
        if not 0 <= partition < self.partition_bound:
            raise ValueError(f"Invalid partition: {partition}")
        if count < 0 or count.bit_length() + self.partition_bits + (vtype.offset if vtype else 0) > TOTAL_BITS:
            raise ValueError(f"Invalid count: {count}")
        vid = (count << self.partition_bits) + partition
        return vtype.add_padding(vid) if vtype else vid

    def get_vertex_id(self, count, partition, vtype: VertexIDType):
        if not 0 < count < self.vertex_count_bound:
            raise ValueError(f"Invalid count for bound: {count}")
        if vtype is VertexIDType.PartitionedVertex:
            if partition != PARTITIONED_VERTEX_PARTITION:
                raise ValueError("partitioned vertices live in PARTITIONED_VERTEX_PARTITION")
            return self._canonical_from_count(count)
        return self._construct_id(count, partition, vtype)

    def to_vertex_id(self, user_id: int) -> int:
        if user_id <= 0:
            raise ValueError(f"Vertex id must be positive: {user_id}")
        if user_id >= self.vertex_count_bound:
            raise ValueError(f"Vertex id is too large: {user_id}")
        return user_id << (self.partition_bits + USERVERTEX_PADDING_BITWIDTH)

    def from_vertex_id(self, vid: int) -> int:
        shift = USERVERTEX_PADDING_BITWIDTH + self.partition_bits
        if not (vid >> shift > 0 and vid <= (self.vertex_count_bound - 1) << shift):
            raise ValueError(f"Invalid vertex id provided: {vid}")
        return vid >> shift

    # --- inspection ---
    def user_vertex_type(self, vid):
        for t in USER_VERTEX_TYPES:
            if t.is_(vid):
                return t
        raise ValueError(f"Vertex ID {vid} has unrecognized type")

    def is_user_vertex_id(self, vid):
        return any(t.is_(vid) for t in USER_VERTEX_TYPES) and (vid >> (self.partition_bits + 3)) > 0

    def get_partition_id(self, vid):
        return (vid >> USERVERTEX_PADDING_BITWIDTH) & (self.partition_bound - 1)

    def is_partitioned_vertex(self, vid):
        return self.is_user_vertex_id(vid) and VertexIDType.PartitionedVertex.is_(vid)

    # --- row keys ---
    def get_key(self, vid) -> int:
        """8-byte row key as an unsigned 64-bit integer (big-endian buffer value)."""
        vtype = self.user_vertex_type(vid)
        partition = self.get_partition_id(vid)
        count = vid >> (self.partition_bits + USERVERTEX_PADDING_BITWIDTH)
        if count <= 0:
            raise ValueError("count must be positive")
        shifted = (partition << (self.partition_offset & 63)) & _MASK64  # Java masks the shift distance
        return shifted | vtype.add_padding(count)

    def get_key_id(self, key: int) -> int:
        value = _signed64(key)
        vtype = self.user_vertex_type(value)
        u = value & _MASK64
        partition = (u >> self.partition_offset) if self.partition_offset < 64 else 0
        count = (u >> USERVERTEX_PADDING_BITWIDTH) & ((1 << (self.partition_offset - USERVERTEX_PADDING_BITWIDTH)) - 1)
        return self._construct_id(count, partition, vtype)

    # --- partitioned (vertex-cut) vertices ---
    def get_partition_hash_for_id(self, vid):
        if vid <= 0 or self.partition_bits <= 0:
            raise ValueError("need a positive id and partition bits")
        result, offset = 0, 0
        while offset < 64:
            result ^= (vid >> offset) & (self.partition_bound - 1)
            offset += self.partition_bits
        return result

    def _canonical_from_count(self, count):
        return self._construct_id(count, self.get_partition_hash_for_id(count), VertexIDType.PartitionedVertex)

    def get_canonical_vertex_id(self, partitioned_vid):
        if not VertexIDType.PartitionedVertex.is_(partitioned_vid):
            raise ValueError("not a partitioned vertex id")
        return self._canonical_from_count(partitioned_vid >> (self.partition_bits + USERVERTEX_PADDING_BITWIDTH))

    def get_partitioned_vertex_representatives(self, partitioned_vid):
        count = partitioned_vid >> (self.partition_bits + USERVERTEX_PADDING_BITWIDTH)
        return [self._construct_id(count, p, VertexIDType.PartitionedVertex) for p in range(self.partition_bound)]

    def canonical_id(self, vid):
        """FulgoraVertexMemory.getCanonicalId: representatives of a partitioned vertex collapse."""
        return self.get_canonical_vertex_id(vid) if self.is_partitioned_vertex(vid) else vid
