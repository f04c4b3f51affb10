"""IDManager mirror against IDManagementTest (janusgraph-test/.../idmanagement/IDManagementTest.java:48-114)."""
import pytest

from janusgraph_amd.idmanager import (PARTITIONED_VERTEX_PARTITION, USER_VERTEX_TYPES, IDManager, VertexIDType)


@pytest.mark.parametrize("pbits,partition,lo,hi", [(12, 2341, 1234123, 1234623), (16, 64000, 582919, 583219),
                                                    (4, 14, 1, 1000), (10, 1, 903392, 903592),
                                                    (0, 0, 242342, 243342)])
def test_entity_id_round_trip(pbits, partition, lo, hi):
    """testEntityID: user vertex ids of every type round-trip through getKey/getKeyID."""
    eid = IDManager(pbits)
    assert eid.partition_bound > 0 and eid.vertex_count_bound > 0
    for count in range(lo, hi):
        for vtype in USER_VERTEX_TYPES:
            if pbits == 0 and vtype is VertexIDType.PartitionedVertex:
                continue
            p = PARTITIONED_VERTEX_PARTITION if vtype is VertexIDType.PartitionedVertex else partition
            vid = eid.get_vertex_id(count, p, vtype)
            assert eid.is_user_vertex_id(vid)
            assert vtype.is_(vid)
            if vtype is not VertexIDType.PartitionedVertex:
                assert eid.get_partition_id(vid) == partition
            assert eid.get_key_id(eid.get_key(vid)) == vid


def test_entity_id_rejects():
    with pytest.raises(ValueError):
        IDManager(0).get_vertex_id(242342, 1, VertexIDType.NormalVertex)  # partition out of bound
    with pytest.raises(ValueError):
        IDManager(0).get_vertex_id(-11, 0, VertexIDType.NormalVertex)
    with pytest.raises(ValueError):
        IDManager(17)


def test_user_ids_set_vertex_id():
    """toVertexId/fromVertexId (IDManager.java:578-595): i << (partitionBits + 3)."""
    idm = IDManager(5)
    for i in (1, 2, 255, 10**9):
        vid = idm.to_vertex_id(i)
        assert vid == i << 8 and idm.from_vertex_id(vid) == i
        assert idm.is_user_vertex_id(vid) and VertexIDType.NormalVertex.is_(vid)
    with pytest.raises(ValueError):
        idm.to_vertex_id(0)


def test_partitioned_vertex_canonical_ids():
    """Representatives of a vertex-cut vertex collapse onto one canonical id (FulgoraVertexMemory:74-77)."""
    idm = IDManager(5)
    canon = idm.get_vertex_id(777, PARTITIONED_VERTEX_PARTITION, VertexIDType.PartitionedVertex)
    reps = idm.get_partitioned_vertex_representatives(canon)
    assert len(reps) == 32 and canon in reps
    assert {idm.canonical_id(r) for r in reps} == {canon}
    normal = idm.get_vertex_id(777, 3, VertexIDType.NormalVertex)
    assert idm.canonical_id(normal) == normal
