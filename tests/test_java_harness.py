"""The Java drop-in and its conformance harness, checked statically against the reference (no JDK here or
on the GPU box, so nothing compiles): both patches apply to the reference tree, every org.janusgraph
import of java/ resolves to a reference source file (or one of ours), and every reference member the
drop-in and the harness use exists with the visibility they need (after the patches).  TinkerPop classes
are third party (gremlin-core 3.4.6, not in the container) and are not checked.  Skipped where the
reference tree is absent."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
JAVA = os.path.join(ROOT, "java")
PATCHES = sorted(os.path.join(JAVA, "patches", p) for p in os.listdir(os.path.join(JAVA, "patches")))

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")

CORE = "janusgraph-core/src/main/java/org/janusgraph"


@pytest.fixture(scope="module")
def patched(tmp_path_factory):
    """janusgraph-core (and the test utilities) with java/patches applied."""
    d = tmp_path_factory.mktemp("ref")
    shutil.copytree(os.path.join(REF, "janusgraph-core"), d / "janusgraph-core")
    for p in PATCHES:
        r = subprocess.run(["patch", "-p1", "-s", "-i", p], cwd=d, capture_output=True, text=True)
        assert r.returncode == 0, f"{os.path.basename(p)} does not apply: {r.stdout}{r.stderr}"
    return d


def java_sources():
    for base, _, files in os.walk(JAVA):
        for f in files:
            if f.endswith(".java"):
                yield os.path.join(base, f)


def reference_classes():
    found = {}
    for module in os.listdir(REF):
        for sub in ("src/main/java", "src/test/java"):
            top = os.path.join(REF, module, sub)
            for base, _, files in os.walk(top):
                for f in files:
                    if f.endswith(".java"):
                        rel = os.path.relpath(os.path.join(base, f[:-5]), top)
                        found[rel.replace(os.sep, ".")] = os.path.join(base, f)
    return found


def test_patches_apply(patched):
    assert (patched / CORE / "graphdb/olap/computer/FulgoraGraphComputer.java").exists()


def test_janusgraph_imports_resolve():
    ref = reference_classes()
    ours = {}
    for path in java_sources():
        pkg = re.search(r"^package ([\w.]+);", open(path).read(), re.M).group(1)
        ours[pkg + "." + os.path.basename(path)[:-5]] = path
    missing = []
    for path in java_sources():
        for imp in re.findall(r"^import (org\.janusgraph\.[\w.]+);", open(path).read(), re.M):
            if imp not in ref and imp not in ours:
                missing.append((os.path.relpath(path, ROOT), imp))
    assert not missing, missing


# (file under the patched janusgraph-core or the reference, regex) for every reference member java/ uses
MEMBERS = [
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected FulgoraMemory memory;"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected FulgoraVertexMemory vertexMemory;"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected int numThreads"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected ResultGraph resultGraphMode"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected Persist persistMode"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected void guardAgainstDuplicateSubmission\(\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected void ensureSettingsAreValid\(\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java", r"protected void initializeMemory\(\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java",
     r"protected Map<MapReduce, FulgoraMapEmitter> collectMapJobs\(\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java",
     r"protected void executeMapJobs\(Map<MapReduce, FulgoraMapEmitter> mapJobs\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java",
     r"protected void executeReducePhase\(Map<MapReduce, FulgoraMapEmitter> mapJobs\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraGraphComputer.java",
     r"public FulgoraGraphComputer\(final StandardJanusGraph graph, final Configuration configuration\)"),
    (f"{CORE}/graphdb/tinkerpop/JanusGraphBlueprintsGraph.java", r"graphComputerClass\.equals\(GpuGraphComputer\.class\)"),
    (f"{CORE}/graphdb/tinkerpop/JanusGraphBlueprintsGraph.java",
     r"getConfiguration\(\)\.getConfiguration\(\)\.get\(GraphDatabaseConfiguration\.COMPUTER_GPU_DEFAULT\)"),
    (f"{CORE}/diskstorage/configuration/ModifiableConfiguration.java",
     r"public ModifiableConfiguration\(ConfigNamespace root, WriteConfiguration config, Restriction restriction\)"),
    (f"{CORE}/diskstorage/configuration/BasicConfiguration.java", r"public enum Restriction \{ LOCAL, GLOBAL, NONE \}"),
    (f"{CORE}/graphdb/olap/computer/FulgoraMemory.java", r"public FulgoraMemory\(final VertexProgram<\?> vertexProgram"),
    (f"{CORE}/graphdb/olap/computer/FulgoraMemory.java", r"void attachReferenceElements\(Graph graph\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraMemory.java", r"void setIteration\(final int iteration\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraVertexMemory.java", r"void setProperty\(long vertexId, String key, V value\)"),
    (f"{CORE}/graphdb/olap/computer/FulgoraMapEmitter.java", r"public void emit\("),
    (f"{CORE}/graphdb/olap/QueryContainer.java", r"public static final int DEFAULT_HARD_QUERY_LIMIT"),
    (f"{CORE}/graphdb/olap/VertexJobConverter.java", r"public static StandardJanusGraphTx startTransaction\("),
    (f"{CORE}/graphdb/idmanagement/IDManager.java", r"public static long stripRelationTypePadding\(long id\)"),
    (f"{CORE}/graphdb/idmanagement/IDManager.java", r"public long getPartitionBound\(\)"),
    (f"{CORE}/graphdb/idmanagement/IDManager.java", r"public long getKeyID\(StaticBuffer b\)"),
    (f"{CORE}/graphdb/internal/InternalRelationType.java", r"long\[\] getSignature\(\);"),
    (f"{CORE}/graphdb/internal/InternalRelationType.java", r"long\[\] getSortKey\(\);"),
    (f"{CORE}/graphdb/database/EdgeSerializer.java", r"public Direction parseDirection\(Entry data\)"),
    (f"{CORE}/graphdb/database/EdgeSerializer.java", r"public RelationCache parseRelation\(Entry data, boolean excludeProperties"),
    (f"{CORE}/graphdb/relations/RelationCache.java", r"public final long typeId;"),
    (f"{CORE}/graphdb/util/WorkerPool.java", r"public void submit\("),
    ("janusgraph-backend-testutils/src/main/java/org/janusgraph/blueprints/AbstractJanusGraphComputerProvider.java",
     r"public ModifiableConfiguration getJanusGraphConfiguration\(String graphName, Class<\?> test, String testMethodName\)"),
    ("janusgraph-backend-testutils/src/main/java/org/janusgraph/StorageSetup.java",
     r"public static ModifiableConfiguration getInMemoryConfiguration\(\)"),
    (f"{CORE}/graphdb/configuration/GraphDatabaseConfiguration.java", r"ConfigOption<Boolean> STORAGE_TRANSACTIONAL"),
    ("janusgraph-inmemory/src/test/java/org/janusgraph/graphdb/inmemory/InMemoryOLAPTest.java",
     r"public class InMemoryOLAPTest extends OLAPTest"),
]


@pytest.mark.parametrize("path,pattern", MEMBERS, ids=[p.split("/")[-1] + ":" + r[:40] for p, r in MEMBERS])
def test_reference_member_exists(patched, path, pattern):
    f = patched / path if path.startswith("janusgraph-core/") else os.path.join(REF, path)
    assert re.search(pattern, open(f).read()), f"{path}: no match for {pattern}"


# computer.gpu.* (VERDICT r03 item 7): the options GpuGraphComputer and the harness read
GPU_OPTIONS = {"COMPUTER_GPU_DEFAULT": ("Boolean", "default"), "COMPUTER_GPU_DEVICES": ("String[]", "devices"),
               "COMPUTER_GPU_UNTRUNCATED": ("Boolean", "untruncated"),
               "COMPUTER_GPU_DIRECT_MEMORY": ("Long", "direct-memory")}


def test_gpu_options_registered_under_computer_ns(patched):
    """Every GraphDatabaseConfiguration.COMPUTER_GPU_* that java/ uses is a ConfigOption of the type the code
    reads, in the computer.gpu namespace (a child of COMPUTER_NS, next to computer.result-mode), MASKABLE
    (per graph), built with a ConfigOption constructor the reference has; no name collides in the namespace."""
    gdc = open(patched / CORE / "graphdb/configuration/GraphDatabaseConfiguration.java").read()
    assert re.search(r'ConfigNamespace COMPUTER_GPU_NS = new ConfigNamespace\(COMPUTER_NS,"gpu",', gdc)
    used = set()
    for path in java_sources():
        used |= set(re.findall(r"GraphDatabaseConfiguration\.(COMPUTER_GPU_\w+)", open(path).read()))
    used |= set(re.findall(r"GraphDatabaseConfiguration\.(COMPUTER_GPU_\w+)",
                           open(patched / CORE / "graphdb/tinkerpop/JanusGraphBlueprintsGraph.java").read()))
    assert used == set(GPU_OPTIONS), used
    names = []
    for const, (typ, name) in GPU_OPTIONS.items():
        m = re.search(r"public static final ConfigOption<" + re.escape(typ) + r"> " + const +
                      r' = new ConfigOption<>\(COMPUTER_GPU_NS,"([\w-]+)",(.*?);\n', gdc, re.S)
        assert m, const
        assert m.group(1) == name and "ConfigOption.Type.MASKABLE" in m.group(2), const
        names.append(m.group(1))
    assert len(set(names)) == len(names)
    opt = open(patched / CORE / "diskstorage/configuration/ConfigOption.java").read()
    assert re.search(r"public ConfigOption\(ConfigNamespace parent, String name, String description, Type type, "
                     r"O defaultValue\)", opt)
    assert re.search(r"enum Type \{", opt) and "MASKABLE" in opt


def test_drop_in_reads_no_system_properties():
    """The drop-in's settings come from the graph's configuration only (two graphs in one JVM may differ)."""
    for path in java_sources():
        src = open(path).read()
        assert "System.getProperty" not in src and "Boolean.getBoolean" not in src, path
