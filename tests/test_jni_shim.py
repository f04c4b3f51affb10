"""The Java drop-in's JNI boundary, checked without a JDK (none is installed here or on the GPU box):
every `static native` method of JanusGpu.java has a JNI function in java/native/janusgpu_jni.c with the
mangled name, the same number of arguments and matching JNI types, and every C-ABI entry point the shim
calls is declared in include/janusgpu.h and exported by libjanusgpu.so."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "org", "janusgraph", "graphdb", "olap", "computer")
SHIM = os.path.join(ROOT, "java", "native", "janusgpu_jni.c")
HEADER = os.path.join(ROOT, "include", "janusgpu.h")

JNI_TYPE = {"int": "jint", "long": "jlong", "double": "jdouble", "ByteBuffer": "jobject", "int[]": "jintArray",
            "long[]": "jlongArray", "double[]": "jdoubleArray", "String": "jstring",
            "ByteBuffer[]": "jobjectArray"}


def java_natives():
    src = open(os.path.join(JAVA, "JanusGpu.java")).read()
    out = {}
    for ret, name, args in re.findall(r"static native (\w+(?:\[\])?) (\w+)\(([^)]*)\);", src, re.S):
        types = [a.strip().rsplit(" ", 1)[0] for a in args.split(",") if a.strip()]
        out[name] = (ret, types)
    return out


def shim_functions():
    src = open(SHIM).read()
    out = {}
    for ret, name, args in re.findall(r"JNIEXPORT (\w+) JNICALL FN\((\w+)\)\(([^)]*)\)", src, re.S):
        types = [a.strip().rsplit(" ", 1)[0].strip() for a in args.split(",")]
        assert types[:2] == ["JNIEnv*", "jclass"], name
        out[name] = (ret, types[2:])
    return out, src


def test_every_native_has_its_jni_function():
    natives = java_natives()
    shim, _ = shim_functions()
    assert natives and set(natives) == set(shim)
    for name, (ret, jtypes) in natives.items():
        cret, ctypes_ = shim[name]
        assert cret == JNI_TYPE[ret], name
        assert ctypes_ == [JNI_TYPE[t] for t in jtypes], name


def test_shim_calls_only_declared_exported_entry_points():
    from janusgraph_amd import _lib
    _, src = shim_functions()
    header = open(HEADER).read()
    called = set(re.findall(r"\b(jg_[a-z_0-9]+)\(", src))
    assert called
    for f in called:
        assert re.search(r"\b" + f + r"\(", header), f
        assert f in _lib.EXPORTS, f


def test_java_sources_reference_existing_natives():
    natives = java_natives()
    used = set()
    for fn in os.listdir(JAVA):
        if fn.endswith(".java") and fn != "JanusGpu.java":
            used |= set(re.findall(r"JanusGpu\.(\w+)\(", open(os.path.join(JAVA, fn)).read()))
    assert used and used <= set(natives) | {"check"}
