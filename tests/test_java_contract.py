"""The Java plugin layer (java/) against the native JNI shim, without a JVM (no JDK in this image).

The shim (csrc/bridge/jni_shim.cc) binds to the Java side by name and JNI descriptor: natives are
found through their mangled symbol names, callbacks through GetStaticMethodID, the index record
through GetFieldID. A mismatch only shows at run time inside Hadoop, so it is pinned here by parsing
both sides. The command ids and the INIT parameter count are checked against csrc/include/uda/cmd.h.
"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java")
SHARED = os.path.join(JAVA, "shared", "com", "mellanox", "hadoop", "mapred")
SHIM = os.path.join(ROOT, "csrc", "bridge", "jni_shim.cc")
LIBUDA = os.path.join(ROOT, "uda_amd", "lib", "libuda.so")

PRIM = {"void": "V", "boolean": "Z", "byte": "B", "char": "C", "short": "S", "int": "I", "long": "J",
        "float": "F", "double": "D"}
CLASSES = {"String": "Ljava/lang/String;", "Object": "Ljava/lang/Object;"}


def _desc(t: str) -> str:
    t = t.strip()
    if t.endswith("[]"):
        return "[" + _desc(t[:-2])
    if t in PRIM:
        return PRIM[t]
    return CLASSES[t]


def _method_desc(ret: str, params: str) -> str:
    args = []
    for p in filter(None, (x.strip() for x in params.split(","))):
        typ, name = p.rsplit(None, 1)
        if name.endswith("[]"):
            typ += "[]"
        args.append(_desc(typ))
    return "(" + "".join(args) + ")" + _desc(ret)


def _read(path):
    with open(path) as f:
        return f.read()


def _bridge_methods():
    src = _read(os.path.join(SHARED, "UdaBridge.java"))
    natives, statics = {}, {}
    for m in re.finditer(r"private static native (\w+(?:\[\])?) (\w+)\(([^)]*)\);", src):
        natives[m.group(2)] = _method_desc(m.group(1), m.group(3))
    for m in re.finditer(r"public static (\w+(?:\[\])?) (\w+)\(([^)]*)\)", src):
        statics[m.group(2)] = _method_desc(m.group(1), m.group(3))
    return natives, statics


def test_native_methods_are_exported_with_jni_names(native):  # `native` ensures the build exists
    natives, _ = _bridge_methods()
    assert natives == {
        "startNative": "(Z[Ljava/lang/String;IZ)I",
        "doCommandNative": "(Ljava/lang/String;)V",
        "reduceExitMsgNative": "()V",
        "setLogLevelNative": "(I)V",
    }
    lib = ctypes.CDLL(LIBUDA)
    for name in natives:
        assert hasattr(lib, "Java_com_mellanox_hadoop_mapred_UdaBridge_" + name), name
    assert hasattr(lib, "JNI_OnLoad")
    # the shim's C signatures take the same JNI types in the same order
    shim = _read(SHIM)
    sig = re.search(r"UdaBridge_startNative\(\s*JNIEnv\* e, jclass, (.*?)\)", shim, re.S).group(1)
    assert [a.split()[0] for a in sig.split(",")] == ["jboolean", "jobjectArray", "jint", "jboolean"]


def test_callbacks_match_shim_method_ids():
    _, statics = _bridge_methods()
    shim = _read(SHIM)
    looked_up = dict(re.findall(r'GetStaticMethodID\(e, g\.bridge, "(\w+)", "([^"]+)"\)', shim))
    assert set(looked_up) == {"fetchOverMessage", "dataFromUda", "getPathUda", "getConfData", "logToJava",
                              "failureInUda"}
    for name, desc in looked_up.items():
        assert statics.get(name) == desc, (name, statics.get(name), desc)
    assert re.search(r'kBridgeClass = "com/mellanox/hadoop/mapred/UdaBridge"', shim)
    assert re.search(r'kExceptionClass = "com/mellanox/hadoop/mapred/UdaRuntimeException"', shim)
    assert os.path.exists(os.path.join(SHARED, "UdaRuntimeException.java"))


def test_index_record_fields_match_shim():
    src = _read(os.path.join(JAVA, "shared", "org", "apache", "hadoop", "mapred", "IndexRecordBridge.java"))
    fields = {name: _desc(typ) for typ, name in re.findall(r"public (long|String) (\w+);", src)}
    shim = _read(SHIM)
    wanted = dict(re.findall(r'GetFieldID\(e, c, "(\w+)", "([^"]+)"\)', shim))
    assert wanted == {"startOffset": "J", "rawLength": "J", "partLength": "J", "pathMOF": "Ljava/lang/String;"}
    assert fields == wanted


def test_command_ids_and_format_match_native(native):
    src = _read(os.path.join(SHARED, "UdaCmd.java"))
    java_ids = {k: int(v) for k, v in re.findall(r"static final int (\w+) = (\d+);", src)}
    hdr = _read(os.path.join(ROOT, "csrc", "include", "uda", "cmd.h"))
    native_ids = {k: int(v) for k, v in re.findall(r"(k\w+) = (\d+),", hdr)}
    pairs = {"EXIT_COMMAND": "kExitMsg", "NEW_MAP_COMMAND": "kNewMapMsg", "FINAL_MERGE_COMMAND": "kFinalMsg",
             "RESULT_COMMAND": "kResult", "FETCH_COMMAND": "kFetchMsg", "FETCH_OVER_COMMAND": "kFetchOverMsg",
             "JOB_OVER_COMMAND": "kJobOverMsg", "INIT_COMMAND": "kInitMsg", "MORE_COMMAND": "kMoreMsg",
             "NETLEV_REDUCE_LAUNCHED": "kRtLaunched"}
    for j, n in pairs.items():
        assert java_ids[j] == native_ids[n], j
    # formCmd: "<params+1>:<id>:p1:...": the Java builder and the native formatter agree
    assert "append(params.size() + 1).append(':').append(id)" in src
    assert native.form_cmd(4, ["h", "job_1", "attempt_1_m_0", "3"]) == "5:4:h:job_1:attempt_1_m_0:3"


def test_init_parameters_in_native_order(native):
    src = _read(os.path.join(SHARED, "UdaPluginRT.java"))
    body = src[src.index("List<String> p = new ArrayList<String>();"):src.index("p.addAll(dirs);")]
    assert body.count("p.add(") == 11  # numMaps .. numDirs, then the dirs
    # the native parser accepts exactly that shape (numDirs = 2 + two dirs)
    params = ["7", "job_1", "attempt_1_r_000000_0", "0", "1048576", "16384", "org.apache.hadoop.io.Text",
              "null", "262144", "0", "2", "/a", "/b"]
    count, cid, got = native.parse_cmd(native.form_cmd(7, params))
    assert cid == 7 and count == len(params) + 1 and got == params


@pytest.mark.parametrize("flavor,classes", [
    ("yarn", ["com/mellanox/hadoop/mapred/UdaShuffleConsumerPlugin.java",
              "com/mellanox/hadoop/mapred/UdaShuffleHandler.java",
              "org/apache/hadoop/mapred/UdaMapredBridge.java"]),
    ("hadoop-1", ["com/mellanox/hadoop/mapred/UdaShuffleConsumerPlugin.java",
                  "com/mellanox/hadoop/mapred/UdaShuffleProviderPlugin.java",
                  "org/apache/hadoop/mapred/UdaMapredBridge.java",
                  "org/apache/hadoop/mapred/LRUCacheBridgeHadoop1.java"]),
    ("hadoop-1-old", ["com/mellanox/hadoop/mapred/UdaShuffleConsumerPlugin.java"]),
    ("yarn-2.0", ["com/mellanox/hadoop/mapred/UdaShuffleHandler.java"]),
])
def test_version_front_ends_present(flavor, classes):
    for c in classes:
        src = _read(os.path.join(JAVA, flavor, c))
        pkg = os.path.dirname(c).replace("/", ".")
        assert f"package {pkg};" in src
        assert f"class {os.path.basename(c)[:-5]}" in src


def test_health_signal_strings():
    """tools/regression.py (and the reference's testStatusAnalyzer.sh) count these log lines."""
    src = _read(os.path.join(SHARED, "UdaShuffleConsumerPluginShared.java"))
    assert "init - Using UdaShuffleConsumerPlugin" in src
    assert "====XXX Successfully closed UdaShuffleConsumerPlugin XXX====" in src


def test_older_front_end_apis():
    """mlx-1.x-old: the consumer extends the abstract ShuffleConsumerPlugin with the 4-argument init;
    mlx-2.0.x: the provider is an AbstractService implementing AuxServices.AuxiliaryService (initApp /
    stopApp), and still sends JOB_OVER when an application stops."""
    old = _read(os.path.join(JAVA, "hadoop-1-old", "com/mellanox/hadoop/mapred/UdaShuffleConsumerPlugin.java"))
    assert "extends ShuffleConsumerPlugin implements UdaConsumerPluginCallable" in old
    assert "init(ReduceTask reduceTask, TaskUmbilicalProtocol umb, JobConf conf, Reporter reporter)" in old
    y20 = _read(os.path.join(JAVA, "yarn-2.0", "com/mellanox/hadoop/mapred/UdaShuffleHandler.java"))
    assert "extends AbstractService" in y20 and "AuxServices.AuxiliaryService" in y20
    assert "public void initApp(String user, ApplicationId appId, ByteBuffer secret)" in y20
    assert "public void stopApp(ApplicationId appId)" in y20 and "JOB_OVER_COMMAND" in y20
