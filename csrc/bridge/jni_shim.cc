// JNI entry points of libuda.so for the unchanged Java plugin classes
// (com.mellanox.hadoop.mapred.UdaBridge, plugins/shared/com/mellanox/hadoop/mapred/UdaBridge.java:49-145).
//
// The shim is a thin adapter from JNI to the C ABI (uda/uda_bridge.h): natives -> uda_start /
// uda_do_command / uda_reduce_exit / uda_set_log_level, and the C callback vtable -> the six static
// Java callbacks. Reference behaviour kept (src/UdaBridge.cc):
//   * JNI_OnLoad caches the JavaVM, a global ref to UdaBridge and the callback method IDs (:110-174);
//   * native threads that call back into Java attach themselves as daemons on first use and detach
//     when the thread exits (attachNativeThread / detachNativeThread, :459-502);
//   * dataFromUda receives a java.nio DirectByteBuffer over the native buffer plus its length
//     (registerDirectByteBuffer, :535-551) — no copy on the native side;
//   * getPathUda returns an IndexRecordBridge whose startOffset/rawLength/partLength/pathMOF fields
//     are read back (:352-415);
//   * a failing native entry point raises com.mellanox.hadoop.mapred.UdaRuntimeException in the
//     calling Java thread (exceptionInJniThread, :81-107); failures on native threads go through
//     failureInUda exactly once (the C ABI's failure latch).
// Differences: the JNI table is called through in-tree declarations (jni_abi.h, no JDK needed to
// build), only non-varargs call forms are used, and local references created on attached native
// threads are deleted eagerly (those threads never return to Java to free them).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "jni_abi.h"
#include "uda/uda_bridge.h"

using namespace uda::jni;

namespace {

constexpr const char* kBridgeClass = "com/mellanox/hadoop/mapred/UdaBridge";
constexpr const char* kExceptionClass = "com/mellanox/hadoop/mapred/UdaRuntimeException";

struct State {
  JavaVM* vm = nullptr;
  jclass bridge = nullptr;
  jmethodID fetch_over = nullptr, data = nullptr, get_path = nullptr, get_conf = nullptr, log = nullptr,
            failure = nullptr;
  std::mutex mu;
  uda_handle* provider = nullptr;
  uda_handle* consumer = nullptr;
  // IndexRecordBridge field IDs, resolved on the first getPathUda
  std::mutex fid_mu;
  jfieldID f_start = nullptr, f_raw = nullptr, f_part = nullptr, f_path = nullptr;
};
State g;

struct ThreadEnv {
  JNIEnv* env = nullptr;
  bool attached = false;
  ~ThreadEnv() {
    if (attached && g.vm) DetachCurrentThread(g.vm);
  }
};
thread_local ThreadEnv t_env;

JNIEnv* thread_env() {
  if (t_env.env) return t_env.env;
  if (!g.vm) return nullptr;
  JNIEnv* e = nullptr;
  if (GetEnv(g.vm, &e, JNI_VERSION_1_4) == JNI_OK && e) {
    t_env.env = e;
    return e;
  }
  if (AttachCurrentThreadAsDaemon(g.vm, &e) == JNI_OK && e) {
    t_env.env = e;
    t_env.attached = true;
    return e;
  }
  return nullptr;
}

// Clear a pending Java exception raised by a callback; true if there was one.
bool take_exception(JNIEnv* e) {
  if (!ExceptionCheck(e)) return false;
  ExceptionDescribe(e);
  ExceptionClear(e);
  return true;
}

void throw_uda(JNIEnv* e, const std::string& msg) {
  jclass c = FindClass(e, kExceptionClass);
  if (c) {
    ThrowNew(e, c, msg.c_str());
    DeleteLocalRef(e, c);
  }  // else NoClassDefFoundError is already pending
}

std::string utf(JNIEnv* e, jstring s) {
  if (!s) return std::string();
  const char* c = GetStringUTFChars(e, s);
  if (!c) return std::string();
  std::string out(c);
  ReleaseStringUTFChars(e, s, c);
  return out;
}

// ---- C ABI callbacks -> static Java methods
void cb_fetch_over(void*) {
  JNIEnv* e = thread_env();
  if (!e) return;
  CallStaticVoidMethodA(e, g.bridge, g.fetch_over, nullptr);
  take_exception(e);
}

int cb_data(void*, const void* buf, int32_t len) {
  JNIEnv* e = thread_env();
  if (!e) return -1;
  jobject bb = NewDirectByteBuffer(e, const_cast<void*>(buf), (jlong)len);
  if (!bb) {
    take_exception(e);
    return -1;
  }
  jvalue a[2];
  a[0].l = bb;
  a[1].i = len;
  CallStaticVoidMethodA(e, g.bridge, g.data, a);
  DeleteLocalRef(e, bb);
  return take_exception(e) ? -1 : 0;
}

int cb_get_path(void*, const char* job, const char* map, int32_t reduce, uda_index_record* out) {
  JNIEnv* e = thread_env();
  if (!e) return -1;
  jstring js = NewStringUTF(e, job), ms = NewStringUTF(e, map);
  jvalue a[3];
  a[0].l = js;
  a[1].l = ms;
  a[2].i = reduce;
  jobject rec = CallStaticObjectMethodA(e, g.bridge, g.get_path, a);
  DeleteLocalRef(e, js);
  DeleteLocalRef(e, ms);
  if (take_exception(e) || !rec) {
    DeleteLocalRef(e, rec);
    return -1;
  }
  {
    std::lock_guard<std::mutex> lk(g.fid_mu);
    if (!g.f_start) {
      jclass c = GetObjectClass(e, rec);
      g.f_start = GetFieldID(e, c, "startOffset", "J");
      g.f_raw = GetFieldID(e, c, "rawLength", "J");
      g.f_part = GetFieldID(e, c, "partLength", "J");
      g.f_path = GetFieldID(e, c, "pathMOF", "Ljava/lang/String;");
      DeleteLocalRef(e, c);
      if (take_exception(e) || !g.f_start || !g.f_raw || !g.f_part || !g.f_path) {
        g.f_start = nullptr;
        DeleteLocalRef(e, rec);
        return -1;
      }
    }
  }
  out->start_offset = GetLongField(e, rec, g.f_start);
  out->raw_length = GetLongField(e, rec, g.f_raw);
  out->part_length = GetLongField(e, rec, g.f_part);
  jstring p = (jstring)GetObjectField(e, rec, g.f_path);
  const std::string path = utf(e, p);
  DeleteLocalRef(e, p);
  DeleteLocalRef(e, rec);
  std::strncpy(out->path, path.c_str(), UDA_PATH_MAX - 1);
  out->path[UDA_PATH_MAX - 1] = 0;
  return 0;
}

int cb_get_conf(void*, const char* key, const char* dflt, char* out, int32_t outlen) {
  JNIEnv* e = thread_env();
  std::string v = dflt ? dflt : "";
  if (e) {
    jstring k = NewStringUTF(e, key), d = NewStringUTF(e, v.c_str());
    jvalue a[2];
    a[0].l = k;
    a[1].l = d;
    jstring r = (jstring)CallStaticObjectMethodA(e, g.bridge, g.get_conf, a);
    if (!take_exception(e) && r) v = utf(e, r);
    DeleteLocalRef(e, r);
    DeleteLocalRef(e, k);
    DeleteLocalRef(e, d);
  }
  if (outlen <= 0) return -1;
  const int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)outlen - 1);
  std::memcpy(out, v.data(), (size_t)n);
  out[n] = 0;
  return n;
}

void cb_log(void*, const char* msg, int32_t sev) {
  JNIEnv* e = thread_env();
  if (!e) return;
  jstring m = NewStringUTF(e, msg);
  jvalue a[2];
  a[0].l = m;
  a[1].i = sev;
  CallStaticVoidMethodA(e, g.bridge, g.log, a);
  DeleteLocalRef(e, m);
  take_exception(e);
}

void cb_failure(void*, const char*) {
  JNIEnv* e = thread_env();
  if (!e) return;
  CallStaticVoidMethodA(e, g.bridge, g.failure, nullptr);
  take_exception(e);
}

uda_callbacks java_callbacks() {
  uda_callbacks cb;
  cb.ctx = nullptr;
  cb.fetch_over = cb_fetch_over;
  cb.data_from_uda = cb_data;
  cb.get_path = cb_get_path;
  cb.get_conf = cb_get_conf;
  cb.log = cb_log;
  cb.failure = cb_failure;
  return cb;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) jint JNI_OnLoad(JavaVM* vm, void*) {
  JNIEnv* e = nullptr;
  if (GetEnv(vm, &e, JNI_VERSION_1_4) != JNI_OK || !e) return -1;
  jclass c = FindClass(e, kBridgeClass);
  if (!c) return -1;
  g.vm = vm;
  g.bridge = (jclass)NewGlobalRef(e, c);
  DeleteLocalRef(e, c);
  g.fetch_over = GetStaticMethodID(e, g.bridge, "fetchOverMessage", "()V");
  g.data = GetStaticMethodID(e, g.bridge, "dataFromUda", "(Ljava/lang/Object;I)V");
  g.get_path = GetStaticMethodID(e, g.bridge, "getPathUda", "(Ljava/lang/String;Ljava/lang/String;I)Ljava/lang/Object;");
  g.get_conf = GetStaticMethodID(e, g.bridge, "getConfData", "(Ljava/lang/String;Ljava/lang/String;)Ljava/lang/String;");
  g.log = GetStaticMethodID(e, g.bridge, "logToJava", "(Ljava/lang/String;I)V");
  g.failure = GetStaticMethodID(e, g.bridge, "failureInUda", "()V");
  if (!g.fetch_over || !g.data || !g.get_path || !g.get_conf || !g.log || !g.failure) return -1;
  return JNI_VERSION_1_4;
}

__attribute__((visibility("default"))) void JNI_OnUnload(JavaVM* vm, void*) {
  JNIEnv* e = nullptr;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    if (g.consumer) {
      uda_reduce_exit(g.consumer);
      uda_destroy(g.consumer);
      g.consumer = nullptr;
    }
    if (g.provider) {
      uda_destroy(g.provider);
      g.provider = nullptr;
    }
  }
  if (GetEnv(vm, &e, JNI_VERSION_1_4) == JNI_OK && e && g.bridge) DeleteGlobalRef(e, g.bridge);
  g.bridge = nullptr;
  g.vm = nullptr;
}

__attribute__((visibility("default"))) jint Java_com_mellanox_hadoop_mapred_UdaBridge_startNative(
    JNIEnv* e, jclass, jboolean is_net_merger, jobjectArray args, jint log_level, jboolean log_to_uda_file) {
  t_env.env = e;  // the calling Java thread
  std::vector<std::string> argv;
  const jsize n = args ? GetArrayLength(e, args) : 0;
  for (jsize i = 0; i < n; ++i) {
    jstring s = (jstring)GetObjectArrayElement(e, args, i);
    argv.push_back(utf(e, s));
    DeleteLocalRef(e, s);
  }
  std::vector<const char*> cargv;
  for (auto& a : argv) cargv.push_back(a.c_str());
  const uda_callbacks cb = java_callbacks();
  uda_handle* h = uda_start(is_net_merger ? 1 : 0, (int)cargv.size(), cargv.data(), log_level, log_to_uda_file ? 1 : 0,
                            &cb);
  if (!h) {
    throw_uda(e, is_net_merger ? "NetMerger failed to start" : "MOFSupplier failed to start");
    return -1;
  }
  std::lock_guard<std::mutex> lk(g.mu);
  uda_handle*& slot = is_net_merger ? g.consumer : g.provider;
  if (slot) uda_destroy(slot);
  slot = h;
  return 0;
}

__attribute__((visibility("default"))) void Java_com_mellanox_hadoop_mapred_UdaBridge_doCommandNative(JNIEnv* e,
                                                                                                    jclass,
                                                                                                    jstring s) {
  t_env.env = e;
  const std::string cmd = utf(e, s);
  uda_handle* h;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    h = g.consumer ? g.consumer : g.provider;  // one role per JVM in production (UdaBridge.cc:218-227)
  }
  if (!h) {
    throw_uda(e, "doCommand before startNative");
    return;
  }
  if (uda_do_command(h, cmd.c_str()) != 0) throw_uda(e, std::string("command failed: ") + uda_last_error(h));
}

__attribute__((visibility("default"))) void Java_com_mellanox_hadoop_mapred_UdaBridge_reduceExitMsgNative(JNIEnv* e,
                                                                                                        jclass) {
  t_env.env = e;
  uda_handle* h;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    h = g.consumer;
    g.consumer = nullptr;
  }
  if (!h) return;
  const int rc = uda_reduce_exit(h);
  const std::string err = uda_last_error(h);
  uda_destroy(h);
  if (rc != 0 && !err.empty()) throw_uda(e, "reduce exit: " + err);
}

__attribute__((visibility("default"))) void Java_com_mellanox_hadoop_mapred_UdaBridge_setLogLevelNative(JNIEnv*, jclass,
                                                                                                      jint level) {
  uda_set_log_level(level);
}

}  // extern "C"
