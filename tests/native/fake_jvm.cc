// A fake JVM that loads libuda.so and drives its JNI entry points the way the Java plugin does
// (UdaBridge.java: startNative / doCommandNative / reduceExitMsgNative / setLogLevelNative), with
// the six static callbacks implemented here. It checks the JNI contract from the JVM side:
// every callback arrives on a thread that is attached to the VM, dataFromUda gets a direct buffer,
// local references are balanced, a bad command raises UdaRuntimeException in the caller.
//
// Usage: fake_jvm <libuda.so> <manifest>   (manifest format: see tests/test_jni_shim.py)
// Prints one JSON line of counters; writes the merged stream to the manifest's `out` path.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

namespace {

using jint = int32_t;
using jlong = int64_t;
using jboolean = uint8_t;
union jvalue {
  jboolean z;
  jint i;
  jlong j;
  void* l;
};
using Table = void* const*;  // JNIEnv / JavaVM: pointer to a function table

enum Kind { kClass, kString, kDirect, kIndexRecord, kArray };
struct Obj {
  Kind kind;
  std::string str;            // class name / string value
  void* addr = nullptr;       // direct buffer
  int64_t cap = 0;
  int64_t start = 0, raw = 0, part = 0;
  Obj* path = nullptr;        // IndexRecordBridge.pathMOF
  std::vector<Obj*> items;    // String[]
};

struct Method {
  std::string name, sig;
};
const Method kMethods[] = {
    {"fetchOverMessage", "()V"},
    {"dataFromUda", "(Ljava/lang/Object;I)V"},
    {"getPathUda", "(Ljava/lang/String;Ljava/lang/String;I)Ljava/lang/Object;"},
    {"getConfData", "(Ljava/lang/String;Ljava/lang/String;)Ljava/lang/String;"},
    {"logToJava", "(Ljava/lang/String;I)V"},
    {"failureInUda", "()V"},
};
enum Field { kFStart = 1, kFRaw, kFPart, kFPath };

struct Jvm {
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, std::string> conf;
  std::map<std::string, std::vector<int64_t>> mofs;  // job|map|reduce -> start raw part
  std::map<std::string, std::string> mof_path;
  std::string out;
  bool eof = false;
  std::atomic<int> fetch_over{0}, buffers{0}, failures{0}, logs{0}, unattached_calls{0}, non_direct{0};
  std::atomic<int> hosted{0};  // log lines saying the NetMerger runs in the merge service
  std::atomic<int> attaches{0}, detaches{0}, bad_slot{0};
  std::atomic<long> live_local{0};
  Obj bridge_cls{kClass, "com/mellanox/hadoop/mapred/UdaBridge"};
  Obj exc_cls{kClass, "com/mellanox/hadoop/mapred/UdaRuntimeException"};
  Obj rec_cls{kClass, "org/apache/hadoop/mapred/IndexRecordBridge"};
} J;

thread_local bool t_attached = false;
thread_local std::string t_exception;  // pending exception: "<class>: <message>"

void* g_env_table[234];
void* g_vm_table[8];
Table g_env = g_env_table;
Table g_vm = g_vm_table;

Obj* local(Obj* o) {
  if (o) J.live_local++;
  return o;
}
void check_thread() {
  if (!t_attached) J.unattached_calls++;
}

// ---- JNIEnv functions used by the shim
void* FindClass(Table*, const char* n) {
  check_thread();
  if (J.bridge_cls.str == n) return local(&J.bridge_cls);
  if (J.exc_cls.str == n) return local(&J.exc_cls);
  t_exception = std::string("java/lang/NoClassDefFoundError: ") + n;
  return nullptr;
}
jint ThrowNew(Table*, Obj* c, const char* msg) {
  t_exception = c->str + ": " + msg;
  return 0;
}
void ExceptionDescribe(Table*) { fprintf(stderr, "[fake jvm] exception: %s\n", t_exception.c_str()); }
void ExceptionClear(Table*) { t_exception.clear(); }
jboolean ExceptionCheck(Table*) { return t_exception.empty() ? 0 : 1; }
void* NewGlobalRef(Table*, void* o) { return o; }
void DeleteGlobalRef(Table*, void*) {}
void DeleteLocalRef(Table*, Obj* o) {
  if (!o) return;
  J.live_local--;
  if (o->kind == kString || o->kind == kDirect || o->kind == kIndexRecord) {
    // objects are owned by their last local ref in this fake (the shim never keeps one)
    if (o->kind == kIndexRecord) {
      // its path string is reached through GetObjectField, which hands out its own reference
    }
  }
}
void* GetObjectClass(Table*, Obj* o) { return local(o->kind == kIndexRecord ? &J.rec_cls : &J.bridge_cls); }
void* GetFieldID(Table*, Obj* c, const char* n, const char* sig) {
  if (c != &J.rec_cls) return nullptr;
  const std::string f(n), s(sig);
  if (f == "startOffset" && s == "J") return (void*)(intptr_t)kFStart;
  if (f == "rawLength" && s == "J") return (void*)(intptr_t)kFRaw;
  if (f == "partLength" && s == "J") return (void*)(intptr_t)kFPart;
  if (f == "pathMOF" && s == "Ljava/lang/String;") return (void*)(intptr_t)kFPath;
  t_exception = std::string("java/lang/NoSuchFieldError: ") + n;
  return nullptr;
}
void* GetObjectField(Table*, Obj* o, void* f) {
  check_thread();
  return (intptr_t)f == kFPath ? local(o->path) : nullptr;
}
jlong GetLongField(Table*, Obj* o, void* f) {
  check_thread();
  switch ((intptr_t)f) {
    case kFStart: return o->start;
    case kFRaw: return o->raw;
    case kFPart: return o->part;
  }
  return -1;
}
void* GetStaticMethodID(Table*, Obj* c, const char* n, const char* sig) {
  if (c != &J.bridge_cls) return nullptr;
  for (size_t i = 0; i < sizeof(kMethods) / sizeof(kMethods[0]); ++i)
    if (kMethods[i].name == n && kMethods[i].sig == sig) return (void*)(intptr_t)(i + 1);
  t_exception = std::string("java/lang/NoSuchMethodError: ") + n;
  return nullptr;
}
Obj* NewStringUTF(Table*, const char* s) {
  check_thread();
  Obj* o = new Obj{kString, s};
  return local(o);
}
const char* GetStringUTFChars(Table*, Obj* s, jboolean*) { return s->str.c_str(); }
void ReleaseStringUTFChars(Table*, Obj*, const char*) {}
jint GetArrayLength(Table*, Obj* a) { return (jint)a->items.size(); }
Obj* GetObjectArrayElement(Table*, Obj* a, jint i) { return local(a->items[(size_t)i]); }
Obj* NewDirectByteBuffer(Table*, void* addr, jlong cap) {
  check_thread();
  Obj* o = new Obj{kDirect};
  o->addr = addr;
  o->cap = cap;
  return local(o);
}

void call_void(Table*, Obj*, void* mid, const jvalue* a) {
  check_thread();
  switch ((intptr_t)mid) {
    case 1:
      J.fetch_over++;
      break;
    case 2: {  // dataFromUda(Object directBuf, int len)
      Obj* b = static_cast<Obj*>(a[0].l);
      if (!b || b->kind != kDirect || b->cap < a[1].i) {
        J.non_direct++;
        break;
      }
      std::lock_guard<std::mutex> lk(J.mu);
      J.out.append(static_cast<const char*>(b->addr), (size_t)a[1].i);
      J.buffers++;
      if (a[1].i >= 2 && std::memcmp(static_cast<const char*>(b->addr) + a[1].i - 2, "\xff\xff", 2) == 0) {
        J.eof = true;
        J.cv.notify_all();
      }
      break;
    }
    case 5:
      J.logs++;
      if (a && a[0].l && static_cast<Obj*>(a[0].l)->str.find("hosted by the merge service") != std::string::npos)
        J.hosted++;
      break;
    case 6: {
      std::lock_guard<std::mutex> lk(J.mu);
      J.failures++;
      J.cv.notify_all();
      break;
    }
    default:
      J.bad_slot++;
  }
}
void* call_object(Table*, Obj*, void* mid, const jvalue* a) {
  check_thread();
  if ((intptr_t)mid == 3) {  // getPathUda(jobId, mapId, reduceId)
    const std::string key = static_cast<Obj*>(a[0].l)->str + "|" + static_cast<Obj*>(a[1].l)->str + "|" +
                            std::to_string(a[2].i);
    auto it = J.mofs.find(key);
    if (it == J.mofs.end()) return nullptr;
    Obj* r = new Obj{kIndexRecord};
    r->start = it->second[0];
    r->raw = it->second[1];
    r->part = it->second[2];
    r->path = new Obj{kString, J.mof_path[key]};
    return local(r);
  }
  if ((intptr_t)mid == 4) {  // getConfData(name, default)
    auto it = J.conf.find(static_cast<Obj*>(a[0].l)->str);
    return local(new Obj{kString, it == J.conf.end() ? static_cast<Obj*>(a[1].l)->str : it->second});
  }
  J.bad_slot++;
  return nullptr;
}

// ---- JavaVM invocation interface
jint GetEnv(Table*, void** env, jint) {
  if (!t_attached) {
    *env = nullptr;
    return -2;  // JNI_EDETACHED
  }
  *env = &g_env;
  return 0;
}
jint AttachDaemon(Table*, void** env, void*) {
  t_attached = true;
  J.attaches++;
  *env = &g_env;
  return 0;
}
jint Detach(Table*) {
  t_attached = false;
  J.detaches++;
  return 0;
}

template <int N>
void trap() {
  fprintf(stderr, "[fake jvm] unimplemented JNI slot %d called\n", N);
  J.bad_slot++;
}
template <int... I>
void fill_traps(std::integer_sequence<int, I...>) {
  ((g_env_table[I] = (void*)&trap<I>), ...);
}

void install() {
  fill_traps(std::make_integer_sequence<int, 234>{});
  g_env_table[6] = (void*)&FindClass;
  g_env_table[14] = (void*)&ThrowNew;
  g_env_table[16] = (void*)&ExceptionDescribe;
  g_env_table[17] = (void*)&ExceptionClear;
  g_env_table[21] = (void*)&NewGlobalRef;
  g_env_table[22] = (void*)&DeleteGlobalRef;
  g_env_table[23] = (void*)&DeleteLocalRef;
  g_env_table[31] = (void*)&GetObjectClass;
  g_env_table[94] = (void*)&GetFieldID;
  g_env_table[95] = (void*)&GetObjectField;
  g_env_table[101] = (void*)&GetLongField;
  g_env_table[113] = (void*)&GetStaticMethodID;
  g_env_table[116] = (void*)&call_object;
  g_env_table[143] = (void*)&call_void;
  g_env_table[167] = (void*)&NewStringUTF;
  g_env_table[169] = (void*)&GetStringUTFChars;
  g_env_table[170] = (void*)&ReleaseStringUTFChars;
  g_env_table[171] = (void*)&GetArrayLength;
  g_env_table[173] = (void*)&GetObjectArrayElement;
  g_env_table[228] = (void*)&ExceptionCheck;
  g_env_table[229] = (void*)&NewDirectByteBuffer;
  for (auto& s : g_vm_table) s = nullptr;
  g_vm_table[5] = (void*)&Detach;
  g_vm_table[6] = (void*)&GetEnv;
  g_vm_table[7] = (void*)&AttachDaemon;
}

Obj* string_array(const std::vector<std::string>& v) {
  Obj* a = new Obj{kArray};
  for (auto& s : v) a->items.push_back(new Obj{kString, s});
  return a;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: fake_jvm <libuda.so> <manifest>\n");
    return 2;
  }
  install();
  t_attached = true;  // this is the "Java main thread"
  std::vector<std::string> prov_args, cons_args, cmds, bad_cmds;
  int log_level = 3;
  std::string exit_cmd, out_path;
  {
    std::ifstream in(argv[2]);
    std::string line;
    while (std::getline(in, line)) {
      std::istringstream ls(line);
      std::string tag;
      ls >> tag;
      std::string rest;
      std::getline(ls, rest);
      if (!rest.empty() && rest[0] == ' ') rest.erase(0, 1);
      if (tag == "parg") prov_args.push_back(rest);
      else if (tag == "carg") cons_args.push_back(rest);
      else if (tag == "cmd") cmds.push_back(rest);
      else if (tag == "bad") bad_cmds.push_back(rest);
      else if (tag == "exit") exit_cmd = rest;
      else if (tag == "out") out_path = rest;
      else if (tag == "loglevel") log_level = std::atoi(rest.c_str());
      else if (tag == "conf") {
        std::istringstream cs(rest);
        std::string k, v;
        cs >> k >> v;
        J.conf[k] = v;
      } else if (tag == "mof") {  // job map reduce start raw part path
        std::istringstream ms(rest);
        std::string job, map, path;
        int reduce;
        int64_t s, r, p;
        ms >> job >> map >> reduce >> s >> r >> p >> path;
        const std::string key = job + "|" + map + "|" + std::to_string(reduce);
        J.mofs[key] = {s, r, p};
        J.mof_path[key] = path;
      }
    }
  }
  void* lib = dlopen(argv[1], RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    fprintf(stderr, "dlopen: %s\n", dlerror());
    return 3;
  }
  using OnLoad = jint (*)(Table*, void*);
  using Start = jint (*)(Table*, void*, jboolean, Obj*, jint, jboolean);
  using DoCmd = void (*)(Table*, void*, Obj*);
  using Exit = void (*)(Table*, void*);
  using SetLog = void (*)(Table*, void*, jint);
  using OnUnload = void (*)(Table*, void*);
  auto on_load = (OnLoad)dlsym(lib, "JNI_OnLoad");
  auto start = (Start)dlsym(lib, "Java_com_mellanox_hadoop_mapred_UdaBridge_startNative");
  auto do_cmd = (DoCmd)dlsym(lib, "Java_com_mellanox_hadoop_mapred_UdaBridge_doCommandNative");
  auto reduce_exit = (Exit)dlsym(lib, "Java_com_mellanox_hadoop_mapred_UdaBridge_reduceExitMsgNative");
  auto set_log = (SetLog)dlsym(lib, "Java_com_mellanox_hadoop_mapred_UdaBridge_setLogLevelNative");
  auto on_unload = (OnUnload)dlsym(lib, "JNI_OnUnload");
  if (!on_load || !start || !do_cmd || !reduce_exit || !set_log || !on_unload) {
    fprintf(stderr, "missing JNI symbol\n");
    return 4;
  }
  Table* env = &g_env;
  const jint ver = on_load(&g_vm, nullptr);
  set_log(env, &J.bridge_cls, log_level);
  int exceptions = 0, unexpected_exceptions = 0;
  std::string first_exception;
  jint rc = start(env, &J.bridge_cls, 0, string_array(prov_args), log_level, 0);
  if (!t_exception.empty()) unexpected_exceptions++, first_exception = t_exception, t_exception.clear();
  rc |= start(env, &J.bridge_cls, 1, string_array(cons_args), log_level, 0);
  if (!t_exception.empty()) unexpected_exceptions++, first_exception = t_exception, t_exception.clear();
  for (auto& b : bad_cmds) {
    do_cmd(env, &J.bridge_cls, new Obj{kString, b});
    if (t_exception.rfind("com/mellanox/hadoop/mapred/UdaRuntimeException", 0) == 0) exceptions++;
    t_exception.clear();
  }
  for (auto& c : cmds) {
    do_cmd(env, &J.bridge_cls, new Obj{kString, c});
    if (!t_exception.empty()) {
      unexpected_exceptions++;
      if (first_exception.empty()) first_exception = t_exception;
      t_exception.clear();
    }
  }
  bool finished;
  {
    std::unique_lock<std::mutex> lk(J.mu);
    finished = J.cv.wait_for(lk, std::chrono::seconds(60), [] { return J.eof || J.failures > 0; });
  }
  reduce_exit(env, &J.bridge_cls);
  if (!t_exception.empty()) unexpected_exceptions++, t_exception.clear();
  if (!exit_cmd.empty()) do_cmd(env, &J.bridge_cls, new Obj{kString, exit_cmd});
  if (!t_exception.empty()) unexpected_exceptions++, t_exception.clear();
  on_unload(&g_vm, nullptr);
  {
    std::ofstream o(out_path, std::ios::binary);
    o.write(J.out.data(), (std::streamsize)J.out.size());
  }
  printf("{\"onload_version\":%d,\"start_rc\":%d,\"finished\":%s,\"fetch_over\":%d,\"buffers\":%d,\"bytes\":%zu,"
         "\"failures\":%d,\"logs\":%d,\"bad_cmd_exceptions\":%d,\"unexpected_exceptions\":%d,\"attaches\":%d,"
         "\"detaches\":%d,\"unattached_calls\":%d,\"non_direct\":%d,\"bad_slot\":%d,\"live_local_refs\":%ld,"
         "\"hosted\":%d,\"first_exception\":\"%s\"}\n",
         ver, rc, finished ? "true" : "false", J.fetch_over.load(), J.buffers.load(), J.out.size(), J.failures.load(),
         J.logs.load(), exceptions, unexpected_exceptions, J.attaches.load(), J.detaches.load(),
         J.unattached_calls.load(), J.non_direct.load(), J.bad_slot.load(), J.live_local.load(), J.hosted.load(),
         first_exception.c_str());
  fflush(stdout);
  // libuda's worker threads are joined by reduce exit / EXIT; leave the library loaded (as a JVM does)
  return 0;
}
