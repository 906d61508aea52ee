// The slice of the JNI binary interface libuda.so needs, declared in-tree (this image has no JDK).
//
// The JNI ABI is fixed by the Java Native Interface specification: a JNIEnv* points at a pointer to
// the function table, whose slots have stable indices across JDK releases (new functions are only
// appended); the invocation interface (JavaVM) works the same way. Only the slots the shim calls are
// named here, and only the non-varargs 'A' call forms are used, so the shim never depends on a
// C varargs calling convention. Indices: JNI spec, chapter 4 "JNI Functions" (interface function
// table) and chapter 5 "The Invocation API".
#pragma once
#include <cstdint>

namespace uda {
namespace jni {

using jint = int32_t;
using jlong = int64_t;
using jboolean = uint8_t;
using jsize = jint;
struct _jobject;
using jobject = _jobject*;
using jclass = jobject;
using jstring = jobject;
using jthrowable = jobject;
using jobjectArray = jobject;
struct _jmethodID;
using jmethodID = _jmethodID*;
struct _jfieldID;
using jfieldID = _jfieldID*;
union jvalue {
  jboolean z;
  int8_t b;
  uint16_t c;
  int16_t s;
  jint i;
  jlong j;
  float f;
  double d;
  jobject l;
};

constexpr jint JNI_OK = 0;
constexpr jint JNI_EDETACHED = -2;
constexpr jint JNI_VERSION_1_4 = 0x00010004;

// JNIEnv / JavaVM as the C binding declares them: pointer to a table of function pointers.
using JNIEnv = void* const*;
using JavaVM = void* const*;

enum EnvSlot : int {
  kFindClass = 6,
  kThrowNew = 14,
  kExceptionDescribe = 16,
  kExceptionClear = 17,
  kNewGlobalRef = 21,
  kDeleteGlobalRef = 22,
  kDeleteLocalRef = 23,
  kGetObjectClass = 31,
  kGetFieldID = 94,
  kGetObjectField = 95,
  kGetLongField = 101,
  kGetStaticMethodID = 113,
  kCallStaticObjectMethodA = 116,
  kCallStaticVoidMethodA = 143,
  kNewStringUTF = 167,
  kGetStringUTFChars = 169,
  kReleaseStringUTFChars = 170,
  kGetArrayLength = 171,
  kGetObjectArrayElement = 173,
  kExceptionCheck = 228,
  kNewDirectByteBuffer = 229,
  kEnvSlots = 234,
};

enum VmSlot : int {
  kDetachCurrentThread = 5,
  kGetEnv = 6,
  kAttachCurrentThreadAsDaemon = 7,
  kVmSlots = 8,
};

template <typename F>
inline F env_fn(JNIEnv* env, int slot) {
  return reinterpret_cast<F>((*env)[slot]);
}
template <typename F>
inline F vm_fn(JavaVM* vm, int slot) {
  return reinterpret_cast<F>((*vm)[slot]);
}

// Typed wrappers (JNICALL is the platform C convention on x86-64 Linux).
inline jclass FindClass(JNIEnv* e, const char* name) {
  return env_fn<jclass (*)(JNIEnv*, const char*)>(e, kFindClass)(e, name);
}
inline jint ThrowNew(JNIEnv* e, jclass c, const char* msg) {
  return env_fn<jint (*)(JNIEnv*, jclass, const char*)>(e, kThrowNew)(e, c, msg);
}
inline void ExceptionDescribe(JNIEnv* e) { env_fn<void (*)(JNIEnv*)>(e, kExceptionDescribe)(e); }
inline void ExceptionClear(JNIEnv* e) { env_fn<void (*)(JNIEnv*)>(e, kExceptionClear)(e); }
inline jboolean ExceptionCheck(JNIEnv* e) { return env_fn<jboolean (*)(JNIEnv*)>(e, kExceptionCheck)(e); }
inline jobject NewGlobalRef(JNIEnv* e, jobject o) {
  return env_fn<jobject (*)(JNIEnv*, jobject)>(e, kNewGlobalRef)(e, o);
}
inline void DeleteGlobalRef(JNIEnv* e, jobject o) { env_fn<void (*)(JNIEnv*, jobject)>(e, kDeleteGlobalRef)(e, o); }
inline void DeleteLocalRef(JNIEnv* e, jobject o) {
  if (o) env_fn<void (*)(JNIEnv*, jobject)>(e, kDeleteLocalRef)(e, o);
}
inline jclass GetObjectClass(JNIEnv* e, jobject o) {
  return env_fn<jclass (*)(JNIEnv*, jobject)>(e, kGetObjectClass)(e, o);
}
inline jfieldID GetFieldID(JNIEnv* e, jclass c, const char* n, const char* sig) {
  return env_fn<jfieldID (*)(JNIEnv*, jclass, const char*, const char*)>(e, kGetFieldID)(e, c, n, sig);
}
inline jobject GetObjectField(JNIEnv* e, jobject o, jfieldID f) {
  return env_fn<jobject (*)(JNIEnv*, jobject, jfieldID)>(e, kGetObjectField)(e, o, f);
}
inline jlong GetLongField(JNIEnv* e, jobject o, jfieldID f) {
  return env_fn<jlong (*)(JNIEnv*, jobject, jfieldID)>(e, kGetLongField)(e, o, f);
}
inline jmethodID GetStaticMethodID(JNIEnv* e, jclass c, const char* n, const char* sig) {
  return env_fn<jmethodID (*)(JNIEnv*, jclass, const char*, const char*)>(e, kGetStaticMethodID)(e, c, n, sig);
}
inline jobject CallStaticObjectMethodA(JNIEnv* e, jclass c, jmethodID m, const jvalue* a) {
  return env_fn<jobject (*)(JNIEnv*, jclass, jmethodID, const jvalue*)>(e, kCallStaticObjectMethodA)(e, c, m, a);
}
inline void CallStaticVoidMethodA(JNIEnv* e, jclass c, jmethodID m, const jvalue* a) {
  env_fn<void (*)(JNIEnv*, jclass, jmethodID, const jvalue*)>(e, kCallStaticVoidMethodA)(e, c, m, a);
}
inline jstring NewStringUTF(JNIEnv* e, const char* s) {
  return env_fn<jstring (*)(JNIEnv*, const char*)>(e, kNewStringUTF)(e, s);
}
inline const char* GetStringUTFChars(JNIEnv* e, jstring s) {
  return env_fn<const char* (*)(JNIEnv*, jstring, jboolean*)>(e, kGetStringUTFChars)(e, s, nullptr);
}
inline void ReleaseStringUTFChars(JNIEnv* e, jstring s, const char* c) {
  env_fn<void (*)(JNIEnv*, jstring, const char*)>(e, kReleaseStringUTFChars)(e, s, c);
}
inline jsize GetArrayLength(JNIEnv* e, jobjectArray a) {
  return env_fn<jsize (*)(JNIEnv*, jobjectArray)>(e, kGetArrayLength)(e, a);
}
inline jobject GetObjectArrayElement(JNIEnv* e, jobjectArray a, jsize i) {
  return env_fn<jobject (*)(JNIEnv*, jobjectArray, jsize)>(e, kGetObjectArrayElement)(e, a, i);
}
inline jobject NewDirectByteBuffer(JNIEnv* e, void* addr, jlong cap) {
  return env_fn<jobject (*)(JNIEnv*, void*, jlong)>(e, kNewDirectByteBuffer)(e, addr, cap);
}

inline jint GetEnv(JavaVM* vm, JNIEnv** env, jint version) {
  return vm_fn<jint (*)(JavaVM*, void**, jint)>(vm, kGetEnv)(vm, reinterpret_cast<void**>(env), version);
}
inline jint AttachCurrentThreadAsDaemon(JavaVM* vm, JNIEnv** env) {
  return vm_fn<jint (*)(JavaVM*, void**, void*)>(vm, kAttachCurrentThreadAsDaemon)(vm, reinterpret_cast<void**>(env),
                                                                                    nullptr);
}
inline jint DetachCurrentThread(JavaVM* vm) { return vm_fn<jint (*)(JavaVM*)>(vm, kDetachCurrentThread)(vm); }

}  // namespace jni
}  // namespace uda
