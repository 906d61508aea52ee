/*
 * JNI surface of libuda.so (uda_amd). Parity: reference
 * plugins/shared/com/mellanox/hadoop/mapred/UdaBridge.java:36-147 — the same class name, the same
 * four natives and the same six static callbacks, because csrc/bridge/jni_shim.cc resolves them by
 * name and JNI descriptor in JNI_OnLoad:
 *
 *   natives    startNative(Z[Ljava/lang/String;IZ)I   doCommandNative(Ljava/lang/String;)V
 *              reduceExitMsgNative()V                  setLogLevelNative(I)V
 *   callbacks  fetchOverMessage()V                     dataFromUda(Ljava/lang/Object;I)V
 *              getPathUda(Ljava/lang/String;Ljava/lang/String;I)Ljava/lang/Object;
 *              getConfData(Ljava/lang/String;Ljava/lang/String;)Ljava/lang/String;
 *              logToJava(Ljava/lang/String;I)V         failureInUda()V
 *
 * Design differences from the reference:
 *  - the library location can be overridden with -Duda.library.path=/dir (default: the directory of
 *    the jar, like the reference), so the same jar runs against an in-tree build;
 *  - the provider-side index resolver and the consumer-side configuration are registered
 *    explicitly (registerProvider / start) instead of being hard-wired to one per-version class;
 *  - a callback that arrives after the consumer closed is dropped instead of dereferencing null.
 */
package com.mellanox.hadoop.mapred;

import java.io.File;

import org.apache.commons.logging.Log;
import org.apache.commons.logging.LogFactory;
import org.apache.hadoop.mapred.IndexRecordBridge;

public final class UdaBridge {

  /** Provider-side resolver of (job, map attempt, reduce) to a MOF partition. */
  interface IndexResolver {
    IndexRecordBridge resolve(String jobId, String mapId, int reduceId);
  }

  /** Configuration source for getConfData (the reducer's JobConf, or the NodeManager conf). */
  interface ConfSource {
    String get(String key, String dflt);
  }

  private static volatile Log log = LogFactory.getLog(UdaBridge.class.getCanonicalName());
  private static volatile UdaCallable consumer;
  private static volatile IndexResolver resolver;
  private static volatile ConfSource conf;

  static {
    String dir = System.getProperty("uda.library.path");
    if (dir == null || dir.isEmpty()) {
      String jar = UdaBridge.class.getProtectionDomain().getCodeSource().getLocation().getPath();
      dir = new File(jar).getParent();
    }
    Runtime.getRuntime().load(new File(dir, "libuda.so").getAbsolutePath());
  }

  private UdaBridge() {}

  // ------------------------------------------------------------------ natives (jni_shim.cc)
  private static native int startNative(boolean isNetMerger, String[] args, int logLevel, boolean logToUdaFile);

  private static native void doCommandNative(String cmd);

  private static native void reduceExitMsgNative();

  private static native void setLogLevelNative(int level);

  // ------------------------------------------------------------------ Java-side entry points
  static void registerProvider(IndexResolver r, ConfSource c) {
    resolver = r;
    conf = c;
  }

  /**
   * Start the native side. For the NetMerger `callable` receives the data and progress callbacks;
   * for the MOFSupplier it is null and the index resolver registered with registerProvider is used.
   */
  static int start(boolean isNetMerger, String[] args, Log sink, int logLevel, boolean logToUdaFile,
                   UdaCallable callable, ConfSource confSource) {
    if (sink != null) log = sink;
    if (isNetMerger) {
      consumer = callable;
      conf = confSource;
    } else if (confSource != null) {
      conf = confSource;
    }
    log.info("UDA: starting native " + (isNetMerger ? "NetMerger" : "MOFSupplier") + " argv=" + String.join(" ", args));
    int rc = startNative(isNetMerger, args, logLevel, logToUdaFile);
    log.info("UDA: native start returned " + rc);
    return rc;
  }

  public static void doCommand(String cmd) {
    if (log.isDebugEnabled()) log.debug("UDA: doCommand " + cmd);
    doCommandNative(cmd);
  }

  public static void reduceExitMsg() {
    try {
      reduceExitMsgNative();
    } finally {
      consumer = null;
    }
  }

  public static void setLogLevel(int level) {
    setLogLevelNative(level);
  }

  // ------------------------------------------------------------------ callbacks from native threads
  public static void fetchOverMessage() throws Throwable {
    UdaCallable c = consumer;
    if (c != null) c.fetchOverMessage();
  }

  public static void dataFromUda(Object directBuffer, int len) throws Throwable {
    UdaCallable c = consumer;
    if (c == null) throw new UdaRuntimeException("dataFromUda after the consumer closed");
    c.dataFromUda(directBuffer, len);
  }

  public static Object getPathUda(String jobId, String mapId, int reduceId) {
    IndexResolver r = resolver;
    if (r == null) {
      log.error("UDA: getPathUda with no provider registered");
      return null;
    }
    return r.resolve(jobId, mapId, reduceId);
  }

  public static String getConfData(String key, String dflt) {
    ConfSource c = conf;
    return c == null ? dflt : c.get(key, dflt);
  }

  /** Native severities 1=fatal .. 6=trace (uda/log.h). */
  public static void logToJava(String msg, int severity) {
    final Log l = log;
    switch (severity) {
      case 1: l.fatal(msg); break;
      case 2: l.error(msg); break;
      case 3: l.warn(msg); break;
      case 5: l.debug(msg); break;
      case 6: l.trace(msg); break;
      default: l.info(msg); break;
    }
  }

  public static void failureInUda() {
    UdaCallable c = consumer;
    if (c != null) c.failureInUda();
    else log.error("UDA: native failure reported with no active consumer");
  }
}
