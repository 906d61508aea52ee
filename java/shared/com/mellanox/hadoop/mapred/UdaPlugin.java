/*
 * Common launcher of the native side for both roles (reference UdaPlugin.java:60-144).
 *
 * - builds the native CLI (-w -r -a -m -g -t -s, parsed by csrc/common/cmd.cc parse_options);
 * - derives the native log threshold from the commons-logging levels that are enabled
 *   (1 = fatal only ... 6 = trace), and, for the long-lived provider, re-syncs it every second;
 * - starts the native side through UdaBridge.
 */
package com.mellanox.hadoop.mapred;

import java.util.ArrayList;
import java.util.List;
import java.util.Timer;
import java.util.TimerTask;

import org.apache.commons.logging.Log;
import org.apache.hadoop.mapred.JobConf;

abstract class UdaPlugin {
  protected final JobConf jobConf;
  protected final Log log;
  private volatile int nativeLevel;
  private Timer levelTimer;

  UdaPlugin(JobConf jobConf, Log log) {
    this.jobConf = jobConf;
    this.log = log;
    this.nativeLevel = levelOf(log);
  }

  /** Native CLI arguments for this role. */
  protected abstract List<String> cliArgs();

  /** Number of enabled log levels == native severity threshold (uda/log.h). */
  static int levelOf(Log l) {
    int n = 0;
    if (l.isFatalEnabled()) n++;
    if (l.isErrorEnabled()) n++;
    if (l.isWarnEnabled()) n++;
    if (l.isInfoEnabled()) n++;
    if (l.isDebugEnabled()) n++;
    if (l.isTraceEnabled()) n++;
    return n;
  }

  /** Options shared by both roles; `logDir` is where per-role native log files go (-g). */
  static List<String> commonArgs(JobConf conf, String logDir) {
    List<String> a = new ArrayList<String>();
    a.add("-w");
    a.add(conf.get("mapred.rdma.wqe.per.conn", "256"));
    a.add("-r");
    a.add(conf.get("mapred.rdma.cma.port", "9011"));
    a.add("-m");
    a.add("1");  // INTEGRATED (inside Hadoop)
    if (logDir != null && !logDir.isEmpty()) {
      a.add("-g");
      a.add(logDir);
    }
    a.add("-s");
    a.add(conf.get("mapred.rdma.buf.size", "1024"));  // KB
    return a;
  }

  static String defaultLogDir() {
    String d = System.getProperty("yarn.app.container.log.dir");
    if (d == null) d = System.getProperty("hadoop.log.dir");
    return d == null ? "" : d;
  }

  protected void launch(boolean netMerger, UdaCallable callable, UdaBridge.ConfSource confSource) {
    List<String> args = cliArgs();
    boolean ownFiles = jobConf.getBoolean("mapred.uda.log.to.unique.file", false);
    try {
      UdaBridge.start(netMerger, args.toArray(new String[0]), log, nativeLevel, ownFiles, callable, confSource);
    } catch (UnsatisfiedLinkError e) {
      log.warn("UDA: cannot load libuda.so (java.library.path=" + System.getProperty("java.library.path") + ")", e);
      throw e;
    }
    if (!netMerger) startLevelSync();
  }

  private void startLevelSync() {
    levelTimer = new Timer("uda-log-level", true);
    levelTimer.schedule(new TimerTask() {
      @Override
      public void run() {
        int now = levelOf(log);
        if (now != nativeLevel) {
          nativeLevel = now;
          UdaBridge.setLogLevel(now);
          log.info("UDA: native log level changed to " + now);
        }
      }
    }, 1000, 1000);
  }

  protected void stopLevelSync() {
    if (levelTimer != null) levelTimer.cancel();
  }
}
