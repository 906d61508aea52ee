/*
 * Version-independent consumer core (reference UdaShuffleConsumerPluginShared.java:115-432).
 *
 * Contract kept from the reference:
 *  - any Throwable in init / fetch / iterator creation, and any native failure (failureInUda),
 *    switches this reduce task to the vanilla Hadoop shuffle, once;
 *  - with mapred.rdma.developer.mode=true a failure aborts the task JVM instead (System.exit(1));
 *  - log lines the regression tools look for: "init - Using UdaShuffleConsumerPlugin" and
 *    "====XXX Successfully closed UdaShuffleConsumerPlugin XXX====" (tools/regression.py).
 */
package com.mellanox.hadoop.mapred;

import java.io.IOException;

import org.apache.commons.logging.Log;
import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.mapred.JobConf;
import org.apache.hadoop.mapred.RawKeyValueIterator;
import org.apache.hadoop.mapred.ReduceTask;
import org.apache.hadoop.mapred.Reporter;

class UdaShuffleConsumerPluginShared {
  static final Log LOG = UdaPluginRT.LOG;
  static final String DEV_MODE_KEY = "mapred.rdma.developer.mode";

  private final UdaConsumerPluginCallable version;
  ReduceTask reduceTask;
  JobConf jobConf;
  Reporter reporter;
  FileSystem fs;

  private UdaPluginRT rt;
  private volatile Object vanilla;  // non-null once fallen back
  private final Object fetchLock = new Object();
  private boolean fetchSignalled;
  private boolean udaFetchDone;
  private boolean vanillaFetchDone;

  UdaShuffleConsumerPluginShared(UdaConsumerPluginCallable version) {
    this.version = version;
  }

  void init(ReduceTask reduceTask, JobConf conf, Reporter reporter, FileSystem fs) throws IOException {
    this.reduceTask = reduceTask;
    this.jobConf = conf;
    this.reporter = reporter;
    this.fs = fs;
    try {
      LOG.info("init - Using UdaShuffleConsumerPlugin");
      rt = new UdaPluginRT(this, conf, reporter, reduceTask.getJobID().toString(), reduceTask.getTaskID().toString(),
          reduceTask.getPartition(), reduceTask.getNumMaps());
    } catch (Throwable t) {
      fallback(t);
    }
  }

  // ------------------------------------------------------------------ failure -> vanilla
  synchronized void fallback(Throwable cause) throws IOException {
    if (vanilla != null) return;
    if (jobConf != null && jobConf.getBoolean(DEV_MODE_KEY, false)) {
      LOG.fatal("UDA failed and " + DEV_MODE_KEY + " is set: aborting instead of falling back", cause);
      System.exit(1);
    }
    if (cause != null) LOG.error("UDA failed; falling back to the vanilla shuffle", cause);
    try {
      vanilla = version.createVanillaPlugin();
    } catch (ClassNotFoundException e) {
      throw new UdaRuntimeException("UDA failed and the vanilla shuffle class cannot be loaded", e);
    }
    LOG.info("UDA: switched to the vanilla shuffle");
  }

  /** Native thread or the events poller: fall back, then wake fetchOutputs. */
  void failureInUda(Throwable cause) {
    try {
      fallback(cause);
    } catch (IOException e) {
      throw new UdaRuntimeException("UDA failed and the fallback to vanilla failed too", e);
    } finally {
      notifyFetchCompleted();
    }
  }

  void notifyFetchCompleted() {
    synchronized (fetchLock) {
      fetchSignalled = true;
      fetchLock.notifyAll();
    }
  }

  // ------------------------------------------------------------------ ShuffleConsumerPlugin flow
  boolean fetchOutputs() throws IOException {
    if (vanilla == null) {
      try {
        return fetchWithUda();
      } catch (Throwable t) {
        fallback(t);
      }
    }
    return fetchWithVanilla();
  }

  private boolean fetchWithUda() throws Exception {
    MapEventsPoller poller = new MapEventsPoller(this, version, rt, LOG);
    poller.start();
    try {
      synchronized (fetchLock) {
        while (!fetchSignalled) fetchLock.wait();
      }
    } finally {
      poller.shutdown();
      poller.join(5000);
    }
    if (vanilla != null) throw new UdaRuntimeException("UDA failure reported while fetching");
    udaFetchDone = true;
    return true;
  }

  private synchronized boolean fetchWithVanilla() throws IOException {
    if (!vanillaFetchDone) {
      fallback(null);
      vanillaFetchDone = version.vanillaFetchOutputs(vanilla);
    }
    return vanillaFetchDone;
  }

  RawKeyValueIterator createKVIterator(JobConf job, FileSystem fs, Reporter reporter) throws IOException {
    if (vanilla == null && udaFetchDone) {
      try {
        LOG.info("createKVIterator - Using UdaShuffleConsumerPlugin");
        return rt.createKVIterator();
      } catch (Throwable t) {
        fallback(t);
      }
    }
    if (!fetchWithVanilla()) throw new IOException("Task " + reduceTask.getTaskID() + ": the vanilla reduce copier failed");
    try {
      return version.vanillaIterator(vanilla, job, fs, reporter);
    } catch (InterruptedException e) {
      Thread.currentThread().interrupt();
      throw new IOException(e);
    }
  }

  void close() {
    if (vanilla == null) {
      rt.close();
      LOG.info("====XXX Successfully closed UdaShuffleConsumerPlugin XXX====");
      return;
    }
    version.closeVanilla(vanilla);
    if (rt != null) {  // stop the native side without holding up the task for long
      final UdaPluginRT r = rt;
      Thread closer = new Thread("uda-closer") {
        @Override
        public void run() {
          r.close();
        }
      };
      closer.setDaemon(true);
      closer.start();
      try {
        closer.join(1000);
      } catch (InterruptedException e) {
        Thread.currentThread().interrupt();
      }
    }
    LOG.info("====XXX Successfully closed fallbackPlugin XXX====");
  }
}
