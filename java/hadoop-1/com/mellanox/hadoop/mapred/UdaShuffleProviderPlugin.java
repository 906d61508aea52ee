/*
 * Hadoop 1.x provider: a TaskTracker ShuffleProviderPlugin hosting the native MOFSupplier
 * (reference plugins/mlx-1.x/.../UdaShuffleProviderPlugin.java + shared UdaPluginTT1.java).
 * getPathUda resolves <local dir>/<TaskTracker.getIntermediateOutputDir(user, job, map)>/file.out[.index]
 * with small LRU caches of the resolved paths, like the TaskTracker's MapOutputServlet.
 */
package com.mellanox.hadoop.mapred;

import java.io.IOException;

import org.apache.commons.logging.Log;
import org.apache.hadoop.fs.LocalDirAllocator;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.mapred.IndexCacheBridge;
import org.apache.hadoop.mapred.IndexRecordBridge;
import org.apache.hadoop.mapred.JobConf;
import org.apache.hadoop.mapred.JobID;
import org.apache.hadoop.mapred.LRUCacheBridgeHadoop1;
import org.apache.hadoop.mapred.ShuffleProviderPlugin;
import org.apache.hadoop.mapred.TaskTracker;

public class UdaShuffleProviderPlugin implements ShuffleProviderPlugin, UdaBridge.IndexResolver {
  private static final Log LOG = UdaShuffleProviderPluginShared.LOG;
  private final LocalDirAllocator localDirs = new LocalDirAllocator("mapred.local.dir");
  private final LRUCacheBridgeHadoop1<String, Path> pathCache = new LRUCacheBridgeHadoop1<String, Path>();
  private TaskTracker tracker;
  private JobConf conf;
  private IndexCacheBridge indexCache;
  private UdaShuffleProviderPluginShared supplier;

  @Override
  public void initialize(TaskTracker tt) {
    tracker = tt;
    conf = tt.getJobConf();
    indexCache = new IndexCacheBridge(conf);
    supplier = new UdaShuffleProviderPluginShared(conf, this);
  }

  @Override
  public void destroy() {
    if (supplier != null) supplier.close();
    supplier = null;
  }

  private Path local(String rel) throws IOException {
    Path p = pathCache.get(rel);
    if (p == null) {
      p = localDirs.getLocalPathToRead(rel, conf);
      pathCache.put(rel, p);
    }
    return p;
  }

  @Override
  public IndexRecordBridge resolve(String jobId, String mapId, int reduceId) {
    try {
      JobConf jc = tracker.getJobConf(JobID.forName(jobId));
      String runAs = tracker.getTaskController().getRunAsUser(jc);
      String dir = TaskTracker.getIntermediateOutputDir(jc.getUser(), jobId, mapId);
      return indexCache.lookup(mapId, reduceId, local(dir + "/file.out.index"), runAs, local(dir + "/file.out"));
    } catch (IOException e) {
      LOG.error("UDA: cannot resolve " + jobId + "/" + mapId + "/" + reduceId, e);
      return null;
    }
  }
}
