/*
 * Hadoop 2.x / 3.x provider: a NodeManager auxiliary service (yarn.nodemanager.aux-services =
 * uda_shuffle, yarn.nodemanager.aux-services.uda_shuffle.class =
 * com.mellanox.hadoop.mapred.UdaShuffleHandler) hosting the native MOFSupplier (reference
 * plugins/mlx-2.x|mlx-3.x UdaShuffleHandler.java + UdaPluginSH.java).
 *
 * getPathUda resolves a map output the way the vanilla ShuffleHandler does:
 *   <nm-local-dir>/usercache/<user>/appcache/<application id>/output/<map attempt>/file.out[.index]
 * with the application's user recorded in initializeApplication, and the index record read through
 * Hadoop's IndexCache (owner-checked, cached).
 */
package com.mellanox.hadoop.mapred;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.Collections;
import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;

import org.apache.commons.logging.Log;
import org.apache.commons.logging.LogFactory;
import org.apache.hadoop.conf.Configuration;
import org.apache.hadoop.fs.LocalDirAllocator;
import org.apache.hadoop.fs.Path;
import org.apache.hadoop.mapred.IndexCacheBridge;
import org.apache.hadoop.mapred.IndexRecordBridge;
import org.apache.hadoop.mapred.JobConf;
import org.apache.hadoop.mapred.JobID;
import org.apache.hadoop.yarn.api.records.ApplicationId;
import org.apache.hadoop.yarn.conf.YarnConfiguration;
import org.apache.hadoop.yarn.server.api.ApplicationInitializationContext;
import org.apache.hadoop.yarn.server.api.ApplicationTerminationContext;
import org.apache.hadoop.yarn.server.api.AuxiliaryService;

public class UdaShuffleHandler extends AuxiliaryService implements UdaBridge.IndexResolver {
  public static final String SERVICE_ID = "uda_shuffle";
  private static final Log LOG = LogFactory.getLog(UdaShuffleHandler.class.getCanonicalName());

  private final Map<String, String> jobUser = new ConcurrentHashMap<String, String>();
  private final LocalDirAllocator nmDirs = new LocalDirAllocator(YarnConfiguration.NM_LOCAL_DIRS);
  private JobConf conf;
  private IndexCacheBridge indexCache;
  private UdaShuffleProviderPluginShared supplier;

  public UdaShuffleHandler() {
    super(SERVICE_ID);
  }

  @Override
  protected void serviceInit(Configuration c) throws Exception {
    conf = new JobConf(c);
    super.serviceInit(new Configuration(c));
  }

  @Override
  protected void serviceStart() throws Exception {
    indexCache = new IndexCacheBridge(conf);
    supplier = new UdaShuffleProviderPluginShared(conf, this);
    LOG.info("UDA MOFSupplier started");
    super.serviceStart();
  }

  @Override
  protected void serviceStop() throws Exception {
    if (supplier != null) supplier.close();
    supplier = null;
    super.serviceStop();
  }

  private static String jobOf(ApplicationId app) {
    return new JobID(Long.toString(app.getClusterTimestamp()), app.getId()).toString();
  }

  @Override
  public void initializeApplication(ApplicationInitializationContext ctx) {
    jobUser.put(jobOf(ctx.getApplicationId()), ctx.getUser());
  }

  @Override
  public void stopApplication(ApplicationTerminationContext ctx) {
    String job = jobOf(ctx.getApplicationId());
    jobUser.remove(job);
    if (supplier != null) {  // the native provider may free the job's MOFs held in its HBM store
      UdaBridge.doCommand(UdaCmd.formCmd(UdaCmd.JOB_OVER_COMMAND, Collections.singletonList(job)));
    }
  }

  @Override
  public ByteBuffer getMetaData() {
    return ByteBuffer.allocate(0);  // never null (YARN-1256)
  }

  @Override
  public IndexRecordBridge resolve(String jobId, String mapId, int reduceId) {
    String user = jobUser.get(jobId);
    if (user == null) {
      LOG.error("UDA: getPathUda for unknown job " + jobId);
      return null;
    }
    JobID job = JobID.forName(jobId);
    ApplicationId app = ApplicationId.newInstance(Long.parseLong(job.getJtIdentifier()), job.getId());
    String base = "usercache/" + user + "/appcache/" + app + "/output/" + mapId;
    try {
      Path index = nmDirs.getLocalPathToRead(base + "/file.out.index", conf);
      Path data = nmDirs.getLocalPathToRead(base + "/file.out", conf);
      return indexCache.lookup(mapId, reduceId, index, user, data);
    } catch (IOException e) {
      LOG.error("UDA: cannot resolve " + jobId + "/" + mapId + "/" + reduceId, e);
      return null;
    }
  }
}
