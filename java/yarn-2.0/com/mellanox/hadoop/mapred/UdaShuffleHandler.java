/*
 * Hadoop 2.0.x-alpha provider: the NodeManager auxiliary service API before Hadoop 2.2 -- an
 * AbstractService implementing AuxServices.AuxiliaryService, with initApp / stopApp callbacks instead of
 * the later AuxiliaryService base class (reference plugins/mlx-2.0.x/UdaShuffleHandler.java). The map
 * output lookup is the yarn flavour's: <nm-local-dir>/usercache/<user>/appcache/<application id>/output/
 * <map attempt>/file.out[.index], the application's user recorded when the application starts, the index
 * record read through Hadoop's IndexCache. java/build.sh yarn-2.0 compiles this directory alone (with the
 * shared classes); the consumer plugin of 2.0.x is the yarn flavour's ShuffleConsumerPlugin.
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
import org.apache.hadoop.yarn.server.nodemanager.containermanager.AuxServices;
import org.apache.hadoop.yarn.service.AbstractService;
import org.apache.hadoop.yarn.util.ConverterUtils;

public class UdaShuffleHandler extends AbstractService
    implements AuxServices.AuxiliaryService, UdaBridge.IndexResolver {
  public static final String SERVICE_ID = "uda_shuffle";
  private static final Log LOG = LogFactory.getLog(UdaShuffleHandler.class.getCanonicalName());

  // job id -> (user, application id as the NodeManager names its directory)
  private final Map<String, String[]> jobs = new ConcurrentHashMap<String, String[]>();
  private final LocalDirAllocator nmDirs = new LocalDirAllocator(YarnConfiguration.NM_LOCAL_DIRS);
  private JobConf conf;
  private IndexCacheBridge indexCache;
  private UdaShuffleProviderPluginShared supplier;

  public UdaShuffleHandler() {
    super(SERVICE_ID);
  }

  @Override
  public synchronized void init(Configuration c) {
    conf = new JobConf(c);
    super.init(new Configuration(c));
  }

  @Override
  public synchronized void start() {
    indexCache = new IndexCacheBridge(conf);
    supplier = new UdaShuffleProviderPluginShared(conf, this);
    LOG.info("UDA MOFSupplier started (Hadoop 2.0.x aux service)");
    super.start();
  }

  @Override
  public synchronized void stop() {
    if (supplier != null) supplier.close();
    supplier = null;
    super.stop();
  }

  private static String jobOf(ApplicationId app) {
    return new JobID(Long.toString(app.getClusterTimestamp()), app.getId()).toString();
  }

  @Override
  public void initApp(String user, ApplicationId appId, ByteBuffer secret) {
    jobs.put(jobOf(appId), new String[] {user, ConverterUtils.toString(appId)});
  }

  @Override
  public void stopApp(ApplicationId appId) {
    String job = jobOf(appId);
    jobs.remove(job);
    if (supplier != null) {  // the native provider may free the job's MOFs held in its HBM store
      UdaBridge.doCommand(UdaCmd.formCmd(UdaCmd.JOB_OVER_COMMAND, Collections.singletonList(job)));
    }
  }

  public synchronized ByteBuffer getMeta() {
    return ByteBuffer.allocate(0);
  }

  @Override
  public IndexRecordBridge resolve(String jobId, String mapId, int reduceId) {
    String[] ua = jobs.get(jobId);
    if (ua == null) {
      LOG.error("UDA: getPathUda for unknown job " + jobId);
      return null;
    }
    String base = "usercache/" + ua[0] + "/appcache/" + ua[1] + "/output/" + mapId;
    try {
      Path index = nmDirs.getLocalPathToRead(base + "/file.out.index", conf);
      Path data = nmDirs.getLocalPathToRead(base + "/file.out", conf);
      return indexCache.lookup(mapId, reduceId, index, ua[0], data);
    } catch (IOException e) {
      LOG.error("UDA: cannot resolve " + jobId + "/" + mapId + "/" + reduceId, e);
      return null;
    }
  }
}
