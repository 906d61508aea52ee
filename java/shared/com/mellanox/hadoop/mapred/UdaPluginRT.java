/*
 * Reduce-task side of the plugin: starts the native NetMerger, sends INIT and FETCH, receives the
 * merged stream (reference UdaPluginRT, UdaPlugin.java:146-556).
 *
 * INIT parameters, in order (parsed by csrc/common/cmd.cc parse_init_params):
 *   numMaps, jobId, reduceTaskId, lpqSize, maxBufBytes, minBufBytes, keyClass, codec|null,
 *   compBlockSize, shuffleMemBytes, numDirs, dir_1..dir_n
 * FETCH parameters: host, jobId, mapAttemptId, reducePartition.
 *
 * Shuffle memory: mapred.rdma.shuffle.total.size if > 0, else Xmx x
 * mapred.job.shuffle.input.buffer.percent (0.7). With the GPU backend
 * (mapred.uda.merge.backend=gpu) the partitions are staged in HBM and this only sizes the host-side
 * fetch buffers.
 */
package com.mellanox.hadoop.mapred;

import java.io.File;
import java.io.IOException;
import java.util.ArrayList;
import java.util.List;

import org.apache.commons.logging.Log;
import org.apache.commons.logging.LogFactory;
import org.apache.hadoop.mapred.JobConf;
import org.apache.hadoop.mapred.RawKeyValueIterator;
import org.apache.hadoop.mapred.Reporter;
import org.apache.hadoop.util.Progress;
import org.apache.hadoop.util.StringUtils;

class UdaPluginRT extends UdaPlugin implements UdaCallable {
  static final Log LOG = LogFactory.getLog("org.apache.hadoop.mapred.ShuffleConsumerPlugin");
  static final int PROGRESS_REPORT_LIMIT = 20;  // MOFs per fetchOverMessage (MergeManager.cc:44)
  static final int KV_BUF_SIZE = 1 << 20;       // dataFromUda buffer (NETLEV_KV_POOL_EXPO)
  static final int KV_BUF_NUM = 2;
  private static final float DEFAULT_SHUFFLE_INPUT_PERCENT = 0.7f;

  private final UdaShuffleConsumerPluginShared owner;
  private final Reporter reporter;
  private final int partition;
  private final int numMaps;
  private final KVBufferRing ring;
  private final Progress progress = new Progress();
  private volatile int mapsReported;

  UdaPluginRT(UdaShuffleConsumerPluginShared owner, JobConf conf, Reporter reporter, String jobId,
              String reduceAttemptId, int partition, int numMaps) throws IOException {
    super(conf, LOG);
    this.owner = owner;
    this.reporter = reporter;
    this.partition = partition;
    this.numMaps = numMaps;
    int kvBuf = conf.getInt("mapred.uda.kv.buf.size", KV_BUF_SIZE);
    this.ring = new KVBufferRing(KV_BUF_NUM, kvBuf);

    long maxBufKb = conf.getLong("mapred.rdma.buf.size", 1024);
    long minBufKb = conf.getLong("mapred.rdma.buf.size.min", 16);
    long shuffleMem = shuffleMemory(conf);
    LOG.info("UDA: numMaps=" + numMaps + " rdma.buf.size=" + maxBufKb + "KB min=" + minBufKb
        + "KB shuffle memory=" + (shuffleMem >> 20) + "MB backend=" + conf.get("mapred.uda.merge.backend", "cpu"));

    launch(true, this, new UdaBridge.ConfSource() {
      @Override
      public String get(String key, String dflt) {
        return jobConf.get(key, dflt);
      }
    });

    List<String> p = new ArrayList<String>();
    p.add(Integer.toString(numMaps));
    p.add(jobId);
    p.add(reduceAttemptId);
    p.add(conf.get("mapred.netmerger.hybrid.lpq.size", "0"));
    p.add(Long.toString(maxBufKb * 1024));
    p.add(Long.toString(minBufKb * 1024));
    p.add(conf.getMapOutputKeyClass().getName());
    String codec = conf.getCompressMapOutput() ? conf.get("mapred.map.output.compression.codec", null) : null;
    p.add(codec == null ? "null" : codec);
    p.add(Integer.toString(codecBlockSize(conf, codec)));
    p.add(Long.toString(shuffleMem));
    List<String> dirs = usableLocalDirs(conf);
    p.add(Integer.toString(dirs.size()));
    p.addAll(dirs);
    LOG.info("UDA: sending INIT " + p);
    UdaBridge.doCommand(UdaCmd.formCmd(UdaCmd.INIT_COMMAND, p));
    progress.set(0.5f);
  }

  @Override
  protected List<String> cliArgs() {
    List<String> a = commonArgs(jobConf, defaultLogDir());
    a.add("-a");
    a.add(jobConf.get("mapred.netmerger.merge.approach", "1"));
    return a;
  }

  static long shuffleMemory(JobConf conf) {
    long total = StringUtils.TraditionalBinaryPrefix.string2long(conf.get("mapred.rdma.shuffle.total.size", "0"));
    if (total > 0) return total;
    float pct = conf.getFloat("mapred.job.shuffle.input.buffer.percent", DEFAULT_SHUFFLE_INPUT_PERCENT);
    if (pct < 0 || pct > 1) pct = DEFAULT_SHUFFLE_INPUT_PERCENT;
    return (long) (Runtime.getRuntime().maxMemory() * pct);
  }

  static int codecBlockSize(JobConf conf, String codec) {
    int dflt = 256 * 1024;
    if (codec == null) return dflt;
    if (codec.contains("Lzo")) return conf.getInt("io.compression.codec.lzo.buffersize", dflt);
    if (codec.contains("Snappy")) return conf.getInt("io.compression.codec.snappy.buffersize", dflt);
    return dflt;
  }

  /** Local dirs that exist or can be created (LPQ spill files go there). */
  static List<String> usableLocalDirs(JobConf conf) throws IOException {
    List<String> out = new ArrayList<String>();
    String[] dirs = conf.getLocalDirs();
    if (dirs == null) return out;
    for (String d : dirs) {
      File f = new File(d.trim());
      if ((f.isDirectory() || f.mkdirs()) && f.canWrite()) out.add(f.getPath());
    }
    return out;
  }

  void sendFetchReq(String host, String jobId, String mapAttemptId) {
    List<String> p = new ArrayList<String>(4);
    p.add(host);
    p.add(jobId);
    p.add(mapAttemptId);
    p.add(Integer.toString(partition));
    UdaBridge.doCommand(UdaCmd.formCmd(UdaCmd.FETCH_COMMAND, p));
  }

  RawKeyValueIterator createKVIterator() {
    return new MergedKVIterator(ring, reporter, progress);
  }

  void close() {
    try {
      UdaBridge.reduceExitMsg();
    } finally {
      ring.close();
    }
  }

  // ------------------------------------------------------------------ UdaCallable (native threads)
  @Override
  public void fetchOverMessage() {
    int n = Math.min(numMaps, mapsReported + PROGRESS_REPORT_LIMIT);
    mapsReported = n;
    if (reporter != null) reporter.progress();
    if (n >= numMaps) owner.notifyFetchCompleted();
  }

  @Override
  public void dataFromUda(Object directBuffer, int len) throws Throwable {
    ring.put(directBuffer, len);
  }

  @Override
  public void failureInUda() {
    owner.failureInUda(new UdaRuntimeException("UDA failure in a native thread"));
  }
}
