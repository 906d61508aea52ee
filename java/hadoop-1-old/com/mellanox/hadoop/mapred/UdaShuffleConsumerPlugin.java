/*
 * Hadoop 1.x with the first form of the shuffle plugin patch, where ShuffleConsumerPlugin is an
 * abstract class whose init takes the reduce task, the umbilical, the job configuration and the
 * reporter directly (reference plugins/mlx-1.x-old). Everything else -- the provider plugin, the
 * vanilla ReduceCopier fallback (UdaMapredBridge) and the LRU path cache -- is the hadoop-1 flavour's:
 * java/build.sh hadoop-1-old compiles this directory over java/hadoop-1.
 */
package com.mellanox.hadoop.mapred;

import java.io.IOException;

import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.mapred.JobConf;
import org.apache.hadoop.mapred.MapTaskCompletionEventsUpdate;
import org.apache.hadoop.mapred.RawKeyValueIterator;
import org.apache.hadoop.mapred.ReduceTask;
import org.apache.hadoop.mapred.Reporter;
import org.apache.hadoop.mapred.ShuffleConsumerPlugin;
import org.apache.hadoop.mapred.TaskUmbilicalProtocol;
import org.apache.hadoop.mapred.UdaMapredBridge;

public class UdaShuffleConsumerPlugin extends ShuffleConsumerPlugin implements UdaConsumerPluginCallable {
  private final UdaShuffleConsumerPluginShared core = new UdaShuffleConsumerPluginShared(this);
  private TaskUmbilicalProtocol umbilical;

  @Override
  public void init(ReduceTask reduceTask, TaskUmbilicalProtocol umb, JobConf conf, Reporter reporter)
      throws IOException {
    umbilical = umb;
    core.init(reduceTask, conf, reporter, FileSystem.getLocal(conf).getRaw());
  }

  @Override
  public boolean fetchOutputs() throws IOException {
    return core.fetchOutputs();
  }

  @Override
  public RawKeyValueIterator createKVIterator(JobConf job, FileSystem fs, Reporter reporter) throws IOException {
    return core.createKVIterator(job, fs, reporter);
  }

  @Override
  public void close() {
    core.close();
  }

  // ------------------------------------------------------------------ UdaConsumerPluginCallable
  @Override
  public Object createVanillaPlugin() throws IOException, ClassNotFoundException {
    return UdaMapredBridge.vanillaCopier(core.reduceTask, umbilical, core.jobConf, core.reporter);
  }

  @Override
  public boolean vanillaFetchOutputs(Object vanilla) throws IOException {
    return ((ShuffleConsumerPlugin) vanilla).fetchOutputs();
  }

  @Override
  public RawKeyValueIterator vanillaIterator(Object vanilla, JobConf job, FileSystem fs, Reporter reporter)
      throws IOException {
    return ((ShuffleConsumerPlugin) vanilla).createKVIterator(job, fs, reporter);
  }

  @Override
  public void closeVanilla(Object vanilla) {
    ((ShuffleConsumerPlugin) vanilla).close();
  }

  @Override
  public MapTaskCompletionEventsUpdate mapCompletionEvents(int fromEventId, int maxEvents) throws IOException {
    ReduceTask rt = core.reduceTask;
    return umbilical.getMapCompletionEvents(rt.getJobID(), fromEventId, maxEvents, rt.getTaskID(), rt.getJvmContext());
  }
}
