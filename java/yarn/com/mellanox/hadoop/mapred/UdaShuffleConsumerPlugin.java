/*
 * Hadoop 2.x / 3.x reduce-side plugin: mapreduce.job.reduce.shuffle.consumer.plugin.class =
 * com.mellanox.hadoop.mapred.UdaShuffleConsumerPlugin (reference plugins/mlx-2.x and mlx-3.x
 * UdaShuffleConsumerPlugin.java). The vanilla fallback is Hadoop's own
 * org.apache.hadoop.mapreduce.task.reduce.Shuffle, initialized with this task's context.
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
import org.apache.hadoop.mapred.UdaMapredBridge;

public class UdaShuffleConsumerPlugin<K, V> implements ShuffleConsumerPlugin<K, V>, UdaConsumerPluginCallable {
  private final UdaShuffleConsumerPluginShared core = new UdaShuffleConsumerPluginShared(this);
  private ShuffleConsumerPlugin.Context<K, V> context;

  @Override
  public void init(ShuffleConsumerPlugin.Context<K, V> ctx) {
    this.context = ctx;
    try {
      core.init((ReduceTask) ctx.getReduceTask(), ctx.getJobConf(), ctx.getReporter(), ctx.getLocalFS());
    } catch (IOException e) {
      UdaShuffleConsumerPluginShared.LOG.error("UDA: plugin init failed", e);
    }
  }

  @Override
  public RawKeyValueIterator run() throws IOException, InterruptedException {
    if (!core.fetchOutputs()) throw new IOException("UDA: fetching the map outputs failed");
    return core.createKVIterator(core.jobConf, core.fs, core.reporter);
  }

  @Override
  public void close() {
    core.close();
  }

  // ------------------------------------------------------------------ UdaConsumerPluginCallable
  @Override
  public Object createVanillaPlugin() throws IOException, ClassNotFoundException {
    return UdaMapredBridge.vanillaShuffle(context);
  }

  @Override
  public boolean vanillaFetchOutputs(Object vanilla) {
    return true;  // the vanilla Shuffle fetches inside run()
  }

  @Override
  @SuppressWarnings("unchecked")
  public RawKeyValueIterator vanillaIterator(Object vanilla, JobConf job, FileSystem fs, Reporter reporter)
      throws IOException, InterruptedException {
    return ((ShuffleConsumerPlugin<K, V>) vanilla).run();
  }

  @Override
  public void closeVanilla(Object vanilla) {
    ((ShuffleConsumerPlugin<?, ?>) vanilla).close();
  }

  @Override
  public MapTaskCompletionEventsUpdate mapCompletionEvents(int fromEventId, int maxEvents) throws IOException {
    ReduceTask rt = core.reduceTask;
    return context.getUmbilical().getMapCompletionEvents(rt.getJobID(), fromEventId, maxEvents, rt.getTaskID());
  }
}
