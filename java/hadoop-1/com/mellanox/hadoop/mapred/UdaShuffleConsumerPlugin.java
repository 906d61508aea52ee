/*
 * Hadoop 1.x (patched with the ShuffleConsumerPlugin API, reference plugins/HADOOP-1.x.y-v2.patch)
 * reduce-side plugin; reference plugins/mlx-1.x/.../UdaShuffleConsumerPlugin.java. CDH renamed
 * Context.getConf -> getJobConf and dropped createKVIterator's arguments: both are looked up by
 * reflection.
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

public class UdaShuffleConsumerPlugin implements ShuffleConsumerPlugin, UdaConsumerPluginCallable {
  private final UdaShuffleConsumerPluginShared core = new UdaShuffleConsumerPluginShared(this);
  private TaskUmbilicalProtocol umbilical;

  @Override
  public void init(ShuffleConsumerPlugin.Context ctx) throws IOException {
    Object conf = Utils.invokeFunctionReflection(ShuffleConsumerPlugin.Context.class, "getConf", new Class<?>[0], ctx,
        new Object[0]);
    if (conf == null)  // CDH
      conf = Utils.invokeFunctionReflection(ShuffleConsumerPlugin.Context.class, "getJobConf", new Class<?>[0], ctx,
          new Object[0]);
    if (conf == null) throw new UdaRuntimeException("ShuffleConsumerPlugin.Context has neither getConf nor getJobConf");
    umbilical = ctx.getUmbilical();
    JobConf jc = (JobConf) conf;
    core.init(ctx.getReduceTask(), jc, ctx.getReporter(), FileSystem.getLocal(jc).getRaw());
  }

  @Override
  public boolean fetchOutputs() throws IOException {
    return core.fetchOutputs();
  }

  public RawKeyValueIterator createKVIterator(JobConf job, FileSystem fs, Reporter reporter) throws IOException {
    return core.createKVIterator(job, fs, reporter);
  }

  public RawKeyValueIterator createKVIterator() throws IOException {  // CDH signature
    return core.createKVIterator(core.jobConf, core.fs, core.reporter);
  }

  @Override
  public Throwable getMergeThrowable() {
    return null;
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
  public RawKeyValueIterator vanillaIterator(Object vanilla, JobConf job, FileSystem fs, Reporter reporter) {
    Object it = Utils.invokeFunctionReflection(ShuffleConsumerPlugin.class, "createKVIterator",
        new Class<?>[] {JobConf.class, FileSystem.class, Reporter.class}, vanilla, new Object[] {job, fs, reporter});
    if (it == null)
      it = Utils.invokeFunctionReflection(ShuffleConsumerPlugin.class, "createKVIterator", new Class<?>[0], vanilla,
          new Object[0]);
    if (it == null) throw new UdaRuntimeException("no createKVIterator on the vanilla ShuffleConsumerPlugin");
    return (RawKeyValueIterator) it;
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
