/*
 * Hadoop 1.x fallback: builds the vanilla ReduceTask.ReduceCopier (a non-static inner class in the
 * v2 plugin patch, static in v3) and its Context (vanilla or CDH argument order); reference
 * plugins/mlx-1.x/org/apache/hadoop/mapred/UdaMapredBridge.java.
 */
package org.apache.hadoop.mapred;

import java.io.IOException;

import org.apache.hadoop.util.ReflectionUtils;

import com.mellanox.hadoop.mapred.UdaRuntimeException;
import com.mellanox.hadoop.mapred.Utils;

public final class UdaMapredBridge {
  private UdaMapredBridge() {}

  public static ShuffleConsumerPlugin vanillaCopier(ReduceTask reduceTask, TaskUmbilicalProtocol umbilical,
                                                    JobConf conf, Reporter reporter) throws IOException {
    ShuffleConsumerPlugin copier =
        (ShuffleConsumerPlugin) Utils.invokeCtorWithArg(ReduceTask.ReduceCopier.class, ReduceTask.class, reduceTask);
    if (copier == null) copier = ReflectionUtils.newInstance(ReduceTask.ReduceCopier.class, conf);
    Task.TaskReporter tr = (Task.TaskReporter) reporter;
    Object ctx = Utils.invokeConstructorReflection(ShuffleConsumerPlugin.Context.class,
        new Class<?>[] {ReduceTask.class, TaskUmbilicalProtocol.class, JobConf.class, Task.TaskReporter.class},
        new Object[] {reduceTask, umbilical, conf, tr});
    if (ctx == null)  // CDH argument order
      ctx = Utils.invokeConstructorReflection(ShuffleConsumerPlugin.Context.class,
          new Class<?>[] {TaskUmbilicalProtocol.class, JobConf.class, Task.TaskReporter.class, ReduceTask.class},
          new Object[] {umbilical, conf, tr, reduceTask});
    if (ctx == null) throw new UdaRuntimeException("cannot build a ShuffleConsumerPlugin.Context");
    copier.init((ShuffleConsumerPlugin.Context) ctx);
    return copier;
  }
}
