/*
 * Creates the vanilla Hadoop 2/3 shuffle for the fallback path (reference plugins/mlx-2.x
 * org/apache/hadoop/mapred/UdaMapredBridge.java). In this package for access to the task types.
 */
package org.apache.hadoop.mapred;

import java.io.IOException;

import org.apache.hadoop.mapreduce.task.reduce.Shuffle;
import org.apache.hadoop.util.ReflectionUtils;

public final class UdaMapredBridge {
  private UdaMapredBridge() {}

  @SuppressWarnings({"unchecked", "rawtypes"})
  public static <K, V> ShuffleConsumerPlugin<K, V> vanillaShuffle(ShuffleConsumerPlugin.Context<K, V> context)
      throws IOException {
    if (context == null) throw new IOException("UDA fallback: no shuffle context (init was never called)");
    ShuffleConsumerPlugin<K, V> plugin = ReflectionUtils.newInstance(Shuffle.class, context.getJobConf());
    plugin.init(context);
    return plugin;
  }
}
