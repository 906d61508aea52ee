/*
 * What the version-independent consumer core needs from a Hadoop line (reference
 * UdaShuffleConsumerPluginShared.java:93-100). The vanilla plugin is passed as Object because its
 * interface differs between Hadoop 1 (fetchOutputs + createKVIterator) and Hadoop 2/3 (run()).
 */
package com.mellanox.hadoop.mapred;

import java.io.IOException;

import org.apache.hadoop.fs.FileSystem;
import org.apache.hadoop.mapred.JobConf;
import org.apache.hadoop.mapred.MapTaskCompletionEventsUpdate;
import org.apache.hadoop.mapred.RawKeyValueIterator;
import org.apache.hadoop.mapred.Reporter;

interface UdaConsumerPluginCallable {
  /** The vanilla shuffle of this Hadoop line, initialized for the current reduce task. */
  Object createVanillaPlugin() throws IOException, ClassNotFoundException;

  /** Hadoop 1: vanilla.fetchOutputs(); Hadoop 2/3: nothing to do before run(). */
  boolean vanillaFetchOutputs(Object vanilla) throws IOException;

  RawKeyValueIterator vanillaIterator(Object vanilla, JobConf job, FileSystem fs, Reporter reporter)
      throws IOException, InterruptedException;

  void closeVanilla(Object vanilla);

  /** umbilical.getMapCompletionEvents for this reduce task. */
  MapTaskCompletionEventsUpdate mapCompletionEvents(int fromEventId, int maxEvents) throws IOException;
}
