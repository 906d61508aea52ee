/*
 * Public door to Hadoop's package-private IndexCache (the file.out.index cache the vanilla shuffle
 * server uses, with its owner check); reference IndexCacheBridge.java:28-38.
 */
package org.apache.hadoop.mapred;

import java.io.IOException;

import org.apache.hadoop.fs.Path;

public class IndexCacheBridge extends IndexCache {
  public IndexCacheBridge(JobConf conf) {
    super(conf);
  }

  /** Index record of (mapId, reduce) from `indexFile`, tagged with the MOF data path. */
  public IndexRecordBridge lookup(String mapId, int reduce, Path indexFile, String expectedOwner, Path dataFile)
      throws IOException {
    IndexRecord r = getIndexInformation(mapId, reduce, indexFile, expectedOwner);
    return IndexRecordBridge.of(r, dataFile.toString());
  }
}
