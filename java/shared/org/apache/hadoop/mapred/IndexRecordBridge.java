/*
 * MOF partition descriptor returned to the native side by getPathUda. csrc/bridge/jni_shim.cc reads
 * the fields startOffset (J), rawLength (J), partLength (J) and pathMOF (Ljava/lang/String;) by name;
 * reference plugins/shared/org/apache/hadoop/mapred/IndexRecordBridge.java:26-34. It lives in this
 * package because Hadoop's IndexRecord is package-private.
 */
package org.apache.hadoop.mapred;

public class IndexRecordBridge {
  public long startOffset;
  public long rawLength;
  public long partLength;
  public String pathMOF;

  public IndexRecordBridge(long startOffset, long rawLength, long partLength, String pathMOF) {
    this.startOffset = startOffset;
    this.rawLength = rawLength;
    this.partLength = partLength;
    this.pathMOF = pathMOF;
  }

  static IndexRecordBridge of(IndexRecord r, String pathMOF) {
    return new IndexRecordBridge(r.startOffset, r.rawLength, r.partLength, pathMOF);
  }

  @Override
  public String toString() {
    return pathMOF + "@" + startOffset + "+" + partLength + " (raw " + rawLength + ")";
  }
}
