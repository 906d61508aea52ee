/*
 * RawKeyValueIterator over the merged stream the native side delivers (reference J2CQueue,
 * UdaPlugin.java:435-555). Each buffer holds whole records `VInt keyLen, VInt valLen, key, value`;
 * the stream ends with VInt(-1) VInt(-1). A buffer is handed back to the native side when the
 * iterator moves past its last record, so the key/value views stay valid until the next next().
 * The Python twin used by the tests is uda_amd/utils/ifile.py J2CQueueReader.
 */
package com.mellanox.hadoop.mapred;

import java.io.IOException;

import org.apache.hadoop.io.DataInputBuffer;
import org.apache.hadoop.io.WritableUtils;
import org.apache.hadoop.mapred.RawKeyValueIterator;
import org.apache.hadoop.mapred.Reporter;
import org.apache.hadoop.util.Progress;

final class MergedKVIterator implements RawKeyValueIterator {
  private static final int PROGRESS_EVERY = 1000;  // records between reporter.progress() calls

  private final KVBufferRing ring;
  private final Reporter reporter;
  private final Progress progress;
  private final DataInputBuffer cur = new DataInputBuffer();
  private final DataInputBuffer key = new DataInputBuffer();
  private final DataInputBuffer value = new DataInputBuffer();
  private KVBufferRing.Slot slot;
  private boolean eof;
  private int sinceProgress;

  MergedKVIterator(KVBufferRing ring, Reporter reporter, Progress progress) {
    this.ring = ring;
    this.reporter = reporter;
    this.progress = progress;
  }

  @Override
  public DataInputBuffer getKey() {
    return key;
  }

  @Override
  public DataInputBuffer getValue() {
    return value;
  }

  @Override
  public boolean next() throws IOException {
    if (eof) return false;
    while (slot == null || cur.getPosition() >= slot.len) {
      if (slot != null) ring.release(slot);
      try {
        slot = ring.take();
      } catch (InterruptedException e) {
        Thread.currentThread().interrupt();
        throw new IOException("interrupted while waiting for merged data", e);
      }
      if (slot == null) {  // closed before EOF
        eof = true;
        return false;
      }
      cur.reset(slot.data, 0, slot.len);
    }
    int kl = WritableUtils.readVInt(cur);
    int vl = WritableUtils.readVInt(cur);
    if (kl < 0 || vl < 0) {
      eof = true;
      ring.release(slot);
      slot = null;
      return false;
    }
    int pos = cur.getPosition();
    if (pos + kl + vl > slot.len) throw new IOException("record split across merged buffers");
    key.reset(slot.data, pos, kl);
    value.reset(slot.data, pos + kl, vl);
    cur.skip(kl + vl);
    if (++sinceProgress >= PROGRESS_EVERY) {
      sinceProgress = 0;
      if (reporter != null) reporter.progress();
    }
    return true;
  }

  @Override
  public void close() {
    ring.close();
  }

  @Override
  public Progress getProgress() {
    return progress;
  }
}
