/*
 * Hand-off of merged buffers from the native merge thread (dataFromUda) to the reducer thread
 * (MergedKVIterator). Parity: the two KVBuf objects and their recv/redc states of the reference
 * (UdaPlugin.java:164-179, 369-402, 421-433, 456-484); here two blocking queues of slots replace the
 * per-buffer monitors, and close() wakes both sides instead of leaving a native thread parked.
 */
package com.mellanox.hadoop.mapred;

import java.nio.ByteBuffer;
import java.util.concurrent.ArrayBlockingQueue;
import java.util.concurrent.BlockingQueue;
import java.util.concurrent.TimeUnit;

final class KVBufferRing {
  /** One delivery buffer: whole IFile records, the last one of the stream ends with (-1,-1). */
  static final class Slot {
    final byte[] data;
    int len;

    Slot(int capacity) {
      data = new byte[capacity];
    }
  }

  private static final Slot CLOSED = new Slot(0);
  private final BlockingQueue<Slot> free;
  private final BlockingQueue<Slot> full;
  private volatile boolean closed;

  KVBufferRing(int slots, int capacity) {
    free = new ArrayBlockingQueue<Slot>(slots);
    full = new ArrayBlockingQueue<Slot>(slots + 1);
    for (int i = 0; i < slots; i++) free.add(new Slot(capacity));
  }

  /** Native thread: copy `len` bytes of a direct buffer into the next free slot (blocks). */
  void put(Object directBuffer, int len) throws InterruptedException {
    Slot s = null;
    while (s == null) {
      if (closed) throw new UdaRuntimeException("reducer closed the merged-data queue");
      s = free.poll(100, TimeUnit.MILLISECONDS);
    }
    if (len > s.data.length) throw new UdaRuntimeException("merged buffer of " + len + " bytes exceeds " + s.data.length);
    ByteBuffer bb = ((ByteBuffer) directBuffer).duplicate();
    bb.position(0);
    bb.get(s.data, 0, len);
    s.len = len;
    full.put(s);
  }

  /** Reducer thread: the next filled slot, or null once closed. */
  Slot take() throws InterruptedException {
    Slot s = full.take();
    return s == CLOSED ? null : s;
  }

  /** Reducer thread: the slot's records have been consumed. */
  void release(Slot s) {
    s.len = 0;
    free.offer(s);
  }

  void close() {
    closed = true;
    full.offer(CLOSED);
  }
}
