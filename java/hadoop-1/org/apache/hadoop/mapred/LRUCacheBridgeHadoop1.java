/*
 * Bounded LRU map for resolved MOF paths on the Hadoop 1 TaskTracker (reference
 * LRUCacheBridgeHadoop1.java wraps the TaskTracker's own LRUCache; this one is self-contained).
 */
package org.apache.hadoop.mapred;

import java.util.LinkedHashMap;
import java.util.Map;

public class LRUCacheBridgeHadoop1<K, V> {
  private static final int DEFAULT_CAPACITY = 10000;
  private final Map<K, V> map;

  public LRUCacheBridgeHadoop1() {
    this(DEFAULT_CAPACITY);
  }

  public LRUCacheBridgeHadoop1(final int capacity) {
    map = new LinkedHashMap<K, V>(16, 0.75f, true) {
      private static final long serialVersionUID = 1L;

      @Override
      protected boolean removeEldestEntry(Map.Entry<K, V> eldest) {
        return size() > capacity;
      }
    };
  }

  public synchronized V get(K key) {
    return map.get(key);
  }

  public synchronized void put(K key, V value) {
    map.put(key, value);
  }

  public synchronized void clear() {
    map.clear();
  }
}
