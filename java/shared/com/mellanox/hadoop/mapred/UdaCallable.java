/*
 * Consumer-side receiver of the native callbacks (reference UdaBridge.java:30-34).
 */
package com.mellanox.hadoop.mapred;

interface UdaCallable {
  /** Progress: called every 20 fetched map outputs and once when fetching is complete. */
  void fetchOverMessage();

  /** One merged buffer: whole IFile records, the last buffer ends with the EOF marker (-1,-1). */
  void dataFromUda(Object directBuffer, int len) throws Throwable;

  /** A native thread failed; the consumer falls back to the vanilla shuffle. */
  void failureInUda();
}
