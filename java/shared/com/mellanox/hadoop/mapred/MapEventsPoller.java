/*
 * Polls the map-completion events of the job and turns every newly succeeded map into a FETCH
 * (reference GetMapEventsThread, UdaShuffleConsumerPluginShared.java:434-602). Rules kept:
 *  - poll every second, at most 10000 events per call;
 *  - the first SUCCEEDED attempt of a map is fetched, later attempts of the same map are ignored;
 *  - FAILED / KILLED / OBSOLETE for an attempt already sent to the native side cannot be undone
 *    there -> the reducer falls back to the vanilla shuffle;
 *  - a reset of the event stream is harmless before any success and a fallback after one.
 * Unlike the reference, the succeeded sets live for the whole task, not for one poll.
 */
package com.mellanox.hadoop.mapred;

import java.net.URI;
import java.util.HashSet;
import java.util.Set;

import org.apache.commons.logging.Log;
import org.apache.hadoop.mapred.MapTaskCompletionEventsUpdate;
import org.apache.hadoop.mapred.TaskAttemptID;
import org.apache.hadoop.mapred.TaskCompletionEvent;
import org.apache.hadoop.mapred.TaskID;

final class MapEventsPoller extends Thread {
  static final long POLL_MS = 1000;
  static final int MAX_EVENTS = 10000;

  private final UdaShuffleConsumerPluginShared owner;
  private final UdaConsumerPluginCallable version;
  private final UdaPluginRT rt;
  private final Log log;
  private final Set<TaskID> succeededTasks = new HashSet<TaskID>();
  private final Set<TaskAttemptID> succeededAttempts = new HashSet<TaskAttemptID>();
  private int fromEventId;
  private volatile boolean stop;

  MapEventsPoller(UdaShuffleConsumerPluginShared owner, UdaConsumerPluginCallable version, UdaPluginRT rt, Log log) {
    this.owner = owner;
    this.version = version;
    this.rt = rt;
    this.log = log;
    setName("uda-map-events");
    setDaemon(true);
  }

  void shutdown() {
    stop = true;
    interrupt();
  }

  @Override
  public void run() {
    try {
      while (!stop) {
        int n = pollOnce();
        if (n > 0 && log.isDebugEnabled()) log.debug("UDA: " + n + " new map outputs");
        Thread.sleep(POLL_MS);
      }
    } catch (InterruptedException e) {
      // shutdown
    } catch (Throwable t) {
      if (!stop) {
        log.error("UDA: map events poller failed", t);
        owner.failureInUda(t);
      }
    }
  }

  int pollOnce() throws Exception {
    MapTaskCompletionEventsUpdate u = version.mapCompletionEvents(fromEventId, MAX_EVENTS);
    if (u.shouldReset()) {
      if (!succeededTasks.isEmpty())
        throw new UdaRuntimeException("map events reset after " + succeededTasks.size() + " maps were fetched");
      log.info("UDA: map events reset before any map succeeded");
      fromEventId = 0;
    }
    TaskCompletionEvent[] events = u.getMapTaskCompletionEvents();
    fromEventId += events.length;
    int fresh = 0;
    for (TaskCompletionEvent ev : events) {
      TaskAttemptID attempt = ev.getTaskAttemptId();
      switch (ev.getTaskStatus()) {
        case SUCCEEDED:
          if (succeededTasks.add(attempt.getTaskID())) {
            succeededAttempts.add(attempt);
            String host = URI.create(ev.getTaskTrackerHttp()).getHost();
            rt.sendFetchReq(host, attempt.getJobID().toString(), attempt.toString());
            fresh++;
          } else {
            log.info("UDA: ignoring another successful attempt " + attempt);
          }
          break;
        case FAILED:
        case KILLED:
        case OBSOLETE:
          if (succeededAttempts.contains(attempt))
            throw new UdaRuntimeException("map attempt " + attempt + " became " + ev.getTaskStatus() + " after it was fetched");
          log.info("UDA: ignoring " + ev.getTaskStatus() + " attempt " + attempt);
          break;
        default:  // TIPFAILED: the job does not need this map's output
          log.info("UDA: ignoring output of failed map TIP " + attempt);
          break;
      }
    }
    return fresh;
  }
}
