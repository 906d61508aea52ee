/*
 * Provider (MOFSupplier) runtime shared by the TaskTracker (Hadoop 1) and NodeManager aux-service
 * (Hadoop 2/3) front ends (reference UdaShuffleProviderPluginShared.java + UdaPluginTT/UdaPluginSH).
 * It starts the native MOFSupplier, answers getPathUda through a version-specific resolver, and
 * sends EXIT on close.
 */
package com.mellanox.hadoop.mapred;

import java.util.ArrayList;
import java.util.List;

import org.apache.commons.logging.Log;
import org.apache.commons.logging.LogFactory;
import org.apache.hadoop.mapred.JobConf;

class UdaShuffleProviderPluginShared extends UdaPlugin {
  static final Log LOG = LogFactory.getLog("org.apache.hadoop.mapred.ShuffleProviderPlugin");

  UdaShuffleProviderPluginShared(final JobConf conf, UdaBridge.IndexResolver resolver) {
    super(conf, LOG);
    UdaBridge.ConfSource src = new UdaBridge.ConfSource() {
      @Override
      public String get(String key, String dflt) {
        return conf.get(key, dflt);
      }
    };
    UdaBridge.registerProvider(resolver, src);
    launch(false, null, src);
  }

  @Override
  protected List<String> cliArgs() {
    String dir = System.getProperty("hadoop.log.dir");
    return commonArgs(jobConf, dir == null ? defaultLogDir() : dir);
  }

  void close() {
    stopLevelSync();
    LOG.info("UDA: sending EXIT to the MOFSupplier");
    UdaBridge.doCommand(UdaCmd.formCmd(UdaCmd.EXIT_COMMAND, new ArrayList<String>()));
  }
}
