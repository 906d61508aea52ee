/*
 * Java -> native command strings "<n>:<id>:p1:...:p(n-1)", n counting the id itself.
 * Ids and format must match csrc/include/uda/cmd.h (CmdId, form_cmd); reference
 * plugins/shared/com/mellanox/hadoop/mapred/UdaPlugin.java:562-587.
 */
package com.mellanox.hadoop.mapred;

import java.util.List;

final class UdaCmd {
  static final int EXIT_COMMAND = 0;
  static final int NEW_MAP_COMMAND = 1;
  static final int FINAL_MERGE_COMMAND = 2;
  static final int RESULT_COMMAND = 3;
  static final int FETCH_COMMAND = 4;
  static final int FETCH_OVER_COMMAND = 5;
  static final int JOB_OVER_COMMAND = 6;
  static final int INIT_COMMAND = 7;
  static final int MORE_COMMAND = 8;
  static final int NETLEV_REDUCE_LAUNCHED = 9;

  private UdaCmd() {}

  static String formCmd(int id, List<String> params) {
    StringBuilder sb = new StringBuilder(64);
    sb.append(params.size() + 1).append(':').append(id);
    for (String p : params) sb.append(':').append(p);  // a null param is sent as "null"
    return sb.toString();
  }
}
