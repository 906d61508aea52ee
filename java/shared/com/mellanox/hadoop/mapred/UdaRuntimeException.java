/*
 * Raised by the JNI shim when a native entry point fails (csrc/bridge/jni_shim.cc throw_uda) and by
 * the plugin on unrecoverable shuffle errors; reference UdaRuntimeException.java.
 */
package com.mellanox.hadoop.mapred;

public class UdaRuntimeException extends RuntimeException {
  private static final long serialVersionUID = 0x0da0a3d1L;

  public UdaRuntimeException(String message) {
    super(message);
  }

  public UdaRuntimeException(String message, Throwable cause) {
    super(message, cause);
  }
}
