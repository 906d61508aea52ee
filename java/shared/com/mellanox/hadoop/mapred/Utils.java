/*
 * Reflection helpers for Hadoop distributions whose plugin signatures differ (vanilla vs CDH);
 * reference Utils.java. A missing method/constructor yields null; a failing call throws.
 */
package com.mellanox.hadoop.mapred;

import java.lang.reflect.Constructor;
import java.lang.reflect.InvocationTargetException;
import java.lang.reflect.Method;

public final class Utils {
  private Utils() {}

  /** Invoke `name(argTypes)` declared on `cls` on `target`; null if no such method. */
  public static Object invokeFunctionReflection(Class<?> cls, String name, Class<?>[] argTypes, Object target,
                                                Object[] args) {
    Method m;
    try {
      m = cls.getDeclaredMethod(name, argTypes);
    } catch (NoSuchMethodException e) {
      return null;
    }
    try {
      m.setAccessible(true);
      return m.invoke(target, args);
    } catch (IllegalAccessException e) {
      throw new UdaRuntimeException("cannot call " + cls.getName() + "." + name, e);
    } catch (InvocationTargetException e) {
      throw new UdaRuntimeException(cls.getName() + "." + name + " failed", e.getCause());
    }
  }

  /** New instance through the public constructor `argTypes`; null if there is none. */
  public static Object invokeConstructorReflection(Class<?> cls, Class<?>[] argTypes, Object[] args) {
    Constructor<?> c;
    try {
      c = cls.getConstructor(argTypes);
    } catch (NoSuchMethodException e) {
      return null;
    }
    return newInstance(c, args);
  }

  /** New instance of a (possibly non-static inner) class through its one-argument constructor. */
  public static Object invokeCtorWithArg(Class<?> cls, Class<?> argType, Object arg) {
    Constructor<?> c;
    try {
      c = cls.getDeclaredConstructor(argType);
    } catch (NoSuchMethodException e) {
      return null;
    }
    c.setAccessible(true);
    return newInstance(c, new Object[] {arg});
  }

  private static Object newInstance(Constructor<?> c, Object[] args) {
    try {
      return c.newInstance(args);
    } catch (InvocationTargetException e) {
      throw new UdaRuntimeException("constructor of " + c.getDeclaringClass().getName() + " failed", e.getCause());
    } catch (ReflectiveOperationException e) {
      throw new UdaRuntimeException("cannot construct " + c.getDeclaringClass().getName(), e);
    }
  }
}
