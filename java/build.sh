#!/bin/bash
# Build the Hadoop plugin jar against an installed Hadoop (needs a JDK and `hadoop classpath`).
#   java/build.sh yarn      -> build/java/uda-amd-hadoop-yarn.jar   (Hadoop 2.x / 3.x)
#   java/build.sh hadoop-1  -> build/java/uda-amd-hadoop-1.jar      (Hadoop 1.x + plugin patch)
# Deploy the jar next to libuda.so (UdaBridge loads libuda.so from the jar's directory, or from
# -Duda.library.path=<dir>).
set -euo pipefail
flavor="${1:-yarn}"
here="$(cd "$(dirname "$0")" && pwd)"
root="$(dirname "$here")"
out="$root/build/java/$flavor"
cp_="${HADOOP_CLASSPATH_OVERRIDE:-$(hadoop classpath)}"
rm -rf "$out" && mkdir -p "$out/classes"
find "$here/shared" "$here/$flavor" -name '*.java' > "$out/sources.txt"
javac -source 8 -target 8 -nowarn -cp "$cp_" -d "$out/classes" @"$out/sources.txt"
jar cf "$root/build/java/uda-amd-hadoop-$flavor.jar" -C "$out/classes" .
cp "$root/uda_amd/lib/libuda.so" "$root/build/java/"
echo "built $root/build/java/uda-amd-hadoop-$flavor.jar (+ libuda.so)"
