#!/bin/bash
# Build the Hadoop plugin jar against an installed Hadoop (needs a JDK and `hadoop classpath`).
#   java/build.sh yarn      -> build/java/uda-amd-hadoop-yarn.jar   (Hadoop 2.x / 3.x)
#   java/build.sh hadoop-1  -> build/java/uda-amd-hadoop-1.jar      (Hadoop 1.x + plugin patch)
#   java/build.sh hadoop-1-old -> Hadoop 1.x with the abstract-class ShuffleConsumerPlugin patch
#   java/build.sh yarn-2.0  -> Hadoop 2.0.x-alpha (AuxServices.AuxiliaryService provider API)
# Deploy the jar next to libuda.so (UdaBridge loads libuda.so from the jar's directory, or from
# -Duda.library.path=<dir>).
set -euo pipefail
flavor="${1:-yarn}"
here="$(cd "$(dirname "$0")" && pwd)"
root="$(dirname "$here")"
out="$root/build/java/$flavor"
cp_="${HADOOP_CLASSPATH_OVERRIDE:-$(hadoop classpath)}"
rm -rf "$out" && mkdir -p "$out/classes"
# a flavour's own classes replace the same-named ones of the flavour it builds on
case "$flavor" in
  hadoop-1-old) dirs="$here/hadoop-1-old $here/hadoop-1" ;;
  yarn-2.0) dirs="$here/yarn-2.0 $here/yarn" ;;
  *) dirs="$here/$flavor" ;;
esac
: > "$out/sources.txt"
for f in $(cd "$here/shared" && find . -name '*.java'); do echo "$here/shared/$f" >> "$out/sources.txt"; done
seen=""
for d in $dirs; do
  for f in $(cd "$d" && find . -name '*.java'); do
    case " $seen " in *" $f "*) continue ;; esac
    seen="$seen $f"
    echo "$d/$f" >> "$out/sources.txt"
  done
done
javac -source 8 -target 8 -nowarn -cp "$cp_" -d "$out/classes" @"$out/sources.txt"
jar cf "$root/build/java/uda-amd-hadoop-$flavor.jar" -C "$out/classes" .
cp "$root/uda_amd/lib/libuda.so" "$root/build/java/"
echo "built $root/build/java/uda-amd-hadoop-$flavor.jar (+ libuda.so)"
