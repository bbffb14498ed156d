#!/bin/sh
# Boundary parity of tests/golden/cdc.json against an ALREADY INSTALLED rabinwindow-1.0.2.jar
# (INTEGRATION.md §4).  Needs javac/java on PATH.  Usage: jar_parity.sh <rabinwindow.jar> [--emit] [--sdfs]
set -e
JAR="$1"; shift || true
[ -f "$JAR" ] || { echo "usage: $0 /path/to/rabinwindow-1.0.2.jar [--emit] [--sdfs]" >&2; exit 2; }
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$(mktemp -d)
javac -cp "$JAR" -d "$OUT" "$ROOT/tools/java/JarParity.java"
EXTRA=""
for a in "$@"; do
  case "$a" in
    --emit) EXTRA="$EXTRA --emit $ROOT/tests/golden/jar_cdc.json" ;;
    --sdfs) EXTRA="$EXTRA --sdfs" ;;
  esac
done
java -cp "$JAR:$OUT:${SDFS_CLASSPATH:-}" JarParity "$ROOT/tests/golden/cdc.json" $EXTRA
