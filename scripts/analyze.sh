#!/bin/bash
# Clang static analyzer over the native core (path-sensitive checks: null/uninitialised
# use, leaks, dead stores, libc argument constraints).  Prints findings; exit 1 if any.
set -u
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CXX=/opt/rocm/lib/llvm/bin/clang++
PYINC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PB=$(python3 -c "import pybind11; print(pybind11.get_include())")
out=$(cd /tmp && for f in "$ROOT"/native/*.cpp; do
  "$CXX" --analyze -std=c++17 -I"$ROOT/native" -I/opt/rocm/include -I"$PYINC" -I"$PB" \
    -Xanalyzer -analyzer-output=text "$f" -o /dev/null 2>&1 | grep -E "warning:"
done | sort -u)
if [ -n "$out" ]; then echo "$out"; exit 1; fi
echo "clang static analyzer: no findings in native/*.cpp"
