#!/bin/bash
# Build a tuning variant of libyk.so: tools/variant.sh NAME "-DKNOB=value ..."
# -> tune/libyk_NAME.so (load it with YK_LIB=$PWD/tune/libyk_NAME.so).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tune"
make -s -j8 -C "$ROOT/core_amd" OUT="$ROOT/tune/libyk_$1.so" BUILD="/tmp/ykbuild_$1" EXTRA="$2"
