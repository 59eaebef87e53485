#!/bin/bash
# Experiment library: the product objects with one unit recompiled under extra flags.
# usage: tools/build_variant.sh NAME UNIT.hip [hipcc flags...]  -> fluidframework_amd/build/libmtreplay_NAME.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/fluidframework_amd/build
NAME=$1; UNIT=$2; shift 2
D=$B/obj-libmtreplay_$NAME
rm -rf "$D"; mkdir -p "$D"
cp $B/obj-libmtreplay/*.o "$D/"
U=$(basename "$UNIT" .hip)
# the unit's product flags (fluidframework_amd/native.py unit_flags), then the experiment's
UF=$(cd "$ROOT" && python3 -c "from fluidframework_amd import native; print(' '.join(native.unit_flags('$U.hip')))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $UF "$@" -c -o "$D/$U.o" "$ROOT/fluidframework_amd/${CSRC:-csrc}/$U.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o "$B/libmtreplay_$NAME.so" "$D"/*.o
echo "$B/libmtreplay_$NAME.so"
