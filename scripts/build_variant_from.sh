#!/bin/bash
# Build the product sources of git revision REV into
# delta-compression_amd/lib/libdeltagpu_NAME.so (an A/B baseline selected with
# DG_LIB_VARIANT=NAME; never loaded by default).
# usage: [NOAB=1] scripts/build_variant_from.sh REV|WT NAME [extra hipcc flags]
# (NOAB=1: the product's flags, no A/B switches, for a like-for-like A/B)
set -e
REV=$1; NAME=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
AB=-DDG_AB_SWITCHES
[ -n "$NOAB" ] && AB=
if [ "$REV" = WT ]; then   # the working tree
  mkdir -p "$T/delta-compression_amd" && cp -r "$ROOT/delta-compression_amd/csrc" "$T/delta-compression_amd/" && cp -r "$ROOT/include" "$T/"
else
  git -C "$ROOT" archive "$REV" delta-compression_amd/csrc include | tar -x -C "$T"
fi
mkdir -p "$T/o" "$ROOT/delta-compression_amd/lib"
for f in "$T"/delta-compression_amd/csrc/*.hip "$T"/delta-compression_amd/csrc/*.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w $AB "$@" -x hip -c "$f" -o "$T/o/$(basename "$f").o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/delta-compression_amd/lib/libdeltagpu_$NAME.so" "$T"/o/*.o
rm -rf "$T"
echo "built lib/libdeltagpu_$NAME.so from $REV"
