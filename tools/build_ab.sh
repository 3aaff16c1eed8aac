#!/bin/bash
# Build a standalone gfx950 shared object of one kernel source variant for A/B timing:
#   tools/build_ab.sh <name> <kernel.hip> [kcommon.h]  ->  tools/ab/<name>.so
set -e
name=$1; src=$2; kc=$3
root=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d /tmp/ab_${name}_XXXX)
mkdir -p "$d/kernels" "$root/tools/ab"
cp -r "$root/csrc/common" "$d/"
cp "$root"/csrc/kernels/*.h "$d/kernels/"
[ -n "$kc" ] && cp "$kc" "$d/kernels/kcommon.h"
cp "$src" "$d/kernels/$(basename "$src" | sed 's/_v[0-9a-z]*\.hip$/.hip/')"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I"$d" -o "$root/tools/ab/$name.so" "$d"/kernels/*.hip
rm -rf "$d"
