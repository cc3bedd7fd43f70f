#!/bin/bash
# Build an alternative libmapa.so with one source file swapped: tools/ab_build.sh <name> <file.hip> <replaces>
# Output: build_ab/<name>/libmapa.so (load with MAPA_LIB_PATH=...; for A/B timing in one GPU session).
set -e
name=$1; src=$2; rep=$3
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/build_ab/$name
rm -rf $d && mkdir -p $d/csrc && cp $root/map-anything_amd/csrc/*.hip $root/map-anything_amd/csrc/*.h $root/map-anything_amd/csrc/*.cpp $root/map-anything_amd/csrc/Makefile $d/csrc/
cp $src $d/csrc/$rep
mkdir -p $d/include && cp $root/include/mapa.h $d/include/
# Makefile includes ../../include/mapa.h relative to csrc: mirror that layout
mkdir -p $d/x && mv $d/csrc $d/x/csrc && mkdir -p $d/include
make -s -C $d/x/csrc -j8 OUT=$d/libmapa.so HIPCC=/opt/rocm/bin/hipcc >/dev/null 2>&1 || make -C $d/x/csrc OUT=$d/libmapa.so
echo $d/libmapa.so
