#!/bin/bash
# Build an alternative libmapa.so with one source file swapped: tools/ab_build.sh <name> <file.hip> <replaces>
# Output: ab_libs/<name>/libmapa.so (bench.py --lib / kbench.py MAPA_AB_LIB=...; A/B timing in one GPU session; ab_libs/ is git-ignored and travels to the box only while it exists — delete it after the A/B).
set -e
name=$1; src=$2; rep=$3
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/ab_libs/$name
rm -rf $d && mkdir -p $d/csrc && cp $root/map-anything_amd/csrc/*.hip $root/map-anything_amd/csrc/*.h $root/map-anything_amd/csrc/*.cpp $root/map-anything_amd/csrc/Makefile $d/csrc/
cp $src $d/csrc/$rep
mkdir -p $d/include && cp $root/include/mapa.h $d/include/
# Makefile includes ../../include/mapa.h relative to csrc: mirror that layout
mkdir -p $d/x && mv $d/csrc $d/x/csrc && mkdir -p $d/include
make -s -C $d/x/csrc -j8 OUT=$d/libmapa.so HIPCC=/opt/rocm/bin/hipcc >/dev/null 2>&1 || make -C $d/x/csrc OUT=$d/libmapa.so
echo $d/libmapa.so
