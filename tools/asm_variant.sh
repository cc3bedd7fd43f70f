#!/bin/bash
# Rebuild one translation unit of libmapa.so from an EDITED device assembly file (hazard experiments):
#   tools/asm_variant.sh <src.hip> <device.s> <out_dir> [extra hipcc flags for the host side]
# -> <out_dir>/libmapa.so = the in-tree objects with <src>.o replaced by (host part of <src>.hip + device.s).
# The host object embeds the code object as an .asciz blob; it is swapped for an .incbin of the new bundle.
set -e
src=$1; dev=$2; out=$3; shift 3
L=/opt/rocm/llvm/bin
root=$(cd "$(dirname "$0")/.." && pwd)
csrc=$root/map-anything_amd/csrc
base=$(basename $src .hip)
mkdir -p $out/tmp && cd $out/tmp
$L/clang -cc1as -triple amdgcn-amd-amdhsa -filetype obj -target-cpu gfx950 -mrelocation-model pic -o dev.o $dev
$L/lld -flavor gnu -m elf64_amdgpu --no-undefined -shared -o dev.out dev.o
$L/clang-offload-bundler -type=o -bundle-align=4096 -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950 -input=/dev/null -input=dev.out -output=dev.hipfb
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-function "$@" -save-temps -c $csrc/$src -o host_ref.o >/dev/null 2>&1
hs=$base-host-x86_64-unknown-linux-gnu.s
python3 - "$hs" <<'PY'
import re, sys
p = sys.argv[1]
s = open(p).read()
m = re.search(r'(\.section\s+\.hip_fatbin[^\n]*\n\s*\.p2align[^\n]*\n(\.L__unnamed_\d+):\n)\s*\.asciz\s+"[^\n]*\n\s*\.size\s+\2, \d+', s)
assert m, "fatbin blob not found"
s = s[:m.start()] + m.group(1) + '\t.incbin "dev.hipfb"\n' + s[m.end():]
open(p, 'w').write(s)
PY
$L/clang -cc1as -triple x86_64-unknown-linux-gnu -filetype obj -target-cpu x86-64 -mrelocation-model pic -o $base.o $hs
objs=""
for o in $csrc/*.o; do [ $(basename $o) = $base.o ] && objs="$objs $PWD/$base.o" || objs="$objs $o"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -Wl,--no-undefined $objs -o $out/libmapa.so
echo $out/libmapa.so
