#!/bin/bash
# A/B builds: yjs_amd/libymerge_<name>.so = the current objects with one kernel source replaced by another
# version (a git revision of it, or a file).  Usage: tools/build_variant.sh <name> <source.hip> <rev|file> [hipcc flags]
set -e
cd "$(dirname "$0")/../yjs_amd/csrc"
name=$1; src=$2; from=$3; shift 3
tmp=_ab_${name}_$src
if [ -f "$from" ]; then cp "$from" $tmp; else git show "$from:yjs_amd/csrc/$src" > $tmp; fi
obj=build/$(basename $src .hip).o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value "$@" -c $tmp -o /tmp/_ab_$name.o
rm -f $tmp
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $(ls build/ym_*.o | grep -v "^$obj$") /tmp/_ab_$name.o -o ../libymerge_$name.so
echo built yjs_amd/libymerge_$name.so
