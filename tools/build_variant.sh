#!/bin/bash
# Builds an experiment variant of libnmf.so with extra defines: tools/build_variant.sh <out.so> -DFOO ...
set -e
OUT=$1; shift
C=$(dirname "$0")/../nmfconsensus_amd/csrc
T=$(mktemp -d)
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c $C/brunet.hip -o $T/b.o
$H --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c $C/engine.hip -o $T/e.o
$H --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c $C/generic.hip -o $T/g.o
$H --offload-arch=gfx950 -O3 -fPIC -std=c++17 "$@" -c $C/solo.hip -o $T/s.o
$H --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c $C/compat.hip -o $T/c.o
$H -O3 -fPIC -std=c++17 -x c++ -c $C/hclust.cpp -o $T/h.o
$H --offload-arch=gfx950 -shared -fPIC -o "$OUT" $T/e.o $T/c.o $T/b.o $T/g.o $T/s.o $T/h.o -Wl,-soname,libnmf.so
rm -rf $T
