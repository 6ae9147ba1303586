#!/usr/bin/env bash
# Lab builds for round-5 A/Bs: the engine with one source's extra -D flags,
# linked from the in-tree objects into profiles/r05/ab/<name>.so.
# Usage: build_lab.sh <name> <source stem, e.g. cksum_api> "<-D flags>"
set -eu
NAME=$1; SRC=$2; FLAGS=$3
cd "$(dirname "$0")/../../../libuinet_amd"
make -s -j8
F="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -I../include -Icsrc"
/opt/rocm/bin/hipcc $F $FLAGS -c csrc/$SRC.hip -o build/lab_$NAME.o
OBJS=$(ls build/*.o | grep -v -e "/$SRC.o" -e lab_)
/opt/rocm/bin/hipcc $F -shared -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -o ../profiles/r05/ab/$NAME.so $OBJS build/lab_$NAME.o
echo built ../profiles/r05/ab/$NAME.so
