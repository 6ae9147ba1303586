#!/usr/bin/env bash
# Lab build for the wait A/B: the engine with -DUINET_WAIT_SPIN (ctx_wait in
# hipEventSynchronize, as before round 5), linked from the in-tree objects.
set -eu
cd "$(dirname "$0")/../../../libuinet_amd"
make -s -j8
F="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -I../include -Icsrc"
/opt/rocm/bin/hipcc $F -DUINET_WAIT_SPIN -c csrc/cksum_api.hip -o build/lab_spin_api.o
OBJS=$(ls build/*.o | grep -v -e cksum_api.o -e lab_)
/opt/rocm/bin/hipcc $F -shared -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined -o ../profiles/r05/ab/spin.so $OBJS build/lab_spin_api.o
echo built ../profiles/r05/ab/spin.so
