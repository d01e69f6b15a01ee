#!/bin/bash
# usage: mkvar.sh name "FLAGS"  -> liblshkm_name.so (fused.hip rebuilt with FLAGS, other objects from build/)
set -e
V=$1; EXTRA=$2
mkdir -p build_$V
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -I../include -Icsrc $EXTRA -x hip -c csrc/fused.hip -o build_$V/fused.hip.o
objs=$(ls build/*.o | grep -v fused.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o liblshkm_$V.so $objs build_$V/fused.hip.o
