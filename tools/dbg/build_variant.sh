#!/bin/bash
# Build a libyoda variant from an alternative yoda_kernels.hip (A/B timing only):
#   tools/dbg/build_variant.sh <kernels.hip> <out.so>
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
SRC=$ROOT/kubernetes-scheduler_amd/csrc
T=$(mktemp -d)
cp "$1" $T/yoda_kernels.hip; cp $SRC/yoda_layout.h $T/
make -s -C $SRC build/yoda_order.o build/yoda_capi.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -c -o $T/k.o $T/yoda_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$2" $T/k.o $SRC/build/yoda_order.o $SRC/build/yoda_capi.o
rm -rf $T
