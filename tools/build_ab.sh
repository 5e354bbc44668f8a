#!/bin/bash
# Build A/B variants of libyoda from the current sources into abl/ (timing runs only; abl/ is
# git-ignored but travels to the GPU box):
#   tools/build_ab.sh <name> [kernel -D flags...]   -> abl/<name>.so (capi with -DYODA_AB_KNOBS)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/kubernetes-scheduler_amd/csrc
NAME=$1; shift
mkdir -p $ROOT/abl
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize"
T=$(mktemp -d)
/opt/rocm/bin/hipcc $F -DYODA_AB_KNOBS "$@" -c -o $T/k.o $SRC/yoda_kernels.hip
/opt/rocm/bin/hipcc $F -c -o $T/o.o $SRC/yoda_order.hip
/opt/rocm/bin/hipcc $F -DYODA_AB_KNOBS -c -o $T/c.o $SRC/yoda_capi.cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/abl/$NAME.so $T/k.o $T/o.o $T/c.o
rm -rf $T
