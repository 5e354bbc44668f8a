#!/bin/bash
# Variants after a stream switch on fresh handles (the race fixed by switch_stream), plus the
# GPU suite: serialised kernels for the first pass so a fault names its kernel.
set -o pipefail
mkdir -p gpurun_out/dbgmix
AMD_SERIALIZE_KERNEL=3 timeout -k 10 180 python3 tools/variants.py mixed50 --steps 1 > gpurun_out/dbgmix/out.txt 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/dbgmix/out.txt; exit 1; }
cut -c1-300 gpurun_out/dbgmix/out.txt
bash tools/gpu_quick.sh gpurun_out/k1mix "" mixed50 c3 het100k c4 bytes
