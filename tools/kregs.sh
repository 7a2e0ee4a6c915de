#!/bin/bash
# Per-kernel VGPRs / SGPRs / LDS / occupancy of one csrc file (hipcc remarks):
#   bash tools/kregs.sh preprocess.hip [extra hipcc flags]
src=$1; shift
extra=""
[ "$src" = "preprocess.hip" ] && extra="-ffp-contract=off"
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -c -fno-slp-vectorize -O3 $extra "$@" \
    -I/root/repo/include -I/root/repo/gsviewer_amd/csrc -Rpass-analysis=kernel-resource-usage \
    /root/repo/gsviewer_amd/csrc/$src -o /tmp/kregs.o 2>&1 | python3 /root/repo/tools/kregs.py
