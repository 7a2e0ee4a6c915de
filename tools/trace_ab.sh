#!/bin/bash
# A/B of the frame-alone kernels: rocprofv3 kernel trace per env variant
# usage: bash tools/trace_ab.sh TAG "VAR=1 VAR2=0" "VAR=0" ...
O=gpurun_out/$1; shift
mkdir -p $O
export TMPDIR=/tmp
i=0
for v in "$@"; do
    i=$((i+1))
    echo "[ab] variant $i: $v" | tee -a $O/variants.txt
    env $v timeout -k 10 240 rocprofv3 --kernel-trace -d $O/p$i -o prof --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench$i.json 2> $O/rocprof$i.err || { echo "variant $i failed"; exit 1; }
    python tools/frame_kernels.py $O/p$i/prof_kernel_trace.csv > $O/frame$i.txt
done
