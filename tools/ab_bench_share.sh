#!/bin/bash
# A/B of library variants on the default (shared-scene-pass) bench, no profile region:
# bash tools/ab_bench_share.sh OUT_PREFIX lib1.so|default [lib2.so ...]
P=$1; shift
for lib in "$@"; do
    name=$(basename $lib .so)
    if [ "$lib" = default ]; then
        timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile > gpurun_out/${P}_$name.json 2>/dev/null || exit 1
    else
        GSR_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile > gpurun_out/${P}_$name.json 2>/dev/null || exit 1
    fi
    python -c "import json; d=json.load(open('gpurun_out/${P}_$name.json')); print('$name', round(d['ms_per_step'],4))"
done
