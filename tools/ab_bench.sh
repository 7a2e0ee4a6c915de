#!/bin/bash
# A/B the bench across library variants: bash tools/ab_bench.sh OUT_PREFIX lib1.so [lib2.so ...]
# (each variant: python bench.py --no-cpu-baseline with GSR_LIB_PATH set; product lib if "default")
P=$1; shift
for lib in "$@"; do
    name=$(basename $lib .so)
    if [ "$lib" = default ]; then
        timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${P}_$name.json 2>/dev/null || exit 1
    else
        GSR_LIB_PATH=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${P}_$name.json 2>/dev/null || exit 1
    fi
    python -c "import json; d=json.load(open('gpurun_out/${P}_$name.json')); print('$name', round(d['ms_per_step'],4), {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
