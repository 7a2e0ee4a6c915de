#!/bin/bash
# A/B two library builds (GSR_LIB_PATH) on the bench, alternating, 20- and 100-frame regions:
# bash tools/lib_ab.sh OUT a.so b.so [reps]
O=$1; A=$2; B=$3; R=${4:-3}; mkdir -p $O
for rep in $(seq 1 $R); do
for lib in $A $B; do
    name=$(basename $lib .so)
    for steps in 20 100; do
        GSR_LIB_PATH=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --steps $steps --warmup 5 > $O/s${steps}_${name}_r$rep.json 2>$O/err.txt || exit 1
        python -c "
import json; d=json.load(open('$O/s${steps}_${name}_r$rep.json')); st=d['stage_ms']
print('steps $steps $name rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4), 'merge', round(st['merge']*1e3,1))"
    done
done
done
