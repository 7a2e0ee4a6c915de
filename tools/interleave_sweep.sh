#!/bin/bash
# A group's compositing dispatch: GSR_VIEWS_INTERLEAVE (0 view-major, 1 class-major over the views) x
# GSR_LEN_CLASSES; 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2; do
for cfg in "0 2" "1 2" "1 4" "1 8" "0 8"; do
    set -- $cfg
    for steps in 20 100; do
        GSR_VIEWS_INTERLEAVE=$1 GSR_LEN_CLASSES=$2 timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 > $O/s${steps}_i$1_c$2_r$rep.json 2>$O/err.txt || exit 1
        python -c "import json; d=json.load(open('$O/s${steps}_i$1_c$2_r$rep.json')); print('steps $steps interleave $1 classes $2 rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4))"
    done
done
done
