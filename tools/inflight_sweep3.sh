#!/bin/bash
# Views in flight x group size for 20- and 100-frame regions (current pipeline).
O=$1; mkdir -p $O
for rep in 1 2; do
for cfg in "20 5" "16 4" "24 6" "32 8" "40 8"; do
    set -- $cfg
    for steps in 20 100; do
        timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 --inflight $1 --share $2 > $O/s${steps}_i$1_g$2_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/s${steps}_i$1_g$2_r$rep.json')); print('steps $steps inflight $1 share $2 rep $rep', round(d['ms_per_step'],4))"
    done
done
done
