#!/bin/bash
# Short (driver: 20 frames) and long timed regions for more views in flight.
O=$1; mkdir -p $O
for rep in 1 2; do
for cfg in "16 4" "20 5" "20 4" "24 6" "24 4" "32 8" "32 4"; do
    set -- $cfg
    for steps in 20 100; do
        timeout -k 10 120 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 --inflight $1 --share $2 > $O/s${steps}_i$1_g$2_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/s${steps}_i$1_g$2_r$rep.json')); print('steps $steps inflight $1 share $2 rep $rep', round(d['ms_per_step'],4))"
    done
done
done
