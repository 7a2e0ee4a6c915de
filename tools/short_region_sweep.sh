#!/bin/bash
# The driver times 20 frames (python3 bench.py --gpus 1 --steps 20 --warmup 5):
# frame rate of short timed regions vs views in flight / group size.
# bash tools/short_region_sweep.sh OUT
O=$1; mkdir -p $O
for rep in 1 2; do
for cfg in "16 4" "8 4" "12 4" "8 2" "4 4" "16 8"; do
    set -- $cfg
    for steps in 20 100; do
        timeout -k 10 120 python bench.py --no-cpu-baseline --steps $steps --warmup 5 --inflight $1 --share $2 > $O/s${steps}_i$1_g$2_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/s${steps}_i$1_g$2_r$rep.json')); print('steps $steps inflight $1 share $2 rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4))"
    done
done
done
