#!/bin/bash
# Views in flight as groups of 5: 10 (2 groups), 15 (3), 20 (4, default), 25 (5); 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2; do
for k in 10 15 20 25; do
    for steps in 20 100; do
        timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 --inflight $k --share 5 > $O/k${k}_s${steps}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/k${k}_s${steps}_r$rep.json')); print('inflight $k steps $steps rep $rep', round(d['ms_per_step'],4))"
    done
done
done
