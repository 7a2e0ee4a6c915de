#!/bin/bash
# 20 views in flight as groups of 5 (4 streams), 7 (7+7+6), 8 (8+8+4); 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2 3; do
for g in 5 7 8; do
    for steps in 20 100; do
        timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 --inflight 20 --share $g > $O/s${steps}_g${g}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/s${steps}_g${g}_r$rep.json')); print('steps $steps share $g rep $rep', round(d['ms_per_step'],4))"
    done
done
done
