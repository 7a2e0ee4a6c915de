#!/bin/bash
# 20 views in flight as groups of 4 (5 groups), 5 (4, default), 8 (8+8+4); 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2; do
for sh in 4 5 8; do
    for steps in 20 100; do
        timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 --inflight 20 --share $sh > $O/sh${sh}_s${steps}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/sh${sh}_s${steps}_r$rep.json')); print('share $sh steps $steps rep $rep', round(d['ms_per_step'],4))"
    done
done
done
