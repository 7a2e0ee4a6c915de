#!/bin/bash
# Group chunk length (GSR_CHUNK_VIEWS) with first-major dispatch; 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2; do
for c in 1536 2048 3072 4096 6144; do
    for steps in 20 100; do
        GSR_CHUNK_VIEWS=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 > $O/c${c}_s${steps}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/c${c}_s${steps}_r$rep.json')); print('chunk_views $c steps $steps rep $rep', round(d['ms_per_step'],4))"
    done
done
done
