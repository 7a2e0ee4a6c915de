#!/bin/bash
# In-flight frame time (20 and 100 frames) vs the group path's compositing chunk (GSR_CHUNK_VIEWS).
O=$1; mkdir -p $O
for rep in 1 2 3; do
for c in 2048 3072 4096; do
    for steps in 20 100; do
        GSR_CHUNK_VIEWS=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 > $O/c${c}_s${steps}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/c${c}_s${steps}_r$rep.json')); print('chunk_views $c steps $steps rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4))"
    done
done
done
