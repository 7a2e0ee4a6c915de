#!/bin/bash
# Compositing dispatch order: GSR_LEN_CLASSES (2 = full chunks then partials in
# tile order; more = partials longest class first); 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2; do
for c in 2 4 8 16; do
    for steps in 20 100; do
        GSR_LEN_CLASSES=$c timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 > $O/s${steps}_c${c}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/s${steps}_c${c}_r$rep.json')); print('steps $steps classes $c rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4))"
    done
done
done
