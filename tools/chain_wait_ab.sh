#!/bin/bash
# Later chunks waiting for their tile's previous chunk (GSR_CHAIN_WAIT=1) vs not (0); 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2 3; do
for cw in 0 1; do
    for steps in 20 100; do
        GSR_CHAIN_WAIT=$cw timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 > $O/cw${cw}_s${steps}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/cw${cw}_s${steps}_r$rep.json')); print('chain_wait $cw steps $steps rep $rep', round(d['ms_per_step'],4))"
    done
done
done
