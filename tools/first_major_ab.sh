#!/bin/bash
# A group's compositing dispatch: first chunks before later chunks (GSR_FIRST_MAJOR=1) vs the full-chunks-first
# order (0); 20- and 100-frame regions.
O=$1; mkdir -p $O
for rep in 1 2 3; do
for fm in 0 1; do
    for steps in 20 100; do
        GSR_FIRST_MAJOR=$fm timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile --steps $steps --warmup 5 > $O/fm${fm}_s${steps}_r$rep.json 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$O/fm${fm}_s${steps}_r$rep.json')); print('first_major $fm steps $steps rep $rep', round(d['ms_per_step'],4))"
    done
done
done
