#!/bin/bash
# In-flight frame time vs compositing chunk length (current default pipeline).
O=$1; mkdir -p $O
for rep in 1 2; do
for c in 1536 2048 4096 8192 32768; do
    GSR_CHUNK=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-profile --steps 100 --warmup 10 > $O/c${c}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/c${c}_r$rep.json')); print('chunk $c rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4))"
done
done
