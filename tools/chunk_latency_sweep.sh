#!/bin/bash
# Single-view latency and in-flight frame time vs compositing chunk length.
O=$1; mkdir -p $O
for rep in 1 2; do
for c in 96 128 160 192; do
    GSR_CHUNK=$c timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/c${c}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/c${c}_r$rep.json')); s=d['stage_ms']; print('chunk $c rep $rep inflight', round(d['ms_per_step'],4), 'latency', round(d['latency_ms_per_frame'],4), 'comp', round(s['composite']*1e3,1), 'merge', round(s['merge']*1e3,1), 'ranges', round(s['tile_ranges']*1e3,1))"
done
done
