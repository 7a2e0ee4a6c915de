#!/bin/bash
# Single-view latency (bench's one-view-at-a-time region) vs GSR_CHUNK (the path of a frame finished alone).
O=$1; mkdir -p $O
for rep in 1 2; do
for c in 128 192 256 384 512; do
    GSR_CHUNK=$c timeout -k 10 150 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/c${c}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/c${c}_r$rep.json')); st=d['stage_ms']; print('chunk $c rep $rep lat', round(d['latency_ms_per_frame'],4), 'composite', round(st['composite']*1e3,1), 'merge', round(st['merge']*1e3,1), 'ranges', round(st['tile_ranges']*1e3,1))"
done
done
