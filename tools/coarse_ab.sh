#!/bin/bash
# Frames' depth sort: GSR_DEPTH_COARSE=16 (2 passes of the top 16 key bits + the tile-list run fix-up)
# vs 0 (the full 4-pass sort); 20- and 100-frame regions, single-view latency and stage times.
O=$1; mkdir -p $O
for rep in 1 2; do
for c in 16 0; do
    for steps in 20 100; do
        GSR_DEPTH_COARSE=$c timeout -k 10 150 python bench.py --no-cpu-baseline --steps $steps --warmup 5 > $O/s${steps}_c${c}_r$rep.json 2>$O/err.txt || exit 1
        python -c "
import json; d=json.load(open('$O/s${steps}_c${c}_r$rep.json')); st=d['stage_ms']
print('steps $steps coarse $c rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4), 'depth_sort', round(st['depth_sort']*1e3,1), 'binning', round(st['binning']*1e3,1), 'tile_sort', round(st['tile_sort']*1e3,1), 'ranges', round(st['tile_ranges']*1e3,1))"
    done
done
done
