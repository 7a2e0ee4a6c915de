#!/bin/bash
# Depth sort passes of a frame rendered alone (gsr_render) (GSR_DEPTH_PASSES_ALONE 3 vs 4): single-view latency and stage times.
O=$1; mkdir -p $O
for rep in 1 2 3; do
for p in 4 3; do
    GSR_DEPTH_PASSES_ALONE=$p timeout -k 10 150 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/p${p}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/p${p}_r$rep.json')); st=d['stage_ms']; print('passes $p rep $rep lat', round(d['latency_ms_per_frame'],4), 'inflight', round(d['ms_per_step'],4), 'depth_sort', round(st['depth_sort']*1e3,1))"
done
done
