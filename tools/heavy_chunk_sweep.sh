#!/bin/bash
# Group chunk length (GSR_CHUNK_VIEWS) on the heavy configs (c2h, c3), 50 frames.
O=$1; mkdir -p $O
for cfg in c2h c3; do
for c in 2048 3072 4096 6144; do
    GSR_CHUNK_VIEWS=$c timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --config $cfg --steps 50 --warmup 5 > $O/${cfg}_c$c.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/${cfg}_c$c.json')); print('$cfg chunk_views $c', round(d['ms_per_step'],4))"
done
done
