#!/bin/bash
# A frame finished alone: first-major dispatch (GSR_FIRST_MAJOR_ALONE) x chunk length (GSR_CHUNK); latency.
O=$1; mkdir -p $O
for rep in 1 2; do
for fm in 0 1; do
for c in 192 384 768 1536; do
    GSR_FIRST_MAJOR_ALONE=$fm GSR_CHUNK=$c timeout -k 10 150 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/fm${fm}_c${c}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/fm${fm}_c${c}_r$rep.json')); st=d['stage_ms']; print('first_major_alone $fm chunk $c rep $rep lat', round(d['latency_ms_per_frame'],4), 'composite', round(st['composite']*1e3,1), 'merge', round(st['merge']*1e3,1))"
done
done
done
