#!/bin/bash
# In-flight frame time vs LDS padding of the batched compositor (caps its blocks per CU).
O=$1; mkdir -p $O
for rep in 1 2; do
for pad in 0 8192 16384 28672 45056; do
    GSR_COMP_LDS_PAD=$pad timeout -k 10 120 python bench.py --no-cpu-baseline --no-profile --steps 100 --warmup 10 > $O/p${pad}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/p${pad}_r$rep.json')); print('pad $pad rep $rep', round(d['ms_per_step'],4))"
done
done
