#!/bin/bash
# Compositor with the scene in given vs 3D Morton order: bench A/B, kernel stats and FETCH_SIZE.
O=$1; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for order in given morton; do
    timeout -k 10 150 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --scene-order $order > $O/${order}_r$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/${order}_r$rep.json')); s=d['stage_ms']; print('$order rep $rep', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4), {k: round(v*1e3,1) for k,v in s.items()})"
done
done
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --inflight 1 --share 1 --no-batched-sorts --no-batched-finish"
for order in given morton; do
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$order -o pmc --output-format csv -- $B --scene-order $order > $O/fetch_$order.log 2>&1 || exit 1
    python profiles/summarize_pmc.py $O/fetch_$order.csv $(find $O/fetch_$order -name '*counter_collection.csv' -printf '%h\n' | sort -u)
    echo "$order"; grep -E "k_composite<0>|k_preprocess<3>|k_bin_write|k_rs_scatter" $O/fetch_$order.csv
done
