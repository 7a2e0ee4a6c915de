#!/bin/bash
# In-flight frame time with and without the depth sort's rect payload (GSR_NO_RECT_PAYLOAD).
O=$1; mkdir -p $O
for rep in 1 2; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/pay_r$rep.json 2>/dev/null || exit 1
    GSR_NO_RECT_PAYLOAD=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/nopay_r$rep.json 2>/dev/null || exit 1
    for v in pay nopay; do python -c "import json; d=json.load(open('$O/${v}_r$rep.json')); s=d['stage_ms']; print('$v', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_frame'],4), 'dsort', round(s['depth_sort']*1e3,1), 'bin', round(s['binning']*1e3,1))"; done
done
