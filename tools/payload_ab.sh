#!/bin/bash
# Depth sort carrying the packed tile rects (default) vs the binning's by-id gather (GSR_NO_RECT_PAYLOAD)
for i in 1 2; do
  for mode in payload gather; do
    if [ $mode = gather ]; then export GSR_NO_RECT_PAYLOAD=1; else unset GSR_NO_RECT_PAYLOAD; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/pab.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/pab.json')); print('$mode', round(d['ms_per_step'],4), {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
  done
done
unset GSR_NO_RECT_PAYLOAD
