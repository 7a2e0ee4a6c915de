#!/bin/bash
# Default (shared-scene-pass) bench throughput over compositing chunk sizes: bash tools/chunk_sweep_share.sh "128 192"
for c in $1; do
  GSR_CHUNK=$c timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile > gpurun_out/css_$c.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/css_$c.json')); print('chunk $c', round(d['ms_per_step'],4))"
done
