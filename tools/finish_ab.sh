#!/bin/bash
# Shared-scene-pass bench: batched group finish (gsr_render_finish_views) vs per-view finishes
for i in 1 2; do
  for flag in "" "--no-batched-finish"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile $flag > gpurun_out/fab.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/fab.json')); print('batched' if '$flag' == '' else 'per-view', round(d['ms_per_step'],4))"
  done
done
