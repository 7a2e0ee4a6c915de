#!/bin/bash
# Throughput over (views in flight, chunk size): bash tools/inflight_chunk_sweep.sh PREFIX "4 6 8" "128 192"
P=$1
for n in $2; do
  for c in $3; do
    GSR_CHUNK=$c timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --inflight $n > gpurun_out/${P}_if${n}_c$c.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${P}_if${n}_c$c.json')); print('inflight $n chunk $c', round(d['ms_per_step'],4), round(d['latency_ms_per_frame'],4))"
  done
done
