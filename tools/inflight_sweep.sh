#!/bin/bash
# Throughput vs views in flight per GPU: bash tools/inflight_sweep.sh OUT_PREFIX N1 N2 ...
P=$1; shift
for n in "$@"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --inflight $n > gpurun_out/${P}_if$n.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${P}_if$n.json')); print('inflight', $n, round(d['ms_per_step'],4), round(d['latency_ms_per_frame'],4))"
done
