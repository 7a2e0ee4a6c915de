#!/bin/bash
# Throughput with views sharing one scene pass: bash tools/share_sweep.sh PREFIX "inflight:share ..."
P=$1
for cfg in $2; do
  n=${cfg%%:*}; sh=${cfg##*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile --inflight $n --share $sh > gpurun_out/${P}_$n_$sh.json 2>gpurun_out/${P}_${n}_$sh.err || { echo "inflight $n share $sh FAILED"; tail -5 gpurun_out/${P}_${n}_$sh.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${P}_$n_$sh.json')); print('inflight $n share $sh', round(d['ms_per_step'],4), '%.3g' % d['value'])"
done
