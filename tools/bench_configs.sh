#!/bin/bash
# Bench lines for the other BASELINE.json configs (the driver's bench runs c2):
# c1 (100k, deg 0, 640x480) with the CPU baseline (the reference's CPU-sort
# OGL path as defined for C1), c3 (6M, 1080p), c5 (1M, 4K) plain / AABB / OBB
# cull, and the c2h heavy-splat stress scene beside c2.
# usage (GPU box): [BENCH_EXTRA="--inflight 1"] bash tools/bench_configs.sh OUT_DIR
O=${1:-gpurun_out/configs}
mkdir -p $O
run() {  # run NAME ARGS...
    local name=$1
    shift
    echo "[bench_configs] $name"
    timeout -k 10 300 python bench.py $BENCH_EXTRA "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; exit 1; }
}
run c1 --config c1 --cpu-seconds 15
BENCH_EXTRA="--no-cpu-baseline $BENCH_EXTRA"
run c2h --config c2h --steps 50
run c3 --config c3 --steps 50
run c5 --config c5 --steps 50
run c5_aabb --config c5 --box aabb --steps 50
run c5_obb --config c5 --box obb --steps 50
for f in $O/*.json; do
    python -c "import json,sys; d=json.load(open('$f')); print('$(basename $f .json)', d['config']['workload'], 'ms', round(d['ms_per_step'],4), 'splats/s %.3g' % d['value'], 'vis', d['frame_stats']['n_visible'], 'inst', d['frame_stats']['n_instances'], 'p99', d['frame_stats']['tile_len_p99'], 'cpu', (d['cpu_baseline'] or {}).get('ms_per_frame'))"
done
