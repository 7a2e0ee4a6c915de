#!/bin/bash
# The driver's bench region (--steps 20 --warmup 5) on one box: interleaved
# repeats of the bench variants given, then one rocprofv3 kernel trace of the
# first variant.  usage: bash tools/region20.sh TAG ROUNDS VARIANT...
TAG=$1; ROUNDS=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
bash tools/ab.sh $TAG $ROUNDS "$@" -- --steps 20 --warmup 5 --no-profile || exit $?
read -r -a first <<< "$1"
[ "$1" = "-" ] && first=()
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/trace -o prof --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-profile "${first[@]}" > $O/trace_bench.json 2> $O/trace.err || exit $?
echo "[region20] done"
