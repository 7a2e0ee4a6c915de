#!/bin/bash
# rocprofv3 kernel stats of a short bench run: bash tools/kstats_run.sh OUT [bench args...]
# (writes OUT/kernel_stats.csv and prints the top kernels)
O=$1; shift
export TMPDIR=/tmp
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- \
    python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $O/bench.json 2> $O/rocprof.err || exit 1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
python tools/kstats.py $O/kernel_stats.csv 1 | head -40
