#!/bin/bash
# GPU check of the current tree on one MI355X (run through gpurun):
# load, parity tests, smoke, bench, rocprofv3 kernel stats, HBM PMC passes.
# usage: gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG [quick|full]
#   quick: load, parity tests, smoke, bench (no CPU baseline), kernel stats
#   full: + the CPU baseline and the PMC traffic passes (tools/pmc.sh TAG traffic)
# Every step has its own time limit; the first failing step ends the script.
TAG=${1:-run}
MODE=${2:-full}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"  # the driver's region (BENCH_rNN: --steps 20 --warmup 5)

step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2
    shift 2
    echo "[gpu_round] $name"
    timeout -k 10 "$secs" "$@"
    local rc=$?
    if [ $rc -ne 0 ]; then
        echo "[gpu_round] $name FAILED rc=$rc"
        exit $rc
    fi
}

# (the library is built here, in-tree, and travels with the tree: the driver runs without building;
# the load step fails on a library older than its sources: gsviewer_amd/_srcid.py)
step load 120 bash -c "python -c 'from gsviewer_amd import _lib; _lib.load()' > $O/load.log 2>&1"
step pytest_gpu 600 bash -c "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1"
step smoke 120 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1"
if [ "$MODE" = quick ]; then
    step bench 300 bash -c "python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err"
else
    step bench 300 bash -c "python bench.py > $O/bench.json 2> $O/bench.err"
fi
step rocprof_stats 240 bash -c "rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- $B > $O/bench_under_rocprof.json 2> $O/rocprof.err"
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
# the compositing kernel's busy time per view (union of its overlapping launches), bench.py's cross-check
step busy_union 60 bash -c "python tools/busy_union.py \$(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/composite_busy.json"
# every kernel's busy time in the timed region (bench.py's per-kernel roofline table), and the trace itself (gzip)
step region_kernels 60 bash -c "T=\$(find $O/prof -name '*kernel_trace.csv' | head -1); python tools/region_kernels.py \$T > $O/region_kernels.json && gzip -9 -c \$T > $O/prof/prof_kernel_trace.csv.gz"
if [ "$MODE" != quick ]; then
    step pmc 800 bash tools/pmc.sh $TAG traffic
    step pmc_stalls 600 bash tools/pmc.sh ${TAG}_stalls stalls
fi
echo "[gpu_round] done"
