#!/bin/bash
# Full GPU check of the current tree on one MI355X (run through gpurun):
# build, parity tests, smoke, bench, rocprofv3 kernel stats, HBM PMC passes.
# usage: gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --steps 50 --warmup 10 --no-cpu-baseline"
echo "[gpu_round] build" && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 && \
echo "[gpu_round] pytest -m gpu" && \
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
echo "[gpu_round] smoke" && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
echo "[gpu_round] bench" && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
echo "[gpu_round] rocprof stats" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- $B > $O/bench_under_rocprof.json 2> $O/rocprof.err && \
echo "[gpu_round] pmc fetch" && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- $B > $O/pmc_fetch.log 2>&1 && \
echo "[gpu_round] pmc write" && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- $B > $O/pmc_write.log 2>&1 && \
python profiles/summarize_pmc.py $O/pmc_summary.csv $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv' -printf '%h\n' | sort -u) && \
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \; && \
echo "[gpu_round] done"
