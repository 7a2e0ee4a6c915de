# coarse depth order with the keys carried by the binning and the tile sort: GPU tests, kernel traces, bench A/B
set -o pipefail
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 600 bash tools/trace_ab.sh c5 "GSR_DEPTH_COARSE=0" "GSR_AB_DEFAULT=1" || exit 2
for rep in 1 2; do
for cfg in "D" "C GSR_DEPTH_COARSE=0"; do
  set -- $cfg; tag=$1; shift
  for st in 20 100; do
    timeout -k 10 120 env "$@" python bench.py --steps $st --warmup 5 --no-cpu-baseline >> $O/bench_${tag}_${st}.jsonl 2>> $O/bench.err || exit 3
  done
done
done
