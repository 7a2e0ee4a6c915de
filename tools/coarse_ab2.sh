# the run repair loading the slots only when a run needs sorting: GPU tests of the order, frame-alone traces, bench
set -o pipefail
O=gpurun_out/c7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_coarse_depth.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 600 bash tools/trace_ab.sh c7 "GSR_DEPTH_COARSE=0" "GSR_AB_DEFAULT=1" || exit 2
for rep in 1 2; do
  timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu-baseline >> $O/bench_D_100.jsonl 2>> $O/bench.err || exit 3
done
