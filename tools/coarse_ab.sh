# A/B of the coarse depth order on one box (profiles/r4_s32, run c6): GPU tests, frame-alone kernel traces, bench
set -o pipefail
O=gpurun_out/c6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_coarse_depth.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_variants.py tests/test_gpu_large_splats.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 600 bash tools/trace_ab.sh c6 "GSR_DEPTH_COARSE=0" "GSR_AB_DEFAULT=1" || exit 2
for rep in 1 2; do
for cfg in "D" "C GSR_DEPTH_COARSE=0"; do
  set -- $cfg; tag=$1; shift
  for st in 20 100; do
    timeout -k 10 120 env "$@" python bench.py --steps $st --warmup 5 --no-cpu-baseline >> $O/bench_${tag}_${st}.jsonl 2>> $O/bench.err || exit 3
  done
done
done
