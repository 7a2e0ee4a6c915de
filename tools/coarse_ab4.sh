# the repairing kernel's instances per thread (16, 8, 12): order tests per build, frame-alone traces
set -o pipefail
O=gpurun_out/c9
mkdir -p $O
for lib in fix8 fix12; do
  GSR_LIB_PATH=varlib/$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_coarse_depth.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$lib.log 2>&1 || exit 1
done
timeout -k 10 600 bash tools/trace_ab.sh c9 "GSR_AB_DEFAULT=1" "GSR_LIB_PATH=varlib/fix8.so" "GSR_LIB_PATH=varlib/fix12.so" || exit 2
