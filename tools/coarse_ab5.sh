# the repairing kernel at 4 instances per thread against the product's 8: order tests, frame-alone traces
set -o pipefail
O=gpurun_out/c10
mkdir -p $O
GSR_LIB_PATH=varlib/fix4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_coarse_depth.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_fix4.log 2>&1 || exit 1
timeout -k 10 600 bash tools/trace_ab.sh c10 "GSR_AB_DEFAULT=1" "GSR_LIB_PATH=varlib/fix4.so" || exit 2
