set -e
mkdir -p gpurun_out/r5_s15
timeout -k 10 600 python -u -m pytest tests/test_gpu_long_runs.py tests/test_gpu_coarse_depth.py tests/test_gpu_parity.py tests/test_gpu_unorm8.py tests/test_gpu_variants.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r5_s15/pytest.log 2>&1
bash tools/ab.sh r5_s15_c3 1 "GSR_CHUNK=192" "GSR_CHUNK=384" "GSR_CHUNK=768" "GSR_CHUNK=1536" -- --config c3 --steps 20 --warmup 5 > gpurun_out/r5_s15_c3.log 2>&1
bash tools/ab.sh r5_s15_c2 1 "GSR_CHUNK=192" "GSR_CHUNK=256" "GSR_CHUNK=384" "GSR_CHUNK=768" -- --steps 20 --warmup 5 > gpurun_out/r5_s15_c2.log 2>&1
