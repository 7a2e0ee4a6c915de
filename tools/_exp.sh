set -e
export TMPDIR=/tmp
O=gpurun_out/r5_s17
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_long_runs.py tests/test_gpu_coarse_depth.py tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_multiview.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o prof --output-format csv -- python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o prof --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c2.json 2> $O/c2.err
bash tools/ab.sh r5_s17_c3 1 "GSR_CHUNK_TARGET=0" "GSR_CHUNK_TARGET=16384" "GSR_CHUNK_TARGET=8192" -- --config c3 --steps 20 --warmup 5 > $O/ab_c3.log 2>&1
bash tools/ab.sh r5_s17_c2h 1 "GSR_CHUNK_TARGET=0" "GSR_CHUNK_TARGET=16384" "GSR_CHUNK_TARGET=8192" -- --config c2h --steps 20 --warmup 5 > $O/ab_c2h.log 2>&1
bash tools/ab.sh r5_s17_c5 1 "GSR_CHUNK_TARGET=0" "GSR_CHUNK_TARGET=8192" -- --config c5 --steps 20 --warmup 5 > $O/ab_c5.log 2>&1
