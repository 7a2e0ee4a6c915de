#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r2_s10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ply_load.py tests/test_ply.py tests/test_gpu_unorm8.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest_ply.log 2>&1 || exit 1
timeout -k 10 300 python tools/ply_load_bench.py 1000000 $O/ply_load.json > $O/ply_load.log 2>&1
