#!/bin/bash
# Record-pair compositor A/B (round 2): parity with the variant, then the bench per variant.
export TMPDIR=/tmp
O=gpurun_out/r2_s5; mkdir -p $O
GSR_LIB_PATH=varlib/pair6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiview.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pair6.log 2>&1 || exit 1
bash tools/ab_bench.sh r2_s5/ab varlib/base.so varlib/pair6.so varlib/pair7.so varlib/pair8.so varlib/base.so varlib/pair6.so > $O/ab.log 2>&1
