set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final2/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/final2/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final2/bench20.json 2> gpurun_out/final2/bench20.err
