export TMPDIR=/tmp
O=gpurun_out/r2_s4
mkdir -p $O
timeout -k 10 900 bash tools/bench_configs.sh $O/configs > $O/configs.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c2h -o prof --output-format csv -- python bench.py --config c2h --steps 30 --no-cpu-baseline > $O/c2h_rocprof.json 2> $O/c2h_rocprof.err
