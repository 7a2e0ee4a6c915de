set -e
mkdir -p gpurun_out/r2_s44
bash tools/lib_ab.sh gpurun_out/r2_s44/r ab_libs/base.so ab_libs/depthr16.so 2
bash tools/lib_ab.sh gpurun_out/r2_s44/t ab_libs/base.so ab_libs/tiler32.so 2
bash tools/chunk_views_sweep.sh gpurun_out/r2_s44/cv
