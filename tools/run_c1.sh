# coarse depth order: frame-alone kernel traces (exact, coarse 16, coarse 16 without the repair's sort)
set -o pipefail
timeout -k 10 900 bash tools/trace_ab.sh c4 "GSR_DEPTH_COARSE=0" "GSR_DEPTH_COARSE_ALONE=16 GSR_DEPTH_COARSE_VIEWS=0" "GSR_DEPTH_COARSE_ALONE=16 GSR_DEPTH_COARSE_VIEWS=0 GSR_LIB_PATH=varlib/nosort.so"
