# where the run repair's time goes: the product against a build that stops after the window's tests
set -o pipefail
timeout -k 10 600 bash tools/trace_ab.sh c8 "GSR_AB_DEFAULT=1" "GSR_LIB_PATH=varlib/nosort.so"
