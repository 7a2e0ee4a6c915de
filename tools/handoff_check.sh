#!/bin/bash
# The tail-merge hand-off tests (tests/test_gpu_handoff.py, and the 1080p
# repeatability test in which round 3 saw the two visibility bugs) against the
# product library and the two verification builds that restore the code
# before each round-3 fix (varlib/revert_sc1.so: -DGSR_TAIL_REVERT_SC1_LOADS,
# varlib/revert_sat.so: -DGSR_TAIL_REVERT_SAT_ATOMIC).
# usage: bash tools/handoff_check.sh TAG [REPEATS]
O=gpurun_out/$1
R=${2:-1}
mkdir -p $O
for v in product revert_sc1 revert_sat; do
    if [ $v = product ]; then lib=""; else lib="GSR_LIB_PATH=varlib/$v.so"; fi
    for r in $(seq 1 $R); do
        env $lib timeout -k 10 300 python -u -m pytest tests/test_gpu_handoff.py \
            tests/test_gpu_variants.py::test_group_frames_repeatable -q --timeout 240 --timeout-method thread \
            > $O/handoff_${v}_$r.log 2>&1
        rc=$?
        echo "[handoff] $v run $r rc=$rc $(tail -1 $O/handoff_${v}_$r.log)"
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # 1 = test failures
    done
done
