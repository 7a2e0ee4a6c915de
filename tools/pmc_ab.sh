#!/bin/bash
# Composite-kernel PMC passes for several library variants (A/B of stall
# sources): bash tools/pmc_ab.sh OUT_PREFIX lib1.so|default [lib2.so ...]
# -> gpurun_out/<prefix>_<lib>.csv (profiles/summarize_pmc.py format)
export TMPDIR=/tmp
P=$1; shift
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --inflight 1 --no-profile"
pass() {  # pass DIR COUNTERS...
    local d=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" -d $d -o pmc --output-format csv -- $B > $d.log 2>&1
}
for lib in "$@"; do
    name=$(basename $lib .so)
    O=gpurun_out/${P}_$name
    if [ "$lib" = default ]; then unset GSR_LIB_PATH; else export GSR_LIB_PATH=$lib; fi
    pass ${O}_a SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH || exit 1
    pass ${O}_b SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS || exit 1
    pass ${O}_c SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit 1
    python profiles/summarize_pmc.py $O.csv $(find ${O}_a ${O}_b ${O}_c -name '*counter_collection.csv' -printf '%h\n' | sort -u)
    grep "k_composite<0>" $O.csv
done
