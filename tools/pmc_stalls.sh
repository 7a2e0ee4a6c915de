#!/bin/bash
# Stall/issue counters of the single-view frame's kernels for library variants:
# bash tools/pmc_stalls.sh OUTDIR lib1.so [lib2.so ...]   (default = product lib)
# -> OUTDIR/NAME_summary.csv per variant (profiles/summarize_pmc.py format)
O=$1; shift
export TMPDIR=/tmp
mkdir -p $O
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --inflight 1 --share 1 --no-batched-sorts --no-batched-finish"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU"
P3="SQ_THREAD_CYCLES_VALU SQ_IFETCH SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAVES"
for lib in "$@"; do
    name=$(basename $lib .so)
    dirs=""
    i=0
    for P in "$P1" "$P2" "$P3"; do
        i=$((i+1))
        d=$O/${name}_p$i
        if [ "$lib" = default ]; then
            timeout -s KILL 90 rocprofv3 --pmc $P -d $d -o pmc --output-format csv -- $B > $d.log 2>&1 || exit 1
        else
            GSR_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $P -d $d -o pmc --output-format csv -- $B > $d.log 2>&1 || exit 1
        fi
        dirs="$dirs $(find $d -name '*counter_collection.csv' -printf '%h\n' | sort -u)"
    done
    python profiles/summarize_pmc.py $O/${name}_summary.csv $dirs
    grep "k_composite<0>" $O/${name}_summary.csv
done
