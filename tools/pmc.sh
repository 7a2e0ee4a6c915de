#!/bin/bash
# rocprofv3 PMC passes of a bench command, one counter pass per run:
#   bash tools/pmc.sh TAG PRESET [-- extra bench.py args]
# PRESET: traffic (FETCH_SIZE, WRITE_SIZE, VALU and LDS counts: the roofline's inputs),
#         stalls (issue / wait / LDS counters of the compositor),
#         lds (LDS instructions, bank conflicts, LDS-busy cycles).
# Env GSR_LIB_PATH selects a variant library.  Writes gpurun_out/TAG/pmc_summary.csv
# (profiles/summarize_pmc.py: FETCH_SIZE doubled per the gfx950 correction).
TAG=$1
PRESET=$2
shift 2
[ "$1" = "--" ] && shift
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline $*"  # the driver's region
case $PRESET in
    traffic) PASSES=("FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT") ;;
    stalls) PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
                    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU") ;;
    lds) PASSES=("SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES") ;;
    *) echo "unknown preset $PRESET"; exit 2 ;;
esac
dirs=""
i=0
for P in "${PASSES[@]}"; do
    i=$((i + 1))
    d=$O/pmc_p$i
    echo "[pmc] pass $i: $P"
    timeout -s KILL 240 rocprofv3 --pmc $P -d $d -o pmc --output-format csv -- $B > $d.log 2>&1 || { echo "[pmc] pass $i FAILED"; exit 1; }
    dirs="$dirs $(find $d -name '*counter_collection.csv' -printf '%h\n' | sort -u)"
done
python profiles/summarize_pmc.py $O/pmc_summary.csv $dirs
