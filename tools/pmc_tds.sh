#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r5_s11
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES"
i=0
dirs=""
for P in "$P1" "$P2"; do
  i=$((i+1)); d=$O/pmc_p$i
  echo "[pmc] pass $i"
  timeout -s KILL 200 rocprofv3 --pmc $P -d $d -o pmc --output-format csv -- python tools/tds_probe.py --frames 10 0 > $d.log 2>&1 || { echo "pass $i failed"; exit 1; }
  dirs="$dirs $(find $d -name '*counter_collection.csv' -printf '%h\n' | sort -u)"
done
python profiles/summarize_pmc.py $O/pmc_summary.csv $dirs
