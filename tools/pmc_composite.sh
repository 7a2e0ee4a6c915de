export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_VMEM -d gpurun_out/pmc5_a -o pmc --output-format csv -- $B > gpurun_out/pmc5_a.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d gpurun_out/pmc5_b -o pmc --output-format csv -- $B > gpurun_out/pmc5_b.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_IFETCH SQC_ICACHE_MISSES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/pmc5_c -o pmc --output-format csv -- $B > gpurun_out/pmc5_c.log 2>&1
