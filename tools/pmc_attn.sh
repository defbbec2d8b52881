# PMC counters of the attention kernels (one pass per counter group; never mixed with traces).
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc/p1 -o p --output-format csv -- python3 tools/bench_attn.py --iters 2 > gpurun_out/pmc/p1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA -d gpurun_out/pmc/p2 -o p --output-format csv -- python3 tools/bench_attn.py --iters 2 > gpurun_out/pmc/p2.log 2>&1
