cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--kernel-include-regex segment_sort_kernel|radix_scatter_kernel"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -T $R -d gpurun_out/pmc1 -o p --output-format csv -- python tools/run_sort.py 3 > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -T $R -d gpurun_out/pmc2 -o p --output-format csv -- python tools/run_sort.py 3 > gpurun_out/pmc2.log 2>&1
