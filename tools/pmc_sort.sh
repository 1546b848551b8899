# PMC passes (one counter group per rocprofv3 run) over the binning sort's kernels; tools/pmc_table.py reads them.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--kernel-include-regex segment_sort_kernel|radix_scatter_kernel|radix_hist_kernel|identify_ranges_kernel"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -T $R -d gpurun_out/pmc1 -o p --output-format csv -- python tools/run_sort.py 3 > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -T $R -d gpurun_out/pmc2 -o p --output-format csv -- python tools/run_sort.py 3 > gpurun_out/pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -T $R -d gpurun_out/pmc3 -o p --output-format csv -- python tools/run_sort.py 3 > gpurun_out/pmc3.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -T $R -d gpurun_out/pmc4 -o p --output-format csv -- python tools/run_sort.py 3 > gpurun_out/pmc4.log 2>&1
