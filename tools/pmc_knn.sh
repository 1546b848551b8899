cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--kernel-include-regex knn_leaf_kernel"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM -T $R -d gpurun_out/pmck1 -o p --output-format csv -- python tools/run_knn.py 2 > gpurun_out/pmck1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -T $R -d gpurun_out/pmck2 -o p --output-format csv -- python tools/run_knn.py 2 > gpurun_out/pmck2.log 2>&1
