# L2 hit rate and wave-state counters of distCUDA2's phase-1 kernel (one counter group per pass).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R="--kernel-include-regex knn_leaf_kernel"
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T $R -d gpurun_out/pk1 -o p --output-format csv -- python tools/knn_time.py > gpurun_out/pk1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -T $R -d gpurun_out/pk2 -o p --output-format csv -- python tools/knn_time.py > gpurun_out/pk2.log 2>&1
