cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export HIDEGS_KNN_ABLATE=2
R="--kernel-include-regex knn_leaf_kernel"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_VMEM -T $R -d gpurun_out/pmck3 -o p --output-format csv -- python tools/run_knn_plane.py > gpurun_out/pmck3.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS -T $R -d gpurun_out/pmck4 -o p --output-format csv -- python tools/run_knn_plane.py > gpurun_out/pmck4.log 2>&1
