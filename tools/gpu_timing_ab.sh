# In-bench per-kernel timing (fence-free HIP events) against rocprofv3 on the same bench command, then
# the unskewed bench view product vs the variants named on the command line (tools/gpu_common_ab.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
B="--steps 50 --warmup 5 --knn-steps 1 --no-cpu-baseline --no-config5 --no-skewed --no-adam --no-exchange"
timeout -k 10 300 python bench.py $B > gpurun_out/tbench.json 2> gpurun_out/tbench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/tprof -o kt --output-format csv -- python bench.py $B > gpurun_out/tprof.log 2>&1 && \
bash tools/gpu_common_ab.sh "$@"
echo rc=$?
