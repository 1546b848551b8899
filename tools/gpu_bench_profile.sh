cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_kt -o kt --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof_fetch -o fetch --output-format csv -- python bench.py --steps 5 --warmup 1 --knn-steps 1 --no-cpu-baseline --no-exchange > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof_write -o write --output-format csv -- python bench.py --steps 5 --warmup 1 --knn-steps 1 --no-cpu-baseline --no-exchange > gpurun_out/prof_write.log 2>&1
