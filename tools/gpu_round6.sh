# Round-6 GPU session: the full GPU suite and smoke, each timed (profiles/r06_evidence.md), the driver's
# bench, its rocprofv3 kernel trace and PMC passes, and the distCUDA2 VALU-issue PMC pass.  Every GPU
# step has its own time limit; steps chained by &&.  gpurun_out/sources.sha256: the kernel sources'
# hash (bench.sources_sha256); gpurun_out/maps_gputest.txt: the in-tree .so files the test process mapped.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
python -c "import bench; print(bench.sources_sha256())" > gpurun_out/sources.sha256 && \
ls -l --time-style=+%s.%N hidegs_amd/libhidegs.so hidegs_amd/csrc/* include/hidegs.h > gpurun_out/mtimes.txt && \
date +%s.%N > gpurun_out/t_gputest0 && \
HIDEGS_MAPS_OUT=gpurun_out/maps_gputest.txt timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --durations=10 -s > gpurun_out/gputest.log 2>&1 && \
date +%s.%N > gpurun_out/t_gputest1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
date +%s.%N > gpurun_out/t_smoke1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_kt -o kt --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-config5 > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d gpurun_out/prof_fetch -o fetch --output-format csv -- python bench.py --steps 5 --warmup 1 --knn-steps 1 --no-cpu-baseline --no-exchange --no-config5 --no-adam > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d gpurun_out/prof_write -o write --output-format csv -- python bench.py --steps 5 --warmup 1 --knn-steps 1 --no-cpu-baseline --no-exchange --no-config5 --no-adam > gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM SQ_BUSY_CYCLES -T -d gpurun_out/prof_knn -o knn --output-format csv -- python tools/run_knn.py 2 > gpurun_out/prof_knn.log 2>&1
echo rc=$?
