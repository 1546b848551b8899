# Binning-primitive GPU tests, per-kernel sort timing, then the bench line.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_binning_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bin.log 2>&1 && \
timeout -k 10 120 python tools/seg_time.py >> gpurun_out/bin.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
