cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_binning_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/bt.log 2>&1 && bash tools/gpu_queue_ab.sh nodefer
