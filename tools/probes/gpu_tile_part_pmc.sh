# The one-pass tile-partition probe under rocprofv3: kernel trace, then FETCH_SIZE and WRITE_SIZE passes
# (one counter per pass), for profiles/r05_tile_part_ab.md.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R="--kernel-include-regex tp_|radix_|segment_sort"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T $R -d gpurun_out/tp_kt -o kt --output-format csv -- python tools/probes/tile_part.py > gpurun_out/tp_kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T $R -d gpurun_out/tp_fetch -o fetch --output-format csv -- python tools/probes/tile_part.py > gpurun_out/tp_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T $R -d gpurun_out/tp_write -o write --output-format csv -- python tools/probes/tile_part.py > gpurun_out/tp_write.log 2>&1
echo rc=$?
