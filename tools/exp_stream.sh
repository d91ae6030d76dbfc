#!/bin/bash
# Streaming wavefront (stream_kernel) on the GPU: smoke, the -m gpu suite, then
# A/B against per-bounce launches (MRT_STREAM=0) on C2 and one GPU's 1/8 share,
# alternating in one call, and a kernel trace of the share.
export TMPDIR=/tmp
B="python3 bench.py --config c2 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh "smoke:90:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "c2_stream_a:100:$B --steps 5" "c2_bounce_a:100:MRT_STREAM=0 $B --steps 5" \
 "s8_stream_a:100:$B --steps 10 --shard-of 8" "s8_bounce_a:100:MRT_STREAM=0 $B --steps 10 --shard-of 8" \
 "c2_stream_b:100:$B --steps 5" "c2_bounce_b:100:MRT_STREAM=0 $B --steps 5" \
 "s8_stream_b:100:$B --steps 10 --shard-of 8" "s8_bounce_b:100:MRT_STREAM=0 $B --steps 10 --shard-of 8" \
 "c1:100:$B --config c1 --steps 5" "c2L5:100:$B --steps 3 --max-path-length 5" \
 "s8trace:200:rocprofv3 --kernel-trace -d gpurun_out/s8s -o run -f csv -- python3 bench.py --config c2 --steps 3 --warmup 1 --shard-of 8 --no-cpu-baseline"
