#!/bin/bash
# Chained wavefront (chain_kernel) on the GPU: smoke, the -m gpu suite, then
# A/B against per-bounce launches (MRT_CHAIN=0) on C2 and one GPU's 1/8 share,
# alternating in one call; then the C3g partition A/B (tools/exp_classes.sh).
export TMPDIR=/tmp
B="python3 bench.py --config c2 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh "smoke:90:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "c2_chain_a:100:$B --steps 5" "c2_bounce_a:100:MRT_CHAIN=0 $B --steps 5" \
 "s8_chain_a:100:$B --steps 10 --shard-of 8" "s8_bounce_a:100:MRT_CHAIN=0 $B --steps 10 --shard-of 8" \
 "c2_chain_b:100:$B --steps 5" "c2_bounce_b:100:MRT_CHAIN=0 $B --steps 5" \
 "s8_chain_b:100:$B --steps 10 --shard-of 8" "s8_bounce_b:100:MRT_CHAIN=0 $B --steps 10 --shard-of 8" \
 "s8trace:200:rocprofv3 --kernel-trace -d gpurun_out/s8c -o run -f csv -- python3 bench.py --config c2 --steps 3 --warmup 1 --shard-of 8 --no-cpu-baseline" \
 && bash tools/exp_classes.sh
