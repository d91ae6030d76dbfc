#!/bin/bash
# Accumulate pass overlapped with the next kernel (MRT_OVERLAP, default on):
# the -m gpu suite, then A/B against MRT_OVERLAP=0 on C2, the 1/8 share and C4,
# alternating in one call.
export TMPDIR=/tmp
B="python3 bench.py --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh "smoke:90:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "c2_ov_a:100:$B --config c2 --steps 5" "c2_seq_a:100:MRT_OVERLAP=0 $B --config c2 --steps 5" \
 "s8_ov_a:100:$B --config c2 --steps 10 --shard-of 8" "s8_seq_a:100:MRT_OVERLAP=0 $B --config c2 --steps 10 --shard-of 8" \
 "c2_ov_b:100:$B --config c2 --steps 5" "c2_seq_b:100:MRT_OVERLAP=0 $B --config c2 --steps 5" \
 "s8_ov_b:100:$B --config c2 --steps 10 --shard-of 8" "s8_seq_b:100:MRT_OVERLAP=0 $B --config c2 --steps 10 --shard-of 8" \
 "c4_ov:200:$B --config c4 --steps 3" "c4_seq:200:MRT_OVERLAP=0 $B --config c4 --steps 3" \
 "s8trace:200:rocprofv3 --kernel-trace -d gpurun_out/s8o -o run -f csv -- python3 bench.py --config c2 --steps 3 --warmup 1 --shard-of 8 --no-cpu-baseline"
