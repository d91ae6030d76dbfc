#!/bin/bash
# A/B of the survivor partition on C3g (all four BSDFs) with the lane-refill
# wavefront: 2 classes (diffuse vs the rest) vs 4 (one per BSDF), alternating
# in one call, plus the path kernel (the product default) for reference.
export TMPDIR=/tmp
B="python3 bench.py --config c3g --steps 2 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh "test4:300:python -u -m pytest tests/test_gpu_configs.py -x -q -k four_class --timeout 240 --timeout-method thread" \
 "w2a:200:MRT_KERNEL=wave MRT_CLASSES=2 $B" "w4a:200:MRT_KERNEL=wave MRT_CLASSES=4 $B" \
 "w2b:200:MRT_KERNEL=wave MRT_CLASSES=2 $B" "w4b:200:MRT_KERNEL=wave MRT_CLASSES=4 $B" \
 "path:200:$B"
