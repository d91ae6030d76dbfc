# r3: C4 memory-pipeline counters; non-temporal radiance stores A/B
B="python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh \
 "probe_c4:600:tools/pmc_probe.sh r3c c4" \
 "c_base:120:$B" "c_nt:120:MRT_LIB=metal-renderer_amd/lib/libmrt_nt.so $B" \
 "c_base2:120:$B" "c_nt2:120:MRT_LIB=metal-renderer_amd/lib/libmrt_nt.so $B"
