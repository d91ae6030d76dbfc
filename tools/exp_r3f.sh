# r3: kernel traces of one GPU's 1/8 tile share of C2 vs the whole frame
export TMPDIR=/tmp
B="python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
 "f_s8:120:$B --shard-of 8" "f_full:120:$B" \
 "f_tr_s8:200:rocprofv3 --kernel-trace --stats -d gpurun_out/tr_s8 -o run -f csv -- $B --shard-of 8" \
 "f_tr_full:200:rocprofv3 --kernel-trace --stats -d gpurun_out/tr_full -o run -f csv -- $B"
PASSES=valu timeout -k 10 200 bash tools/pmc_probe.sh r3f c4 > gpurun_out/probe_valu_c4.txt 2>&1 && cat gpurun_out/probe_valu_c4.txt && PASSES=valu timeout -k 10 200 bash tools/pmc_probe.sh r3f c2 > gpurun_out/probe_valu_c2.txt 2>&1 && cat gpurun_out/probe_valu_c2.txt
