tools/gpu_run.sh \
 "counters:60:rocprofv3 --list-avail" \
 "c2:300:python3 bench.py --config c2 --steps 10 --warmup 2" \
 "c4:400:python3 bench.py --config c4 --steps 3 --warmup 1" \
 "c4_base:120:python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "c4_mode0:120:MRT_MODE=0 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "c4_mode0_s12:120:MRT_MODE=0 MRT_STACK=12 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "c4_mode0_s16:120:MRT_MODE=0 MRT_STACK=16 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "c4_grid4:120:MRT_GRID=1024 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "c4_base2:120:python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "prof_c4:700:tools/profile.sh r3a c4"
