# r6y: the c2i profile again without the bench's image-check leg (its batched
# launches had joined the single-frame launches' averages), then the c2i line
set -o pipefail
mkdir -p gpurun_out
LPS=64 STEPS=6 bash tools/profile.sh r6a c2i --no-image-check || exit $?
timeout -k 10 300 python3 bench.py --config c2i --steps 80 --warmup 5 > gpurun_out/r6y_cfg_c2i.json 2> gpurun_out/r6y_cfg_c2i.log
rc=$?; tail -c 400 gpurun_out/r6y_cfg_c2i.json; exit $rc
