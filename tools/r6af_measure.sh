# r6af: camera-ray grab size for the per-frame cadence (c2i: 2 M paths per
# launch, ~405 per wave) and batched C2: 192 against the default 128 (64: r6af_c2i in profiles/r6/ab/grab_size_c2i.log)
set -o pipefail
mkdir -p gpurun_out
bash tools/lib_sweep.sh "--steps 20 --no-image-check" c2i -- libmrt.so libmrt_fg192.so libmrt.so libmrt_fg192.so > gpurun_out/r6af_c2i.log 2>&1 || exit $?
cat gpurun_out/r6af_c2i.log
bash tools/lib_sweep.sh "--sustain 0" c2 -- libmrt.so libmrt_fg192.so > gpurun_out/r6af_c2.log 2>&1
rc=$?; cat gpurun_out/r6af_c2.log; exit $rc
