# r6t: stream kernel occupancy / grid at the r6q library: 5 / 7 waves of
# registers (w5, w7) and 0 / 2 block slots left free by the persistent grid
# (sp0, sp2; default 1), alternating on C2 and L=5
set -o pipefail
mkdir -p gpurun_out
bash tools/lib_sweep.sh "--sustain 0" c2 c2l5 -- libmrt.so libmrt_fw5.so libmrt_fw7.so libmrt_fsp0.so libmrt_fsp2.so libmrt.so libmrt_fw5.so libmrt_fsp0.so libmrt_fsp2.so > gpurun_out/r6t_ab.log 2>&1
rc=$?; cat gpurun_out/r6t_ab.log; exit $rc
