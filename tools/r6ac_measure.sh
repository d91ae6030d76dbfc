# r6ac: unit-triangle (Woop) leaf tests in the all-in-LDS fast kernels
# (libmrt_fwoop.so, MRT_WOOP=1; A/B) against Moller-Trumbore: C2 / L=5
# alternating, then one C2 line of the variant with the CPU oracle's image
# parity (fast gate)
set -o pipefail
mkdir -p gpurun_out
bash tools/lib_sweep.sh "--sustain 0" c2 c2l5 -- libmrt.so libmrt_fwoop.so libmrt.so libmrt_fwoop.so > gpurun_out/r6ac_ab.log 2>&1 || exit $?
cat gpurun_out/r6ac_ab.log
MRT_LIB=metal-renderer_amd/lib/libmrt_fwoop.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --sustain 0 > gpurun_out/r6ac_woop_c2.json 2> gpurun_out/r6ac_woop_c2.log
rc=$?; python3 -c "import json; d=json.loads(open('gpurun_out/r6ac_woop_c2.json').read().strip().splitlines()[-1]); print(d['value'], d.get('parity'))"; exit $rc
