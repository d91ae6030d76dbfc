# r3: path kernel re-tune with both slacks (variants rebuilt at the current ABI); LDS stack 12/16;
# display ring GPU test; FETCH_SIZE gather calibration
export TMPDIR=/tmp
tools/gpu_run.sh "o_ring:200:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'ring or golden_compare'" \
 "o_fetch:120:timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_probe -o run -f csv -- tools/fetch_probe" \
 "o_sweep:900:bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 -- libmrt.so libmrt_ps8.so libmrt_ps16.so libmrt_w6.so" \
 "o_st12:200:MRT_STACK=12 bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 c3g -- libmrt.so" \
 "o_st16:200:MRT_STACK=16 bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 c3g -- libmrt.so" \
 "o_st8:200:bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 c3g -- libmrt.so"
