# r3: path kernel re-tune with both slacks: interior slack 8/16, 6 waves/SIMD, service 20, 12-entry LDS stack
export TMPDIR=/tmp
tools/gpu_run.sh \
 "n_sweep:900:bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 c3g -- libmrt.so libmrt_ps8.so libmrt_ps16.so libmrt_w6.so libmrt_sv20.so libmrt.so" \
 "n_stack12:200:MRT_STACK=12 bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 -- libmrt.so"
tools/gpu_run.sh "n_ring:200:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'ring or golden_compare'" \
 "n_fetch:120:timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_probe -o run -f csv -- tools/fetch_probe"
