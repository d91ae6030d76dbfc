# r6m: where the phase-4 last-bounce query loses: MRT_DEBUG=64 (no last-bounce
# query) on the new and the previous library
set -o pipefail
mkdir -p gpurun_out
MRT_DIAG=1 MRT_DEBUG=64 bash tools/lib_sweep.sh "--sustain 0" c2 -- libmrt.so libmrt_prev.so libmrt.so libmrt_prev.so > gpurun_out/r6m_ab.log 2>&1; cat gpurun_out/r6m_ab.log
