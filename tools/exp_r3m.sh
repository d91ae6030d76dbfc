# r3: read-back on the main stream (3 streams per renderer); pipelined share vs one stream;
# GPU_MAX_HW_QUEUES=8 (allowed <= 32) as a check of the queue-sharing explanation
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --config c2 --shard-of 8"
tools/gpu_run.sh "m_a1:100:$B" "m_c1:100:MRT_INFLIGHT=1 $B" "m_q1:100:GPU_MAX_HW_QUEUES=8 $B" \
 "m_a2:100:$B" "m_c2:100:MRT_INFLIGHT=1 $B" "m_q2:100:GPU_MAX_HW_QUEUES=8 $B" \
 "m_g2:200:python3 bench.py --gpus 2 --exchange-backend host --check-image --steps 4 --warmup 1 --no-cpu-baseline"
