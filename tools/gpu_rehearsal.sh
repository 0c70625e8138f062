#!/bin/bash
# Multi-rank rehearsal on ONE GPU (every rank on cuda:0; never a measurement): C4 x 2 / x 4, C3 x 2 (one window and
# 1M-edge windows), C5 x 2 (256 windows: the delta merge) through bench.py
# under torch.distributed.run — the production merge loop (gcc_forest_group_merge) with its collectives through the
# shared-memory stand-in for librccl (tests/cpp/shm_rccl.cpp, GELLY_RCCL_LIB); gloo only bootstraps the id and runs
# the bench's barriers. The JSON line is the last line. A failing step ends the session.
# Usage (GPU box): bash tools/gpu_rehearsal.sh
set -o pipefail
O=${O:-gpurun_out/rehearsal}; mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
B="bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-extras"
export GELLY_SHARE_GPU=1 GELLY_DIST_BACKEND=gloo GELLY_RCCL_LIB=$PWD/tests/cpp/build/libshm_rccl.so
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29511 $B --gpus 2 > $O/c4_2.json 2> $O/c4_2.err && echo c4x2 ok && \
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29512 $B --gpus 4 > $O/c4_4.json 2> $O/c4_4.err && echo c4x4 ok && \
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29513 $B --gpus 2 --workload c3_gnm24 > $O/c3_2.json 2> $O/c3_2.err && echo c3x2 ok && \
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29514 $B --gpus 2 --workload c3_gnm24 --window-edges 1048576 > $O/c3w1M_2.json 2> $O/c3w1M_2.err && echo c3w1Mx2 ok && \
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29515 $B --gpus 2 --workload c5_adversarial > $O/c5_2.json 2> $O/c5_2.err && echo c5x2 ok
rc=$?
for f in $O/*.json; do tail -1 $f | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); m=d.get('merge') or {}; print('$f', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', d.get('parity'), d.get('n_gpus'), d.get('scaling'), 'merge', m.get('kind_last_window'), m.get('message_bytes'), round(m.get('ms_per_window') or 0, 4))" || tail -5 ${f%.json}.err; done
exit $rc
