#!/bin/bash
# C5 profile session: a kernel trace of the short-window bench (per-launch durations and the gaps between them),
# then PMC passes (SQ issue/wait counters, HBM bytes) of the same command, one counter group per run.
# Usage (GPU box): bash tools/gpu_c5prof.sh <tag> [workload]
set -o pipefail
TAG=${1:-r3}
WL=${2:-c5_adversarial}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $ROOT/bench.py --workload $WL --steps 2 --warmup 1 --cpu-seconds 0 --no-extras --no-parity"
echo "== trace" && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.json" 2> "$OUT/trace.err" && \
echo "== sq a" && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sqa" -o run -- $CMD > "$OUT/sqa.json" 2> "$OUT/sqa.err" && \
echo "== sq b" && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --output-format csv -d "$OUT/sqb" -o run -- $CMD > "$OUT/sqb.json" 2> "$OUT/sqb.err" && \
echo "== fetch" && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $CMD > "$OUT/fetch.json" 2> "$OUT/fetch.err" && \
echo "== write" && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $CMD > "$OUT/write.json" 2> "$OUT/write.err"
rc=$?
echo "exit $rc"
exit $rc
