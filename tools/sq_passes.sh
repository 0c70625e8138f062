#!/bin/bash
# SQ counter passes over one workload's fold (tools/fold_once.py), one rocprofv3 --pmc run per pass (each block's
# counter limits respected). Usage on the GPU box: bash tools/sq_passes.sh <tag> [workload] [reps]
set -o pipefail
TAG=$1; WL=${2:-c4_kron26}; REPS=${3:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD"
  "SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAVES SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/fold_once.py" "$WL" "$REPS" > "$OUT/p$i.out" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.out"; exit 1; }
done
python3 "$ROOT/tools/sq_summary.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
