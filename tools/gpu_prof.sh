#!/bin/bash
# C4 profiling session: bench A/B of the P1 geometry, rocprofv3 PMC passes of the default bench (HBM bytes per kernel
# and per step: tools/pmc_passes.sh) and SQ counter passes of one C4 fold per P1 geometry (wave waits, LDS, VMEM).
# Every step is time-limited and the chain stops at the first failure. Usage: bash tools/gpu_prof.sh <tag>
set -o pipefail
TAG=${1:-r3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras"
for p1 in 1 2 0; do
  echo "== c4 bucket_p1=$p1"
  timeout -k 10 240 $B --tune bucket_p1=$p1 > "$OUT/c4_p1_$p1.json" 2> "$OUT/c4_p1_$p1.err" || exit $?
done
echo "== pmc passes" && bash tools/pmc_passes.sh "$TAG" > "$OUT/pmc_passes.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for p1 in 1 2; do
  S=$OUT/sq_p1_$p1
  mkdir -p "$S"
  echo "== sq p1=$p1"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$S/a" -o run -- python3 "$ROOT/tools/fold_once.py" c4_kron26 2 bucket_p1=$p1 > "$S/a.out" 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$S/b" -o run -- python3 "$ROOT/tools/fold_once.py" c4_kron26 2 bucket_p1=$p1 > "$S/b.out" 2>&1 || exit $?
done
cd "$ROOT"
for f in "$OUT"/c4_p1_*.json; do python3 -c "
import json
d=json.load(open('$f'));r=d['roofline']
print('$f'.split('/')[-1], round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', d['parity'],
      {k: round(v['ms_per_step'],3) for k,v in r['kernels'].items() if v['ms_per_step'] > 0.05})"; done
echo "exit 0"
