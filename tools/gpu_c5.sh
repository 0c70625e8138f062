#!/bin/bash
# Short-window session: parity of the incremental compress (windowed + parity tests), the C5 / C2 x16 / C3 benches
# of the in-tree library against saved builds (GELLY_CC_LIB), then SQ counter passes of one C4 fold (P1 / P2 bounds).
# Every GPU step is time-limited; the chain stops at the first failure.
# Usage (GPU box): [SQ=1] bash tools/gpu_c5.sh <tag> <old .so> [variant .so]
set -o pipefail
TAG=${1:-r3}
OLD=$2
VAR=$3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "== windowed + parity tests"
timeout -k 10 700 python -u -m pytest tests/test_gpu_windows.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
trc=$?
tail -3 "$OUT/tests.log"
if [ $trc -ne 0 ]; then grep -E "FAILED|Error|inc_check" "$OUT/tests.log" | head -20; exit $trc; fi
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras"
run() {  # name, lib ("" = in-tree), bench args...
  local name=$1 lib=$2; shift 2
  echo "== $name"
  if [ -n "$lib" ]; then GELLY_CC_LIB=$ROOT/$lib timeout -k 10 240 $B "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  else timeout -k 10 240 $B "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; fi
}
run c5_new "" --workload c5_adversarial || exit $?
run c5_old "$OLD" --workload c5_adversarial || exit $?
if [ -n "$VAR" ]; then run c5_var "$VAR" --workload c5_adversarial || exit $?; fi
run c5_new_b "" --workload c5_adversarial || exit $?
run c2w16_new "" --workload c2_rmat20 --window-edges 1048576 || exit $?
run c2w16_old "$OLD" --workload c2_rmat20 --window-edges 1048576 || exit $?
run c3_new "" --workload c3_gnm24 || exit $?
run c3_old "$OLD" --workload c3_gnm24 || exit $?
run c4_new "" || exit $?
for f in "$OUT"/c*.json; do python3 -c "
import json
d=json.load(open('$f'));r=d.get('roofline',{})
print('$f'.split('/')[-1], round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms', d.get('parity'),
      {k: round(v['ms_per_step'],3) for k,v in r.get('kernels',{}).items()})"; done
[ "$SQ" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
S=$OUT/sq
mkdir -p "$S"
echo "== sq passes (c4 fold)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$S/a" -o run -- python3 "$ROOT/tools/fold_once.py" c4_kron26 2 > "$S/a.out" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$S/b" -o run -- python3 "$ROOT/tools/fold_once.py" c4_kron26 2 > "$S/b.out" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$S/c" -o run -- python3 "$ROOT/tools/fold_once.py" c4_kron26 2 > "$S/c.out" 2>&1
rc=$?
echo "exit $rc"
exit $rc
