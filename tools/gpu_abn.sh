#!/bin/bash
# Interleaved A/B/n of library builds on one box (GELLY_CC_LIB; "-" = the in-tree build), two rounds each, bench only.
# A step that fails ends the session. Usage (GPU box):
#   bash tools/gpu_abn.sh <tag> "<bench args>" name=lib.so[@k=v,...] [name=lib.so[@k=v,...] ...]
set -o pipefail
TAG=$1
ARGS=$2
shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
B="python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras $ARGS"
for r in 1 2; do
  for nl in "$@"; do
    name=${nl%%=*}
    lib=${nl#*=}
    tune=""
    case $lib in *@*) tune="--tune ${lib#*@}"; lib=${lib%%@*} ;; esac
    echo "== $name round $r"
    if [ "$lib" = "-" ]; then timeout -k 10 240 $B $tune > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit $?
    else GELLY_CC_LIB=$ROOT/$lib timeout -k 10 240 $B $tune > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err" || exit $?; fi
  done
done
for f in "$OUT"/*_[12].json; do python3 -c "
import json
d=json.load(open('$f'));r=d.get('roofline',{})
print('$f'.split('/')[-1], round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', d.get('parity'),
      {k: round(v['ms_per_step'],3) for k,v in r.get('kernels',{}).items() if v['ms_per_step'] > 0.02})"; done
exit 0
