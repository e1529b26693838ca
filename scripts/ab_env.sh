#!/bin/bash
# A/B of one environment switch on the bench, alternating on one box:
#   bash scripts/ab_env.sh VAR "v1 v2 ..." REPS [bench args]
# prints per value and repetition the V-cycles/s and the roofline kernel's time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VAR=$1; VALS=$2; REPS=$3; shift 3
for i in $(seq 1 "$REPS"); do
  for v in $VALS; do
    out=gpurun_out/ab_${VAR}_${v}_$i.json
    env "$VAR=$v" timeout -k 10 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-general --no-abi "$@" \
        > "$out" 2> "${out%.json}.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], 'rep', sys.argv[4], d['value'], 'V-cycles/s', 'roofline', r['ms_per_launch'], 'ms', r['frac'])" "$out" "$VAR" "$v" "$i"
  done
done
