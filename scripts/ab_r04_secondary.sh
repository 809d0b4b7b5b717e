#!/bin/bash
# Same-box A/B of the round-4 tree (_r04: git worktree at d040214, built in
# place) against this tree on the driver's batch-16 secondaries (train_320,
# train_ivd_400): the driver's own window (5 steps, 2 warmup) and a longer one
# (20 steps, 5 warmup), alternating trees.  -> gpurun_out/r6/ab_r04/
set -u
OUT=gpurun_out/r6/ab_r04
mkdir -p $OUT
run() {  # tree name steps warmup args...
  local tree=$1 name=$2 st=$3 wu=$4; shift 4
  (cd $tree && timeout -k 10 200 python -u bench.py --batch 16 --steps $st --warmup $wu "$@" 2>/dev/null | tail -1) \
    | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$tree $name st=$st', round(r.get('pairs_per_s', r.get('value', 0)), 1))" \
    >> $OUT/results.txt || exit 1
}
for rep in 1 2 3; do
  for tree in _r04 .; do
    run $tree train_320 5 2 --only-secondary train --image-size 320 || exit 1
    run $tree train_320 20 5 --only-secondary train --image-size 320 || exit 1
    run $tree train_ivd 5 2 --only-secondary train_ivd --image-size 400 || exit 1
    run $tree train_ivd 20 5 --only-secondary train_ivd --image-size 400 || exit 1
  done
done
cat $OUT/results.txt
