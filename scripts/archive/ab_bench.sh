#!/usr/bin/env bash
# A/B: headline bench of ./ab_old (a git worktree of an older commit) vs this tree, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for t in old new; do
    d=.; [ $t = old ] && d=ab_old
    (cd $d && timeout -k 10 300 python bench.py --ref-events 0 --steps 10 --warmup 2) > gpurun_out/ab/$t-$i.json 2>gpurun_out/ab/$t-$i.err || { echo "$t $i failed"; tail -5 gpurun_out/ab/$t-$i.err; exit 1; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab/$t-$i.json').read().strip().splitlines()[-1]);print('$t',$i,d['value'],d['cpu_util_rank0'])"
  done
done
