#!/bin/bash
# Same-box A/B of the current tree against an older tree exported (with its built library) under
# build/ab/oldtree: bench.py from each, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
R=$PWD
for i in 1 2 3; do for v in old new; do
  d=$R; [ $v = old ] && d=$R/build/ab/oldtree
  (cd $d && timeout -k 10 300 python bench.py --steps 12 --warmup 4 ${AB_ARGS:-}) > gpurun_out/abtree_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/abtree_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
