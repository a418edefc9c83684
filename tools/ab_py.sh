#!/bin/bash
# Same-box A/B of a Python-side change: build/ab/<file>_old.py is swapped into a copy of the tree
# (AB_FILE = its path in the package), both benches run interleaved.  bash tools/ab_py.sh
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
F=${AB_FILE:-distributedpytorch_amd/models/hip_unet.py}
rm -rf /tmp/ab_old && cp -r "$PWD" /tmp/ab_old && cp build/ab/$(basename "$F" .py)_old.py /tmp/ab_old/$F
for i in 1 2; do for v in old new; do
  d=$PWD; [ $v = old ] && d=/tmp/ab_old
  (cd $d && timeout -k 10 200 python bench.py --steps 12 --warmup 4 ${AB_ARGS:-}) > gpurun_out/abpy_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/abpy_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
