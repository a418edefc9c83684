#!/bin/bash
# Does stream/queue concurrency on one MI355X pay for this workload?  Two bench processes at half the
# batch running at the same time vs one at the full batch (sum of their img/s vs the single rate).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/cc_single.log 2>&1 || exit 1
echo "single b256: $(tail -1 gpurun_out/cc_single.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
timeout -k 10 200 python bench.py --steps 40 --warmup 4 --batch 128 > gpurun_out/cc_a.log 2>&1 &
pa=$!
timeout -k 10 200 python bench.py --steps 40 --warmup 4 --batch 128 > gpurun_out/cc_b.log 2>&1 &
pb=$!
wait $pa; ra=$?; wait $pb; rb=$?
[ $ra -ne 0 -o $rb -ne 0 ] && { echo "pair failed $ra $rb"; exit 1; }
for f in a b; do echo "pair $f b128: $(tail -1 gpurun_out/cc_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
timeout -k 10 200 python bench.py --steps 12 --warmup 4 --batch 128 > gpurun_out/cc_half.log 2>&1 || exit 1
echo "single b128: $(tail -1 gpurun_out/cc_half.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
