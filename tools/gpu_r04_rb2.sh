#!/bin/bash
# Two-phase row-block GEMMs (cfg 16/17): fp32-anchored + bitwise tests, per-layer A/B against pp2h,
# end-to-end A/B (DPA_GLDS_RB2=0/1 interleaved).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/rb2
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rowblock.py > gpurun_out/rb2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/rb2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py --batch 256 --paths "" --no-wgrad --gvar 14 65536 15 131072 --reps 7 --only "L2,L3,mid" > gpurun_out/rb2/kbench.log 2>&1 || { echo kbench failed; tail gpurun_out/rb2/kbench.log; exit 1; }
grep -v "n/a" gpurun_out/rb2/kbench.log
for r in 1 2; do
  for v in 0 1; do
    DPA_GLDS_RB2=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > gpurun_out/rb2/bench_rb2_${v}_$r.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/rb2/bench_rb2_${v}_$r.log; exit 1; }
    echo "rb2=$v run $r: $(tail -1 gpurun_out/rb2/bench_rb2_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
