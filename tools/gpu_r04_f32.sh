#!/bin/bash
# Round-4: fp32 engine -- numerics tests, bench, kernel profile.
set -o pipefail
cd "$(dirname "$0")/.." && R=$(pwd) && export TMPDIR=/tmp && mkdir -p gpurun_out/f32
O=$R/gpurun_out/f32
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_fp32_engine.py tests/test_fp32_backend.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python tools/f32_kbench.py > $O/kbench.txt 2>&1 || { echo "kbench failed"; tail -3 $O/kbench.txt; exit 1; }
tail -1 $O/kbench.txt
timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 6 --warmup 2 > $O/bench.log 2>&1 || { echo "bench failed"; tail -3 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --dtype fp32 --batch 16 --steps 4 --warmup 2 > $O/prof.log 2>&1) || { echo "prof failed"; tail -3 $O/prof.log; exit 1; }
head -8 $O/prof/run_kernel_stats.csv | cut -c1-150
