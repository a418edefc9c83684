#!/bin/bash
# Round 5: fp32 engine (packed weights, in-place gradients) -- tests, bench, kernel-trace timeline; the
# deferral-cap test and the fp32 DDP multirank cases.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/f32
R=$PWD; O=gpurun_out/f32
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fp32_engine.py tests/test_defer_cap.py "tests/test_hip_multirank.py::test_ddp_hip_allreduce_equals_mean_of_rank_grads" tests/test_fp32_backend.py > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 10 --warmup 3 > $O/bench_fp32.log 2>&1 || { echo "fp32 bench failed"; tail $O/bench_fp32.log; exit 1; }
tail -1 $O/bench_fp32.log | cut -c1-300
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --dtype fp32 --batch 16 --steps 4 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof --timeline > $O/prof_summary.txt 2>&1; head -40 $O/prof_summary.txt
