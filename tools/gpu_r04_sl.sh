#!/bin/bash
# Round-4: slice-staged 128-channel default -- kernel tests, bench, kernel-trace profile.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/sl2
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rowblock.py tests/test_hip_kernels.py tests/test_hip_model.py tests/test_bn_on_load.py tests/test_bwd_fused.py > gpurun_out/sl2/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sl2/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/sl2/bench_$i.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/sl2/bench_$i.log; exit 1; }
tail -1 gpurun_out/sl2/bench_$i.log | cut -c80-200
done
timeout -k 10 300 python bench.py --model unet-bn > gpurun_out/sl2/bench_bn.log 2>&1 || { echo "bench bn failed"; exit 1; }
tail -1 gpurun_out/sl2/bench_bn.log | cut -c80-200
rm -rf gpurun_out/sl2/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sl2/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/sl2/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py gpurun_out/sl2/prof > gpurun_out/sl2/prof_summary.txt 2>&1; head -36 gpurun_out/sl2/prof_summary.txt
