#!/bin/bash
# BatchNorm UNet after the round-5 fusions (BN sums from the head / pool backward and the first conv's epilogue)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn5
R=$PWD; O=gpurun_out/bn5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_hip_variants.py tests/test_bn_on_load.py tests/test_bwd_fused.py tests/test_hip_model.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/bench_bn_$i.log 2>&1 || { echo "bn bench failed"; tail $O/bench_bn_$i.log; exit 1; }
  echo "bn $i: $(tail -1 $O/bench_bn_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_unet.log 2>&1 || { echo "bench failed"; exit 1; }
echo "unet: $(tail -1 $O/bench_unet.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --model unet-bn --steps 4 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof > $O/prof_summary.txt 2>&1; head -36 $O/prof_summary.txt | cut -c1-120
