#!/bin/bash
# BN re-measure after issuing the pool backward's y loads up front; UNet-XL kernel summary
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn6
R=$PWD; O=gpurun_out/bn6
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_hip_variants.py tests/test_bn_on_load.py tests/test_bwd_fused.py tests/test_hip_model.py tests/test_split_blocks.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/bench_bn_$i.log 2>&1 || { echo "bn bench failed"; tail $O/bench_bn_$i.log; exit 1; }
  echo "bn $i: $(tail -1 $O/bench_bn_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
rm -rf $O/prof $O/profxl
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --model unet-bn --steps 4 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof > $O/prof_summary.txt 2>&1; grep -E "pool_bwd|bn_partial|total kernel|last step" $O/prof_summary.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/profxl -o run -- python3 $R/bench.py --model unet-xl --img 1024 --batch 16 --steps 4 --warmup 2 > $R/$O/profxl.log 2>&1) || { echo "xl prof failed"; exit 1; }
python tools/prof_summary.py $O/profxl --timeline > $O/profxl_summary.txt 2>&1; head -34 $O/profxl_summary.txt | cut -c1-120
