#!/bin/bash
# fp32 engine A/B on one GPU: the engine's tests, the per-layer kernel bench, then bench.py --dtype fp32 b16
# alternating ENV unset / ENV=VAL (default 1).   usage: tools/gpu_r05_ab.sh ENV[=VAL] "f32_kbench args" [test file]
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
O=gpurun_out/ab
ENV=${1%%=*}; VAL=1; [[ $1 == *=* ]] && VAL=${1#*=}; KB=$2; T=${3:-tests/test_fp32_engine.py}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/f32_kbench.py --batch 16 --img 512 $KB > $O/kbench.txt 2>&1 || { echo kbench failed; tail $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export $ENV=$VAL; else unset $ENV; fi
  timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 10 --warmup 3 > $O/bench_$v.log 2>&1 || { echo bench failed; exit 1; }
  echo "$ENV=$v $(tail -1 $O/bench_$v.log | cut -c80-140)"
done
