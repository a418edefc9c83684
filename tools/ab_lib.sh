set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
[ -z "$SKIP_TESTS" ] && { timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_hip_model.py tests/test_hip_variants.py -m gpu > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc; }
for i in 1 2; do for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python bench.py --steps 12 --warmup 4 ${AB_ARGS:-} > gpurun_out/ab_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/ab_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
