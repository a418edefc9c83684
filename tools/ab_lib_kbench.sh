set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -m gpu -k "rowblock or pingpong" > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python tools/glds_variant_check.py --base 0 --new --only "L1,L2" > gpurun_out/abk_$v$i.log 2>&1 || exit 1
  echo "$v$i"; grep -v amdgpu gpurun_out/abk_$v$i.log
done; done
