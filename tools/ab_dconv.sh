# Same-box A/B of the fused first-level forward (csrc/dconv_fwd.hip) against the two streaming kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dconv_fwd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dc.log 2>&1; tail -1 gpurun_out/pytest_dc.log
for i in 1 2; do for E in "DPA_FUSED_DCONV1=0" "DPA_FUSED_DCONV1=1 DPA_DCONV1_BP=64" "DPA_FUSED_DCONV1=1 DPA_DCONV1_BP=128"; do
  env $E timeout -k 10 300 python bench.py --steps 12 --warmup 4 > gpurun_out/ab3.log 2>&1 || exit 1
  echo "$E $(tail -1 gpurun_out/ab3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
