#!/bin/bash
# Build + an arbitrary list of quick GPU steps selected by env: KBENCH (args), DDP_REHEARSAL, BENCH
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
if [ -n "$PYTEST" ]; then timeout -k 10 600 python -m pytest $PYTEST > gpurun_out/pytest_sel.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sel.log; [ $rc -ne 0 ] && exit $rc; fi
if [ -n "$KBENCH" ]; then timeout -k 10 400 python tools/kbench.py $KBENCH > gpurun_out/kbench.log 2>&1; rc=$?; echo "kbench rc=$rc"; grep -v amdgpu gpurun_out/kbench.log; [ $rc -ne 0 ] && exit $rc; fi
if [ -n "$BENCH" ]; then timeout -k 10 300 python bench.py $BENCH > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc; fi
if [ -n "$BENCH2" ]; then timeout -k 10 300 python bench.py $BENCH2 > gpurun_out/bench2.log 2>&1; rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2.log; [ $rc -ne 0 ] && exit $rc; fi
if [ -n "$PROF" ]; then
  R=$PWD; rm -rf gpurun_out/prof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py $PROF > $R/gpurun_out/prof.log 2>&1); echo "prof rc=$?"
  python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt 2>&1; head -40 gpurun_out/prof_summary.txt
fi
if [ -n "$PMC" ]; then
  # hardware counters (own pass, kernel-trace only): PMC="<counters>" PMC_ARGS="<kbench args>"
  R=$PWD; rm -rf gpurun_out/pmc
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o run -- python3 $R/tools/kbench.py $PMC_ARGS > $R/gpurun_out/pmc.log 2>&1); echo "pmc rc=$?"
  python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1; cat gpurun_out/pmc_summary.txt | head -40
fi
if [ -n "$DDP_REHEARSAL" ]; then
  DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --batch 4 > gpurun_out/ddp_rehearsal.log 2>&1; echo "ddp rehearsal rc=$?"; grep -v amdgpu.ids gpurun_out/ddp_rehearsal.log | tail -4
  DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 train.py -t DDP --synthetic --synthetic-len 16 --img-size 128 -e 1 -b 2 --out-dir /tmp/ddp_train > gpurun_out/ddp_train.log 2>&1; echo "ddp train rc=$?"; grep -v amdgpu.ids gpurun_out/ddp_train.log | tail -4
fi
exit 0
