#!/bin/bash
# rocprofv3 kernel stats of the 1-GPU 2-stage GPipe rehearsal (bench.py --parallelism mp).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_mp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mp -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 --batch ${BATCH:-256} --parallelism mp --stages ${STAGES:-2} --microbatches ${MB:-8} \
  ${EXTRA:-} > $R/gpurun_out/prof_mp.log 2>&1; echo "prof rc=$?"
