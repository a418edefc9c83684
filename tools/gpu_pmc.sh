#!/bin/bash
# Three rocprofv3 counter passes (SQ+GRBM, FETCH_SIZE, WRITE_SIZE) over a short bench.py run, each in
# its own process with --kernel-trace only, then tools/pmc_report.py.  Usage: bash tools/gpu_pmc.sh [bench args]
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
ARGS=${*:-"--batch 32 --steps 2 --warmup 1"}
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write
run() {  # $1 = out dir, rest = counters
  local out=$1; shift
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$R/$out" -o run \
     -- python3 "$R/bench.py" $ARGS > "$R/$out.log" 2>&1)
}
run gpurun_out/pmc_sq SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || { echo "sq pass failed"; exit 1; }
run gpurun_out/pmc_fetch FETCH_SIZE || { echo "fetch pass failed"; exit 1; }
run gpurun_out/pmc_write WRITE_SIZE || { echo "write pass failed"; exit 1; }
python tools/pmc_report.py gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_report.txt
cat gpurun_out/pmc_report.txt
