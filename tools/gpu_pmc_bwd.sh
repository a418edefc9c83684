#!/bin/bash
# SQ counter pass over the fused-backward kernel benchmark (tools/kbench_bwd.py --only-fused).
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_bwd
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
   SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace \
   --output-format csv -d "$R/gpurun_out/pmc_bwd" -o run -- python3 "$R/tools/kbench_bwd.py" --batch 128 --iters 2 --only-fused \
   > "$R/gpurun_out/pmc_bwd.log" 2>&1) || { echo "pmc pass failed"; tail -5 gpurun_out/pmc_bwd.log; exit 1; }
python tools/pmc_report.py gpurun_out/pmc_bwd > gpurun_out/pmc_bwd_report.txt 2>&1; grep -E "kernel|bwd_stream|wgrad_reduce" gpurun_out/pmc_bwd_report.txt | head -20
