#!/bin/bash
# Round-4: fp32 kernel-library A/B (tools/f32_kbench.py with DPA_LIB_PATH = each library under build/ab).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/f32ab
for v in ${AB_VARIANTS:-base bk16 base}; do
  DPA_LIB_PATH=$PWD/build/ab/libdpa_hip_$v.so timeout -k 10 200 python tools/f32_kbench.py > gpurun_out/f32ab/kbench_$v.txt 2>&1 || { echo "$v failed"; tail -3 gpurun_out/f32ab/kbench_$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/f32ab/kbench_$v.txt)"
done
