#!/bin/bash
# first-level backward chunk count: kernel-trace wall per step, plain UNet b256, default (4) vs 8, twice
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/chunks
R=$PWD; O=gpurun_out/chunks
prof() {
  local tag=$1; shift
  rm -rf $O/$tag
  (cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$tag -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/$tag.log 2>&1) || { echo "$tag prof failed"; exit 1; }
  python tools/prof_summary.py $O/$tag > $O/sum_$tag.txt 2>&1
  echo "== $tag: $(grep 'total kernel time' $O/sum_$tag.txt) | $(grep 'last step' $O/sum_$tag.txt | cut -c1-40) | bench $(tail -1 $O/$tag.log | cut -c80-110)"
}
prof c4a DPA_X=0
prof c8a DPA_ENC0_CHUNKS=8
prof c4b DPA_X=0
prof c8b DPA_ENC0_CHUNKS=8
