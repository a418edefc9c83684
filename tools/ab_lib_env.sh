set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for i in 1 2; do for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/ab_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/ab_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python bench.py --model unet-xl --img 1024 --batch 16 --steps 5 --warmup 2 --parallelism mp --stages 8 --microbatches 4 > gpurun_out/abxl_$v$i.log 2>&1 || exit 1
  echo "xl8mb4 $v $(tail -1 gpurun_out/abxl_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
