#!/bin/bash
# Host-side AddressSanitizer run of the HIP kernel library (SURVEY §5 "race detection / sanitizers").
# GPU ASan / xnack+ builds are not available on the MI355X pool, so only the HOST code of every
# csrc/*.hip translation unit (argument validation, tiling arithmetic, launch plumbing) is
# instrumented: `-Xarch_host -fsanitize=address` leaves the gfx950 device code unchanged.  The
# instrumented library is loaded through DPA_LIB_PATH by the CPU contract tests, which call every
# launcher's validation path without launching anything, under the ASan runtime (LD_PRELOAD).
#   bash tools/asan_host.sh            # build build/asan/libdpa_hip_asan.so + run tests/test_host_contracts.py
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=build/asan
mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
TORCH_LIB=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
objs=()
for src in csrc/*.hip; do
  obj="$OUT/$(basename "${src%.hip}").o"
  $HIPCC --offload-arch=gfx950 -O1 -g -fPIC -std=c++17 -c "$src" -o "$obj" -I csrc \
    -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -Wno-unused-result &
  objs+=("$obj")
done
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT/libdpa_hip_asan.so" "${objs[@]}" -fsanitize=address -shared-libasan \
  -L"$TORCH_LIB" -lamdhip64 -Wl,-rpath,"$TORCH_LIB"
ASAN_RT=$($HIPCC -print-file-name=libclang_rt.asan-x86_64.so)
echo "ASan runtime: $ASAN_RT"
LD_PRELOAD="$ASAN_RT" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 DPA_LIB_PATH="$PWD/$OUT/libdpa_hip_asan.so" \
  python -m pytest -q -p no:cacheprovider tests/test_host_contracts.py
