#!/bin/bash
# Environment setup (reference install.sh:1-10 installed numpy / pytorch+cudatoolkit / pandas / tqdm
# with conda).  Here the stack is the ROCm image's PyTorch-ROCm; nothing is downloaded: this checks
# the Python dependencies, builds the gfx950 HIP kernel library in-tree and runs the CPU smoke test.
#   bash install.sh            # build + check
#   bash install.sh --editable # also `pip install -e .` (offline, no dependency resolution)
set -euo pipefail
cd "$(dirname "$0")"
python - <<'PY'
import importlib, sys
missing = [m for m in ("torch", "numpy", "pandas", "tqdm") if importlib.util.find_spec(m) is None]
if missing:
    sys.exit(f"missing python packages: {missing} (use the ROCm PyTorch image)")
import torch
print(f"torch {torch.__version__} hip {torch.version.hip} gpus {torch.cuda.device_count()}")
PY
command -v hipcc >/dev/null || [ -x /opt/rocm/bin/hipcc ] || { echo "hipcc not found (ROCm required)"; exit 1; }
python -c "import __graft_entry__ as g; g.build()"
python -m distributedpytorch_amd.models.unet unet-tiny
if [ "${1:-}" = "--editable" ]; then
  pip install --no-deps --no-build-isolation -e .
fi
echo "ok: python train.py --synthetic   (see README.md)"
