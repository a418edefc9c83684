#!/usr/bin/env python3
"""Build a variant of the HIP kernel library with extra compiler flags into build/ab/NAME/libdpa_hip.so, for
same-box A/B runs (``DPA_LIB_PATH=build/ab/NAME/libdpa_hip.so python bench.py``).

    python tools/build_variant.py prio -DDPA_PRIO_STATIC
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import build_hip  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
root = Path(build_hip.ROOT)
build_hip.BUILD = root / "build" / "ab" / name / "obj"
build_hip.OUT = root / "build" / "ab" / name
print(build_hip.build(force=False, flags=flags))
