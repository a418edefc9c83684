"""Kernel-dispatch switches (ops/config.py): one documented table, and nothing outside it changes
which kernels run."""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_every_dpa_variable_in_the_package_is_documented():
    from distributedpytorch_amd.ops.config import allowed_env
    allowed = allowed_env()
    found = set()
    for f in (ROOT / "distributedpytorch_amd").rglob("*.py"):
        if f.name != "config.py" or f.parent.name != "ops":     # the table itself
            found |= set(re.findall(r"DPA_[A-Z0-9_]+", f.read_text()))
    for f in ("bench.py", "train.py", "__graft_entry__.py", "tools/build_hip.py"):
        found |= set(re.findall(r"DPA_[A-Z0-9_]+", (ROOT / f).read_text()))
    undocumented = sorted(found - set(allowed))
    assert not undocumented, f"DPA_* names read outside the documented allow-list: {undocumented}"
    assert all(len(doc) > 10 for doc in allowed.values())


def test_unknown_variables_do_not_change_dispatch():
    """A fresh interpreter with stray DPA_* variables (including the removed DPA_ABLATE timing switch and
    retired A/B knobs) builds the default kernel config and no timing ablation."""
    code = ("import json; from distributedpytorch_amd.ops import kernels as K; "
            "print(json.dumps({'nd': K.CFG.non_default(), 'ablate': sorted(K._ABLATE), "
            "'sl': K.USE_GLDS_SL, 'halo': K.USE_HALO}))")
    env = dict(os.environ, DPA_ABLATE="glds,halo,bwd", DPA_WGRAD_ROWS="1", DPA_FUSED_DCONV1="1",
               DPA_GLDS_TAP_MAJOR="1", DPA_GLDS_NO_PP="1", DPA_GLDS_RB2="1", DPA_SOMETHING_NEW="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"nd": {}, "ablate": [], "sl": True, "halo": True}


def test_documented_switches_parse():
    from distributedpytorch_amd.ops.config import KernelConfig
    c = KernelConfig.from_env({"DPA_NO_HALO": "1", "DPA_BWD_BLOCKS": "2048", "DPA_NO_FUSED_BWD": "1"})
    assert not c.halo and c.bwd_blocks == 2048 and c.bwd_blocks_set
    assert not c.fused_bwd and not c.fused_pool_bwd and not c.fused_head_bwd     # dependent modes follow
    assert set(c.non_default()) == {"halo", "bwd_blocks", "bwd_blocks_set", "fused_bwd", "fused_head_bwd",
                                    "fused_halves", "fused_pool_bwd", "fused_bn_bwd"}
    assert "halo=False" in c.describe()
    assert KernelConfig.from_env({}).describe() == "kernel config: defaults"


def test_timing_ablation_is_explicit_only():
    import pytest
    from distributedpytorch_amd.ops import kernels as K
    assert K._ABLATE == frozenset()
    K.set_timing_ablation({"wgrad"})
    try:
        assert K._ABLATE == {"wgrad"}
    finally:
        K.set_timing_ablation(())
    with pytest.raises(AssertionError):
        K.set_timing_ablation({"not_a_family"})
