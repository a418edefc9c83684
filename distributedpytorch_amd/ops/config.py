"""Kernel-dispatch configuration of the HIP engine: every environment switch, in ONE documented table.

The engine picks a kernel family per layer automatically (``ops/kernels.py``); the switches below
exist to fall back to a simpler path when triaging a problem on a GPU box, or to A/B launch geometry.
They are read once, at import, from the variables named here and NOWHERE else: an environment
variable outside :data:`KNOBS` / :data:`RUNTIME_ENV` cannot change which kernels run
(``tests/test_kernel_config.py`` checks the package source and a fresh interpreter).  The run's
non-default switches are logged once (:func:`log_once`; bench.py also puts them in its JSON line).

Timing ablation (skipping kernel families to see what they cost; numerically WRONG) is not an
environment switch: only :func:`..ops.kernels.set_timing_ablation` enables it, called explicitly by
the measurement tools (``bench.py --timing-ablation``, ``tools/block_times.py``), and bench marks
such a run invalid in its output.
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass, fields
from typing import Dict, Mapping

log = logging.getLogger("dpa.kernels")


@dataclass(frozen=True)
class Knob:
    attr: str
    env: str
    default: object
    doc: str


def _flag_off(env):      # DPA_NO_X=1 turns feature X off
    return lambda e: e.get(env, "0") != "1"


KNOBS = (
    # kernel families (a switch falls back to the next family / the generic register-staged GEMM)
    Knob("halo", "DPA_NO_HALO", True, "row-halo conv3x3 (csrc/halo.hip) for <= 128-output-channel layers"),
    Knob("stream", "DPA_NO_STREAM", True, "row-streaming conv3x3 / weight gradients (csrc/halo.hip) at 32/64 channels"),
    Knob("glds", "DPA_NO_GLDS", True, "LDS-DMA implicit GEMMs (csrc/igemm_glds.hip) for the deep layers"),
    Knob("glds128", "DPA_NO_GLDS128", True, "128-output-channel convs on the row-block GEMM instead of the row-halo conv"),
    Knob("glds_bn", "DPA_NO_GLDS_BN", True, "BatchNorm partial sums in the row-block GEMM epilogue"),
    Knob("glds_sl", "DPA_NO_GLDS_SL", True, "128-output-channel convs on rows <= 128 px: the slice-staged 128 x 512 GEMM (cfg 18)"),
    Knob("wgrad_gemm", "DPA_NO_WGRAD_GEMM", True, "deep weight gradients as a dense LDS-DMA GEMM (csrc/wgrad_gemm.hip)"),
    Knob("wgrad_presum_y", "DPA_WGRAD_PRESUM_Y", 0, "cap on the in-place presum grid's group blocks (0 = one block per 32-row group)"),
    Knob("slp256", "DPA_SLP256", False, "256-channel convs on 32/64-wide grids as slice-staged ping-pong (igemm_slp_kernel<EP, 256>) instead of the row-block kernel"),
    Knob("slpp", "DPA_NO_SLPP", True, "128-output-channel slice-staged convs on the ping-pong schedule (csrc/igemm_glds.hip igemm_slp_kernel)"),
    Knob("halo_cfg", "DPA_HALO_CFG", 0, "row-halo conv tile override (csrc/halo.hip dpa_igemm_halo cfg; 0 = auto)"),
    Knob("slp64", "DPA_SLP64", False, "64-output-channel convs over >= 64 input channels on rows <= 256 px: slice-staged "
         "ping-pong 64 x 512 (igemm_slp_kernel<EP, 64>, cfg 19) instead of the row-halo conv. Off: bitwise equal but "
         "slower at b256 (3619 vs 3113 us at 256^2 128 -> 64, 1015 vs 875 us at the 128^2 dgrad; 16 MFMAs per phase do "
         "not cover the phase barriers, profiles/kbench_slp64_halo_r06.txt)"),
    Knob("wgrad_up", "DPA_NO_WGRAD_UP", True, "transposed-conv weight gradients (Cin % 256 == 0) on the dense LDS-DMA GEMM "
         "(csrc/wgrad_gemm.hip up mode) instead of the register-staged split-K kernel"),
    Knob("wgrad_band", "DPA_NO_WGRAD_BAND", True, "deep weight gradients with the input band staged once for all 9 taps (csrc/wgrad_band.hip)"),
    Knob("side_wgrad", "DPA_NO_SIDE_WGRAD", True, "weight gradients on a side HIP stream, overlapping the dgrad chain"),
    # fusions
    Knob("fused_head", "DPA_NO_FUSED_HEAD", True, "segmentation head + loss partials in the last decoder conv's epilogue"),
    Knob("fused_bn", "DPA_NO_FUSED_BN", True, "BatchNorm statistics in the producing streaming conv's epilogue"),
    Knob("fold_bn_eval", "DPA_NO_FOLD_BN", True, "eval-mode BatchNorm folded into the conv weights"),
    Knob("fused_bwd", "DPA_NO_FUSED_BWD", True, "fused conv backward (dgrad + weight gradient, csrc/bwd_stream.hip)"),
    Knob("fused_head_bwd", "DPA_NO_FUSED_HEAD_BWD", True, "head backward folded into the last conv's fused backward"),
    Knob("fused_halves", "DPA_NO_FUSED_HALVES", True, "concat-input convs: one fused backward per half"),
    Knob("fused_pool_bwd", "DPA_NO_FUSED_POOL_BWD", True, "max-pool backward folded into the fused backward"),
    Knob("fused_bn_bwd", "DPA_FUSED_BN_BWD", True, "BatchNorm backward formed in the fused backward's loader (=0 opts out)"),
    Knob("fused_w1", "DPA_FUSED_W1", False, "first conv's weight gradient in the pool-mode fused backward (slower at b256)"),
    Knob("fused_deconv", "DPA_NO_FUSED_DECONV", True, "full-resolution transposed conv: fused forward / backward"),
    Knob("bn_on_load", "DPA_NO_BN_ON_LOAD", True, "DoubleConv with BatchNorm: the second conv forms relu(bn(z)) of the "
         "first on load (forward and fused backward); the first conv's BN output is never stored"),
    Knob("dual_input", "DPA_NO_DUAL_INPUT", True, "32-channel level: skip and up half as two dense tensors read by the "
         "decoder conv (no concat buffer)"),
    Knob("f32_wgrad_halo", "DPA_NO_F32_WGRAD_HALO", True, "fp32 engine: 3x3 weight gradients over 32 / 64 input channels "
         "stage the input halo once per 2 x 32-pixel patch (csrc/fp32.hip wgrad3_f32_kernel)"),
    Knob("f32_wgrad_big", "DPA_NO_F32_WGRAD_BIG", True, "fp32 engine: 256 x 256 8-wave weight-gradient tiles for the "
         "256-output-channel layers over >= 256 inputs instead of 128 x 128"),
    Knob("f32_igemm_wide", "DPA_NO_F32_IGEMM_WIDE", True, "fp32 engine: 256-pixel x 128-channel 8-wave conv / dgrad "
         "tiles for GEMM-N % 128 == 0 when the grid has >= 512 of them (the 128 x 128 4-wave tile otherwise)"),
    Knob("f32_wgrad_px", "DPA_NO_F32_WGRAD_PX", True, "fp32 engine: weight-gradient operands staged pixel-major "
         "(no loader transpose; ds_read_b32 operand columns) -- same result bit for bit, 19.9 vs 20.2 ms of "
         "weight gradients at b16 512^2 (profiles/f32_kbench_b16_512_r05_px.txt)"),
    Knob("f32_wgrad3_halves", "DPA_NO_F32_WGRAD3_HALVES", True, "fp32 engine: the halo weight gradient over 64 input "
         "channels as two 32-column blocks (56 KB, 2 blocks per CU) instead of one 104 KB 64-column block: 0.88 vs "
         "1.16 ms at enc1.c2, 312 -> 321 img/s at b16 (profiles/f32_kbench_b16_512_r05_halves.txt)"),
    Knob("bn_sums_pool", "DPA_NO_BN_SUMS_POOL", True, "BatchNorm UNet: the encoder BN's backward partial sums from the "
         "max-pool backward (reads the skip once more) instead of a statistics pass over (g, z)"),
    Knob("bn_sums_deconv", "DPA_NO_BN_SUMS_DECONV", True, "BatchNorm UNet: the decoder BN's backward partial sums from the "
         "fused transposed-conv backward's dx epilogue instead of a statistics pass"),
    Knob("bn_sums_pool_z", "DPA_NO_BN_SUMS_POOL_Z", True, "BatchNorm UNet: the pool backward's BN partial sums read the "
         "dense pre-BN z and re-form relu(bn(z)) instead of reading the skip (a strided concat half)"),
    Knob("wgrad_presum", "DPA_NO_WGRAD_PRESUM", True, "split-K weight-gradient reduction over >= 1024 slab rows of a "
         "small weight: rows summed in groups of 32 in place first (the first conv's [9][32][8] gradient: one "
         "block column per element walked 16k rows, 0.9 ms)"),
    Knob("bn_wgrad_on_load", "DPA_NO_BN_WGRAD_ON_LOAD", True, "BatchNorm UNet: the first conv's BN backward formed "
         "in its weight gradient's loader (dz = a g + b z + c) instead of a dz pass over HBM"),
    Knob("bn_deconv_on_load", "DPA_NO_BN_DECONV_ON_LOAD", True, "BatchNorm UNet: a decoder block's output BN is "
         "applied on load by the next block's fused transposed conv (forward and backward), never written"),
    Knob("bn_dual", "DPA_NO_BN_DUAL", True, "BatchNorm UNet (training): the full-resolution skip and up-sampled "
         "halves stay two dense tensors (dual input, as in the plain UNet) instead of a concat buffer"),
    Knob("bn_halves", "DPA_NO_BN_HALVES", True, "BatchNorm UNet: the 256^2 decoder conv over the 128-channel concat "
         "takes the two-pass fused backward (BN backward on load) instead of dz pass + split dgrad + weight gradient"),
    Knob("bn_skip_z", "DPA_NO_BN_SKIP_Z", True, "BatchNorm UNet: at a dual-input level the encoder's skip is its BN "
         "input z (only the pooled tensor is normalised); the decoder conv forms relu(bn(z)) on load"),
    Knob("bn_head_fold", "DPA_BN_HEAD_FOLD", False, "BatchNorm UNet: the head backward folded into the last decoder "
         "conv's fused backward (a statistics pass, then gy and dz formed on load; the head gradient is never stored). "
         "Off: measured 1.1-1.3 % slower end to end on one box (profiles/bn_knobs_ab_r05.txt, box G)"),
    Knob("bn_head_defer", "DPA_NO_BN_HEAD_DEFER", True, "BatchNorm UNet, head on load: the head backward runs inside the "
         "last decoder level's backward, so its full-resolution gradient is freed there (peak HBM)"),
    Knob("bn_head_on_load", "DPA_NO_BN_HEAD_ON_LOAD", True, "BatchNorm UNet: the segmentation head forms the last decoder "
         "BN's output relu(bn(z)) on load in its forward and backward, so that full-resolution tensor is never written"),
    Knob("f32_wgrad_c4", "DPA_NO_F32_WGRAD_C4", True, "fp32 engine: the first conv's weight gradient (4 padded input "
         "channels, 32 outputs) with 48 MFMA columns straight from global memory instead of a 128-column tile "
         "(0.27 vs 0.58 ms at b16 512^2, profiles/f32_kbench_b16_512_r05_halo.txt)"),
    Knob("f32_conv_halo", "DPA_F32_CONV_HALO", 2, "fp32 engine: 3x3 conv / dgrad with GEMM-N 32 (1; 2: also 64; 0: off) "
         "over 32-channel input slices staged once per 8 x 32 output pixels with the halo (csrc/fp32.hip "
         "conv3_halo_f32_kernel) instead of per tap: enc0.c2 forward 0.89 vs 1.07 ms, dec3.c1 1.42 vs 1.71 ms"),
    # launch geometry / streams
    Knob("side_priority", "DPA_SIDE_PRIORITY", 0, "HIP priority of the weight-gradient side stream (torch convention)"),
    Knob("wgrad_stream_blocks", "DPA_WGRAD_STREAM_BLOCKS", 2048, "target workgroups of a row-streaming weight gradient"),
    Knob("wgrad_gemm_blocks", "DPA_WGRAD_GEMM_BLOCKS", 768, "target workgroups of a dense-GEMM weight gradient"),
    Knob("bwd_blocks", "DPA_BWD_BLOCKS", 1024, "minimum workgroups of a fused backward launch"),
    Knob("bwd_blocks_small", "DPA_BWD_BLOCKS_SMALL", 512, "the same for launches over < 2^25 pixels"),
    Knob("chunk_sink", "DPA_NO_CHUNK_SINK", True, "first-level image chunks: each conv's weight-gradient slab rows "
         "of all chunks in one buffer, reduced once after the chunks (kernels.SlabSink) instead of per chunk"),
    Knob("enc0_chunks", "DPA_ENC0_CHUNKS", 8, "first encoder level backward in this many image chunks, so the first "
         "conv's side-stream weight gradient of one chunk overlaps the next chunk's fused backward (1 = off); 8 vs "
         "4: step wall 86.02 / 85.98 vs 86.61 / 86.04 ms in kernel traces at b256 (profiles/enc0_chunks_r05.txt)"),
)

# process / launcher environment (not kernel dispatch): documented here so the allow-list is complete
RUNTIME_ENV = {
    "DPA_LIB_PATH": "load the HIP kernel library from this path instead of distributedpytorch_amd/_C",
    "DPA_DEBUG_SYNC": "synchronise after every kernel launch (fault triage; same as --debug-sync)",
    "DPA_ROCTX": "emit roctx ranges (same as --trace-ranges)",
    "DPA_SAME_DEVICE": "multi-rank rehearsal: every rank on cuda:0 (tests, one-GPU boxes)",
    "DPA_DIST_BACKEND": "process-group backend override (gloo for the one-GPU rehearsal)",
    "DPA_DP_NATIVE_COMM": "-t DP: the native single-process RCCL clique (=0: torch collectives)",
    "DPA_DP_REPLICAS": "-t DP rehearsal: this many replicas over the visible GPUs round-robin (one-GPU boxes)",
    "DPA_ARCH": "tools/build_hip.py: --offload-arch (default gfx950)",
}

# variables earlier rounds read and that now do nothing: setting one is warned about, not ignored silently
REMOVED_ENV = {
    "DPA_DP_OVERLAP": "removed in round 3: use --no-comm-overlap (DDP / DP) for one reduction after the backward",
}

# the DPA_NO_* switches turn a default-on feature off; the others carry their value
_NEGATED = {k.env for k in KNOBS if k.env.startswith("DPA_NO_")}


def _read(k: Knob, env: Mapping[str, str]):
    raw = env.get(k.env)
    if raw is None:
        return k.default
    if isinstance(k.default, bool):
        on = raw == "1"
        return (not on) if k.env in _NEGATED else on
    return int(raw)


@dataclass(frozen=True)
class KernelConfig:
    halo: bool = True
    stream: bool = True
    glds: bool = True
    glds128: bool = True
    glds_bn: bool = True
    glds_sl: bool = True
    wgrad_gemm: bool = True
    wgrad_band: bool = True
    slpp: bool = True
    slp256: bool = False
    slp64: bool = False
    wgrad_up: bool = True
    chunk_sink: bool = True
    halo_cfg: int = 0
    wgrad_presum_y: int = 0
    side_wgrad: bool = True
    fused_head: bool = True
    fused_bn: bool = True
    fold_bn_eval: bool = True
    fused_bwd: bool = True
    fused_head_bwd: bool = True
    fused_halves: bool = True
    fused_pool_bwd: bool = True
    fused_bn_bwd: bool = True
    fused_w1: bool = False
    fused_deconv: bool = True
    dual_input: bool = True
    bn_on_load: bool = True
    f32_wgrad_halo: bool = True
    f32_wgrad_big: bool = True
    f32_igemm_wide: bool = True
    f32_wgrad_px: bool = True
    f32_wgrad3_halves: bool = True
    f32_conv_halo: int = 2
    bn_sums_pool: bool = True
    bn_sums_deconv: bool = True
    bn_sums_pool_z: bool = True
    bn_head_on_load: bool = True
    bn_head_defer: bool = True
    wgrad_presum: bool = True
    bn_wgrad_on_load: bool = True
    bn_deconv_on_load: bool = True
    bn_dual: bool = True
    bn_halves: bool = True
    bn_skip_z: bool = True
    bn_head_fold: bool = False
    f32_wgrad_c4: bool = True
    side_priority: int = 0
    wgrad_stream_blocks: int = 2048
    wgrad_gemm_blocks: int = 768
    bwd_blocks: int = 1024
    bwd_blocks_small: int = 512
    enc0_chunks: int = 8
    bwd_blocks_set: bool = False          # DPA_BWD_BLOCKS given explicitly: applies to every launch

    @classmethod
    def from_env(cls, env: Mapping[str, str] = None) -> "KernelConfig":
        env = os.environ if env is None else env
        vals = {k.attr: _read(k, env) for k in KNOBS}
        # dependent switches: the fused-backward modes need the fused backward
        for dep in ("fused_head_bwd", "fused_halves", "fused_pool_bwd", "fused_bn_bwd"):
            vals[dep] = vals[dep] and vals["fused_bwd"]
        vals["fused_w1"] = vals["fused_w1"] and vals["fused_pool_bwd"]
        vals["bwd_blocks_set"] = "DPA_BWD_BLOCKS" in env
        return cls(**vals)

    def non_default(self) -> Dict[str, object]:
        ref = KernelConfig()
        return {f.name: getattr(self, f.name) for f in fields(self) if getattr(self, f.name) != getattr(ref, f.name)}

    def describe(self) -> str:
        nd = self.non_default()
        return "kernel config: defaults" if not nd else "kernel config: " + ", ".join(f"{k}={v}" for k, v in nd.items())


def allowed_env() -> Dict[str, str]:
    """Every DPA_* variable the package reads, with its meaning."""
    out = {k.env: k.doc for k in KNOBS}
    out.update(RUNTIME_ENV)
    out.update({k: "(no effect) " + v for k, v in REMOVED_ENV.items()})
    return out


_logged = [False]


def removed_in_env(env: Mapping[str, str] = None) -> Dict[str, str]:
    env = os.environ if env is None else env
    return {k: v for k, v in REMOVED_ENV.items() if k in env}


def log_once(cfg: KernelConfig) -> None:
    if not _logged[0]:
        _logged[0] = True
        log.info(cfg.describe())
        for k, why in removed_in_env().items():
            log.warning("%s is set but has no effect: %s", k, why)
