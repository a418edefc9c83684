"""Host-side contracts of the HIP kernel library, checked on the CPU (no GPU, no kernel launch).

Every ``dpa_*`` launcher validates its shapes, alignments and tiling before it touches the device
and returns ``hipErrorInvalidValue`` (1) instead of launching a kernel whose grid or addressing
would not match -- the guard against out-of-bounds waves that the GPU tests cannot exercise
safely.  The Python wrappers (ops/kernels.py) assert the tensor-level contracts before building
the argument blocks.  The same checks run under AddressSanitizer (host code) via
``tools/asan_host.sh``.
"""
import ctypes
import os

import pytest
import torch

from distributedpytorch_amd.ops import _lib

INVALID = 1   # hipErrorInvalidValue

pytestmark = pytest.mark.skipif(not _lib.LIB_PATH.exists(), reason="HIP library not built")


@pytest.fixture(scope="module")
def L():
    return _lib.lib()


def _igemm_args(**kw):
    from distributedpytorch_amd.ops import kernels as K
    a = K.IgemmArgs()
    base = dict(ldx=32, ldy=32, N=1, Ho=64, Wo=64, Hs=64, Ws=64, Cs=32, KH=3, KW=3, stride=1, pad=1, Ngemm=32,
                Kpad=288, mode=0, ximg=64 * 64 * 32 * 2)
    base.update(kw)
    for k, v in base.items():
        setattr(a, k, v)
    return a


def _wgrad_args(**kw):
    from distributedpytorch_amd.ops import kernels as K
    a = K.WgradArgs()
    base = dict(lda=32, ldb=32, N=1, Hg=64, Wg=64, HA=64, WA=64, HB=64, WB=64, M=32, Nc=32, s=1, pad=1, KW=3,
                pix_per_split=4096, splits=1)
    base.update(kw)
    for k, v in base.items():
        setattr(a, k, v)
    return a


def test_library_exports_and_version(L):
    assert L.dpa_version() > 0
    for name in ("dpa_igemm", "dpa_igemm_glds", "dpa_igemm_halo", "dpa_igemm_stream", "dpa_wgrad", "dpa_wgrad_halo",
                 "dpa_wgrad_stream", "dpa_wgrad_gemm", "dpa_wgrad_band", "dpa_wgrad_band128", "dpa_wgrad_reduce", "dpa_deconv_fwd", "dpa_deconv_bwd", "dpa_maxpool2",
                 "dpa_pool_bwd", "dpa_pool_bwd_code", "dpa_head_fwd", "dpa_head_bwd", "dpa_bn_fwd", "dpa_bn_bwd",
                 "dpa_up2_fwd", "dpa_up2_bwd", "dpa_adam_flat", "dpa_adam_flat_dev", "dpa_pack_weights",
                 "dpa_slab_fold", "dpa_loss_finish", "dpa_loss_grad"):
        assert hasattr(L, name), name
    assert L.dpa_error_string(INVALID).decode() == "invalid argument"


@pytest.mark.parametrize("kw", [dict(Cs=12), dict(ldx=30), dict(Kpad=300), dict(Ngemm=48), dict(mode=1, Cout=6)])
def test_generic_igemm_rejects(L, kw):
    assert L.dpa_igemm(ctypes.byref(_igemm_args(**kw)), 0, None) == INVALID


@pytest.mark.parametrize("kw", [dict(Cs=32), dict(Kpad=288), dict(KH=7, KW=7, Cs=64, Kpad=64 * 49)])
def test_glds_igemm_rejects(L, kw):
    a = _igemm_args(Cs=64, Kpad=576, Ngemm=256, ldx=64)
    for k, v in kw.items():
        setattr(a, k, v)
    assert L.dpa_igemm_glds(ctypes.byref(a), 0, None) == INVALID


@pytest.mark.parametrize("kw", [dict(Wo=96, Ws=96), dict(relu=1), dict(Kpad=640), dict(Ngemm=192),
                                dict(mask=1, mask_ch=128, ldm=256)])
def test_glds_bn_sums_refuse_other_shapes(L, kw):
    """BatchNorm partial sums (bnslab) exist only in the row-block kernels' forward (bias, no ReLU) and
    full-mask dgrad epilogues: every other launch is refused before anything runs (the caller then
    computes the statistics with the BN pass), never silently run without them."""
    a = _igemm_args(Cs=64, Kpad=576, Ngemm=256, ldx=64, ldy=256, N=2, Ho=32, Wo=64, Hs=32, Ws=64)
    a.bnslab = 0x1000     # never dereferenced: the host checks return first
    for k, v in kw.items():
        setattr(a, k, v)
    assert L.dpa_igemm_glds(ctypes.byref(a), 0, None) == INVALID


@pytest.mark.parametrize("kw", [dict(mode=1), dict(KH=1, KW=1), dict(stride=2), dict(Cs=48, Kpad=448),
                                dict(Hs=66), dict(Kpad=256), dict(Wo=96, Ws=96), dict(ximg=0),
                                dict(ximg=64 * 64 * 32 * 2 - 66)])
def test_halo_igemm_rejects(L, kw):
    assert L.dpa_igemm_halo(ctypes.byref(_igemm_args(**kw)), 0, None) == INVALID


# any row width >= 16 streams (a ragged last strip is masked); narrower rows and a fused pool over an
# odd width (half a 2x2 window) are rejected
@pytest.mark.parametrize("kw", [dict(Wo=8, Ws=8), dict(mode=1), dict(pad=0), dict(Kpad=256), dict(Ngemm=128, Kpad=288),
                                dict(Wo=97, Ws=97, pool=16, ldp=32), dict(ximg=0), dict(ximg=64 * 64 * 32 * 2 - 66)])
def test_stream_igemm_rejects(L, kw):
    assert L.dpa_igemm_stream(ctypes.byref(_igemm_args(**kw)), 0, None) == INVALID


def test_dual_input_only_on_the_stream_kernels(L):
    """A dual conv input (IgemmArgs.x2 / BwdArgs.x2: channels 32-63 from a second tensor) is read only
    by the row-streaming forward at Cs = 64 and the fused backward at 64 input channels; every other
    launcher refuses it instead of silently reading [x | garbage]."""
    dual = dict(Cs=64, Kpad=576, ldx=32, ximg=64 * 64 * 32 * 2)
    for launch in (lambda a: L.dpa_igemm(ctypes.byref(a), 0, None), lambda a: L.dpa_igemm_halo(ctypes.byref(a), 0, None),
                   lambda a: L.dpa_igemm_glds(ctypes.byref(a), 0, None)):
        a = _igemm_args(**dual)
        a.x2 = 0x1000
        assert launch(a) == INVALID
    for kw in (dict(Cs=32, Kpad=288), dict(ldx=16), dict(ximg=64 * 64 * 32 * 2 - 66)):
        a = _igemm_args(**{**dual, **kw})
        a.x2 = 0x1000
        assert L.dpa_igemm_stream(ctypes.byref(a), 0, None) == INVALID, kw
    from distributedpytorch_amd.ops import kernels as K
    b = K.BwdArgs(ldg=32, ldx=32, ldy=32, Kd=288, N=1, H=64, W=64, rh=64, ipb=1)
    b.x2 = 0x1000
    assert L.dpa_bwd_stream(ctypes.byref(b), 32, 32, 0, None) == INVALID            # 32 input channels
    b.ldx = 16
    assert L.dpa_bwd_stream(ctypes.byref(b), 64, 32, 0, None) == INVALID            # a plane is 32 channels


def test_bn_on_load_only_in_bn_statistics_launches(L):
    """IgemmArgs.xbn (BN + ReLU of the input formed on load) exists only in the row-streaming kernel's
    BN-statistics forward epilogue; every other launch that would ignore it is refused.  BwdArgs.xbn
    needs the BN mode with the layer-below statistics."""
    for launch in (lambda a: L.dpa_igemm(ctypes.byref(a), 0, None), lambda a: L.dpa_igemm_halo(ctypes.byref(a), 0, None),
                   lambda a: L.dpa_igemm_glds(ctypes.byref(a), 0, None), lambda a: L.dpa_igemm_stream(ctypes.byref(a), 0, None)):
        a = _igemm_args()
        a.xbn = 0x1000                      # no bnslab: not the BN-statistics epilogue
        assert launch(a) == INVALID
    for kw in (dict(mask=0x2000, mask_ch=32, ldm=32), dict(pool=0x2000, ldp=32, relu=1), dict(Cs=8, Kpad=96, ldx=8)):
        a = _igemm_args(**kw)
        a.xbn, a.bnslab = 0x1000, 0x3000
        assert L.dpa_igemm_stream(ctypes.byref(a), 0, None) == INVALID, kw
    from distributedpytorch_amd.ops import kernels as K
    b = K.BwdArgs(ldg=32, ldx=32, ldy=32, Kd=288, N=1, H=64, W=64, rh=64, ipb=1)
    b.xbn = 0x1000
    assert L.dpa_bwd_stream(ctypes.byref(b), 32, 32, 0, None) == INVALID            # no BN mode


def test_stream_block_count_matches_launch_geometry(L):
    # variant 1 (Cs = Ngemm = 32): 128-pixel strips, 32-row segments when there are >= 1024 of them
    a = _igemm_args(N=128, Ho=512, Wo=512, Hs=512, Ws=512)
    assert L.dpa_igemm_stream_blocks(ctypes.byref(a)) == 128 * (512 // 32) * (512 // 128)
    a = _igemm_args(N=2, Ho=40, Wo=128, Hs=40, Ws=128)
    assert L.dpa_igemm_stream_blocks(ctypes.byref(a)) == 2 * 3 * 1       # 16-row segments: ceil(40/16)


@pytest.mark.parametrize("kw", [dict(M=48), dict(lda=30), dict(pix_per_split=100), dict(splits=0)])
def test_wgrad_rejects(L, kw):
    assert L.dpa_wgrad(ctypes.byref(_wgrad_args(**kw)), 0, 0, None) == INVALID


@pytest.mark.parametrize("kw", [dict(Wg=48, WA=48, WB=48), dict(Nc=48), dict(KW=2), dict(HB=32)])
def test_wgrad_halo_rejects(L, kw):
    assert L.dpa_wgrad_halo(ctypes.byref(_wgrad_args(**kw)), 0, None) == INVALID


def test_wgrad_stream_checks_split_count(L):
    # splits must equal ceil(N/ipb) * ceil(Hg/rh) * (Wg/bp): 1 image, rh 64, bp 64 -> 1 split
    assert L.dpa_wgrad_stream(ctypes.byref(_wgrad_args(splits=2)), 1, 64, 64, 1, None) == INVALID
    assert L.dpa_wgrad_stream(ctypes.byref(_wgrad_args(Wg=96, WA=96, WB=96)), 1, 64, 64, 1, None) == INVALID
    assert L.dpa_wgrad_stream(ctypes.byref(_wgrad_args()), 1, 64, 64, 0, None) == INVALID   # ipb < 1


@pytest.mark.parametrize("kw", [dict(M=128), dict(Nc=36), dict(Wg=96, WA=96, WB=96), dict(Hg=3, HA=3, HB=3, Wg=32, WA=32, WB=32),
                                dict(KW=2), dict(HB=32), dict(splits=2), dict(pix_per_split=0), dict(lda=36),
                                dict(abytes=1024), dict(N=1, Hg=1, HA=1, HB=1),
                                dict(N=3, pix_per_split=2, splits=2, Hg=1, HA=1, HB=1, abytes=2 * 64 * 256 * 2,
                                     bbytes=2 * 64 * 64 * 2)])
def test_wgrad_gemm_rejects(L, kw):
    """csrc/wgrad_gemm.hip: M % 256, Nc % 8, W % 64 or 32, H*W % 64, 3x3 s1 p1 on one grid, split count =
    ceil(N / images per split), 16-B strides, >= 2 K-steps per split (the ragged last one too: 3 one-row
    images of 64 pixels in splits of 2 leave the last split ONE K-step), 32-bit split extents."""
    base = dict(M=256, Nc=64, lda=256, ldb=64, pix_per_split=1, splits=1,
                abytes=64 * 64 * 256 * 2, bbytes=64 * 64 * 64 * 2)
    assert L.dpa_wgrad_gemm(ctypes.byref(_wgrad_args(**base)), None) != INVALID     # the valid case passes
    base.update(kw)
    assert L.dpa_wgrad_gemm(ctypes.byref(_wgrad_args(**base)), None) == INVALID


@pytest.mark.parametrize("kw", [dict(M=128), dict(Nc=48), dict(Nc=16, ldb=16), dict(Wg=128, WA=128, WB=128),
                                dict(Hg=3, HA=3, HB=3, Wg=32, WA=32, WB=32), dict(KW=2), dict(pad=0), dict(HB=32),
                                dict(splits=2), dict(pix_per_split=0), dict(lda=260), dict(abytes=1024),
                                dict(N=0), dict(atab=1)])
def test_wgrad_band_rejects(L, kw):
    """csrc/wgrad_band.hip: M % 256, Nc % 32, W in {32, 64}, H % (64 / W), 3x3 s1 p1 on one grid, split count =
    ceil(N / images per split), 16-B strides, both or neither per-image table, 32-bit split extents (a
    one-K-step split is valid here: no peeled tail)."""
    base = dict(M=256, Nc=64, lda=256, ldb=64, pix_per_split=1, splits=1,
                abytes=64 * 64 * 256 * 2, bbytes=64 * 64 * 64 * 2)
    assert L.dpa_wgrad_band(ctypes.byref(_wgrad_args(**base)), None) != INVALID     # the valid case passes
    one_step = dict(base, Hg=1, HA=1, HB=1)
    assert L.dpa_wgrad_band(ctypes.byref(_wgrad_args(**one_step)), None) != INVALID
    base.update(kw)
    assert L.dpa_wgrad_band(ctypes.byref(_wgrad_args(**base)), None) == INVALID


@pytest.mark.parametrize("kw", [dict(M=64, lda=64), dict(Nc=32, ldb=32), dict(Wg=96, WA=96, WB=96), dict(KW=2),
                                dict(HB=32), dict(splits=2), dict(pix_per_split=96), dict(pix_per_split=0),
                                dict(lda=132), dict(atab=1), dict(atab=1, btab=1, pix_per_split=64 * 32)])
def test_wgrad_band128_rejects(L, kw):
    """csrc/wgrad_band.hip 128-channel form: M % 128, Nc % 64, W % 64, 3x3 s1 p1 on one grid, pixels per
    split a multiple of 64 and splits = ceil(N H W / it), both or neither per-image table, whole-image splits
    with tables."""
    base = dict(M=128, Nc=64, lda=128, ldb=64, pix_per_split=64 * 64, splits=1, Hg=64, Wg=64, HA=64, WA=64,
                HB=64, WB=64)
    assert L.dpa_wgrad_band128(ctypes.byref(_wgrad_args(**base)), None) != INVALID     # the valid case passes
    assert L.dpa_wgrad_band128(ctypes.byref(_wgrad_args(**dict(base, pix_per_split=64 * 16, splits=4))),
                               None) != INVALID                                         # splits inside an image
    base.update(kw)
    assert L.dpa_wgrad_band128(ctypes.byref(_wgrad_args(**base)), None) == INVALID


def test_elementwise_launchers_reject(L):
    n = None
    i = ctypes.c_int
    assert L.dpa_maxpool2(n, i(12), n, i(12), i(1), i(8), i(8), i(12), n, n) == INVALID            # C % 8
    assert L.dpa_pool_bwd_code(n, n, i(8), n, i(8), n, i(8), i(1), i(7), i(8), i(8), n, i(0), n, n, n) == INVALID  # odd H
    assert L.dpa_up2_fwd(n, i(8), n, i(8), i(1), i(0), i(4), i(8), n) == INVALID                   # h < 1
    assert L.dpa_up2_bwd(n, i(8), n, i(8), i(1), i(4), i(4), i(12), n) == INVALID                  # C % 8
    assert L.dpa_slab_fold(n, i(0), i(64), i(8), n, n) == INVALID
    assert L.dpa_deconv_bwd(n, i(64), n, i(64), n, n, i(64), n, n, i(1), i(8), i(8), i(64), i(32), i(0),
                            ctypes.c_uint(0), ctypes.c_uint(0), n, n, n) == INVALID                 # splits < 1
    assert L.dpa_deconv_fwd(n, i(60), n, n, n, i(64), i(1), i(8), i(8), i(64), i(32), i(1), ctypes.c_uint(0),
                            n, n) == INVALID                                                        # ldx % 8


def test_bn_shapes(L):
    assert L.dpa_bn_slab_rows(ctypes.c_longlong(1000), ctypes.c_int(12)) == 0     # C % 8
    rows = L.dpa_bn_slab_rows(ctypes.c_longlong(128 * 512 * 512), ctypes.c_int(32))
    assert 0 < rows <= 512
    assert L.dpa_head_slab_blocks(ctypes.c_longlong(1 << 20)) > 0


def test_python_wrappers_assert_before_launch():
    """Tensor-level checks in ops/kernels.py fire before any argument block is built."""
    from distributedpytorch_amd.ops import kernels as K
    x = torch.zeros(1, 8, 8, 32, dtype=torch.bfloat16)
    w = torch.zeros(32 * 288, dtype=torch.bfloat16)
    y = torch.zeros(1, 8, 8, 16, dtype=torch.bfloat16)            # fewer channels than Ngemm
    with pytest.raises(AssertionError):
        K.igemm(x, w, y, Ngemm=32, Kpad=288, KH=3, KW=3, stride=1, pad=1, Cs=32, out_grid=(1, 8, 8))
    with pytest.raises(AssertionError):                          # packed weights too short
        K.igemm(x, w[:100], torch.zeros(1, 8, 8, 32, dtype=torch.bfloat16), Ngemm=32, Kpad=288, KH=3, KW=3,
                stride=1, pad=1, Cs=32, out_grid=(1, 8, 8))
    with pytest.raises(AssertionError):                          # fp32 activations
        K.igemm(x.float(), w, y, Ngemm=32, Kpad=288, KH=3, KW=3, stride=1, pad=1, Cs=32, out_grid=(1, 8, 8))


def test_native_dp_comm_rejects_bad_args():
    from distributedpytorch_amd.parallel import dp_comm
    if not dp_comm.LIB_PATH.exists():
        pytest.skip("comm library not built")
    L = dp_comm.lib()
    h = ctypes.c_void_p()
    assert L.dpa_dp_comm_init(ctypes.c_int(0), None, ctypes.byref(h)) != 0
    assert L.dpa_dp_all_reduce(None, None, ctypes.c_longlong(4), ctypes.c_int(0), ctypes.c_int(0), None) != 0
    assert L.dpa_dp_broadcast(None, None, ctypes.c_longlong(4), ctypes.c_int(0), ctypes.c_int(0), None) != 0
    assert L.dpa_dp_comm_size(None) == 0
    assert L.dpa_dp_version() > 0


def test_fused_bwd_bn_combinations():
    """HipBlocks.fusable's BatchNorm rule: the fused backward pairs the conv's BN backward
    (loader) with the BN partial sums of the layer below (dx epilogue); a masked dx with BN on one side
    only must take the unfused path instead of failing in the kernel host code."""
    from distributedpytorch_amd.models.hip_unet import bn_combo_ok
    assert bn_combo_ok(False, None, False) and bn_combo_ok(False, False, False)   # no BN anywhere
    assert bn_combo_ok(True, True, True) and bn_combo_ok(True, None, True)        # BN both sides / unmasked dx
    assert not bn_combo_ok(True, True, False) and not bn_combo_ok(True, None, False)   # BN fusion off
    assert not bn_combo_ok(False, True, True)     # no BN here, BN below: no epilogue-only instantiation
    assert not bn_combo_ok(True, False, True)     # BN here, plain layer below: no loader-only masked mode
