"""Half-block pipeline cuts (a stage boundary between the two convs of a DoubleConv, ``b + 0.5``):
segment units, crossing tensors, stage I/O and parameter ownership, on the CPU."""
import pytest

from distributedpytorch_amd.models.blocks import boundary_names, segment_units
from distributedpytorch_amd.models.unet import build_model
from distributedpytorch_amd.parallel.pipeline import stage_io, stage_param_names


def test_segment_units():
    # depth 2: enc0 enc1 mid dec0 dec1 head
    assert segment_units(0, 6, 2) == [(0, "full"), (1, "full"), (2, "full"), (3, "full"), (4, "full"), (5, "full")]
    assert segment_units(0, 1.5, 2) == [(0, "full"), (1, "a")]
    assert segment_units(1.5, 3.5, 2) == [(1, "b"), (2, "full"), (3, "a")]
    assert segment_units(3.5, 6, 2) == [(3, "b"), (4, "full"), (5, "full")]
    assert segment_units(2.5, 3, 2) == [(2, "b")]
    with pytest.raises(AssertionError):
        segment_units(0, 5.5, 2)          # the head has no halves
    with pytest.raises(AssertionError):
        segment_units(0, 1.25, 2)


def test_boundary_names_and_stage_io():
    # a skip is produced at the END of its encoder block (part b), consumed at the START of its decoder
    # block (part a): a cut inside enc1 does not carry skip1, a cut inside dec0 carries skip0 but not skip1
    assert boundary_names(1.5, 2) == ["x", "skip0"]
    assert boundary_names(2, 2) == ["x", "skip0", "skip1"]
    assert boundary_names(3.5, 2) == ["x", "skip0"]
    assert boundary_names(4.5, 2) == ["x"]
    # skips go straight from producer to consumer stage: skip0 (enc0, stage 0) -> dec1 (stage 2),
    # skip1 (enc1 part b, stage 1) -> dec0 part a (stage 1): internal
    recv, send = stage_io([0, 1.5, 3.5, 6], 2)
    assert recv[1] == [("x", 0)]
    assert sorted(recv[2]) == sorted([("x", 1), ("skip0", 0)])
    assert sorted(send[0]) == sorted([("x", 1), ("skip0", 2)]) and send[1] == [("x", 2)]


@pytest.mark.parametrize("name", ["unet-tiny", "unet-tiny-bn"])
def test_half_cut_parameter_ownership(name):
    model = build_model(name)
    cuts = [0, 0.5, 1.5, 2.5, 3.5, 4.5, 6]
    owned = [set(stage_param_names(model, a, b)) for a, b in zip(cuts, cuts[1:])]
    allp = {n for n, _ in model.named_parameters()}
    assert set().union(*owned) == allp and sum(len(o) for o in owned) == len(allp)   # a partition
    assert owned[0] and all(n.startswith("encoder.conv1.conv_block.0") or n.startswith("encoder.conv1.conv_block.1")
                            for n in owned[0])                      # enc0 part a: the first conv (+ its BN)
    # the decoder's transposed conv belongs to the part that concatenates its output (part a)
    assert any(n.startswith("decoder.deconv2.") for n in owned[4])   # stage [3.5, 4.5): dec0 part b + dec1 part a
    assert any(n.startswith("decoder.deconv1.") for n in owned[3])   # stage [2.5, 3.5): mid part b + dec0 part a
    assert not any(n.startswith("decoder.deconv2.") for n in owned[3])
