"""The config-5 shape device generator (evs_config5_shape, libevmsynth.so)
against its numpy twin, byte for byte (the bench's config5_shape leg input)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("O,n", [(1000, 50_000), (7, 1234), (100_000, 200_000)])
def test_config5_shape_generator_matches_numpy_twin(O, n):
    import torch

    from evolu_amd import synth

    gen = synth.DeviceSynth()
    ts, owner, keep = synth.device_config5_shape(gen, 0xE7010005, O, n, torch.device("cuda", 0))
    t_np, o_np, k_np = synth.config5_shape(0xE7010005, O, n)
    assert np.array_equal(ts.cpu().numpy(), t_np)
    assert np.array_equal(owner.cpu().numpy().view(np.uint32), o_np)
    assert np.array_equal(keep.cpu().numpy().astype(bool), k_np)
