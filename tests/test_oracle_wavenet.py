"""WaveNet oracle self-consistency (parity UNPINNED: wavenet_vocoder 0.1.1 is absent from
the reference and from this image, and the reference holds no WaveNet golden vector).

What pins the restatement as far as this container allows:
  * Philox4x32-10 against the Random123 known-answer vectors;
  * the written-out upsample formula against torch's own conv_transpose2d (the op the
    reference's upsample_conv runs);
  * the incremental (buffered, linearised-conv) step loop against an independent
    full-sequence causal dilated conv1d formulation (what r9y9's own tests assert);
  * weight-norm folding against torch.nn.utils.remove_weight_norm;
  * the HIP-side module (autovc_amd.wavenet.WaveNet) exposing the r9y9 state_dict keys;
  * the reference's own outputs pin only the output length: results/*.wav have 256*Tc
    samples."""
import os
import warnings

import numpy as np
import pytest
import torch

from oracle import wavenet as ow

from conftest import REFERENCE


def test_philox_known_answers():
    m = 0xFFFFFFFF
    assert [int(x) for x in ow.philox4x32(0, 0, 0, 0, 0, 0)] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert [int(x) for x in ow.philox4x32(m, m, m, m, m, m)] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    got = ow.philox4x32(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0)
    assert [int(x) for x in got] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_uniform_range_and_independence_of_grouping():
    u = ow.philox_uniforms(99, [0, 1, 2], 0, 200)
    assert u.dtype == np.float32 and u.shape == (3, 200, 11)
    assert u.min() >= np.float32(1e-5) and u.max() <= np.float32(1 - 1e-5)
    assert abs(float(u.mean()) - 0.5) < 0.02
    # the draw of (utterance, sample) does not depend on the batch or chunk it is part of
    assert np.array_equal(ow.philox_uniforms(99, [2], 50, 120)[0], u[2, 50:120])


def test_upsample_formula_matches_conv_transpose2d():
    hp = ow.small_hparams()
    o = ow.OracleWaveNet(ow.make_weights(hp), hp)
    c = torch.from_numpy(np.random.RandomState(1).rand(2, 80, 3).astype(np.float32))
    a, b = o.upsample(c), o.upsample_loops(c)
    assert a.shape == (2, 80, 3 * 256)
    assert (a - b).abs().max().item() < 1e-12


def test_incremental_matches_full_sequence_formulation():
    hp = ow.small_hparams(layers=8, stacks=2)
    o = ow.OracleWaveNet(ow.make_weights(hp), hp)
    rs = np.random.RandomState(2)
    c = torch.from_numpy(np.clip(rs.normal(0.43, 0.18, (2, 80, 1)), 0, 1).astype(np.float32))
    cu = o.upsample(c)
    T = cu.shape[-1]
    inputs = torch.from_numpy(rs.uniform(-0.9, 0.9, (2, T)))
    _, mol = o.incremental(cu, T, teacher=inputs, return_mol=True)
    full = o.teacher_forced_full(cu, inputs)
    assert (mol - full).abs().max().item() < 1e-12 * max(1.0, full.abs().max().item()) * 100


def test_free_running_is_stable_in_fp32():
    """fp32 vs fp64 restatement with identical uniforms stays together (the GPU parity test
    relies on this: an argmax flip would make sample-wise comparison meaningless)."""
    hp = ow.small_hparams(layers=6, stacks=1)
    W = ow.make_weights(hp)
    o64, o32 = ow.OracleWaveNet(W, hp), ow.OracleWaveNet(W, hp, dtype=torch.float32)
    c = torch.from_numpy(np.clip(np.random.RandomState(3).normal(0.43, 0.18, (1, 80, 1)), 0, 1).astype(np.float32))
    cu = o64.upsample(c)
    u = ow.philox_uniforms(5, [0], 0, 256)
    y64 = o64.incremental(cu, 256, uniforms=u)
    y32 = o32.incremental(cu.float(), 256, uniforms=u)
    assert (y64 - y32.double()).abs().max().item() < 1e-4
    assert y64.abs().max().item() <= 1.0


def test_weight_norm_folding_matches_torch():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        m = torch.nn.utils.weight_norm(torch.nn.Conv1d(6, 10, 3))
    with torch.no_grad():
        m.weight_g.mul_(1.7)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    folded = ow.fold_weight_norm(sd)
    torch.nn.utils.remove_weight_norm(m)
    assert torch.allclose(folded["weight"], m.weight, rtol=1e-6, atol=1e-7)


def test_module_keys_match_r9y9_layout():
    from autovc_amd.synthesis import build_model
    model = build_model()
    want = [k for k, _ in ow.wavenet_keys(weight_norm=True)]
    got = list(model.state_dict().keys())
    assert sorted(got) == sorted(want)
    shapes = dict(ow.wavenet_keys(weight_norm=True))
    assert all(tuple(v.shape) == tuple(shapes[k]) for k, v in model.state_dict().items())
    model.make_generation_fast_()
    assert sorted(model.state_dict().keys()) == sorted(k for k, _ in ow.wavenet_keys(weight_norm=False))
    assert model.receptive_field == 505  # (k-1) * sum(dilations) + 1, SURVEY a23


def test_checkpoint_without_conditioning_bias_loads():
    """wavenet_vocoder 0.1.1 (the reference's pin) gives conv1x1c a bias; later releases do
    not.  A state_dict without the conv1x1c.bias keys loads strictly, as zeros;
    one with them round-trips unchanged."""
    from autovc_amd.synthesis import build_model
    src = build_model()
    sd = src.state_dict()
    for k in sd:
        if k.endswith("conv1x1c.bias"):
            sd[k] = torch.randn_like(sd[k])
    dst = build_model()
    dst.load_state_dict(sd, strict=True)
    assert all(torch.equal(dst.state_dict()[k], v) for k, v in sd.items())
    nobias = {k: v for k, v in sd.items() if not k.endswith("conv1x1c.bias")}
    assert len(nobias) == len(sd) - 24
    dst.load_state_dict(nobias, strict=True)
    for k, v in dst.state_dict().items():
        if k.endswith("conv1x1c.bias"):
            assert not bool(v.any()), k
        else:
            assert torch.equal(v, sd[k]), k


def test_module_rejects_unsupported_configs():
    from autovc_amd.wavenet import WaveNet
    with pytest.raises(NotImplementedError):
        WaveNet(out_channels=256, scalar_input=False, cin_channels=80)
    with pytest.raises(NotImplementedError):
        WaveNet(out_channels=30, scalar_input=True, cin_channels=80, gin_channels=16)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, "results")), reason="reference tree absent")
def test_reference_outputs_pin_length_only():
    """The only WaveNet facts the reference holds: wav length = 256 * Tc."""
    import wave
    root = os.path.join(REFERENCE, "results")
    lens = []
    for d, _, files in os.walk(root):
        for f in files:
            if f.endswith(".wav"):
                try:
                    with wave.open(os.path.join(d, f)) as w:
                        lens.append(w.getnframes())
                except (wave.Error, EOFError):
                    continue
    if not lens:
        pytest.skip("no readable wav in results/")
    assert all(n % 256 == 0 for n in lens)
