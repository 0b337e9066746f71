"""End-to-end chain (BASELINE config 5): wav -> GPU STFT+mel -> Generator conversion ->
WaveNet, each stage checked against its oracle on the same inputs, plus the batching and
sharding invariances the pipeline relies on."""
import numpy as np
import pytest
import torch

from oracle import frontend as fe
from oracle import generator as og
from oracle import wavenet as ow

pytestmark = pytest.mark.gpu


def _wavs(n, seed=3):
    """SURVEY §8d C5 synthetic audio: 3 sinusoids (100-4000 Hz, amp <= 0.3) + N(0, 0.01)."""
    rs = np.random.RandomState(seed)
    out = []
    for _ in range(n):
        L = int(rs.randint(6000, 12000))
        t = np.arange(L) / 16000.0
        w = sum(rs.uniform(0.05, 0.3) * np.sin(2 * np.pi * rs.uniform(100, 4000) * t) for _ in range(3))
        out.append(np.clip(w + rs.normal(0, 0.01, L), -0.99, 0.99))
    return out


def _models(cuda):
    from autovc_amd.model_vc_mel import Generator
    from autovc_amd.wavenet import WaveNet
    G = Generator(32, 256, 512, 32)
    G.load_state_dict(og.make_weights())
    hp = ow.small_hparams(layers=6, stacks=2)
    V = WaveNet(out_channels=30, layers=6, stacks=2, residual_channels=512, gate_channels=512,
                skip_out_channels=256, cin_channels=80, upsample_conditional_features=True,
                upsample_scales=[4, 4, 4, 4], scalar_input=True)
    V.make_generation_fast_()
    V.load_state_dict(ow.make_weights(hp))
    return G.to(cuda).eval(), V.to(cuda).eval()


def test_end_to_end_stages_vs_oracles(cuda):
    from autovc_amd import pipeline
    wavs = _wavs(3)
    G, V = _models(cuda)
    g = torch.Generator().manual_seed(9)
    e = torch.randn(3, 256, generator=g)
    e = e / e.norm(dim=1, keepdim=True) * 0.8
    e_org, e_trg = e.to(cuda), e.roll(1, 0).to(cuda)
    mels, waves = pipeline.convert_and_vocode(wavs, G, V, e_org, e_trg, seed=11)
    specs = pipeline.spectrograms(wavs, device=cuda, seeds=[0, 1, 2])
    ref_gen = og.OracleGenerator(og.make_weights(), training=False)
    for i, w in enumerate(wavs):
        # front end vs oracle (same host preprocessing stream)
        pre = fe.preprocess(np.asarray(w, np.float64), np.random.RandomState(i))
        spec_ref = fe.spmel_from_wav(pre)
        assert np.abs(specs[i].cpu().numpy() - spec_ref).max() <= 1e-4
        # conversion vs oracle, B=1 as conversion.py
        x, len_pad = pipeline.pad_seq(specs[i].cpu().numpy())
        with torch.no_grad():
            _, ref_psnt, _ = ref_gen.forward(torch.from_numpy(x[None]), e[i:i + 1], e.roll(1, 0)[i:i + 1])
        ref = ref_psnt[0, 0, : specs[i].shape[0]]
        err = (mels[i].cpu().double() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-4, (i, err)
        # vocoder output contract
        assert waves[i].shape == (256 * specs[i].shape[0],) and np.isfinite(waves[i]).all()
        assert np.abs(waves[i]).max() <= 1.0


def test_batched_conversion_equals_per_utterance(cuda):
    from autovc_amd import pipeline
    G, _ = _models(cuda)
    wavs = _wavs(4, seed=5)
    wavs[1] = wavs[0][:len(wavs[0]) - 300]      # same padded length as utterance 0 -> batched together
    specs = pipeline.spectrograms(wavs, device=cuda)
    e = torch.nn.functional.normalize(torch.randn(4, 256), dim=1).to(cuda) * 0.8
    a = pipeline.convert(G, specs, e, e.flip(0), batch=True)
    b = pipeline.convert(G, specs, e, e.flip(0), batch=False)
    for x, y in zip(a, b):
        assert x.shape == y.shape
        assert (x - y).abs().max().item() <= 1e-5 * max(1.0, y.abs().max().item())


def test_stft_model_output_projected_to_mels(cuda):
    from autovc_amd import dsp, pipeline
    y = torch.rand(37, 513, device=cuda)
    got = pipeline._mel_project(y).cpu().double()
    ref = y.cpu().double() @ torch.from_numpy(dsp.mel_basis().T).double()
    assert got.shape == (37, 80)
    assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
