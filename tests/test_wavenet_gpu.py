"""WaveNet vocoder on the MI355X (libautovc_hip.so) against the CPU restatement
oracle/wavenet.py (parity UNPINNED upstream: see tests/test_oracle_wavenet.py).

Bars (WaveNet row):
  (1) teacher-forced per-step MoL parameters: <= 1e-4 relative (max-abs / max);
  (2) deterministic sampling with the shared Philox uniforms: every sample within 1e-4;
  (3) output length 256 * Tc, samples in [-1, 1].
Plus properties of the HIP path itself: hipGraph replay == direct launches (bit-exact),
batch / shard / chunk invariance, and the reference's error behaviour."""
import numpy as np
import pytest
import torch

from oracle import wavenet as ow

pytestmark = pytest.mark.gpu

LSM = ow.HPARAMS["log_scale_min"]


def _model(hp, cuda, seed=4322):
    from autovc_amd.wavenet import WaveNet
    m = WaveNet(out_channels=hp["out_channels"], layers=hp["layers"], stacks=hp["stacks"],
                residual_channels=hp["residual_channels"], gate_channels=hp["gate_channels"],
                skip_out_channels=hp["skip_out_channels"], kernel_size=hp["kernel_size"],
                cin_channels=hp["cin_channels"], upsample_conditional_features=True,
                upsample_scales=list(hp["upsample_scales"]), scalar_input=True, legacy=True)
    m.make_generation_fast_()
    W = ow.make_weights(hp, seed)
    m.load_state_dict(W)
    return m.to(cuda).eval(), W


def _cond(B, Tc, seed=4321):
    rs = np.random.RandomState(seed)
    return torch.from_numpy(np.clip(rs.normal(0.43, 0.18, (B, 80, Tc)), 0, 1).astype(np.float32))


def _restore_mode(prev, explicit):
    from autovc_amd import _lib
    if explicit:
        _lib.call("autovc_wavenet_set_grid", prev)
    else:
        _lib.call("autovc_wavenet_reset_grid")


@pytest.fixture(params=[0, 1, 3], ids=["launches", "grid", "pipe"])
def wn_mode(request):
    """Run a test with the per-layer launches, the all-CU weight-resident generation
    (wn_grid_kernel: B <= 8, 8..24 layers, 256 CUs) and the layer-pipelined one (wn_pipe_kernel:
    B <= 8, 24 layers); other shapes use the launches either way.  (The XCD-local form this
    fixture also ran until round 4 is retired: tools/retired/.)"""
    from autovc_amd import _lib
    lib = _lib.load()
    prev, explicit = lib.autovc_wavenet_get_grid(), lib.autovc_wavenet_grid_explicit()
    _lib.call("autovc_wavenet_set_grid", request.param)
    yield request.param
    _restore_mode(prev, explicit)


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def test_upsample_matches_oracle(cuda):
    hp = ow.small_hparams()
    m, W = _model(hp, cuda)
    c = _cond(3, 5)
    got = m.upsample(c.to(cuda)).permute(1, 2, 0)          # (T, B, C) -> (B, C, T)
    want = ow.OracleWaveNet(W, hp).upsample(c)
    assert got.shape == want.shape == (3, 80, 5 * 256)
    assert rel(got, want) < 1e-6


@pytest.mark.parametrize("B,layers,stacks", [(3, 24, 4), (9, 6, 2)])
def test_teacher_forced_mol_and_samples(cuda, B, layers, stacks, wn_mode):
    hp = ow.small_hparams(layers=layers, stacks=stacks)
    m, W = _model(hp, cuda)
    c = _cond(B, 2)
    T = 512
    rs = np.random.RandomState(11)
    teacher = torch.from_numpy(rs.uniform(-0.9, 0.9, (B, T)).astype(np.float32))
    seed = 1234567
    y, mol = m.generate(c.to(cuda), T=T, seed=seed, teacher=teacher.to(cuda), return_mol=True, log_scale_min=LSM)
    o = ow.OracleWaveNet(W, hp)
    u = ow.philox_uniforms(seed, list(range(B)), 0, T)
    y_ref, mol_ref = o.incremental(o.upsample(c), T, uniforms=u, teacher=teacher.double(), return_mol=True)
    assert rel(mol, mol_ref) < 1e-4
    assert (y.double().cpu() - y_ref).abs().max().item() < 1e-4


def test_free_running_matches_oracle(cuda, wn_mode):
    hp = ow.HPARAMS
    m, W = _model(hp, cuda)
    c = _cond(2, 2, seed=7)
    seed = 2024
    y = m.generate(c.to(cuda), seed=seed, log_scale_min=LSM)
    o = ow.OracleWaveNet(W, hp)
    u = ow.philox_uniforms(seed, [0, 1], 0, 512)
    y_ref = o.incremental(o.upsample(c), 512, uniforms=u)
    assert y.shape == (2, 512)
    assert (y.double().cpu() - y_ref).abs().max().item() < 1e-4


def test_graph_replay_is_bit_exact(cuda):
    hp = ow.small_hparams()
    m, _ = _model(hp, cuda)
    c = _cond(4, 2).to(cuda)
    a = m.generate(c, seed=5, log_scale_min=LSM, graph_steps=0)
    b = m.generate(c, seed=5, log_scale_min=LSM, graph_steps=32)
    d = m.generate(c, seed=5, log_scale_min=LSM, graph_steps=7)      # graph + direct remainder
    assert torch.equal(a, b) and torch.equal(a, d)


def test_batch_shard_and_chunk_invariance(cuda, wn_mode):
    hp = ow.small_hparams()
    m, _ = _model(hp, cuda)
    c = _cond(3, 2).to(cuda)
    full = m.generate(c, seed=77, log_scale_min=LSM)
    alone = m.generate(c[2:3], seed=77, utt_base=2, log_scale_min=LSM)
    chunked = m.generate(c, seed=77, log_scale_min=LSM, chunk=96)
    assert (full[2:3] - alone).abs().max().item() < 1e-5
    assert (full - chunked).abs().max().item() < 1e-5


def test_wavegen_api(cuda, wn_mode):
    from autovc_amd import synthesis
    torch.manual_seed(0)
    model = synthesis.build_model().to(cuda)      # r9y9 init, weight norm still attached
    torch.manual_seed(0)
    mel = np.clip(np.random.RandomState(3).normal(0.43, 0.18, (3, 80)), 0, 1).astype(np.float32)
    y = synthesis.wavegen(model, c=mel)
    assert y.shape == (3 * 256,) and y.dtype == np.float32
    assert np.isfinite(y).all() and np.abs(y).max() <= 1.0
    mels = [mel, mel[:2]]
    ys = synthesis.wavegen_batch(model, mels, seed=9)
    assert [len(v) for v in ys] == [768, 512]
    solo = synthesis.wavegen_batch(model, [mel[:2]], seed=9, utt_offset=1)[0]
    assert np.abs(solo - ys[1]).max() < 1e-5


def test_error_behaviour(cuda):
    hp = ow.small_hparams()
    m, _ = _model(hp, cuda)
    c = _cond(1, 1).to(cuda)
    with pytest.raises(ValueError):
        m.generate(c, T=100)
    m.train()
    with pytest.raises(RuntimeError, match="eval"):
        m.generate(c)
    m.eval()
    with pytest.raises(RuntimeError, match="cuda"):
        m.generate(c.cpu())


def test_full_size_config4_shard_invariance(cuda, wn_mode):
    """BASELINE config 4 at full size (8 utterances x 32,768 samples, 24 layers): sharding the
    batch by rank (utt_base) reproduces the single-batch run over 256 ring wraps and 256
    conditioning chunks; every sample finite and in [-1, 1]."""
    hp = ow.HPARAMS
    m, _ = _model(hp, cuda)
    c = _cond(8, 128, seed=19).to(cuda)
    full = m.generate(c, seed=31, log_scale_min=LSM)
    assert full.shape == (8, 32768)
    assert torch.isfinite(full).all() and full.abs().max().item() <= 1.0
    lo = m.generate(c[:4], seed=31, log_scale_min=LSM)
    hi = m.generate(c[4:], seed=31, utt_base=4, log_scale_min=LSM)
    assert (full - torch.cat([lo, hi])).abs().max().item() < 1e-5
    # not a constant or collapsed signal
    assert full.std(dim=1).min().item() > 1e-3


def test_two_tiles_direct_launches_equal_graphs(cuda):
    """16 utterances (two 8-utterance tiles of every kernel), 24 layers, 4,096 samples (32 ring
    wraps): direct launches, 32-step graphs and 7-step graphs with a direct remainder agree
    bit for bit."""
    hp = ow.HPARAMS
    m, _ = _model(hp, cuda)
    c = _cond(16, 16, seed=23).to(cuda)
    a = m.generate(c, seed=3, log_scale_min=LSM, graph_steps=0)
    b = m.generate(c, seed=3, log_scale_min=LSM)
    d = m.generate(c, seed=3, log_scale_min=LSM, graph_steps=7)
    assert a.shape == (16, 4096)
    assert torch.equal(a, b) and torch.equal(a, d)


def _set_modes(grid):
    from autovc_amd import _lib
    _lib.call("autovc_wavenet_set_grid", grid)


@pytest.mark.parametrize("mode", [1, 3], ids=["grid", "pipe"])
@pytest.mark.parametrize("B", [8, 1])
def test_grid_generation_matches_launches(cuda, B, mode):
    """The all-CU weight-resident generation (wn_grid_kernel: every gate weight of the chain
    on chip, each phase's outputs handed on in tagged granules, the past taps computed a step
    ahead by the same workgroups) against the per-layer launches: 24 layers, 2,048 free-running samples (16 ring wraps, 16 conditioning
    chunks = 16 persistent launches, so the past taps cross launch seams), within fp32
    summation-order noise, the MoL parameters of a teacher-forced run within 1e-5; B = 8 and
    the reference's wavegen batch of one; no fault recorded."""
    import ctypes
    from autovc_amd import _lib
    lib = _lib.load()
    if lib.autovc_lstm_xcd_supported(64, 512) == 0:
        pytest.skip("needs 8 XCDs x 32 CUs")
    hp = ow.HPARAMS
    m, _ = _model(hp, cuda)
    c = _cond(B, 8, seed=31).to(cuda)
    rs = np.random.RandomState(6)
    teacher = torch.from_numpy(rs.uniform(-0.9, 0.9, (B, 2048)).astype(np.float32)).to(cuda)
    prev, explicit = lib.autovc_wavenet_get_grid(), lib.autovc_wavenet_grid_explicit()
    out = {}
    try:
        for md in (0, mode):
            _set_modes(md)
            y = m.generate(c, seed=17, log_scale_min=LSM)
            assert lib.autovc_wavenet_last_path() == {0: 0, 1: 1, 3: 2}[md]
            _, mol = m.generate(c, seed=17, log_scale_min=LSM, teacher=teacher, return_mol=True)
            out[md] = (y, mol)
    finally:
        _restore_mode(prev, explicit)
    (y0, m0), (y1, m1) = out[0], out[mode]
    assert torch.isfinite(y1).all() and torch.isfinite(m1).all()
    assert rel(m1, m0) < 1e-5
    assert (y1 - y0).abs().max().item() < 1e-4
    f = ctypes.c_int(0)
    _lib.call("autovc_wavenet_fault", 1, ctypes.addressof(f))
    assert f.value == 0


def test_grid_generation_timeout_surfaces(cuda):
    """A hand-off wait that gives up (forced: a 1-tick timeout) with the all-CU form requested
    (mode 1) poisons the outputs and raises DeviceFault; the next call runs clean."""
    from autovc_amd import _lib, functional as AF
    lib = _lib.load()
    if lib.autovc_lstm_xcd_supported(64, 512) == 0:
        pytest.skip("needs 8 XCDs x 32 CUs")
    hp = ow.small_hparams(layers=8, stacks=2)
    m, _ = _model(hp, cuda)
    c = _cond(2, 1).to(cuda)
    prev, explicit = lib.autovc_wavenet_get_grid(), lib.autovc_wavenet_grid_explicit()
    try:
        _set_modes(1)
        _lib.call("autovc_wavenet_set_timeout_ticks", 1)
        with pytest.raises(AF.DeviceFault, match="wn_grid_kernel.*AVC_WN_GRID=0"):
            m.generate(c, seed=1, log_scale_min=LSM)
        _lib.call("autovc_wavenet_set_timeout_ticks", 0)
        y = m.generate(c, seed=1, log_scale_min=LSM)      # the next call runs clean
        assert torch.isfinite(y).all()
    finally:
        _lib.call("autovc_wavenet_set_timeout_ticks", 0)
        _restore_mode(prev, explicit)


def test_grid_default_mode_small_batches(cuda):
    """Mode 2 runs the all-CU form for up to two utterances: B = 1 and B = 2
    equal mode 1 bit for bit, B = 3 equals the launches bit for bit.  If its wait gives up
    (forced: a 1-tick timeout) the call raises DeviceFault naming AVC_WN_GRID=0 — it does not
    regenerate on the launches — and the mode is unchanged."""
    from autovc_amd import _lib, functional as AF
    lib = _lib.load()
    if lib.autovc_lstm_xcd_supported(64, 512) == 0:
        pytest.skip("needs 8 XCDs x 32 CUs")
    hp = ow.small_hparams(layers=8, stacks=2)
    m, _ = _model(hp, cuda)
    c1, c2, c3 = _cond(1, 2, seed=3).to(cuda), _cond(2, 2, seed=4).to(cuda), _cond(3, 2, seed=5).to(cuda)
    prev, explicit = lib.autovc_wavenet_get_grid(), lib.autovc_wavenet_grid_explicit()
    try:
        out = {}
        for mode in (0, 1, 2):
            _set_modes(mode)
            out[mode] = tuple(m.generate(c, seed=5, log_scale_min=LSM) for c in (c1, c2, c3))
            assert lib.autovc_wavenet_last_path() == (1 if mode == 1 else 0)   # the last call was B = 3
        assert torch.equal(out[2][0], out[1][0]) and torch.equal(out[2][1], out[1][1])
        assert torch.equal(out[2][2], out[0][2])
        _set_modes(2)
        _lib.call("autovc_wavenet_set_timeout_ticks", 1)
        with pytest.raises(AF.DeviceFault, match="wn_grid_kernel.*AVC_WN_GRID=0"):
            m.generate(c1, seed=5, log_scale_min=LSM)
        assert lib.autovc_wavenet_get_grid() == 2
        _lib.call("autovc_wavenet_set_timeout_ticks", 0)
        assert torch.equal(m.generate(c1, seed=5, log_scale_min=LSM), out[2][0])   # the next call runs clean
    finally:
        _lib.call("autovc_wavenet_set_timeout_ticks", 0)
        _restore_mode(prev, explicit)


def test_pipe_default_mode_and_fallback(cuda):
    """The library default (AVC_WN_GRID unset: mode 3) runs the layer-pipelined kernel for
    B <= 8 at the r9y9 shape (24 layers) and the per-layer launches otherwise (B = 9, 8 layers).
    A default-mode call whose wait gives up (forced: a 1-tick timeout) warns and regenerates on
    the launches — the samples equal mode 0's — and the mode stays the unchosen default; the same
    timeout with mode 3 chosen explicitly raises DeviceFault (ADVICE r5 on the default path)."""
    from autovc_amd import _lib, functional as AF
    lib = _lib.load()
    if lib.autovc_lstm_xcd_supported(64, 512) == 0:
        pytest.skip("needs 8 XCDs x 32 CUs")
    prev, explicit = lib.autovc_wavenet_get_grid(), lib.autovc_wavenet_grid_explicit()
    m, _ = _model(ow.HPARAMS, cuda)
    small, _ = _model(ow.small_hparams(layers=8, stacks=2), cuda)
    c1, c9 = _cond(1, 1, seed=3).to(cuda), _cond(9, 1, seed=4).to(cuda)
    try:
        _lib.call("autovc_wavenet_reset_grid")
        assert lib.autovc_wavenet_get_grid() == 3 and lib.autovc_wavenet_grid_explicit() == 0
        y = m.generate(c1, seed=5, log_scale_min=LSM)
        assert lib.autovc_wavenet_last_path() == 2
        m.generate(c9, seed=5, log_scale_min=LSM)
        assert lib.autovc_wavenet_last_path() == 0
        small.generate(c1, seed=5, log_scale_min=LSM)
        assert lib.autovc_wavenet_last_path() == 0
        _lib.call("autovc_wavenet_set_grid", 0)
        y0 = m.generate(c1, seed=5, log_scale_min=LSM)
        assert (y - y0).abs().max().item() < 1e-4
        _lib.call("autovc_wavenet_reset_grid")
        _lib.call("autovc_wavenet_set_timeout_ticks", 1)
        with pytest.warns(RuntimeWarning, match="wn_pipe_kernel.*regenerating"):
            yf = m.generate(c1, seed=5, log_scale_min=LSM)
        assert torch.equal(yf, y0)
        assert lib.autovc_wavenet_get_grid() == 3 and lib.autovc_wavenet_grid_explicit() == 0
        _lib.call("autovc_wavenet_set_grid", 3)
        with pytest.raises(AF.DeviceFault, match="wn_pipe_kernel.*AVC_WN_GRID=0"):
            m.generate(c1, seed=5, log_scale_min=LSM)
        _lib.call("autovc_wavenet_set_timeout_ticks", 0)
        assert torch.equal(m.generate(c1, seed=5, log_scale_min=LSM), y)   # the next call runs clean
    finally:
        _lib.call("autovc_wavenet_set_timeout_ticks", 0)
        _restore_mode(prev, explicit)
