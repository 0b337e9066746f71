"""autovc_amd — MI355X-native (gfx950) hot path of AutoVC.

Host modules keep the reference's Python API (model_vc_mel.Generator, solver_encoder.Solver,
make_spect.Spect, synthesis.build_model/wavegen, ...); the arithmetic runs in the
hand-written HIP kernels of libautovc_hip.so (csrc/), reached through _lib (ctypes).
"""
__version__ = "0.1.0"
