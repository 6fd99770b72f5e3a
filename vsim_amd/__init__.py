"""vsim_amd — MI355X-native Q4_0 decode path for the NAIST-Archlab/vsim ggml runner.

The compute lives in libvsim_hip.so (vsim_amd/csrc, HIP for gfx950) behind the C-ABI
in include/vsim_hip.h; `vsim_amd.hip` is its ctypes binding and `vsim_amd.modelgen`
writes deterministic synthetic ggml model files.
"""
__all__ = ["hip", "modelgen"]
