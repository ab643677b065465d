"""memo_amd -- MI355X-native (gfx950) block erasure codec for memo.

The hot path (RS encode / rebuild of batched blocks) lives in
memo_amd/csrc (HIP kernels + C ABI, built into memo_amd/_lib/libmemo_ec.so);
memo_amd.ec is its ctypes binding.  See DESIGN.md.
"""
from . import ec  # noqa: F401
