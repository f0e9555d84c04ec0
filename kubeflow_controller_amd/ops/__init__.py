"""Hand-written CDNA4 (gfx950) HIP kernels and their torch autograd wrappers.

All kernels live in ONE in-tree shared object (``ops/_hip_kernels.so``) built
from ``csrc/kernels/*.hip`` by ``hipcc --offload-arch=gfx950`` (see
``_build.py``) and bound with ctypes (``_lib.py``).
"""
