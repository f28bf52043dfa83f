"""MI355X drop-in for the reference's `simple_knn` extension (submodules/simple-knn).

`from simple_knn._C import distCUDA2` works as in scene/gaussian_model.py:22: distCUDA2(points) returns
the mean squared distance of every point to its 3 nearest other points, computed by libgs4d's HIP
kernels (csrc/knn.hip) through the in-tree `_C` binding.  Importing `_C` without the built extension
raises ImportError -- there is no CPU fallback.
"""
from . import _C  # noqa: F401

__all__ = ["_C"]
