"""Caller-side mirror of the reference's rasterizer call path.

The reference's caller (gaussian_renderer/__init__.py) and harness (train.py) cannot travel to the
GPU box, so this package restates the parts of them that touch the rasterizer: camera matrices
(scene/cameras.py, utils/graphics_utils.py), the render() argument mapping, the synthetic scenes
used by the parity tests and bench.py, and the train-step harness.
"""
