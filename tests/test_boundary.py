"""CPU tests of the drop-in boundary (no GPU calls): the C-ABI library loads and exports every entry
point include/gs4d.h declares, argument errors come back as status codes, and the Python API mirror
keeps the reference's names, field order and argument-exclusivity errors
(diff_gaussian_rasterization/__init__.py:157-220 of the reference)."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("gs4d.h", "gs4d_train.h")]
PKG = os.path.join(ROOT, "4dgaussians-fast-train_amd", "diff_gaussian_rasterization")
LIB = os.path.join(PKG, "libgs4d.so")


def declared():
    text = "".join(open(h).read() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gs4d_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("libgs4d.so is not built (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB)
    L.gs4d_version.restype = ctypes.c_char_p
    L.gs4d_last_error.restype = ctypes.c_char_p
    return L


def test_header_declares_the_reference_entry_points():
    names = declared()
    for n in ("gs4d_forward", "gs4d_backward", "gs4d_mark_visible", "gs4d_last_error", "gs4d_version",
              "gs4d_knn_mean_dist", "gs4d_l1_loss_forward", "gs4d_adam_step", "gs4d_densify_stats",
              "gs4d_hexplane_forward", "gs4d_hexplane_backward", "gs4d_hexplane_backward_scratch_bytes", "gs4d_hexplane_order",
              "gs4d_hexplane_reg_forward", "gs4d_hexplane_reg_backward"):
        assert n in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_version_and_error_strings(lib):
    assert lib.gs4d_version().startswith(b"gs4d")
    assert isinstance(lib.gs4d_last_error(), bytes)


def test_argument_errors_are_status_codes(lib):
    # P < 0 is rejected before any HIP call (GS4D_ERR_ARG = 1)
    nr = ctypes.c_int(-7)
    null = ctypes.c_void_p(0)
    args = [null] * 6 + [ctypes.c_int(-1), ctypes.c_int(0), ctypes.c_int(0), null, ctypes.c_int(16),
                         ctypes.c_int(16)] + [null] * 4 + [null, ctypes.c_float(1.0), null, null, null, null, null,
                                                           ctypes.c_float(1.0), ctypes.c_float(1.0), ctypes.c_int(0),
                                                           null, null, null, ctypes.c_int(0), null, ctypes.byref(nr)]
    assert lib.gs4d_forward(*args) == 1
    assert nr.value == 0
    assert b"P" in lib.gs4d_last_error()
    # P == 0 is a no-op success, like the reference's `if (P != 0)` (rasterize_points.cu:79)
    args[6] = ctypes.c_int(0)
    assert lib.gs4d_forward(*args) == 0 and nr.value == 0
    assert lib.gs4d_mark_visible(ctypes.c_int(-1), null, null, null, null, null) == 1
    assert lib.gs4d_mark_visible(ctypes.c_int(0), null, null, null, null, null) == 0


def test_python_api_surface():
    import diff_gaussian_rasterization as dgr
    assert dgr.GaussianRasterizationSettings._fields == (
        "image_height", "image_width", "tanfovx", "tanfovy", "bg", "scale_modifier", "viewmatrix", "projmatrix",
        "sh_degree", "campos", "prefiltered", "debug")
    for name in ("GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians"):
        assert hasattr(dgr, name)
    for name in ("rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible"):
        assert hasattr(dgr._C, name)


def _settings():
    import diff_gaussian_rasterization as dgr
    e = torch.zeros(4, 4)
    return dgr.GaussianRasterizationSettings(8, 8, 0.5, 0.5, torch.ones(3), 1.0, e, e, 0, torch.zeros(3), False,
                                             False)


def test_argument_exclusivity_raises_like_the_reference():
    import diff_gaussian_rasterization as dgr
    r = dgr.GaussianRasterizer(_settings())
    m = torch.zeros(4, 3)
    o = torch.ones(4, 1)
    with pytest.raises(Exception, match="either SHs or precomputed colors"):
        r(m, m, o)  # neither
    with pytest.raises(Exception, match="either SHs or precomputed colors"):
        r(m, m, o, shs=torch.zeros(4, 1, 3), colors_precomp=torch.zeros(4, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m, o, shs=torch.zeros(4, 1, 3))


def test_cpu_tensors_are_refused_loudly():
    import diff_gaussian_rasterization as dgr
    e = torch.empty(0)
    z = torch.zeros(4, 3)
    with pytest.raises(RuntimeError):
        dgr._C.rasterize_gaussians(torch.ones(3), z, e, torch.ones(4, 1), z, torch.zeros(4, 4), 1.0, e,
                                   torch.eye(4), torch.eye(4), 0.5, 0.5, 8, 8, torch.zeros(4, 1, 3), 0,
                                   torch.zeros(3), False, False)


def test_product_package_has_no_oracle_or_cpu_fallback():
    for dirpath, _, files in os.walk(os.path.dirname(PKG)):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), f
                assert "gs4d_oracle" not in src, f


def test_knn_and_train_bindings_load_and_refuse_cpu():
    from simple_knn._C import distCUDA2
    import gs4d_train.kernels as K
    with pytest.raises(RuntimeError):
        distCUDA2(torch.zeros(5, 3))
    with pytest.raises(RuntimeError):
        K._C.l1_forward(torch.zeros(4), torch.zeros(4))
    with pytest.raises(RuntimeError):
        K._C.hexplane_forward(torch.zeros(4, 4), [torch.zeros(1, 4, 2, 2)] * 6)


def test_adam_batch_argument_errors(lib):
    # a descriptor table whose chunk offsets do not chain is refused before any launch
    class T(ctypes.Structure):
        _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("m", ctypes.c_void_p),
                    ("v", ctypes.c_void_p), ("n", ctypes.c_int64), ("first_chunk", ctypes.c_int64),
                    ("s", ctypes.c_float), ("b", ctypes.c_float)]

    class B(ctypes.Structure):
        _fields_ = [("count", ctypes.c_int), ("b1", ctypes.c_float), ("omb1", ctypes.c_float),
                    ("b2", ctypes.c_float), ("omb2", ctypes.c_float), ("eps", ctypes.c_float), ("t", T * 48)]

    b = B()
    b.count = 1
    b.t[0].n = 10
    b.t[0].first_chunk = 3
    assert lib.gs4d_adam_step(ctypes.byref(b), None) == 1
    b.count = 49
    assert lib.gs4d_adam_step(ctypes.byref(b), None) == 1
