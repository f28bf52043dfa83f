"""ctypes wrapper around the CPU parity oracle (oracle/gs4d_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  The C restatement follows
submodules/depth-diff-gaussian-rasterization/cuda_rasterizer/{forward,backward,rasterizer_impl}.cu
of the reference; see the header of gs4d_oracle.c for the function-by-function citations.

Arrays are numpy float32/int32/uint32, C-contiguous.  Semantics mirror the reference `_C`
entry points (rasterize_points.cu:36-198): forward returns (num_rendered, color (3,H,W),
depth (1,H,W), radii (P,)) plus the internal state needed by backward; backward returns the
8-tuple (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
dL_drotations) in the reference's order.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgs4d_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def build():
    """Compile the oracle with its Makefile (gcc + OpenMP)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    lib = ctypes.CDLL(_LIB_PATH)
    lib.gs4d_oracle_forward.restype = ctypes.c_void_p
    lib.gs4d_oracle_forward.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int,
        _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_float, _f32p, _f32p, _f32p, _f32p, _f32p,
        ctypes.c_float, ctypes.c_float, ctypes.c_int, _f32p, _f32p, _i32p, _i32p, _i32p]
    lib.gs4d_oracle_backward.restype = None
    lib.gs4d_oracle_backward.argtypes = [
        ctypes.c_void_p, _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_float, _f32p, _f32p, _f32p,
        _f32p, _f32p, ctypes.c_float, ctypes.c_float, _i32p, _f32p,
        _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
    lib.gs4d_oracle_free.argtypes = [ctypes.c_void_p]
    lib.gs4d_oracle_state_L.argtypes = [ctypes.c_void_p]
    lib.gs4d_oracle_state_L.restype = ctypes.c_int
    lib.gs4d_oracle_state_export.argtypes = [ctypes.c_void_p, _f32p, _f32p, _f32p, _f32p, _u8p, _u32p,
                                             _u32p, _u32p, _f32p, _u32p, _f32p]
    lib.gs4d_oracle_mark_visible.argtypes = [ctypes.c_int, _f32p, _f32p, _f32p, _u8p]
    lib.gs4d_oracle_sh_forward.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _u8p]
    lib.gs4d_oracle_knn.argtypes = [ctypes.c_int, _f32p, _f32p]
    lib.gs4d_oracle_flip_flags.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, _u8p, _u8p]
    lib.gs4d_oracle_flip_flags.restype = ctypes.c_int
    lib.gs4d_oracle_flip_bounds.argtypes = [ctypes.c_void_p, _f32p, _f32p, _f32p, ctypes.c_float, ctypes.c_float, _u8p,
                                            _u8p, _f32p, _f32p, ctypes.POINTER(ctypes.c_double)]
    lib.gs4d_oracle_flip_bounds.restype = ctypes.c_int
    lib.gs4d_oracle_near_pairs.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int, _i32p, _i32p, _i32p,
                                           _f32p, _f32p]
    lib.gs4d_oracle_near_pairs.restype = ctypes.c_int
    lib.gs4d_oracle_backward_tail.restype = None
    lib.gs4d_oracle_backward_tail.argtypes = [
        ctypes.c_void_p, _f32p, _f32p, _f32p, ctypes.c_float, _f32p, _f32p, _f32p, _f32p, _f32p, ctypes.c_float,
        ctypes.c_float, _i32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
    lib.gs4d_oracle_set_threads.argtypes = [ctypes.c_int]
    lib.gs4d_oracle_get_threads.restype = ctypes.c_int
    _lib = lib
    return lib


def set_threads(n):
    _load().gs4d_oracle_set_threads(int(n))


def get_threads():
    return _load().gs4d_oracle_get_threads()


def _arr(a, dtype=np.float32):
    """None / empty -> NULL (the reference's empty-tensor convention)."""
    if a is None:
        return None, None
    a = np.ascontiguousarray(np.asarray(a, dtype=dtype))
    if a.size == 0:
        return None, None
    ctype = {np.float32: _f32p, np.int32: _i32p, np.uint8: _u8p, np.uint32: _u32p}[dtype]
    return a, a.ctypes.data_as(ctype)


class OracleState:
    """Owns the C-side forward state (GeometryState/BinningState/ImageState analogue)."""

    def __init__(self, handle, P, W, H):
        self.handle = handle
        self.P, self.W, self.H = P, W, H

    def __del__(self):
        if getattr(self, "handle", None) and _lib is not None:
            _lib.gs4d_oracle_free(self.handle)
            self.handle = None

    def export(self):
        """Internal forward buffers, for white-box tests."""
        lib = _load()
        P, W, H = self.P, self.W, self.H
        L = lib.gs4d_oracle_state_L(self.handle)
        gx, gy = (W + 15) // 16, (H + 15) // 16
        out = dict(
            depths=np.zeros(P, np.float32), means2D=np.zeros((P, 2), np.float32),
            conic_opacity=np.zeros((P, 4), np.float32), rgb=np.zeros((P, 3), np.float32),
            clamped=np.zeros(P, np.uint8), tiles_touched=np.zeros(P, np.uint32),
            point_list=np.zeros(max(L, 1), np.uint32), ranges=np.zeros((gx * gy, 2), np.uint32),
            final_T=np.zeros((H, W), np.float32), n_contrib=np.zeros((H, W), np.uint32),
            cov3D=np.zeros((P, 6), np.float32))
        p = lambda k, t: out[k].ctypes.data_as(t)
        lib.gs4d_oracle_state_export(self.handle, p("depths", _f32p), p("means2D", _f32p),
                                     p("conic_opacity", _f32p), p("rgb", _f32p), p("clamped", _u8p),
                                     p("tiles_touched", _u32p), p("point_list", _u32p), p("ranges", _u32p),
                                     p("final_T", _f32p), p("n_contrib", _u32p), p("cov3D", _f32p))
        out["point_list"] = out["point_list"][:L]
        out["L"] = L
        return out


def rasterize_forward(bg, means3D, colors_precomp, opacities, scales, rotations, scale_modifier, cov3D_precomp,
                      viewmatrix, projmatrix, tanfovx, tanfovy, image_height, image_width, sh, degree, campos,
                      prefiltered=False):
    """Mirror of _C.rasterize_gaussians (rasterize_points.cu:36-117), CPU/numpy."""
    lib = _load()
    means3D = np.ascontiguousarray(np.asarray(means3D, np.float32))
    if means3D.ndim != 2 or means3D.shape[1] != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    P = means3D.shape[0]
    H, W = int(image_height), int(image_width)
    color = np.zeros((3, H, W), np.float32)
    depth = np.zeros((1, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    if P == 0:
        return 0, color, depth, radii, None
    sh_a, sh_p = _arr(sh)
    M = sh_a.shape[1] if sh_a is not None else 0
    keep = [_arr(x) for x in (bg, colors_precomp, opacities, scales, rotations, cov3D_precomp, viewmatrix,
                              projmatrix, campos)]
    (bg_a, bg_p), (cp_a, cp_p), (op_a, op_p), (sc_a, sc_p), (ro_a, ro_p), (c3_a, c3_p), (vm_a, vm_p), \
        (pm_a, pm_p), (cam_a, cam_p) = keep
    nr = ctypes.c_int(0)
    status = ctypes.c_int(0)
    h = lib.gs4d_oracle_forward(
        P, int(degree), M, bg_p, W, H, means3D.ctypes.data_as(_f32p), sh_p, cp_p, op_p, sc_p,
        float(scale_modifier), ro_p, c3_p, vm_p, pm_p, cam_p, float(tanfovx), float(tanfovy), int(bool(prefiltered)),
        color.ctypes.data_as(_f32p), depth.ctypes.data_as(_f32p), radii.ctypes.data_as(_i32p), ctypes.byref(nr),
        ctypes.byref(status))
    state = OracleState(h, P, W, H)
    if status.value != 0:
        raise RuntimeError("Point is filtered although prefiltered is set. This shouldn't happen!")
    return nr.value, color, depth, radii, state


def rasterize_backward(state, bg, means3D, radii, colors_precomp, scales, rotations, scale_modifier, cov3D_precomp,
                       viewmatrix, projmatrix, tanfovx, tanfovy, dL_dout_color, sh, degree, campos):
    """Mirror of _C.rasterize_gaussians_backward (rasterize_points.cu:119-198), CPU/numpy."""
    lib = _load()
    means3D = np.ascontiguousarray(np.asarray(means3D, np.float32))
    P = means3D.shape[0]
    sh_a, sh_p = _arr(sh)
    M = sh_a.shape[1] if sh_a is not None else 0
    g = dict(
        dL_dmeans2D=np.zeros((P, 3), np.float32), dL_dconic=np.zeros((P, 4), np.float32),
        dL_dopacity=np.zeros((P, 1), np.float32), dL_dcolors=np.zeros((P, 3), np.float32),
        dL_dmeans3D=np.zeros((P, 3), np.float32), dL_dcov3D=np.zeros((P, 6), np.float32),
        dL_dsh=np.zeros((P, M, 3), np.float32), dL_dscales=np.zeros((P, 3), np.float32),
        dL_drotations=np.zeros((P, 4), np.float32))
    if P != 0:
        keep = [_arr(x) for x in (bg, colors_precomp, scales, rotations, cov3D_precomp, viewmatrix, projmatrix,
                                  campos, dL_dout_color)]
        (bg_a, bg_p), (cp_a, cp_p), (sc_a, sc_p), (ro_a, ro_p), (c3_a, c3_p), (vm_a, vm_p), (pm_a, pm_p), \
            (cam_a, cam_p), (dl_a, dl_p) = keep
        ra, rp = _arr(radii, np.int32)
        q = lambda k: g[k].ctypes.data_as(_f32p)
        lib.gs4d_oracle_backward(
            state.handle, bg_p, means3D.ctypes.data_as(_f32p), sh_p, cp_p, sc_p, float(scale_modifier), ro_p, c3_p,
            vm_p, pm_p, cam_p, float(tanfovx), float(tanfovy), rp, dl_p, q("dL_dmeans2D"), q("dL_dconic"),
            q("dL_dopacity"), q("dL_dcolors"), q("dL_dmeans3D"), q("dL_dcov3D"),
            g["dL_dsh"].ctypes.data_as(_f32p) if M > 0 else None, q("dL_dscales"), q("dL_drotations"))
    return (g["dL_dmeans2D"], g["dL_dcolors"], g["dL_dopacity"], g["dL_dmeans3D"], g["dL_dcov3D"], g["dL_dsh"],
            g["dL_dscales"], g["dL_drotations"]), g["dL_dconic"]


def flip_flags(state, band_alpha, band_T):
    """Near-threshold flags of the forward's two discrete decisions (gs4d_oracle_flip_flags): returns
    (pix_flag (H, W) uint8, gauss_flag (P,) uint8); bit 0 = alpha within band_alpha (relative) of
    1/255, bit 1 = T(1 - alpha) within band_T (relative) of 1e-4."""
    lib = _load()
    pix = np.zeros((state.H, state.W), np.uint8)
    gau = np.zeros(max(state.P, 1), np.uint8)
    if state.handle:
        lib.gs4d_oracle_flip_flags(state.handle, float(band_alpha), float(band_T), pix.ctypes.data_as(_u8p),
                                   gau.ctypes.data_as(_u8p))
    return pix, gau[:state.P]


def backward_tail(state, means3D, radii, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                  tanfovx, tanfovy, sh, degree, campos, dL_dmean2D, dL_dconic, dL_dcolor):
    """K8 + K9 (backward.cu:144-274, 346-396) from given K7 totals: dL_dmean2D (P,3), dL_dconic (P,4),
    dL_dcolor (P,3) -> (dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations).  Linear in the totals."""
    lib = _load()
    means3D = np.ascontiguousarray(np.asarray(means3D, np.float32))
    P = means3D.shape[0]
    sh_a, sh_p = _arr(sh)
    M = sh_a.shape[1] if sh_a is not None else 0
    out = dict(m=np.zeros((P, 3), np.float32), c=np.zeros((P, 6), np.float32), sh=np.zeros((P, M, 3), np.float32),
               s=np.zeros((P, 3), np.float32), r=np.zeros((P, 4), np.float32))
    if P:
        keep = [_arr(x) for x in (scales, rotations, cov3D_precomp, viewmatrix, projmatrix, campos, dL_dmean2D,
                                  dL_dconic, dL_dcolor)]
        (sc_a, sc_p), (ro_a, ro_p), (c3_a, c3_p), (vm_a, vm_p), (pm_a, pm_p), (cam_a, cam_p), (m2_a, m2_p), \
            (cn_a, cn_p), (cl_a, cl_p) = keep
        ra, rp = _arr(radii, np.int32)
        q = lambda k: out[k].ctypes.data_as(_f32p)
        lib.gs4d_oracle_backward_tail(state.handle, means3D.ctypes.data_as(_f32p), sh_p, sc_p, float(scale_modifier),
                                      ro_p, c3_p, vm_p, pm_p, cam_p, float(tanfovx), float(tanfovy), rp, m2_p, cn_p,
                                      cl_p, q("m"), q("c"), out["sh"].ctypes.data_as(_f32p) if M > 0 else None, q("s"),
                                      q("r"))
    return out["m"], out["c"], out["sh"], out["s"], out["r"]


def flip_bounds(state, band_alpha, band_T, bg, means3D, radii, colors_precomp, scales, rotations, scale_modifier,
                cov3D_precomp, viewmatrix, projmatrix, tanfovx, tanfovy, dL_dout_color, sh, degree, campos):
    """Near-threshold flags AND bounds (gs4d_oracle_flip_bounds): every decision of the forward within
    band_alpha of 1/255 or band_T of 1e-4 (relative) is replayed the other way, pixel by pixel, and the
    differences it makes are summed.  The arguments after the bands are rasterize_backward's.  Returns a dict:
      pflag (H, W) / gflag (P,)  bit 0 near-1/255, bit 1 near-termination (pixels; the Gaussians whose own
                                 decision it is)
      pix_rad, depth_rad (H, W)  bound on |colour| (max over channels) and |depth| changes at the pixel
      grad_rad                   8-tuple aligned with rasterize_backward's outputs: per-element bounds on the
                                 gradient changes, the K7 terms' bounds carried through the (linear) K8 + K9
                                 by their absolute values (sum_j |M e_j| r_j >= |M r| for every r in the box)."""
    lib = _load()
    means3D = np.ascontiguousarray(np.asarray(means3D, np.float32))
    P = means3D.shape[0]
    H, W = state.H, state.W
    pflag = np.zeros((H, W), np.uint8)
    gflag = np.zeros(max(P, 1), np.uint8)
    pix_rad = np.zeros((H, W), np.float32)
    depth_rad = np.zeros((H, W), np.float32)
    rad9 = np.zeros((max(P, 1), 9), np.float64)
    if state is not None and state.handle:
        bg_a, bg_p = _arr(bg)
        cp_a, cp_p = _arr(colors_precomp)
        dl_a, dl_p = _arr(dL_dout_color)
        lib.gs4d_oracle_flip_bounds(state.handle, bg_p, cp_p, dl_p, float(band_alpha), float(band_T),
                                    pflag.ctypes.data_as(_u8p), gflag.ctypes.data_as(_u8p),
                                    pix_rad.ctypes.data_as(_f32p), depth_rad.ctypes.data_as(_f32p),
                                    rad9.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    rad9 = rad9[:P]
    gflag = gflag[:P]
    sh_a = None if sh is None else np.asarray(sh)
    M = sh_a.shape[1] if sh_a is not None and sh_a.size else 0
    r_m2 = np.zeros((P, 3), np.float32)
    r_m2[:, :2] = rad9[:, :2]
    r_col = rad9[:, 6:9].astype(np.float32)
    r_op = rad9[:, 5:6].astype(np.float32)
    r_m3, r_c3, r_sh, r_s, r_r = (np.zeros((P, 3)), np.zeros((P, 6)), np.zeros((P, M, 3)), np.zeros((P, 3)),
                                  np.zeros((P, 4)))
    live = rad9.any(1)
    if live.any():
        rad_in = np.where(live, np.asarray(radii, np.int32), 0).astype(np.int32)  # the tail skips radius-0 rows
        for j in (0, 1, 2, 3, 4, 6, 7, 8):
            col = rad9[:, j].astype(np.float32)
            if not col.any():
                continue
            m2, cn, cl = np.zeros((P, 3), np.float32), np.zeros((P, 4), np.float32), np.zeros((P, 3), np.float32)
            if j < 2:
                m2[:, j] = col
            elif j < 5:
                cn[:, (0, 1, 3)[j - 2]] = col
            else:
                cl[:, j - 6] = col
            outs = backward_tail(state, means3D, rad_in, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                                 projmatrix, tanfovx, tanfovy, sh, degree, campos, m2, cn, cl)
            for acc, o in zip((r_m3, r_c3, r_sh, r_s, r_r), outs):
                acc += np.abs(o.astype(np.float64)).reshape(acc.shape)
    grad_rad = (r_m2, r_col, r_op, r_m3.astype(np.float32), r_c3.astype(np.float32), r_sh.astype(np.float32),
                r_s.astype(np.float32), r_r.astype(np.float32))
    return dict(pflag=pflag, gflag=gflag, pix_rad=pix_rad, depth_rad=depth_rad, grad_rad=grad_rad)


def near_pairs(state, band, kind=1, max_n=1 << 22):
    """(gid, px, py, o G, mag) of every forward-walk pair near a threshold (gs4d_oracle_near_pairs), in no
    particular order: kind 1, alpha within `band` x mag (relative) of 1/255, mag = 1 + the magnitude of the
    power's terms (near_alpha); kind 2, a blended splat whose T(1 - alpha) lies within `band` (relative) of
    1e-4."""
    lib = _load()
    gid, px, py = (np.zeros(max_n, np.int32) for _ in range(3))
    og, mag = np.zeros(max_n, np.float32), np.zeros(max_n, np.float32)
    n = lib.gs4d_oracle_near_pairs(state.handle, int(kind), float(band), int(max_n), gid.ctypes.data_as(_i32p),
                                   px.ctypes.data_as(_i32p), py.ctypes.data_as(_i32p), og.ctypes.data_as(_f32p),
                                   mag.ctypes.data_as(_f32p))
    if n > max_n:
        raise RuntimeError(f"near_pairs: {n} pairs, more than max_n = {max_n}")
    return gid[:n], px[:n], py[:n], og[:n], mag[:n]


def sh_forward(degree, means, campos, shs):
    """forward.cu:20-71 for every Gaussian: returns (rgb (P,3) float32, clamped (P,) uint8 bitmask)."""
    lib = _load()
    means = np.ascontiguousarray(np.asarray(means, np.float32))
    shs = np.ascontiguousarray(np.asarray(shs, np.float32))
    campos = np.ascontiguousarray(np.asarray(campos, np.float32))
    P, M = shs.shape[0], shs.shape[1]
    rgb = np.zeros((P, 3), np.float32)
    cl = np.zeros(P, np.uint8)
    lib.gs4d_oracle_sh_forward(P, int(degree), M, means.ctypes.data_as(_f32p), campos.ctypes.data_as(_f32p),
                               shs.ctypes.data_as(_f32p), rgb.ctypes.data_as(_f32p), cl.ctypes.data_as(_u8p))
    return rgb, cl


def mark_visible(means3D, viewmatrix, projmatrix):
    lib = _load()
    means3D = np.ascontiguousarray(np.asarray(means3D, np.float32))
    P = means3D.shape[0]
    out = np.zeros(P, np.uint8)
    if P:
        vm, vp = _arr(viewmatrix)
        pm, pp = _arr(projmatrix)
        lib.gs4d_oracle_mark_visible(P, means3D.ctypes.data_as(_f32p), vp, pp, out.ctypes.data_as(_u8p))
    return out.astype(bool)


def knn_mean_dist(points):
    """Mirror of simple_knn._C.distCUDA2 (submodules/simple-knn/spatial.cu:15-25) -- knn_oracle.c."""
    lib = _load()
    pts = np.ascontiguousarray(np.asarray(points, np.float32))
    if pts.ndim != 2 or pts.shape[1] != 3:
        raise RuntimeError("points must have dimensions (num_points, 3)")
    out = np.zeros(pts.shape[0], np.float32)
    lib.gs4d_oracle_knn(pts.shape[0], pts.ctypes.data_as(_f32p), out.ctypes.data_as(_f32p))
    return out
