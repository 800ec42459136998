"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU restatement (oracle/nori_oracle.cpp).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / reported CPU baseline. See nori_oracle.h for what pins this oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "optix-renderer_amd"))
import nori_hip as nh  # noqa: E402  (struct layouts of the shared scene description)

LIB_PATH = os.path.join(_HERE, "_build", "libnori_oracle.so")
_lib = C.CDLL(LIB_PATH)

PER_PATH, NORI_BLOCK = 0, 1
LENS_SERIAL = 0x100  # or into `mode`: lens samples from one sequential stream in the serial loop (nori_oracle.h)
PCG32_DEFAULT_STATE = 0x853C49E6748FEA9B
PCG32_DEFAULT_STREAM = 0xDA3E39CB94B95BDB

_vp, _i32, _u32, _u64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64
_fp = C.POINTER(C.c_float)
_u64p = C.POINTER(C.c_uint64)


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)


_sig("no_scene_create", _i32, C.POINTER(nh.nh_scene_desc), C.POINTER(_vp))
_sig("no_scene_free", None, _vp)
_sig("no_bvh_info", _i32, _vp, C.POINTER(_u32), C.POINTER(_u32))
_sig("no_env_cdf", _i32, _vp, C.POINTER(_fp), C.POINTER(_u32), C.POINTER(C.c_float))
_sig("no_bvh_export", _i32, _vp, C.POINTER(nh.nh_bvh_node), C.POINTER(_u32))
_sig("no_trace_rays", _i32, _vp, C.POINTER(nh.nh_ray_soa), _i32, _i32, C.POINTER(nh.nh_hit_soa))
_sig("no_pcg32_seed", None, _u64p, _u64p, _u64, _u64)
_sig("no_pcg32_next", _u32, _u64p, _u64p)
_sig("no_path_seed", None, _u64, _u64, _u64, _u64p, _u64p)
_sig("no_render", _i32, _vp, _i32, _u64, _i32, _i32, C.POINTER(_i32), _i32, _i32, _fp, _u64p)
_sig("no_path_radiance", _i32, _vp, _u64, _i32, _i32, _i32, _fp, _fp)
_sig("no_ttest_scene", _i32, _vp, _u64p, _u64p, _i32, C.POINTER(C.c_double), C.POINTER(C.c_double))
_sig("no_ttest_bsdf", _i32, C.POINTER(nh.nh_bsdf), C.c_float, _u64p, _u64p, _i32, C.POINTER(C.c_double),
     C.POINTER(C.c_double))
_sig("no_bsdf_sample", _i32, C.POINTER(nh.nh_bsdf), _fp, _fp, _fp, _fp, _fp, C.POINTER(_i32))
_sig("no_bsdf_pdf", C.c_float, C.POINTER(nh.nh_bsdf), _fp, _fp)
_sig("no_texture_eval", _i32, _vp, _u32, _i32, _fp, _fp, _fp)
_sig("no_bsdf_pdf_batch", _i32, C.POINTER(nh.nh_bsdf), _fp, _i32, _fp, _fp)
_sig("no_eigen_ops", _i32, _i32, _fp, _fp)
_sig("no_normal_ops", _i32, _i32, _fp, _fp)
_sig("no_denoise_simple", _i32, _fp, _i32, _i32, _i32, C.POINTER(nh.nh_denoiser))
_sig("no_chi2_histogram", _i32, C.POINTER(nh.nh_bsdf), _fp, _u64p, _u64p, _i32, _i32, _i32, C.POINTER(C.c_double))


class Pcg32:
    """pcg32 restatement handle (state/inc live on the Python side)."""

    def __init__(self, state=PCG32_DEFAULT_STATE, inc=PCG32_DEFAULT_STREAM):
        self.state, self.inc = _u64(state), _u64(inc)

    @classmethod
    def seeded(cls, initstate, initseq=1):
        r = cls()
        _lib.no_pcg32_seed(C.byref(r.state), C.byref(r.inc), initstate, initseq)
        return r

    @classmethod
    def per_path(cls, seed, pixel, sample):
        r = cls()
        _lib.no_path_seed(seed, pixel, sample, C.byref(r.state), C.byref(r.inc))
        return r

    def next_uint(self):
        return _lib.no_pcg32_next(C.byref(self.state), C.byref(self.inc))

    def next_float(self):
        u = (self.next_uint() >> 9) | 0x3F800000
        return float(np.array([u], np.uint32).view(np.float32)[0] - np.float32(1.0))


class OracleScene:
    def __init__(self, scene: "nh.Scene"):
        self._keep = scene
        d = scene.desc
        h = _vp()
        if _lib.no_scene_create(C.byref(d), C.byref(h)) != 0:
            raise RuntimeError("oracle scene creation failed")
        self._h = h
        self.width, self.height, self.border = d.camera.width, d.camera.height, d.filter.border

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.no_scene_free(self._h)
            self._h = None

    def bvh(self):
        nn, ni = _u32(), _u32()
        _lib.no_bvh_info(self._h, C.byref(nn), C.byref(ni))
        nodes = (nh.nh_bvh_node * max(nn.value, 1))()
        idx = np.zeros(ni.value, np.uint32)
        _lib.no_bvh_export(self._h, nodes, idx.ctypes.data_as(C.POINTER(_u32)))
        raw = np.ctypeslib.as_array(C.cast(nodes, C.POINTER(C.c_uint32)), shape=(max(nn.value, 1) * 8,))
        return raw.reshape(-1, 8)[: nn.value].copy(), idx

    def env_cdf(self):
        """The oracle's own EnvMap::calculateProbs CDF and normalization (None without an envmap)."""
        p, n, norm = _fp(), _u32(), C.c_float()
        if _lib.no_env_cdf(self._h, C.byref(p), C.byref(n), C.byref(norm)) != 0:
            return None
        return np.ctypeslib.as_array(p, shape=(n.value,)).copy(), norm.value

    def texture_eval(self, texture: int, u, v):
        """Albedo texture `texture` (1-based, nh_bsdf.albedo_texture) at the uv pairs: (n, 3) float32."""
        u = np.ascontiguousarray(u, dtype=np.float32)
        v = np.ascontiguousarray(v, dtype=np.float32)
        out = np.zeros((len(u), 3), np.float32)
        if _lib.no_texture_eval(self._h, texture, len(u), u.ctypes.data_as(_fp), v.ctypes.data_as(_fp),
                                out.ctypes.data_as(_fp)) != 0:
            raise RuntimeError("no_texture_eval failed")
        return out

    def trace(self, o, d, mint, maxt, any_hit=False):
        n = len(o)
        cols = [np.ascontiguousarray(x, dtype=np.float32) for x in (o[:, 0], o[:, 1], o[:, 2], d[:, 0], d[:, 1],
                                                                     d[:, 2], mint, maxt)]
        r = nh.nh_ray_soa(*[c.ctypes.data_as(_fp) for c in cols])
        res = {"hit": np.zeros(n, np.uint8), "t": np.zeros(n, np.float32), "u": np.zeros(n, np.float32),
               "v": np.zeros(n, np.float32), "prim": np.zeros(n, np.uint32), "shape": np.zeros(n, np.uint32)}
        h = nh.nh_hit_soa(res["hit"].ctypes.data_as(C.POINTER(C.c_uint8)), res["t"].ctypes.data_as(_fp),
                          res["u"].ctypes.data_as(_fp), res["v"].ctypes.data_as(_fp),
                          res["prim"].ctypes.data_as(C.POINTER(_u32)), res["shape"].ctypes.data_as(C.POINTER(_u32)))
        _lib.no_trace_rays(self._h, C.byref(r), n, int(any_hit), C.byref(h))
        return res

    def render(self, s0, s1, seed=0, mode=PER_PATH, blocks=None, threads=None, rgbw=None):
        if rgbw is None:
            rgbw = np.zeros((self.height + 2 * self.border, self.width + 2 * self.border, 4), np.float32)
        threads = threads or os.cpu_count() or 1
        nb, bp = 0, None
        keep = None
        if blocks is not None:
            keep = np.ascontiguousarray(blocks, np.int32)
            nb, bp = len(keep), keep.ctypes.data_as(C.POINTER(_i32))
        inv = _u64()
        rc = _lib.no_render(self._h, mode, seed, s0, s1, bp, nb, threads, rgbw.ctypes.data_as(_fp), C.byref(inv))
        if rc != 0:
            raise RuntimeError(f"oracle render failed ({rc})")
        self.last_invalid = inv.value
        return rgbw

    def path(self, seed, px, py, sample):
        rgb, jit = np.zeros(3, np.float32), np.zeros(2, np.float32)
        _lib.no_path_radiance(self._h, seed, px, py, sample, rgb.ctypes.data_as(_fp), jit.ctypes.data_as(_fp))
        return rgb, jit

    def ttest(self, rng: Pcg32, n: int):
        m, v = C.c_double(), C.c_double()
        _lib.no_ttest_scene(self._h, C.byref(rng.state), C.byref(rng.inc), n, C.byref(m), C.byref(v))
        return m.value, v.value


def ttest_bsdf(bsdf: "nh.nh_bsdf", angle_deg: float, rng: Pcg32, n: int):
    m, v = C.c_double(), C.c_double()
    _lib.no_ttest_bsdf(C.byref(bsdf), angle_deg, C.byref(rng.state), C.byref(rng.inc), n, C.byref(m), C.byref(v))
    return m.value, v.value


def bsdf_sample(bsdf, wi, sample):
    wi = np.asarray(wi, np.float32)
    s = np.asarray(sample, np.float32)
    wo, w, pdf, meas = np.zeros(3, np.float32), np.zeros(3, np.float32), C.c_float(), _i32()
    _lib.no_bsdf_sample(C.byref(bsdf), wi.ctypes.data_as(_fp), s.ctypes.data_as(_fp), wo.ctypes.data_as(_fp),
                        w.ctypes.data_as(_fp), C.byref(pdf), C.byref(meas))
    return wo, w, pdf.value, meas.value


def bsdf_pdf(bsdf, wi, wo):
    wi = np.asarray(wi, np.float32)
    wo = np.asarray(wo, np.float32)
    return _lib.no_bsdf_pdf(C.byref(bsdf), wi.ctypes.data_as(_fp), wo.ctypes.data_as(_fp))


def bsdf_pdf_batch(bsdf, wi, wo):
    wi = np.ascontiguousarray(wi, np.float32)
    wo = np.ascontiguousarray(wo, np.float32).reshape(-1, 3)
    out = np.zeros(len(wo), np.float32)
    _lib.no_bsdf_pdf_batch(C.byref(bsdf), wi.ctypes.data_as(_fp), len(wo), wo.ctypes.data_as(_fp),
                           out.ctypes.data_as(_fp))
    return out


def chi2_histogram(bsdf, wi, rng: Pcg32, n, res_theta, res_phi):
    wi = np.ascontiguousarray(wi, np.float32)
    obs = np.zeros(res_theta * res_phi, np.float64)
    _lib.no_chi2_histogram(C.byref(bsdf), wi.ctypes.data_as(_fp), C.byref(rng.state), C.byref(rng.inc), n, res_theta,
                           res_phi, obs.ctypes.data_as(C.POINTER(C.c_double)))
    return obs


def denoise_simple(rgbw, border: int, params) -> np.ndarray:
    """SimpleDenoiser (src/denoiser/simple.cpp:29-76), serial row-major order, on a copy of a
    (H+2b, W+2b, 4) float32 ImageBlock. params: nori_hip.nh_denoiser."""
    out = np.array(rgbw, dtype=np.float32, order="C", copy=True)
    h, w = out.shape[0] - 2 * border, out.shape[1] - 2 * border
    if _lib.no_denoise_simple(out.ctypes.data_as(_fp), w, h, border, C.byref(params)) != 0:
        raise RuntimeError("no_denoise_simple: invalid arguments")
    return out


def normal_ops(cases):
    """The oracle's normal-map arithmetic (no_normal_ops) on (n, 13) float32 cases -> (n, 15)."""
    cases = np.ascontiguousarray(cases, np.float32)
    out = np.zeros((len(cases), 15), np.float32)
    _lib.no_normal_ops(len(cases), cases.ctypes.data_as(_fp), out.ctypes.data_as(_fp))
    return out


def eigen_ops(cases):
    """The oracle's restated Eigen arithmetic (no_eigen_ops) on (n, 36) float32 cases -> (n, 28)."""
    cases = np.ascontiguousarray(cases, np.float32)
    out = np.zeros((len(cases), 28), np.float32)
    _lib.no_eigen_ops(len(cases), cases.ctypes.data_as(_fp), out.ctypes.data_as(_fp))
    return out
