"""Python binding of the nori_hip C-ABI (include/nori_hip.h) via ctypes.

This is the host-side mirror of the reference's render entry points for tests and the
benchmark: `Scene` ~ loadFromXML + Scene::cloneAndInit/update
(src/utils/parser.cpp:28-378, src/utils/scene.cpp:59-202), `Bvh` ~ BVH::build
(src/utils/bvh.cpp:327-380), `Context.render` ~ RenderThread::renderThreadMain over a
sample range (src/utils/render.cpp:232-459), `Context.trace` ~ Scene::rayIntersect
(include/nori/scene.h:114-137).

The library is the in-tree build optix-renderer_amd/lib/libnori_hip.so. There is no
fallback: if it is missing, importing raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NH_LIB_PATH: an alternative in-tree build, for A/B measurements in one GPU session
LIB_PATH = os.environ.get("NH_LIB_PATH") or os.path.join(_HERE, "lib", "libnori_hip.so")

from nh_env import raise_hw_queues  # noqa: E402  (nori_hip's own directory is on sys.path)

if not os.path.exists(LIB_PATH):
    raise ImportError(f"nori_hip: HIP library not built ({LIB_PATH}); run `make` or __graft_entry__.build()")
_lib = C.CDLL(LIB_PATH)

NH_OK = 0
SHAPE_MESH, SHAPE_SPHERE = 0, 1
BSDF_DIFFUSE, BSDF_MIRROR, BSDF_DIELECTRIC, BSDF_MICROFACET = 0, 1, 2, 3
EMITTER_AREA, EMITTER_POINT, EMITTER_ENVMAP = 0, 1, 2
INTEGRATOR_PATH_MIS, INTEGRATOR_PATH_MATS, INTEGRATOR_DIRECT_EMS, INTEGRATOR_DIRECT_MATS, INTEGRATOR_DIRECT_MIS = 0, 1, 2, 3, 4
INTEGRATOR_DIRECT = 5  # the point-light `direct` integrator of scenes/pa1 (direct.cpp)
INTEGRATOR_NORMALS = 6  # the `normals` integrator of the normal-map scenes (normals.cpp)
MODE_MEGAKERNEL, MODE_WAVEFRONT = 0, 1
TRAVERSAL_REFERENCE, TRAVERSAL_ORDERED, TRAVERSAL_WIDE = 0, 1, 2
DENOISER_NONE, DENOISER_SIMPLE = 0, 1
LENS_DRAWS_LTR, LENS_DRAWS_RTL = 0, 1

_f = C.c_float
_i32 = C.c_int32
_u32 = C.c_uint32
_fp = C.POINTER(C.c_float)
_u32p = C.POINTER(C.c_uint32)


class nh_shape(C.Structure):
    _fields_ = [("type", _i32), ("bsdf", _i32), ("emitter", _i32), ("v_offset", _u32), ("n_vertices", _u32),
                ("f_offset", _u32), ("n_faces", _u32), ("has_normals", _i32), ("has_uvs", _i32),
                ("center", _f * 3), ("radius", _f), ("bbox_min", _f * 3), ("bbox_max", _f * 3),
                ("pdf_offset", _u32), ("pdf_normalization", _f), ("normal_map", _u32)]


class nh_bsdf(C.Structure):
    _fields_ = [("type", _i32), ("albedo", _f * 3), ("alpha", _f), ("int_ior", _f), ("ext_ior", _f),
                ("kd", _f * 3), ("ks", _f), ("albedo_texture", _u32)]


TEXTURE_CONSTANT, TEXTURE_CHECKERBOARD, TEXTURE_PNG = 0, 1, 2


class nh_texture(C.Structure):
    _fields_ = [("type", _i32), ("value1", _f * 3), ("value2", _f * 3), ("delta", _f * 2), ("scale", _f * 2),
                ("width", _i32), ("height", _i32), ("texel_offset", C.c_uint64), ("scale_u", _f), ("scale_v", _f),
                ("offset_u", _f), ("offset_v", _f), ("spherical", _i32), ("rotation", _f * 9), ("linear", _i32),
                ("intensity", _f), ("pad", _i32)]


class nh_emitter(C.Structure):
    _fields_ = [("type", _i32), ("shape", _i32), ("radiance", _f * 3), ("light_prob", _f),
                ("position", _f * 3), ("pad", _f)]


class nh_camera(C.Structure):
    _fields_ = [("width", _i32), ("height", _i32), ("sample_to_camera", _f * 16), ("camera_to_world", _f * 16),
                ("inv_output_size", _f * 2), ("near_clip", _f), ("far_clip", _f), ("lens_radius", _f),
                ("focal_distance", _f), ("lens_draw_order", _i32)]


class nh_filter(C.Structure):
    _fields_ = [("radius", _f), ("border", _i32), ("lookup_factor", _f), ("table", _f * 33)]


class nh_envmap(C.Structure):
    _fields_ = [("width", _i32), ("height", _i32), ("rgba", _fp), ("radiance", _f * 3), ("scale_u", _f),
                ("scale_v", _f), ("offset_u", _f), ("offset_v", _f), ("spherical", _i32), ("constant", _i32),
                ("cdf", _fp), ("normalization", _f), ("rotation", _f * 9)]


class nh_denoiser(C.Structure):
    _fields_ = [("type", _i32), ("sigma_d", _f), ("sigma_vr", _f), ("range", _i32), ("amount", _i32)]


def simple_denoiser(sigma_d: float = 0.0, sigma_vr: float = 0.6, range: int = 1, amount: int = 1) -> nh_denoiser:
    """SimpleDenoiser's parameters with its constructor's defaults and clamps (src/denoiser/simple.cpp:15-24,
    Nori's clamp and Epsilon = 1e-4f)."""
    eps = np.float32(1e-4)

    def clampf(v, lo, hi):
        v = np.float32(v)
        return float(lo if v < lo else (hi if v > hi else v))
    d = nh_denoiser()
    d.type = DENOISER_SIMPLE
    d.sigma_d = clampf(sigma_d, eps, np.float32(10))
    d.sigma_vr = clampf(sigma_vr, eps, np.float32(10))
    d.range = int(min(max(range, 0), 50))
    d.amount = int(min(max(amount, 1), 10))
    return d


class nh_scene_desc(C.Structure):
    _fields_ = [("camera", nh_camera), ("filter", nh_filter), ("integrator", _i32), ("sample_count", _i32),
                ("n_shapes", _u32), ("shapes", C.POINTER(nh_shape)), ("n_bsdfs", _u32),
                ("bsdfs", C.POINTER(nh_bsdf)), ("n_emitters", _u32), ("emitters", C.POINTER(nh_emitter)),
                ("emitter_cdf", _fp), ("envmap", _i32), ("n_vertices", _u32), ("V", _fp), ("N", _fp),
                ("UV", _fp), ("T", _fp), ("BT", _fp), ("n_faces", _u32), ("F", _u32p), ("n_area_cdf", _u32),
                ("area_cdf", _fp), ("env", nh_envmap), ("denoiser", nh_denoiser), ("n_textures", _u32),
                ("textures", C.POINTER(nh_texture)), ("n_texels", C.c_uint64), ("texels", _fp),
                ("normals_direction", _f * 3)]


class nh_bvh_node(C.Structure):
    _fields_ = [("word0", _u32), ("word1", _u32), ("bbox_min", _f * 3), ("bbox_max", _f * 3)]


class nh_bvh_desc(C.Structure):
    _fields_ = [("n_nodes", _u32), ("nodes", C.POINTER(nh_bvh_node)), ("n_indices", _u32), ("indices", _u32p),
                ("n_shapes", _u32), ("shape_offset", _u32p), ("bbox_min", _f * 3), ("bbox_max", _f * 3),
                ("max_depth", _u32)]


class nh_ray_soa(C.Structure):
    _fields_ = [(n, _fp) for n in ("ox", "oy", "oz", "dx", "dy", "dz", "mint", "maxt")]


class nh_hit_soa(C.Structure):
    _fields_ = [("hit", C.POINTER(C.c_uint8)), ("t", _fp), ("u", _fp), ("v", _fp), ("prim", _u32p),
                ("shape", _u32p)]


class nh_render_req(C.Structure):
    _fields_ = [("sample_begin", _i32), ("sample_end", _i32), ("seed", C.c_uint64), ("n_blocks", _i32),
                ("blocks", C.POINTER(_i32)), ("mode", _i32), ("traversal", _i32), ("clear", _i32),
                ("collect_stats", _i32)]


class nh_render_stats(C.Structure):
    _fields_ = [("kernel_ms_path", C.c_double), ("kernel_ms_splat", C.c_double), ("kernel_ms_extend", C.c_double),
                ("kernel_ms_shadow", C.c_double), ("kernel_ms_shade", C.c_double), ("launches_path", C.c_uint64),
                ("launches_splat", C.c_uint64), ("launches_extend", C.c_uint64), ("launches_shadow", C.c_uint64),
                ("launches_shade", C.c_uint64), ("samples", C.c_uint64), ("ray_queries", C.c_uint64),
                ("nodes_visited", C.c_uint64), ("boxes_tested", C.c_uint64), ("prims_tested", C.c_uint64),
                ("invalid_samples", C.c_uint64), ("shadow_queries", C.c_uint64),
                ("shadow_nodes_visited", C.c_uint64), ("shadow_boxes_tested", C.c_uint64),
                ("shadow_prims_tested", C.c_uint64), ("shade_state_bytes", C.c_uint64),
                ("extend_queue_bytes", C.c_uint64), ("shadow_queue_bytes", C.c_uint64),
                ("paths_shaded", C.c_uint64), ("kernel_ms_tail", C.c_double), ("launches_tail", C.c_uint64),
                ("node_bytes", C.c_uint64)] + [
        (n, C.c_uint64) for n in ("tail_queries", "tail_nodes_visited", "tail_boxes_tested", "tail_prims_tested",
                                  "tail_shadow_queries", "tail_shadow_nodes_visited", "tail_shadow_boxes_tested",
                                  "tail_shadow_prims_tested", "lds_scene", "fused_bounce", "comm_inits")] + [
        ("kernel_ms_denoise", C.c_double), ("launches_denoise", C.c_uint64), ("tails_async", C.c_uint64),
        ("pools_active", C.c_uint64), ("trace_fused", C.c_uint64)] + [
        (n, C.c_uint64) for n in ("tail_cycles_body", "tail_cycles_shadow", "tail_cycles_closest", "tail_cycles_head",
                                  "tail_bounces", "tail_max_bounces", "tail_coop_cycles_body",
                                  "tail_coop_cycles_shadow", "tail_coop_cycles_closest", "tail_coop_cycles_head",
                                  "tail_coop_bounces", "bounce_cycles_load", "bounce_cycles_body",
                                  "bounce_cycles_shadow", "bounce_cycles_closest", "bounce_cycles_head",
                                  "bounce_cycles_store", "bounce_bounces")]


def _sig(name, res, *args):
    fn = getattr(_lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_vp = C.c_void_p
_sig("nh_scene_load_xml", _i32, C.c_char_p, C.POINTER(_vp))
_sig("nh_scene_load_xml_index", _i32, C.c_char_p, _i32, C.POINTER(_vp))
_sig("nh_scene_get_desc", _i32, _vp, C.POINTER(nh_scene_desc))
_sig("nh_scene_set_resolution", _i32, _vp, _i32, _i32)
_sig("nh_scene_set_sample_count", _i32, _vp, _i32)
_sig("nh_scene_set_bsdf", _i32, _vp, _u32, C.POINTER(nh_bsdf))
_sig("nh_scene_set_integrator", _i32, _vp, _i32)
_sig("nh_scene_add_texture", _u32, _vp, C.POINTER(nh_texture), _fp)
_sig("nh_scene_set_normal_map", _i32, _vp, _u32, _u32)
_sig("nh_scene_set_lens_draw_order", _i32, _vp, _i32)
_sig("nh_texture_decode", _i32, C.POINTER(C.c_uint8), C.c_uint64, _i32, _fp)
_sig("nh_scene_free", None, _vp)
_sig("nh_host_last_error", C.c_char_p)
_sig("nh_debug_transform", _i32, C.c_char_p, _fp, _i32)
_sig("nh_bvh_build", _i32, C.POINTER(nh_scene_desc), _i32, C.POINTER(_vp))
_sig("nh_bvh_get_desc", _i32, _vp, C.POINTER(nh_bvh_desc))
_sig("nh_bvh_free", None, _vp)
_sig("nh_framebuffer_to_rgb", _i32, _fp, _i32, _i32, _i32, _fp)
_sig("nh_write_pfm", _i32, C.c_char_p, _fp, _i32, _i32)
_sig("nh_image_load_png", _i32, C.c_char_p, C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(_i32), C.POINTER(_i32))
_sig("nh_write_exr", _i32, C.c_char_p, _fp, _i32, _i32)
_sig("nh_write_png", _i32, C.c_char_p, _fp, _i32, _i32)
_sig("nh_rgb_to_ldr", _i32, _fp, _i32, _i32, C.POINTER(C.c_uint8))
_sig("nh_get_device_count", _i32, C.POINTER(C.c_int))
_sig("nh_create", _i32, C.c_int, C.POINTER(_vp))
_sig("nh_destroy", None, _vp)
_sig("nh_upload_scene", _i32, _vp, C.POINTER(nh_scene_desc))
_sig("nh_upload_bvh", _i32, _vp, C.POINTER(nh_bvh_desc))
_sig("nh_trace_rays", _i32, _vp, C.POINTER(nh_ray_soa), _i32, _i32, _i32, C.POINTER(nh_hit_soa))
_sig("nh_render", _i32, _vp, C.POINTER(nh_render_req))
_sig("nh_synchronize", _i32, _vp)
_sig("nh_get_framebuffer", _i32, _vp, _fp, C.c_size_t)
_sig("nh_framebuffer_device_ptr", _i32, _vp, C.POINTER(_vp), C.POINTER(C.c_size_t))
_sig("nh_get_stats", _i32, _vp, C.POINTER(nh_render_stats))
_sig("nh_reset_stats", _i32, _vp)
_sig("nh_reduce_framebuffers", _i32, C.POINTER(_vp), _i32, _i32)
_sig("nh_denoise", _i32, _vp, C.POINTER(nh_denoiser))
_sig("nh_denoise_image", _i32, _vp, _fp, _i32, _i32, _i32, C.POINTER(nh_denoiser))
_sig("nh_last_error", C.c_char_p, _vp)

lib = _lib
_hip_used = False  # set by the first call that initialises the HIP runtime (device_count, Context)


def configure_runtime(min_hw_queues: int = 8) -> int:
    """Process settings the HIP runtime reads once, when it initialises: GPU_MAX_HW_QUEUES raised to min_hw_queues
    (one hardware queue per path-pool stream, nh_env.py) unless a larger value is set or NH_KEEP_HW_QUEUES keeps the
    caller's. An explicit call, not an import side effect; it must come before the first device_count() / Context().
    Returns the value the runtime will see."""
    if _hip_used:
        raise RuntimeError("configure_runtime: the HIP runtime is already initialised in this process")
    return raise_hw_queues(min_hw_queues)


class NoriError(RuntimeError):
    pass


def _fptr(a):
    return a.ctypes.data_as(_fp)


def _host_check(rc, what):
    if rc != NH_OK:
        raise NoriError(f"{what}: {_lib.nh_host_last_error().decode()}")


class Scene:
    """A loaded Nori XML scene (host-owned flattened arrays)."""

    def __init__(self, path: str, index: int = 0):
        h = _vp()
        _host_check(_lib.nh_scene_load_xml_index(path.encode(), index, C.byref(h)), f"load {path}")
        self._h = h
        self.path = path

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.nh_scene_free(self._h)
            self._h = None

    @property
    def desc(self) -> nh_scene_desc:
        d = nh_scene_desc()
        _host_check(_lib.nh_scene_get_desc(self._h, C.byref(d)), "get_desc")
        return d

    def set_resolution(self, w: int, h: int):
        _host_check(_lib.nh_scene_set_resolution(self._h, w, h), "set_resolution")

    def set_sample_count(self, spp: int):
        _host_check(_lib.nh_scene_set_sample_count(self._h, spp), "set_sample_count")

    def set_integrator(self, integ: int):
        _host_check(_lib.nh_scene_set_integrator(self._h, integ), "set_integrator")

    def set_bsdf(self, shape: int, **kw):
        b = nh_bsdf()
        b.type = kw.get("type", BSDF_DIFFUSE)
        for i, v in enumerate(kw.get("albedo", (0.5, 0.5, 0.5))):
            b.albedo[i] = v
        b.alpha = kw.get("alpha", 0.1)
        b.int_ior = kw.get("int_ior", 1.5046)
        b.ext_ior = kw.get("ext_ior", 1.000277)
        kd = kw.get("kd", (0.5, 0.5, 0.5))
        for i, v in enumerate(kd):
            b.kd[i] = v
        kdf = np.asarray(kd, dtype=np.float32)
        m = kdf[1] if not (kdf[1] < kdf[2]) else kdf[2]
        m = kdf[0] if not (kdf[0] < m) else m
        b.ks = float(np.float32(1) - np.float32(m))
        b.albedo_texture = kw.get("albedo_texture", 0)
        _host_check(_lib.nh_scene_set_bsdf(self._h, shape, C.byref(b)), "set_bsdf")

    def add_texture(self, type: int, value1=(0, 0, 0), value2=(1, 1, 1), delta=(0, 0), scale=(1, 1), texels=None,
                    scale_uv=(1, 1), offset_uv=(0, 0), spherical=False, linear=False, intensity=1.0) -> int:
        """Append a texture (nh_scene_add_texture); returns the value naming it in nh_bsdf.albedo_texture or
        nh_shape.normal_map (set_normal_map). texels: (H, W, 4) float32 RGBA for TEXTURE_PNG, already decoded
        (texture_decode), row 0 first; linear: sRGB = false (normal-map texels, eval blends by intensity)."""
        t = nh_texture()
        t.type = type
        t.linear = int(linear)
        t.intensity = intensity
        for i in range(3):
            t.value1[i], t.value2[i] = value1[i], value2[i]
        t.delta[0], t.delta[1] = delta
        t.scale[0], t.scale[1] = scale
        t.scale_u, t.scale_v = scale_uv
        t.offset_u, t.offset_v = offset_uv
        t.spherical = int(spherical)
        for i in range(9):
            t.rotation[i] = 1.0 if i % 4 == 0 else 0.0
        ptr = None
        if texels is not None:
            tx = np.ascontiguousarray(texels, dtype=np.float32)
            t.height, t.width = tx.shape[0], tx.shape[1]
            ptr = _fptr(tx)
        idx = _lib.nh_scene_add_texture(self._h, C.byref(t), ptr)
        if idx == 0:
            raise NoriError(f"add_texture: {_lib.nh_host_last_error().decode()}")
        return idx

    def set_lens_draw_order(self, order: int):
        """LENS_DRAWS_RTL (default, g++'s evaluation of Point2f(nextFloat(), nextFloat())) or LENS_DRAWS_LTR."""
        _host_check(_lib.nh_scene_set_lens_draw_order(self._h, order), "set_lens_draw_order")

    def set_normal_map(self, shape: int, texture: int):
        """Shape::addChild(<texture name="normal">): texture = an add_texture value, 0 removes the map."""
        _host_check(_lib.nh_scene_set_normal_map(self._h, shape, texture), "set_normal_map")

    @property
    def width(self):
        return self.desc.camera.width

    @property
    def height(self):
        return self.desc.camera.height

    @property
    def border(self):
        return self.desc.filter.border

    @property
    def spp(self):
        """the sampler's sampleCount"""
        return self.desc.sample_count

    def framebuffer_shape(self):
        d = self.desc
        b = d.filter.border
        return (d.camera.height + 2 * b, d.camera.width + 2 * b, 4)


def texture_decode(rgba8, srgb: bool) -> np.ndarray:
    """PNGTexture::loadFromFile's byte -> float loop (nh_texture_decode): sRGB or the normal-map decode."""
    b = np.ascontiguousarray(rgba8, dtype=np.uint8).ravel()
    out = np.empty(b.size, dtype=np.float32)
    _host_check(_lib.nh_texture_decode(b.ctypes.data_as(C.POINTER(C.c_uint8)), b.size, int(srgb), _fptr(out)),
                "texture_decode")
    return out


class Bvh:
    def __init__(self, scene: Scene, n_threads: int = 0):
        self._scene = scene
        d = scene.desc
        h = _vp()
        _host_check(_lib.nh_bvh_build(C.byref(d), n_threads, C.byref(h)), "bvh_build")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.nh_bvh_free(self._h)
            self._h = None

    @property
    def desc(self) -> nh_bvh_desc:
        d = nh_bvh_desc()
        _host_check(_lib.nh_bvh_get_desc(self._h, C.byref(d)), "bvh_get_desc")
        return d

    def nodes(self) -> np.ndarray:
        d = self.desc
        raw = np.ctypeslib.as_array(C.cast(d.nodes, C.POINTER(C.c_uint32)), shape=(d.n_nodes * 8,))
        return raw.reshape(d.n_nodes, 8).copy()

    def indices(self) -> np.ndarray:
        d = self.desc
        return np.ctypeslib.as_array(d.indices, shape=(d.n_indices,)).copy()


def debug_transform(request: str) -> np.ndarray:
    """The loader's transform arithmetic on one request of oracle/eigen_xform_probe.cpp's protocol
    (parity hook, include/nori_hip.h nh_debug_transform): float32 results."""
    out = np.zeros(64, np.float32)
    n = _lib.nh_debug_transform(request.encode(), _fptr(out), out.size)
    if n < 0:
        raise NoriError(f"debug_transform: {_lib.nh_host_last_error().decode()}")
    return out[:n].copy()


def device_count() -> int:
    global _hip_used
    _hip_used = True
    n = C.c_int(0)
    _lib.nh_get_device_count(C.byref(n))
    return n.value


class Context:
    """One GPU: device scene, BVH, master framebuffer (nh_ctx)."""

    def __init__(self, device: int = 0):
        global _hip_used
        _hip_used = True
        h = _vp()
        rc = _lib.nh_create(device, C.byref(h))
        if rc != NH_OK:
            raise NoriError(f"nh_create(device={device}) failed with {rc}")
        self._h = h
        self.scene = None

    def close(self):
        if getattr(self, "_h", None):
            _lib.nh_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, rc, what):
        if rc != NH_OK:
            raise NoriError(f"{what}: {_lib.nh_last_error(self._h).decode()} (rc={rc})")

    def upload(self, scene: Scene, bvh: Bvh):
        self.scene = scene
        d = scene.desc
        self._check(_lib.nh_upload_scene(self._h, C.byref(d)), "upload_scene")
        b = bvh.desc
        self._check(_lib.nh_upload_bvh(self._h, C.byref(b)), "upload_bvh")

    def render(self, s0: int, s1: int, seed: int = 0, blocks=None, traversal: int = TRAVERSAL_REFERENCE,
               clear: bool = False, stats: bool = False, mode: int = MODE_MEGAKERNEL):
        q = nh_render_req()
        q.sample_begin, q.sample_end, q.seed = s0, s1, seed
        keep = None
        if blocks is not None:
            keep = np.ascontiguousarray(blocks, dtype=np.int32)
            q.n_blocks = len(keep)
            q.blocks = keep.ctypes.data_as(C.POINTER(_i32))
        q.mode, q.traversal, q.clear, q.collect_stats = mode, traversal, int(clear), int(stats)
        self._check(_lib.nh_render(self._h, C.byref(q)), "render")

    def synchronize(self):
        self._check(_lib.nh_synchronize(self._h), "synchronize")

    def framebuffer(self) -> np.ndarray:
        shp = self.scene.framebuffer_shape()
        out = np.zeros(shp, dtype=np.float32)
        self._check(_lib.nh_get_framebuffer(self._h, _fptr(out), out.size), "get_framebuffer")
        return out

    def framebuffer_device_ptr(self):
        p, n = _vp(), C.c_size_t()
        self._check(_lib.nh_framebuffer_device_ptr(self._h, C.byref(p), C.byref(n)), "framebuffer_device_ptr")
        return p.value, n.value

    def stats(self) -> dict:
        s = nh_render_stats()
        self._check(_lib.nh_get_stats(self._h, C.byref(s)), "get_stats")
        return {f: getattr(s, f) for f, _ in s._fields_}

    def reset_stats(self):
        self._check(_lib.nh_reset_stats(self._h), "reset_stats")

    def denoise(self, params: nh_denoiser = None):
        """Denoiser::denoise on the master ImageBlock (src/utils/render.cpp:368-369): the scene's
        <denoiser> unless params are given."""
        if params is None:
            params = self.scene.desc.denoiser
        self._check(_lib.nh_denoise(self._h, C.byref(params)), "denoise")

    def denoise_image(self, rgbw: np.ndarray, border: int, params: nh_denoiser) -> np.ndarray:
        """SimpleDenoiser on a host (H+2b, W+2b, 4) float32 ImageBlock; returns the denoised copy."""
        out = np.array(rgbw, dtype=np.float32, order="C", copy=True)
        h, w = out.shape[0] - 2 * border, out.shape[1] - 2 * border
        self._check(_lib.nh_denoise_image(self._h, _fptr(out), w, h, border, C.byref(params)), "denoise_image")
        return out

    def trace(self, o: np.ndarray, d: np.ndarray, mint: np.ndarray, maxt: np.ndarray, any_hit=False,
              traversal: int = TRAVERSAL_REFERENCE) -> dict:
        n = len(o)
        cols = [np.ascontiguousarray(x, dtype=np.float32) for x in (o[:, 0], o[:, 1], o[:, 2], d[:, 0], d[:, 1],
                                                                     d[:, 2], mint, maxt)]
        r = nh_ray_soa(*[_fptr(c) for c in cols])
        res = {"hit": np.zeros(n, np.uint8), "t": np.zeros(n, np.float32), "u": np.zeros(n, np.float32),
               "v": np.zeros(n, np.float32), "prim": np.zeros(n, np.uint32), "shape": np.zeros(n, np.uint32)}
        h = nh_hit_soa(res["hit"].ctypes.data_as(C.POINTER(C.c_uint8)), _fptr(res["t"]), _fptr(res["u"]),
                       _fptr(res["v"]), res["prim"].ctypes.data_as(_u32p), res["shape"].ctypes.data_as(_u32p))
        self._check(_lib.nh_trace_rays(self._h, C.byref(r), n, int(any_hit), traversal, C.byref(h)), "trace_rays")
        return res


def tile_shard(width: int, height: int, world: int, rank: int) -> list:
    """32x32 image blocks (block id = by*nbx + bx, BlockGenerator numbering) dealt
    round-robin to ranks: the multi-GPU partition of the image."""
    nbx, nby = (width + 31) // 32, (height + 31) // 32
    return [b for b in range(nbx * nby) if b % world == rank]


def reduce_framebuffers(ctxs, root: int = 0):
    arr = (_vp * len(ctxs))(*[c._h for c in ctxs])
    rc = _lib.nh_reduce_framebuffers(arr, len(ctxs), root)
    if rc != NH_OK:
        raise NoriError(f"nh_reduce_framebuffers failed ({rc})")


def to_rgb(rgbw: np.ndarray, border: int) -> np.ndarray:
    """ImageBlock::toBitmap via the C-ABI (block.cpp:76-82)."""
    h, w = rgbw.shape[0] - 2 * border, rgbw.shape[1] - 2 * border
    src = np.ascontiguousarray(rgbw, dtype=np.float32)
    out = np.zeros((h, w, 3), np.float32)
    rc = _lib.nh_framebuffer_to_rgb(_fptr(src), w, h, border, _fptr(out))
    if rc != NH_OK:
        raise NoriError("framebuffer_to_rgb failed")
    return out


def write_exr(path: str, rgb: np.ndarray):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    _host_check(_lib.nh_write_exr(path.encode(), _fptr(rgb), rgb.shape[1], rgb.shape[0]), "write_exr")


def write_png(path: str, rgb: np.ndarray):
    """8-bit sRGB PNG as Bitmap::saveToLDR (src/utils/bitmap.cpp:122-140)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    _host_check(_lib.nh_write_png(path.encode(), _fptr(rgb), rgb.shape[1], rgb.shape[0]), "write_png")


def rgb_to_ldr(rgb: np.ndarray) -> np.ndarray:
    """The bytes write_png stores: (H, W, 3) uint8."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.empty(rgb.shape[:2] + (3,), np.uint8)
    _host_check(_lib.nh_rgb_to_ldr(_fptr(rgb), rgb.shape[1], rgb.shape[0],
                                   out.ctypes.data_as(C.POINTER(C.c_uint8))), "rgb_to_ldr")
    return out


def write_pfm(path: str, rgb: np.ndarray):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    _host_check(_lib.nh_write_pfm(path.encode(), _fptr(rgb), rgb.shape[1], rgb.shape[0]), "write_pfm")


def load_png(path: str) -> np.ndarray:
    """PNG -> (H, W, 4) uint8 through the library's decoder (nh_image_load_png)."""
    w, h = _i32(), _i32()
    _host_check(_lib.nh_image_load_png(path.encode(), None, 0, C.byref(w), C.byref(h)), "load_png")
    out = np.zeros((h.value, w.value, 4), np.uint8)
    _host_check(_lib.nh_image_load_png(path.encode(), out.ctypes.data_as(C.POINTER(C.c_uint8)), out.nbytes,
                                       C.byref(w), C.byref(h)), "load_png")
    return out
