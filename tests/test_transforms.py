"""The loader's host transform arithmetic against the reference's own Eigen, bit for bit (CPU only).

The reference builds every camera ray and every baked mesh vertex from Eigen float arithmetic on the host:
  - parser.cpp:308-360 composes <transform> operations onto an Eigen::Affine3f (Translation, DiagonalMatrix,
    AngleAxis, Affine3f(matrix) and lookat products);
  - nori::Transform(Matrix4f) stores Matrix4f::inverse() (transform.cpp:9-10), Eigen's SSE 4x4 float inverse
    (ext/eigen/Eigen/src/LU/arch/Inverse_SSE.h:35-163);
  - PerspectiveCamera::update sets sampleToCamera = Transform(D * T * P).inverse() (perspective.cpp:68-95);
  - WavefrontOBJ bakes toWorld into points and (trafo * n).normalized() normals (obj.cpp:107,121).
oracle/_ref/eigen_xform_probe (oracle/eigen_xform_probe.cpp compiled by oracle/build_ref.sh against the
reference's vendored, unmodified Eigen 3.3.8) evaluates those Eigen expressions; the product's restatement
(optix-renderer_amd/host/nori_transform.h) is compared with it bit for bit, on random inputs through the
nh_debug_transform hook and on real scenes through the product loader itself, whose camera and vertex arrays
are checked against matrices the probe recomputes from the XML (parsed here, independently of the loader).
Only where the reference checkout is present (this container); skipped elsewhere.
"""
import ctypes
import os
import subprocess
import xml.etree.ElementTree as ET

import numpy as np
import pytest

import nori_hip as nh
import scenegen

PROBE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                     "eigen_xform_probe")
pytestmark = pytest.mark.skipif(not os.path.exists(PROBE),
                                reason="oracle/_ref/eigen_xform_probe not built (needs /root/reference/ext/eigen)")

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


def strtof(s: str) -> np.float32:
    """toFloat (common.cpp:105-112) / istream >> float: C strtof, no double rounding."""
    return np.float32(_libc.strtof(s.strip().encode(), None))


def hx(v) -> str:
    return " ".join(f"{int(u):08x}" for u in np.asarray(v, np.float32).reshape(-1).view(np.uint32))


def probe(requests):
    out = subprocess.run([PROBE], input="\n".join(requests) + "\n", capture_output=True, text=True, check=True,
                         timeout=300).stdout.splitlines()
    assert len(out) == len(requests)
    return [np.array([int(t, 16) for t in line.split()], np.uint32).view(np.float32) for line in out]


def product(requests):
    return [nh.debug_transform(r) for r in requests]


def assert_bits(ref, mine, what):
    bad = []
    for i, (r, m) in enumerate(zip(ref, mine)):
        assert r.shape == m.shape, (what, i)
        same = (r.view(np.uint32) == m.view(np.uint32)) | (np.isnan(r) & np.isnan(m))
        if not same.all():
            bad.append(i)
    assert not bad, f"{what}: {len(bad)} of {len(ref)} mismatch, first request #{bad[0]}"


# ------------------------------------------------------------------------------------------------
def random_matrices(rng, n):
    """Affine, projective, rotation x scale, wide exponent, near-singular and singular 4x4 matrices."""
    out = []
    for k in range(n):
        kind = k % 6
        m = rng.normal(size=(4, 4))
        if kind == 1:
            m[3] = [0, 0, 0, 1]
        elif kind == 2:
            q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
            m = np.eye(4)
            m[:3, :3] = q * rng.uniform(0.01, 100, size=3)
            m[:3, 3] = rng.normal(size=3) * 10
        elif kind == 3:
            m *= 2.0 ** rng.integers(-30, 31, size=(4, 4))
        elif kind == 4:
            m[3] = m[2] * (1 + 1e-6 * rng.normal())
        elif kind == 5 and k % 12 == 5:
            m[2] = m[1]  # exactly singular: the determinant's reciprocal is infinite
        out.append(m.astype(np.float32))
    return out


def test_inverse_matches_eigen_sse():
    rng = np.random.default_rng(11)
    reqs = ["inv " + hx(m) for m in random_matrices(rng, 6000)]
    assert_bits(probe(reqs), product(reqs), "Matrix4f::inverse")


def random_ops(rng, n_ops):
    ops = []
    for _ in range(n_ops):
        kind = rng.integers(0, 5)
        v = (rng.normal(size=3) * 2.0 ** rng.integers(-4, 5)).astype(np.float32)
        if kind == 0:
            ops.append("t " + hx(v))
        elif kind == 1:
            v[rng.random(3) < 0.2] *= -1
            ops.append("s " + hx(v))
        elif kind == 2:
            ang = np.float32(rng.uniform(-360, 360))
            ops.append("r " + hx([ang]) + " " + hx(v))  # axis used as given (not normalised)
        elif kind == 3:
            m = rng.normal(size=(4, 4)).astype(np.float32)
            ops.append("m " + hx(m))
        else:
            o, t, u = (rng.normal(size=(3, 3)) * 3).astype(np.float32)
            ops.append("l " + hx(o) + " " + hx(t) + " " + hx(u))
    return ops


def test_transform_composition_matches_eigen():
    """<transform> children pre-multiplied onto an Affine3f, then Transform(matrix) with its inverse."""
    rng = np.random.default_rng(5)
    reqs = []
    for k in range(3000):
        ops = random_ops(rng, int(rng.integers(1, 6)))
        reqs.append(f"xf {len(ops)} " + " ".join(ops))
    assert_bits(probe(reqs), product(reqs), "parser transform composition")


def test_camera_projection_matches_eigen():
    rng = np.random.default_rng(3)
    reqs = []
    cases = [(800, 600, 27.7856, 1e-4, 1e4), (1024, 1024, 27.7856, 1e-4, 1e4), (2048, 2048, 27.7856, 1e-4, 1e4),
             (4096, 4096, 30.0, 1e-4, 1e4), (1, 1, 1e-9, 1e-4, 1e4), (64, 48, 45.0, 1e-4, 1e4), (1280, 720, 30, 1e-4, 1e4)]
    for _ in range(400):
        cases.append((int(rng.integers(1, 5000)), int(rng.integers(1, 5000)), float(rng.uniform(1e-3, 170)),
                      float(10 ** rng.uniform(-6, 0)), float(10 ** rng.uniform(1, 6))))
    for w, h, fov, n, f in cases:
        reqs.append("cam " + hx([w, h, fov, n, f]))
    assert_bits(probe(reqs), product(reqs), "sampleToCamera")


def test_point_vector_normal_application_matches_eigen():
    rng = np.random.default_rng(9)
    reqs = []
    for m in random_matrices(rng, 1500):
        for cmd in ("pt", "vec", "nrm"):
            v = (rng.normal(size=3) * 2.0 ** rng.integers(-8, 9)).astype(np.float32)
            reqs.append(f"{cmd} {hx(m)} {hx(v)}")
    assert_bits(probe(reqs), product(reqs), "Transform * Point3f / Vector3f / Normal3f")


def test_png_texture_rotation_matches_eigen():
    """PNGTexture's spherical-lookup rotation for eulerAngles (PNGTexture.cpp:28, :133-139: quaternion products of
    AngleAxisf rotations in Eigen's SSE arithmetic, toRotationMatrix, a 3x3 product) and the lookup's rot * wi,
    restated in host/nori_transform.h (png_rotation) and applied by the loader, the oracle and the kernels."""
    rng = np.random.default_rng(17)
    reqs = ["prot " + hx([0, 270, 0]), "prot " + hx([0, 0, 0])]
    for k in range(3000):
        e = rng.uniform(-720, 720, 3).astype(np.float32)
        if k % 5 == 0:
            e = np.round(e / 45) * 45  # the right angles scenes use
        if k % 7 == 0:
            e[rng.integers(0, 3)] = 0
        reqs.append("prot " + hx(e))
    for _ in range(3000):
        reqs.append("pdir " + hx(rng.normal(size=9)) + " " + hx(rng.normal(size=3)))
    assert_bits(probe(reqs), product(reqs), "PNGTexture rotation / rot * wi")


# ------------------------------------------------------------------------------------------------
# whole scenes through the product loader, checked against matrices recomputed from the XML by the probe

def xform_request(tnode):
    ops = []
    for op in tnode:
        a = {k: v for k, v in op.attrib.items()}
        vec = lambda s: [strtof(x) for x in s.replace(",", " ").split()]  # noqa: E731 (tokenize + toFloat)
        if op.tag == "translate":
            ops.append("t " + hx(vec(a["value"])))
        elif op.tag == "scale":
            ops.append("s " + hx(vec(a["value"])))
        elif op.tag == "rotate":
            ops.append("r " + hx([strtof(a["angle"])]) + " " + hx(vec(a["axis"])))
        elif op.tag == "matrix":
            ops.append("m " + hx(vec(a["value"])))
        elif op.tag == "lookat":
            ops.append("l " + hx(vec(a["origin"])) + " " + hx(vec(a["target"])) + " " + hx(vec(a["up"])))
    return f"xf {len(ops)} " + " ".join(ops)


def obj_vertices(path, matrix):
    """WavefrontOBJ::loadFromFile's vertex list (obj.cpp:96-179: (p, uv, n) dedup in face order, quads
    split), positions transformed by the probe: returns (expected V, normal requests per vertex or None)."""
    pos, nrm, order, seen = [], [], [], {}
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            pos.append([strtof(x) for x in t[1:4]])
        elif t[0] == "vn":
            nrm.append([strtof(x) for x in t[1:4]])
        elif t[0] == "f":
            vs = t[1:5]
            verts = vs[:3] + ([vs[3], vs[0], vs[2]] if len(vs) > 3 else [])
            for v in verts:
                key = tuple((v.split("/") + ["", ""])[:3])
                if key not in seen:
                    seen[key] = len(order)
                    order.append(key)
    mh = hx(matrix)
    pts = probe([f"pt {mh} {hx(p)}" for p in pos])
    nrms = probe([f"nrm {mh} {hx(n)}" for n in nrm]) if nrm else []
    V = np.array([pts[int(k[0]) - 1] for k in order], np.float32)
    N = np.array([nrms[int(k[2]) - 1] for k in order], np.float32) if nrm else None
    return V, N


def scenes_of(path):
    root = ET.parse(path).getroot()
    return [root] if root.tag == "scene" else root.findall("scene")


def check_scene(path, index=0, size=None):
    s = nh.Scene(path, index)
    if size:
        s.set_resolution(*size)
    d = s.desc
    sc = scenes_of(path)[index]
    cam = sc.find("camera")
    props = {c.get("name"): c.get("value") for c in cam if c.tag in ("float", "integer")}
    tw = cam.find("transform")
    w, h = size or (int(props.get("width", 1280)), int(props.get("height", 720)))
    fov, near, far = (strtof(props.get(k, dflt)) for k, dflt in (("fov", "30"), ("nearClip", "1e-4"),
                                                                  ("farClip", "1e4")))
    reqs = ["cam " + hx([w, h, fov, near, far])]
    if tw is not None:
        reqs.append(xform_request(tw))
    res = probe(reqs)
    s2c = np.array(d.camera.sample_to_camera[:], np.float32)
    np.testing.assert_array_equal(s2c.view(np.uint32), res[0][:16].view(np.uint32), "sampleToCamera")
    c2w = np.array(d.camera.camera_to_world[:], np.float32)
    ref_c2w = res[1][:16] if tw is not None else np.eye(4, dtype=np.float32).reshape(-1)
    np.testing.assert_array_equal(c2w.view(np.uint32), ref_c2w.view(np.uint32), "cameraToWorld")
    # baked meshes, in shape order
    base = os.path.dirname(path)
    meshes = [sh for sh in sc.findall("shape") if sh.get("type") == "obj"]
    dshapes = [d.shapes[i] for i in range(d.n_shapes) if d.shapes[i].type == nh.SHAPE_MESH]
    assert len(meshes) == len(dshapes)
    Vall = np.ctypeslib.as_array(d.V, shape=(d.n_vertices * 3,)).reshape(-1, 3)
    Nall = np.ctypeslib.as_array(d.N, shape=(d.n_vertices * 3,)).reshape(-1, 3)
    checked = 0
    for sh, ds in zip(meshes, dshapes):
        fn = next(c.get("value") for c in sh if c.tag == "string" and c.get("name") == "filename")
        t = sh.find("transform")
        m = probe([xform_request(t)])[0][:16] if t is not None else np.eye(4, dtype=np.float32).reshape(-1)
        V, N = obj_vertices(os.path.join(base, fn), m)
        mine = Vall[ds.v_offset:ds.v_offset + ds.n_vertices]
        np.testing.assert_array_equal(mine.view(np.uint32), V.view(np.uint32), f"V of {fn}")
        if N is not None:
            np.testing.assert_array_equal(Nall[ds.v_offset:ds.v_offset + ds.n_vertices].view(np.uint32),
                                          N.view(np.uint32), f"N of {fn}")
        checked += 1
    return checked


@pytest.mark.parametrize("name", ["pa4/cbox/cbox_path_mis.xml", "pa4/tests/test-direct.xml", "pa1/test-direct.xml",
                                  "pa3/tests/test-mesh.xml", "pa4/tests/test-furnace.xml"])
def test_reference_scenes_camera_and_meshes_match_eigen(scene_dir, name):
    path = os.path.join(scene_dir, "scenes", name)
    for i in range(len(scenes_of(path))):
        check_scene(path, i)


@pytest.mark.parametrize("size", [(1024, 1024), (2048, 2048), (256, 256)])
def test_bench_cbox_camera_matches_eigen(scene_dir, size):
    """C1 / C2 / C4 (the cbox camera resized by the benchmark, PerspectiveCamera::update recomputed)."""
    check_scene(os.path.join(scene_dir, "scenes/pa4/cbox/cbox_path_mis.xml"), 0, size)


def test_c5_toworld_copies_match_eigen(tmp_path):
    """C5's ten scale / rotate / translate copies of one mesh (obj.cpp:107 bakes each), a small mesh."""
    xml, _ = scenegen.c5_xml(str(tmp_path), n_copies=10, n_phi=40, n_theta=12, width=64, height=64)
    assert check_scene(xml) >= 10
