"""Shape normal maps: `<texture name="normal">` children of shapes.

Reference pieces, all restated in the product loader (host/scene_loader.cpp), the kernels (csrc/nh_shade.h hit_info /
tex_eval) and the oracle (oracle/nori_oracle.cpp set_hit_information / texture_eval):
  * Shape::addChild takes a texture named "normal" (src/shapes/shape.cpp:138-147);
  * PNGTexture defaults sRGB to false for it (src/textures/PNGTexture.cpp:26) and decodes lodepng's RGBA8 bytes as
    x / 255 * 2 - 1, normalizing every third float of the RGBA array as an Eigen Vector3f (:85-95) -- the triples
    straddle pixels and take in alpha; reproduced, not fixed;
  * eval blends the texel towards +z by `intensity` and normalizes it (:155-161);
  * Mesh::setHitInformation applies normalize(TBN * eval(uv)) when the mesh has normals and uvs (mesh.cpp:165-185);
  * Sphere::setHitInformation re-derives its frame from shFrame.toWorld(eval(uv)) (sphere.cpp:115-121).

Pins (CPU, this file): the decode against a numpy restatement on a crafted RGBA PNG whose triples straddle pixels,
and -- where the reference checkout is present -- against oracle/_ref/normalmap_probe, which runs the reference's
own lodepng + Eigen 3.3.8 on the same bytes and on the reference's shipped normal-map PNGs (product PNG decoder
included), and the oracle's TBN / sphere / blend arithmetic against the same probe. The GPU renders are compared
with the oracle in test_gpu_project_scenes.py.
"""
import os
import subprocess

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen

REF = "/root/reference"
PROBE = os.path.join(os.path.dirname(no.__file__), "_ref", "normalmap_probe")
PROBE_CLANG = PROBE + "_clang"
NORMALMAP_SCENES = ["scenes/project/normalmap/normals-identity-direct.xml",
                    "scenes/project/normalmap/normals-primitives-direct.xml",
                    "scenes/project/normalmap/normals-camel.xml",
                    "scenes/project/normalmap/normals-identity.xml",
                    "scenes/project/normalmap/normals-identity-x.xml",
                    "scenes/project/normalmap/normals-identity-y.xml",
                    "scenes/project/normalmap/normals-primitives.xml"]


@pytest.fixture(scope="module")
def proj_dir(tmp_path_factory):
    return scenegen.materialize(str(tmp_path_factory.mktemp("nmap")))


def decode_restated(b: np.ndarray, srgb: bool) -> np.ndarray:
    """numpy restatement of PNGTexture::loadFromFile's loop (float32 arithmetic, one rounding per operation)."""
    b = np.asarray(b, np.uint8).ravel()
    f32 = np.float32
    if srgb:
        x = b.astype(f32) / f32(255)
        lin = x * f32(1) / f32(12.92)
        gam = np.power(((x + f32(0.055)) * f32(1) / f32(1.055)).astype(np.float64), float(f32(2.4))).astype(f32)
        return np.where(x <= f32(0.04045), lin, gam).astype(f32)
    d = b.astype(f32) / f32(255) * f32(2) - f32(1)
    n3 = (d.size // 3) * 3
    t = d[:n3].reshape(-1, 3)  # a view: the triples of the RGBA array, straddling pixels
    z = t[:, 0] * t[:, 0] + (t[:, 1] * t[:, 1] + t[:, 2] * t[:, 2])
    pos = z > 0
    s = np.sqrt(z[pos])
    t[pos] = t[pos] / s[:, None]
    return d


def nmap_scene_xml(tmp_path, png_name, intensity=None, srgb=None, extra=""):
    """A direct_mis scene: a plane (normals + uvs) and a sphere, both with the given normal map."""
    proj = scenegen.materialize(str(tmp_path))
    tex = f'<texture type="png_texture" name="normal"><string name="filename" value="{png_name}"/>'
    if intensity is not None:
        tex += f'<float name="intensity" value="{intensity}"/>'
    if srgb is not None:
        tex += f'<boolean name="sRGB" value="{"true" if srgb else "false"}"/>'
    tex += "</texture>"
    xml = f"""<scene>
  <integrator type="direct_mis"/>
  <camera type="perspective">
    <transform name="toWorld"><lookat origin="0,4,-6" target="0,0.5,0" up="0,1,0"/></transform>
    <float name="fov" value="40"/><integer name="width" value="64"/><integer name="height" value="48"/>
  </camera>
  <shape type="obj"><string name="filename" value="../meshes/plane.obj"/>{tex}
    <transform name="toWorld"><scale value="3,3,3"/></transform></shape>
  <shape type="sphere"><point name="center" value="0,1,0"/><float name="radius" value="1"/>{tex}</shape>
  {extra}
  <emitter type="point"><point name="position" value="0,3,-2"/><color name="power" value="200,200,200"/></emitter>
</scene>"""
    path = os.path.join(proj, "scenes/project/normalmap", "test_nmap.xml")
    with open(path, "w") as f:
        f.write(xml)
    return path


def crafted_rgba(h=5, w=7, seed=3):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    img[0, 0] = (128, 128, 128, 0)      # a near-zero triple (no byte decodes to exactly 0: x / 255 * 2 - 1)
    img[1, :, 3] = 17                   # alpha that is not 255: the straddling triples take it in
    return img


def test_decode_quirk_numpy_restatement(tmp_path):
    """A crafted RGBA PNG whose triples straddle pixels (5x7, random bytes, non-opaque alpha): the
    loader's texels equal the numpy restatement of the stride-3 normalize over the RGBA array bit for bit."""
    proj = scenegen.materialize(str(tmp_path))
    img = crafted_rgba()
    png = os.path.join(proj, "scenes/project/res/crafted-rgba.png")
    scenegen.write_png(png, img)
    s = nh.Scene(nmap_scene_xml(tmp_path, "../res/crafted-rgba.png"))
    d = s.desc
    assert d.n_textures == 2 and [d.shapes[i].normal_map for i in range(d.n_shapes)] == [1, 2]
    t = d.textures[0]
    assert (t.type, t.linear, t.width, t.height, t.intensity) == (nh.TEXTURE_PNG, 1, 7, 5, np.float32(1))
    texels = np.ctypeslib.as_array(d.texels, shape=(int(d.n_texels) * 4,))[: 7 * 5 * 4]
    ref = decode_restated(img, srgb=False)
    np.testing.assert_array_equal(texels.view(np.uint32), ref.view(np.uint32))
    # the quirk is real: pixel 1's RGB is part of two triples (A0 R1 G1) and (B1 A1 R2), so it is not a unit vector
    p1 = texels[4:7].astype(np.float64)
    assert abs(np.linalg.norm(p1) - 1.0) > 1e-3
    # pixel 0's RGB is the first triple: a unit vector
    assert abs(np.linalg.norm(texels[0:3].astype(np.float64)) - 1.0) < 1e-6
    # the C-ABI decode hook is the same loop
    np.testing.assert_array_equal(nh.texture_decode(img, srgb=False).view(np.uint32), ref.view(np.uint32))
    np.testing.assert_array_equal(nh.texture_decode(img, srgb=True).view(np.uint32),
                                  decode_restated(img, srgb=True).view(np.uint32))


def test_shape_texture_errors(tmp_path):
    """Shape::addChild's checks (shape.cpp:138-147): a second normal map and a texture with another name throw."""
    proj = scenegen.materialize(str(tmp_path))
    base = open(nmap_scene_xml(tmp_path, "../res/normal-identity.png")).read()
    tex = '<texture type="png_texture" name="normal"><string name="filename" value="../res/normal-identity.png"/></texture>'
    twice = base.replace(tex, tex + tex, 1)
    other = base.replace('name="normal"', 'name="bump"', 1)
    for text, msg in ((twice, "already a normal map"), (other, "does not have a texture with name: bump")):
        p = os.path.join(proj, "scenes/project/normalmap/bad.xml")
        with open(p, "w") as f:
            f.write(text)
        with pytest.raises(nh.NoriError, match=msg):
            nh.Scene(p)


def test_reference_normalmap_scenes_load(proj_dir):
    """The reference's three normal-mapped scenes with in-scope integrators load from the fixtures: every
    `<texture name="normal">` becomes a linear (sRGB = false) png texture of intensity 1 on its shape."""
    expect = {"normals-identity-direct.xml": ([1, 2, 3, 4], nh.INTEGRATOR_DIRECT_MIS, (1024, 1024)),
              "normals-primitives-direct.xml": ([1, 0, 2, 0], nh.INTEGRATOR_DIRECT_MIS, (1024, 1024)),
              "normals-camel.xml": ([1, 0], nh.INTEGRATOR_DIRECT, (200, 200)),
              "normals-identity.xml": ([1, 2, 3, 4], nh.INTEGRATOR_NORMALS, (1024, 1024)),
              "normals-identity-x.xml": ([1, 2, 3, 4], nh.INTEGRATOR_NORMALS, (1024, 1024)),
              "normals-identity-y.xml": ([1, 2, 3, 4], nh.INTEGRATOR_NORMALS, (1024, 1024)),
              "normals-primitives.xml": ([1, 0, 2, 0], nh.INTEGRATOR_NORMALS, (1024, 1024))}
    for rel in NORMALMAP_SCENES:
        s = nh.Scene(os.path.join(proj_dir, rel))
        d = s.desc
        maps, integ, size = expect[os.path.basename(rel)]
        assert [d.shapes[i].normal_map for i in range(d.n_shapes)] == maps
        assert d.integrator == integ
        for i in range(d.n_textures):
            t = d.textures[i]
            assert (t.linear, t.intensity, (t.width, t.height)) == (1, np.float32(1), size)
        # meshes with normals and uvs take the TBN branch (mesh.cpp:173-183); the spheres take sphere.cpp:115-121
        for i in range(d.n_shapes):
            sh = d.shapes[i]
            if sh.normal_map and sh.type == nh.SHAPE_MESH:
                assert sh.has_normals and sh.has_uvs


def test_oracle_normal_map_changes_shading(proj_dir):
    """normals-primitives-direct.xml at 96x72: the normal maps change the oracle's image (removing them changes
    the shaded pixels of the plane and the cube), and the render is finite."""
    path = os.path.join(proj_dir, "scenes/project/normalmap/normals-primitives-direct.xml")
    s = nh.Scene(path)
    s.set_resolution(96, 72)
    a = no.OracleScene(s).render(0, 2, seed=5)
    s2 = nh.Scene(path)
    s2.set_resolution(96, 72)
    for i in range(s2.desc.n_shapes):
        s2.set_normal_map(i, 0)
    b = no.OracleScene(s2).render(0, 2, seed=5)
    assert np.isfinite(a).all() and np.abs(a[..., :3]).sum() > 0
    assert (np.abs(a - b).max(axis=-1) > 0).sum() > 100


def test_intensity_and_srgb_properties(tmp_path):
    """`intensity` is read for every png_texture, and an explicit sRGB = true keeps the gamma decode (no blend)."""
    s = nh.Scene(nmap_scene_xml(tmp_path, "../res/normal-test.png", intensity=0.25))
    assert s.desc.textures[0].intensity == np.float32(0.25) and s.desc.textures[0].linear == 1
    s = nh.Scene(nmap_scene_xml(tmp_path, "../res/normal-test.png", srgb=True))
    assert s.desc.textures[0].linear == 0


# ---- pins against the reference's own lodepng + Eigen (this container only) ------------------------------------

def run_probe(exe, *args):
    subprocess.run([exe, *map(str, args)], check=True, timeout=120)


needs_probe = pytest.mark.skipif(not os.path.exists(PROBE), reason="oracle/_ref/normalmap_probe not built "
                                 "(needs /root/reference/ext/lodepng and ext/eigen)")


@needs_probe
@pytest.mark.parametrize("srgb", [False, True])
def test_decode_matches_reference_lodepng_eigen_bytes(tmp_path, srgb):
    """PNGTexture's decode loop run by the reference's Eigen on 3M crafted bytes (random, and every combination of
    16 edge byte values in a triple) equals nh_texture_decode bit for bit."""
    rng = np.random.default_rng(11)
    edge = np.array([0, 1, 2, 63, 64, 126, 127, 128, 129, 130, 191, 192, 253, 254, 255, 10], np.uint8)
    combos = np.stack(np.meshgrid(edge, edge, edge, indexing="ij"), -1).reshape(-1)
    b = np.concatenate([combos, rng.integers(0, 256, size=3_000_000, dtype=np.uint8), np.uint8([7, 9])])
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    b.tofile(inp)
    run_probe(PROBE, "bytes", inp, out, int(srgb))
    ref = np.fromfile(out, np.float32)
    mine = nh.texture_decode(b, srgb=srgb)
    assert ref.size == mine.size == b.size
    bad = ref.view(np.uint32) != mine.view(np.uint32)
    assert not bad.any(), f"{bad.sum()} mismatches, first at {np.argmax(bad)}"
    np.testing.assert_array_equal(decode_restated(b, srgb).view(np.uint32), mine.view(np.uint32))


@needs_probe
@pytest.mark.parametrize("rel,srgb", [("scenes/project/res/normal-identity.png", False),
                                      ("scenes/project/res/normal-primitives.png", False),
                                      ("scenes/project/res/normal-test.png", False),
                                      ("scenes/project/res/envmap-test.png", True),
                                      ("scenes/project/res/wooden_motel.png", True)])
def test_png_texels_match_reference_lodepng(tmp_path, rel, srgb):
    """The reference's shipped PNGs through the reference's lodepng + decode loop equal the product loader's PNG
    decoder (host/png_decode.cpp) + decode loop bit for bit: this pins the texels of the normal maps and of the
    sRGB textures (InverseGammaCorrect with g++'s std::pow(float, float))."""
    src = os.path.join(REF, rel)
    if not os.path.exists(src):
        pytest.skip(f"{rel} not in the reference checkout")
    out = tmp_path / "out.bin"
    run_probe(PROBE, "png", src, out, int(srgb))
    raw = np.fromfile(out, np.uint8)
    w, h = raw[:8].view(np.uint32)
    ref = raw[8:].view(np.float32)
    W, H = C_int(), C_int()
    assert nh.lib.nh_image_load_png(src.encode(), None, 0, nh.C.byref(W), nh.C.byref(H)) == 0
    buf = np.empty(W.value * H.value * 4, np.uint8)
    assert nh.lib.nh_image_load_png(src.encode(), buf.ctypes.data_as(nh.C.POINTER(nh.C.c_uint8)), buf.size,
                                    nh.C.byref(W), nh.C.byref(H)) == 0
    assert (W.value, H.value) == (w, h)
    mine = nh.texture_decode(buf, srgb=srgb)
    bad = ref.view(np.uint32) != mine.view(np.uint32)
    assert not bad.any(), f"{bad.sum()} of {ref.size} texel floats differ"


def C_int():
    return nh.C.c_int32()


@needs_probe
def test_normal_ops_match_reference_eigen(tmp_path):
    """The oracle's TBN product, sphere re-framing and eval blend (no_normal_ops) equal the reference's Eigen
    expressions bit for bit on 200k cases: unit frames and texels, random vectors, wide exponents, zeros, and
    intensities in [0, 1] with the endpoints."""
    rng = np.random.default_rng(5)
    n = 200_000
    c = rng.normal(size=(n, 13)).astype(np.float32)
    for k in (0, 3, 6, 9):
        v = c[: n // 2, k:k + 3].astype(np.float64)
        c[: n // 2, k:k + 3] = (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)
    c[n // 2:, :12] *= (2.0 ** rng.integers(-20, 21, size=(n - n // 2, 12))).astype(np.float32)
    c[:, 12] = rng.random(n).astype(np.float32)
    c[::7, 12] = 1.0
    c[1::7, 12] = 0.0
    c[2::101, 9:12] = 0.0                 # a zero texel: normalize leaves it
    c[3::103, 6:9] = c[3::103, 0:3]       # degenerate frames
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    c.tofile(inp)
    run_probe(PROBE, "ops", inp, out)
    ref = np.fromfile(out, np.float32).reshape(n, 15)
    mine = no.normal_ops(c)
    names = ["tbn"] * 3 + ["sphere n"] * 3 + ["sphere t"] * 3 + ["sphere b"] * 3 + ["blend"] * 3
    for j, name in enumerate(names):
        nan_both = np.isnan(ref[:, j]) & np.isnan(mine[:, j])
        bad = (ref[:, j].view(np.uint32) != mine[:, j].view(np.uint32)) & ~nan_both
        assert not bad.any(), f"{name} (column {j}): {bad.sum()} mismatches, e.g. case {np.argmax(bad)}"


@needs_probe
def test_next2d_argument_order_is_compiler_dependent(tmp_path):
    """Independent::next2D is `Point2f(m_random.nextFloat(), m_random.nextFloat())` (independent.cpp:74-78): C++
    leaves the order of the two calls unspecified. g++ (this image's compiler) evaluates them right to left -- x is
    the second draw -- and clang left to right. The lens sample of the thin-lens camera follows the g++ order
    (DESIGN.md section 7); the per-path sample streams are this framework's own contract either way."""
    first = no.Pcg32()
    a, b = first.next_float(), first.next_float()
    run_probe(PROBE, "order", tmp_path / "g.bin")
    g = np.fromfile(tmp_path / "g.bin", np.float32)
    assert (g[0], g[1]) == (np.float32(b), np.float32(a))
    if os.path.exists(PROBE_CLANG):
        run_probe(PROBE_CLANG, "order", tmp_path / "c.bin")
        c = np.fromfile(tmp_path / "c.bin", np.float32)
        assert (c[0], c[1]) == (np.float32(a), np.float32(b))


def test_normals_integrator_shows_the_mapped_frames(proj_dir):
    """The `normals` integrator (normals.cpp:15-33) renders |shFrame.toWorld((0, 0, 1))|: the identity map and the
    x- and y-tilted maps of the reference's scenes give finite images that differ visibly from one another."""
    def render(name):
        s = nh.Scene(os.path.join(proj_dir, "scenes/project/normalmap", name))
        assert s.desc.integrator == nh.INTEGRATOR_NORMALS
        s.set_resolution(96, 72)
        return no.OracleScene(s).render(0, 1, seed=2)
    ident, x, y = render("normals-identity.xml"), render("normals-identity-x.xml"), render("normals-identity-y.xml")
    for img in (ident, x, y):
        assert np.isfinite(img).all() and img[..., 3].sum() > 0
    assert np.abs(x - ident).max() > 0.05 and np.abs(y - ident).max() > 0.05 and np.abs(x - y).max() > 0.05
