"""Textured diffuse albedo: Diffuse's Texture<Color3f> child (src/bsdf/diffuse.cpp:32-91) --
constant_color (src/textures/consttexture.cpp), checkerboard_color (src/textures/checkerboard.cpp:29-47) and
png_texture (src/textures/PNGTexture.cpp:125-160) -- through the loader, the C-ABI and the oracle.

CPU tests: the reference's textured scenes load with the reference's parameters; the oracle's texture lookups
equal an independent numpy restatement of the reference's formulas (float32 arithmetic, and the float -> int /
unsigned casts as the reference's x86-64 build executes them: cvttss2si) on random and edge-case uvs; the
loader raises the reference's errors. The GPU lookups are compared with the oracle in test_gpu_textures.py.
Parity with the reference renderer itself is pinned only through these restatements (the reference cannot be
built here).
"""
import os

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen

F = np.float32


def x86_f2i(x):
    """int(float) on x86-64 (cvttss2si, 32 bits): trunc toward zero, NaN / out of range -> INT_MIN."""
    x = np.asarray(x, np.float32)
    ok = np.abs(x) < F(2.0 ** 31)
    out = np.full(x.shape, -2 ** 31, np.int64)
    out[ok] = np.trunc(x[ok]).astype(np.int64)
    return out


def x86_f2u(x):
    """static_cast<unsigned int>(float) on x86-64 (cvttss2si to 64 bits, low word)."""
    x = np.asarray(x, np.float32)
    ok = np.abs(x) < F(2.0 ** 63)
    out = np.zeros(x.shape, np.uint64)
    out[ok] = (np.trunc(x[ok].astype(np.float64)).astype(np.int64).astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    return out


def checker_ref(u, v, scale, delta, c1, c2):
    """Checkerboard<Color3f>::eval (checkerboard.cpp:29-47)."""
    with np.errstate(all="ignore"):
        ox = np.asarray(u, F) / F(scale[0]) - F(delta[0])
        oy = np.asarray(v, F) / F(scale[1]) - F(delta[1])
    x = x86_f2i(ox) + (ox < 0)
    y = x86_f2i(oy) + (oy < 0)
    even = ((x + y) & 1) == 0  # (x + y) % 2 == 0 on wrapping 32-bit ints: the low bit
    return np.where(even[:, None], np.asarray(c1, F)[None], np.asarray(c2, F)[None]).astype(F)


def png_ref(texels, u, v, scale=(1, 1), offset=(0, 0)):
    """PNGTexture::eval for a non-spherical texture (PNGTexture.cpp:125-160): nearest texel, row 0 first."""
    H, W = texels.shape[:2]
    with np.errstate(all="ignore"):
        u = np.asarray(u, F) + F(offset[0])
        v = np.asarray(v, F) + F(offset[1])
        w = x86_f2u(u * F(scale[0]) * F(W))
        hh = x86_f2u(v * F(scale[1]) * F(H))
    h = (np.uint64(H) - hh) & np.uint64(0xFFFFFFFF)
    idx = ((h * np.uint64(W) + w) & np.uint64(0xFFFFFFFF)) % np.uint64(W * H)
    return texels.reshape(-1, 4)[idx.astype(np.int64), :3]


def uv_cases(n, seed):
    rng = np.random.default_rng(seed)
    u = rng.uniform(-3, 3, n).astype(F)
    v = rng.uniform(-3, 3, n).astype(F)
    edge = np.array([0, -0.0, 1, 0.5, -0.5, 1e-30, -1e-30, 0.1, 0.2, 0.3, 1e10, -1e10, 3e9, -3e9, 1e30, -1e30,
                     np.inf, -np.inf, np.nan, 0.999999, 1.000001, 2 ** 31, -2 ** 31], F)
    uu, vv = np.meshgrid(edge, edge)
    return np.concatenate([u, uu.ravel()]), np.concatenate([v, vv.ravel()])


def textured_dir(tmp_path_factory):
    return scenegen.materialize(str(tmp_path_factory.mktemp("tex")))


@pytest.fixture(scope="module")
def tex_dir(tmp_path_factory):
    return textured_dir(tmp_path_factory)


def test_reference_textured_scenes_load(tex_dir):
    """denoiser-test.xml (checkerboard floor, the scene of the reference's published timing), mesh-texture.xml and
    sphere-texture.xml load unchanged with the reference's texture parameters."""
    cases = {
        "scenes/project/denoiser/denoiser-test.xml": ((0.1, 0.2), (0.0, 0.0), 3),
        "scenes/pa1/mesh-texture.xml": ((0.1, 0.2), (0.5, 0.5), 0),
        "scenes/pa1/sphere-texture.xml": ((0.1, 0.2), (0.0, 0.0), 0),
    }
    for rel, (scale, delta, shape) in cases.items():
        s = nh.Scene(os.path.join(tex_dir, rel))
        d = s.desc
        assert d.n_textures == 1, rel
        t = d.textures[0]
        assert t.type == nh.TEXTURE_CHECKERBOARD
        assert np.allclose(list(t.scale), scale) and np.allclose(list(t.delta), delta), rel
        assert np.allclose(list(t.value1), [0.8] * 3) and np.allclose(list(t.value2), [0.2] * 3)
        sh = d.shapes[shape]
        assert d.bsdfs[sh.bsdf].albedo_texture == 1, rel
        # every other diffuse BSDF keeps its constant albedo
        assert sum(d.bsdfs[i].albedo_texture != 0 for i in range(d.n_bsdfs)) == 1


def test_denoiser_test_scene_parameters(tex_dir):
    s = nh.Scene(os.path.join(tex_dir, "scenes/project/denoiser/denoiser-test.xml"))
    d = s.desc
    assert (d.camera.width, d.camera.height) == (800, 600)
    assert d.integrator == nh.INTEGRATOR_PATH_MIS and d.sample_count == 16
    assert d.denoiser.type == nh.DENOISER_SIMPLE and d.denoiser.range == 7
    assert d.n_emitters == 2 and d.n_shapes == 4


def test_checkerboard_matches_numpy_restatement(tex_dir):
    for rel in ("scenes/pa1/mesh-texture.xml", "scenes/project/denoiser/denoiser-test.xml"):
        s = nh.Scene(os.path.join(tex_dir, rel))
        t = s.desc.textures[0]
        u, v = uv_cases(20000, 3)
        got = no.OracleScene(s).texture_eval(1, u, v)
        ref = checker_ref(u, v, list(t.scale), list(t.delta), list(t.value1), list(t.value2))
        np.testing.assert_array_equal(got, ref, err_msg=rel)
        # both colours occur on the [0, 1]^2 uv square
        m = (u >= 0) & (u <= 1) & (v >= 0) & (v <= 1)
        assert len(np.unique(got[m][:, 0])) == 2


def png_scene(tmp_path, tex_w=37, tex_h=23, scale=None, offset=None, spherical=False, seed=5):
    """A Cornell box whose walls and floor (walls.obj: no texture coordinates, so uv = barycentric) carry a
    png_texture albedo; returns (xml, decoded RGBA texels)."""
    d = str(tmp_path)
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, size=(tex_h, tex_w, 4), dtype=np.uint8)
    img[..., 3] = 255
    png = os.path.join(d, "albedo.png")
    scenegen.write_png(png, img)
    props = ""
    if scale:
        props += f'<float name="scaleU" value="{scale[0]}"/><float name="scaleV" value="{scale[1]}"/>'
    if offset:
        props += f'<float name="offsetU" value="{offset[0]}"/><float name="offsetV" value="{offset[1]}"/>'
    if spherical:
        props += '<boolean name="sphericalTexture" value="true"/>'
    tex = (f'<bsdf type="diffuse"><texture type="png_texture" name="albedo"><string name="filename" '
           f'value="{png}"/>{props}</texture></bsdf>')
    xml = scenegen.cbox_xml(d, "c2", walls_bsdf=tex)
    return xml, img


def inverse_gamma_f32(img):
    """InverseGammaCorrect (PNGTexture.cpp:442-447) of v = byte / 255.f, std::pow in double, rounded."""
    x = img.astype(F) / F(255.0)
    lo = x * F(1.0) / F(12.92)
    hi = np.power(((x + F(0.055)) * F(1.0) / F(1.055)).astype(np.float64), np.float64(F(2.4))).astype(F)
    return np.where(x <= F(0.04045), lo, hi).astype(F)


@pytest.mark.parametrize("scale,offset", [(None, None), ((2.5, 0.75), (-0.3, 0.6))])
def test_png_albedo_matches_numpy_restatement(tmp_path, scale, offset):
    xml, img = png_scene(tmp_path, scale=scale, offset=offset)
    s = nh.Scene(xml)
    d = s.desc
    assert d.n_textures == 1 and d.textures[0].type == nh.TEXTURE_PNG
    texels = np.ctypeslib.as_array(d.texels, shape=(d.n_texels * 4,)).reshape(img.shape).copy()
    np.testing.assert_array_equal(texels, inverse_gamma_f32(img))
    u, v = uv_cases(20000, 4)
    got = no.OracleScene(s).texture_eval(1, u, v)
    ref = png_ref(texels, u, v, scale or (1, 1), offset or (0, 0))
    np.testing.assert_array_equal(got, ref)


def test_texture_through_cabi_add_texture(tmp_path):
    """nh_scene_add_texture + nh_bsdf.albedo_texture: a C caller builds the same texture the XML describes."""
    xml = scenegen.cbox_xml(str(tmp_path), "c2")
    s = nh.Scene(xml)
    idx = s.add_texture(nh.TEXTURE_CHECKERBOARD, value1=(0.8, 0.1, 0.1), value2=(0.1, 0.8, 0.1), scale=(0.25, 0.5),
                        delta=(0.5, 0.0))
    assert idx == 1
    s.set_bsdf(0, type=nh.BSDF_DIFFUSE, albedo=(0.5, 0.5, 0.5), albedo_texture=idx)
    assert s.desc.bsdfs[s.desc.shapes[0].bsdf].albedo_texture == 1
    u, v = uv_cases(5000, 6)
    got = no.OracleScene(s).texture_eval(1, u, v)
    np.testing.assert_array_equal(got, checker_ref(u, v, (0.25, 0.5), (0.5, 0.0), (0.8, 0.1, 0.1), (0.1, 0.8, 0.1)))
    texels = np.random.default_rng(1).random((5, 7, 4)).astype(F)
    idx2 = s.add_texture(nh.TEXTURE_PNG, texels=texels, scale_uv=(1.5, 1.0))
    assert idx2 == 2
    np.testing.assert_array_equal(no.OracleScene(s).texture_eval(2, u, v), png_ref(texels, u, v, (1.5, 1.0)))
    with pytest.raises(nh.NoriError):
        s.add_texture(nh.TEXTURE_PNG)  # png without texels


def test_textured_render_differs_from_constant(tmp_path, tex_dir):
    """The oracle renders the checkerboard: the textured sphere scene is not the constant-albedo one."""
    path = os.path.join(tex_dir, "scenes/pa1/sphere-texture.xml")
    s = nh.Scene(path)
    s.set_resolution(48, 48)
    a = no.OracleScene(s).render(0, 2, seed=1)
    s.set_bsdf(0, type=nh.BSDF_DIFFUSE, albedo=(0.5, 0.5, 0.5))
    b = no.OracleScene(s).render(0, 2, seed=1)
    assert np.abs(a - b).max() > 0.01


def test_texture_loader_errors(tmp_path):
    d = str(tmp_path)
    png = os.path.join(d, "t.png")
    scenegen.write_png(png, np.full((4, 4, 4), 128, np.uint8))
    open(png[:-4] + ".hdr", "wb").write(b"#?RADIANCE\n")  # a truncated .hdr image (test_hdr.py: the decoder)
    cases = {
        # an albedo colour already creates the albedo texture (diffuse.cpp:33-40, :75-79)
        '<bsdf type="diffuse"><color name="albedo" value="0.5,0.5,0.5"/><texture type="constant_color" name="albedo">'
        '<color name="value" value="1,1,1"/></texture></bsdf>': "There is already an albedo defined!",
        '<bsdf type="diffuse"><texture type="constant_color" name="kd"><color name="value" value="1,1,1"/></texture>'
        '</bsdf>': "does not match any field",
        f'<bsdf type="diffuse"><texture type="png_texture" name="albedo"><string name="filename" value="{png[:-4]}.hdr"/>'
        '</texture></bsdf>': "Could not load HDR file",
        '<bsdf type="diffuse"><texture type="png_texture" name="albedo"><string name="filename" value="nope.png"/>'
        '</texture></bsdf>': "image file not found",
        '<bsdf type="diffuse"><texture type="checkerboard_color" name="albedo"><vector name="scale" value="1,2,3,4"/>'
        '</texture></bsdf>': "is not of size 2 or 3",
    }
    for bsdf, msg in cases.items():
        xml = scenegen.cbox_xml(d, "c2", walls_bsdf=bsdf)
        with pytest.raises(nh.NoriError, match=msg):
            nh.Scene(xml)
    # constant_color child: its value is the albedo
    xml = scenegen.cbox_xml(d, "c2", walls_bsdf='<bsdf type="diffuse"><texture type="constant_color" name="albedo">'
                                               '<color name="value" value="0.25,0.5,0.75"/></texture></bsdf>')
    s = nh.Scene(xml)
    assert s.desc.textures[0].type == nh.TEXTURE_CONSTANT
    np.testing.assert_array_equal(no.OracleScene(s).texture_eval(1, [0.3, -7.0], [0.1, 2.0]),
                                  np.array([[0.25, 0.5, 0.75]] * 2, F))


def aircraft_substituted(tex_dir):
    """aircraft.xml with synthetic stand-ins for its two absent images, written where the scene expects them: a
    random 128x64 res/aircraft_base.png and a 96x48 run-length Radiance sky as res/dikhololo_night_4k.hdr (so the
    scene file loads unmodified); returns the scene file's path."""
    src = os.path.join(tex_dir, "scenes/project/textures/aircraft.xml")
    res = os.path.join(tex_dir, "scenes/project/res")
    os.makedirs(res, exist_ok=True)
    rng = np.random.default_rng(2)
    scenegen.write_png(os.path.join(res, "aircraft_base.png"), rng.integers(0, 256, (64, 128, 4), dtype=np.uint8))
    sky = scenegen.sky_image(96, 48).astype(np.float64) / 255.0 * 4.0
    scenegen.write_hdr(os.path.join(res, "dikhololo_night_4k.hdr"), scenegen.rgbe_encode(sky), mode="rle")
    return src


def test_aircraft_scene(tex_dir, tmp_path):
    """scenes/project/textures/aircraft.xml: png_texture albedo on the aircraft body, glass dielectric, spherical
    envmap texture with eulerAngles (0, 270, 0). Its two images (res/aircraft_base.png, res/dikhololo_night_4k.hdr)
    are absent from the reference checkout, so it fails to load as the reference would (PNGTexture: image file not
    found); with a synthetic aircraft_base.png and a synthetic Radiance sky in their places it loads, with the
    reference's rotation (Eigen-pinned, test_transforms.py), the .hdr texels and the aircraft's texture
    coordinates."""
    src = os.path.join(tex_dir, "scenes/project/textures/aircraft.xml")
    if not os.path.exists(os.path.join(tex_dir, "scenes/project/res/aircraft_base.png")):
        with pytest.raises(nh.NoriError, match="image file not found"):
            nh.Scene(src)
    s = nh.Scene(aircraft_substituted(tex_dir))
    d = s.desc
    assert d.n_textures == 1 and d.textures[0].type == nh.TEXTURE_PNG and d.textures[0].spherical == 0
    assert (d.textures[0].width, d.textures[0].height) == (128, 64)
    assert d.envmap >= 0 and d.env.spherical == 1 and (d.env.width, d.env.height) == (96, 48)
    hdr = scenegen.rgbe_encode(scenegen.sky_image(96, 48).astype(np.float64) / 255.0 * 4.0)
    np.testing.assert_array_equal(np.ctypeslib.as_array(d.env.rgba, shape=(48, 96, 4)),
                                  scenegen.rgbe_decode_reference(hdr))
    rot = np.array(list(d.env.rotation), np.float32).reshape(3, 3)
    assert not np.array_equal(rot, np.eye(3, dtype=np.float32))  # eulerAngles (0, 270, 0): a rotation about x
    assert abs(abs(rot[1, 2]) - 1) < 1e-6 and abs(rot[0, 0] - 1) < 1e-6
    body = d.shapes[0]
    assert body.has_uvs == 1 and d.bsdfs[body.bsdf].albedo_texture == 1
    assert d.bsdfs[d.shapes[1].bsdf].type == nh.BSDF_DIELECTRIC
    s.set_resolution(40, 30)
    img = no.OracleScene(s).render(0, 1, seed=1)
    assert np.isfinite(img).all() and img[..., :3].sum() > 0
