"""Textured diffuse albedo on the GPU: checkerboard_color / png_texture / constant_color children
of Diffuse (src/bsdf/diffuse.cpp:32-91) rendered by the HIP path equal the oracle bit for bit -- on crops (block
subsets) of the reference's own textured scenes (scenes/project/denoiser/denoiser-test.xml, scenes/pa1/mesh-texture.xml,
scenes/pa1/sphere-texture.xml) and on a png-textured Cornell box with scale / offset (negative uvs after the offset,
the reference's x86 cast semantics), in both render modes."""
import os

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen
from test_textures import aircraft_substituted, png_scene

pytestmark = pytest.mark.gpu

MODES = [pytest.param(nh.MODE_MEGAKERNEL, id="megakernel"), pytest.param(nh.MODE_WAVEFRONT, id="wavefront")]


@pytest.fixture(scope="module")
def tex_dir(tmp_path_factory):
    return scenegen.materialize(str(tmp_path_factory.mktemp("tex")))


def blocks_of(w, h, x0, y0, x1, y1):
    """32x32 block ids (by * nbx + bx) of the pixel rectangle [x0, x1) x [y0, y1)."""
    nbx = (w + 31) // 32
    return [by * nbx + bx for by in range(y0 // 32, (y1 + 31) // 32) for bx in range(x0 // 32, (x1 + 31) // 32)]


def render_both(s, spp, blocks, mode, seed=7, traversal=nh.TRAVERSAL_ORDERED):
    b = nh.Bvh(s)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(0, spp, seed=seed, blocks=blocks, traversal=traversal, clear=True, mode=mode)
    g = ctx.framebuffer()
    r = no.OracleScene(s).render(0, spp, seed=seed, blocks=blocks)
    return g, r


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("rel,rect", [
    # the checkerboard floor under the bowl and both lights' reflections (800x600 camera)
    ("scenes/project/denoiser/denoiser-test.xml", (224, 320, 608, 512)),
    ("scenes/pa1/mesh-texture.xml", (256, 224, 512, 480)),    # camel head (checkerboard) + plane, point light
    ("scenes/pa1/sphere-texture.xml", (224, 160, 480, 416)),  # checkerboard sphere, point light
])
def test_reference_textured_scene_crops(gpu, tex_dir, rel, rect, mode):
    s = nh.Scene(os.path.join(tex_dir, rel))
    d = s.desc
    blocks = blocks_of(d.camera.width, d.camera.height, *rect)
    g, r = render_both(s, 4, blocks, mode)
    print(f"{rel} mode={mode}: {len(blocks)} blocks, max|d| {np.abs(g - r).max():.3e}")
    np.testing.assert_array_equal(g, r)
    assert np.abs(r).sum() > 0


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("scale,offset,spherical", [(None, None, False), ((2.5, 0.75), (-0.3, 0.6), False),
                                                    (None, None, True)])
def test_png_albedo_cbox(gpu, tmp_path, scale, offset, spherical, mode):
    xml, _ = png_scene(tmp_path, scale=scale, offset=offset, spherical=spherical)
    s = nh.Scene(xml)
    s.set_resolution(64, 48)
    g, r = render_both(s, 8, None, mode)
    np.testing.assert_array_equal(g, r)
    # the texture shows: the same scene with the walls' constant albedo renders differently
    s2 = nh.Scene(scenegen.cbox_xml(str(tmp_path), "c2"))
    s2.set_resolution(64, 48)
    assert np.abs(no.OracleScene(s2).render(0, 8, seed=7) - r).max() > 1e-3


def test_checkerboard_through_cabi(gpu, tmp_path):
    """A texture added through nh_scene_add_texture (no XML) on the Cornell box walls, path_mis and path_mats."""
    s = nh.Scene(scenegen.cbox_xml(str(tmp_path), "c1"))
    s.set_resolution(48, 40)
    idx = s.add_texture(nh.TEXTURE_CHECKERBOARD, value1=(0.8, 0.2, 0.1), value2=(0.1, 0.3, 0.9), scale=(0.05, 0.1),
                        delta=(0.25, 0.0))
    s.set_bsdf(0, type=nh.BSDF_DIFFUSE, albedo=(0.5, 0.5, 0.5), albedo_texture=idx)
    for integ in (nh.INTEGRATOR_PATH_MIS, nh.INTEGRATOR_PATH_MATS):
        s.set_integrator(integ)
        for mode in (nh.MODE_MEGAKERNEL, nh.MODE_WAVEFRONT):
            g, r = render_both(s, 8, None, mode)
            np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("euler", [(0, 270, 0), (30, -45, 110)])
def test_envmap_euler_rotation(gpu, tmp_path, euler):
    """A spherical png envmap with eulerAngles (PNGTexture.cpp:133-139; the rotation is pinned against Eigen by
    test_transforms.py): NEE by the rotated luminance CDF, escaped rays, both modes, GPU = oracle."""
    xml = scenegen.envmap_xml(str(tmp_path), texture="png", tex_size=(96, 48), euler=euler)
    s = nh.Scene(xml)
    s.set_resolution(64, 48)
    for mode in (nh.MODE_MEGAKERNEL, nh.MODE_WAVEFRONT):
        g, r = render_both(s, 8, None, mode)
        np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("mode", MODES)
def test_aircraft_substituted_crop(gpu, tex_dir, mode):
    """scenes/project/textures/aircraft.xml (png_texture albedo on the aircraft's own texture coordinates, glass,
    envmap with eulerAngles 0,270,0) with synthetic stand-ins for its two absent images, a crop of its 800x600
    camera at 2 spp."""
    s = nh.Scene(aircraft_substituted(tex_dir))
    blocks = blocks_of(800, 600, 256, 192, 544, 416)
    g, r = render_both(s, 2, blocks, mode)
    np.testing.assert_array_equal(g, r)
    assert np.abs(r).sum() > 0
