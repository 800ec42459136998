"""The reference's project scenes on the GPU, HIP path vs oracle bit for bit (tests/golden/project_scenes.json.gz).

* Thin-lens depth of field (src/cameras/perspective.cpp:114-130): scenes/project/dof/dof-val.xml
  (fstop 1 -> lensRadius 18) and dof/table_path_mis.xml (lensRadius 1, a dielectric wine glass) on crops, in both
  render modes, with the crop's blocks split over two renders (as two ranks would take them) and over a round range
  that does not start at 0. Each ray's lens sample is the serial-order draw of the camera's static pcg32 stream
  (test_dof.py pins that mapping against the literal sequential stream); parity with the multi-threaded reference is
  unpinned (its lens draws race between threads).
* The reference's own envmap scene, scenes/project/envmap/envmap_sphere.xml with the shipped res/wooden_motel.png
  (environmentmap.cpp:73-169, PNGTexture eulerAngles 180,180,0): parity unpinned (no reference output exists), but
  the input is the reference's own instead of a synthetic sky.
"""
import os

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen

pytestmark = pytest.mark.gpu

MODES = [pytest.param(nh.MODE_MEGAKERNEL, id="megakernel"), pytest.param(nh.MODE_WAVEFRONT, id="wavefront")]


@pytest.fixture(scope="module")
def proj_dir(tmp_path_factory):
    return scenegen.materialize(str(tmp_path_factory.mktemp("proj")))


def blocks_of(w, h, x0, y0, x1, y1):
    """32x32 block ids (by * nbx + bx) of the pixel rectangle [x0, x1) x [y0, y1)."""
    nbx = (w + 31) // 32
    return [by * nbx + bx for by in range(y0 // 32, (y1 + 31) // 32) for bx in range(x0 // 32, (x1 + 31) // 32)]


def gpu_render(s, s0, s1, blocks, mode, seed=7):
    b = nh.Bvh(s)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(s0, s1, seed=seed, blocks=blocks, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=mode)
    return ctx.framebuffer()


DOF_CROPS = [
    ("scenes/project/dof/dof-val.xml", (320, 128, 512, 288)),           # the centre cube, in focus, and the lights
    ("scenes/project/dof/table_path_mis.xml", (288, 192, 544, 416)),    # the glasses and bowls on the table
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("rel,rect", DOF_CROPS)
def test_reference_dof_scene_crops(gpu, proj_dir, rel, rect, mode):
    s = nh.Scene(os.path.join(proj_dir, rel))
    d = s.desc.camera
    assert d.lens_radius > 1e-4
    blocks = blocks_of(d.width, d.height, *rect)
    g = gpu_render(s, 0, 4, blocks, mode)
    r = no.OracleScene(s).render(0, 4, seed=7, blocks=blocks)
    print(f"{rel} mode={mode}: {len(blocks)} blocks, max|d| {np.abs(g - r).max():.3e}")
    np.testing.assert_array_equal(g, r)
    assert r[..., 3].sum() > 0 and np.abs(r[..., :3]).sum() > 0


@pytest.mark.parametrize("mode", MODES)
def test_dof_crop_clang_draw_order_and_late_rounds(gpu, proj_dir, mode):
    """dof-val.xml with the other next2D argument order (x = draw 2k, as clang compiles Independent::next2D) over
    rounds [300, 302) and [255, 257) (the lens tables' low / high round split at 256): GPU = oracle bit for bit."""
    s = nh.Scene(os.path.join(proj_dir, "scenes/project/dof/dof-val.xml"))
    s.set_lens_draw_order(nh.LENS_DRAWS_LTR)
    d = s.desc.camera
    blocks = blocks_of(d.width, d.height, 352, 160, 480, 256)
    orc = no.OracleScene(s)
    for r0 in (300, 255):
        g = gpu_render(s, r0, r0 + 2, blocks, mode, seed=5)
        r = orc.render(r0, r0 + 2, seed=5, blocks=blocks)
        np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("mode", MODES)
def test_dof_block_split_and_round_offset(gpu, proj_dir, mode):
    """dof-val.xml: the crop's blocks split in two renders (alternate blocks, as two ranks take them) over rounds
    [3, 5): each half equals the oracle's render of the same blocks and rounds."""
    s = nh.Scene(os.path.join(proj_dir, "scenes/project/dof/dof-val.xml"))
    d = s.desc.camera
    blocks = blocks_of(d.width, d.height, 256, 96, 544, 320)
    orc = no.OracleScene(s)
    for half in (blocks[0::2], blocks[1::2]):
        g = gpu_render(s, 3, 5, half, mode, seed=11)
        r = orc.render(3, 5, seed=11, blocks=half)
        np.testing.assert_array_equal(g, r)


def test_dof_cbox_full_image_wavefront(gpu, tmp_path):
    """A thin-lens Cornell box (c1: mirror + dielectric spheres) at 160x120, 6 spp, whole image through the default
    wavefront pipeline (path pools, tails) equals the oracle."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    text = open(xml).read().replace('<camera type="perspective">',
                                    '<camera type="perspective"><float name="lensRadius" value="0.1"/>'
                                    '<float name="focalDistance" value="4.5"/>', 1)
    path = os.path.join(os.path.dirname(xml), "cbox_c1_dof.xml")
    with open(path, "w") as f:
        f.write(text)
    s = nh.Scene(path)
    s.set_resolution(160, 120)
    g = gpu_render(s, 0, 6, None, nh.MODE_WAVEFRONT, seed=2)
    r = no.OracleScene(s).render(0, 6, seed=2)
    np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("knobs", [{"NH_PERSISTENT": "1", "NH_LDS_SCENE": "0"},
                                   {"NH_PERSISTENT": "1", "NH_LDS_SCENE": "0", "NH_TRACE2": "0"},
                                   {"NH_PERSISTENT": "1", "NH_LDS_SCENE": "0", "NH_WIDE": "0"}])
def test_dof_persistent_camera_rays(gpu, tmp_path, monkeypatch, knobs):
    """Thin-lens scenes on the persistent traversal kernels: bounce 0's camera rays (with their lens samples) are
    written by wf_camera_rays and read by the persistent refill (4-wide both-queries launch, 4-wide split launches,
    binary tree). A thin-lens Cornell box forced off the LDS-staged path, 96x64, 4 spp: GPU = oracle bit for bit."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    text = open(xml).read().replace('<camera type="perspective">',
                                    '<camera type="perspective"><float name="lensRadius" value="0.1"/>'
                                    '<float name="focalDistance" value="4.5"/>', 1)
    path = os.path.join(os.path.dirname(xml), "cbox_c1_dof_pt.xml")
    with open(path, "w") as f:
        f.write(text)
    s = nh.Scene(path)
    s.set_resolution(96, 64)
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    g = gpu_render(s, 0, 4, None, nh.MODE_WAVEFRONT, seed=6)
    r = no.OracleScene(s).render(0, 4, seed=6)
    np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("mode", MODES)
def test_reference_envmap_sphere_crop(gpu, proj_dir, mode):
    """envmap_sphere.xml (800x800, path_mis, the shipped wooden_motel.png envmap rotated by eulerAngles 180,180,0
    around a diffuse sphere): a crop over the sphere's limb and the background."""
    s = nh.Scene(os.path.join(proj_dir, "scenes/project/envmap/envmap_sphere.xml"))
    d = s.desc.camera
    assert (d.width, d.height) == (800, 800)
    blocks = blocks_of(d.width, d.height, 256, 320, 544, 480)
    g = gpu_render(s, 0, 4, blocks, mode)
    r = no.OracleScene(s).render(0, 4, seed=7, blocks=blocks)
    print(f"envmap_sphere mode={mode}: {len(blocks)} blocks, max|d| {np.abs(g - r).max():.3e}")
    np.testing.assert_array_equal(g, r)
    assert np.abs(r[..., :3]).sum() > 0


# ---- shape normal maps (tests/golden/normalmap_scenes.json.gz) -------------------------
# Mesh::setHitInformation's TBN branch (mesh.cpp:173-183), Sphere::setHitInformation's re-framing (sphere.cpp:115-121)
# and PNGTexture's normal-map decode + eval (PNGTexture.cpp:26, :85-95, :155-161); the decode and the arithmetic are
# pinned against the reference's own lodepng + Eigen in test_normalmap.py.
NORMALMAP_CROPS = [
    ("scenes/project/normalmap/normals-identity-direct.xml", (224, 160, 576, 416)),    # sphere, cube, cone, plane
    ("scenes/project/normalmap/normals-primitives-direct.xml", (224, 160, 576, 416)),
    ("scenes/project/normalmap/normals-camel.xml", (224, 128, 544, 448)),              # the camel head (22.7k tris)
    # the `normals` integrator (normals.cpp): |shFrame.n| itself, the most direct view of the mapped frames
    ("scenes/project/normalmap/normals-identity.xml", (224, 160, 576, 416)),
    ("scenes/project/normalmap/normals-identity-x.xml", (224, 160, 576, 416)),
    ("scenes/project/normalmap/normals-identity-y.xml", (224, 160, 576, 416)),
    ("scenes/project/normalmap/normals-primitives.xml", (224, 160, 576, 416)),
    ("scenes/project/normalmap/normals-identity-ref.xml", (224, 160, 576, 416)),  # no maps: the reference view
]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("rel,rect", NORMALMAP_CROPS)
def test_reference_normalmap_scene_crops(gpu, proj_dir, rel, rect, mode):
    s = nh.Scene(os.path.join(proj_dir, rel))
    d = s.desc
    assert any(d.shapes[i].normal_map for i in range(d.n_shapes)) or rel.endswith("-ref.xml")
    blocks = blocks_of(d.camera.width, d.camera.height, *rect)
    g = gpu_render(s, 0, 3, blocks, mode)
    r = no.OracleScene(s).render(0, 3, seed=7, blocks=blocks)
    print(f"{rel} mode={mode}: {len(blocks)} blocks, max|d| {np.abs(g - r).max():.3e}")
    np.testing.assert_array_equal(g, r)
    assert np.abs(r[..., :3]).sum() > 0


def normalmap_cbox(tmp_path, variant="c1", camel=False):
    """The Cornell box (path_mis) with normal maps: both spheres (c1: mirror + dielectric) take normal-test.png, a
    cube mesh with normals and uvs takes normal-primitives.png at intensity 0.7; camel = the camel head (normals +
    uvs, 22.7k triangles: a BVH past the LDS-staged size) with normal-test.png in place of the cube."""
    proj = scenegen.materialize(str(tmp_path))
    nm = ('<texture type="png_texture" name="normal"><string name="filename" value="../../project/res/{}"/>'
          '{}</texture>')
    if camel:
        mesh = ('<shape type="obj"><string name="filename" value="../../project/meshes/camelhead.obj"/>'
                + nm.format("normal-test.png", "") +
                '<bsdf type="diffuse"><color name="albedo" value="0.6 0.5 0.4"/></bsdf>'
                '<transform name="toWorld"><scale value="1.4,1.4,1.4"/><translate value="0,0.55,-0.1"/></transform>'
                '</shape>')
    else:
        mesh = ('<shape type="obj"><string name="filename" value="../../project/meshes/cube.obj"/>'
                + nm.format("normal-primitives.png", '<float name="intensity" value="0.7"/>') +
                '<bsdf type="diffuse"><color name="albedo" value="0.5 0.6 0.7"/></bsdf>'
                '<transform name="toWorld"><scale value="0.3,0.3,0.3"/><rotate axis="0,1,0" angle="30"/>'
                '<translate value="0.1,0.15,-0.55"/></transform></shape>')
    xml = scenegen.cbox_xml(str(tmp_path), variant, extra_shapes=mesh, drop_spheres=camel)
    text = open(xml).read()
    if not camel:
        text = text.replace('<float name="radius" value="0.3263" />',
                            '<float name="radius" value="0.3263" />' + nm.format("normal-test.png", ""))
        assert text.count("normal-test.png") == 2
    path = os.path.join(os.path.dirname(xml), f"cbox_{variant}_nmap{'_camel' if camel else ''}.xml")
    with open(path, "w") as f:
        f.write(text)
    return path


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("variant", ["c1", "c2"])
def test_normalmap_cbox_path_mis(gpu, tmp_path, variant, mode):
    """path_mis on a Cornell box whose spheres and a cube mesh carry normal maps, whole image (96x72, 6 spp) through
    the default pipelines: GPU = oracle bit for bit (c1: mirror + dielectric spheres; c2: diffuse spheres)."""
    s = nh.Scene(normalmap_cbox(tmp_path, variant))
    d = s.desc
    assert [d.shapes[i].normal_map != 0 for i in range(d.n_shapes)].count(True) == 3
    s.set_resolution(96, 72)
    g = gpu_render(s, 0, 6, None, mode, seed=4)
    r = no.OracleScene(s).render(0, 6, seed=4)
    np.testing.assert_array_equal(g, r)
    s2 = nh.Scene(normalmap_cbox(tmp_path, variant))
    s2.set_resolution(96, 72)
    for i in range(s2.desc.n_shapes):
        s2.set_normal_map(i, 0)
    plain = no.OracleScene(s2).render(0, 6, seed=4)
    assert not np.array_equal(plain, r)  # the maps do change the image


@pytest.mark.parametrize("mode", MODES)
def test_normalmap_deep_bvh_path_mis(gpu, tmp_path, mode):
    """The camel head (normals + uvs, 22.7k triangles, a BVH the kernels traverse from HBM) with a normal map in the
    Cornell box, path_mis, 64x64, 4 spp: GPU = oracle bit for bit."""
    s = nh.Scene(normalmap_cbox(tmp_path, "c2", camel=True))
    s.set_resolution(64, 64)
    g = gpu_render(s, 0, 4, None, mode, seed=8)
    r = no.OracleScene(s).render(0, 4, seed=8)
    np.testing.assert_array_equal(g, r)
