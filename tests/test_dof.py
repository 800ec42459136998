"""Thin-lens depth of field (PerspectiveCamera::sampleRay, src/cameras/perspective.cpp:114-130).

The reference takes the lens sample from one static Independent sampler created inside sampleRay
(perspective.cpp:118-119): a default-state pcg32 (ext/pcg32/pcg32.h:40) that is never prepare()d, two floats per
call, shared by every render thread. Its serial (one-thread) render order -- sample rounds (render.cpp:281-347),
blocks in BlockGenerator spiral order with clipped edge blocks (block.cpp:151-199), a block's pixels x-major
(independent.cpp:85-99) -- gives camera ray k = round * W * H + (position in the round) the draws 2k and 2k + 1.
The oracle and the HIP path reach them with pcg32::advance (pcg32.h:131-150). These CPU tests pin that mapping
against a literal sequential stream inside the oracle's serial loop (NO_RENDER_LENS_SERIAL), on a ragged image over
several rounds, in both sampler modes. The GPU comparison is in test_gpu_project_scenes.py.
"""
import os

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen


@pytest.fixture(scope="module")
def proj_dir(tmp_path_factory):
    return scenegen.materialize(str(tmp_path_factory.mktemp("proj")))


def dof_cbox(tmp_path, lens=0.08, focal=3.2):
    xml = scenegen.cbox_xml(str(tmp_path), "c2")
    text = open(xml).read()
    assert "<camera type=\"perspective\">" in text
    text = text.replace("<camera type=\"perspective\">",
                        f"<camera type=\"perspective\"><float name=\"lensRadius\" value=\"{lens}\"/>"
                        f"<float name=\"focalDistance\" value=\"{focal}\"/>", 1)
    path = os.path.join(os.path.dirname(xml), f"cbox_dof_{lens}_{focal}.xml")
    with open(path, "w") as f:
        f.write(text)
    return path


@pytest.mark.parametrize("order", [nh.LENS_DRAWS_RTL, nh.LENS_DRAWS_LTR])
@pytest.mark.parametrize("mode", [no.PER_PATH, no.NORI_BLOCK])
def test_lens_advance_equals_serial_stream(tmp_path, mode, order):
    """70x45 (3x2 blocks, ragged right and bottom edges), 3 rounds: every ray's lens sample by advance(2k) equals
    the literal sequential stream of the serial render loop, bit for bit, in both next2D argument orders."""
    s = nh.Scene(dof_cbox(tmp_path))
    s.set_resolution(70, 45)
    s.set_lens_draw_order(order)
    orc = no.OracleScene(s)
    serial = orc.render(0, 3, seed=3, mode=mode | no.LENS_SERIAL, threads=1)
    jump = orc.render(0, 3, seed=3, mode=mode, threads=4)
    np.testing.assert_array_equal(serial, jump)
    # depth of field is on: the image differs from the pinhole render of the same scene
    s0 = nh.Scene(dof_cbox(tmp_path, lens=0.0))
    s0.set_resolution(70, 45)
    pin = no.OracleScene(s0).render(0, 3, seed=3, mode=mode, threads=4)
    assert not np.array_equal(pin, jump)
    assert np.isfinite(jump).all() and jump[..., 3].sum() > 0


def test_lens_serial_needs_the_serial_loop(tmp_path):
    s = nh.Scene(dof_cbox(tmp_path))
    s.set_resolution(40, 40)
    orc = no.OracleScene(s)
    for kw in ({"threads": 2}, {"threads": 1, "blocks": [0]}):
        with pytest.raises(RuntimeError):
            orc.render(0, 1, mode=no.LENS_SERIAL, **kw)
    with pytest.raises(RuntimeError):
        orc.render(1, 2, mode=no.LENS_SERIAL, threads=1)


def test_lens_rounds_split_and_block_subsets(tmp_path):
    """Round ranges and block subsets place each ray at the same k: [0, 2) + [2, 3) = [0, 3), and two disjoint
    block subsets each equal the full render on their own blocks' interior pixels."""
    s = nh.Scene(dof_cbox(tmp_path))
    s.set_resolution(96, 64)
    orc = no.OracleScene(s)
    full = orc.render(0, 3, seed=9, threads=4)
    part = orc.render(0, 2, seed=9, threads=4)
    part = orc.render(2, 3, seed=9, threads=4, rgbw=part)
    np.testing.assert_allclose(part, full, rtol=1e-6, atol=1e-6)
    a = orc.render(0, 3, seed=9, threads=4, blocks=[0, 2, 4])
    b = orc.render(0, 3, seed=9, threads=4, blocks=[1, 3, 5])
    np.testing.assert_allclose(a + b, full, rtol=1e-5, atol=1e-6)


def test_reference_dof_scenes_load(proj_dir):
    """The reference's two thin-lens path_mis scenes load with the camera's fstop <-> lensRadius coupling
    (perspective.cpp:39-42): dof-val (fstop 1, focalDistance 18 -> lensRadius 18) and table_path_mis (lensRadius 1,
    focalDistance 80)."""
    a = nh.Scene(os.path.join(proj_dir, "scenes/project/dof/dof-val.xml")).desc.camera
    assert (a.width, a.height) == (800, 400)
    assert a.focal_distance == np.float32(18) and a.lens_radius == np.float32(18)
    b = nh.Scene(os.path.join(proj_dir, "scenes/project/dof/table_path_mis.xml")).desc.camera
    assert (b.width, b.height) == (800, 600)
    assert b.focal_distance == np.float32(80) and b.lens_radius == np.float32(1)


def test_reference_dof_scene_oracle_crop_serial(proj_dir):
    """dof-val.xml at a reduced 80x40 resolution, 2 rounds: the oracle's advance mapping equals the literal serial
    stream on the reference's own DOF scene."""
    s = nh.Scene(os.path.join(proj_dir, "scenes/project/dof/dof-val.xml"))
    s.set_resolution(80, 40)
    orc = no.OracleScene(s)
    np.testing.assert_array_equal(orc.render(0, 2, seed=1, mode=no.LENS_SERIAL, threads=1),
                                  orc.render(0, 2, seed=1, threads=4))


def test_lens_draw_order_default_and_effect(tmp_path):
    """The loader defaults to g++'s evaluation of Point2f(nextFloat(), nextFloat()) (right to left: x = draw 2k + 1,
    pinned by oracle/normalmap_probe "order" in test_normalmap.py); the other order gives another image."""
    s = nh.Scene(dof_cbox(tmp_path))
    assert s.desc.camera.lens_draw_order == nh.LENS_DRAWS_RTL
    s.set_resolution(48, 40)
    rtl = no.OracleScene(s).render(0, 2, seed=3)
    s.set_lens_draw_order(nh.LENS_DRAWS_LTR)
    assert s.desc.camera.lens_draw_order == nh.LENS_DRAWS_LTR
    ltr = no.OracleScene(s).render(0, 2, seed=3)
    assert not np.array_equal(rtl, ltr)
    with pytest.raises(nh.NoriError):
        s.set_lens_draw_order(2)
