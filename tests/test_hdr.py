"""Radiance .hdr textures (PNGTexture::loadFromFile's ".hdr" branch, src/textures/PNGTexture.cpp:97-117, through
include/nori/HDRLoader.h): the loader's texels (host/hdr_decode.cpp) against a numpy restatement of HDRLoader's
per-pixel arithmetic (scenegen.rgbe_decode_reference: (m / 256.0f) * (float)pow(2, e - 128), alpha 0,
HDRLoader.h:28-46) on synthetic files in all three scanline encodings the reader accepts -- new-style run-length
(HDRLoader.h:98-131), flat RGBE pixels and the old (1, 1, 1, n) repeat codes with the chained << 8 count
(HDRLoader.h:49-83) -- including widths outside [8, 0x7fff], where every scanline is read the old way (:89-90), and a
flat scanline whose first pixel starts with byte 2 but is not a run-length header (:103-108). Rows land in file order
(:196-203). No .hdr ships with the reference; the reference's own decoder (include/nori/HDRLoader.h, a
self-contained header) is compiled here into oracle/_ref/hdr_probe (oracle/build_ref.sh), and
test_hdr_texels_match_reference_hdrloader pins the loader against it bit for bit on well-formed files of every
encoding (this container only: the GPU box has no reference checkout). Malformed files the reference reads into
undefined memory are errors here.
"""
import os

import numpy as np
import pytest

import nori_hip as nh
import scenegen


def envmap_scene(tmp_path, rgbe, mode, name="sky.hdr"):
    """An envmap scene whose spherical png_texture is `name`, holding `rgbe` in encoding `mode`."""
    d = str(tmp_path)
    h, w, _ = rgbe.shape
    xml = scenegen.envmap_xml(d, texture="hdr", tex_size=(w, h))
    path = os.path.join(d, name)
    scenegen.write_hdr(path, rgbe, mode=mode)
    text = open(xml).read().replace(f"sky_{w}x{h}.hdr", name)
    out = os.path.join(d, f"scene_{name}.xml")
    open(out, "w").write(text)
    return out


def env_texels(scene):
    e = scene.desc.env
    return np.ctypeslib.as_array(e.rgba, shape=(e.height, e.width, 4)).copy()


def random_rgbe(h, w, seed):
    """Random RGBE bytes with runs of equal pixels and equal components, every exponent from 0 to 255 somewhere;
    no literal pixel reads as an old repeat code (RGB = 1, 1, 1) and no scanline opens like a run-length header."""
    rng = np.random.default_rng(seed)
    px = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    px[..., 3] = rng.integers(0, 256, (h, w), dtype=np.uint8)
    for y in range(h):  # runs: a pixel repeated, a component repeated
        a = int(rng.integers(0, w))
        b = min(w, a + int(rng.integers(2, 300)))
        px[y, a:b] = px[y, a]
        c = int(rng.integers(0, 4))
        a = int(rng.integers(0, w))
        px[y, a:min(w, a + 140), c] = 7
    flat = px.reshape(-1, 4)
    flat[: min(256, flat.shape[0]), 3] = np.arange(min(256, flat.shape[0]), dtype=np.uint8)
    ones = (px[..., :3] == 1).all(-1)
    px[ones, 0] = 3
    px[:, 0, 0] = np.where(px[:, 0, 0] == 2, 5, px[:, 0, 0])
    return px


@pytest.mark.parametrize("mode", ["rle", "flat", "old"])
@pytest.mark.parametrize("w,h", [(37, 9), (300, 3), (5, 4), (1, 2)])
def test_hdr_texels_equal_the_restatement(tmp_path, mode, w, h):
    rgbe = random_rgbe(h, w, seed=w * 31 + h)
    if mode == "rle" and not 8 <= w <= 0x7FFF:
        mode = "flat"  # HDRLoader.h:89-90: such scanlines are never run-length encoded
    s = nh.Scene(envmap_scene(tmp_path, rgbe, mode))
    assert (s.desc.env.width, s.desc.env.height, s.desc.env.spherical) == (w, h, 1)
    want = scenegen.rgbe_decode_reference(rgbe)
    np.testing.assert_array_equal(env_texels(s), want)
    assert (want[..., 3] == 0).all()


def test_hdr_encodings_agree_and_rows_in_file_order(tmp_path):
    """The same pixels in the three encodings give the same texels; row 0 is the file's first scanline."""
    rgbe = random_rgbe(6, 40, seed=3)
    rgbe[0] = [200, 100, 50, 130]  # a bright first scanline
    out = [env_texels(nh.Scene(envmap_scene(tmp_path, rgbe, m, name=f"s_{m}.hdr"))) for m in ("rle", "flat", "old")]
    np.testing.assert_array_equal(out[0], out[1])
    np.testing.assert_array_equal(out[0], out[2])
    np.testing.assert_array_equal(out[0][0, :, :3], np.broadcast_to(np.float32([200, 100, 50]) / 256 * 4, (40, 3)))


def test_hdr_old_repeat_counts_chain(tmp_path):
    """Old-style scanlines: a repeat code repeats the previous pixel n times, a second code in a row n << 8 times
    (HDRLoader.h:63-73): a 700-pixel run is one literal pixel and (1,1,1,187) (1,1,1,2): 187 + 2 * 256 repeats."""
    w = 702
    rgbe = np.zeros((2, w, 4), np.uint8)
    rgbe[:, 0] = [9, 8, 7, 140]
    rgbe[:, 1:701] = [50, 60, 70, 129]
    rgbe[:, 701] = [10, 20, 30, 120]
    s = nh.Scene(envmap_scene(tmp_path, rgbe, "old"))
    np.testing.assert_array_equal(env_texels(s), scenegen.rgbe_decode_reference(rgbe))
    raw = open(os.path.join(str(tmp_path), "sky.hdr"), "rb").read()
    assert bytes([1, 1, 1, 699 & 255, 1, 1, 1, 699 >> 8]) in raw


def test_hdr_flat_scanline_opening_with_byte_2(tmp_path):
    """A flat scanline whose first pixel is (2, 2, 200, e) (200 has the high bit set: not a run-length header) is
    read as that pixel followed by old-style pixels (HDRLoader.h:103-108)."""
    rgbe = random_rgbe(3, 16, seed=5)
    rgbe[:, 0] = [2, 2, 200, 131]
    rgbe[1, 0] = [2, 7, 9, 126]  # (2, 7, ...): not (2, 2, ...), also a plain pixel
    s = nh.Scene(envmap_scene(tmp_path, rgbe, "flat"))
    np.testing.assert_array_equal(env_texels(s), scenegen.rgbe_decode_reference(rgbe))


def test_hdr_exponent_extremes(tmp_path):
    """Exponent bytes 0 and 255 (2^-128 is a float32 subnormal, 2^127 the largest power) and zero mantissas."""
    rgbe = np.array([[[255, 128, 1, 0], [255, 255, 254, 255], [0, 0, 0, 0], [0, 0, 0, 255], [17, 0, 3, 1],
                      [128, 64, 32, 128], [255, 1, 0, 136], [1, 2, 3, 100]]], np.uint8)
    s = nh.Scene(envmap_scene(tmp_path, rgbe, "flat"))
    got = env_texels(s)
    want = scenegen.rgbe_decode_reference(rgbe)
    np.testing.assert_array_equal(got, want)
    assert got[0, 0, 0] == np.float32(255 / 256) * np.float32(2.0 ** -128) and got[0, 0, 0] > 0
    assert got[0, 1, 0] == np.float32(255 / 256 * 2.0 ** 127)


def test_hdr_envmap_cdf_uses_the_texels(tmp_path):
    """EnvMap::calculateProbs over .hdr texels: the loader's CDF is monotone, ends at 1, and a sky twice as bright
    has the same CDF (normalised) and half the normalization."""
    rgbe = scenegen.rgbe_encode(scenegen.sky_image(32, 16).astype(np.float64) / 255.0 * 2.0)
    sa = nh.Scene(envmap_scene(tmp_path, rgbe, "rle", name="a.hdr"))  # (the scene owns the texels and CDF)
    a = sa.desc.env
    b_rgbe = rgbe.copy()
    b_rgbe[..., 3] = np.where(b_rgbe[..., 3] > 0, b_rgbe[..., 3] + 1, 0)
    sb = nh.Scene(envmap_scene(tmp_path, b_rgbe, "rle", name="b.hdr"))
    b = sb.desc.env
    ca = np.ctypeslib.as_array(a.cdf, shape=(32 * 16 + 1,))
    cb = np.ctypeslib.as_array(b.cdf, shape=(32 * 16 + 1,))
    assert ca[-1] == 1.0 and (np.diff(ca) >= 0).all()
    np.testing.assert_array_equal(ca, cb)
    assert b.normalization == np.float32(a.normalization) / 2


H = b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n"
BAD_FILES = {  # name: (file, the decoder's reason)
    "signature": (b"#?RGBE\nFORMAT=32-bit_rle_rgbe\n\n-Y 1 +X 1\n\x80\x80\x80\x80", "not a Radiance"),
    "truncated_header": (b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n", "truncated header"),
    # no header line: the newline after the signature is skipped (HDRLoader.h:152), so the reader looks for the empty
    # line past the resolution line (:157-164) -- the reference reads on into the pixels as well
    "empty_header": (b"#?RADIANCE\n\n-Y 1 +X 1\n\x80\x80\x80\x80", "truncated header"),
    "orientation": (H + b"+Y 1 +X 1\n\x80\x80\x80\x80", "resolution line"),
    "zero_size": (H + b"-Y 0 +X 4\n", "resolution line"),
    "truncated_flat": (H + b"-Y 2 +X 2\n" + b"\x80\x80\x80\x80" * 3, "scanline 1: truncated"),
    "repeat_first": (H + b"-Y 1 +X 2\n\x01\x01\x01\x02", "before the first pixel"),
    "repeat_past_end": (H + b"-Y 1 +X 2\n\x80\x80\x80\x80\x01\x01\x01\x05", "past the end"),
    "run_past_end": (H + b"-Y 1 +X 8\n\x02\x02\x00\x08" + b"\x89\x10" + b"\x88\x10" * 3, "run past the end"),
    # chained repeat codes: the count n << 8k must be checked before it is formed -- after three codes in
    # a row the reference's int shift is at 24 (n >= 128: negative), after four at 32 (undefined); both are errors,
    # not a silently skipped repeat
    "repeat_chain_24": (H + b"-Y 1 +X 4\n\x80\x80\x80\x80" + b"\x01\x01\x01\x00" * 3 + b"\x01\x01\x01\x80",
                        "past the end"),
    "repeat_chain_32": (H + b"-Y 1 +X 4\n\x80\x80\x80\x80" + b"\x01\x01\x01\x00" * 4 + b"\x01\x01\x01\x01",
                        "past the end"),
    "repeat_chain_64": (H + b"-Y 1 +X 4\n\x80\x80\x80\x80" + b"\x01\x01\x01\x00" * 9 + b"\x01\x01\x01\xff",
                        "past the end"),
    "truncated_rle": (H + b"-Y 1 +X 8\n\x02\x02\x00\x08\x88\x10\x88\x10", "scanline 0: truncated"),
}


@pytest.mark.parametrize("name", sorted(BAD_FILES))
def test_hdr_malformed_files_are_errors(tmp_path, name):
    d = str(tmp_path)
    xml = scenegen.envmap_xml(d, texture="hdr", tex_size=(8, 4))
    raw, why = BAD_FILES[name]
    open(os.path.join(d, "sky_8x4.hdr"), "wb").write(raw)
    with pytest.raises(nh.NoriError, match=r"Could not load HDR file\.\.\. \(.*" + why):
        nh.Scene(xml)


def test_hdr_well_formed_minimal_files(tmp_path):
    """The smallest files each encoding allows load: one flat pixel, and an 8-wide run-length scanline whose
    components are single runs (the header lines are skipped up to the empty line, HDRLoader.h:154-164)."""
    d = str(tmp_path)
    xml = scenegen.envmap_xml(d, texture="hdr", tex_size=(8, 4))
    cases = {
        b"#?RADIANCE\n# a comment\nEXPOSURE=1\n\n-Y 1 +X 1\n\x80\x40\x20\x81": np.uint8([[[128, 64, 32, 129]]]),
        H + b"-Y 1 +X 8\n\x02\x02\x00\x08\x88\x10\x88\x20\x88\x30\x88\x80":
            np.broadcast_to(np.uint8([16, 32, 48, 128]), (1, 8, 4)),
    }
    # zero-count repeat codes chain without effect (each only shifts the next count), then a literal pixel resets it
    cases[H + b"-Y 1 +X 2\n\x80\x40\x20\x81" + b"\x01\x01\x01\x00" * 6 + b"\x10\x20\x30\x82"] = \
        np.uint8([[[128, 64, 32, 129], [16, 32, 48, 130]]])
    for raw, rgbe in cases.items():
        open(os.path.join(d, "sky_8x4.hdr"), "wb").write(raw)
        np.testing.assert_array_equal(env_texels(nh.Scene(xml)), scenegen.rgbe_decode_reference(rgbe))


HDR_PROBE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "hdr_probe")


@pytest.mark.skipif(not os.path.exists(HDR_PROBE), reason="oracle/_ref/hdr_probe not built (needs /root/reference)")
@pytest.mark.parametrize("mode", ["rle", "flat", "old"])
@pytest.mark.parametrize("w,h", [(37, 9), (300, 3), (5, 4), (1, 2), (40000, 2)])
def test_hdr_texels_match_reference_hdrloader(tmp_path, mode, w, h):
    """The reference's HDRLoader::load (its own header, compiled into oracle/_ref/hdr_probe) and the product loader
    give the same texels bit for bit -- every encoding, widths inside and outside [8, 0x7fff] (40000: every scanline
    read the old way), every exponent."""
    import subprocess
    if mode == "rle" and not 8 <= w <= 0x7FFF:
        pytest.skip("run-length scanlines need 8 <= width <= 0x7fff")
    rgbe = random_rgbe(h, w, seed=w * 31 + h)
    xml = envmap_scene(tmp_path, rgbe, mode)
    mine = env_texels(nh.Scene(xml))
    out = tmp_path / "ref.bin"
    subprocess.run([HDR_PROBE, str(tmp_path / "sky.hdr"), str(out)], check=True, timeout=60)
    raw = np.fromfile(out, np.uint8)
    W, H = raw[:8].view(np.int32)
    assert (W, H) == (w, h)
    ref = raw[8:].view(np.float32).reshape(h, w, 4)
    np.testing.assert_array_equal(mine.view(np.uint32), ref.view(np.uint32))
