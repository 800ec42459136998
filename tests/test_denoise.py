"""SimpleDenoiser (src/denoiser/simple.cpp:29-76, computeVarianceFromImage src/utils/common.cpp:339-398), the
denoiser the reference's render loop applies to the master ImageBlock (src/utils/render.cpp:368-369).

The reference ships no output of this denoiser (its report shows images only), so the oracle
(oracle/nori_oracle.cpp no_denoise_simple) is pinned by (a) the Eigen evaluation order of its colour
distance (Vector4f::lpNorm<1>, checked against ext/eigen in test_oracle_kat.py) and (b) a second,
independent restatement below in plain Python float32 arithmetic. The order is the reference's serial
loop (one TBB thread; with more its in-place rows race). GPU: nh_denoise / nh_denoise_image against the
oracle -- the same float operations in the same order; the only libm difference is exp() in double
(ROCm's vs glibc's) before rounding to float, so the tolerance is rel-L2 < 1e-6 and in practice every
pixel matches bit for bit.
"""
import math
import os

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen

F32 = np.float32


def py_denoise(blk, bs, sigma_d, sigma_vr, r, amount):
    """simple.cpp + common.cpp:339-398 restated with numpy float32 scalars (pure-Python loops)."""
    b = blk.astype(np.float32).copy()
    H, W = b.shape[0] - 2 * bs, b.shape[1] - 2 * bs

    def lum(px):
        c = [F32(px[k]) / F32(px[3]) for k in range(3)] if abs(px[3]) > F32(1e-4) else [F32(0)] * 3
        return F32(F32(F32(c[0] * F32(0.212671)) + F32(c[1] * F32(0.715160))) + F32(c[2] * F32(0.072169)))
    for _ in range(amount):
        var = np.zeros((H, W), np.float32)
        for i in range(H):
            for j in range(W):
                nb = [(i - 1 + k, j - 1 + l) for k in range(3) for l in range(3)
                      if 0 <= i - 1 + k < H and 0 <= j - 1 + l < W]
                mean, s = F32(0), F32(0)
                for a, c in nb:
                    mean = F32(mean + abs(lum(b[a + bs, c + bs])))
                    s = F32(s + 1)
                mean = F32(mean / s)
                col = F32(0)
                for a, c in nb:  # std::pow(float, 2): double
                    d = float(F32(abs(lum(b[a + bs, c + bs])) - mean))
                    col = F32(float(col) + float(F32(1) / s) * (d * d))
                var[i, j] = col
        mx, mn = var.max(), var.min()
        if F32(mx - mn) < F32(1e-4):
            var[:] = 0
        else:
            var = (F32(1) + (var - mn) / F32(mx - mn) * F32(0.254)).astype(np.float32)
        for i in range(H):
            for j in range(W):
                res, sw, ip = [F32(0)] * 4, F32(0), b[i + bs, j + bs].copy()
                for i_ in range(max(i - r, 0), min(i + r + 1, H)):
                    for j_ in range(max(j - r, 0), min(j + r + 1, W)):
                        dsq = (i - i_) ** 2 + (j - j_) ** 2
                        g = F32(math.exp(float(F32(F32(F32(F32(-dsq) / F32(2)) / F32(sigma_d)) / F32(sigma_d)))))
                        iq = b[i_ + bs, j_ + bs]
                        dd = [F32(ip[k] - iq[k]) for k in range(4)]
                        l1 = F32(F32(abs(dd[0]) + abs(dd[2])) + F32(abs(dd[1]) + abs(dd[3])))
                        x = F32(F32(l1 * var[i, j]) / F32(sigma_vr))
                        w = F32(g * F32(math.exp(-0.5 * (float(x) * float(x)))))
                        for k in range(4):
                            res[k] = F32(res[k] + F32(iq[k] * w))
                        sw = F32(sw + w)
                for k in range(4):
                    b[i + bs, j + bs, k] = F32(res[k] / sw)
    return b


def random_block(h, w, bs, seed):
    rng = np.random.default_rng(seed)
    blk = (rng.random((h + 2 * bs, w + 2 * bs, 4)) * 3).astype(np.float32)
    blk[..., 3] = rng.random(blk.shape[:2]).astype(np.float32) * 2
    blk[::3, ::4, 3] = 0.0  # zero filter weight: divideByFilterWeight's Color3f(0) branch
    return blk


@pytest.mark.parametrize("h,w,bs,r,amount,sigma_d,sigma_vr", [
    (5, 7, 2, 2, 1, 1.5, 0.6), (6, 4, 0, 1, 2, 6.0, 1.5), (3, 3, 1, 0, 1, 1.0, 1.0), (8, 9, 2, 3, 1, 2.0, 0.3),
    (1, 6, 2, 2, 1, 1.0, 0.6), (7, 1, 0, 3, 3, 0.0, 0.6)])
def test_oracle_denoise_matches_python_restatement(h, w, bs, r, amount, sigma_d, sigma_vr):
    blk = random_block(h, w, bs, h * 100 + w)
    p = nh.simple_denoiser(sigma_d, sigma_vr, r, amount)
    a = no.denoise_simple(blk, bs, p)
    b = py_denoise(blk, bs, p.sigma_d, p.sigma_vr, p.range, p.amount)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    # the border is not touched
    inner = np.zeros(blk.shape[:2], bool)
    inner[bs:bs + h, bs:bs + w] = True
    np.testing.assert_array_equal(a[~inner], blk[~inner])


def test_oracle_denoise_properties():
    blk = random_block(12, 10, 2, 9)
    # range 0: the window is p alone, weight exp(0) * exp(-0) = 1 -> unchanged, bit for bit
    np.testing.assert_array_equal(no.denoise_simple(blk, 2, nh.simple_denoiser(1.0, 0.6, 0, 3)), blk)
    # in place, row-major: the result differs from a two-buffer (Jacobi) sweep, and depends on it
    p = nh.simple_denoiser(2.0, 1.0, 2, 1)
    a = no.denoise_simple(blk, 2, p)
    assert not np.array_equal(a, blk)
    # the constructor's clamps (simple.cpp:15-24)
    q = nh.simple_denoiser(0.0, 99.0, 100, 0)
    assert q.sigma_d == np.float32(1e-4) and q.sigma_vr == 10.0 and q.range == 50 and q.amount == 1


def test_scene_loader_parses_denoiser(tmp_path):
    xml = scenegen.cbox_xml(str(tmp_path), "c2", 32, 24, 4, denoiser=(
        '<denoiser type="simple"><float name="sigma_d" value="6.0"/><float name="sigma_vr" value="1.5"/>'
        '<integer name="range" value="7"/></denoiser>'))
    d = nh.Scene(xml).desc.denoiser
    assert (d.type, d.sigma_d, d.sigma_vr, d.range, d.amount) == (nh.DENOISER_SIMPLE, 6.0, 1.5, 7, 1)
    # defaults and clamps: sigma_d 0 -> Epsilon, range 100 -> 50, amount 0 -> 1
    xml = scenegen.cbox_xml(str(tmp_path), "c2", 32, 24, 4, denoiser=(
        '<denoiser type="simple"><integer name="range" value="100"/><integer name="amount" value="0"/></denoiser>'))
    d = nh.Scene(xml).desc.denoiser
    assert (d.sigma_d, d.sigma_vr, d.range, d.amount) == (np.float32(1e-4), np.float32(0.6), 50, 1)
    assert nh.Scene(scenegen.cbox_xml(str(tmp_path), "c2", 32, 24, 4)).desc.denoiser.type == nh.DENOISER_NONE
    for bad in ('<denoiser type="simple"/><denoiser type="simple"/>', '<denoiser type="optix"/>'):
        with pytest.raises(nh.NoriError):
            nh.Scene(scenegen.cbox_xml(str(tmp_path), "c2", 32, 24, 4, denoiser=bad))


def rel_l2(a, b):
    return float(np.sqrt(np.sum((a.astype(np.float64) - b) ** 2) / max(np.sum(b.astype(np.float64) ** 2), 1e-300)))


@pytest.mark.gpu
@pytest.mark.parametrize("h,w,bs,r,amount,sigma_d,sigma_vr", [
    (1, 1, 0, 1, 1, 1.0, 0.6),        # single pixel
    (3, 70, 2, 2, 2, 1.5, 0.6),       # fewer rows than a band, two passes
    (37, 29, 2, 7, 1, 6.0, 1.5),      # ragged bands, the denoiser-test.xml parameters
    (64, 48, 1, 3, 3, 2.0, 0.3),      # three passes (the result ends in the framebuffer)
    (20, 23, 0, 12, 1, 4.0, 1.0),     # 625-term windows: several LDS chunks per pixel
    (16, 16, 2, 0, 1, 1.0, 0.6),      # range 0: identity
    (40, 5, 2, 9, 1, 3.0, 0.6),       # narrower than the window
    (50, 3, 0, 15, 2, 5.0, 0.9),      # range 15: the largest chunk the tiled kernel precomputes
    (24, 30, 2, 20, 1, 6.0, 1.5),     # range 20: chunk 21 > 16 precomputed steps -> the untiled kernel
    (70, 100, 2, 9, 1, 6.0, 1.5),     # range 9: full-size tile (45 KB) + the kernel's static LDS
    (64, 96, 2, 10, 1, 6.0, 1.5),     # range 10: full-size tile 48 KB, with the static LDS 74 KB
    (72, 112, 1, 11, 1, 6.0, 1.5),    # range 11: full-size tile 57 KB, with the static LDS 83 KB
])
@pytest.mark.parametrize("tile", [True, False], ids=["tile", "global"])
def test_denoise_image_matches_oracle(gpu, monkeypatch, tile, h, w, bs, r, amount, sigma_d, sigma_vr):
    if not tile:
        monkeypatch.setenv("NH_DENOISE_NO_TILE", "1")
    blk = random_block(h, w, bs, 7 * h + w)
    p = nh.simple_denoiser(sigma_d, sigma_vr, r, amount)
    ctx = nh.Context(0)
    g = ctx.denoise_image(blk, bs, p)
    o = no.denoise_simple(blk, bs, p)
    exact = float(np.mean(g.view(np.uint32) == o.view(np.uint32)))
    e = rel_l2(g, o)
    print(f"{h}x{w} b{bs} r{r} x{amount}: rel-L2 {e:.3e}, bit-exact {exact:.6f}")
    assert e < 1e-6 and exact > 0.999
    assert ctx.stats()["launches_denoise"] > 0


@pytest.mark.gpu
def test_denoise_after_render_matches_oracle(gpu, tmp_path):
    """render (wavefront, default knobs) -> Denoiser::denoise on the master block, as render.cpp:368-369"""
    xml = scenegen.cbox_xml(str(tmp_path), "c1", 96, 72, 8, denoiser=(
        '<denoiser type="simple"><float name="sigma_d" value="6.0"/><float name="sigma_vr" value="1.5"/>'
        '<integer name="range" value="7"/></denoiser>'))
    s = nh.Scene(xml)
    ctx = nh.Context(0)
    ctx.upload(s, nh.Bvh(s))
    ctx.render(0, 8, seed=3, clear=True, mode=nh.MODE_WAVEFRONT, traversal=nh.TRAVERSAL_ORDERED)
    ctx.denoise()
    g = ctx.framebuffer()
    r = no.OracleScene(s).render(0, 8, seed=3)
    o = no.denoise_simple(r, s.border, s.desc.denoiser)
    e = rel_l2(g, o)
    exact = float(np.mean(g.view(np.uint32) == o.view(np.uint32)))
    print(f"render + denoise: rel-L2 {e:.3e}, bit-exact {exact:.6f}")
    assert e < 1e-6 and exact > 0.999
    assert not np.array_equal(g, r)  # the denoiser changed the image
    # an invalid parameter set is refused, not clamped
    bad = nh.simple_denoiser()
    bad.range = 51
    with pytest.raises(nh.NoriError):
        ctx.denoise(bad)
