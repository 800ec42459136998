"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on identical inputs.

Traversal results are integer/index work plus fp32 arithmetic done in the same order, so
they must be bit-exact. Images: rel-L2 < 1e-4 (BASELINE.json north_star tolerance); the
megakernel and oracle evaluate the same fp32 operations in the same order, so in practice
they agree to the last bit and the test also reports the max abs difference.
"""
import os

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen

pytestmark = pytest.mark.gpu

TOL_REL_L2 = 1e-4


def rel_l2(a, b):
    return float(np.sqrt(np.sum((a.astype(np.float64) - b) ** 2) / max(np.sum(b.astype(np.float64) ** 2), 1e-300)))


def random_rays(n, lo, hi, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    mint = np.full(n, 1e-4, np.float32)
    maxt = np.full(n, np.inf, np.float32)
    # some finite segments and some axis-aligned directions (the d == 0 slab branch)
    maxt[::7] = rng.uniform(0.1, 3.0, size=maxt[::7].shape).astype(np.float32)
    d[::11, 0] = 0.0
    d[::13, 1] = 0.0
    # a denormal component (1/d = inf: the general slab path) and a tiny one (huge finite 1/d)
    d[5::17, 2] = 1e-39
    d[3::19, 1] = 3e-30
    return o, d.astype(np.float32), mint, maxt


def secondary_rays(oracle, n, seed):
    """Rays leaving surface points (origins on geometry, adaptive epsilon in play)."""
    o, d, mint, maxt = random_rays(n, -1.0, 2.0, seed)
    h = oracle.trace(o, d, mint, maxt)
    m = h["hit"] == 1
    with np.errstate(invalid="ignore", over="ignore"):
        p = o[m] + h["t"][m][:, None] * d[m]
    # a hit at t = inf is legal for an unbounded ray (t <= maxt, mesh.cpp:138) but has no surface point
    p = p[np.isfinite(p).all(axis=1)]
    assert len(p) > 0.9 * m.sum()
    rng = np.random.default_rng(seed + 1)
    d2 = rng.normal(size=p.shape).astype(np.float32)
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    return p.astype(np.float32), d2.astype(np.float32), np.full(len(p), 1e-4, np.float32), \
        np.full(len(p), np.inf, np.float32)


def compare_trace(ctx, oracle, o, d, mint, maxt, traversal):
    g = ctx.trace(o, d, mint, maxt, any_hit=False, traversal=traversal)
    r = oracle.trace(o, d, mint, maxt, any_hit=False)
    np.testing.assert_array_equal(g["hit"], r["hit"])
    m = r["hit"] == 1
    np.testing.assert_array_equal(g["t"][m], r["t"][m])
    np.testing.assert_array_equal(g["prim"][m], r["prim"][m])
    np.testing.assert_array_equal(g["shape"][m], r["shape"][m])
    np.testing.assert_array_equal(g["u"][m], r["u"][m])
    np.testing.assert_array_equal(g["v"][m], r["v"][m])
    ga = ctx.trace(o, d, mint, maxt, any_hit=True, traversal=traversal)
    ra = oracle.trace(o, d, mint, maxt, any_hit=True)
    np.testing.assert_array_equal(ga["hit"], ra["hit"])
    return int(m.sum())


def setup(xml, width=None, height=None):
    s = nh.Scene(xml)
    if width:
        s.set_resolution(width, height)
    b = nh.Bvh(s)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    return s, b, ctx


TRAVERSALS = [pytest.param(nh.TRAVERSAL_REFERENCE, id="reference"), pytest.param(nh.TRAVERSAL_ORDERED, id="ordered"),
              pytest.param(nh.TRAVERSAL_WIDE, id="wide")]


@pytest.mark.parametrize("traversal", TRAVERSALS)
def test_trace_parity_cbox(gpu, scene_dir, traversal):
    s, b, ctx = setup(os.path.join(scene_dir, "scenes/pa4/cbox/cbox_path_mis.xml"))
    orc = no.OracleScene(s)
    hits = compare_trace(ctx, orc, *random_rays(20000, -1.2, 2.0, 7), traversal)
    assert hits > 5000
    compare_trace(ctx, orc, *secondary_rays(orc, 20000, 11), traversal)


@pytest.mark.parametrize("traversal", TRAVERSALS + [pytest.param("wide8", id="wide8")])
def test_trace_parity_bumpy_mesh(gpu, tmp_path, monkeypatch, traversal):
    xml, ntri = scenegen.bumpy_cbox_xml(str(tmp_path), 200, 100)
    assert ntri > 30000
    if traversal == "wide8":  # the 8-wide collapse (NH_WIDE8=1, read when the BVH is uploaded)
        monkeypatch.setenv("NH_WIDE8", "1")
        traversal = nh.TRAVERSAL_WIDE
    s, b, ctx = setup(xml)
    orc = no.OracleScene(s)
    compare_trace(ctx, orc, *random_rays(20000, -0.6, 1.2, 3), traversal)
    compare_trace(ctx, orc, *secondary_rays(orc, 20000, 5), traversal)


MODES = [pytest.param(nh.MODE_MEGAKERNEL, id="mega"), pytest.param(nh.MODE_WAVEFRONT, id="wave")]


def render_pair(xml, w, h, spp, seed=5, traversal=nh.TRAVERSAL_REFERENCE, integrator=None, mode=nh.MODE_MEGAKERNEL):
    s = nh.Scene(xml)
    s.set_resolution(w, h)
    if integrator is not None:
        s.set_integrator(integrator)
    b = nh.Bvh(s)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(0, spp, seed=seed, traversal=traversal, clear=True, mode=mode)
    g = ctx.framebuffer()
    r = no.OracleScene(s).render(0, spp, seed=seed)
    return g, r, s


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("variant", ["c1", "c2"])
@pytest.mark.parametrize("traversal", [nh.TRAVERSAL_REFERENCE, nh.TRAVERSAL_ORDERED])
def test_render_parity_cbox(gpu, tmp_path, variant, traversal, mode):
    xml = scenegen.cbox_xml(str(tmp_path), variant)
    g, r, s = render_pair(xml, 64, 48, 16, traversal=traversal, mode=mode)
    e = rel_l2(g, r)
    print(f"{variant} traversal={traversal} mode={mode}: rel-L2 {e:.3e}, max|d| {np.abs(g - r).max():.3e}")
    assert e < TOL_REL_L2
    img_g, img_r = nh.to_rgb(g, s.border), nh.to_rgb(r, s.border)
    assert rel_l2(img_g, img_r) < TOL_REL_L2
    assert img_r.mean() > 0.05


@pytest.mark.parametrize("mode", MODES)
def test_render_parity_path_mats(gpu, tmp_path, mode):
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    g, r, _ = render_pair(xml, 48, 48, 16, integrator=nh.INTEGRATOR_PATH_MATS, mode=mode)
    assert rel_l2(g, r) < TOL_REL_L2


DIRECT = [pytest.param(nh.INTEGRATOR_DIRECT_EMS, id="direct_ems"), pytest.param(nh.INTEGRATOR_DIRECT_MATS, id="direct_mats"),
          pytest.param(nh.INTEGRATOR_DIRECT_MIS, id="direct_mis")]


@pytest.mark.parametrize("integrator", DIRECT)
@pytest.mark.parametrize("scene", ["c1", "envmap"])
def test_render_parity_direct(gpu, tmp_path, scene, integrator):
    """direct_ems / direct_mats / direct_mis (single bounce, run as the megakernel also when the
    wavefront mode is asked for) against the oracle: Cornell box with mirror + dielectric, and the
    PNG environment map scene (env terms of misses, occluded light samples and BSDF rays)."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1") if scene == "c1" else \
        scenegen.envmap_xml(str(tmp_path), texture="png", tex_size=(96, 48))
    for mode in (nh.MODE_WAVEFRONT, nh.MODE_MEGAKERNEL):
        g, r, s = render_pair(xml, 48, 40, 16, integrator=integrator, mode=mode, traversal=nh.TRAVERSAL_ORDERED)
        print(f"{scene} integrator={integrator} mode={mode}: rel-L2 {rel_l2(g, r):.3e}, max|d| {np.abs(g - r).max():.3e}")
        np.testing.assert_array_equal(g, r)
        assert nh.to_rgb(r, s.border).mean() > 0.01


def test_direct_ttest_scenes_match_oracle(gpu, scene_dir):
    """The reference's direct-integrator known-answer scenes (scenes/pa3/tests/test-mesh*.xml, 1x1
    pixel cameras) and the point-light scenes of the `direct` integrator (scenes/pa1/test-direct.xml,
    PointLight::sample/eval, pointlight.cpp:47-78): GPU render equals the oracle's bit for bit at 64 spp."""
    for name in ("pa3/tests/test-mesh.xml", "pa3/tests/test-mesh-furnace.xml", "pa1/test-direct.xml"):
        path = os.path.join(scene_dir, "scenes", name)
        for i in range(len(scenegen.test_references(path))):
            s = nh.Scene(path, i)
            b = nh.Bvh(s)
            ctx = nh.Context(0)
            ctx.upload(s, b)
            ctx.render(0, 64, seed=3, clear=True, mode=nh.MODE_MEGAKERNEL)
            np.testing.assert_array_equal(ctx.framebuffer(), no.OracleScene(s).render(0, 64, seed=3))


@pytest.mark.parametrize("mode", MODES)
def test_render_parity_microfacet_mesh(gpu, tmp_path, mode):
    xml, _ = scenegen.bumpy_cbox_xml(str(tmp_path), 120, 60)
    g, r, _ = render_pair(xml, 48, 40, 8, traversal=nh.TRAVERSAL_ORDERED, mode=mode)
    e = rel_l2(g, r)
    print(f"microfacet mesh rel-L2 {e:.3e}")
    assert e < TOL_REL_L2


def test_render_deterministic_and_sharded(gpu, tmp_path):
    """Two identical renders are bitwise equal; rendering two disjoint block sets into two
    framebuffers and summing equals the full render up to fp32 summation order."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    s = nh.Scene(xml)
    s.set_resolution(96, 80)
    b = nh.Bvh(s)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(0, 8, seed=3, clear=True)
    full = ctx.framebuffer()
    ctx.render(0, 8, seed=3, clear=True)
    np.testing.assert_array_equal(full, ctx.framebuffer())
    nb = 3 * 3
    parts = []
    for r in range(2):
        c2 = nh.Context(0)
        c2.upload(s, b)
        c2.render(0, 8, seed=3, blocks=list(range(r, nb, 2)), clear=True)
        parts.append(c2.framebuffer())
    assert rel_l2(parts[0] + parts[1], full) < 1e-6
    # sample-range split accumulates: [0,3) + [3,8) == [0,8) up to summation order
    ctx.render(0, 3, seed=3, clear=True)
    ctx.render(3, 8, seed=3, clear=False)
    assert rel_l2(ctx.framebuffer(), full) < 1e-6


@pytest.mark.parametrize("res,spp,blocks", [((100, 70), 6, None), ((33, 31), 4, None), ((200, 40), 5, [0, 2, 3, 5, 6, 9, 11]),
                                            ((64, 64), 3, [1, 2]), ((96, 96), 2, [4])])
def test_fused_splat_matches_staged_and_oracle(gpu, tmp_path, monkeypatch, res, spp, blocks):
    """The fused splat + merge (NH_SPLAT_FUSED=1: one workgroup per master tile, rounds in order, blocks in spiral
    order, no staging) and the staged pair -- one workgroup per block taking all rounds of the pixels only that block
    covers (default), or per round group with its first workgroup adding its rounds of those pixels straight into the
    master (NH_SPLAT_DIRECT=0, at 1 / 4 / 8 rounds per workgroup), every workgroup staging (NH_SPLAT_LEAD=0), the jitter read
    from a per-record array instead of recomputed from the path stream (NH_SPLAT_JITTER=stored), a persistent grid of
    3 workgroups walking the items (NH_SPLAT_WGS=3), 256-thread workgroups with 6-row strips instead of the default
    512 threads with 3-row strips (NH_SPLAT_T512=0, staged and all-direct), the all-direct splat in one launch with every
    band pixel staged and merged (NH_SPLAT_PAIR=0) instead of the default pair splat -- give the same
    framebuffer bit for bit, and the oracle's: partial blocks and the master border of the last block column / row
    (100x70, 33x31), block subsets whose neighbours are absent (every tile quadrant case), several chunks (1 MiB path
    budget) and both render modes."""
    xml = scenegen.cbox_xml(str(tmp_path), "c2")
    s = nh.Scene(xml)
    s.set_resolution(*res)
    b = nh.Bvh(s)
    out = {}
    d0 = {"NH_SPLAT_DIRECT": "0"}
    variants = ({}, d0, {**d0, "NH_SPLAT_LEAD": "0"}, {**d0, "NH_SPLAT_ROUNDS": "4"}, {**d0, "NH_SPLAT_ROUNDS": "1"},
                {"NH_SPLAT_FUSED": "1"}, {"NH_SPLAT_JITTER": "stored"}, {**d0, "NH_SPLAT_JITTER": "stored"},
                {**d0, "NH_SPLAT_WGS": "3"}, {"NH_SPLAT_T512": "0"}, {**d0, "NH_SPLAT_T512": "0"}, {"NH_SPLAT_PAIR": "0"})
    for env in variants:
        for name in ("NH_SPLAT_DIRECT", "NH_SPLAT_LEAD", "NH_SPLAT_ROUNDS", "NH_SPLAT_FUSED", "NH_SPLAT_JITTER",
                     "NH_SPLAT_WGS", "NH_SPLAT_T512", "NH_SPLAT_PAIR"):
            monkeypatch.delenv(name, raising=False)
        for name, val in env.items():
            monkeypatch.setenv(name, val)
        fused, direct = env.get("NH_SPLAT_FUSED", "0"), repr(sorted(env.items()))
        for mode in (nh.MODE_MEGAKERNEL, nh.MODE_WAVEFRONT):
            for budget in (None, "1"):
                if budget:
                    monkeypatch.setenv("NH_WF_BUDGET_MB", budget)
                    monkeypatch.setenv("NH_RECORD_BUDGET_MB", budget)
                ctx = nh.Context(0)
                ctx.upload(s, b)
                ctx.render(0, spp, seed=21, clear=True, mode=mode, blocks=blocks)
                out[(fused, direct, mode, budget)] = ctx.framebuffer()
                monkeypatch.delenv("NH_WF_BUDGET_MB", raising=False)
                monkeypatch.delenv("NH_RECORD_BUDGET_MB", raising=False)
    ref = no.OracleScene(s).render(0, spp, seed=21, blocks=blocks)
    assert np.abs(ref).sum() > 0
    for k, g in out.items():
        np.testing.assert_array_equal(g, ref, err_msg=str(k))


def test_wavefront_matches_megakernel(gpu, tmp_path, monkeypatch):
    """Same per-path random streams and arithmetic: the two schedules give bitwise-equal
    framebuffers and identical traversal work, also when the wavefront splits the rounds into
    several chunks (a 1 MiB path-state budget) and renders a block subset."""
    xml = scenegen.cbox_xml(str(tmp_path), "c2")
    s = nh.Scene(xml)
    s.set_resolution(160, 96)
    b = nh.Bvh(s)
    out = {}
    for mode in (nh.MODE_MEGAKERNEL, nh.MODE_WAVEFRONT):
        ctx = nh.Context(0)
        ctx.upload(s, b)
        ctx.render(0, 12, seed=9, traversal=nh.TRAVERSAL_ORDERED, clear=True, stats=True, mode=mode,
                   blocks=[0, 2, 3, 5, 7, 8, 11])
        out[mode] = (ctx.framebuffer(), ctx.stats())
    np.testing.assert_array_equal(out[0][0], out[1][0])
    for k in ("samples", "ray_queries", "nodes_visited", "prims_tested", "invalid_samples"):
        assert out[0][1][k] == out[1][1][k], k
    assert out[1][1]["launches_extend"] > 5
    monkeypatch.setenv("NH_WF_BUDGET_MB", "1")
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(0, 12, seed=9, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_WAVEFRONT,
               blocks=[0, 2, 3, 5, 7, 8, 11])
    np.testing.assert_array_equal(out[0][0], ctx.framebuffer())
    assert ctx.stats()["launches_splat"] > 1


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("texture,integrator", [("png", nh.INTEGRATOR_PATH_MIS), ("png", nh.INTEGRATOR_PATH_MATS),
                                                ("hdr", nh.INTEGRATOR_PATH_MIS), ("constant", nh.INTEGRATOR_PATH_MIS),
                                                ("none", nh.INTEGRATOR_PATH_MIS)])
def test_render_parity_envmap(gpu, tmp_path, texture, integrator, mode):
    """EnvMap emitter (NEE by luminance CDF, escaped-ray term) + png_texture lookups (a PNG or a Radiance .hdr sky),
    GPU vs oracle."""
    xml = scenegen.envmap_xml(str(tmp_path), texture=texture, tex_size=(96, 48))
    g, r, s = render_pair(xml, 64, 48, 8, integrator=integrator, mode=mode, traversal=nh.TRAVERSAL_ORDERED)
    e = rel_l2(g, r)
    print(f"envmap {texture} integrator={integrator} mode={mode}: rel-L2 {e:.3e}, max|d| {np.abs(g - r).max():.3e}")
    assert e < TOL_REL_L2
    assert nh.to_rgb(r, s.border).mean() > 0.05


@pytest.mark.parametrize("mode", MODES)
def test_envmap_guide_table(gpu, tmp_path, monkeypatch, mode):
    """EnvMap::sample's CDF search bracketed by the guide table (nh_device.h dpdf_sample_guided) gives the plain binary
    search's texel: images with and without the table (NH_ENV_GUIDE=0) equal each other and the oracle, on a sky large
    enough for a 2^12-entry table and with a hot spot (the bright sun: most samples land in a few brackets)."""
    xml = scenegen.envmap_xml(str(tmp_path), texture="png", tex_size=(256, 128))
    out = []
    for guide in ("1", "0"):
        monkeypatch.setenv("NH_ENV_GUIDE", guide)
        g, r, s = render_pair(xml, 48, 32, 8, mode=mode, traversal=nh.TRAVERSAL_ORDERED)
        out.append((g, r))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][0], out[0][1])


@pytest.mark.parametrize("mode", MODES)
def test_render_parity_black_envmap_mirror(gpu, tmp_path, mode):
    """An all-black PNG envmap (luminance table sums to 0: DiscretePDF's normalization 0) beside an area light and a
    mirror sphere. The reference's envmap light sample is then non-finite, so the light-sample skip at mirror hits
    must stay off (nee_finite); GPU vs oracle bit for bit. Parity unpinned (no reference output)."""
    xml = scenegen.envmap_xml(str(tmp_path), texture="png", tex_size=(32, 16), black=True)
    g, r, s = render_pair(xml, 64, 48, 8, mode=mode, traversal=nh.TRAVERSAL_ORDERED)
    np.testing.assert_array_equal(g, r)
    assert np.isfinite(g).all()


@pytest.mark.parametrize("knob", ["NH_PERSISTENT=1", "NH_PERSISTENT=1,NH_WIDE=0", "NH_PERSISTENT=0",
                                  "NH_LDS_SCENE=0", "NH_TAIL=0", "NH_TAIL=1000000", "NH_PERSISTENT=1,NH_TAIL=1000000",
                                  "NH_FUSED=0", "NH_SORT=0", "NH_SORT=1", "NH_FUSED=1,NH_TAIL=0",
                                  "NH_SORT_SHADE=1", "NH_FUSED=0,NH_SORT_SHADE=1", "NH_RR_AHEAD=0",
                                  "NH_RR_AHEAD=0,NH_TAIL=0", "NH_TRACE2=0", "NH_PERSISTENT=1,NH_TRACE2=0",
                                  "NH_LDS_FRAMES=0", "NH_EMIT_FACES=0",
                                  # the count kernel's handoff: the runtime copy + memset fallback, alone
                                  # and with in-place chunk ends
                                  "NH_COUNT_KERNEL=0", "NH_COUNT_KERNEL=0,NH_TAIL=0",
                                  # the 8-wide collapse: both-queries launch, split launches, tails
                                  "NH_WIDE8=1", "NH_WIDE8=1,NH_TRACE2=0", "NH_WIDE8=1,NH_PERSISTENT=1,NH_TAIL=1000000"])
def test_wavefront_variants_match(gpu, tmp_path, monkeypatch, knob):
    """The traversal variants the wavefront picks per scene (persistent ray-fetching traversal for
    deep BVHs over the binary or the 4-wide tree, per-lane traversal, LDS-staged small BVHs) all give
    the megakernel's framebuffer bit for bit, on a microfacet mesh (deep BVH) and on the Cornell box
    (LDS-sized BVH). Binary-tree variants also visit exactly the megakernel's nodes and primitives."""
    knobs = [k.split("=") for k in knob.split(",")]
    # the fused kernels answer rays inside an isolated sphere without walking the tree and the ray-queue kernels do
    # not (test_isolated_sphere_shortcut): traversal work is compared with the shortcut off in both contexts
    monkeypatch.setenv("NH_ISO_SPHERE", "0")
    for xml in (scenegen.bumpy_cbox_xml(str(tmp_path), 160, 80)[0], scenegen.cbox_xml(str(tmp_path), "c1")):
        s = nh.Scene(xml)
        s.set_resolution(48, 40)
        b = nh.Bvh(s)
        ref = nh.Context(0)
        ref.upload(s, b)
        ref.render(0, 6, seed=11, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_MEGAKERNEL, stats=True)
        for name, val in knobs:
            monkeypatch.setenv(name, val)
        ctx = nh.Context(0)
        ctx.upload(s, b)
        ctx.render(0, 6, seed=11, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_WAVEFRONT, stats=True)
        for name, _ in knobs:
            monkeypatch.delenv(name)
        np.testing.assert_array_equal(ref.framebuffer(), ctx.framebuffer())
        wide = ctx.stats()["node_bytes"] in (128, 256)
        if wide:
            assert (ctx.stats()["node_bytes"] == 256) == (dict(knobs).get("NH_WIDE8") == "1")
        env = dict(knobs)
        # the fused bounce kernel runs exactly when the BVH is traversed from LDS, unless NH_FUSED=0
        assert ctx.stats()["fused_bounce"] == int(ctx.stats()["lds_scene"] == 1 and env.get("NH_FUSED") != "0"), xml
        if s.desc.n_faces < 100 and not any(k in env for k in ("NH_LDS_SCENE", "NH_PERSISTENT")):  # the Cornell box
            assert ctx.stats()["lds_scene"] == 1
        persistent = env["NH_PERSISTENT"] == "1" if "NH_PERSISTENT" in env else b.desc.max_depth + 2 > 20
        assert wide == (persistent and env.get("NH_WIDE") != "0"), xml
        for k in ("ray_queries",) if wide else ("ray_queries", "nodes_visited", "prims_tested"):
            assert ref.stats()[k] == ctx.stats()[k], (xml, k)


@pytest.mark.parametrize("variant,tail,coop,waves", [("c1", "4096", "16", "4"), ("c1", "4096", "1", "4"),
                                                     ("c1", "200000", "16", "1"), ("c1", "64", "16", "4"),
                                                     ("c1", "4096", "16", "2"),
                                                     # C2 (diffuse only): the lean tail body (FULL = false)
                                                     ("c2", "4096", "16", "2"), ("c2", "4096", "1", "4"),
                                                     ("c2", "200000", "16", "2")])
def test_cooperative_tail_matches_oracle(gpu, tmp_path, monkeypatch, variant, tail, coop, waves):
    """The RR-ahead tail kernel's cooperative finish (NH_TAIL_COOP=16: once a tail wave carries <= 4 paths, each is
    carried by a 16-lane group that tests a leaf's primitives in one parallel step and reduces to the smallest t,
    ties to the later primitive) on the mirror + dielectric Cornell box (long specular chains), forced early by a
    small tail threshold, and the per-lane tail (NH_TAIL_COOP=1), at both register budgets: framebuffer and traversal
    counters equal the megakernel's, the framebuffer equals the oracle's. c2: the diffuse-only box, whose tail runs
    the lean body (no discrete-BSDF skip, texture lookup or isolated-sphere test compiled in) at 2 or 4 waves/SIMD."""
    xml = scenegen.cbox_xml(str(tmp_path), variant)
    s = nh.Scene(xml)
    s.set_resolution(64, 48)
    b = nh.Bvh(s)
    ref = nh.Context(0)
    ref.upload(s, b)
    ref.render(0, 8, seed=17, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_MEGAKERNEL, stats=True)
    for name, val in (("NH_TAIL", tail), ("NH_TAIL_COOP", coop), ("NH_TAIL_RR_WAVES", waves)):
        monkeypatch.setenv(name, val)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(0, 8, seed=17, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_WAVEFRONT, stats=True)
    st = ctx.stats()
    assert st["fused_bounce"] == 1 and st["launches_tail"] >= 1 and st["tail_bounces"] > 0
    assert (st["tail_coop_bounces"] > 0) == (coop == "16")  # the cooperative finish ran (its own clock slots)
    np.testing.assert_array_equal(ref.framebuffer(), ctx.framebuffer())
    for k in ("ray_queries", "nodes_visited", "prims_tested"):  # (the megakernel does not split off any-hit counts)
        assert ref.stats()[k] == st[k], k
    np.testing.assert_array_equal(ctx.framebuffer(), no.OracleScene(s).render(0, 8, seed=17))


def _render_stats(s, b, mode, integrator=None, **env):
    import os as _os
    old = {k: _os.environ.get(k) for k in env}
    _os.environ.update(env)
    try:
        ctx = nh.Context(0)
        ctx.upload(s, b)
        ctx.render(0, 8, seed=17, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=mode, stats=True)
        return ctx.framebuffer(), ctx.stats()
    finally:
        for k, v in old.items():
            if v is None:
                _os.environ.pop(k, None)
            else:
                _os.environ[k] = v


@pytest.mark.parametrize("integrator", [nh.INTEGRATOR_PATH_MIS, nh.INTEGRATOR_PATH_MATS])
def test_isolated_sphere_shortcut(gpu, tmp_path, integrator):
    """Rays leaving the surface of an isolated sphere (its box, grown by the host's margin, apart from every other
    primitive's: both Cornell-box spheres) that meet it again are answered by the sphere test alone
    (nh_traverse.h trace_next) in the megakernel and the fused wavefront kernels (RR-ahead bounce, its tail with and
    without the cooperative finish, the round-2 bounce, the per-lane tail). Every image equals the oracle's and the
    one rendered with the shortcut off (NH_ISO_SPHERE=0); the megakernel and the RR-ahead wavefront still do the
    same traversal work, and less of it than without the shortcut. Spheres sunk into the floor (boxes overlap) are
    not marked: the same work with the shortcut on or off."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    sunk = open(xml).read().replace(' 0.332100 ', ' 0.200000 ')  # both spheres into the floor
    assert sunk != open(xml).read()
    sunk_xml = os.path.join(os.path.dirname(xml), "cbox_sunk.xml")
    open(sunk_xml, "w").write(sunk)
    for path, isolated in ((xml, True), (sunk_xml, False)):
        s = nh.Scene(path)
        s.set_resolution(64, 48)
        s.set_integrator(integrator)
        b = nh.Bvh(s)
        ref = no.OracleScene(s).render(0, 8, seed=17)
        off, st_off = _render_stats(s, b, nh.MODE_MEGAKERNEL, NH_ISO_SPHERE="0")
        np.testing.assert_array_equal(off, ref)
        mk, st_mk = _render_stats(s, b, nh.MODE_MEGAKERNEL)
        np.testing.assert_array_equal(mk, ref)
        assert st_mk["ray_queries"] == st_off["ray_queries"]
        if isolated:
            assert st_mk["prims_tested"] < st_off["prims_tested"] and st_mk["nodes_visited"] < st_off["nodes_visited"]
        else:
            assert st_mk["prims_tested"] == st_off["prims_tested"] and st_mk["nodes_visited"] == st_off["nodes_visited"]
        for env in ({}, {"NH_TAIL": "1000000"}, {"NH_TAIL": "1000000", "NH_TAIL_COOP": "1"}, {"NH_RR_AHEAD": "0"},
                    {"NH_RR_AHEAD": "0", "NH_TAIL": "1000000"}, {"NH_FUSED": "0"}):
            wf, st_wf = _render_stats(s, b, nh.MODE_WAVEFRONT, **env)
            np.testing.assert_array_equal(wf, ref, err_msg=f"{path} {env}")
            if "NH_FUSED" not in env:  # every closest-hit query in a fused kernel: the megakernel's work
                for k in ("ray_queries", "nodes_visited", "prims_tested"):
                    assert st_wf[k] == st_mk[k], (path, env, k)


@pytest.mark.parametrize("mode", MODES)
def test_render_parity_c5_small(gpu, tmp_path, mode):
    """C5-shaped scene at test size: flattened transformed bumpy meshes (microfacet + diffuse),
    png envmap (sphericalTexture) + area light."""
    xml, ntri = scenegen.c5_xml(str(tmp_path), n_copies=4, n_phi=240, n_theta=60, width=48, height=40, spp=4,
                                sky=(120, 60))
    assert ntri > 50000
    g, r, s = render_pair(xml, 48, 40, 4, mode=mode, traversal=nh.TRAVERSAL_ORDERED)
    e = rel_l2(g, r)
    print(f"c5-small mode={mode}: rel-L2 {e:.3e}")
    assert e < TOL_REL_L2


_TORCH_WRAP = r"""
import os, sys
import numpy as np
import torch                      # first: the library then shares torch's HIP runtime (one per process)
torch.zeros(1, device="cuda:0")   # torch initialises the device before the library, as bench.py at N > 1
sys.path[:0] = [os.path.join(sys.argv[1], "optix-renderer_amd"), sys.argv[1]]
import importlib.util
import nori_hip as nh
import scenegen
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(sys.argv[1], "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
s = nh.Scene(scenegen.cbox_xml(sys.argv[2], "c2", width=64, height=48))
b = nh.Bvh(s)
ctx = nh.Context(0)
ctx.upload(s, b)
ctx.render(0, 4, seed=2, clear=True, mode=nh.MODE_WAVEFRONT, traversal=nh.TRAVERSAL_ORDERED)
# no nh_synchronize: the pointer call completes the submitted chunks (the pipeline advances only
# inside library calls), so a torch-side device sync is enough
ptr, n = ctx.framebuffer_device_ptr()
t = bench._wrap_device(ptr, n, 0)
torch.cuda.synchronize()
host = ctx.framebuffer().reshape(-1)
assert np.array_equal(t.cpu().numpy(), host)
t.mul_(2.0)  # writes through to the context's buffer
torch.cuda.synchronize()
assert np.array_equal(ctx.framebuffer().reshape(-1), host * np.float32(2.0))
print("torch-wrap ok", float(host.sum()))
"""


def test_framebuffer_device_pointer_wraps_in_torch(gpu, tmp_path):
    """bench.py hands the device framebuffer to torch.distributed (RCCL) through
    __cuda_array_interface__; the wrapped tensor must alias the context's framebuffer. Run in a fresh
    process that imports and initialises torch first, as bench.py's multi-GPU path does: the library
    then binds to torch's HIP runtime (two HIP runtimes in one process do not coexist)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "wrap.py"
    script.write_text(_TORCH_WRAP)
    r = subprocess.run([sys.executable, str(script), repo, str(tmp_path)], capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0 and "torch-wrap ok" in r.stdout


def test_persistent_traversal_deep_tree_spills(gpu, tmp_path, monkeypatch):
    """A tree deeper than the persistent kernel's 16-entry LDS stack window: entries spill to the
    global spill area and come back; the image and traversal counters still equal the
    megakernel's (which keeps the whole stack in LDS)."""
    xml, ntri = scenegen.bumpy_cbox_xml(str(tmp_path), 700, 250)
    s = nh.Scene(xml)
    s.set_resolution(40, 32)
    b = nh.Bvh(s, n_threads=8)
    assert b.desc.max_depth > 20, b.desc.max_depth
    monkeypatch.setenv("NH_WIDE", "0")
    out = []
    for mode, knob in ((nh.MODE_MEGAKERNEL, "0"), (nh.MODE_WAVEFRONT, "1")):
        monkeypatch.setenv("NH_PERSISTENT", knob)
        ctx = nh.Context(0)
        ctx.upload(s, b)
        ctx.render(0, 4, seed=21, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=mode, stats=True)
        out.append((ctx.framebuffer(), ctx.stats()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    for k in ("ray_queries", "nodes_visited", "prims_tested"):
        assert out[0][1][k] == out[1][1][k], k


@pytest.mark.parametrize("width", [4, 8])
def test_wide_traversal_deep_tree(gpu, tmp_path, monkeypatch, width):
    """The 4-wide (and 8-wide, NH_WIDE8=1) collapse on a deep tree (stack deeper than its 8-entry LDS window, so
    entries spill): closest and any hit bit-exact against the oracle's binary traversal, and the persistent
    wavefront render over it equals the megakernel's image bit for bit."""
    if width == 8:
        monkeypatch.setenv("NH_WIDE8", "1")
    xml, ntri = scenegen.bumpy_cbox_xml(str(tmp_path), 700, 250)
    s = nh.Scene(xml)
    s.set_resolution(40, 32)
    b = nh.Bvh(s, n_threads=8)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    orc = no.OracleScene(s)
    compare_trace(ctx, orc, *random_rays(20000, -0.6, 1.2, 13), nh.TRAVERSAL_WIDE)
    compare_trace(ctx, orc, *secondary_rays(orc, 20000, 17), nh.TRAVERSAL_WIDE)
    ctx.render(0, 4, seed=21, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_MEGAKERNEL, stats=True)
    ref, q = ctx.framebuffer(), ctx.stats()["ray_queries"]
    monkeypatch.setenv("NH_PERSISTENT", "1")
    ctx.reset_stats()
    ctx.render(0, 4, seed=21, traversal=nh.TRAVERSAL_ORDERED, clear=True, mode=nh.MODE_WAVEFRONT, stats=True)
    assert ctx.stats()["node_bytes"] == 32 * width
    assert ctx.stats()["ray_queries"] == q
    np.testing.assert_array_equal(ref, ctx.framebuffer())


def test_pipelined_chunks_match_one_pool(gpu, tmp_path, monkeypatch):
    """Asynchronous wavefront renders: several nh_render calls, several chunks per call (small
    memory budget), two path pools overlapping one chunk's last bounces with the next chunk.
    Splats land in submission order, so the framebuffer equals the one-pool run bit for bit, and
    both match the oracle."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    s = nh.Scene(xml)
    s.set_resolution(64, 48)
    b = nh.Bvh(s)
    monkeypatch.setenv("NH_WF_BUDGET_MB", "2")  # ~3 rounds per chunk at 64x48
    out = []
    for pools in ("2", "1"):
        ctx = nh.Context(0)
        ctx.upload(s, b)
        ctx.render(0, 0, clear=True, mode=nh.MODE_WAVEFRONT)
        for s0 in range(0, 12, 4):
            ctx.render(s0, s0 + 4, seed=9, traversal=nh.TRAVERSAL_ORDERED, mode=nh.MODE_WAVEFRONT)
        ctx.synchronize()
        out.append(ctx.framebuffer())
        monkeypatch.setenv("NH_POOLS", "1")
    np.testing.assert_array_equal(out[0], out[1])
    r = no.OracleScene(s).render(0, 12, seed=9)
    assert rel_l2(out[0], r) < TOL_REL_L2


def test_async_tails_match_in_place(gpu, tmp_path, monkeypatch):
    """Chunk tails handed off to tail slots (the live paths packed into the slot's buffer, the tail kernel and
    splat on the slot's stream, the pool taking the next chunk meanwhile) give the in-place tails' and the
    one-pool framebuffer bit for bit, over several calls of several chunks each; the hand-offs are counted."""
    xml = scenegen.cbox_xml(str(tmp_path), "c1")
    s = nh.Scene(xml)
    s.set_resolution(160, 128)
    b = nh.Bvh(s)
    monkeypatch.setenv("NH_WF_BUDGET_MB", "16")  # 2-3 rounds per chunk
    out = []
    for knobs in ({"NH_TAIL_ASYNC": "1"}, {"NH_TAIL_ASYNC": "1", "NH_POOLS": "2"}, {}, {"NH_POOLS": "1"}):
        for k, v in knobs.items():
            monkeypatch.setenv(k, v)
        ctx = nh.Context(0)
        ctx.upload(s, b)
        ctx.render(0, 0, clear=True, mode=nh.MODE_WAVEFRONT)
        for s0 in range(0, 24, 8):
            ctx.render(s0, s0 + 8, seed=4, traversal=nh.TRAVERSAL_ORDERED, mode=nh.MODE_WAVEFRONT)
        ctx.synchronize()
        out.append((ctx.framebuffer(), ctx.stats()))
        for k in knobs:
            monkeypatch.delenv(k)
    assert out[0][1]["tails_async"] > 3 and out[1][1]["tails_async"] > 3
    assert out[2][1]["tails_async"] == 0 and out[3][1]["tails_async"] == 0
    assert out[0][1]["launches_splat"] > 6
    for fb, _ in out[1:]:
        np.testing.assert_array_equal(out[0][0], fb)
    r = no.OracleScene(s).render(0, 24, seed=4)
    assert rel_l2(out[0][0], r) < TOL_REL_L2


def test_fast_reciprocal_exhaustive(gpu):
    """nhd::rcp_rn (hardware estimate + one FMA Newton step), which the triangle tests use for 1/det,
    equals the correctly rounded 1.0f / x for every one of the 2^32 float inputs in the range the
    kernels use it for (tools/rcp_exhaustive.hip, built by `make`)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "bin", "rcp_exhaustive")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=90)
    print(r.stdout.strip())
    assert r.returncode == 0, r.stdout + r.stderr
    assert "in_range_mismatches 0 " in r.stdout


def test_reduce_framebuffers_reuses_communicator(gpu, tmp_path):
    """nh_reduce_framebuffers (single-process RCCL reduce of per-GPU framebuffers): one box GPU, so a
    one-rank clique -- the sum over one rank is the framebuffer itself; the communicator is created on
    the first call and reused by the next, and a different context set gets its own."""
    s, b, ctx = setup(scenegen.cbox_xml(str(tmp_path), "c2"), 48, 40)
    ctx.render(0, 4, seed=2, clear=True, mode=nh.MODE_WAVEFRONT, traversal=nh.TRAVERSAL_ORDERED)
    ref = ctx.framebuffer()
    nh.reduce_framebuffers([ctx], root=0)
    nh.reduce_framebuffers([ctx], root=0)
    np.testing.assert_array_equal(ctx.framebuffer(), ref)
    assert ctx.stats()["comm_inits"] == 1
    other = nh.Context(0)
    other.upload(s, b)
    other.render(0, 4, seed=2, clear=True, mode=nh.MODE_WAVEFRONT, traversal=nh.TRAVERSAL_ORDERED)
    nh.reduce_framebuffers([other], root=0)
    assert other.stats()["comm_inits"] == 1
    np.testing.assert_array_equal(other.framebuffer(), ref)
    other.close()
    nh.reduce_framebuffers([ctx], root=0)  # the first set's clique is still alive
    assert ctx.stats()["comm_inits"] == 1


def test_manual_scene_description_through_cabi(gpu):
    """The binding path that needs no XML re-parse: a C program fills nh_scene_desc field by field
    (camera matrices, filter table, meshes with area CDFs, two spheres with microfacet / mirror BSDFs,
    an area light -- what per-plugin getHipRecord hooks would export), builds the BVH, renders through
    nh_render and compares with the oracle on the same description (tests/c/manual_scene.c)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "bin", "manual_scene")
    r = subprocess.run([exe, "8"], capture_output=True, text=True, timeout=120)
    print(r.stdout.strip(), r.stderr.strip())
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-identical 1" in r.stdout
