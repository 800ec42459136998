"""The oracle against the reference's own known answers (CPU only).

  - pcg32: ext/pcg32/pcg32-demo.out (5 rounds of u32 / coins / rolls / card shuffles) -- bit-exact;
  - path integrators: scenes/pa4/tests/test-furnace.xml and test-direct.xml, run with the
    reference's StudentsTTest scene procedure (src/utils/ttest.cpp:191-240: one default-seeded
    Independent sampler drawn sequentially across the file's scenes, 100k paths each, Welford
    mean/variance, Student-t test with Sidak correction at alpha = 0.01);
  - microfacet BSDF: scenes/pa3/tests/ttest-microfacet.xml (ttest.cpp:147-190) and
    chi2test-microfacet.xml (src/utils/chi2test.cpp:121-230: 10x20 cos(theta)/phi table,
    5000 samples per cell, pooled cells below 5 expected, Sidak-corrected chi^2 test).
Where the reference checkout is present, every verdict is also taken from the reference's own test procedures
(ext/hypothesis/hypothesis.h compiled into oracle/_ref/hypothesis_probe) on the same estimates, and must agree.
"""
import json
import math
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest
from scipy import stats

import nori_hip as nh
import nori_oracle as no
import scenegen

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---------------------------------------------------------------------------------------
def pcg_bounded(r, bound):
    """pcg32::nextUInt(bound) (ext/pcg32/pcg32.h:69-98)."""
    threshold = ((1 << 32) - bound) % bound
    while True:
        x = r.next_uint()
        if x >= threshold:
            return x % bound


def test_pcg32_demo_known_answers():
    kat = json.load(open(os.path.join(GOLDEN, "pcg32_kat.json")))
    r = no.Pcg32.seeded(*kat["seed"])
    number, suit = "A23456789TJQK", "hcds"
    for rnd in kat["rounds"]:
        assert [r.next_uint() for _ in range(6)] == rnd["u32"]
        assert "".join("H" if pcg_bounded(r, 2) else "T" for _ in range(65)) == rnd["coins"]
        assert [pcg_bounded(r, 6) + 1 for _ in range(33)] == rnd["rolls"]
        cards = list(range(52))
        for i in range(51, 0, -1):  # pcg32::shuffle (Knuth)
            j = pcg_bounded(r, i + 1)
            cards[i], cards[j] = cards[j], cards[i]
        assert [number[c // 4] + suit[c % 4] for c in cards] == rnd["cards"]


def splitmix64(x):
    m = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def pcg_seed_py(initstate, initseq):
    m = (1 << 64) - 1
    mult = 0x5851F42D4C957F2D
    inc = ((initseq << 1) | 1) & m
    state = 0
    state = (state * mult + inc) & m
    state = (state + initstate) & m
    state = (state * mult + inc) & m
    return state, inc


@pytest.mark.parametrize("seed,pixel,sample", [(0, 0, 0), (1234, 1023 * 1024 + 5, 255), (2**63 + 7, 12345, 99999)])
def test_per_path_seeding_contract(seed, pixel, sample):
    """pcg32.seed(splitmix64(seed ^ pixel), sample) -- the contract the GPU uses."""
    r = no.Pcg32.per_path(seed, pixel, sample)
    st, inc = pcg_seed_py(splitmix64(seed ^ pixel), sample)
    assert (r.state.value, r.inc.value) == (st, inc)


# ---------------------------------------------------------------------------------------
HYP_PROBE = os.path.join(os.path.dirname(no.__file__), "_ref", "hypothesis_probe")


def reference_verdicts(requests, tmp_dir):
    """The reference's hypothesis::students_t_test / chi2_test (oracle/_ref/hypothesis_probe) on the given requests:
    ("t", mean, var, ref, n, alpha, k) or ("chi2", obs, exp, n, min_exp, alpha, k). None without the probe."""
    import subprocess
    import tempfile
    if not os.path.exists(HYP_PROBE):
        return None
    d = tempfile.mkdtemp(dir=tmp_dir)
    lines = []
    for i, r in enumerate(requests):
        if r[0] == "t":
            lines.append("t " + " ".join(repr(float(x)) if j < 3 or j == 4 else str(int(x)) for j, x in enumerate(r[1:])))
        else:
            _, obs, exp, n, min_exp, alpha, k = r
            f = os.path.join(d, f"c{i}.bin")
            np.concatenate([np.asarray(obs, np.float64), np.asarray(exp, np.float64)]).tofile(f)
            lines.append(f"chi2 {f} {len(obs)} {int(n)} {float(min_exp)!r} {float(alpha)!r} {int(k)}")
    inp, out = os.path.join(d, "in.txt"), os.path.join(d, "out.txt")
    open(inp, "w").write("\n".join(lines) + "\n")
    subprocess.run([HYP_PROBE, inp, out], check=True, timeout=120)
    return [x.strip() == "1" for x in open(out)]


def students_t_test(mean, variance, reference, n, alpha, num_tests):
    """hypothesis::students_t_test (ext/hypothesis/hypothesis.h:314-346)."""
    t = abs(mean - reference) * math.sqrt(n / max(variance, 1e-5))
    pval = 2 * (1 - stats.t.cdf(t, n - 1))
    sidak = 1.0 - (1.0 - alpha) ** (1.0 / num_tests)
    return not (pval < sidak or not math.isfinite(pval)), pval


@pytest.mark.parametrize("name", ["pa4/tests/test-furnace.xml", "pa4/tests/test-direct.xml",
                                  "pa3/tests/test-mesh.xml", "pa3/tests/test-mesh-furnace.xml",
                                  "pa1/test-direct.xml"])
def test_scene_ttests(scene_dir, tmp_path, name):
    """pa4: path_mats / path_mis; pa3: direct_ems / direct_mats / direct_mis (5 + 2 scenes each);
    pa1: the point-light `direct` integrator (4 scenes: visible, visible, hidden, all three lights)."""
    path = os.path.join(scene_dir, "scenes", name)
    refs = scenegen.test_references(path)
    rng = no.Pcg32()  # Independent sampler created once, never prepare()d (ttest.cpp:193-194)
    results = []
    for i, ref in enumerate(refs):
        s = nh.Scene(path, i)
        mean, var = no.OracleScene(s).ttest(rng, 100000)
        ok, p = students_t_test(mean, var, ref, 100000, 0.01, len(refs))
        results.append((i, mean, ref, p, ok, var))
    assert all(r[4] for r in results), results
    theirs = reference_verdicts([("t", m, v, r, 100000, 0.01, len(refs)) for _, m, r, _, _, v in results], tmp_path)
    if theirs is not None:  # the reference's own hypothesis.h agrees
        assert theirs == [r[4] for r in results], (theirs, results)


def microfacet_from_xml(node):
    b = nh.nh_bsdf()
    b.type = nh.BSDF_MICROFACET
    vals = {f.get("name"): f.get("value") for f in node}
    b.alpha = float(vals.get("alpha", 0.1))
    b.int_ior = float(vals.get("intIOR", 1.5046))
    b.ext_ior = float(vals.get("extIOR", 1.000277))
    kd = np.array([float(x) for x in vals.get("kd", "0.5 0.5 0.5").replace(",", " ").split()], np.float32)
    for i in range(3):
        b.kd[i] = kd[i]
    m = kd[1] if not (kd[1] < kd[2]) else kd[2]
    m = kd[0] if not (kd[0] < m) else m
    b.ks = float(np.float32(1) - m)
    return b


def test_microfacet_ttest(scene_dir, tmp_path):
    root = ET.parse(os.path.join(scene_dir, "scenes/pa3/tests/ttest-microfacet.xml")).getroot()
    strings = {s.get("name"): s.get("value") for s in root.findall("string")}
    angles = [float(x) for x in strings["angles"].replace(",", " ").split()]
    refs = [float(x) for x in strings["references"].replace(",", " ").split()]
    rng = no.Pcg32()
    reqs = []
    for bnode in root.findall("bsdf"):
        b = microfacet_from_xml(bnode)
        for angle, ref in zip(angles, refs):
            mean, var = no.ttest_bsdf(b, angle, rng, 100000)
            ok, p = students_t_test(mean, var, ref, 100000, 0.01, len(refs))
            assert ok, (angle, mean, ref, p)
            reqs.append(("t", mean, var, ref, 100000, 0.01, len(refs)))
    theirs = reference_verdicts(reqs, tmp_path)
    if theirs is not None:
        assert all(theirs), theirs


def chi2_test(obs, exp, n, min_exp, alpha, num_tests):
    """hypothesis::chi2_test: pool low-expectation cells, Pearson statistic, Sidak correction."""
    order = np.argsort(exp, kind="stable")
    pooled_o = pooled_e = 0.0
    chsq, dof = 0.0, 0
    for i in order:
        if exp[i] == 0:
            if obs[i] > n * 1e-5:
                return False
        elif exp[i] < min_exp:
            pooled_o += obs[i]
            pooled_e += exp[i]
        elif pooled_e > 0 and pooled_e < min_exp:
            pooled_o += obs[i]
            pooled_e += exp[i]
        else:
            chsq += (obs[i] - exp[i]) ** 2 / exp[i]
            dof += 1
    if pooled_e > 0 or pooled_o > 0:
        chsq += (pooled_o - pooled_e) ** 2 / max(pooled_e, 1e-300)
        dof += 1
    dof -= 1
    pval = 1 - stats.chi2.cdf(chsq, dof)
    sidak = 1.0 - (1.0 - alpha) ** (1.0 / num_tests)
    return not (pval < sidak or not math.isfinite(pval))


def expected_frequencies(b, wi, res_t, res_p, n, quad=48):
    """Integral of pdf(wi, .) over each cos(theta) x phi cell (Gauss-Legendre per cell)."""
    x, w = np.polynomial.legendre.leggauss(quad)
    exp = np.zeros(res_t * res_p)
    for i in range(res_t):
        c0, c1 = -1.0 + i * 2.0 / res_t, -1.0 + (i + 1) * 2.0 / res_t
        ct = 0.5 * (c1 - c0) * x + 0.5 * (c1 + c0)
        for j in range(res_p):
            p0, p1 = j * 2 * math.pi / res_p, (j + 1) * 2 * math.pi / res_p
            ph = 0.5 * (p1 - p0) * x + 0.5 * (p1 + p0)
            CT, PH = np.meshgrid(ct, ph, indexing="ij")
            st = np.sqrt(1 - CT * CT)
            wo = np.stack([st * np.cos(PH), st * np.sin(PH), CT], -1).astype(np.float32)
            pdf = no.bsdf_pdf_batch(b, wi, wo.reshape(-1, 3)).reshape(CT.shape).astype(np.float64)
            exp[i * res_p + j] = (np.outer(w, w) * pdf).sum() * 0.25 * (c1 - c0) * (p1 - p0) * n
    return exp


def test_microfacet_chi2(scene_dir, tmp_path):
    root = ET.parse(os.path.join(scene_dir, "scenes/pa3/tests/chi2test-microfacet.xml")).getroot()
    res_t, res_p, tests_per_bsdf = 10, 20, 5
    n = res_t * res_p * 5000
    bsdfs = [microfacet_from_xml(b) for b in root.findall("bsdf")]
    rng = no.Pcg32()
    passed = 0
    reqs = []
    for b in bsdfs:
        for _ in range(tests_per_bsdf):
            cos_t = rng.next_float()
            sin_t = math.sqrt(max(0.0, 1 - cos_t * cos_t))
            phi = np.float32(2.0 * np.float32(math.pi)) * np.float32(rng.next_float())
            wi = np.array([math.cos(phi) * sin_t, math.sin(phi) * sin_t, cos_t], np.float32)
            obs = no.chi2_histogram(b, wi, rng, n, res_t, res_p)
            exp = expected_frequencies(b, wi, res_t, res_p, n)
            passed += chi2_test(obs, exp, n, 5, 0.01, tests_per_bsdf * len(bsdfs))
            reqs.append(("chi2", obs, exp, n, 5, 0.01, tests_per_bsdf * len(bsdfs)))
    assert passed == tests_per_bsdf * len(bsdfs), passed
    theirs = reference_verdicts(reqs, tmp_path)
    if theirs is not None:
        assert all(theirs), theirs


def test_oracle_arithmetic_matches_reference_eigen(tmp_path):
    """The oracle's restated Eigen arithmetic (dot = x0*y0 + (x1*y1 + x2*y2), normalized, maxCoeff,
    squaredNorm/norm, cross, 3x3 and 4x4 matrix-vector products, Color3f cwise chains, the denoiser's
    Vector4f lpNorm<1> = (|x0|+|x2|) + (|x1|+|x3|) and Color3f / w) is bit-identical
    to the reference's own vendored Eigen 3.3.8 (ext/eigen, compiled unmodified into
    oracle/_ref/eigen_probe by oracle/build_ref.sh) on random inputs, including wide exponent ranges,
    signed zeros and denormals. Only where the reference checkout is present (this container)."""
    import subprocess
    exe = os.path.join(os.path.dirname(no.__file__), "_ref", "eigen_probe")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/eigen_probe not built (needs /root/reference/ext/eigen)")
    rng = np.random.default_rng(2024)
    n = 200000
    cases = rng.normal(size=(n, 36)).astype(np.float32)
    scale = (2.0 ** rng.integers(-20, 21, size=(n, 36))).astype(np.float32)
    cases[n // 2:] *= scale[n // 2:]          # wide exponent ranges
    cases[::97, 0] = 0.0                       # exact zeros / signed zeros
    cases[1::97, 1] = -0.0
    cases[2::89, 2] = np.float32(1e-40)        # denormals
    cases[3::83, 3:6] = cases[3::83, 0:3]      # a == b (zero differences)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    cases.tofile(inp)
    subprocess.run([exe, str(inp), str(out)], check=True, timeout=120)
    ref = np.fromfile(out, np.float32).reshape(n, 28)
    mine = no.eigen_ops(cases)
    names = ["dot"] + ["normalized"] * 3 + ["maxCoeff"] + ["mat3*v"] * 3 + ["mat4*v"] * 4 + ["squaredNorm", "norm"] + \
            ["(a*s)*b"] * 3 + ["a*b*c"] * 3 + ["cross"] * 3 + ["(a-b).norm"] + \
            ["Vector4f.lpNorm<1>"] + ["Color3f/w"] * 3
    for j, name in enumerate(names):
        r, m = ref[:, j].view(np.uint32), mine[:, j].view(np.uint32)
        nan_both = np.isnan(ref[:, j]) & np.isnan(mine[:, j])
        bad = (r != m) & ~nan_both
        assert not bad.any(), f"{name} (column {j}): {bad.sum()} mismatches, e.g. case {np.argmax(bad)}"
