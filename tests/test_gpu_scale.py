"""GPU parity at the benchmark configurations' own sizes (BASELINE.json configs), through the
default bench pipeline: wavefront mode, two path pools, ordered traversal (4-wide persistent
traversal for the deep mesh BVHs), default knobs. Compared with the CPU oracle on the same per-path
seeds; tolerance: per-image relative L2 < 1e-4 (north star). Each test also reports whether the
images are bit-identical.

  C2  Cornell box diffuse, 1024^2, 4 spp: all 1024 blocks, several chunks (small path-state budget)
      with both pools overlapping
  C4  Cornell box mirror + dielectric, 2048^2, 16 spp in one 2^26-path chunk: the full 26-bit
      path-id packing of the wavefront state (nh_wavefront.hip kPidBits)
  C3  the 498k-triangle bumpy mesh (microfacet), 128^2, 4 spp
  C5  the full C5 geometry -- ten flattened toWorld copies of the 996k-triangle mesh (9.96M
      triangles, scenegen.c5_xml) + the PNG envmap (sphericalTexture) + area light -- at 64^2, 2 spp
"""
import os
import time

import numpy as np
import pytest

import nori_hip as nh
import nori_oracle as no
import scenegen

pytestmark = pytest.mark.gpu

TOL_REL_L2 = 1e-4


def rel_l2(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    return float(np.sqrt(np.sum((a - b) ** 2) / max(np.sum(b ** 2), 1e-300)))


def bench_pipeline_vs_oracle(xml, w, h, spp, seed=1234, rounds_per_call=None):
    t0 = time.time()
    s = nh.Scene(xml)
    s.set_resolution(w, h)
    b = nh.Bvh(s, n_threads=16)
    ctx = nh.Context(0)
    ctx.upload(s, b)
    ctx.render(0, 0, seed=seed, clear=True, mode=nh.MODE_WAVEFRONT)
    step = rounds_per_call or spp
    for s0 in range(0, spp, step):  # asynchronous calls, as bench.py issues them
        ctx.render(s0, min(spp, s0 + step), seed=seed, traversal=nh.TRAVERSAL_ORDERED, mode=nh.MODE_WAVEFRONT)
    g = ctx.framebuffer()
    st = ctx.stats()
    t_gpu = time.time() - t0
    t0 = time.time()
    r = no.OracleScene(s).render(0, spp, seed=seed)
    t_cpu = time.time() - t0
    e = rel_l2(g, r)
    same = bool(np.array_equal(g, r))
    print(f"{os.path.basename(xml)} {w}x{h} {spp} spp: rel-L2 {e:.3e}, bit-identical {same}, "
          f"max|d| {np.abs(g.astype(np.float64) - r).max():.3e}, splat launches {st['launches_splat']}, "
          f"node bytes {st['node_bytes']} (gpu side {t_gpu:.1f} s, oracle {t_cpu:.1f} s)")
    assert np.isfinite(g).all()
    assert e < TOL_REL_L2, e
    img = nh.to_rgb(r, s.border)
    assert img.mean() > 0.01
    return g, r, st


def test_c2_full_image_multi_chunk(gpu, tmp_path, monkeypatch):
    """C2 at its bench resolution: every one of the 1024 blocks, 4 spp split into 2-round chunks by a
    small path-state budget, issued as two asynchronous calls so both pools overlap."""
    monkeypatch.setenv("NH_WF_BUDGET_MB", "700")
    xml = scenegen.cbox_xml(str(tmp_path), "c2", width=1024, height=1024)
    _, _, st = bench_pipeline_vs_oracle(xml, 1024, 1024, 4, rounds_per_call=2)
    assert st["launches_splat"] >= 2  # several chunks


def test_c4_full_path_id_range(gpu, tmp_path, monkeypatch):
    """C4 at 2048^2: 16 rounds x 4M pixels = 2^26 paths in one chunk (the largest path id the
    wavefront state packs); mirror + dielectric paths (long specular chains, tail kernel)."""
    monkeypatch.setenv("NH_WF_BUDGET_MB", "24000")
    xml = scenegen.cbox_xml(str(tmp_path), "c1", width=2048, height=2048)
    _, _, st = bench_pipeline_vs_oracle(xml, 2048, 2048, 16)
    assert st["samples"] == 16 * 2048 * 2048


@pytest.mark.parametrize("sort_shade", ["0", "1"])
def test_c3_full_mesh(gpu, tmp_path, monkeypatch, sort_shade):
    """C3's 498k-triangle Beckmann-microfacet mesh (the bench scene itself) at 128^2, 4 spp; with NH_SORT_SHADE=1
    the deep-BVH material-sorted shade (wf_shade<true>: the workgroup's entries shaded in BSDF-type order, the
    north star's material-sorted queues on the split pipeline) against the oracle too."""
    monkeypatch.setenv("NH_SORT_SHADE", sort_shade)
    xml, ntri = scenegen.bumpy_cbox_xml(str(tmp_path), 1000, 250, width=128, height=128)
    assert ntri == 498000
    _, _, st = bench_pipeline_vs_oracle(xml, 128, 128, 4)
    assert st["node_bytes"] == 128  # the persistent 4-wide traversal the bench uses


def test_c5_full_geometry(gpu, tmp_path):
    """C5's geometry at full size: ten toWorld-baked copies of the 996k-triangle mesh (9.96M
    triangles, BVH far larger than the MALL) + PNG envmap + area light, 64^2 x 2 spp."""
    xml, ntri = scenegen.c5_xml(str(tmp_path), n_copies=10, width=64, height=64, spp=2)
    assert ntri > 9_900_000
    _, _, st = bench_pipeline_vs_oracle(xml, 64, 64, 2)
    assert st["node_bytes"] == 128
