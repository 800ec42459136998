"""Scene inputs for tests and benchmarks (SURVEY.md 8(d) configurations).

The reference's own scene files (Cornell box, path-integrator KAT scenes) ship as the data
fixture tests/golden/reference_scenes.json; `materialize()` writes them to a directory so
they load through nh_scene_load_xml exactly like the reference loads them. Large-mesh
configurations use a deterministic synthetic "bumpy sphere" because the reference's
large meshes (scenes/pa1/ajax.obj) are missing blobs:
  r = 0.3 * (1 + 0.05 sin(12 theta) cos(9 phi) + 0.01 N(0,1)),  numpy seed 1234.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(_REPO, "tests", "golden", "reference_scenes.json")

C2_ALBEDO = "0.725 0.71 0.68"


def materialize(out_dir: str) -> str:
    """Write the reference scene fixtures under out_dir; returns out_dir."""
    with open(FIXTURE) as f:
        files = json.load(f)
    for rel, text in files.items():
        p = os.path.join(out_dir, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as g:
            g.write(text)
    return out_dir


def cbox_xml(out_dir: str, variant: str = "c1", width: int | None = None, height: int | None = None,
             spp: int | None = None, extra_shapes: str = "", drop_spheres: bool = False) -> str:
    """Cornell box scene file. variant: c1/c4 = reference (mirror + dielectric spheres),
    c2 = both spheres diffuse (albedo of the walls), as SURVEY.md 8(d) defines."""
    materialize(out_dir)
    src = os.path.join(out_dir, "scenes/pa4/cbox/cbox_path_mis.xml")
    text = open(src).read()
    if variant == "c2":
        text = text.replace('<bsdf type="mirror"/>', f'<bsdf type="diffuse"><color name="albedo" value="{C2_ALBEDO}"/></bsdf>')
        text = text.replace('<bsdf type="dielectric"/>', f'<bsdf type="diffuse"><color name="albedo" value="{C2_ALBEDO}"/></bsdf>')
    if drop_spheres:
        import re
        text = re.sub(r'<shape type="sphere">.*?</shape>', "", text, flags=re.S)
    if extra_shapes:
        text = text.replace("</scene>", extra_shapes + "\n</scene>")
    if width:
        text = text.replace('<integer name="width" value="800"/>', f'<integer name="width" value="{width}"/>')
    if height:
        text = text.replace('<integer name="height" value="600"/>', f'<integer name="height" value="{height}"/>')
    if spp:
        text = text.replace('<integer name="sampleCount" value="512"/>', f'<integer name="sampleCount" value="{spp}"/>')
    key = repr((width, height, spp, extra_shapes, drop_spheres)).encode()
    name = f"cbox_{variant}_{hashlib.sha1(key).hexdigest()[:10]}.xml"
    dst = os.path.join(out_dir, "scenes/pa4/cbox", name)
    with open(dst, "w") as f:
        f.write(text)
    return dst


def bumpy_sphere_obj(path: str, n_phi: int, n_theta: int, center=(0.0, 0.35, 0.0), radius=0.3, seed=1234) -> int:
    """UV sphere with n_phi x n_theta quads (2 triangles each, poles as triangle fans
    emitted as degenerate-free quads) written as OBJ; returns the triangle count."""
    rng = np.random.default_rng(seed)
    th = np.linspace(0.0, np.pi, n_theta + 1)[1:-1]          # interior rings
    ph = np.linspace(0.0, 2 * np.pi, n_phi, endpoint=False)
    T, P = np.meshgrid(th, ph, indexing="ij")
    r = radius * (1 + 0.05 * np.sin(12 * T) * np.cos(9 * P) + 0.01 * rng.standard_normal(T.shape))
    x = center[0] + r * np.sin(T) * np.cos(P)
    y = center[1] + r * np.cos(T)
    z = center[2] + r * np.sin(T) * np.sin(P)
    verts = np.stack([x, y, z], -1).reshape(-1, 3)
    top = np.array([[center[0], center[1] + radius, center[2]]])
    bot = np.array([[center[0], center[1] - radius, center[2]]])
    V = np.concatenate([verts, top, bot]).astype(np.float32)
    nr = n_theta - 1
    idx = np.arange(nr * n_phi).reshape(nr, n_phi)
    faces = []
    a = idx[:-1, :]
    b = np.roll(idx[:-1, :], -1, axis=1)
    c = idx[1:, :]
    d = np.roll(idx[1:, :], -1, axis=1)
    faces.append(np.stack([a, c, d], -1).reshape(-1, 3))
    faces.append(np.stack([a, d, b], -1).reshape(-1, 3))
    it, ib = len(verts), len(verts) + 1
    r0 = idx[0]
    faces.append(np.stack([np.full(n_phi, it), r0, np.roll(r0, -1)], -1))
    rl = idx[-1]
    faces.append(np.stack([np.full(n_phi, ib), np.roll(rl, -1), rl], -1))
    F = np.concatenate(faces).astype(np.int64) + 1
    with open(path, "w") as f:
        f.write("\n".join("v %.7g %.7g %.7g" % tuple(v) for v in V))
        f.write("\n")
        f.write("\n".join("f %d %d %d" % tuple(t) for t in F))
        f.write("\n")
    return len(F)


def bumpy_cbox_xml(out_dir: str, n_phi: int, n_theta: int, bsdf: str | None = None, width=None, height=None,
                   spp=None) -> tuple[str, int]:
    """Cornell box walls + light with the synthetic bumpy sphere in place of the two spheres
    (C3 / perf-1M). Default BSDF: Nori's Beckmann microfacet, alpha 0.2, kd (0.3,0.3,0.5)."""
    materialize(out_dir)
    mesh = os.path.join(out_dir, "scenes/pa4/cbox/meshes", f"bumpy_{n_phi}x{n_theta}.obj")
    ntri = bumpy_sphere_obj(mesh, n_phi, n_theta)
    bsdf = bsdf or ('<bsdf type="microfacet"><float name="alpha" value="0.2"/>'
                    '<color name="kd" value="0.3 0.3 0.5"/></bsdf>')
    shape = f'<shape type="obj"><string name="filename" value="meshes/{os.path.basename(mesh)}"/>{bsdf}</shape>'
    return cbox_xml(out_dir, "c1", width, height, spp, extra_shapes=shape, drop_spheres=True), ntri


def furnace_xml(out_dir: str) -> str:
    materialize(out_dir)
    return os.path.join(out_dir, "scenes/pa4/tests/test-furnace.xml")


def direct_xml(out_dir: str) -> str:
    materialize(out_dir)
    return os.path.join(out_dir, "scenes/pa4/tests/test-direct.xml")


def test_references(xml_path: str) -> list[float]:
    import xml.etree.ElementTree as ET
    root = ET.parse(xml_path).getroot()
    for s in root.findall("string"):
        if s.get("name") == "references":
            return [float(x) for x in s.get("value").replace(",", " ").split()]
    return []
