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
TEXTURED_FIXTURE = os.path.join(_REPO, "tests", "golden", "textured_scenes.json.gz")
PROJECT_FIXTURE = os.path.join(_REPO, "tests", "golden", "project_scenes.json.gz")
NORMALMAP_FIXTURE = os.path.join(_REPO, "tests", "golden", "normalmap_scenes.json.gz")

C2_ALBEDO = "0.725 0.71 0.68"


def materialize(out_dir: str) -> str:
    """Write the reference scene fixtures (reference_scenes.json, the textured scenes of textured_scenes.json.gz and
    the depth-of-field / envmap scenes of project_scenes.json.gz, the normal-mapped scenes of
    normalmap_scenes.json.gz) under out_dir; returns out_dir."""
    import base64
    import gzip
    with open(FIXTURE) as f:
        files = json.load(f)
    for bundle in (TEXTURED_FIXTURE, PROJECT_FIXTURE, NORMALMAP_FIXTURE):
        if os.path.exists(bundle):
            with gzip.open(bundle, "rt") as f:
                files.update(json.load(f))
    for rel, text in files.items():
        p = os.path.join(out_dir, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        if isinstance(text, dict):  # binary file (a PNG)
            with open(p, "wb") as g:
                g.write(base64.b64decode(text["base64"]))
        else:
            with open(p, "w") as g:
                g.write(text)
    return out_dir


def cbox_xml(out_dir: str, variant: str = "c1", width: int | None = None, height: int | None = None,
             spp: int | None = None, extra_shapes: str = "", drop_spheres: bool = False, denoiser: str = "",
             walls_bsdf: str = "") -> str:
    """Cornell box scene file. variant: c1/c4 = reference (mirror + dielectric spheres),
    c2 = both spheres diffuse (albedo of the walls), as SURVEY.md 8(d) defines. denoiser: a
    <denoiser> element to add (scenes/project/denoiser/denoiser-test.xml:28-32 form). walls_bsdf: a <bsdf>
    element replacing the one of walls.obj (floor, ceiling, back wall), e.g. a textured diffuse."""
    materialize(out_dir)
    src = os.path.join(out_dir, "scenes/pa4/cbox/cbox_path_mis.xml")
    text = open(src).read()
    if variant == "c2":
        text = text.replace('<bsdf type="mirror"/>', f'<bsdf type="diffuse"><color name="albedo" value="{C2_ALBEDO}"/></bsdf>')
        text = text.replace('<bsdf type="dielectric"/>', f'<bsdf type="diffuse"><color name="albedo" value="{C2_ALBEDO}"/></bsdf>')
    if walls_bsdf:
        old = '<bsdf type="diffuse">\n\t\t\t<color name="albedo" value="0.725 0.71 0.68"/>\n\t\t</bsdf>'
        assert text.count(old) == 1
        text = text.replace(old, walls_bsdf)
    if drop_spheres:
        import re
        text = re.sub(r'<shape type="sphere">.*?</shape>', "", text, flags=re.S)
    if extra_shapes:
        text = text.replace("</scene>", extra_shapes + "\n</scene>")
    if denoiser:
        text = text.replace("</scene>", denoiser + "\n</scene>")
    if width:
        text = text.replace('<integer name="width" value="800"/>', f'<integer name="width" value="{width}"/>')
    if height:
        text = text.replace('<integer name="height" value="600"/>', f'<integer name="height" value="{height}"/>')
    if spp:
        text = text.replace('<integer name="sampleCount" value="512"/>', f'<integer name="sampleCount" value="{spp}"/>')
    key = repr((width, height, spp, extra_shapes, drop_spheres, denoiser, walls_bsdf)).encode()
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


# ---------------------------------------------------------------------------------------
# Environment-map scenes (C5's envmap). The reference's probe image
# (scenes/project/res/rooitou_park.png) is not shipped to the GPU box, so the sky is a
# deterministic synthetic PNG: a vertical gradient, a bright "sun" disc and a seeded noise
# texture, written with every PNG scanline filter type so the decoder is exercised.

def _png_filter_row(kind: int, row: np.ndarray, prev: np.ndarray, bpp: int) -> bytes:
    r = row.astype(np.int32)
    p = prev.astype(np.int32)
    left = np.concatenate([np.zeros(bpp, np.int32), r[:-bpp]])
    upleft = np.concatenate([np.zeros(bpp, np.int32), p[:-bpp]])
    if kind == 0:
        out = r
    elif kind == 1:
        out = r - left
    elif kind == 2:
        out = r - p
    elif kind == 3:
        out = r - ((left + p) >> 1)
    else:
        pa = np.abs(p - upleft)
        pb = np.abs(left - upleft)
        pc = np.abs(left + p - 2 * upleft)
        pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, p, upleft))
        out = r - pred
    return bytes([kind]) + (out & 0xFF).astype(np.uint8).tobytes()


def write_png(path: str, img: np.ndarray) -> None:
    """8-bit RGB (H, W, 3) or RGBA (H, W, 4) PNG; scanline filter type = row index mod 5."""
    import struct
    import zlib
    h, w, ch = img.shape
    ctype = {3: 2, 4: 6}[ch]
    raw = bytearray()
    prev = np.zeros(w * ch, np.uint8)
    for y in range(h):
        row = img[y].reshape(-1)
        raw += _png_filter_row(y % 5, row, prev, ch)
        prev = row

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(bytes(raw), 6)))
        f.write(chunk(b"IEND", b""))


def rgbe_encode(rgb: np.ndarray) -> np.ndarray:
    """float RGB (h, w, 3) -> RGBE bytes (h, w, 4): shared exponent of the largest channel, mantissas m such that
    (m / 256) * 2^(e - 128) approximates each channel (any RGBE bytes are valid input for the decoder tests)."""
    rgb = np.asarray(rgb, np.float64)
    mx = rgb.max(axis=-1)
    out = np.zeros(rgb.shape[:-1] + (4,), np.uint8)
    nz = mx > 1e-32
    e = np.floor(np.log2(mx[nz])) + 1
    out[nz, 3] = np.clip(e + 128, 0, 255)
    scale = 256.0 / np.exp2(out[nz, 3].astype(np.float64) - 128)
    out[nz, :3] = np.clip(np.floor(rgb[nz] * scale[:, None]), 0, 255)
    return out


def write_hdr(path: str, rgbe: np.ndarray, mode: str = "rle", header: str = "FORMAT=32-bit_rle_rgbe") -> None:
    """Radiance .hdr of RGBE bytes (h, w, 4) in one of the encodings HDRLoader reads (include/nori/HDRLoader.h):
    rle   new-style scanlines (2, 2, w >> 8, w & 255, then each component as runs / literal chunks);
    flat  plain RGBE pixels;
    old   plain pixels with the old (1, 1, 1, n) repeat codes for runs of identical pixels (n << 8 chained for long
          runs)."""
    h, w, _ = rgbe.shape
    out = bytearray(b"#?RADIANCE\n" + header.encode() + b"\n\n" + f"-Y {h} +X {w}\n".encode())
    if mode == "rle" and not 8 <= w <= 0x7FFF:
        raise ValueError("run-length scanlines need 8 <= width <= 0x7fff (HDRLoader.h:89-90)")
    for y in range(h):
        line = rgbe[y]
        if mode == "rle":
            out += bytes([2, 2, w >> 8, w & 255])
            for c in range(4):
                comp = line[:, c]
                j = 0
                while j < w:
                    r = 1
                    while j + r < w and r < 127 and comp[j + r] == comp[j]:
                        r += 1
                    if r >= 3:
                        out += bytes([128 + r, int(comp[j])])
                        j += r
                    else:
                        k = j
                        while k < w and k - j < 128 and not (k + 2 < w and comp[k] == comp[k + 1] == comp[k + 2]):
                            k += 1
                        k = max(k, j + 1)
                        out += bytes([k - j]) + bytes(int(v) for v in comp[j:k])
                        j = k
        elif mode == "flat":
            out += line.astype(np.uint8).tobytes()
        elif mode == "old":
            x = 0
            while x < w:
                out += line[x].astype(np.uint8).tobytes()
                r = 0
                while x + 1 + r < w and (line[x + 1 + r] == line[x]).all():
                    r += 1
                x += 1
                # runs of identical pixels: (1, 1, 1, n) repeats the previous pixel n times; a second code in a row
                # counts n << 8 (HDRLoader.h oldDecrunch)
                if r >= 2 and not (line[x - 1][:3] == 1).all():
                    hi, lo = r >> 8, r & 255
                    out += bytes([1, 1, 1, lo])  # (a zero count still shifts the next code by 8)
                    if hi:
                        out += bytes([1, 1, 1, hi])
                    x += r
        else:
            raise ValueError(mode)
    with open(path, "wb") as f:
        f.write(bytes(out))


def rgbe_decode_reference(rgbe: np.ndarray) -> np.ndarray:
    """HDRLoader's floats (HDRLoader.h:27-44) of RGBE bytes: (m / 256.0f) * (float)pow(2, e - 128), alpha 0 -- float32
    arithmetic as the reference's."""
    m = rgbe[..., :3].astype(np.float32) / np.float32(256.0)
    d = np.exp2(rgbe[..., 3:4].astype(np.float64) - 128.0).astype(np.float32)
    out = np.zeros(rgbe.shape[:-1] + (4,), np.float32)
    out[..., :3] = m * d
    return out


def sky_image(width: int, height: int, seed: int = 7) -> np.ndarray:
    """Synthetic lat-long sky (rows = polar angle), uint8 RGB."""
    rng = np.random.default_rng(seed)
    v = (np.arange(height) + 0.5) / height
    u = (np.arange(width) + 0.5) / width
    V, U = np.meshgrid(v, u, indexing="ij")
    sky = np.stack([0.35 + 0.4 * V, 0.5 + 0.3 * V, 0.9 - 0.2 * V], -1)
    ground = np.stack([0.25 + 0 * V, 0.2 + 0 * V, 0.15 + 0 * V], -1)
    img = np.where((V > 0.5)[..., None], ground, sky)
    d2 = ((U - 0.3) * 2) ** 2 + (V - 0.25) ** 2
    img = img + 4.0 * np.exp(-d2 / (2 * 0.02 ** 2))[..., None] * np.array([1.0, 0.9, 0.7])
    img = img * (0.9 + 0.2 * rng.random((height, width, 1)))
    return np.clip(img * 200, 0, 255).astype(np.uint8)


def envmap_xml(out_dir: str, width: int = 64, height: int = 48, spp: int = 16, texture: str = "png",
               tex_size=(96, 48), spherical: bool = True, area_light: bool = True, integrator: str = "path_mis",
               mesh: str | None = None, euler=None, black: bool = False) -> str:
    """Open scene lit by an envmap (+ optionally a small area light): a ground quad, a diffuse
    and a microfacet sphere, a mirror sphere. texture: png | hdr | constant | none (EnvMap's 0.5
    fallback); hdr is a Radiance RGBE sky (.hdr, run-length scanlines). mesh: optional OBJ path added with a diffuse BSDF. euler: the png_texture's eulerAngles
    (degrees) of the spherical lookup. black: an all-black PNG (its luminance table sums to 0)."""
    os.makedirs(out_dir, exist_ok=True)
    tex_xml = ""
    if texture == "png":
        png = os.path.join(out_dir, f"{'black' if black else 'sky'}_{tex_size[0]}x{tex_size[1]}.png")
        if not os.path.exists(png):
            img = sky_image(*tex_size)
            write_png(png, np.zeros_like(img) if black else img)
        tex_xml = f"""<texture type="png_texture" name="albedo">
      <string name="filename" value="{os.path.basename(png)}"/>
      <boolean name="sphericalTexture" value="{'true' if spherical else 'false'}"/>
      {f'<vector name="eulerAngles" value="{euler[0]},{euler[1]},{euler[2]}"/>' if euler else ''}
    </texture>"""
    elif texture == "hdr":  # a Radiance RGBE sky (PNGTexture's .hdr branch)
        hdr = os.path.join(out_dir, f"sky_{tex_size[0]}x{tex_size[1]}.hdr")
        if not os.path.exists(hdr):
            sky = sky_image(*tex_size).astype(np.float64) / 255.0 * 3.0
            write_hdr(hdr, rgbe_encode(sky), mode="rle" if 8 <= tex_size[0] <= 0x7FFF else "flat")
        tex_xml = f"""<texture type="png_texture" name="albedo">
      <string name="filename" value="{os.path.basename(hdr)}"/>
      <boolean name="sphericalTexture" value="{'true' if spherical else 'false'}"/>
    </texture>"""
    elif texture == "constant":
        tex_xml = '<texture type="constant_color" name="albedo"><color name="value" value="0.8 0.7 0.6"/></texture>'
    quad = os.path.join(out_dir, "ground.obj")
    with open(quad, "w") as f:
        f.write("v -4 0 -4\nv 4 0 -4\nv 4 0 4\nv -4 0 4\nvt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\nf 1/1 4/4 3/3 2/2\n")
    light = ""
    if area_light:
        lq = os.path.join(out_dir, "lightquad.obj")
        with open(lq, "w") as f:
            f.write("v -0.3 2.5 -0.3\nv 0.3 2.5 -0.3\nv 0.3 2.5 0.3\nv -0.3 2.5 0.3\nf 1 2 3 4\n")
        light = f"""<shape type="obj"><string name="filename" value="lightquad.obj"/>
    <emitter type="area"><color name="radiance" value="6 6 6"/></emitter></shape>"""
    extra = ""
    if mesh:
        extra = f"""<shape type="obj"><string name="filename" value="{os.path.relpath(mesh, out_dir)}"/>
    <bsdf type="diffuse"><color name="albedo" value="0.6 0.6 0.6"/></bsdf></shape>"""
    text = f"""<?xml version="1.0" encoding="utf-8"?>
<scene>
  <integrator type="{integrator}"/>
  <sampler type="independent"><integer name="sampleCount" value="{spp}"/></sampler>
  <camera type="perspective">
    <transform name="toWorld"><lookat target="0, 0.4, 0" origin="0, 1.2, 3.2" up="0, 1, 0"/></transform>
    <float name="fov" value="40"/>
    <integer name="width" value="{width}"/><integer name="height" value="{height}"/>
  </camera>
  <emitter type="envmap">
    <color name="radiance" value="1.5 1.5 1.5"/>
    {tex_xml}
  </emitter>
  {light}
  <shape type="obj"><string name="filename" value="ground.obj"/>
    <bsdf type="diffuse"><color name="albedo" value="0.5 0.5 0.45"/></bsdf></shape>
  <shape type="sphere"><point name="center" value="-0.7 0.4 0"/><float name="radius" value="0.4"/>
    <bsdf type="diffuse"><color name="albedo" value="0.7 0.3 0.2"/></bsdf></shape>
  <shape type="sphere"><point name="center" value="0.1 0.35 0.3"/><float name="radius" value="0.35"/>
    <bsdf type="microfacet"><float name="alpha" value="0.15"/><color name="kd" value="0.2 0.3 0.5"/></bsdf></shape>
  <shape type="sphere"><point name="center" value="0.8 0.3 -0.3"/><float name="radius" value="0.3"/>
    <bsdf type="mirror"/></shape>
  {extra}
</scene>
"""
    key = repr((width, height, spp, texture, tex_size, spherical, area_light, integrator, mesh, euler, black)).encode()
    dst = os.path.join(out_dir, f"envmap_{hashlib.sha1(key).hexdigest()[:10]}.xml")
    with open(dst, "w") as f:
        f.write(text)
    return dst


def c5_xml(out_dir: str, n_copies: int = 10, n_phi: int = 2000, n_theta: int = 250, width: int = 4096,
           height: int = 4096, spp: int = 16, sky=(1500, 750)) -> tuple[str, int]:
    """C5: n_copies bumpy meshes with distinct affine transforms, flattened
    (Nori bakes toWorld, obj.cpp:107-121; no instancing), lit by an envmap png_texture with
    sphericalTexture=true (a synthetic sky of the size of scenes/project/res/rooitou_park.png,
    which does not travel to the GPU box) and a small area light. Returns (xml, triangle count)."""
    os.makedirs(out_dir, exist_ok=True)
    mesh = os.path.join(out_dir, f"bumpy_{n_phi}x{n_theta}_c0.obj")
    ntri = bumpy_sphere_obj(mesh, n_phi, n_theta, center=(0.0, 0.0, 0.0), radius=1.0)
    rng = np.random.default_rng(5)
    shapes = []
    for i in range(n_copies):
        ang = i * 360.0 / n_copies
        x, z = 2.2 * np.cos(np.radians(ang)), 2.2 * np.sin(np.radians(ang))
        sc = 0.45 + 0.2 * rng.random()
        rot = 360.0 * rng.random()
        kd = rng.random(3) * 0.5 + 0.2
        bsdf = (f'<bsdf type="microfacet"><float name="alpha" value="{0.1 + 0.3 * rng.random():.3f}"/>'
                f'<color name="kd" value="{kd[0]:.3f} {kd[1]:.3f} {kd[2]:.3f}"/></bsdf>' if i % 2 == 0 else
                f'<bsdf type="diffuse"><color name="albedo" value="{kd[0]:.3f} {kd[1]:.3f} {kd[2]:.3f}"/></bsdf>')
        shapes.append(f"""  <shape type="obj"><string name="filename" value="{os.path.basename(mesh)}"/>
    <transform name="toWorld"><scale value="{sc:.3f},{sc * 1.1:.3f},{sc:.3f}"/><rotate axis="0,1,0" angle="{rot:.2f}"/>
      <translate value="{x:.3f},{sc * 1.1:.3f},{z:.3f}"/></transform>
    {bsdf}</shape>""")
    png = os.path.join(out_dir, f"sky_{sky[0]}x{sky[1]}.png")
    if not os.path.exists(png):
        write_png(png, sky_image(*sky))
    quad = os.path.join(out_dir, "c5_ground.obj")
    with open(quad, "w") as f:
        f.write("v -8 0 -8\nv 8 0 -8\nv 8 0 8\nv -8 0 8\nf 1 4 3 2\n")
    lq = os.path.join(out_dir, "c5_light.obj")
    with open(lq, "w") as f:
        f.write("v -0.5 4 -0.5\nv 0.5 4 -0.5\nv 0.5 4 0.5\nv -0.5 4 0.5\nf 1 2 3 4\n")
    text = f"""<?xml version="1.0" encoding="utf-8"?>
<scene>
  <integrator type="path_mis"/>
  <sampler type="independent"><integer name="sampleCount" value="{spp}"/></sampler>
  <camera type="perspective">
    <transform name="toWorld"><lookat target="0, 0.5, 0" origin="0, 3.5, 7.5" up="0, 1, 0"/></transform>
    <float name="fov" value="45"/>
    <integer name="width" value="{width}"/><integer name="height" value="{height}"/>
  </camera>
  <emitter type="envmap">
    <texture type="png_texture" name="albedo">
      <string name="filename" value="{os.path.basename(png)}"/>
      <boolean name="sphericalTexture" value="true"/>
    </texture>
  </emitter>
  <shape type="obj"><string name="filename" value="c5_light.obj"/>
    <emitter type="area"><color name="radiance" value="8 8 8"/></emitter></shape>
  <shape type="obj"><string name="filename" value="c5_ground.obj"/>
    <bsdf type="diffuse"><color name="albedo" value="0.4 0.4 0.4"/></bsdf></shape>
{chr(10).join(shapes)}
</scene>
"""
    dst = os.path.join(out_dir, f"c5_{n_copies}x{n_phi}x{n_theta}_{width}x{height}_{spp}.xml")
    with open(dst, "w") as f:
        f.write(text)
    return dst, ntri * n_copies + 4
