"""Regenerates the committed golden fixtures from the reference checkout (this container only).

    python tests/golden/make_fixtures.py [/root/reference]

Writes (all data, no reference source):
  pcg32_kat.json          the pcg32 known-answer output (ext/pcg32/pcg32-demo.out), parsed,
                          cross-checked against oracle/_ref/pcg32-demo built from the reference's
                          own pcg32-demo.cpp when that binary exists
  reference_scenes.json   scene inputs the reference's own tests and benchmarks use: the Cornell
                          box (scenes/pa4/cbox), the path-integrator known-answer tests
                          (scenes/pa4/tests), the microfacet BSDF tests (scenes/pa3/tests
                          ttest/chi2test XML) and the point-light tests (scenes/pa1/test-direct.xml). Stored as {relative path: file text}; tests write
                          them to a temporary directory and load them through nh_scene_load_xml.
  textured_scenes.json.gz the reference's textured-albedo scenes with their meshes (gzip of the same
                          {relative path: file text} form): scenes/project/denoiser/denoiser-test.xml (the
                          scene of the reference's only published timing, checkerboard_color floor),
                          scenes/pa1/mesh-texture.xml and sphere-texture.xml (checkerboard_color),
                          scenes/project/textures/aircraft.xml (png_texture; its aircraft_base.png and .hdr
                          envmap are absent from the reference checkout)
  project_scenes.json.gz  the reference's depth-of-field scenes (scenes/project/dof/dof-val.xml and
                          table_path_mis.xml, path_mis, thin lens) with their meshes, and its envmap scene
                          scenes/project/envmap/envmap_sphere.xml with the shipped res/wooden_motel.png (binary
                          files stored as {"base64": ...})
  normalmap_scenes.json.gz the reference's normal-mapped scenes (scenes/project/normalmap/: the direct_mis / direct
                          ones, normals-identity-direct.xml, normals-primitives-direct.xml, normals-camel.xml, and
                          the `normals` integrator's normals-identity{,-x,-y,-ref}.xml, normals-primitives.xml) with
                          their meshes and the shipped normal maps res/normal-identity{,-x,-y}.png,
                          normal-primitives.png, normal-test.png (same form)
"""
import base64
import gzip
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

SCENE_FILES = [
    "scenes/pa4/cbox/cbox_path_mis.xml",
    "scenes/pa4/cbox/cbox_path_mats.xml",
    "scenes/pa4/cbox/meshes/walls.obj",
    "scenes/pa4/cbox/meshes/leftwall.obj",
    "scenes/pa4/cbox/meshes/rightwall.obj",
    "scenes/pa4/cbox/meshes/light.obj",
    "scenes/pa4/tests/test-furnace.xml",
    "scenes/pa4/tests/test-direct.xml",
    "scenes/pa4/tests/furnace.obj",
    "scenes/pa4/tests/floor.obj",
    "scenes/pa4/tests/polylum1.obj",
    "scenes/pa4/tests/polylum2.obj",
    "scenes/pa4/tests/polylum3.obj",
    "scenes/pa4/tests/polylum4.obj",
    "scenes/pa4/tests/polylum5.obj",
    "scenes/pa3/tests/ttest-microfacet.xml",
    "scenes/pa3/tests/chi2test-microfacet.xml",
    # direct_ems / direct_mats / direct_mis known-answer scenes (t-tests)
    "scenes/pa3/tests/test-mesh.xml",
    "scenes/pa3/tests/test-mesh-furnace.xml",
    "scenes/pa3/tests/furnace.obj",
    "scenes/pa3/tests/floor.obj",
    "scenes/pa3/tests/polylum1.obj",
    "scenes/pa3/tests/polylum2.obj",
    "scenes/pa3/tests/polylum3.obj",
    "scenes/pa3/tests/polylum4.obj",
    "scenes/pa3/tests/polylum5.obj",
    # point-light known-answer scenes of the `direct` integrator (PointLight, pointlight.cpp:47-78)
    "scenes/pa1/test-direct.xml",
    "scenes/pa1/disk.obj",
]

TEXTURED_FILES = [
    "scenes/project/denoiser/denoiser-test.xml",
    "scenes/project/meshes/table/plane.obj",
    "scenes/project/meshes/table/curvy_bowl.obj",
    "scenes/pa1/mesh-texture.xml",
    "scenes/pa1/sphere-texture.xml",
    "scenes/pa1/camelhead.obj",
    "scenes/pa1/plane.obj",
    "scenes/project/textures/aircraft.xml",
    "scenes/project/meshes/aircraft/aircraft_base.obj",
    "scenes/project/meshes/aircraft/aircraft_glass.obj",
]

PROJECT_FILES = [
    "scenes/project/dof/dof-val.xml",
    "scenes/project/dof/center-cube.obj",
    "scenes/project/dof/center-lights.obj",
    "scenes/project/dof/cube-array.obj",
    "scenes/project/dof/floor.obj",
    "scenes/project/dof/light-array.obj",
    "scenes/project/dof/table_path_mis.xml",
    "scenes/project/meshes/table/plane.obj",
    "scenes/project/meshes/table/curvy_bowl.obj",
    "scenes/project/meshes/table/circle.obj",
    "scenes/project/meshes/table/wine_glass.obj",
    "scenes/project/meshes/table/wine_glass_inner.obj",
    "scenes/project/envmap/envmap_sphere.xml",
    "scenes/project/res/wooden_motel.png",
]


NORMALMAP_FILES = [
    "scenes/project/normalmap/normals-identity-direct.xml",
    "scenes/project/normalmap/normals-primitives-direct.xml",
    "scenes/project/normalmap/normals-camel.xml",
    # the `normals` integrator's views of the same maps (normals.cpp)
    "scenes/project/normalmap/normals-identity.xml",
    "scenes/project/normalmap/normals-identity-x.xml",
    "scenes/project/normalmap/normals-identity-y.xml",
    "scenes/project/normalmap/normals-identity-ref.xml",
    "scenes/project/normalmap/normals-primitives.xml",
    "scenes/project/meshes/sphere.obj",
    "scenes/project/res/normal-identity-x.png",
    "scenes/project/res/normal-identity-y.png",
    "scenes/project/meshes/plane.obj",
    "scenes/project/meshes/cube.obj",
    "scenes/project/meshes/cone.obj",
    "scenes/project/meshes/camelhead.obj",
    "scenes/project/res/normal-identity.png",
    "scenes/project/res/normal-primitives.png",
    "scenes/project/res/normal-test.png",
]


def read_fixture(ref, rel):
    data = open(os.path.join(ref, rel), "rb").read()
    try:
        return data.decode("utf-8")
    except UnicodeDecodeError:
        return {"base64": base64.b64encode(data).decode("ascii")}


def parse_demo(text):
    rounds = []
    cur = None
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        if s.startswith("Round"):
            cur = {"u32": [], "coins": "", "rolls": [], "cards": []}
            rounds.append(cur)
        elif s.startswith("32bit:"):
            cur["u32"] = [int(x, 16) for x in s.split()[1:]]
        elif s.startswith("Coins:"):
            cur["coins"] = s.split()[1]
        elif s.startswith("Rolls:"):
            cur["rolls"] = [int(x) for x in s.split()[1:]]
        elif s.startswith("Cards:"):
            cards = s.split()[1:]
            j = i + 1
            while j < len(lines) and lines[j].startswith("\t"):
                cards += lines[j].split()
                j += 1
            cur["cards"] = cards
            i = j - 1
        i += 1
    return rounds


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    demo_out = open(os.path.join(ref, "ext/pcg32/pcg32-demo.out")).read()
    kat = {"seed": [42, 54], "source": "ext/pcg32/pcg32-demo.out", "rounds": parse_demo(demo_out)}
    exe = os.path.join(REPO, "oracle", "_ref", "pcg32-demo")
    if os.path.exists(exe):
        built = subprocess.run([exe, "5"], capture_output=True, text=True, check=True).stdout
        assert parse_demo(built) == kat["rounds"], "reference pcg32-demo build disagrees with pcg32-demo.out"
        kat["cross_checked_with"] = "oracle/_ref/pcg32-demo (built from ext/pcg32/pcg32-demo.cpp)"
    with open(os.path.join(HERE, "pcg32_kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    scenes = {p: open(os.path.join(ref, p)).read() for p in SCENE_FILES}
    with open(os.path.join(HERE, "reference_scenes.json"), "w") as f:
        json.dump(scenes, f, indent=0)
    textured = {p: open(os.path.join(ref, p)).read() for p in TEXTURED_FILES}
    with open(os.path.join(HERE, "textured_scenes.json.gz"), "wb") as f:
        f.write(gzip.compress(json.dumps(textured, indent=0).encode(), mtime=0))
    project = {p: read_fixture(ref, p) for p in PROJECT_FILES}
    with open(os.path.join(HERE, "project_scenes.json.gz"), "wb") as f:
        f.write(gzip.compress(json.dumps(project, indent=0).encode(), mtime=0))
    normalmap = {p: read_fixture(ref, p) for p in NORMALMAP_FILES}
    with open(os.path.join(HERE, "normalmap_scenes.json.gz"), "wb") as f:
        f.write(gzip.compress(json.dumps(normalmap, indent=0).encode(), mtime=0))
    print("wrote pcg32_kat.json, reference_scenes.json, textured_scenes.json.gz, project_scenes.json.gz, "
          "normalmap_scenes.json.gz")


if __name__ == "__main__":
    main()
