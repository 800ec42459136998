// Host-side Nori scene ingestion: XML subset -> flattened nh_scene_desc.
//
// Follows the reference's object model (include/nori/object.h:38-291) and parser
// (src/utils/parser.cpp:28-378): children are parsed first, the object is then
// created from its PropertyList and receives its children in document order;
// transform operations pre-multiply (parser.cpp:312-366). Shape/emitter wiring
// mirrors Scene::addChild (src/utils/scene.cpp:203-266) and Shape::addChild
// (src/shapes/shape.cpp:118-153); the OBJ loader mirrors WavefrontOBJ::loadFromFile
// (src/shapes/obj.cpp:77-238: vertex dedup on the (p, uv, n) triple, quad split
// into (0,1,2),(3,0,2), toWorld baked in). Derived quantities follow
// PerspectiveCamera::update (src/cameras/perspective.cpp:48-96), ImageBlock::init's
// filter table (src/utils/block.cpp:54-70), Mesh::update's area DiscretePDF
// (src/shapes/mesh.cpp:35-48) and Scene::update's emitter DiscretePDF
// (src/utils/scene.cpp:178-184).
//
// Floating-point conventions: per-element arithmetic is fp32 with no contraction;
// 3-element dot products / squared norms are evaluated x0*y0 + (x1*y1 + x2*y2),
// which is what the reference's vendored Eigen 3.3.8 emits for Vector3f (measured,
// DESIGN.md). Transform composition, Matrix4f::inverse (Eigen's SSE path) and the camera matrices
// are restated bit for bit in nori_transform.h (pinned against the reference's Eigen by
// tests/test_transforms.py).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "nori_hip.h"
#include "nh_host.h"
#include "nori_transform.h"
#include "xml_lite.h"

namespace nh {

thread_local std::string g_host_error;

void set_host_error(const std::string &msg) { g_host_error = msg; }

struct SceneError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------------------
// small fp32 math helpers in the reference's evaluation order
// ---------------------------------------------------------------------------
namespace {

struct V3 {
    float x = 0, y = 0, z = 0;
};
inline V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline float dot3(V3 a, V3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
inline V3 cross3(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline V3 normalized(V3 a) {
    float n = dot3(a, a);
    if (n > 0.0f) {
        float s = std::sqrt(n);
        return v3(a.x / s, a.y / s, a.z / s);
    }
    return a;
}

using M4 = xf::Mat4;

inline xf::Vec3 to_xf(V3 a) { return {a.x, a.y, a.z}; }
inline V3 from_xf(xf::Vec3 a) { return v3(a.x, a.y, a.z); }

// nori::Transform applied to points / vectors / normals (include/nori/transform.h:73-86)
V3 xform_point(const M4 &t, V3 p) { return from_xf(xf::apply_point(t, to_xf(p))); }
V3 xform_vector(const M4 &t, V3 v) { return from_xf(xf::apply_vector(t, to_xf(v))); }
V3 xform_normal(const M4 &inv, V3 n) { return from_xf(xf::apply_normal(inv, to_xf(n))); }

float to_float(const std::string &str) {
    const char *c = str.c_str();
    char *end = nullptr;
    float r = std::strtof(c, &end);
    while (end && *end && std::isspace((unsigned char)*end)) ++end;
    if (end == c || *end != '\0') throw SceneError("could not parse floating point value \"" + str + "\"");
    return r;
}
int to_int(const std::string &str) {
    const char *c = str.c_str();
    char *end = nullptr;
    long r = std::strtol(c, &end, 10);
    if (end == c || *end != '\0') throw SceneError("could not parse integer value \"" + str + "\"");
    return (int)r;
}
bool to_bool(const std::string &str) {
    std::string v = str;
    std::transform(v.begin(), v.end(), v.begin(), ::tolower);
    if (v == "true") return true;
    if (v == "false") return false;
    throw SceneError("could not parse boolean value \"" + str + "\"");
}
// common.cpp tokenize(): delimiters ", ", empty tokens dropped
std::vector<std::string> tokenize(const std::string &s, const std::string &delim = ", ", bool include_empty = false) {
    std::vector<std::string> out;
    std::string::size_type last = 0, pos = s.find_first_of(delim, last);
    while (last != std::string::npos) {
        if (pos != last || include_empty) out.push_back(s.substr(last, pos - last));
        last = pos;
        if (last != std::string::npos) {
            last += 1;
            pos = s.find_first_of(delim, last);
        }
    }
    return out;
}
V3 to_v3(const std::string &s) {
    auto t = tokenize(s);
    if (t.size() != 3) throw SceneError("expected 3 values in \"" + s + "\"");
    return v3(to_float(t[0]), to_float(t[1]), to_float(t[2]));
}

// ---------------------------------------------------------------------------
// PropertyList (src/utils/proplist.cpp)
// ---------------------------------------------------------------------------
struct Prop {
    enum Kind { Bool, Int, Float, String, Point, Vector, Color, Transform, Point2, Vector2 } kind;
    bool b = false;
    int i = 0;
    float f = 0;
    std::string s;
    V3 v;
    float v2[2] = {0, 0};  // Point2 / Vector2 (parser.cpp:268-294: <point> / <vector> of 2 components)
    M4 t;
};

struct PropList {
    std::map<std::string, Prop> props;
    void set(const std::string &name, const Prop &p) {
        if (props.count(name)) throw SceneError("property \"" + name + "\" was specified multiple times");
        props[name] = p;
    }
    bool has(const std::string &n) const { return props.count(n) != 0; }
    const Prop *get(const std::string &n, Prop::Kind k) const {
        auto it = props.find(n);
        if (it == props.end()) return nullptr;
        if (it->second.kind != k) throw SceneError("property \"" + n + "\" has the wrong type");
        return &it->second;
    }
    float get_float(const std::string &n, float def) const { auto p = get(n, Prop::Float); return p ? p->f : def; }
    float get_float(const std::string &n) const {
        auto p = get(n, Prop::Float);
        if (!p) throw SceneError("property \"" + n + "\" is missing");
        return p->f;
    }
    int get_int(const std::string &n, int def) const { auto p = get(n, Prop::Int); return p ? p->i : def; }
    std::string get_string(const std::string &n, const std::string &def) const { auto p = get(n, Prop::String); return p ? p->s : def; }
    std::string get_string(const std::string &n) const {
        auto p = get(n, Prop::String);
        if (!p) throw SceneError("property \"" + n + "\" is missing");
        return p->s;
    }
    V3 get_point(const std::string &n, V3 def) const { auto p = get(n, Prop::Point); return p ? p->v : def; }
    V3 get_color(const std::string &n, V3 def) const { auto p = get(n, Prop::Color); return p ? p->v : def; }
    V3 get_color(const std::string &n) const {
        auto p = get(n, Prop::Color);
        if (!p) throw SceneError("property \"" + n + "\" is missing");
        return p->v;
    }
    M4 get_transform(const std::string &n, const M4 &def) const { auto p = get(n, Prop::Transform); return p ? p->t : def; }
    bool get_bool(const std::string &n, bool def) const { auto p = get(n, Prop::Bool); return p ? p->b : def; }
    V3 get_vector(const std::string &n, V3 def) const { auto p = get(n, Prop::Vector); return p ? p->v : def; }
    void get_point2(const std::string &n, float def0, float def1, float out[2]) const {
        auto p = get(n, Prop::Point2);
        out[0] = p ? p->v2[0] : def0;
        out[1] = p ? p->v2[1] : def1;
    }
    void get_vector2(const std::string &n, float def0, float def1, float out[2]) const {
        auto p = get(n, Prop::Vector2);
        out[0] = p ? p->v2[0] : def0;
        out[1] = p ? p->v2[1] : def1;
    }
};

// ---------------------------------------------------------------------------
// object tree produced by the parser
// ---------------------------------------------------------------------------
struct Obj {
    std::string tag;   // scene, shape, bsdf, emitter, camera, integrator, sampler, rfilter, ...
    std::string type;  // plugin name
    PropList props;
    std::vector<std::unique_ptr<Obj>> children;
    size_t offset = 0;
};

}  // namespace

// Owning scene (the C handle).
struct ObjKey {
    uint32_t p, uv, n;
    bool operator==(const ObjKey &o) const { return p == o.p && uv == o.uv && n == o.n; }
};
struct ObjText {
    std::vector<V3> positions, normals;
    std::vector<std::pair<float, float>> texcoords;
    std::vector<uint32_t> indices;
    std::vector<ObjKey> vertices;
};

struct SceneData {
    // OBJ files parsed while loading (released once the scene is assembled)
    std::map<std::string, std::shared_ptr<ObjText>> obj_cache;
    nh_camera camera{};
    nh_filter filter{};
    int32_t integrator = NH_INTEGRATOR_PATH_MIS;
    float normals_dir[3] = {0.f, 0.f, 1.f};  // NormalIntegrator's `direction`
    int32_t sample_count = 1;
    std::vector<nh_shape> shapes;
    std::vector<nh_bsdf> bsdfs;
    std::vector<nh_emitter> emitters;
    std::vector<float> emitter_cdf;
    int32_t envmap = -1;
    std::vector<float> V, N, UV, T, BT;
    std::vector<uint32_t> F;
    std::vector<float> area_cdf;
    nh_envmap env{};
    std::vector<float> env_rgba, env_cdf;
    std::vector<nh_texture> textures;  // BSDF albedo textures (nh_bsdf.albedo_texture = index + 1)
    std::vector<float> texels;         // RGBA texels of the png textures
    nh_denoiser denoiser{};  // type NH_DENOISER_NONE unless the scene has a <denoiser>
    // camera parameters kept for re-projection on resize
    float fov = 30.f, near_clip = 1e-4f, far_clip = 1e4f, focal = 10.f, fstop = 0.f, lens = 0.f;
    // Independent::next2D's argument order as g++ compiles it (nh_camera.lens_draw_order)
    int32_t lens_draw_order = NH_LENS_DRAWS_RTL;
    M4 to_world = M4::identity();
};

namespace {

const char *kObjectTags[] = {"scene", "shape", "texture", "volume", "bsdf", "phase", "emitter", "medium", "camera",
                             "integrator", "sampler", "pxsampler", "denoiser", "test", "rfilter", "renderer"};
const char *kPropTags[] = {"boolean", "integer", "float", "string", "point", "vector", "color", "transform"};
const char *kXformTags[] = {"translate", "matrix", "rotate", "scale", "lookat"};

bool in_list(const std::string &s, const char *const *list, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (s == list[i]) return true;
    return false;
}

struct ParseCtx {
    const std::string &text;
    const std::string &filename;
    std::string pos(size_t off) const { return xml_position(text, off); }
};

void check_attrs(const XmlNode &n, std::initializer_list<const char *> allowed, const ParseCtx &c) {
    std::vector<std::string> need(allowed.begin(), allowed.end());
    for (auto &kv : n.attrs) {
        auto it = std::find(need.begin(), need.end(), kv.first);
        if (it == need.end())
            throw SceneError("unexpected attribute \"" + kv.first + "\" in \"" + n.name + "\" at " + c.pos(n.offset));
        need.erase(it);
    }
    if (!need.empty()) throw SceneError("missing attribute \"" + need[0] + "\" in \"" + n.name + "\" at " + c.pos(n.offset));
}

// One transform operation pre-multiplied onto the Affine3f being composed (parser.cpp:308-360).
void apply_xform_op(M4 &t, const XmlNode &n, const ParseCtx &c) {
    if (n.name == "translate") {
        check_attrs(n, {"value"}, c);
        xf::pre_translate(t, to_xf(to_v3(*n.attr("value"))));
    } else if (n.name == "scale") {
        check_attrs(n, {"value"}, c);
        xf::pre_scale(t, to_xf(to_v3(*n.attr("value"))));
    } else if (n.name == "matrix") {
        check_attrs(n, {"value"}, c);
        auto tk = tokenize(*n.attr("value"));
        if (tk.size() != 16) throw SceneError("expected 16 values");
        M4 m;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) m.m[i][j] = to_float(tk[i * 4 + j]);
        xf::pre_affine(t, m);
    } else if (n.name == "rotate") {
        check_attrs(n, {"angle", "axis"}, c);
        const float angle = xf::deg_to_rad(to_float(*n.attr("angle")));
        xf::pre_rotate(t, angle, to_xf(to_v3(*n.attr("axis"))));
    } else if (n.name == "lookat") {
        check_attrs(n, {"origin", "target", "up"}, c);
        xf::pre_affine(t, xf::lookat_matrix(to_xf(to_v3(*n.attr("origin"))), to_xf(to_v3(*n.attr("target"))),
                                            to_xf(to_v3(*n.attr("up")))));
    } else {
        throw SceneError("unhandled transform element \"" + n.name + "\"");
    }
}

std::unique_ptr<Obj> parse_node(const XmlNode &n, PropList *parent_props, const std::string &parent_tag,
                                const ParseCtx &c) {
    const bool is_obj = in_list(n.name, kObjectTags, sizeof(kObjectTags) / sizeof(*kObjectTags));
    const bool is_prop = in_list(n.name, kPropTags, sizeof(kPropTags) / sizeof(*kPropTags));
    const bool is_xop = in_list(n.name, kXformTags, sizeof(kXformTags) / sizeof(*kXformTags));
    if (!is_obj && !is_prop && !is_xop)
        throw SceneError("unexpected tag \"" + n.name + "\" at " + c.pos(n.offset));
    const bool has_parent = !parent_tag.empty();
    if (!has_parent && !is_obj)
        throw SceneError("root element \"" + n.name + "\" must be a Nori object (at " + c.pos(n.offset) + ")");
    if ((parent_tag == "transform") != is_xop)
        throw SceneError("transform nodes can only contain transform operations (at " + c.pos(n.offset) + ")");
    if (is_obj) {
        auto o = std::make_unique<Obj>();
        o->tag = n.name;
        o->offset = n.offset;
        const std::string *t = n.attr("type");
        o->type = (n.name == "scene") ? "scene" : (t ? *t : "");
        for (auto &ch : n.children) {
            auto child = parse_node(*ch, &o->props, n.name, c);
            if (child) o->children.push_back(std::move(child));
        }
        const std::string *nm = n.attr("name");
        Prop p; p.kind = Prop::String; p.s = nm ? *nm : "";
        if (!o->props.has("name")) o->props.props["name"] = p;
        return o;
    }
    if (!parent_props) throw SceneError("property outside of an object at " + c.pos(n.offset));
    if (n.name == "transform") {
        check_attrs(n, {"name"}, c);
        M4 acc = M4::identity();
        for (auto &ch : n.children) {
            if (!in_list(ch->name, kXformTags, sizeof(kXformTags) / sizeof(*kXformTags)))
                throw SceneError("transform nodes can only contain transform operations (at " + c.pos(ch->offset) + ")");
            apply_xform_op(acc, *ch, c);  // pre-multiply: later operations apply last
        }
        Prop p; p.kind = Prop::Transform; p.t = acc;
        parent_props->set(*n.attr("name"), p);
        return nullptr;
    }
    check_attrs(n, {"name", "value"}, c);
    const std::string &name = *n.attr("name"), &val = *n.attr("value");
    Prop p;
    if (n.name == "boolean") { p.kind = Prop::Bool; p.b = to_bool(val); }
    else if (n.name == "integer") { p.kind = Prop::Int; p.i = to_int(val); }
    else if (n.name == "float") { p.kind = Prop::Float; p.f = to_float(val); }
    else if (n.name == "string") { p.kind = Prop::String; p.s = val; }
    else if (n.name == "point" || n.name == "vector") {
        // parser.cpp:268-294: two components make a Point2f / Vector2f, three a Point3f / Vector3f
        auto tk = tokenize(val);
        const bool pt = n.name == "point";
        if (tk.size() == 2) {
            p.kind = pt ? Prop::Point2 : Prop::Vector2;
            p.v2[0] = to_float(tk[0]);
            p.v2[1] = to_float(tk[1]);
        } else if (tk.size() == 3) {
            p.kind = pt ? Prop::Point : Prop::Vector;
            p.v = to_v3(val);
        } else {
            throw SceneError(std::string(pt ? "Point" : "Vector") + " " + name + " (value: " + val +
                             ") is not of size 2 or 3");
        }
    } else if (n.name == "color") { p.kind = Prop::Color; p.v = to_v3(val); }
    parent_props->set(name, p);
    return nullptr;
}

// ---------------------------------------------------------------------------
// scene assembly
// ---------------------------------------------------------------------------

std::string join_path(const std::string &base_dir, const std::string &rel) {
    if (!rel.empty() && rel[0] == '/') return rel;
    if (base_dir.empty()) return rel;
    return base_dir + "/" + rel;
}

// Parsed OBJ text of WavefrontOBJ::loadFromFile before toWorld is applied: positions / normals as
// read, texcoords, the dedup'd (p, uv, n) vertex keys and the triangle indices (quads split into
// verts[0..2], verts[0], verts[2], verts[3] order as obj.cpp:130-160 does).
ObjText parse_obj(const std::string &path) {
    std::ifstream is(path);
    if (is.fail()) throw SceneError("unable to open OBJ file \"" + path + "\"");
    struct KeyHash {
        size_t operator()(const ObjKey &k) const {
            size_t h = std::hash<uint32_t>()(k.p);
            h = h * 37 + std::hash<uint32_t>()(k.uv);
            h = h * 37 + std::hash<uint32_t>()(k.n);
            return h;
        }
    };
    ObjText o;
    std::unordered_map<ObjKey, uint32_t, KeyHash> vmap;
    auto parse_vertex = [&](const std::string &s) {
        auto tk = tokenize(s, "/", true);
        if (tk.size() < 1 || tk.size() > 3) throw SceneError("invalid vertex data \"" + s + "\"");
        ObjKey k{(uint32_t)-1, (uint32_t)-1, (uint32_t)-1};
        k.p = (uint32_t)std::stoul(tk[0]);
        if (tk.size() >= 2 && !tk[1].empty()) k.uv = (uint32_t)std::stoul(tk[1]);
        if (tk.size() >= 3 && !tk[2].empty()) k.n = (uint32_t)std::stoul(tk[2]);
        return k;
    };
    std::string line_str;
    while (std::getline(is, line_str)) {
        std::istringstream line(line_str);
        std::string prefix;
        line >> prefix;
        if (prefix == "v") {
            V3 p;
            line >> p.x >> p.y >> p.z;
            o.positions.push_back(p);
        } else if (prefix == "vt") {
            float u = 0, v = 0;
            line >> u >> v;
            o.texcoords.emplace_back(u, v);
        } else if (prefix == "vn") {
            V3 n;
            line >> n.x >> n.y >> n.z;
            o.normals.push_back(n);
        } else if (prefix == "f") {
            std::string s1, s2, s3, s4;
            line >> s1 >> s2 >> s3 >> s4;
            ObjKey verts[6];
            int nv = 3;
            verts[0] = parse_vertex(s1);
            verts[1] = parse_vertex(s2);
            verts[2] = parse_vertex(s3);
            if (!s4.empty()) {
                verts[3] = parse_vertex(s4);
                verts[4] = verts[0];
                verts[5] = verts[2];
                nv = 6;
            }
            for (int i = 0; i < nv; ++i) {
                auto it = vmap.find(verts[i]);
                if (it == vmap.end()) {
                    vmap[verts[i]] = (uint32_t)o.vertices.size();
                    o.indices.push_back((uint32_t)o.vertices.size());
                    o.vertices.push_back(verts[i]);
                } else {
                    o.indices.push_back(it->second);
                }
            }
        }
    }
    return o;
}

// WavefrontOBJ::loadFromFile. A scene that instantiates one OBJ file several times (Nori has no
// instancing: C5 bakes ten transforms of one mesh) parses the text once; toWorld is applied to
// the parsed values per shape, as the reference applies it while reading, so the floats are equal.
void load_obj(const std::string &path, const M4 &trafo, SceneData &sd, nh_shape &sh) {
    auto it_cache = sd.obj_cache.find(path);
    if (it_cache == sd.obj_cache.end()) it_cache = sd.obj_cache.emplace(path, std::make_shared<ObjText>(parse_obj(path))).first;
    const ObjText &obj = *it_cache->second;
    const M4 inv = xf::inverse(trafo);  // nori::Transform(Matrix4f) keeps Matrix4f::inverse()
    std::vector<V3> positions(obj.positions.size()), normals(obj.normals.size());
    V3 bmin = v3(INFINITY, INFINITY, INFINITY), bmax = v3(-INFINITY, -INFINITY, -INFINITY);
    for (size_t i = 0; i < positions.size(); ++i) {
        const V3 p = xform_point(trafo, obj.positions[i]);
        bmin = v3(std::min(bmin.x, p.x), std::min(bmin.y, p.y), std::min(bmin.z, p.z));
        bmax = v3(std::max(bmax.x, p.x), std::max(bmax.y, p.y), std::max(bmax.z, p.z));
        positions[i] = p;
    }
    for (size_t i = 0; i < normals.size(); ++i) normals[i] = normalized(xform_normal(inv, obj.normals[i]));
    const auto &texcoords = obj.texcoords;
    const auto &indices = obj.indices;
    const auto &vertices = obj.vertices;
    const uint32_t nvert = (uint32_t)vertices.size(), nface = (uint32_t)(indices.size() / 3);
    sh.type = NH_SHAPE_MESH;
    sh.v_offset = (uint32_t)(sd.V.size() / 3);
    sh.n_vertices = nvert;
    sh.f_offset = (uint32_t)(sd.F.size() / 3);
    sh.n_faces = nface;
    sh.has_normals = normals.empty() ? 0 : 1;
    sh.has_uvs = texcoords.empty() ? 0 : 1;
    sh.bbox_min[0] = bmin.x; sh.bbox_min[1] = bmin.y; sh.bbox_min[2] = bmin.z;
    sh.bbox_max[0] = bmax.x; sh.bbox_max[1] = bmax.y; sh.bbox_max[2] = bmax.z;

    std::vector<V3> P(nvert), Nn(nvert), Tt(nvert), Bt(nvert);
    std::vector<std::pair<float, float>> Uv(nvert, {0.f, 0.f});
    for (uint32_t i = 0; i < nvert; ++i) {
        if (vertices[i].p - 1 >= positions.size()) throw SceneError("OBJ position index out of range in " + path);
        P[i] = positions[vertices[i].p - 1];
        if (sh.has_normals) {
            if (vertices[i].n - 1 >= normals.size()) throw SceneError("OBJ normal index out of range in " + path);
            Nn[i] = normals[vertices[i].n - 1];
        }
        if (sh.has_uvs) {
            if (vertices[i].uv - 1 >= texcoords.size()) throw SceneError("OBJ texcoord index out of range in " + path);
            Uv[i] = texcoords[vertices[i].uv - 1];
        }
    }
    if (sh.has_normals && sh.has_uvs) {  // obj.cpp:180-224 tangent accumulation
        for (uint32_t t = 0; t < nface; ++t) {
            uint32_t i1 = indices[3 * t], i2 = indices[3 * t + 1], i3 = indices[3 * t + 2];
            V3 e1 = sub(P[i2], P[i1]), e2 = sub(P[i3], P[i1]);
            float du1 = Uv[i2].first - Uv[i1].first, dv1 = Uv[i2].second - Uv[i1].second;
            float du2 = Uv[i3].first - Uv[i1].first, dv2 = Uv[i3].second - Uv[i1].second;
            float frac = du1 * dv2 - du2 * dv1;
            float f = 1.f / (frac == 0.f ? 1e-4f : frac);
            V3 tan = v3(f * (dv2 * e1.x - dv1 * e2.x), f * (dv2 * e1.y - dv1 * e2.y), f * (dv2 * e1.z - dv1 * e2.z));
            V3 tw = xform_vector(trafo, tan);
            for (uint32_t k : {i1, i2, i3}) {
                Tt[k] = v3(Tt[k].x + tw.x, Tt[k].y + tw.y, Tt[k].z + tw.z);
                V3 bw = xform_vector(trafo, cross3(Nn[k], tan));
                Bt[k] = v3(Bt[k].x + bw.x, Bt[k].y + bw.y, Bt[k].z + bw.z);
            }
        }
    }
    for (uint32_t i = 0; i < nvert; ++i) {
        sd.V.insert(sd.V.end(), {P[i].x, P[i].y, P[i].z});
        sd.N.insert(sd.N.end(), {Nn[i].x, Nn[i].y, Nn[i].z});
        sd.UV.insert(sd.UV.end(), {Uv[i].first, Uv[i].second});
        sd.T.insert(sd.T.end(), {Tt[i].x, Tt[i].y, Tt[i].z});
        sd.BT.insert(sd.BT.end(), {Bt[i].x, Bt[i].y, Bt[i].z});
    }
    sd.F.insert(sd.F.end(), indices.begin(), indices.end());
}

// Mesh::update: DiscretePDF over triangle areas (mesh.cpp:35-48, 92-99; dpdf.h)
void build_area_pdf(SceneData &sd, nh_shape &sh) {
    sh.pdf_offset = (uint32_t)sd.area_cdf.size();
    std::vector<float> cdf;
    cdf.reserve(sh.n_faces + 1);
    cdf.push_back(0.0f);
    const float *V = sd.V.data() + 3 * (size_t)sh.v_offset;
    const uint32_t *F = sd.F.data() + 3 * (size_t)sh.f_offset;
    for (uint32_t i = 0; i < sh.n_faces; ++i) {
        const float *p0 = V + 3 * F[3 * i], *p1 = V + 3 * F[3 * i + 1], *p2 = V + 3 * F[3 * i + 2];
        V3 a = v3(p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]);
        V3 b = v3(p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]);
        V3 cr = cross3(a, b);
        float area = 0.5f * std::sqrt(dot3(cr, cr));
        cdf.push_back(cdf.back() + area);
    }
    float sum = cdf.back();
    if (sum > 0) {
        float norm = 1.0f / sum;
        for (size_t i = 1; i < cdf.size(); ++i) cdf[i] *= norm;
        cdf.back() = 1.0f;
        sh.pdf_normalization = norm;
    } else {
        sh.pdf_normalization = 0.0f;
    }
    sd.area_cdf.insert(sd.area_cdf.end(), cdf.begin(), cdf.end());
}

float filter_eval(int type, float radius, float stddev, float B, float C, float x) {
    switch (type) {
        case 0: {  // gaussian (rfilter.cpp:41-47)
            float alpha = -1.0f / (2.0f * stddev * stddev);
            float a = (float)std::exp((double)(alpha * x * x));
            float b = (float)std::exp((double)(alpha * radius * radius));
            return std::max(0.0f, a - b);
        }
        case 1: {  // mitchell (rfilter.cpp:95-111)
            x = std::fabs(2.0f * x / radius);
            float x2 = x * x, x3 = x2 * x;
            if (x < 1)
                return 1.0f / 6.0f * ((12 - 9 * B - 6 * C) * x3 + (-18 + 12 * B + 6 * C) * x2 + (6 - 2 * B));
            else if (x < 2)
                return 1.0f / 6.0f * ((-B - 6 * C) * x3 + (6 * B + 30 * C) * x2 + (-12 * B - 48 * C) * x + (8 * B + 24 * C));
            return 0.0f;
        }
        case 2: return std::max(0.0f, 1.0f - std::fabs(x));  // tent
        default: return 1.0f;                                 // box
    }
}

void set_filter(nh_filter &f, int type, float radius, float stddev, float B, float C) {
    f.radius = radius;
    f.border = (int)std::ceil(radius - 0.5f);
    for (int i = 0; i < 32; ++i) {
        float pos = (radius * (float)i) / 32.0f;
        f.table[i] = filter_eval(type, radius, stddev, B, C, pos);
    }
    f.table[32] = 0.0f;
    f.lookup_factor = 32.0f / radius;
}

}  // namespace

// PerspectiveCamera::update (perspective.cpp:67-95)
void camera_update(SceneData &sd) {
    nh_camera &c = sd.camera;
    c.inv_output_size[0] = 1.0f / (float)c.width;
    c.inv_output_size[1] = 1.0f / (float)c.height;
    // sampleToCamera = Transform(D * T * P).inverse(): the inverse Eigen stored for D * T * P
    const M4 s2c = xf::inverse(xf::camera_projection(c.width, c.height, sd.fov, sd.near_clip, sd.far_clip));
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            c.sample_to_camera[i * 4 + j] = s2c.m[i][j];
            c.camera_to_world[i * 4 + j] = sd.to_world.m[i][j];
        }
    c.near_clip = sd.near_clip;
    c.far_clip = sd.far_clip;
    c.focal_distance = sd.focal;
    // cloneAndInit: fstop/lensRadius coupling (perspective.cpp:39-42)
    c.lens_radius = sd.lens;
    c.lens_draw_order = sd.lens_draw_order;
}

namespace {

// PNGTexture::loadFromFile (PNGTexture.cpp:63-117): lodepng RGBA8 -> InverseGammaCorrect(v / 255) for sRGB images,
// the normal-map decode otherwise (decode_texels); a .hdr file's floats as they are
void load_png_texels(const std::string &fn, std::vector<float> &out, unsigned &w, unsigned &h, bool srgb = true);

// A Texture<Color3f> child (src/textures/consttexture.cpp, checkerboard.cpp, PNGTexture.cpp) -> nh_texture: a
// diffuse albedo, or a shape's normal map (Texture<Normal3f>, the same classes)
nh_texture make_texture(const Obj &t, const std::string &base_dir, SceneData &sd) {
    nh_texture x{};
    const PropList &p = t.props;
    if (t.type == "constant_color") {  // ConstantTexture<Color3f>: value [0]
        x.type = NH_TEXTURE_CONSTANT;
        V3 c = p.get_color("value", v3(0, 0, 0));
        x.value1[0] = c.x; x.value1[1] = c.y; x.value1[2] = c.z;
    } else if (t.type == "checkerboard_color") {  // Checkerboard<Color3f> (checkerboard.cpp:80-87)
        x.type = NH_TEXTURE_CHECKERBOARD;
        p.get_point2("delta", 0.f, 0.f, x.delta);
        p.get_vector2("scale", 1.f, 1.f, x.scale);
        V3 a = p.get_color("value1", v3(0, 0, 0)), b = p.get_color("value2", v3(1, 1, 1));
        x.value1[0] = a.x; x.value1[1] = a.y; x.value1[2] = a.z;
        x.value2[0] = b.x; x.value2[1] = b.y; x.value2[2] = b.z;
    } else if (t.type == "png_texture") {  // PNGTexture (PNGTexture.cpp:23-34, 125-160)
        x.type = NH_TEXTURE_PNG;
        // sRGB defaults to false for the texture named "normal" (PNGTexture.cpp:26)
        x.linear = p.get_bool("sRGB", p.get_string("name", "") != "normal") ? 0 : 1;
        x.intensity = p.get_float("intensity", 1.f);
        x.spherical = p.get_bool("sphericalTexture", false) ? 1 : 0;
        xf::png_rotation(to_xf(p.get_vector("eulerAngles", v3(0, 0, 0))), x.rotation);
        x.scale_u = p.get_float("scaleU", 1.f);
        x.scale_v = p.get_float("scaleV", 1.f);
        x.offset_u = p.get_float("offsetU", 0.f);
        x.offset_v = p.get_float("offsetV", 0.f);
        unsigned w = 0, h = 0;
        std::vector<float> px;
        load_png_texels(join_path(base_dir, p.get_string("filename")), px, w, h, x.linear == 0);
        x.width = (int32_t)w;
        x.height = (int32_t)h;
        x.texel_offset = sd.texels.size() / 4;
        sd.texels.insert(sd.texels.end(), px.begin(), px.end());
    } else {
        throw SceneError("texture \"" + t.type + "\" is not supported as a diffuse albedo or normal map");
    }
    return x;
}

nh_bsdf make_bsdf(const Obj &o, const std::string &base_dir, SceneData &sd) {
    nh_bsdf b{};
    const PropList &p = o.props;
    if (o.type == "diffuse") {
        // Diffuse (diffuse.cpp:32-91): an "albedo" colour becomes a constant texture; a <texture name="albedo">
        // child is the albedo otherwise; neither: the constant 0.5 fallback of cloneAndInit
        b.type = NH_BSDF_DIFFUSE;
        const bool has_color = p.has("albedo");
        V3 a = p.get_color("albedo", v3(0.5f, 0.5f, 0.5f));
        b.albedo[0] = a.x; b.albedo[1] = a.y; b.albedo[2] = a.z;
        bool have = has_color;
        for (auto &ch : o.children) {
            if (ch->tag != "texture") throw SceneError("Diffuse::addChild(<" + ch->tag + ">) is not supported!");
            if (ch->props.get_string("name", "") != "albedo")
                throw SceneError("The name of this texture does not match any field!");
            if (have) throw SceneError("There is already an albedo defined!");
            have = true;
            sd.textures.push_back(make_texture(*ch, base_dir, sd));
            b.albedo_texture = (uint32_t)sd.textures.size();
        }
    } else if (o.type == "mirror") {
        b.type = NH_BSDF_MIRROR;
    } else if (o.type == "dielectric") {
        b.type = NH_BSDF_DIELECTRIC;
        b.int_ior = p.get_float("intIOR", 1.5046f);
        b.ext_ior = p.get_float("extIOR", 1.000277f);
    } else if (o.type == "microfacet") {
        b.type = NH_BSDF_MICROFACET;
        b.alpha = p.get_float("alpha", 0.1f);
        b.int_ior = p.get_float("intIOR", 1.5046f);
        b.ext_ior = p.get_float("extIOR", 1.000277f);
        V3 kd = p.get_color("kd", v3(0.5f, 0.5f, 0.5f));
        b.kd[0] = kd.x; b.kd[1] = kd.y; b.kd[2] = kd.z;
        // m_ks = 1 - m_kd.maxCoeff()  (Eigen max redux: f(c0, f(c1, c2)), f(a,b) = a < b ? b : a)
        float m12 = kd.y < kd.z ? kd.z : kd.y;
        float mx = kd.x < m12 ? m12 : kd.x;
        b.ks = 1 - mx;
    } else {
        throw SceneError("BSDF type \"" + o.type + "\" is not supported by the HIP path");
    }
    return b;
}

nh_bsdf default_diffuse() {
    nh_bsdf b{};
    b.type = NH_BSDF_DIFFUSE;
    b.albedo[0] = b.albedo[1] = b.albedo[2] = 0.5f;
    return b;
}


// ---------------------------------------------------------------------------
// EnvMap + albedo texture (src/emitters/environmentmap.cpp, src/textures/PNGTexture.cpp,
// src/textures/consttexture.cpp). M_PI is Nori's float constant (common.h:59-61), so every
// angle expression is fp32; sincosf/acosf/atan2f/powf are evaluated in fp64 and rounded.
// ---------------------------------------------------------------------------
constexpr float kPiF = 3.14159265358979323846f;

V3 spherical_direction(float theta, float phi) {  // common.cpp:270-281
    const float st = (float)std::sin((double)theta), ct = (float)std::cos((double)theta);
    const float sp = (float)std::sin((double)phi), cp = (float)std::cos((double)phi);
    return v3(st * cp, st * sp, ct);
}
void spherical_coordinates(V3 v, float &theta, float &phi) {  // common.cpp:283-291
    theta = (float)std::acos((double)v.z);
    phi = (float)std::atan2((double)v.y, (double)v.x);
    if (phi < 0) phi += 2 * kPiF;
}
float inverse_gamma(float x) {  // PNGTexture.cpp:442-447
    if (x <= 0.04045f) return x * 1.f / 12.92f;
    return (float)std::pow((double)((x + 0.055f) * 1.f / 1.055f), (double)2.4f);
}

}  // namespace

// PNGTexture::loadFromFile's byte -> float loop over lodepng's RGBA8 array (PNGTexture.cpp:78-95). sRGB: every byte
// through InverseGammaCorrect(b / 255.f). Otherwise the normal-map decode: b / 255 * 2 - 1 (float / int: 255.f, 2.f,
// 1.f), and after every third float `Eigen::Map<Eigen::Vector3f>(data + i - 2).normalize()` -- the triples run over
// the RGBA array, so after the first pixel they straddle pixels and take in alpha (reproduced,
// not fixed). Eigen 3.3.8's normalize(): z = squaredNorm() = x0^2 + (x1^2 + x2^2), and if z > 0 each component is
// divided by sqrt(z) (Dot.h:145-150). Pinned against the reference's own lodepng + Eigen (oracle/normalmap_probe.cpp).
void decode_texels(const uint8_t *px, size_t n, bool srgb, float *out) {
    if (srgb) {
        for (size_t i = 0; i < n; ++i) out[i] = inverse_gamma(static_cast<float>(px[i]) / 255.f);
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        out[i] = static_cast<float>(px[i]) / 255 * 2 - 1;
        if ((i + 1) % 3 == 0) {
            float *v = out + i - 2;
            const float z = v[0] * v[0] + (v[1] * v[1] + v[2] * v[2]);
            if (z > 0.f) {
                const float s = std::sqrt(z);
                v[0] /= s;
                v[1] /= s;
                v[2] /= s;
            }
        }
    }
}

namespace {

void load_png_texels(const std::string &fn, std::vector<float> &out, unsigned &w, unsigned &h, bool srgb) {
    const auto dot = fn.find_last_of('.');
    const std::string ext = dot == std::string::npos ? std::string() : fn.substr(dot);
    // PNGTexture::loadFromFile's order (PNGTexture.cpp:63-72): existence first, then the extension
    if (!std::ifstream(fn).good()) throw SceneError("PNGTexture: image file not found " + fn);
    if (ext == ".hdr") {  // PNGTexture.cpp:97-117: the HDRLoader's floats as they are (no gamma)
        std::string err;
        if (!hdr_decode_rgba(fn, out, w, h, err)) throw SceneError("Could not load HDR file... (" + err + ")");
        return;
    }
    if (ext != ".png") throw SceneError("PNGTexture: file extension " + ext + " unknown.");
    std::vector<uint8_t> px;
    std::string err;
    if (!png_decode_rgba8(fn, px, w, h, err)) throw SceneError("PNGTexture: " + err);
    out.resize(px.size());
    decode_texels(px.data(), px.size(), srgb, out.data());
}

// static_cast<unsigned int>(float) as the reference's x86-64 build executes it: cvttss2si to 64 bits and the low
// word (trunc(x) mod 2^32 for |x| < 2^63, else 0) -- stated explicitly, the C++ cast is undefined for such values
unsigned x86_f2u(float x) { return std::fabs(x) < 0x1p63f ? (unsigned)(uint64_t)(int64_t)x : 0u; }

// PNGTexture::eval (PNGTexture.cpp:125-160) / ConstantTexture::eval, spherical lookups rotated by eulerAngles
V3 env_tex_eval(const nh_envmap &e, const float *rgba, float u, float v) {
    if (e.constant) return v3(rgba[0], rgba[1], rgba[2]);
    if (e.spherical) {
        V3 wi = spherical_direction(v * kPiF, u * 2.f * kPiF);
        // rot * wi (Matrix3f * Vector3f: x0*y0 + (x1*y1 + x2*y2) per row, pinned by the probe's "pdir")
        const float *m = e.rotation;
        wi = v3(m[0] * wi.x + (m[1] * wi.y + m[2] * wi.z), m[3] * wi.x + (m[4] * wi.y + m[5] * wi.z),
                m[6] * wi.x + (m[7] * wi.y + m[8] * wi.z));
        float th, ph;
        spherical_coordinates(wi, th, ph);
        u = ph / (2.f * kPiF);
        v = th / kPiF;
    } else {
        u += e.offset_u;
        v += e.offset_v;
    }
    const unsigned W = (unsigned)e.width, H = (unsigned)e.height;
    const unsigned w = x86_f2u(u * e.scale_u * (float)W);
    const unsigned h = H - x86_f2u(v * e.scale_v * (float)H);
    const unsigned index = (h * W + w) % (W * H);
    return v3(rgba[4 * (size_t)index], rgba[4 * (size_t)index + 1], rgba[4 * (size_t)index + 2]);
}

void build_envmap(const Obj &o, const std::string &base_dir, SceneData &sd, nh_emitter &em) {
    em.type = NH_EMITTER_ENVMAP;
    V3 rad = o.props.get_color("radiance", v3(1, 1, 1));
    em.radiance[0] = rad.x; em.radiance[1] = rad.y; em.radiance[2] = rad.z;
    nh_envmap &e = sd.env;
    e = nh_envmap{};
    e.radiance[0] = rad.x; e.radiance[1] = rad.y; e.radiance[2] = rad.z;
    e.scale_u = e.scale_v = 1.f;
    xf::png_rotation(xf::Vec3{0.f, 0.f, 0.f}, e.rotation);
    const Obj *tex = nullptr;
    for (auto &ch : o.children) {
        if (ch->tag != "texture") throw SceneError("EnvMap::addChild(<" + ch->tag + ">) is not supported!");
        if (ch->props.get_string("name", "") != "albedo")
            throw SceneError("The name of this texture does not match any field!");
        if (tex) throw SceneError("There is already an albedo defined!");
        tex = ch.get();
    }
    if (!tex || tex->type == "constant_color") {  // EnvMap::cloneAndInit fallback: constant 0.5
        V3 c = tex ? tex->props.get_color("value", v3(0, 0, 0)) : v3(0.5f, 0.5f, 0.5f);
        e.width = e.height = 1;
        e.constant = 1;
        sd.env_rgba = {c.x, c.y, c.z, 1.f};
    } else if (tex->type == "png_texture") {
        const PropList &p = tex->props;
        const std::string fn = join_path(base_dir, p.get_string("filename"));
        if (!p.get_bool("sRGB", true)) throw SceneError("png_texture: normal-map (sRGB=false) lookups are not supported");
        xf::png_rotation(to_xf(p.get_vector("eulerAngles", v3(0, 0, 0))), e.rotation);
        e.scale_u = p.get_float("scaleU", 1.f);
        e.scale_v = p.get_float("scaleV", 1.f);
        e.offset_u = p.get_float("offsetU", 0.f);
        e.offset_v = p.get_float("offsetV", 0.f);
        e.spherical = p.get_bool("sphericalTexture", false) ? 1 : 0;
        unsigned w = 0, h = 0;
        load_png_texels(fn, sd.env_rgba, w, h);
        e.width = (int32_t)w;
        e.height = (int32_t)h;
    } else {
        throw SceneError("texture \"" + tex->type + "\" is not supported for environment maps");
    }
    // EnvMap::calculateProbs (environmentmap.cpp:155-169): note the (row, col) -> (u, v) swap
    const unsigned W = (unsigned)e.width, H = (unsigned)e.height;
    sd.env_cdf.assign(1, 0.0f);
    sd.env_cdf.reserve((size_t)W * H + 1);
    for (unsigned i = 0; i < H; ++i)
        for (unsigned j = 0; j < W; ++j) {
            V3 c = env_tex_eval(e, sd.env_rgba.data(), i / (float)H, j / (float)W);
            float lum = c.x * 0.212671f + c.y * 0.715160f + c.z * 0.072169f;
            sd.env_cdf.push_back(sd.env_cdf.back() + std::fabs(lum));
        }
    const float sum = sd.env_cdf.back();
    if (sum > 0) {
        e.normalization = 1.0f / sum;
        for (size_t i = 1; i < sd.env_cdf.size(); ++i) sd.env_cdf[i] *= e.normalization;
        sd.env_cdf.back() = 1.0f;
    } else {
        e.normalization = 0.0f;
    }
}

void build_scene(const Obj &scene, const std::string &base_dir, SceneData &sd) {
    bool have_camera = false, have_integrator = false, have_sampler = false;
    set_filter(sd.filter, 0, 2.0f, 0.5f, 1.0f / 3.0f, 1.0f / 3.0f);
    for (auto &chp : scene.children) {
        const Obj &ch = *chp;
        if (ch.tag == "integrator") {
            if (have_integrator) throw SceneError("there can only be one integrator per scene");
            have_integrator = true;
            if (ch.type == "path_mis") sd.integrator = NH_INTEGRATOR_PATH_MIS;
            else if (ch.type == "path_mats") sd.integrator = NH_INTEGRATOR_PATH_MATS;
            else if (ch.type == "direct_ems") sd.integrator = NH_INTEGRATOR_DIRECT_EMS;
            else if (ch.type == "direct_mats") sd.integrator = NH_INTEGRATOR_DIRECT_MATS;
            else if (ch.type == "direct_mis") sd.integrator = NH_INTEGRATOR_DIRECT_MIS;
            else if (ch.type == "direct") sd.integrator = NH_INTEGRATOR_DIRECT;
            else if (ch.type == "normals") {  // NormalIntegrator (normals.cpp:10-12)
                sd.integrator = NH_INTEGRATOR_NORMALS;
                const V3 dir = ch.props.get_point("direction", v3(0, 0, 1));
                sd.normals_dir[0] = dir.x; sd.normals_dir[1] = dir.y; sd.normals_dir[2] = dir.z;
            }
            else throw SceneError("integrator \"" + ch.type + "\" is not supported by the HIP path");
        } else if (ch.tag == "camera") {
            if (have_camera) throw SceneError("there can only be one camera per scene");
            have_camera = true;
            if (ch.type != "perspective") throw SceneError("camera \"" + ch.type + "\" is not supported");
            sd.camera.width = ch.props.get_int("width", 1280);
            sd.camera.height = ch.props.get_int("height", 720);
            sd.to_world = ch.props.get_transform("toWorld", M4::identity());
            sd.fov = ch.props.get_float("fov", 30.0f);
            sd.near_clip = ch.props.get_float("nearClip", 1e-4f);
            sd.far_clip = ch.props.get_float("farClip", 1e4f);
            sd.focal = ch.props.get_float("focalDistance", 10.f);
            sd.fstop = ch.props.get_float("fstop", 0.f);
            sd.lens = ch.props.get_float("lensRadius", 0.f);
            if (sd.fstop == 0.f) sd.fstop = sd.focal / sd.lens;
            else sd.lens = sd.focal / sd.fstop;
            for (auto &rf : ch.children) {
                if (rf->tag != "rfilter") throw SceneError("camera child <" + rf->tag + "> is not supported");
                const PropList &p = rf->props;
                if (rf->type == "gaussian")
                    set_filter(sd.filter, 0, p.get_float("radius", 2.0f), p.get_float("stddev", 0.5f), 0, 0);
                else if (rf->type == "mitchell")
                    set_filter(sd.filter, 1, p.get_float("radius", 2.0f), 0, p.get_float("B", 1.0f / 3.0f),
                               p.get_float("C", 1.0f / 3.0f));
                else if (rf->type == "tent") set_filter(sd.filter, 2, 1.0f, 0, 0, 0);
                else if (rf->type == "box") set_filter(sd.filter, 3, 0.5f, 0, 0, 0);
                else throw SceneError("rfilter \"" + rf->type + "\" is not supported");
            }
        } else if (ch.tag == "sampler") {
            if (have_sampler) throw SceneError("there can only be one sampler per scene");
            have_sampler = true;
            if (ch.type != "independent")
                throw SceneError("sampler \"" + ch.type + "\" is not supported (the HIP path uses per-path pcg32)");
            sd.sample_count = ch.props.get_int("sampleCount", 1);
        } else if (ch.tag == "shape") {
            nh_shape sh{};
            sh.emitter = -1;
            int bsdf = -1, emitter = -1;
            nh_emitter em{};
            for (auto &sc : ch.children) {
                if (sc->tag == "bsdf") {
                    if (bsdf >= 0) throw SceneError("Shape: tried to register multiple BSDF instances");
                    sd.bsdfs.push_back(make_bsdf(*sc, base_dir, sd));
                    bsdf = (int)sd.bsdfs.size() - 1;
                } else if (sc->tag == "emitter") {
                    if (emitter >= 0) throw SceneError("Shape: tried to register multiple Emitter instances");
                    if (sc->type != "area") throw SceneError("shape emitter \"" + sc->type + "\" is not supported");
                    em.type = NH_EMITTER_AREA;
                    V3 r = sc->props.get_color("radiance");
                    em.radiance[0] = r.x; em.radiance[1] = r.y; em.radiance[2] = r.z;
                    em.light_prob = sc->props.get_float("lightWeight", 1.f);
                    emitter = 1;
                } else if (sc->tag == "medium") {
                    throw SceneError("participating media are out of scope for path_mis");
                } else if (sc->tag == "texture") {  // Shape::addChild ETexture (shape.cpp:138-147)
                    const std::string nm = sc->props.get_string("name", "");
                    if (nm != "normal") throw SceneError("Shape does not have a texture with name: " + nm);
                    if (sh.normal_map) throw SceneError("There is already a normal map defined!");
                    sd.textures.push_back(make_texture(*sc, base_dir, sd));
                    sh.normal_map = (uint32_t)sd.textures.size();
                } else {
                    throw SceneError("shape child <" + sc->tag + "> is not supported");
                }
            }
            if (bsdf < 0) {  // Shape::cloneAndInit default diffuse
                sd.bsdfs.push_back(default_diffuse());
                bsdf = (int)sd.bsdfs.size() - 1;
            }
            sh.bsdf = bsdf;
            if (ch.type == "obj") {
                std::string fn = join_path(base_dir, ch.props.get_string("filename"));
                load_obj(fn, ch.props.get_transform("toWorld", M4::identity()), sd, sh);
            } else if (ch.type == "sphere") {
                sh.type = NH_SHAPE_SPHERE;
                V3 c = ch.props.get_point("center", v3(0, 0, 0));
                float r = ch.props.get_float("radius", 1.f);
                sh.center[0] = c.x; sh.center[1] = c.y; sh.center[2] = c.z;
                sh.radius = r;
                sh.v_offset = (uint32_t)(sd.V.size() / 3);
                sh.f_offset = (uint32_t)(sd.F.size() / 3);
                sh.bbox_min[0] = c.x - r; sh.bbox_min[1] = c.y - r; sh.bbox_min[2] = c.z - r;
                sh.bbox_max[0] = c.x + r; sh.bbox_max[1] = c.y + r; sh.bbox_max[2] = c.z + r;
            } else {
                throw SceneError("shape \"" + ch.type + "\" is not supported");
            }
            if (sh.type == NH_SHAPE_MESH) build_area_pdf(sd, sh);
            if (emitter >= 0) {
                em.shape = (int32_t)sd.shapes.size();
                sd.emitters.push_back(em);
                sh.emitter = (int32_t)sd.emitters.size() - 1;
            }
            sd.shapes.push_back(sh);
        } else if (ch.tag == "emitter") {
            nh_emitter em{};
            em.shape = -1;
            em.light_prob = ch.props.get_float("lightWeight", 1.f);
            if (ch.type == "point") {
                em.type = NH_EMITTER_POINT;
                V3 p = ch.props.get_point("position", v3(0, 0, 0));
                V3 pw = ch.props.get_color("power", v3(1, 1, 1));
                em.position[0] = p.x; em.position[1] = p.y; em.position[2] = p.z;
                // PointLight::update: m_radiance = m_power / (4 * M_PI)
                float d = 4 * 3.14159265358979323846f;
                em.radiance[0] = pw.x / d; em.radiance[1] = pw.y / d; em.radiance[2] = pw.z / d;
            } else if (ch.type == "envmap") {
                if (sd.envmap >= 0) throw SceneError("only one environment map per scene is supported");
                build_envmap(ch, base_dir, sd, em);
                sd.envmap = (int32_t)sd.emitters.size();
            } else {
                throw SceneError("emitter \"" + ch.type + "\" is not supported yet");
            }
            sd.emitters.push_back(em);
        } else if (ch.tag == "denoiser") {
            // Scene::addChild (scene.cpp:242-245) + SimpleDenoiser's constructor clamps (simple.cpp:15-24)
            if (sd.denoiser.type != NH_DENOISER_NONE) throw SceneError("There can only be one denoiser per scene!");
            if (ch.type != "simple") throw SceneError("denoiser \"" + ch.type + "\" is not supported");
            const float eps = 1e-4f;
            auto clampf = [](float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); };
            auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
            sd.denoiser.type = NH_DENOISER_SIMPLE;
            sd.denoiser.sigma_d = clampf(ch.props.get_float("sigma_d", 0.f), eps, 10.f);
            sd.denoiser.sigma_vr = clampf(ch.props.get_float("sigma_vr", 0.6f), eps, 10.f);
            sd.denoiser.range = clampi(ch.props.get_int("range", 1), 0, 50);
            sd.denoiser.amount = clampi(ch.props.get_int("amount", 1), 1, 10);
        } else if (ch.tag == "renderer") {
            // OptixRenderer settings object (OptixRenderer.h:17-36): no effect on the path_mis hot path
        } else if (ch.tag == "medium") {
            if (ch.type != "vacuum") throw SceneError("participating media are out of scope for path_mis");
        } else {
            throw SceneError("Scene::addChild(<" + ch.tag + ">) is not supported");
        }
    }
    if (!have_integrator) throw SceneError("No integrator was specified!");
    if (!have_camera) throw SceneError("No camera was specified!");
    // Scene::update: emitter DiscretePDF
    sd.emitter_cdf.assign(1, 0.0f);
    for (auto &e : sd.emitters) sd.emitter_cdf.push_back(sd.emitter_cdf.back() + e.light_prob);
    float sum = sd.emitter_cdf.back();
    if (sum > 0) {
        float norm = 1.0f / sum;
        for (size_t i = 1; i < sd.emitter_cdf.size(); ++i) sd.emitter_cdf[i] *= norm;
        sd.emitter_cdf.back() = 1.0f;
    }
    camera_update(sd);
}

}  // namespace

SceneData *load_scene(const std::string &path, int scene_index) {
    std::ifstream is(path, std::ios::binary);
    if (is.fail()) throw SceneError("unable to open scene file \"" + path + "\"");
    std::stringstream ss;
    ss << is.rdbuf();
    std::string text = ss.str();
    std::unique_ptr<XmlNode> root;
    try {
        root = xml_parse(text);
    } catch (const XmlError &e) {
        throw SceneError("Error while parsing \"" + path + "\": " + e.what());
    }
    ParseCtx c{text, path};
    auto obj = parse_node(*root, nullptr, "", c);
    const Obj *scene = nullptr;
    if (obj->tag == "scene") {
        if (scene_index > 0) throw SceneError("scene index out of range");
        scene = obj.get();
    } else if (obj->tag == "test") {
        int k = 0;
        for (auto &ch : obj->children)
            if (ch->tag == "scene" && k++ == scene_index) { scene = ch.get(); break; }
        if (!scene) throw SceneError("scene index out of range in test file");
    } else {
        throw SceneError("root element <" + obj->tag + "> is not a scene");
    }
    std::string base_dir;
    auto slash = path.find_last_of('/');
    if (slash != std::string::npos) base_dir = path.substr(0, slash);
    auto sd = std::make_unique<SceneData>();
    build_scene(*scene, base_dir, *sd);
    sd->obj_cache.clear();
    return sd.release();
}

void fill_desc(const SceneData &sd, nh_scene_desc *d) {
    std::memset(d, 0, sizeof(*d));
    d->camera = sd.camera;
    d->filter = sd.filter;
    d->integrator = sd.integrator;
    d->sample_count = sd.sample_count;
    d->n_shapes = (uint32_t)sd.shapes.size();
    d->shapes = sd.shapes.data();
    d->n_bsdfs = (uint32_t)sd.bsdfs.size();
    d->bsdfs = sd.bsdfs.data();
    d->n_emitters = (uint32_t)sd.emitters.size();
    d->emitters = sd.emitters.data();
    d->emitter_cdf = sd.emitter_cdf.data();
    d->envmap = sd.envmap;
    d->denoiser = sd.denoiser;
    d->n_vertices = (uint32_t)(sd.V.size() / 3);
    d->V = sd.V.data();
    d->N = sd.N.data();
    d->UV = sd.UV.data();
    d->T = sd.T.data();
    d->BT = sd.BT.data();
    d->n_faces = (uint32_t)(sd.F.size() / 3);
    d->F = sd.F.data();
    d->n_area_cdf = (uint32_t)sd.area_cdf.size();
    d->area_cdf = sd.area_cdf.data();
    d->n_textures = (uint32_t)sd.textures.size();
    d->textures = sd.textures.data();
    d->n_texels = sd.texels.size() / 4;
    d->texels = sd.texels.data();
    for (int i = 0; i < 3; ++i) d->normals_direction[i] = sd.normals_dir[i];
    if (sd.envmap >= 0) {
        d->env = sd.env;
        d->env.rgba = sd.env_rgba.data();
        d->env.cdf = sd.env_cdf.data();
    }
}

}  // namespace nh

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
struct nh_scene {
    nh::SceneData *data;
};

extern "C" {

const char *nh_host_last_error(void) { return nh::g_host_error.c_str(); }

static int load_impl(const char *path, int index, nh_scene **out) {
    if (!path || !out) { nh::set_host_error("null argument"); return NH_ERR_INVALID; }
    try {
        auto *s = new nh_scene{nh::load_scene(path, index)};
        *out = s;
        return NH_OK;
    } catch (const std::exception &e) {
        nh::set_host_error(e.what());
        return NH_ERR_IO;
    }
}

int nh_scene_load_xml(const char *path, nh_scene **out) { return load_impl(path, 0, out); }
int nh_scene_load_xml_index(const char *path, int32_t index, nh_scene **out) { return load_impl(path, index, out); }

int nh_scene_get_desc(const nh_scene *scene, nh_scene_desc *out) {
    if (!scene || !out) { nh::set_host_error("null argument"); return NH_ERR_INVALID; }
    nh::fill_desc(*scene->data, out);
    return NH_OK;
}

int nh_scene_set_resolution(nh_scene *scene, int32_t width, int32_t height) {
    if (!scene || width <= 0 || height <= 0) { nh::set_host_error("invalid resolution"); return NH_ERR_INVALID; }
    scene->data->camera.width = width;
    scene->data->camera.height = height;
    nh::camera_update(*scene->data);
    return NH_OK;
}

int nh_scene_set_sample_count(nh_scene *scene, int32_t spp) {
    if (!scene || spp <= 0) { nh::set_host_error("invalid sample count"); return NH_ERR_INVALID; }
    scene->data->sample_count = spp;
    return NH_OK;
}

int nh_scene_set_bsdf(nh_scene *scene, uint32_t shape, const nh_bsdf *bsdf) {
    if (!scene || !bsdf || shape >= scene->data->shapes.size()) { nh::set_host_error("invalid shape index"); return NH_ERR_INVALID; }
    scene->data->bsdfs.push_back(*bsdf);
    scene->data->shapes[shape].bsdf = (int32_t)scene->data->bsdfs.size() - 1;
    return NH_OK;
}

uint32_t nh_scene_add_texture(nh_scene *scene, const nh_texture *tex, const float *texels) {
    if (!scene || !tex || tex->type < NH_TEXTURE_CONSTANT || tex->type > NH_TEXTURE_PNG) {
        nh::set_host_error("invalid texture");
        return 0;
    }
    nh_texture t = *tex;
    if (t.type == NH_TEXTURE_PNG) {
        if (!texels || t.width <= 0 || t.height <= 0) { nh::set_host_error("png texture without texels"); return 0; }
        auto &v = scene->data->texels;
        t.texel_offset = v.size() / 4;
        v.insert(v.end(), texels, texels + (size_t)t.width * (size_t)t.height * 4);
    }
    scene->data->textures.push_back(t);
    return (uint32_t)scene->data->textures.size();
}

int nh_scene_set_normal_map(nh_scene *scene, uint32_t shape, uint32_t texture) {
    if (!scene || shape >= scene->data->shapes.size() || texture > scene->data->textures.size()) {
        nh::set_host_error("invalid shape or texture index");
        return NH_ERR_INVALID;
    }
    scene->data->shapes[shape].normal_map = texture;
    return NH_OK;
}

int nh_scene_set_lens_draw_order(nh_scene *scene, int32_t order) {
    if (!scene || (order != NH_LENS_DRAWS_LTR && order != NH_LENS_DRAWS_RTL)) {
        nh::set_host_error("invalid lens draw order");
        return NH_ERR_INVALID;
    }
    scene->data->lens_draw_order = order;
    nh::camera_update(*scene->data);
    return NH_OK;
}

int nh_texture_decode(const uint8_t *rgba8, uint64_t n, int32_t srgb, float *out) {
    if ((!rgba8 || !out) && n) { nh::set_host_error("null argument"); return NH_ERR_INVALID; }
    nh::decode_texels(rgba8, (size_t)n, srgb != 0, out);
    return NH_OK;
}

int nh_scene_set_integrator(nh_scene *scene, int32_t integrator) {
    if (!scene || integrator < NH_INTEGRATOR_PATH_MIS || integrator > NH_INTEGRATOR_NORMALS) {
        nh::set_host_error("invalid integrator");
        return NH_ERR_INVALID;
    }
    scene->data->integrator = integrator;
    return NH_OK;
}

void nh_scene_free(nh_scene *scene) {
    if (!scene) return;
    delete scene->data;
    delete scene;
}

// The loader's own transform functions (nori_transform.h) behind oracle/eigen_xform_probe.cpp's protocol.
int nh_debug_transform(const char *request, float *out, int32_t cap) {
    namespace xf = nh::xf;
    if (!request || !out) { nh::set_host_error("null argument"); return -1; }
    std::istringstream in(request);
    auto next = [&in]() -> float {
        std::string t;
        if (!(in >> t)) throw std::runtime_error("truncated request");
        uint32_t u = (uint32_t)std::stoul(t, nullptr, 16);
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    };
    auto m4 = [&next]() {
        xf::Mat4 m;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) m.m[i][j] = next();
        return m;
    };
    auto v3 = [&next]() {
        const float x = next(), y = next(), z = next();
        return xf::Vec3{x, y, z};
    };
    std::vector<float> r;
    auto put_m4 = [&r](const xf::Mat4 &m) {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.push_back(m.m[i][j]);
    };
    try {
        std::string cmd;
        in >> cmd;
        if (cmd == "inv") {
            put_m4(xf::inverse(m4()));
        } else if (cmd == "xf") {
            int n = 0;
            in >> n;
            xf::Mat4 t = xf::Mat4::identity();
            for (int k = 0; k < n; ++k) {
                std::string op;
                in >> op;
                if (op == "t") xf::pre_translate(t, v3());
                else if (op == "s") xf::pre_scale(t, v3());
                else if (op == "r") {
                    const float angle = xf::deg_to_rad(next());
                    xf::pre_rotate(t, angle, v3());
                } else if (op == "m") xf::pre_affine(t, m4());
                else if (op == "l") {
                    const xf::Vec3 o = v3(), tg = v3(), up = v3();
                    xf::pre_affine(t, xf::lookat_matrix(o, tg, up));
                } else throw std::runtime_error("unknown transform op " + op);
            }
            put_m4(t);
            put_m4(xf::inverse(t));
        } else if (cmd == "cam") {
            const float w = next(), h = next(), fov = next(), n = next(), f = next();
            const xf::Mat4 p = xf::camera_projection((int)w, (int)h, fov, n, f);
            put_m4(xf::inverse(p));
            put_m4(p);
        } else if (cmd == "prot") {
            float rot[9];
            xf::png_rotation(v3(), rot);
            r.insert(r.end(), rot, rot + 9);
        } else if (cmd == "pdir") {
            float m[9];
            for (float &x : m) x = next();
            const xf::Vec3 v = v3();
            r.insert(r.end(), {xf::dot3(m[0], m[1], m[2], v.x, v.y, v.z), xf::dot3(m[3], m[4], m[5], v.x, v.y, v.z),
                               xf::dot3(m[6], m[7], m[8], v.x, v.y, v.z)});
        } else if (cmd == "pt" || cmd == "vec" || cmd == "nrm") {
            const xf::Mat4 m = m4();
            const xf::Vec3 v = v3();
            xf::Vec3 o;
            if (cmd == "pt") o = xf::apply_point(m, v);
            else if (cmd == "vec") o = xf::apply_vector(m, v);
            else o = xf::normalized(xf::apply_normal(xf::inverse(m), v));
            r.insert(r.end(), {o.x, o.y, o.z});
        } else {
            throw std::runtime_error("unknown request " + cmd);
        }
    } catch (const std::exception &e) {
        nh::set_host_error(e.what());
        return -1;
    }
    if ((int32_t)r.size() > cap) { nh::set_host_error("output capacity too small"); return -1; }
    std::memcpy(out, r.data(), r.size() * sizeof(float));
    return (int32_t)r.size();
}

}  // extern "C"
