// .rrscene loading and host-side per-frame evaluation. See scene.hpp.
#include "scene.hpp"

#include <cfloat>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "json.hpp"

namespace rr {

namespace {

std::string read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open scene file: " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

std::string dirname_of(const std::string& p) {
    size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

void vec3(const Json& j, double out[3]) {
    if (j.size() < 3) throw std::runtime_error("expected 3-vector");
    for (int i = 0; i < 3; ++i) out[i] = j[i].as_num();
}

int ipo_of(const std::string& s) {
    if (s == "CONSTANT") return IPO_CONSTANT;
    if (s == "LINEAR") return IPO_LINEAR;
    if (s == "BEZIER") return IPO_BEZIER;
    throw std::runtime_error("unsupported keyframe interpolation: " + s);
}

// ---- procedural meshes (stand-in scenes) -------------------
void gen_cube(MeshDesc& m, double size) {
    const double h = size * 0.5;
    const int q[6][4] = {{0, 4, 6, 2}, {3, 2, 6, 7}, {7, 6, 4, 5}, {5, 1, 3, 7}, {1, 0, 2, 3}, {5, 4, 0, 1}};
    for (int i = 0; i < 8; ++i) {
        m.verts.push_back((float)((i & 4) ? h : -h));
        m.verts.push_back((float)((i & 2) ? h : -h));
        m.verts.push_back((float)((i & 1) ? h : -h));
    }
    for (auto& f : q) {
        m.tris.insert(m.tris.end(), {(uint32_t)f[0], (uint32_t)f[1], (uint32_t)f[2],
                                     (uint32_t)f[0], (uint32_t)f[2], (uint32_t)f[3]});
        m.mat_idx.push_back(0);
        m.mat_idx.push_back(0);
    }
}

// size x size plane at z = 0 cut into n x n quads (n = 1: Blender's 2-triangle
// plane). Large scenes use n > 1: a 2-triangle ground spanning the whole scene
// inflates every LBVH ancestor box of its Morton neighbourhood.
void gen_plane(MeshDesc& m, double size, int n) {
    if (n < 1) n = 1;
    for (int y = 0; y <= n; ++y)
        for (int x = 0; x <= n; ++x) {
            m.verts.push_back((float)(size * ((double)x / n - 0.5)));
            m.verts.push_back((float)(size * ((double)y / n - 0.5)));
            m.verts.push_back(0.0f);
        }
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) {
            const uint32_t a = (uint32_t)(y * (n + 1) + x), b = a + 1, c = a + (uint32_t)(n + 1) + 1,
                           d = a + (uint32_t)(n + 1);
            m.tris.insert(m.tris.end(), {a, b, c, a, c, d});
            m.mat_idx.push_back(0);
            m.mat_idx.push_back(0);
        }
}

void gen_icosphere(MeshDesc& m, int subdiv, double radius) {
    const double t = (1.0 + std::sqrt(5.0)) / 2.0;
    std::vector<double> v = {-1, t, 0, 1, t, 0, -1, -t, 0, 1, -t, 0, 0, -1, t, 0, 1, t,
                             0, -1, -t, 0, 1, -t, t, 0, -1, t, 0, 1, -t, 0, -1, -t, 0, 1};
    std::vector<uint32_t> f = {0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4,
                               11, 10, 2, 10, 7, 6, 7, 1, 8, 3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8,
                               3, 8, 9, 4, 9, 5, 2, 4, 11, 6, 2, 10, 8, 6, 7, 9, 8, 1};
    auto norm = [&](size_t i) {
        double l = std::sqrt(v[3 * i] * v[3 * i] + v[3 * i + 1] * v[3 * i + 1] + v[3 * i + 2] * v[3 * i + 2]);
        v[3 * i] /= l; v[3 * i + 1] /= l; v[3 * i + 2] /= l;
    };
    for (size_t i = 0; i < v.size() / 3; ++i) norm(i);
    for (int s = 0; s < subdiv; ++s) {
        std::vector<uint32_t> nf;
        nf.reserve(f.size() * 4);
        std::vector<std::pair<uint64_t, uint32_t>> cache;
        std::vector<std::vector<std::pair<uint32_t, uint32_t>>> edge(v.size() / 3);
        auto mid = [&](uint32_t a, uint32_t b) {
            uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
            for (auto& e : edge[lo]) if (e.first == hi) return e.second;
            uint32_t id = (uint32_t)(v.size() / 3);
            v.push_back((v[3 * a] + v[3 * b]) * 0.5);
            v.push_back((v[3 * a + 1] + v[3 * b + 1]) * 0.5);
            v.push_back((v[3 * a + 2] + v[3 * b + 2]) * 0.5);
            norm(id);
            edge.emplace_back();
            edge[lo].push_back({hi, id});
            return id;
        };
        for (size_t k = 0; k < f.size(); k += 3) {
            uint32_t a = f[k], b = f[k + 1], c = f[k + 2];
            uint32_t ab = mid(a, b), bc = mid(b, c), ca = mid(c, a);
            nf.insert(nf.end(), {a, ab, ca, b, bc, ab, c, ca, bc, ab, bc, ca});
        }
        f.swap(nf);
    }
    m.verts.resize(v.size());
    for (size_t i = 0; i < v.size(); ++i) m.verts[i] = (float)(v[i] * radius);
    m.tris = f;
    m.mat_idx.assign(f.size() / 3, 0);
}

// Icosphere whose vertices are pushed along the normal by a smooth
// deterministic field, r' = r (1 + amp sin(f x + 1.3) sin(f y + 0.7) sin(f z + 2.1))
// on the unit sphere (the C5 synthetic scene's "displaced icospheres",
// SURVEY.md §8d C5). Triangle count = 20 * 4^subdivisions.
void gen_displaced_icosphere(MeshDesc& m, int subdiv, double radius, double amp, double freq) {
    gen_icosphere(m, subdiv, 1.0);
    for (size_t i = 0; i + 2 < m.verts.size(); i += 3) {
        const double x = m.verts[i], y = m.verts[i + 1], z = m.verts[i + 2];
        const double k = radius * (1.0 + amp * std::sin(freq * x + 1.3) * std::sin(freq * y + 0.7) *
                                              std::sin(freq * z + 2.1));
        m.verts[i] = (float)(x * k);
        m.verts[i + 1] = (float)(y * k);
        m.verts[i + 2] = (float)(z * k);
    }
}

void parse_mesh(const Json& jm, MeshDesc& m) {
    m.name = jm.get_str("name", "");
    if (jm.has("generator")) {
        const Json& g = jm["generator"];
        const std::string t = g["type"].as_str();
        if (t == "cube") gen_cube(m, g.get_num("size", 2.0));
        else if (t == "plane") gen_plane(m, g.get_num("size", 2.0), (int)g.get_num("subdivisions", 1));
        else if (t == "icosphere") gen_icosphere(m, (int)g.get_num("subdivisions", 2), g.get_num("radius", 1.0));
        else if (t == "displaced_icosphere")
            gen_displaced_icosphere(m, (int)g.get_num("subdivisions", 3), g.get_num("radius", 1.0),
                                    g.get_num("amplitude", 0.15), g.get_num("frequency", 5.0));
        else throw std::runtime_error("unknown mesh generator: " + t);
    } else {
        const Json& v = jm["vertices"];
        m.verts.resize(v.size());
        for (size_t i = 0; i < v.size(); ++i) m.verts[i] = (float)v[i].as_num();
        const Json& t = jm["triangles"];
        m.tris.resize(t.size());
        for (size_t i = 0; i < t.size(); ++i) m.tris[i] = (uint32_t)t[i].as_num();
        m.mat_idx.assign(m.tris.size() / 3, 0);
        if (jm.has("material_indices")) {
            const Json& mi = jm["material_indices"];
            for (size_t i = 0; i < mi.size() && i < m.mat_idx.size(); ++i) m.mat_idx[i] = (int)mi[i].as_num();
        }
    }
    if (m.tris.size() % 3) throw std::runtime_error("mesh '" + m.name + "': triangle index count not a multiple of 3");
    const uint32_t nv = (uint32_t)(m.verts.size() / 3);
    for (uint32_t i : m.tris)
        if (i >= nv) throw std::runtime_error("mesh '" + m.name + "': vertex index out of range");
    if (jm.has("material_slots")) {
        const Json& s = jm["material_slots"];
        for (size_t i = 0; i < s.size(); ++i) m.slots.push_back((int)s[i].as_num());
    }
}

// ---- Blender F-Curve evaluation ------------------------------------------
// Restated from Blender's published fcurve evaluation (BKE fcurve.cc of
// Blender 3.6, the version the reference pins: pull-blender-image.sh:3-4):
// fcurve_eval_keyframes -> _extrapolate / _interpolate, correct_bezpart,
// findzero/solve_cubic (double), berekeny (float).
constexpr double kSmall = -1.0e-10;

double sqrt3d(double d) {
    if (d == 0.0) return 0.0;
    if (d < 0.0) return -std::exp(std::log(-d) / 3.0);
    return std::exp(std::log(d) / 3.0);
}

inline bool in01(float x) { return x >= (float)kSmall && x <= 1.000001f; }

int solve_cubic(double c0, double c1, double c2, double c3, float* o) {
    double a, b, c, p, q, d, t, phi;
    int nr = 0;
    if (c3 != 0.0) {
        a = c2 / c3;
        b = c1 / c3;
        c = c0 / c3;
        a = a / 3;
        p = b / 3 - a * a;
        q = (2 * a * a * a - a * b + c) / 2;
        d = q * q + p * p * p;
        if (d > 0.0) {
            t = std::sqrt(d);
            o[0] = (float)(sqrt3d(-q + t) + sqrt3d(-q - t) - a);
            return in01(o[0]) ? 1 : 0;
        }
        if (d == 0.0) {
            t = sqrt3d(-q);
            o[0] = (float)(2 * t - a);
            if (in01(o[0])) nr++;
            o[nr] = (float)(-t - a);
            return in01(o[nr]) ? nr + 1 : nr;
        }
        phi = std::acos(-q / std::sqrt(-(p * p * p)));
        t = std::sqrt(-p);
        p = std::cos(phi / 3);
        q = std::sqrt(3 - 3 * p * p);
        o[0] = (float)(2 * t * p - a);
        if (in01(o[0])) nr++;
        o[nr] = (float)(-t * (p + q) - a);
        if (in01(o[nr])) nr++;
        o[nr] = (float)(-t * (p - q) - a);
        return in01(o[nr]) ? nr + 1 : nr;
    }
    a = c2;
    b = c1;
    c = c0;
    if (a != 0.0) {
        p = b * b - 4 * a * c;
        if (p > 0) {
            p = std::sqrt(p);
            o[0] = (float)((-b - p) / (2 * a));
            if (in01(o[0])) nr++;
            o[nr] = (float)((-b + p) / (2 * a));
            return in01(o[nr]) ? nr + 1 : nr;
        }
        if (p == 0) {
            o[0] = (float)(-b / (2 * a));
            if (in01(o[0])) return 1;
        }
        return 0;
    }
    if (b != 0.0) {
        o[0] = (float)(-c / b);
        return in01(o[0]) ? 1 : 0;
    }
    if (c == 0.0) {
        o[0] = 0.0f;
        return 1;
    }
    return 0;
}

int findzero(float x, float q0, float q1, float q2, float q3, float* o) {
    // float arithmetic widened to double, as Blender writes it
    const double c0 = q0 - x;
    const double c1 = 3.0f * (q1 - q0);
    const double c2 = 3.0f * (q0 - 2.0f * q1 + q2);
    const double c3 = q3 - q0 + 3.0f * (q1 - q2);
    return solve_cubic(c0, c1, c2, c3, o);
}

float berekeny(float f1, float f2, float f3, float f4, float t) {
    const float c0 = f1;
    const float c1 = 3.0f * (f2 - f1);
    const float c2 = 3.0f * (f1 - 2.0f * f2 + f3);
    const float c3 = f4 - f1 + 3.0f * (f2 - f3);
    return c0 + t * c1 + t * t * c2 + t * t * t * c3;
}

void correct_bezpart(const float v1[2], float v2[2], float v3[2], const float v4[2]) {
    float h1[2] = {v1[0] - v2[0], v1[1] - v2[1]};
    float h2[2] = {v4[0] - v3[0], v4[1] - v3[1]};
    const float len = v4[0] - v1[0];
    const float len1 = std::fabs(h1[0]);
    const float len2 = std::fabs(h2[0]);
    if ((len1 + len2) == 0.0f) return;
    if ((len1 + len2) > len) {
        const float fac = len / (len1 + len2);
        v2[0] = (v1[0] - fac * h1[0]);
        v2[1] = (v1[1] - fac * h1[1]);
        v3[0] = (v4[0] - fac * h2[0]);
        v3[1] = (v4[1] - fac * h2[1]);
    }
}

float extrapolate(const FCurve& fc, float evaltime, int endpoint, int dir) {
    const Keyframe& e = fc.keys[endpoint];
    if (e.ipo == IPO_CONSTANT || fc.extrapolation == 0) return e.co[1];
    if (e.ipo == IPO_LINEAR) {
        if (fc.keys.size() == 1) return e.co[1];
        const Keyframe& nb = fc.keys[endpoint + dir];
        const float dx = e.co[0] - evaltime;
        float fac = nb.co[0] - e.co[0];
        if (fac == 0.0f) return e.co[1];
        fac = (nb.co[1] - e.co[1]) / fac;
        return e.co[1] - (fac * dx);
    }
    const float* h = dir > 0 ? e.hl : e.hr;
    const float dx = e.co[0] - evaltime;
    float fac = e.co[0] - h[0];
    if (fac == 0.0f) return e.co[1];
    fac = (e.co[1] - h[1]) / fac;
    return e.co[1] - (fac * dx);
}

inline bool is_eqt(float a, float b, float c) { return (a > b) ? ((a - b) <= c) : ((b - a) <= c); }

size_t bezt_binarysearch(const std::vector<Keyframe>& k, float frame, float threshold, bool* exact) {
    *exact = false;
    const size_t n = k.size();
    float f = k[0].co[0];
    if (is_eqt(frame, f, threshold)) { *exact = true; return 0; }
    if (frame < f) return 0;
    f = k[n - 1].co[0];
    if (is_eqt(frame, f, threshold)) { *exact = true; return n - 1; }
    if (frame > f) return n;
    long start = 0, end = (long)n;
    for (size_t loop = 0; loop <= n; ++loop) {
        if (start > end) break;
        const long mid = start + ((end - start) / 2);
        const float midf = k[mid].co[0];
        if (is_eqt(frame, midf, threshold)) { *exact = true; return (size_t)mid; }
        if (frame > midf) start = mid + 1;
        else if (frame < midf) end = mid - 1;
    }
    return (size_t)start;
}

float interpolate(const FCurve& fc, float evaltime) {
    const float eps = 1.e-8f;
    bool exact = false;
    const size_t a = bezt_binarysearch(fc.keys, evaltime, 0.0001f, &exact);
    const Keyframe& bz = fc.keys[a];
    if (exact) return bz.co[1];
    const Keyframe& prev = a > 0 ? fc.keys[a - 1] : bz;
    if (std::fabs(bz.co[0] - evaltime) < eps) return bz.co[1];
    if (evaltime < prev.co[0] || bz.co[0] < evaltime) return 0.0f;
    const float begin = prev.co[1];
    const float change = bz.co[1] - prev.co[1];
    const float duration = bz.co[0] - prev.co[0];
    const float time = evaltime - prev.co[0];
    if (prev.ipo == IPO_CONSTANT || duration == 0) return prev.co[1];
    if (prev.ipo == IPO_LINEAR) return change * time / duration + begin;
    float v1[2] = {prev.co[0], prev.co[1]}, v2[2] = {prev.hr[0], prev.hr[1]};
    float v3[2] = {bz.hl[0], bz.hl[1]}, v4[2] = {bz.co[0], bz.co[1]};
    if (std::fabs(v1[1] - v4[1]) < FLT_EPSILON && std::fabs(v2[1] - v3[1]) < FLT_EPSILON &&
        std::fabs(v3[1] - v4[1]) < FLT_EPSILON)
        return v1[1];
    correct_bezpart(v1, v2, v3, v4);
    float opl[4];
    if (!findzero(evaltime, v1[0], v2[0], v3[0], v4[0], opl)) return 0.0f;
    return berekeny(v1[1], v2[1], v3[1], v4[1], opl[0]);
}

// ---- matrices --------------------------------------------------------------
void mat_mul(const double a[16], const double b[16], double out[16]) {
    double r[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0.0;
            for (int k = 0; k < 4; ++k) s += a[4 * i + k] * b[4 * k + j];
            r[4 * i + j] = s;
        }
    std::memcpy(out, r, sizeof r);
}

// Rotation matrix (row-major R, world = R * local) for Blender Euler orders.
// XYZ uses the expanded form of Blender's eul_to_mat3; other orders compose
// the elementary rotations (first axis of the order applied first).
void euler_to_mat3(const double e[3], const std::string& order, double R[9]) {
    if (order == "XYZ") {
        const double ci = std::cos(e[0]), cj = std::cos(e[1]), ch = std::cos(e[2]);
        const double si = std::sin(e[0]), sj = std::sin(e[1]), sh = std::sin(e[2]);
        const double cc = ci * ch, cs = ci * sh, sc = si * ch, ss = si * sh;
        // Blender mat[col][row]; here R[row*3+col]
        R[0] = cj * ch; R[1] = sj * sc - cs; R[2] = sj * cc + ss;
        R[3] = cj * sh; R[4] = sj * ss + cc; R[5] = sj * cs - sc;
        R[6] = -sj;     R[7] = cj * si;      R[8] = cj * ci;
        return;
    }
    if (order.size() != 3) throw std::runtime_error("unsupported rotation mode: " + order);
    double acc[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (char ax : order) {
        const int i = ax - 'X';
        if (i < 0 || i > 2) throw std::runtime_error("unsupported rotation mode: " + order);
        const double c = std::cos(e[i]), s = std::sin(e[i]);
        double r[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const int a = (i + 1) % 3, b = (i + 2) % 3;
        r[3 * a + a] = c; r[3 * a + b] = -s;
        r[3 * b + a] = s; r[3 * b + b] = c;
        double t[9];
        for (int y = 0; y < 3; ++y)
            for (int x = 0; x < 3; ++x)
                t[3 * y + x] = r[3 * y] * acc[x] + r[3 * y + 1] * acc[3 + x] + r[3 * y + 2] * acc[6 + x];
        std::memcpy(acc, t, sizeof t);
    }
    std::memcpy(R, acc, sizeof acc);
}

void local_matrix(const ObjectDesc& o, double frame, double m[16]) {
    double loc[3], rot[3], scl[3];
    std::memcpy(loc, o.loc, sizeof loc);
    std::memcpy(rot, o.rot, sizeof rot);
    std::memcpy(scl, o.scale, sizeof scl);
    for (const FCurve& fc : o.fcurves) {
        if (fc.keys.empty() || fc.index < 0 || fc.index > 2) continue;
        const double v = eval_fcurve(fc, (float)frame);
        if (fc.data_path == "location") loc[fc.index] = v;
        else if (fc.data_path == "rotation_euler") rot[fc.index] = v;
        else if (fc.data_path == "scale") scl[fc.index] = v;
    }
    double R[9];
    euler_to_mat3(rot, o.rotation_mode, R);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) m[4 * r + c] = R[3 * r + c] * scl[c];
        m[4 * r + 3] = loc[r];
    }
    m[12] = m[13] = m[14] = 0.0;
    m[15] = 1.0;
}

double clamp01d(double x) { return x < 0 ? 0 : (x > 1 ? 1 : x); }

// ---- rigid-body stand-ins (RigidMotion, scene.hpp) --------------------------
// splitmix64 stream per body: state = seed ^ (index * 0xD1B54A32D192ED03).
struct SplitMix {
    uint64_t s;
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double u01() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// Pose at time t (seconds since frame_start): row-major 4x4 object_to_world.
void rigid_matrix(const RigidMotion& r, double t, double m[16]) {
    double travel = 0.0, zr = 0.0;  // weighted flight time, height above rest
    const double trel = t - r.t_spawn;
    const double g = r.gravity;
    if (trel > 0.0) {
        double z = r.p0[2] - r.ground_z - r.rest_height;
        if (z < 0.0) z = 0.0;
        double vz = r.v0[2], tt = trel, fac = 1.0;
        double tau = (vz + std::sqrt(vz * vz + 2.0 * g * z)) / g;
        int k = 0;
        for (;;) {
            if (tt <= tau) {
                zr = z + vz * tt - 0.5 * g * tt * tt;
                travel += fac * tt;
                break;
            }
            travel += fac * tau;
            tt -= tau;
            const double vimp = g * tau - vz;
            vz = r.restitution * vimp;
            z = 0.0;
            fac = fac * r.friction;
            k += 1;
            tau = 2.0 * vz / g;
            if (k > r.max_bounces || vz < r.min_speed) {
                zr = 0.0;
                break;
            }
        }
        if (zr < 0.0) zr = 0.0;
    } else {
        zr = r.p0[2] - r.ground_z - r.rest_height;
    }
    const double th = r.w * travel;
    const double c = std::cos(th), sn = std::sin(th), oc = 1.0 - c;
    const double x = r.axis[0], y = r.axis[1], z = r.axis[2];
    const double R[9] = {c + x * x * oc,     x * y * oc - z * sn, x * z * oc + y * sn,
                         y * x * oc + z * sn, c + y * y * oc,     y * z * oc - x * sn,
                         z * x * oc - y * sn, z * y * oc + x * sn, c + z * z * oc};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[4 * i + j] = R[3 * i + j] * r.scale;
    m[3] = r.p0[0] + r.v0[0] * travel;
    m[7] = r.p0[1] + r.v0[1] * travel;
    m[11] = r.ground_z + r.rest_height + zr;
    m[12] = m[13] = m[14] = 0.0;
    m[15] = 1.0;
}

// Expands one "rigid_bodies" group into `count` mesh objects (draw order per
// body fixed: position xyz, scale, velocity xyz, axis xyz, spin, spawn time).
void expand_rigid_group(const Json& g, const RenderDesc& rd, int n_meshes, std::vector<ObjectDesc>& out) {
    const int count = (int)g["count"].as_num();
    const uint64_t seed = (uint64_t)g.get_num("seed", 0);
    std::vector<int> meshes;
    for (const Json& x : g["meshes"].arr) meshes.push_back((int)x.as_num());
    if (count < 0 || meshes.empty()) throw std::runtime_error("rigid_bodies: bad count or meshes");
    for (int mi : meshes)
        if (mi < 0 || mi >= n_meshes) throw std::runtime_error("rigid_bodies: mesh index out of range");
    double c[3] = {0, 0, 5}, e[3] = {10, 10, 4}, sc[2] = {0.3, 0.6};
    if (g.has("spawn_center")) vec3(g["spawn_center"], c);
    if (g.has("spawn_extent")) vec3(g["spawn_extent"], e);
    if (g.has("scale")) {
        sc[0] = g["scale"][0].as_num();
        sc[1] = g["scale"][1].as_num();
    }
    const double speed = g.get_num("speed", 1.0), vup = g.get_num("up_speed", 1.0), spin = g.get_num("spin", 2.0);
    double win[2] = {(double)rd.frame_start, (double)rd.frame_start};
    if (g.has("spawn_window")) {
        win[0] = g["spawn_window"][0].as_num();
        win[1] = g["spawn_window"][1].as_num();
    }
    const std::string prefix = g.get_str("name", "body");
    for (int i = 0; i < count; ++i) {
        SplitMix rng{seed ^ ((uint64_t)i * 0xD1B54A32D192ED03ull)};
        ObjectDesc o;
        o.name = prefix + "." + std::to_string(i);
        o.type = OBJ_MESH;
        o.mesh = meshes[(size_t)i % meshes.size()];
        RigidMotion& r = o.motion;
        r.on = 1;
        for (int k = 0; k < 3; ++k) r.p0[k] = c[k] + (rng.u01() - 0.5) * e[k];
        r.scale = sc[0] + rng.u01() * (sc[1] - sc[0]);
        r.v0[0] = (rng.u01() - 0.5) * 2.0 * speed;
        r.v0[1] = (rng.u01() - 0.5) * 2.0 * speed;
        r.v0[2] = rng.u01() * vup;
        double a[3];
        for (int k = 0; k < 3; ++k) a[k] = rng.u01() * 2.0 - 1.0;
        double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        if (l < 1e-6) {
            a[0] = 0.0; a[1] = 0.0; a[2] = 1.0; l = 1.0;
        }
        for (int k = 0; k < 3; ++k) r.axis[k] = a[k] / l;
        r.w = spin * (0.5 + rng.u01());
        const double f = win[0] + rng.u01() * (win[1] - win[0]);
        r.t_spawn = (f - rd.frame_start) / rd.fps;
        r.gravity = g.get_num("gravity", 9.81);
        r.restitution = g.get_num("restitution", 0.5);
        r.friction = g.get_num("friction", 0.7);
        r.ground_z = g.get_num("ground_z", 0.0);
        r.rest_height = r.scale * g.get_num("mesh_half_height", 1.0);
        r.min_speed = g.get_num("min_speed", 0.05);
        r.max_bounces = (int)g.get_num("max_bounces", 8);
        for (int k = 0; k < 3; ++k) {
            o.loc[k] = r.p0[k];
            o.scale[k] = r.scale;
        }
        out.push_back(std::move(o));
    }
}

}  // namespace

float eval_fcurve(const FCurve& fc, float evaltime) {
    if (fc.keys.empty()) return 0.0f;
    if (evaltime <= fc.keys.front().co[0]) return extrapolate(fc, evaltime, 0, +1);
    if (fc.keys.back().co[0] <= evaltime) return extrapolate(fc, evaltime, (int)fc.keys.size() - 1, -1);
    return interpolate(fc, evaltime);
}

void object_matrix(const SceneDesc& s, int obj, double frame, double m[16]) {
    if (obj < 0 || obj >= (int)s.objects.size()) throw std::runtime_error("object index out of range");
    const ObjectDesc& o = s.objects[obj];
    if (o.motion.on) {
        rigid_matrix(o.motion, (frame - s.render.frame_start) / s.render.fps, m);
    } else if (o.baked_frames > 0) {
        long f = (long)std::floor(frame) - o.baked_start;
        if (f < 0) f = 0;
        if (f >= o.baked_frames) f = o.baked_frames - 1;
        const float* b = &o.baked[(size_t)f * 12];
        for (int i = 0; i < 12; ++i) m[i] = b[i];
        m[12] = m[13] = m[14] = 0.0;
        m[15] = 1.0;
    } else {
        local_matrix(o, frame, m);
    }
    int guard = 0;
    for (int p = o.parent; p >= 0; p = s.objects[p].parent) {
        if (++guard > 64) throw std::runtime_error("parent cycle");
        double pm[16];
        const ObjectDesc& po = s.objects[p];
        if (po.baked_frames > 0 || po.motion.on) {
            double tmp[16];
            object_matrix(s, p, frame, tmp);
            mat_mul(tmp, m, m);
            break;
        }
        local_matrix(po, frame, pm);
        mat_mul(pm, m, m);
    }
}

void build_filter_table(float width, float* table) {
    // Blackman-Harris importance-sampling table (Cycles doubles the BH width:
    // support [-width, width] pixels). Inverse CDF tabulated at
    // u = i / (N - 1); integration by the midpoint rule on 16*N cells.
    const int N = kFilterTableSize;
    const int M = 16 * N;
    const double w = 2.0 * (double)width;
    std::vector<double> cdf(M + 1, 0.0);
    for (int i = 0; i < M; ++i) {
        const double x = ((double)i + 0.5) / M;  // in [0,1] across the support
        const double v = 2.0 * M_PI * x;
        const double f = 0.35875 - 0.48829 * std::cos(v) + 0.14128 * std::cos(2.0 * v) - 0.01168 * std::cos(3.0 * v);
        cdf[i + 1] = cdf[i] + (f > 0.0 ? f : 0.0);
    }
    for (int i = 0; i <= M; ++i) cdf[i] /= cdf[M];
    int j = 0;
    for (int i = 0; i < N; ++i) {
        const double u = (double)i / (N - 1);
        while (j < M - 1 && cdf[j + 1] < u) ++j;
        const double d = cdf[j + 1] - cdf[j];
        const double frac = d > 0.0 ? (u - cdf[j]) / d : 0.0;
        const double x = ((double)j + clamp01d(frac)) / M;
        table[i] = (float)(w * (x - 0.5));
    }
}

void build_srgb_lut(float* lut) {
    for (int i = 0; i <= kSrgbLutSize; ++i)
        lut[i] = (float)(1.055 * std::pow((double)i / kSrgbLutSize, 1.0 / 2.4) - 0.055);
}

SceneDesc load_scene(const std::string& path) {
    SceneDesc s;
    s.path = path;
    Json j = JsonParser(read_file(path)).parse();
    if (j.get_str("format", "") != "rrscene") throw std::runtime_error("not an rrscene file: " + path);
    if ((int)j.get_num("version", 0) != 1) throw std::runtime_error("unsupported rrscene version");
    s.name = j.get_str("name", "");
    if (j.has("render")) {
        const Json& r = j["render"];
        RenderDesc& d = s.render;
        d.resx = (int)r.get_num("resolution_x", d.resx);
        d.resy = (int)r.get_num("resolution_y", d.resy);
        d.percent = (int)r.get_num("resolution_percentage", d.percent);
        d.fps = r.get_num("fps", d.fps);
        d.frame_start = (int)r.get_num("frame_start", d.frame_start);
        d.frame_end = (int)r.get_num("frame_end", d.frame_end);
        d.samples = (int)r.get_num("samples", d.samples);
        d.max_bounces = (int)r.get_num("max_bounces", d.max_bounces);
        d.max_diffuse_bounces = (int)r.get_num("max_diffuse_bounces", d.max_diffuse_bounces);
        d.max_glossy_bounces = (int)r.get_num("max_glossy_bounces", d.max_glossy_bounces);
        d.clamp_indirect = r.get_num("clamp_indirect", d.clamp_indirect);
        d.filter_width = r.get_num("filter_width", d.filter_width);
        d.exposure = r.get_num("exposure", d.exposure);
        d.seed = (uint32_t)r.get_num("seed", d.seed);
        d.spp_per_chunk = (int)r.get_num("spp_per_chunk", 0);
        d.view_transform_name = r.get_str("view_transform", "Standard");
        // "Filmic" is applied through Blender's OCIO LUTs when the context has
        // them (rr_set_ocio_config); otherwise the frame falls back to Standard
        // and says so (rr_frame_stats.view_transform_substituted). Any other
        // Blender 3.6 view ("Filmic Log", "False Color", "Standard" looks, ...)
        // renders as Standard with the same flag and a warning naming it, as
        // does a look or a display gamma the renderer does not apply: the job
        // still renders, and the substitution is never silent.
        if (d.view_transform_name == "Standard") d.view_transform = VIEW_STANDARD;
        else if (d.view_transform_name == "Raw") d.view_transform = VIEW_RAW;
        else if (d.view_transform_name == "Filmic") d.view_transform = VIEW_FILMIC;
        else {
            d.view_transform = VIEW_STANDARD;
            d.view_note = "view transform '" + d.view_transform_name + "' is not supported, rendered as Standard";
        }
        const std::string look = r.get_str("look", "None");
        auto note = [&](const std::string& m) { d.view_note += (d.view_note.empty() ? "" : "; ") + m; };
        if (look != "None" && !look.empty()) note("look '" + look + "' ignored");
        const double gamma = r.get_num("gamma", 1.0);
        if (gamma != 1.0) note("display gamma " + std::to_string(gamma) + " ignored");
    }
    if (s.render.resx <= 0 || s.render.resy <= 0 || s.render.percent <= 0)
        throw std::runtime_error("invalid resolution");
    if (j.has("world")) {
        vec3(j["world"]["color"], s.world_color);
        s.world_strength = j["world"].get_num("strength", 1.0);
    }
    if (j.has("materials"))
        for (const Json& jm : j["materials"].arr) {
            MaterialDesc m;
            m.name = jm.get_str("name", "");
            if (jm.has("base_color")) vec3(jm["base_color"], m.base);
            m.metallic = jm.get_num("metallic", m.metallic);
            m.specular = jm.get_num("specular", m.specular);
            m.roughness = jm.get_num("roughness", m.roughness);
            m.ior = jm.get_num("ior", m.ior);
            if (jm.has("emission")) vec3(jm["emission"], m.emission);
            m.emission_strength = jm.get_num("emission_strength", m.emission_strength);
            const std::string model = jm.get_str("model", "principled");
            if (model == "lambert") m.model = 1;
            else if (model != "principled") throw std::runtime_error("unknown material model: " + model);
            s.materials.push_back(m);
        }
    const int default_mat = (int)s.materials.size();
    s.materials.push_back(MaterialDesc{});  // fallback for empty slots (Cycles default surface)
    s.materials.back().name = "__default__";
    if (j.has("meshes"))
        for (const Json& jm : j["meshes"].arr) {
            s.meshes.emplace_back();
            parse_mesh(jm, s.meshes.back());
        }
    const std::string dir = dirname_of(path);
    if (!j.has("objects")) throw std::runtime_error("scene has no objects");
    for (const Json& jo : j["objects"].arr) {
        ObjectDesc o;
        o.name = jo.get_str("name", "");
        const std::string t = jo.get_str("type", "EMPTY");
        o.type = t == "MESH" ? OBJ_MESH : t == "CAMERA" ? OBJ_CAMERA : t == "LIGHT" ? OBJ_LIGHT : OBJ_EMPTY;
        if (jo.has("location")) vec3(jo["location"], o.loc);
        if (jo.has("rotation_euler")) vec3(jo["rotation_euler"], o.rot);
        if (jo.has("scale")) vec3(jo["scale"], o.scale);
        o.rotation_mode = jo.get_str("rotation_mode", "XYZ");
        o.parent = (int)jo.get_num("parent", -1);
        if (o.type == OBJ_MESH) {
            o.mesh = (int)jo["mesh"].as_num();
            if (o.mesh < 0 || o.mesh >= (int)s.meshes.size()) throw std::runtime_error("object mesh index out of range");
        }
        if (o.type == OBJ_CAMERA && jo.has("camera")) {
            const Json& c = jo["camera"];
            if (c.get_str("type", "PERSP") != "PERSP")
                throw std::runtime_error("only perspective cameras are supported");
            o.camera.lens = c.get_num("lens", 50.0);
            o.camera.sensor_w = c.get_num("sensor_width", 36.0);
            o.camera.sensor_h = c.get_num("sensor_height", 24.0);
            const std::string fit = c.get_str("sensor_fit", "AUTO");
            o.camera.fit = fit == "HORIZONTAL" ? FIT_HORIZONTAL : fit == "VERTICAL" ? FIT_VERTICAL : FIT_AUTO;
            o.camera.clip_start = c.get_num("clip_start", 0.1);
            o.camera.clip_end = c.get_num("clip_end", 100.0);
        }
        if (o.type == OBJ_LIGHT && jo.has("light")) {
            const Json& l = jo["light"];
            const std::string lt = l.get_str("type", "POINT");
            if (lt == "POINT") o.light.type = LIGHT_POINT;
            else if (lt == "SUN") o.light.type = LIGHT_SUN;
            else throw std::runtime_error("unsupported light type: " + lt);
            o.light.energy = l.get_num("energy", 1000.0);
            if (l.has("color")) vec3(l["color"], o.light.color);
            o.light.radius = l.get_num("radius", 0.0);
        }
        if (jo.has("animation") && jo["animation"].has("fcurves")) {
            for (const Json& jf : jo["animation"]["fcurves"].arr) {
                FCurve fc;
                fc.data_path = jf.get_str("data_path", "");
                fc.index = (int)jf.get_num("index", 0);
                fc.extrapolation = jf.get_str("extrapolation", "CONSTANT") == "LINEAR" ? 1 : 0;
                for (const Json& jk : jf["keyframes"].arr) {
                    Keyframe k;
                    for (int i = 0; i < 2; ++i) {
                        k.co[i] = (float)jk["co"][i].as_num();
                        k.hl[i] = (float)jk["handle_left"][i].as_num();
                        k.hr[i] = (float)jk["handle_right"][i].as_num();
                    }
                    k.ipo = ipo_of(jk.get_str("interpolation", "BEZIER"));
                    fc.keys.push_back(k);
                }
                if (!fc.keys.empty()) s.animated = true;
                o.fcurves.push_back(fc);
            }
        }
        if (jo.has("baked")) {
            const Json& b = jo["baked"];
            o.baked_start = (int)b.get_num("frame_start", 1);
            if (b.has("file")) {
                std::string f = b["file"].as_str();
                if (!f.empty() && f[0] != '/') f = dir + "/" + f;
                std::ifstream in(f, std::ios::binary);
                if (!in) throw std::runtime_error("cannot open baked transform file: " + f);
                const long offset = (long)b.get_num("offset_floats", 0);
                const long stride = (long)b.get_num("stride_floats", 12);
                o.baked_frames = (int)b["frames"].as_num();
                o.baked.resize((size_t)o.baked_frames * 12);
                for (int k = 0; k < o.baked_frames; ++k) {
                    in.seekg((std::streamoff)((offset + (long)k * stride) * 4));
                    in.read(reinterpret_cast<char*>(&o.baked[(size_t)k * 12]), 48);
                    if (!in) throw std::runtime_error("baked transform file too short: " + f);
                }
            } else {
                const Json& fr = b["matrices"];
                o.baked_frames = (int)fr.size();
                for (const Json& row : fr.arr)
                    for (int i = 0; i < 12; ++i) o.baked.push_back((float)row[i].as_num());
            }
            if (o.baked_frames > 1) s.animated = true;
        }
        s.objects.push_back(o);
    }
    if (j.has("rigid_bodies"))
        for (const Json& g : j["rigid_bodies"].arr) {
            expand_rigid_group(g, s.render, (int)s.meshes.size(), s.objects);
            s.animated = true;
        }
    for (size_t i = 0; i < s.objects.size(); ++i) {
        const int p = s.objects[i].parent;
        if (p >= (int)s.objects.size() || p == (int)i) throw std::runtime_error("bad parent index");
    }
    s.camera = (int)j.get_num("camera", -1);
    if (s.camera < 0)
        for (size_t i = 0; i < s.objects.size(); ++i)
            if (s.objects[i].type == OBJ_CAMERA) { s.camera = (int)i; break; }
    if (s.camera < 0 || s.camera >= (int)s.objects.size() || s.objects[s.camera].type != OBJ_CAMERA)
        throw std::runtime_error("scene has no camera");
    // flatten triangles
    for (size_t oi = 0; oi < s.objects.size(); ++oi) {
        const ObjectDesc& o = s.objects[oi];
        if (o.type != OBJ_MESH) continue;
        const MeshDesc& m = s.meshes[o.mesh];
        const size_t nt = m.tris.size() / 3;
        for (size_t t = 0; t < nt; ++t) {
            for (int k = 0; k < 3; ++k) {
                const uint32_t vi = m.tris[3 * t + k];
                s.tri_local.push_back(m.verts[3 * vi]);
                s.tri_local.push_back(m.verts[3 * vi + 1]);
                s.tri_local.push_back(m.verts[3 * vi + 2]);
                s.tri_local.push_back(0.0f);
            }
            s.tri_obj.push_back((int32_t)oi);
            const int slot = m.mat_idx[t];
            int g = (slot >= 0 && slot < (int)m.slots.size()) ? m.slots[slot] : -1;
            if (m.slots.empty() && slot >= 0 && slot < default_mat) g = -1;
            s.tri_mat.push_back(g >= 0 && g < default_mat ? g : default_mat);
        }
    }
    if (s.tri_obj.size() > (size_t)0x0fffffff) throw std::runtime_error("too many triangles (max 2^28 - 1: leaf refs)");
    return s;
}

namespace {
// Cycles fresnel_dielectric_cos (bsdf_util.h), in double for the tables.
double fresnel_dielectric_d(double cosi, double eta) {
    const double c = std::fabs(cosi);
    double g = eta * eta - 1.0 + c * c;
    if (g > 0.0) {
        g = std::sqrt(g);
        const double A = (g - c) / (g + c);
        const double B = (c * (g + c) - 1.0) / (c * (g - c) + 1.0);
        return 0.5 * A * A * (1.0 + B * B);
    }
    return 1.0;
}
double clamp01(double x) { return x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x); }
}  // namespace

void build_material_lut(const float* m, float* out) {
    const int N = kMatLutIntervals;
    const double spec = m[4], met = m[3];
    const double b[3] = {m[0], m[1], m[2]};
    const int model = (int)m[10];
    const bool spec_on = m[4] > 1.0e-5f || m[3] > 1.0e-5f;
    // Cycles principled closure setup: ior = 2 / (1 - sqrt(0.08 specular)) - 1,
    // cspec0 = 0.08 specular (1 - metallic) + base metallic (specular tint 0)
    const double eta = 2.0 / (1.0 - std::sqrt(0.08 * spec)) - 1.0;
    const double f0 = fresnel_dielectric_d(1.0, eta);
    double c0[3];
    for (int k = 0; k < 3; ++k) c0[k] = clamp01(spec * 0.08 * (1.0 - met) + b[k] * met);
    const double wd = (1.0 - met) * ((b[0] + b[1] + b[2]) / 3.0);
    for (int i = 0; i <= N; ++i) {
        const double c = (double)i / N;  // cos of the half angle
        out[i] = (float)((fresnel_dielectric_d(c, eta) - f0) / (1.0 - f0));
    }
    for (int i = 0; i <= N; ++i) {
        const double c = (double)i / N;  // cos of the view angle
        const double fh = (fresnel_dielectric_d(c, eta) - f0) / (1.0 - f0);
        const double wsp = ((c0[0] * (1.0 - fh) + fh) + (c0[1] * (1.0 - fh) + fh) + (c0[2] * (1.0 - fh) + fh)) / 3.0;
        double ps = 0.0;
        if (model != 1 && spec_on) ps = wsp + wd > 0.0 ? wsp / (wsp + wd) : 1.0;
        out[kMatLutPsOffset + i] = (float)ps;
    }
    // each channel's last entry repeated once: the device reads the tables with
    // a branch-free lerp that touches t[i + 1] also at u = 1 (rr_device.h lut_at)
    out[N + 1] = out[N];
    out[kMatLutPsOffset + N + 1] = out[kMatLutPsOffset + N];
}

FrameSetup setup_frame(const SceneDesc& s, int frame, const rr_render_params* p) {
    rr_render_params d;
    rr_render_params_default(&d);
    if (!p) p = &d;
    FrameSetup f;
    const RenderDesc& r = s.render;
    f.W = p->width > 0 ? p->width : (r.resx * r.percent) / 100;
    f.H = p->height > 0 ? p->height : (r.resy * r.percent) / 100;
    if (f.W <= 0 || f.H <= 0 || (int64_t)f.W * f.H > (int64_t)1 << 28)
        throw std::runtime_error("invalid output resolution");
    f.spp = p->spp > 0 ? p->spp : r.samples;
    if (f.spp <= 0) f.spp = 1;
    // Bounce caps as Cycles applies them (path_state_next): a scatter that
    // takes a counter to its cap ends the path at the next hit. The camera hit
    // always scatters, so a cap of 0 ("direct light only") acts as a cap of 1.
    f.max_bounces = p->max_bounces >= 0 ? p->max_bounces : r.max_bounces;
    if (f.max_bounces > 64) f.max_bounces = 64;
    if (f.max_bounces < 1) f.max_bounces = 1;
    f.max_diffuse = p->max_diffuse_bounces >= 0 ? p->max_diffuse_bounces : r.max_diffuse_bounces;
    f.max_glossy = p->max_glossy_bounces >= 0 ? p->max_glossy_bounces : r.max_glossy_bounces;
    f.max_diffuse = std::min(std::max(f.max_diffuse, 1), 0xffff);
    f.max_glossy = std::min(std::max(f.max_glossy, 1), 0xffff);
    f.clamp_indirect = (float)(p->clamp_indirect >= 0.f ? p->clamp_indirect : r.clamp_indirect);
    f.seed = p->use_scene_seed ? r.seed : p->seed;
    f.view_transform = p->view_transform >= 0 ? p->view_transform : r.view_transform;
    if (p->view_transform < 0) f.view_note = r.view_note;
    if (f.view_transform != VIEW_STANDARD && f.view_transform != VIEW_RAW && f.view_transform != VIEW_FILMIC)
        throw std::runtime_error("unsupported view transform");
    f.spp_per_chunk = p->spp_per_chunk > 0 ? p->spp_per_chunk : r.spp_per_chunk;
    f.flags = p->flags;
    f.filter_width = (float)r.filter_width;
    f.exposure_scale = (float)std::pow(2.0, r.exposure);

    // camera
    double m[16];
    object_matrix(s, s.camera, frame, m);
    const CameraDesc& c = s.objects[s.camera].camera;
    double axes[3][3];
    for (int a = 0; a < 3; ++a) {
        const double x = m[a], y = m[4 + a], z = m[8 + a];
        const double l = std::sqrt(x * x + y * y + z * z);
        axes[a][0] = x / l; axes[a][1] = y / l; axes[a][2] = z / l;
    }
    int fit = c.fit;
    if (fit == FIT_AUTO) fit = f.W >= f.H ? FIT_HORIZONTAL : FIT_VERTICAL;
    const double sensor = (c.fit == FIT_VERTICAL) ? c.sensor_h : c.sensor_w;
    double half_w, half_h;
    if (fit == FIT_HORIZONTAL) {
        half_w = 0.5 * sensor / c.lens;
        half_h = half_w * (double)f.H / (double)f.W;
    } else {
        half_h = 0.5 * sensor / c.lens;
        half_w = half_h * (double)f.W / (double)f.H;
    }
    f.cam[0] = (float)m[3]; f.cam[1] = (float)m[7]; f.cam[2] = (float)m[11];
    for (int a = 0; a < 3; ++a)
        for (int k = 0; k < 3; ++k) f.cam[3 + 3 * a + k] = (float)axes[a][k];
    f.cam[12] = (float)half_w;
    f.cam[13] = (float)half_h;
    f.cam[14] = (float)c.clip_start;
    f.cam[15] = (float)c.clip_end;

    // lights
    for (size_t i = 0; i < s.objects.size(); ++i) {
        const ObjectDesc& o = s.objects[i];
        if (o.type != OBJ_LIGHT) continue;
        object_matrix(s, (int)i, frame, m);
        float L[RR_LIGHT_FLOATS] = {};
        L[0] = (float)o.light.type;
        L[1] = (float)m[3]; L[2] = (float)m[7]; L[3] = (float)m[11];
        // light's -Z axis = emission direction (sun)
        double dz[3] = {-m[2], -m[6], -m[10]};
        const double l = std::sqrt(dz[0] * dz[0] + dz[1] * dz[1] + dz[2] * dz[2]);
        for (int k = 0; k < 3; ++k) L[4 + k] = (float)(dz[k] / l);
        L[7] = (float)(o.light.type == LIGHT_POINT ? o.light.radius : 0.0);
        // point: radiant intensity P/(4*pi) W/sr (Cycles eval_fac = 1/(4 pi) * invarea
        // over a disk of area pi r^2); sun: irradiance = strength.
        const double k = o.light.type == LIGHT_POINT ? o.light.energy / (4.0 * M_PI) : o.light.energy;
        for (int c3 = 0; c3 < 3; ++c3) L[8 + c3] = (float)(k * o.light.color[c3]);
        f.lights.insert(f.lights.end(), L, L + RR_LIGHT_FLOATS);
    }
    if (f.lights.size() / RR_LIGHT_FLOATS > 64) throw std::runtime_error("more than 64 lights");
    // materials
    for (const MaterialDesc& md : s.materials) {
        float M[RR_MAT_FLOATS] = {};
        for (int k = 0; k < 3; ++k) M[k] = (float)md.base[k];
        M[3] = (float)md.metallic;
        M[4] = (float)md.specular;
        M[5] = (float)md.roughness;
        M[6] = (float)md.ior;
        for (int k = 0; k < 3; ++k) M[7 + k] = (float)(md.emission[k] * md.emission_strength);
        M[10] = (float)md.model;
        f.materials.insert(f.materials.end(), M, M + RR_MAT_FLOATS);
        float lut[kMatLutFloatsPerMat];
        build_material_lut(M, lut);
        f.mat_lut.insert(f.mat_lut.end(), lut, lut + kMatLutFloatsPerMat);
    }
    for (int k = 0; k < 3; ++k) f.world[k] = (float)(s.world_color[k] * s.world_strength);
    // object transforms (row-major 3x4, float)
    f.obj_xform.resize(s.objects.size() * 12);
    for (size_t i = 0; i < s.objects.size(); ++i) {
        object_matrix(s, (int)i, frame, m);
        for (int k = 0; k < 12; ++k) f.obj_xform[i * 12 + k] = (float)m[k];
    }
    return f;
}

}  // namespace rr
