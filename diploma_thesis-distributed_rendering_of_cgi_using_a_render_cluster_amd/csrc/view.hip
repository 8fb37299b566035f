// Filmic view transform: OCIO LUT parsing (host) and the per-pixel chain
// (device). See view.hpp for the chain and where it comes from. The float
// operations are written in the order oracle/rr_oracle.c orc_filmic uses, so
// the 8-bit output is bit-identical to the oracle's (tests/test_gpu_view.py).
#pragma clang fp contract(off)

#include "view.hpp"

#include <fstream>
#include <sstream>

namespace rr {

namespace {

// log2 for normal positive x without libm: x = 2^e m, m in [1, 2) folded
// into [sqrt(1/2), sqrt(2)); log2 m = 2/ln 2 atanh(t), t = (m - 1)/(m + 1),
// by its odd series to t^9 (|t| < 0.172: truncation < 4e-10).
RR_HD float log2_fixed(float x) {
    const int bits = f2i(x);
    int e = ((bits >> 23) & 0xff) - 127;
    float m = i2f((bits & 0x007fffff) | 0x3f800000);
    if (m > 1.41421356f) {
        m = m * 0.5f;
        e = e + 1;
    }
    const float t = (m - 1.0f) / (m + 1.0f);
    const float t2 = t * t;
    const float p = ((((t2 * 0.111111112f + 0.142857149f) * t2 + 0.2f) * t2 + 0.333333343f) * t2 + 1.0f) * t;
    return (float)e + p * 2.88539004f;
}

RR_HD float sat(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

// OCIO Lut1D, linear interpolation over the domain [lo, hi] (clamped).
RR_D float lut1d(const float* __restrict__ t, int n, int comps, int c, float lo, float hi, float x) {
    float f = (x - lo) / (hi - lo) * (float)(n - 1);
    f = fminf(fmaxf(f, 0.0f), (float)(n - 1));
    const int i = (int)f;
    if (i >= n - 1) return t[(n - 1) * comps + c];
    const float fr = f - (float)i;
    const float a = t[i * comps + c], b = t[(i + 1) * comps + c];
    return a + (b - a) * fr;
}

RR_D float3 ld3(const float4* __restrict__ cube, int i) {
    const float4 v = cube[i];
    return make_float3(v.x, v.y, v.z);
}

// OCIO Lut3D tetrahedral interpolation; input clamped to [0, 1].
RR_D float3 lut3d_tetra(const float4* __restrict__ cube, int n, float r, float g, float b) {
    const float s = (float)(n - 1);
    float fr = sat(r) * s, fg = sat(g) * s, fb = sat(b) * s;
    const int ir = min((int)fr, n - 2), ig = min((int)fg, n - 2), ib = min((int)fb, n - 2);
    fr = fr - (float)ir;
    fg = fg - (float)ig;
    fb = fb - (float)ib;
    auto at = [&](int di, int dj, int dk) { return ld3(cube, ((ir + di) * n + (ig + dj)) * n + (ib + dk)); };
    const float3 c000 = at(0, 0, 0), c111 = at(1, 1, 1);
    float3 c1, c2;
    float w0, w1, w2, w3;
    if (fr > fg) {
        if (fg > fb) {  // r > g > b
            c1 = at(1, 0, 0); c2 = at(1, 1, 0);
            w0 = 1.0f - fr; w1 = fr - fg; w2 = fg - fb; w3 = fb;
        } else if (fr > fb) {  // r > b >= g
            c1 = at(1, 0, 0); c2 = at(1, 0, 1);
            w0 = 1.0f - fr; w1 = fr - fb; w2 = fb - fg; w3 = fg;
        } else {  // b >= r > g
            c1 = at(0, 0, 1); c2 = at(1, 0, 1);
            w0 = 1.0f - fb; w1 = fb - fr; w2 = fr - fg; w3 = fg;
        }
    } else {
        if (fb > fg) {  // b > g >= r
            c1 = at(0, 0, 1); c2 = at(0, 1, 1);
            w0 = 1.0f - fb; w1 = fb - fg; w2 = fg - fr; w3 = fr;
        } else if (fb > fr) {  // g >= b > r
            c1 = at(0, 1, 0); c2 = at(0, 1, 1);
            w0 = 1.0f - fg; w1 = fg - fb; w2 = fb - fr; w3 = fr;
        } else {  // g >= r >= b
            c1 = at(0, 1, 0); c2 = at(1, 1, 0);
            w0 = 1.0f - fg; w1 = fg - fr; w2 = fr - fb; w3 = fb;
        }
    }
    return make_float3(((w0 * c000.x + w1 * c1.x) + w2 * c2.x) + w3 * c111.x,
                       ((w0 * c000.y + w1 * c1.y) + w2 * c2.y) + w3 * c111.y,
                       ((w0 * c000.z + w1 * c1.z) + w2 * c2.z) + w3 * c111.z);
}

struct FilmicArgs {
    const float4* cube;
    const float* lut1;
    int n3, n1, comps;
    float lo1, hi1;
};

__global__ __launch_bounds__(256) void k_view_filmic(FrameConsts fc, FilmicArgs f, const float4* __restrict__ film,
                                                     uchar4* __restrict__ out) {
    for (int pix = blockIdx.x * 256 + threadIdx.x; pix < fc.npix; pix += gridDim.x * 256) {
        const float4 acc = film[pix];
        const float c[3] = {acc.x * fc.inv_spp * fc.exposure_scale, acc.y * fc.inv_spp * fc.exposure_scale,
                            acc.z * fc.inv_spp * fc.exposure_scale};
        float a[3];
        for (int k = 0; k < 3; ++k) a[k] = (log2_fixed(fmaxf(c[k], 1.17549435e-38f)) + 12.473931188f) / 25.0f;
        const float3 b = lut3d_tetra(f.cube, f.n3, a[0], a[1], a[2]);
        const float bb[3] = {b.x, b.y, b.z};
        uint8_t q[3];
        for (int k = 0; k < 3; ++k)
            q[k] = quantize8(lut1d(f.lut1, f.n1, f.comps, f.comps == 3 ? k : 0, f.lo1, f.hi1, bb[k] / 0.66f));
        out[pix] = make_uchar4(q[0], q[1], q[2], 255);
    }
}

bool read_lines(const std::string& path, std::vector<std::string>& lines, std::string& err) {
    std::ifstream in(path);
    if (!in) {
        err = "cannot open " + path;
        return false;
    }
    std::string l;
    while (std::getline(in, l)) {
        if (!l.empty() && l.back() == '\r') l.pop_back();
        lines.push_back(l);
    }
    return true;
}

}  // namespace

// OCIO's .spi3d (Sony Pictures Imageworks): "SPILUT 1.0", "3 3", "N N N",
// then one line "i j k r g b" per cube entry (i indexes red).
bool parse_spi3d(const std::string& path, FilmicLuts& out, std::string& err) {
    std::vector<std::string> L;
    if (!read_lines(path, L, err)) return false;
    if (L.size() < 3 || L[0].rfind("SPILUT", 0) != 0) {
        err = path + ": not an SPILUT file";
        return false;
    }
    int na = 0, nb = 0, nc = 0;
    {
        std::istringstream s(L[2]);
        if (!(s >> na >> nb >> nc) || na != nb || na != nc || na < 2 || na > 256) {
            err = path + ": bad cube size line '" + L[2] + "'";
            return false;
        }
    }
    const int n = na;
    out.n3 = n;
    out.cube.assign((size_t)n * n * n * 3, 0.f);
    std::vector<char> seen((size_t)n * n * n, 0);
    size_t count = 0;
    for (size_t li = 3; li < L.size(); ++li) {
        std::istringstream s(L[li]);
        int i, j, k;
        double r, g, b;  // decimal -> double -> float, as the oracle's reader rounds
        if (!(s >> i)) continue;  // blank line
        if (!(s >> j >> k >> r >> g >> b) || i < 0 || j < 0 || k < 0 || i >= n || j >= n || k >= n) {
            err = path + ": bad entry line " + std::to_string(li + 1);
            return false;
        }
        const size_t e = ((size_t)i * n + j) * n + k;
        if (!seen[e]) ++count;
        seen[e] = 1;
        out.cube[3 * e] = (float)r;
        out.cube[3 * e + 1] = (float)g;
        out.cube[3 * e + 2] = (float)b;
    }
    if (count != (size_t)n * n * n) {
        err = path + ": " + std::to_string(count) + " of " + std::to_string((size_t)n * n * n) + " cube entries";
        return false;
    }
    return true;
}

// OCIO's .spi1d: "Version 1", "From lo hi", "Length N", "Components C",
// "{", N lines of C values, "}".
bool parse_spi1d(const std::string& path, FilmicLuts& out, std::string& err) {
    std::vector<std::string> L;
    if (!read_lines(path, L, err)) return false;
    int n = -1, comps = -1;
    double lo = 0.0, hi = 1.0;
    size_t li = 0;
    for (; li < L.size(); ++li) {
        std::istringstream s(L[li]);
        std::string key;
        if (!(s >> key)) continue;
        if (key == "Version") continue;
        if (key == "From") {
            if (!(s >> lo >> hi) || !(hi > lo)) {
                err = path + ": bad From line";
                return false;
            }
        } else if (key == "Length") {
            s >> n;
        } else if (key == "Components") {
            s >> comps;
        } else if (key == "{") {
            ++li;
            break;
        } else {
            err = path + ": unexpected '" + key + "'";
            return false;
        }
    }
    if (n < 2 || n > (1 << 20) || (comps != 1 && comps != 3)) {
        err = path + ": bad Length/Components";
        return false;
    }
    out.n1 = n;
    out.comps = comps;
    out.lo1 = (float)lo;
    out.hi1 = (float)hi;
    out.lut1.clear();
    for (; li < L.size(); ++li) {
        std::istringstream s(L[li]);
        std::string tok;
        while (s >> tok) {
            if (tok == "}") goto done;
            out.lut1.push_back((float)std::stod(tok));
        }
    }
done:
    if (out.lut1.size() != (size_t)n * comps) {
        err = path + ": " + std::to_string(out.lut1.size()) + " values, expected " + std::to_string((size_t)n * comps);
        return false;
    }
    return true;
}

bool load_filmic_luts(const std::string& dir, FilmicLuts& out, std::string& err) {
    const char* names[2] = {"filmic_desat65cube.spi3d", "filmic_to_0-70_1-03.spi1d"};
    std::string paths[2];
    for (int k = 0; k < 2; ++k) {
        for (const std::string& sub : {std::string("/luts/"), std::string("/")}) {
            const std::string p = dir + sub + names[k];
            if (std::ifstream(p)) {
                paths[k] = p;
                break;
            }
        }
        if (paths[k].empty()) {
            err = std::string("no ") + names[k] + " under " + dir + " (or its luts/)";
            return false;
        }
    }
    return parse_spi3d(paths[0], out, err) && parse_spi1d(paths[1], out, err);
}

void FilmicDev::upload(const FilmicLuts& l, const std::string& from) {
    const size_t n3c = (size_t)l.n3 * l.n3 * l.n3;
    std::vector<float4> c(n3c);
    for (size_t i = 0; i < n3c; ++i) c[i] = make_float4(l.cube[3 * i], l.cube[3 * i + 1], l.cube[3 * i + 2], 0.f);
    cube.ensure(n3c);
    lut1.ensure(l.lut1.size());
    RR_HIP(hipMemcpy(cube.ptr, c.data(), n3c * sizeof(float4), hipMemcpyHostToDevice));
    RR_HIP(hipMemcpy(lut1.ptr, l.lut1.data(), l.lut1.size() * sizeof(float), hipMemcpyHostToDevice));
    n3 = l.n3;
    n1 = l.n1;
    comps = l.comps;
    lo1 = l.lo1;
    hi1 = l.hi1;
    dir = from;
    ready = true;
}

void FilmicDev::release() {
    cube.release();
    lut1.release();
    ready = false;
    dir.clear();
}

void view_filmic_device(const FilmicDev& f, const FrameConsts& fc, const float4* film, uchar4* out,
                        hipStream_t st) {
    if (!f.ready) throw std::runtime_error("Filmic view transform without LUTs");
    const FilmicArgs a{f.cube.ptr, f.lut1.ptr, f.n3, f.n1, f.comps, f.lo1, f.hi1};
    const int grid = std::max(1, std::min((fc.npix + 255) / 256, 4096));
    k_view_filmic<<<grid, 256, 0, st>>>(fc, a, film, out);
    RR_HIP(hipGetLastError());
}

}  // namespace rr
