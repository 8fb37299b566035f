// Filmic view transform (RR_VIEW_FILMIC) through the OCIO LUTs of a Blender
// colour-management directory ("View transforms").
//
// The reference renders 01_simple-animation with Blender 3.6's "Filmic" view
// (the .blend's view settings), which Blender applies through
// OpenColorIO with its bundled config (datafiles/colormanagement/config.ocio,
// third-party, not in the reference tree). For display "sRGB", view "Filmic",
// look "None" that config's chain is, per channel unless noted:
//   1. AllocationTransform lg2 [-12.473931188, 12.526068812]:
//        a = (log2(max(x, FLT_MIN)) + 12.473931188) / 25
//   2. FileTransform filmic_desat65cube.spi3d, interpolation best
//        (tetrahedral, RGB -> RGB, input clamped to the cube)
//   3. AllocationTransform uniform [0, 0.66]:  c = b / 0.66
//   4. FileTransform filmic_to_0-70_1-03.spi1d, interpolation linear
//        (display-referred sRGB code values)
// The constants are restated from that config (not present here); Blender's
// LUT files are not in the image either, so the chain is tested bit-exact
// against the oracle on synthetic LUTs written in the same formats, and its
// parity with Blender's own Filmic output stays unpinned.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "device.hpp"

namespace rr {

// LUTs as parsed from the files (host).
struct FilmicLuts {
    int n3 = 0;                // cube edge
    std::vector<float> cube;   // n3^3 x (r, g, b); entry (i, j, k) at (i * n3 + j) * n3 + k
    int n1 = 0, comps = 1;     // 1D LUT length, components (1: one curve for every channel)
    std::vector<float> lut1;   // n1 x comps
    float lo1 = 0.f, hi1 = 1.f;  // 1D LUT input domain ("From")
};

// Parse an OCIO .spi3d / .spi1d file. false + err on failure.
bool parse_spi3d(const std::string& path, FilmicLuts& out, std::string& err);
bool parse_spi1d(const std::string& path, FilmicLuts& out, std::string& err);

// Find and parse Blender's two Filmic LUTs under `dir` (dir/luts/ or dir/).
bool load_filmic_luts(const std::string& dir, FilmicLuts& out, std::string& err);

// The LUTs on one device.
struct FilmicDev {
    DevBuf<float4> cube;  // n3^3, (r, g, b, 0)
    DevBuf<float> lut1;
    int n3 = 0, n1 = 0, comps = 1;
    float lo1 = 0.f, hi1 = 1.f;
    bool ready = false;
    std::string dir;
    void upload(const FilmicLuts& l, const std::string& from);
    void release();
};

// rgba8 = Filmic(film sums * inv_spp * exposure_scale) for every pixel.
void view_filmic_device(const FilmicDev& f, const FrameConsts& fc, const float4* film, uchar4* out,
                        hipStream_t st);

}  // namespace rr
