// Scene model of the .rrscene format and the host-side per-frame
// evaluation (animation -> object matrices -> camera / lights / materials).
//
// Stands in for what Blender does between `.blend` load and the start of the
// Cycles render in the reference: scene.frame_set(N)
// (/root/reference/scripts/render-timing-script.py:81) evaluates F-Curves and
// object transforms; Cycles' scene sync then converts camera, lights and
// materials. Parity anchors: the F-Curve golden table of SURVEY.md §8c (01 cube
// z) and the oracle restatement oracle/host_oracle.py.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rr.h"

namespace rr {

enum ObjType { OBJ_EMPTY = 0, OBJ_MESH = 1, OBJ_CAMERA = 2, OBJ_LIGHT = 3 };
enum LightType { LIGHT_POINT = 0, LIGHT_SUN = 1 };
enum Ipo { IPO_CONSTANT = 0, IPO_LINEAR = 1, IPO_BEZIER = 2 };
enum SensorFit { FIT_AUTO = 0, FIT_HORIZONTAL = 1, FIT_VERTICAL = 2 };
enum ViewTransform { VIEW_STANDARD = 0, VIEW_RAW = 1, VIEW_FILMIC = 2 };

// Blender stores BezTriple coordinates as float; evaluation happens in float
// (with double inside the cubic solver), see eval_fcurve().
struct Keyframe {
    float co[2], hl[2], hr[2];
    int ipo;
};

struct FCurve {
    std::string data_path;  // "location" | "rotation_euler" | "scale"
    int index = 0;
    int extrapolation = 0;  // 0 constant, 1 linear
    std::vector<Keyframe> keys;
};

struct CameraDesc {
    double lens = 50.0, sensor_w = 36.0, sensor_h = 24.0;
    int fit = FIT_AUTO;
    double clip_start = 0.1, clip_end = 100.0;
};

struct LightDesc {
    int type = LIGHT_POINT;
    double energy = 1000.0;
    double color[3] = {1, 1, 1};
    double radius = 0.0;
};

// Closed-form rigid-body motion of the physics stand-ins (SURVEY.md §8d C4/C5:
// the 02/03 .blend files and their simulation caches are missing from the
// reference, .MISSING_LARGE_BLOBS). A body hangs at p0 until t_spawn, then
// flies ballistically (gravity g) and bounces on the ground plane z = ground_z
// with restitution e; every bounce scales its horizontal and angular travel
// rate by `friction`; it rests after max_bounces or below min_speed. The pose
// is a pure function of the frame, so frames stay independent. Expanded from
// a scene's "rigid_bodies" groups at load; restated in oracle/host_oracle.py.
struct RigidMotion {
    int on = 0;
    double p0[3] = {0, 0, 0}, v0[3] = {0, 0, 0}, axis[3] = {0, 0, 1};
    double w = 0.0, scale = 1.0, t_spawn = 0.0;
    double gravity = 9.81, restitution = 0.5, friction = 0.7, ground_z = 0.0, rest_height = 1.0;
    double min_speed = 0.05;
    int max_bounces = 8;
};

struct ObjectDesc {
    std::string name;
    int type = OBJ_EMPTY;
    double loc[3] = {0, 0, 0}, rot[3] = {0, 0, 0}, scale[3] = {1, 1, 1};
    std::string rotation_mode = "XYZ";
    int parent = -1;
    int mesh = -1;
    CameraDesc camera;
    LightDesc light;
    std::vector<FCurve> fcurves;
    // Baked rigid transforms (stand-ins for simulation caches): frames x 12
    // floats (3x4 row-major object_to_world); frame f uses row f - baked_start,
    // clamped to the baked range.
    int baked_start = 0;
    int baked_frames = 0;
    std::vector<float> baked;
    RigidMotion motion;
};

struct MeshDesc {
    std::string name;
    std::vector<float> verts;      // xyz per vertex
    std::vector<uint32_t> tris;    // 3 per triangle
    std::vector<int> mat_idx;      // slot index per triangle
    std::vector<int> slots;        // slot -> global material
};

struct MaterialDesc {
    std::string name;
    double base[3] = {0.8, 0.8, 0.8};
    double metallic = 0.0, specular = 0.5, roughness = 0.5, ior = 1.45;
    double emission[3] = {0, 0, 0};
    double emission_strength = 1.0;
    int model = 0;  // 0 Principled subset, 1 pure Lambert (analytic test scenes)
};

struct RenderDesc {
    int resx = 1920, resy = 1080, percent = 100;
    double fps = 24;
    int frame_start = 1, frame_end = 250;
    // Cycles 3.6 defaults (scene.cycles): max_bounces 12, diffuse 4, glossy 4
    int samples = 128, max_bounces = 12, max_diffuse_bounces = 4, max_glossy_bounces = 4;
    double clamp_indirect = 10.0, filter_width = 1.5, exposure = 0.0;
    int view_transform = VIEW_STANDARD;
    std::string view_transform_name = "Standard";
    // What of the scene's colour management a frame does not apply, for the
    // frame's warning ("" when all of it is applied): a view transform other
    // than Standard / Raw / Filmic (rendered as Standard), a look other than
    // None, a display gamma other than 1 (both ignored).
    std::string view_note;
    uint32_t seed = 0;
    int spp_per_chunk = 0;
};

struct SceneDesc {
    std::string name, path;
    RenderDesc render;
    double world_color[3] = {0.05, 0.05, 0.05};
    double world_strength = 1.0;
    std::vector<MaterialDesc> materials;
    std::vector<MeshDesc> meshes;
    std::vector<ObjectDesc> objects;
    int camera = -1;
    // Flattened triangle soup in object-local space (built at load).
    std::vector<float> tri_local;  // n * 12 : v0.xyzw v1.xyzw v2.xyzw (w = 0)
    std::vector<int32_t> tri_obj;  // object index per triangle
    std::vector<int32_t> tri_mat;  // global material per triangle
    bool animated = false;         // any object transform depends on the frame
};

// Everything the device needs for one frame (DESIGN.md §4 "frame constants").
struct FrameSetup {
    int32_t W = 0, H = 0, spp = 0, max_bounces = 0, view_transform = 0, spp_per_chunk = 0, flags = 0;
    int32_t max_diffuse = 4, max_glossy = 4;
    std::string view_note;  // RenderDesc::view_note when the view comes from the scene
    uint32_t seed = 0;
    float clamp_indirect = 0.f, filter_width = 1.5f, exposure_scale = 1.f;
    float cam[RR_CAM_FLOATS] = {};
    std::vector<float> lights;     // n * RR_LIGHT_FLOATS
    std::vector<float> materials;  // n * RR_MAT_FLOATS
    std::vector<float> mat_lut;    // n * kMatLutFloatsPerMat (build_material_lut)
    float world[3] = {0, 0, 0};
    std::vector<float> obj_xform;  // n_objects * 12 (3x4 row-major, float)
};

SceneDesc load_scene(const std::string& path);  // throws std::runtime_error

// Blender F-Curve evaluation (fcurve_eval_keyframes semantics).
float eval_fcurve(const FCurve& fc, float evaltime);

// object_to_world (row-major 4x4) at `frame`, parents applied.
void object_matrix(const SceneDesc& s, int obj, double frame, double m[16]);

FrameSetup setup_frame(const SceneDesc& s, int frame, const rr_render_params* p);

// Shared tables (identical double-precision construction in oracle/rr_oracle.c).
constexpr int kFilterTableSize = 1024;
constexpr int kSrgbLutSize = 4096;
void build_filter_table(float width, float* table /* kFilterTableSize */);
// Per-material tables of the Principled closures (rr_device.h kMatLutN,
// kMatLutStride): Cycles' Fresnel blend FH against cos of the half angle and
// the specular-lobe pick probability against cos of the view angle, in double
// from the material's RR_MAT_FLOATS floats (oracle/rr_oracle.c builds them the
// same way).
constexpr int kMatLutIntervals = 128;
constexpr int kMatLutFloatsPerMat = 260;
// layout: FH [0, 128] + a repeat of [128] at 129 | ps [130, 258] + a repeat at 259
constexpr int kMatLutPsOffset = 130;
void build_material_lut(const float* mat12, float* out /* kMatLutFloatsPerMat */);
void build_srgb_lut(float* lut /* kSrgbLutSize + 1 */);

}  // namespace rr
