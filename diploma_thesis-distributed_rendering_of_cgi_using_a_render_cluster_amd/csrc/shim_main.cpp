// rr-blender-shim: a drop-in for the `blender` binary the reference worker
// spawns per frame (--blenderBinary, /root/reference/worker/src/cli.rs:6-45).
//
// Accepts the reference argv (worker/src/rendering/runner/mod.rs:140-158):
//   [prepend...] <project> --background --python <script> --
//       --render-output <dir>/<name_fmt> --render-format <FMT> --render-frame <N> [append...]
// renders frame N through the C ABI and prints the stdout protocol that
// extract_blender_render_information parses (utilities.rs:105-203):
//   Saved: '<path>'
//    Time: MM:SS.ff (Saving: MM:SS.ff)
//   RESULTS={"project_loaded_at": ..., "project_started_rendering_at": ...,
//            "project_finished_rendering_at": ...}
// project_finished_rendering_at includes the save, as in render-timing-script.py:92-98.
//
// <project> may be a .rrscene, or a .blend whose export sits next to it as
// <stem>.rrscene. Environment: RR_DEVICE (ordinal, default 0), RR_SPP,
// RR_MAX_BOUNCES, RR_WIDTH, RR_HEIGHT override the scene's render settings.
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rr.h"

namespace {

double unix_now() {
    timeval tv;
    gettimeofday(&tv, nullptr);
    return (double)tv.tv_sec + (double)tv.tv_usec * 1e-6;
}

// render-timing-script.py:69-78: count every '#', replace the run of exactly
// that many '#' with the zero-padded frame number (no truncation).
std::string format_hash_frame_placeholders(const std::string& path, long frame) {
    size_t count = 0;
    for (char ch : path) count += ch == '#';
    std::string num = std::to_string(frame);
    if (num.size() < count) num = std::string(count - num.size(), '0') + num;
    std::string out;
    if (count == 0) {  // Python str.replace("", s): s before every char and at the end
        for (char ch : path) out += num + ch;
        return out + num;
    }
    const std::string run(count, '#');
    size_t pos = 0;
    for (;;) {  // str.replace replaces every non-overlapping occurrence
        size_t k = path.find(run, pos);
        if (k == std::string::npos) break;
        out += path.substr(pos, k - pos) + num;
        pos = k + run.size();
    }
    out += path.substr(pos);
    return out;
}

std::string blender_time(double seconds) {  // "MM:SS.ff"
    if (seconds < 0) seconds = 0;
    long cs = (long)(seconds * 100.0 + 0.5);
    char buf[64];
    std::snprintf(buf, sizeof buf, "%02ld:%02ld.%02ld", cs / 6000, (cs / 100) % 60, cs % 100);
    return buf;
}

int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

}  // namespace

int main(int argc, char** argv) {
    std::vector<std::string> args(argv + 1, argv + argc);
    // project file: first argument naming a .blend or .rrscene before "--"
    std::string project;
    size_t last_dd = std::string::npos;
    for (size_t i = 0; i < args.size(); ++i)
        if (args[i] == "--") last_dd = i;
    for (size_t i = 0; i < args.size() && (last_dd == std::string::npos || i < last_dd); ++i)
        if (ends_with(args[i], ".blend") || ends_with(args[i], ".rrscene")) {
            project = args[i];
            break;
        }
    // script arguments: after the LAST "--" (render-timing-script.py:48-50)
    std::string out_fmt, fmt;
    long frame = 0;
    bool have_out = false, have_fmt = false, have_frame = false;
    if (last_dd != std::string::npos) {
        for (size_t i = last_dd + 1; i < args.size(); ++i) {
            const std::string& a = args[i];
            auto next = [&](std::string& dst, bool& flag) {
                if (i + 1 < args.size()) { dst = args[++i]; flag = true; }
            };
            std::string tmp;
            if (a == "--render-output") next(out_fmt, have_out);
            else if (a == "--render-format") next(fmt, have_fmt);
            else if (a == "--render-frame") {
                bool ok = false;
                next(tmp, ok);
                char* end = nullptr;
                frame = std::strtol(tmp.c_str(), &end, 10);
                if (ok && end && *end == '\0' && !tmp.empty()) have_frame = true;
                else { std::printf("Invalid render-and-timing-script arguments!\n"); return 0; }
            }
        }
    }
    if (!have_out || !have_fmt || !have_frame) {
        std::printf("Missing render-and-timing-script arguments!\n");
        return 0;
    }
    if (project.empty()) {
        std::fprintf(stderr, "rr-blender-shim: no project file on the command line\n");
        return 1;
    }
    std::string scene_path = project;
    if (ends_with(project, ".blend")) scene_path = project.substr(0, project.size() - 6) + ".rrscene";
    std::printf("rr-blender-shim (MI355X renderer, ABI %d)\n", rr_abi_version());
    std::printf("Read scene: \"%s\"\n", scene_path.c_str());

    rr_ctx* ctx = nullptr;
    rr_scene* scene = nullptr;
    if (rr_create(env_int("RR_DEVICE", 0), &ctx) != 0 || rr_scene_load(ctx, scene_path.c_str(), &scene) != 0) {
        std::fprintf(stderr, "rr-blender-shim: %s\n", rr_last_error(ctx));
        std::printf("Error: %s\n", rr_last_error(ctx));
        if (ctx) rr_destroy(ctx);
        return 1;
    }
    const double time_init = unix_now();  // script start, after the project is loaded
    rr_render_params p;
    rr_render_params_default(&p);
    p.spp = env_int("RR_SPP", 0);
    p.max_bounces = env_int("RR_MAX_BOUNCES", -1);
    p.width = env_int("RR_WIDTH", 0);
    p.height = env_int("RR_HEIGHT", 0);
    const std::string out_path = format_hash_frame_placeholders(out_fmt, frame);
    rr_frame_timing t{};
    rr_frame_stats st{};
    const int rc = rr_render_frame(ctx, scene, (int32_t)frame, &p, out_path.c_str(), fmt.c_str(), 90, &t, &st);
    if (rc != 0) {
        std::printf("Error: %s\n", rr_last_error(ctx));
        rr_scene_free(scene);
        rr_destroy(ctx);
        return 1;
    }
    const std::string ext = fmt == "PNG" ? ".png" : ".jpg";
    std::printf("Fra:%ld Mem:0M | Rendered %d x %d, %d spp, %.3f ms device\n", frame, st.width, st.height, st.spp,
                st.build_ms + st.trace_ms);
    std::printf("Saved: '%s%s'\n", out_path.c_str(), ext.c_str());
    std::printf(" Time: %s (Saving: %s)\n", blender_time(t.file_saving_finished_at - t.started_rendering_at).c_str(),
                blender_time(t.file_saving_finished_at - t.file_saving_started_at).c_str());
    std::printf("\n");
    std::printf("RESULTS={\"project_loaded_at\": %.6f, \"project_started_rendering_at\": %.6f, "
                "\"project_finished_rendering_at\": %.6f}\n",
                time_init, t.started_rendering_at, t.file_saving_finished_at);
    std::printf("\nBlender quit\n");
    std::fflush(stdout);
    rr_scene_free(scene);
    rr_destroy(ctx);
    return 0;
}
