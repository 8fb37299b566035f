"""GPU parity of the Cycles-default behaviours restated this round: the
Filmic view transform through OCIO LUT files (csrc/view.hip vs the oracle's
orc_filmic, on synthetic LUTs in Blender's two formats: Blender's own LUTs are
not in the image, so parity with Blender's Filmic output stays unpinned), and
the per-lobe bounce caps (both the LDS-resident k_tiles path and the split
path), against the oracle bit for bit and against the analytic answer."""
import numpy as np
import pytest

from conftest import scene_path
from oracle import host_oracle as HO
from oracle import oracle as O

pytestmark = pytest.mark.gpu

S01 = scene_path("01_simple-animation.rrscene")


@pytest.fixture()
def luts(tmp_path):
    HO.write_synthetic_filmic_luts(str(tmp_path), n3=33, n1=4096)
    return str(tmp_path), HO.load_filmic_luts(str(tmp_path))


def test_filmic_without_luts_is_flagged(ctx, rr):
    ctx.set_ocio_config(None)
    s = ctx.load_scene(S01)
    try:
        p = rr.default_params(width=64, height=36, spp=4)
        film, rgba, st = ctx.render_to_memory(s, 30, p)
        assert st.view_transform == rr.native.RR_VIEW_STANDARD and st.view_transform_substituted == 1
        t, st2 = ctx.render_frame(s, 30, p, None, None, 90)
        assert st2.view_transform_substituted == 1 and "Filmic" in ctx.last_warning()
        # the substitute is exactly the Standard render
        _, rgba_std, st3 = ctx.render_to_memory(s, 30, rr.default_params(width=64, height=36, spp=4,
                                                                          view_transform=0))
        assert np.array_equal(rgba, rgba_std) and st3.view_transform_substituted == 0
    finally:
        s.close()


def test_filmic_lut_path_bit_exact(ctx, rr, luts):
    d, host = luts
    ctx.set_ocio_config(d)
    O.set_filmic(host)
    s = ctx.load_scene(S01)
    try:
        for frame, (w, h, spp) in ((30, (96, 54, 8)), (1, (160, 90, 40))):
            p = rr.default_params(width=w, height=h, spp=spp)
            film, rgba, st = ctx.render_to_memory(s, frame, p)
            assert st.view_transform == rr.native.RR_VIEW_FILMIC and st.view_transform_substituted == 0
            state = ctx.frame_state(s, frame, p)
            assert int(state.render_ints[5]) == 2
            of, orgba = O.render_state(state)
            assert np.array_equal(film, of)
            nbad = int(np.count_nonzero(rgba != orgba))
            assert nbad == 0, f"{nbad} 8-bit mismatches"
            # the chain itself, on the film the oracle agrees with
            assert np.array_equal(orgba[..., :3].reshape(-1, 3), O.filmic(of[..., :3].reshape(-1, 3)))
        # a JPEG frame takes the same 8-bit image through the device encoder
        t, st = ctx.render_frame(s, 30, rr.default_params(width=96, height=54, spp=8), None, None, 90)
        assert st.view_transform == 2
    finally:
        s.close()
        ctx.set_ocio_config(None)
        O.set_filmic(None)


def test_ocio_config_errors(ctx, rr, tmp_path):
    with pytest.raises(rr.RRError) as e:
        ctx.set_ocio_config(str(tmp_path / "nowhere"))
    assert e.value.code == -2
    (tmp_path / "luts").mkdir()
    (tmp_path / "luts" / HO.FILMIC_LUT_FILES[0]).write_text("SPILUT 1.0\n3 3\n2 2 2\n0 0 0 0 0 0\n")
    (tmp_path / "luts" / HO.FILMIC_LUT_FILES[1]).write_text("Version 1\nFrom 0 1\nLength 2\nComponents 1\n{\n0\n1\n}\n")
    with pytest.raises(rr.RRError) as e:
        ctx.set_ocio_config(str(tmp_path))  # 1 of 8 cube entries
    assert e.value.code == -22
    s = ctx.load_scene(S01)
    try:  # a failed configuration leaves no LUTs behind
        _, _, st = ctx.render_to_memory(s, 1, rr.default_params(width=16, height=16, spp=1))
        assert st.view_transform_substituted == 1
    finally:
        s.close()


@pytest.mark.parametrize("name,caps,hits", [
    ("test_enclosure_diffuse.rrscene", (12, 4, 4), 5),    # k_tiles (80 triangles, LDS-resident)
    ("test_enclosure_diffuse.rrscene", (12, 2, 4), 3),
    ("test_enclosure_diffuse.rrscene", (3, 4, 4), 4),
    ("test_enclosure_glossy.rrscene", (12, 4, 4), 5),     # split path (1,280 triangles)
    ("test_enclosure_glossy.rrscene", (12, 4, 2), 3),
])
def test_bounce_caps_bit_exact_and_known_answer(ctx, rr, name, caps, hits):
    s = ctx.load_scene(scene_path(name))
    try:
        mb, md, mg = caps
        p = rr.default_params(max_bounces=mb, max_diffuse_bounces=md, max_glossy_bounces=mg)
        film, rgba, st = ctx.render_to_memory(s, 1, p)
        state = ctx.frame_state(s, 1, p)
        assert list(state.render_ints[8:10]) == [md, mg]
        of, orgba = O.render_state(state)
        assert np.array_equal(film, of), f"{np.count_nonzero(film != of)} film mismatches"
        assert np.array_equal(rgba, orgba)
        mean = float(film[..., :3].mean())
        assert abs(mean - 0.25 * hits) < 2e-3 * hits, mean
        # hits = camera ray + (hits - 1) continuations per path
        assert st.extension_rays == pytest.approx(st.camera_rays * (hits - 1), rel=2e-3)
    finally:
        s.close()


def test_unsupported_view_settings_render_standard_and_say_so(ctx, rr, tmp_path):
    """A Blender 3.6 view the renderer does not implement ('Filmic Log') and a
    look ('Medium Contrast') do not fail the job: the frame renders with
    Standard, bit-identical to the Standard scene, is flagged
    (view_transform_substituted) and the warning names both."""
    import json
    with open(scene_path("04_very-simple-standin.rrscene")) as f:
        sc = json.load(f)
    sc["render"]["view_transform"] = "Filmic Log"
    sc["render"]["look"] = "Medium Contrast"
    path = str(tmp_path / "filmic_log.rrscene")
    with open(path, "w") as f:
        json.dump(sc, f)
    p = rr.default_params(width=96, height=54, spp=4)
    s_log, s_std = ctx.load_scene(path), ctx.load_scene(scene_path("04_very-simple-standin.rrscene"))
    try:
        film, rgba, st = ctx.render_to_memory(s_log, 12, p)
        w = ctx.last_warning()
        assert st.view_transform_substituted == 1 and st.view_transform == 0
        assert "Filmic Log" in w and "Medium Contrast" in w, w
        film2, rgba2, st2 = ctx.render_to_memory(s_std, 12, p)
        assert st2.view_transform_substituted == 0 and ctx.last_warning() == ""
        assert np.array_equal(film, film2) and np.array_equal(rgba, rgba2)
        # the oracle's Standard render of the same frame
        _, orgba = O.render_state(ctx.frame_state(s_log, 12, p))
        assert np.array_equal(rgba, orgba)
    finally:
        s_log.close()
        s_std.close()


def test_context_warning_survives_frames(rr, tmp_path, monkeypatch):
    """A broken RR_OCIO_DIR is reported by rr_last_warning for the context's
    lifetime, next to each frame's own warning, not only until the first frame."""
    monkeypatch.setenv("RR_OCIO_DIR", str(tmp_path / "no_such_dir"))
    c = rr.RenderContext(0)
    try:
        assert "RR_OCIO_DIR" in c.last_warning()
        s = c.load_scene(scene_path("01_simple-animation.rrscene"))
        _, _, st = c.render_to_memory(s, 5, rr.default_params(width=64, height=36, spp=2))
        w = c.last_warning()
        assert st.view_transform_substituted == 1
        assert "RR_OCIO_DIR" in w and "Filmic rendered as Standard" in w, w
        c.set_ocio_config(None)  # superseded: only the frame's warning is left
        _, _, _ = c.render_to_memory(s, 5, rr.default_params(width=64, height=36, spp=2))
        assert "RR_OCIO_DIR:" not in c.last_warning() and "Filmic rendered as Standard" in c.last_warning()
    finally:
        c.close()
    # the context is gone: the scene handle is host-only again and frees cleanly
    assert s.counts()["triangles"] == 12
    s.close()
