"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/rr.h declares, reports errors errno-style, and its host image
encoders produce valid files."""
import ctypes
import os
import re

import numpy as np
import pytest
from PIL import Image

from conftest import ROOT, scene_path


def header_functions():
    src = open(os.path.join(ROOT, "include", "rr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(rr):
    L = rr.lib()
    names = header_functions()
    assert len(names) >= 16
    for n in names:
        assert hasattr(L, n), f"librr.so does not export {n}"
    assert sorted(rr.EXPORTS) == names


def test_abi_version(rr):
    assert rr.lib().rr_abi_version() == 8 == rr.native.RR_ABI_VERSION


def test_struct_layouts_match_header(rr):
    """The ctypes mirrors have the header's field order (a field added to rr.h
    and not to native.py, or the reverse, shifts every later field)."""
    src = open(os.path.join(ROOT, "include", "rr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    for cname, py in (("rr_render_params", rr.native.RenderParams), ("rr_frame_stats", rr.native.FrameStats),
                      ("rr_frame_timing", rr.native.FrameTiming)):
        body = re.search(r"typedef struct " + cname + r" \{(.*?)\} " + cname, src, flags=re.S).group(1)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names = decl.split(None, 1)[1]
            for nm in names.split(","):
                fields.append(re.sub(r"\[.*\]", "", nm).strip())
        assert [f for f, _ in py._fields_] == fields, cname


def test_default_params_lobe_caps(rr):
    p = rr.default_params()
    assert p.max_diffuse_bounces == -1 and p.max_glossy_bounces == -1


def test_default_params(rr):
    p = rr.default_params()
    assert p.spp == 0 and p.max_bounces == -1 and p.use_scene_seed == 1 and p.view_transform == -1
    q = rr.default_params(seed=5, spp=3)
    assert q.use_scene_seed == 0 and q.seed == 5 and q.spp == 3


def test_scene_errors(rr, tmp_path):
    with pytest.raises(rr.RRError) as e:
        rr.Scene(str(tmp_path / "nope.rrscene"))
    assert e.value.code == -2
    bad = tmp_path / "bad.rrscene"
    bad.write_text("{not json")
    with pytest.raises(rr.RRError) as e:
        rr.Scene(str(bad))
    assert e.value.code == -22
    bad.write_text('{"format": "rrscene", "version": 1, "objects": [{"type": "MESH", "mesh": 3}]}')
    with pytest.raises(rr.RRError) as e:
        rr.Scene(str(bad))
    assert "mesh index" in str(e.value)


def test_null_arguments(rr):
    L = rr.lib()
    assert L.rr_render_frame(None, None, 1, None, None, None, 90, None, None) == -22
    assert L.rr_create(0, None) == -22
    assert b"NULL" in L.rr_last_error(None) or b"out is" in L.rr_last_error(None)


def test_host_only_scene_queries(rr):
    s = rr.Scene(scene_path("04_very-simple-standin.rrscene"))
    assert s.counts() == {"triangles": 12, "lights": 1, "materials": 3, "objects": 3}
    assert s.resolution() == (1920, 1080)
    assert s.resolution(rr.default_params(width=64, height=36)) == (64, 36)
    fc = s.frame_constants(1)
    assert list(fc.render_ints[:4]) == [1920, 1080, 128, 12]
    assert list(fc.render_ints[8:10]) == [4, 4]  # Cycles' diffuse / glossy bounce defaults
    fc = s.frame_constants(1, rr.default_params(max_bounces=0, max_diffuse_bounces=2, max_glossy_bounces=0))
    # a cap of 0 acts as 1 (the camera hit always scatters, Cycles path_state_next)
    assert fc.render_ints[3] == 1 and list(fc.render_ints[8:10]) == [2, 1]
    s.close()
    s01 = rr.Scene(scene_path("01_simple-animation.rrscene"))
    # host-only query: the transform the scene asks for (a context may substitute it)
    assert s01.frame_constants(1).render_ints[5] == rr.native.RR_VIEW_FILMIC
    s01.close()


def _test_image(w=67, h=45):
    y, x = np.mgrid[0:h, 0:w]
    img = np.zeros((h, w, 4), np.uint8)
    img[..., 0] = (x * 255 // max(w - 1, 1)).astype(np.uint8)
    img[..., 1] = (y * 255 // max(h - 1, 1)).astype(np.uint8)
    img[..., 2] = (128 + 100 * np.sin(x / 7.0) * np.cos(y / 5.0)).astype(np.uint8)
    img[..., 3] = 255
    return img


@pytest.mark.parametrize("w,h", [(67, 45), (1, 1), (33, 17), (1920, 1080), (300, 1000)])
def test_png_encoder_is_lossless(rr, tmp_path, w, h):
    """Band-parallel deflate (one band below 32 rows, up to 16 bands): one
    valid zlib stream whose pixels decode exactly (zlib and PIL check the
    Adler-32 and the stored/final block structure)."""
    import zlib
    img = _test_image(w, h)
    n = rr.encode_image(img, str(tmp_path / "frame"), "PNG")
    path = tmp_path / "frame.png"
    assert path.is_file() and path.stat().st_size == n
    back = np.asarray(Image.open(path).convert("RGBA"))
    assert np.array_equal(back, img)
    data = path.read_bytes()
    i = data.index(b"IDAT")
    ln = int.from_bytes(data[i - 4:i], "big")
    raw = zlib.decompress(data[i + 4:i + 4 + ln])  # raises on a bad checksum or stream
    assert len(raw) == (4 * w + 1) * h


@pytest.mark.parametrize("w,h", [(67, 45), (16, 16), (1, 1), (1920, 1080)])
def test_jpeg_encoder_quality90(rr, tmp_path, w, h):
    img = _test_image(w, h)
    rr.encode_image(img, str(tmp_path / "f"), "JPEG", 90)
    path = tmp_path / "f.jpg"
    im = Image.open(path)
    assert im.format == "JPEG" and im.size == (w, h)
    back = np.asarray(im.convert("RGB")).astype(np.float64)
    mse = np.mean((back - img[..., :3]) ** 2)
    psnr = 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)
    assert psnr > 35.0, psnr


def test_unsupported_format(rr, tmp_path):
    with pytest.raises(rr.RRError) as e:
        rr.encode_image(_test_image(), str(tmp_path / "f"), "OPEN_EXR")
    assert e.value.code == -95


def test_product_has_no_cpu_fallback(rr, monkeypatch):
    """Without a HIP device rr_create fails loudly (ENODEV); it never renders on the CPU."""
    import ctypes as C
    h = C.c_void_p()
    rc = rr.lib().rr_create(0, C.byref(h))
    if rc == 0:  # running on a GPU box
        rr.lib().rr_destroy(h)
        pytest.skip("a HIP device is present")
    assert rc == -19
