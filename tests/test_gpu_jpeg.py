"""The device JPEG path (jpeg.hip: forward DCT + quantisation + Huffman coding,
restart interval per MCU row, byte stuffing, RSTn/EOI markers) produces the
same file bytes as the host encoder (image_io.cpp encode_jpeg) on the same
RGBA8 image. Cases: ragged and tiny sizes (edge replication, partial MCUs),
uniform noise (long codes, ZRL-free blocks, many 0xFF bytes to stuff), flat
images (EOB-only blocks), gradients, qualities 50 / 90 / 100, and a full
1080p noise frame (the largest rows the coder sees at C2's resolution)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host(rr, tmp_path, rgba, q):
    rr.encode_image(rgba, str(tmp_path / "host"), "JPEG", q)
    return (tmp_path / "host.jpg").read_bytes()


def _img(kind, w, h, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        a = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    elif kind == "flat":
        a = np.full((h, w, 4), 77, np.uint8)
    elif kind == "gradient":
        y, x = np.mgrid[0:h, 0:w]
        a = np.stack([(x * 255 // max(w - 1, 1)), (y * 255 // max(h - 1, 1)), ((x + y) % 256), np.full_like(x, 255)],
                     -1).astype(np.uint8)
    elif kind == "sparse":  # mostly flat with isolated spikes: long zero runs (ZRL) in the AC scan
        a = np.full((h, w, 4), 128, np.uint8)
        m = rng.random((h, w)) < 0.01
        a[m, :3] = 255
    a[..., 3] = 255
    return a


@pytest.mark.parametrize("kind,w,h,q", [
    ("noise", 1, 1, 90), ("noise", 8, 8, 90), ("noise", 17, 9, 90), ("gradient", 333, 257, 90),
    ("flat", 64, 48, 90), ("sparse", 320, 200, 90), ("noise", 256, 64, 100), ("gradient", 640, 360, 50),
    ("sparse", 1920, 1080, 90), ("noise", 1920, 1080, 90)])
def test_device_jpeg_equals_host(ctx, rr, tmp_path, kind, w, h, q):
    rgba = _img(kind, w, h, seed=w * 7 + h)
    dev = ctx.jpeg_device(rgba, q)
    host = _host(rr, tmp_path, rgba, q)
    assert len(dev) == len(host)
    assert dev == host


def test_rendered_frame_file_equals_host_encoding(ctx, rr, tmp_path):
    """rr_render_frame's JPEG (device entropy coding) == the host encoder on the
    frame's RGBA, for a small frame of the 04vs stand-in."""
    from conftest import scene_path
    s = ctx.load_scene(scene_path("04_very-simple-standin.rrscene"))
    try:
        p = rr.default_params(spp=4, width=250, height=141)
        ctx.render_frame(s, 9, p, str(tmp_path / "f9"), "JPEG", 90)
        _, rgba, _ = ctx.render_to_memory(s, 9, p)
        assert (tmp_path / "f9.jpg").read_bytes() == _host(rr, tmp_path, rgba, 90)
    finally:
        s.close()
