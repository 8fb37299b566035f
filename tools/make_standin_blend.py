#!/usr/bin/env python3
"""Writes the 04_very-simple stand-in project (.blend) from the 01 project.

The reference's 04_very-simple.blend is not in the tree (its job TOMLs name
%BASE%/blender-projects/04_very-simple/04_very-simple.blend, e.g.
/root/reference/blender-projects/04_very-simple/04_very-simple_demo_10f-1w.toml:4,
and the file is listed in .MISSING_LARGE_BLOBS). The stand-in the renderer
measures (scenes/04_very-simple-standin.rrscene, SURVEY.md §8d "04vs-standin")
is the 01_simple-animation content at 1920x1080, 128 samples, view transform
Standard. This tool makes the matching .blend, so that the 04 jobs under
jobs/ name a project file Blender itself can open (the reference worker passes
project_file_path to `blender` as the project, worker/src/rendering/runner/
mod.rs:140-146): a byte copy of 01_simple-animation.blend with one field
changed, the scene's ColorManagedViewSettings.view_transform "Filmic" ->
"Standard" (char[64], located through the file's own SDNA by tools/sdna.py).
Resolution (1920x1080 at 100 %) and frame range are already the 01 file's.

Usage: python tools/make_standin_blend.py <01_simple-animation.blend> <out.blend>
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sdna import BlendFile  # noqa: E402


def set_view_transform(data: bytearray, bf: BlendFile, name: str) -> str:
    """Overwrite every scene's view transform in `data` (the bytes bf was read
    from); returns the previous name of the first scene."""
    old = None
    for sc in bf.blocks_with_code(b"SC"):
        vs = bf.get(sc, "view_settings")  # absolute offset of the nested struct
        f = bf.struct_by_name["ColorManagedViewSettings"].fields["view_transform"]
        raw = name.encode()
        if len(raw) >= f.size:
            raise ValueError(f"view transform name longer than {f.size - 1} bytes")
        if old is None:
            old = bf.read_struct_at(vs, "ColorManagedViewSettings", "view_transform")
        data[vs + f.offset:vs + f.offset + f.size] = raw + b"\0" * (f.size - len(raw))
    if old is None:
        raise ValueError("no scene block in the file")
    return old


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("src")
    ap.add_argument("out")
    ap.add_argument("--view-transform", default="Standard")
    a = ap.parse_args(argv)
    bf = BlendFile(a.src)
    data = bytearray(bf.data)
    old = set_view_transform(data, bf, a.view_transform)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "wb") as f:
        f.write(bytes(data))
    check = BlendFile(a.out)
    sc = check.blocks_with_code(b"SC")[0]
    now = check.read_struct_at(check.get(sc, "view_settings"), "ColorManagedViewSettings", "view_transform")
    assert now == a.view_transform, now
    print(f"wrote {a.out}: view transform {old!r} -> {now!r}, {len(data)} bytes")


if __name__ == "__main__":
    main()
