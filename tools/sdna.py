"""Minimal reader for Blender .blend files (SDNA-described binary).

Used once per project by tools/blend_export.py to export a .blend into the
renderer's .rrscene format. The reference reads the .blend inside
Blender on every frame (/root/reference/worker/src/rendering/runner/mod.rs:142-146);
the MI355X renderer reads an exported scene once.

File layout (Blender's published format, pinned by the reference to Blender
3.6.0 via /root/reference/pull-blender-image.sh:3-4; the one project file
present, blender-projects/01_simple-animation/01_simple-animation.blend, was
written by 3.5 "v305"):
  header  "BLENDER" + ptr-size ('_' 4 / '-' 8) + endian ('v' little / 'V' big) + version
  blocks  code[4] len:i32 old_ptr:ptr sdna_index:i32 count:i32 + payload
  DNA1    "SDNA" NAME/TYPE/TLEN/STRC tables describing every struct
"""
from __future__ import annotations

import re
import struct
from dataclasses import dataclass, field


@dataclass
class Field:
    type: str
    name: str  # bare name, e.g. "loc"
    full: str  # as in SDNA, e.g. "loc[3]" / "*next"
    is_ptr: bool
    dims: tuple
    offset: int
    size: int


@dataclass
class Struct:
    name: str
    size: int
    fields: dict = field(default_factory=dict)


@dataclass
class Block:
    code: bytes
    size: int
    old_ptr: int
    sdna: int
    count: int
    offset: int  # file offset of payload


class BlendFile:
    def __init__(self, path: str):
        with open(path, "rb") as f:
            self.data = f.read()
        d = self.data
        if d[:7] != b"BLENDER":
            raise ValueError("not a .blend file (compressed .blend files are not supported)")
        self.ptr = 8 if d[7:8] == b"-" else 4
        self.endian = "<" if d[8:9] == b"v" else ">"
        self.version = d[9:12].decode()
        self.blocks: list[Block] = []
        self.by_ptr: dict[int, Block] = {}
        off = 12
        pfmt = "Q" if self.ptr == 8 else "I"
        hdr = struct.Struct(self.endian + "4si" + pfmt + "ii")
        while off < len(d):
            code, size, old, sdna, count = hdr.unpack_from(d, off)
            off += hdr.size
            b = Block(code, size, old, sdna, count, off)
            off += size
            if code == b"ENDB":
                break
            self.blocks.append(b)
            if old:
                self.by_ptr[old] = b
        dna = next(b for b in self.blocks if b.code == b"DNA1")
        self._parse_sdna(dna)

    # -- SDNA ------------------------------------------------------------
    def _parse_sdna(self, blk: Block):
        d, e = self.data, self.endian
        p = blk.offset
        assert d[p:p + 4] == b"SDNA"
        p += 4

        def tag(name):
            nonlocal p
            assert d[p:p + 4] == name, (d[p:p + 4], name)
            p += 4

        def strings(n):
            nonlocal p
            out = []
            for _ in range(n):
                q = d.index(b"\0", p)
                out.append(d[p:q].decode("latin-1"))
                p = q + 1
            p = (p + 3) & ~3
            return out

        tag(b"NAME")
        (n,) = struct.unpack_from(e + "i", d, p); p += 4
        names = strings(n)
        tag(b"TYPE")
        (n,) = struct.unpack_from(e + "i", d, p); p += 4
        types = strings(n)
        tag(b"TLEN")
        tlen = list(struct.unpack_from(e + f"{n}h", d, p)); p += 2 * n
        p = (p + 3) & ~3
        tag(b"STRC")
        (ns,) = struct.unpack_from(e + "i", d, p); p += 4
        self.types, self.tlen = types, tlen
        self.structs: list[Struct] = []
        self.struct_by_name: dict[str, Struct] = {}
        for _ in range(ns):
            t, nf = struct.unpack_from(e + "hh", d, p); p += 4
            s = Struct(types[t], tlen[t])
            o = 0
            for _ in range(nf):
                ft, fn = struct.unpack_from(e + "hh", d, p); p += 4
                full = names[fn]
                is_ptr = full.startswith("*") or full.startswith("(*")
                dims = tuple(int(x) for x in re.findall(r"\[(\d+)\]", full))
                bare = re.sub(r"[\*\(\)]|\[\d+\]", "", full)
                count = 1
                for x in dims:
                    count *= x
                size = (self.ptr if is_ptr else tlen[ft]) * count
                s.fields[bare] = Field(types[ft], bare, full, is_ptr, dims, o, size)
                o += size
            self.structs.append(s)
            self.struct_by_name[s.name] = s

    # -- access ----------------------------------------------------------
    def struct_of(self, blk: Block) -> Struct:
        return self.structs[blk.sdna]

    def blocks_with_code(self, code: bytes):
        return [b for b in self.blocks if b.code.rstrip(b"\0") == code]

    def get(self, blk: Block, path: str, base: int = 0, sname: str | None = None):
        """Read a (possibly nested, dotted) field of the struct stored at blk.offset+base."""
        s = self.struct_by_name[sname] if sname else self.struct_of(blk)
        off = blk.offset + base
        parts = path.split(".")
        for i, part in enumerate(parts):
            f = s.fields[part]
            off += f.offset
            if i < len(parts) - 1:
                s = self.struct_by_name[f.type]
        return self._read(f, off)

    def _read(self, f: Field, off: int):
        d, e = self.data, self.endian
        if f.is_ptr:
            n = f.size // self.ptr
            fmt = ("Q" if self.ptr == 8 else "I") * n
            v = struct.unpack_from(e + fmt, d, off)
            return v[0] if n == 1 else list(v)
        prim = {"float": "f", "double": "d", "int": "i", "short": "h", "char": "b",
                "uchar": "B", "int8_t": "b", "uint8_t": "B", "int16_t": "h",
                "uint16_t": "H", "int32_t": "i", "uint32_t": "I", "int64_t": "q",
                "uint64_t": "Q", "ushort": "H", "uint": "I"}.get(f.type)
        if prim is None:
            return off  # nested struct: return absolute offset
        if f.type == "char" and f.dims:
            raw = d[off:off + f.size]
            return raw.split(b"\0", 1)[0].decode("utf-8", "replace")
        n = f.size // struct.calcsize(prim)
        v = struct.unpack_from(e + prim * n, d, off)
        return v[0] if n == 1 else list(v)

    def deref(self, ptr: int) -> Block | None:
        return self.by_ptr.get(ptr) if ptr else None

    def read_struct_at(self, abs_off: int, sname: str, fieldname: str):
        s = self.struct_by_name[sname]
        f = s.fields[fieldname]
        return self._read(f, abs_off + f.offset)

    def listbase(self, first_ptr: int, sname: str):
        """Walk a ListBase of structs whose first member is *next."""
        out = []
        ptr = first_ptr
        seen = set()
        while ptr and ptr not in seen:
            seen.add(ptr)
            b = self.by_ptr.get(ptr)
            if b is None:
                break
            out.append(b)
            ptr = self.read_struct_at(b.offset, sname, "next")
        return out
