"""Kernel resource metadata of the built library, read without a GPU.

libairscmp.so carries one clang offload bundle per HIP translation unit in its
.hip_fatbin section; each holds the gfx950 code object (an ELF), whose
NT_AMDGPU_METADATA note (msgpack) lists every kernel with its register counts
and spill counts (.sgpr_spill_count, .vgpr_spill_count, .vgpr_count,
.sgpr_count, .group_segment_fixed_size, .private_segment_fixed_size)."""
import struct

import msgpack

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NT_AMDGPU_METADATA = 32


def _code_objects(blob):
    pos = blob.find(BUNDLE_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", blob, p)
            ident = blob[p + 24:p + 24 + idlen].decode()
            p += 24 + idlen
            if "gfx950" in ident and size:
                yield blob[pos + off:pos + off + size]
        pos = blob.find(BUNDLE_MAGIC, pos + 32)


def _notes(elf):
    assert elf[:4] == b"\x7fELF" and elf[4] == 2  # ELF64
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for i in range(shnum):
        sh = shoff + i * shentsize
        stype = struct.unpack_from("<I", elf, sh + 4)[0]
        if stype != 7:  # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p, end = off, off + size
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            name_end = p + 12 + ((namesz + 3) & ~3)
            yield ntype, elf[name_end:name_end + descsz]
            p = name_end + ((descsz + 3) & ~3)


def kernels(lib_path):
    """{kernel symbol: metadata dict} for every gfx950 kernel in the library."""
    with open(lib_path, "rb") as f:
        blob = f.read()
    out = {}
    for co in _code_objects(blob):
        for ntype, desc in _notes(co):
            if ntype == NT_AMDGPU_METADATA:
                meta = msgpack.unpackb(desc, raw=False, strict_map_key=False)
                for k in meta.get("amdhsa.kernels", []):
                    out[k[".name"]] = k
    return out
