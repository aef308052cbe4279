"""Per-kernel register / scratch usage of the gfx950 code in a built .so.

    python tools/kernel_resources.py [raft-stereo_amd/_build/libraftcorr.so] [--filter NAME]

Reads the HIP fat binary (clang offload bundle in the ``.hip_fatbin``
section), the amdgcn code object inside it, and the code object's AMDGPU
metadata note (msgpack): for every kernel its VGPR / SGPR counts, spills and
private (scratch) segment size.  tests/test_kernel_resources.py uses it to
keep every product kernel free of scratch memory (a dynamically indexed
register array silently becomes per-lane scratch traffic).
"""
import argparse
import struct
import sys

import msgpack

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    """name -> (offset, size) of an ELF64 little-endian image."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stro = hdrs[shstrndx][4]
    out = {}
    for h in hdrs:
        name = elf[stro + h[0]: elf.index(b"\0", stro + h[0])].decode()
        out.setdefault(name, []).append((h[1], h[4], h[5]))   # type, offset, size
    return out


def code_objects(path, arch="gfx950"):
    data = open(path, "rb").read()
    secs = _sections(data)
    for _, off, size in secs.get(".hip_fatbin", []):
        blob = data[off:off + size]
        pos = 0
        while True:
            pos = blob.find(BUNDLE_MAGIC, pos)
            if pos < 0:
                break
            n, = struct.unpack_from("<Q", blob, pos + 24)
            p = pos + 32
            for _ in range(n):
                eoff, esize, tlen = struct.unpack_from("<QQQ", blob, p)
                triple = blob[p + 24: p + 24 + tlen].decode()
                p += 24 + tlen
                if arch in triple and esize:
                    yield blob[pos + eoff: pos + eoff + esize]
            pos += len(BUNDLE_MAGIC)


def kernels(path):
    """[{name, vgpr, sgpr, agpr, vgpr_spill, sgpr_spill, scratch}] of every kernel."""
    res = []
    for co in code_objects(path):
        for stype, off, size in sum(_sections(co).values(), []):
            if stype != 7:                                   # SHT_NOTE
                continue
            p = off
            while p < off + size:
                namesz, descsz, ntype = struct.unpack_from("<III", co, p)
                name = co[p + 12: p + 12 + namesz]
                d0 = p + 12 + ((namesz + 3) & ~3)
                if ntype == 32 and name.startswith(b"AMDGPU"):
                    meta = msgpack.unpackb(co[d0: d0 + descsz], raw=False)
                    for k in meta.get("amdhsa.kernels", []):
                        res.append({"name": k.get(".name"), "vgpr": k.get(".vgpr_count"),
                                    "agpr": k.get(".agpr_count"), "sgpr": k.get(".sgpr_count"),
                                    "vgpr_spill": k.get(".vgpr_spill_count", 0),
                                    "sgpr_spill": k.get(".sgpr_spill_count", 0),
                                    "scratch": k.get(".private_segment_fixed_size", 0),
                                    "lds": k.get(".group_segment_fixed_size", 0)})
                p = d0 + ((descsz + 3) & ~3)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default="raft-stereo_amd/_build/libraftcorr.so")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    ks = [k for k in kernels(a.lib) if a.filter in k["name"]]
    for k in sorted(ks, key=lambda k: k["name"]):
        print(f"{k['name'][:90]:90s} vgpr={k['vgpr']} agpr={k['agpr']} sgpr={k['sgpr']} "
              f"scratch={k['scratch']} spill={k['vgpr_spill']}/{k['sgpr_spill']} lds={k['lds']}")
    print(f"{len(ks)} kernels", file=sys.stderr)


if __name__ == "__main__":
    main()
