"""Per-kernel register / LDS / scratch use of the gfx950 code objects inside an object file or
shared library (the .hip_fatbin offload bundle), from the AMDGPU metadata note.

    python tools/kernel_regs.py neural_raytracing_amd/build_obj/nrt_shade_ring.o [name-regex]
"""
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    data = open(path, "rb").read()
    pos = 0
    while True:
        pos = data.find(MAGIC, pos)
        if pos < 0:
            return
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if "gfx950" in triple:
                yield data[pos + off:pos + off + size]
        pos += 1


def kernels(blob):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(blob)
        f.flush()
        out = subprocess.run([LLVM + "llvm-readelf", "--notes", f.name], capture_output=True,
                             text=True).stdout
    cur = {}
    for line in out.splitlines():
        s = line.strip()
        m = re.match(r"-?\s*\.(\w+):\s*(.*)", s)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count" and cur:
            yield cur
            cur = {}
        cur[k] = v
    if cur:
        yield cur


def main():
    path = sys.argv[1]
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    for blob in code_objects(path):
        for k in kernels(blob):
            name = k.get("name", "?")
            if rx and not rx.search(name):
                continue
            print(f"vgpr {k.get('vgpr_count', '?'):>4} agpr {k.get('agpr_count', '?'):>4} "
                  f"sgpr {k.get('sgpr_count', '?'):>3} lds {k.get('group_segment_fixed_size', '?'):>6} "
                  f"scratch {k.get('private_segment_fixed_size', '?'):>5}  {name[:150]}")


if __name__ == "__main__":
    main()
