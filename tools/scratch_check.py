"""Per-kernel scratch (private segment) and VGPR use of the gfx950 code objects inside the built
library: a kernel with a non-zero private segment keeps registers (usually an MFMA accumulator array
indexed with a runtime value) in scratch memory -- often 10x slower, and not reported as a "spill".

The library's .hip_fatbin section holds one clang offload bundle per translation unit; each bundle's
gfx950 entry is an ELF code object whose note metadata (llvm-readelf --notes) lists every kernel's
.private_segment_fixed_size and .vgpr_count.

usage: python tools/scratch_check.py [lib.so]   (exit 1 if any kernel uses scratch)"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(fat: bytes, arch: str = "gfx950"):
    """(triple, ELF bytes) of every bundle entry for `arch`."""
    out = []
    for m in re.finditer(re.escape(MAGIC), fat):
        base = m.start()
        pos = base + len(MAGIC)
        (n,) = struct.unpack_from("<Q", fat, pos)
        pos += 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, pos)
            pos += 24
            triple = fat[pos:pos + tlen].decode()
            pos += tlen
            if arch in triple and size:
                out.append((triple, fat[base + off:base + off + size]))
    return out


def kernel_resources(lib: str):
    """{kernel symbol: (private segment bytes, vgprs)} over the library's gfx950 code objects."""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(td, "x.so")],
                       check=True, capture_output=True)
        for i, (_, elf) in enumerate(code_objects(open(fat, "rb").read())):
            path = os.path.join(td, f"co{i}.o")
            open(path, "wb").write(elf)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", path], check=True, capture_output=True,
                                   text=True).stdout
            # one YAML-ish block per kernel: collect the keys of each "- .args" ... block by its .symbol
            for blk in re.split(r"\n\s*- \.agpr_count:", notes)[1:]:
                sym = re.search(r"\.symbol:\s+(\S+)", blk)
                priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
                vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
                if sym and priv:
                    res[sym.group(1)] = (int(priv.group(1)), int(vg.group(1)) if vg else -1)
    return res


def main():
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "distributed-training-comparison_amd", "_lib",
                                                             "libdtc_amd.so")
    res = kernel_resources(lib)
    bad = {k: v for k, v in res.items() if v[0] > 0}
    print(f"{len(res)} kernels, {len(bad)} with scratch")
    for k, (p, v) in sorted(bad.items()):
        print(f"  {p:6d} B/lane  {v:4d} VGPRs  {k}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
