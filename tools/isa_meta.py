"""Register counts, scratch and static instruction mix of the render kernels in one or more
builds of the render library (product build or tools/build_variant.py experiments).
Usage: python tools/isa_meta.py [lib.so ...]   (default: the product build)"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = ("rtx_render_kernelILb0ELi0E", "rtx_render_kernelILb0ELi1E", "rtx_render_kernelILb0ELi2E",
           "rtx_render_kernelILb0ELi3E")


def code_object(lib: str, tmp: Path) -> Path:
    fb, co = tmp / "fatbin.bin", tmp / "gfx950.co"
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fb)], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"], check=True)
    return co


def main() -> None:
    libs = sys.argv[1:] or [str(ROOT / "gp1_raytracer_2223_amd" / "lib" / "librtx_hip.so")]
    for lib in libs:
        with tempfile.TemporaryDirectory() as d:
            co = code_object(lib, Path(d))
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(co)], check=True,
                                 capture_output=True, text=True).stdout
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True,
                                   capture_output=True, text=True).stdout
        names = sorted(set(re.findall(r"<(_Z\d+rtx_(?:render|split)_kernel[^>]*)>:", dis)))
        for name in names:
            start = dis.index(f"<{name}>:")
            body = dis[start:dis.index("s_endpgm", start)]
            ops = collections.Counter()
            for line in body.splitlines():
                t = line.strip().split()
                if t and (t[0].startswith("v_") or t[0].startswith("s_")):
                    ops["valu" if t[0].startswith("v_") else "salu"] += 1
            meta = {}
            for block in notes.split("  - .")[1:]:
                if re.search(rf"\.name:\s+{re.escape(name)}\s", block):
                    for key in ("vgpr_count", "sgpr_count", "private_segment_fixed_size"):
                        mm = re.search(rf"\.{key}:\s+(\d+)", block)
                        if mm:
                            meta[key] = int(mm.group(1))
            k = re.sub(r"^_Z\d+rtx_((?:render|split)_kernel)I(.*)EvN4rtxd.*$", r"\1<\2>", name)
            print(f"{Path(lib).name:28s} {k:22s} vgpr {meta.get('vgpr_count')} sgpr {meta.get('sgpr_count')} "
                  f"scratch {meta.get('private_segment_fixed_size')}  static v_* {ops['valu']} s_* {ops['salu']}")


if __name__ == "__main__":
    main()
