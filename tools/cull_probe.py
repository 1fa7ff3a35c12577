"""Diagnostic: reference BVH work vs work left after a tight-box cull (tools/cull_probe.c).

python tools/cull_probe.py [scene] [step] [delta ...]
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402


def lib() -> C.CDLL:
    out = ROOT / "tools" / "bin" / "libcull_probe.so"
    src = ROOT / "tools" / "cull_probe.c"
    if not out.exists() or out.stat().st_mtime < src.stat().st_mtime:
        out.parent.mkdir(exist_ok=True)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", f"-I{ROOT / 'include'}", str(src),
                        "-o", str(out), "-lm"], check=True)
    return C.CDLL(str(out))


def main() -> None:
    name = sys.argv[1] if len(sys.argv) > 1 else "Synthetic100k"
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    deltas = [float(x) for x in sys.argv[3:]] or [-1.0, 1e-3, 1e-2, 0.1]
    L = lib()
    import os
    if os.environ.get("ORDERED"):
        L.cull_probe_ordered(int(os.environ["ORDERED"]), C.c_double(float(os.environ.get("TSLACK", "1e-3"))))
    if os.environ.get("CAP"):   # UNSOUND: clip triangle margins (prices the margin distribution's tail)
        L.cull_probe_cap(C.c_double(float(os.environ["CAP"])))
    if os.environ.get("CONE"):
        L.cull_probe_cone(int(os.environ["CONE"]))
    if os.environ.get("FIXED_GRID"):
        L.cull_probe_fixed_grid(int(os.environ["FIXED_GRID"]))
    hs = HostScene(name)
    s, cam = hs.view()
    for d in deltas:
        out = (C.c_uint64 * 10)()
        rc = L.cull_probe(C.byref(s), C.byref(cam), 1920, 1080, step, C.c_double(d), out)
        assert rc == 0
        o = list(out)
        print(f"{name} step {step} margin {'bound' if d < 0 else d}: slabs {o[0]} -> {o[2]} ({o[2] / o[0]:.3f}), tris {o[1]} -> {o[3]}"
              f" ({o[3] / max(o[1], 1):.3f}), shadow slabs {o[6]} -> {o[7]}, shadow tris {o[8]} -> {o[9]},"
              f" mismatches {o[4]} / {o[5]} rays",
              flush=True)


if __name__ == "__main__":
    main()
