"""Build an experiment variant of the render library into lib/exp/librtx_hip_<name>.so
(same flags as build.py's product build, plus extra -D / compiler flags), optionally from
another source file.  Usage: python tools/build_variant.py <name> [--src file.hip] [flags...]
Select it at run time with RTX_HIP_LIB (kernel experiments only; tools/ab.sh)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "gp1_raytracer_2223_amd"


def main() -> int:
    name, args = sys.argv[1], sys.argv[2:]
    src = PKG / "csrc" / "rtx_hip.hip"
    if args[:1] == ["--src"]:
        src, args = Path(args[1]).resolve(), args[2:]
    out = PKG / "lib" / "exp" / f"librtx_hip_{name}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    flags = {"-DRTX_MIN_WAVES_PER_EU=6"}
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O3", "-ffp-contract=off",
           "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize",
           "-mllvm", "-structurizecfg-skip-uniform-regions=true",
           *([f for f in flags if not any(a.startswith(f.split("=")[0]) for a in args)]), "-fPIC", "-shared",
           "-Wall", f"-I{ROOT / 'include'}", f"-I{PKG / 'csrc'}", *args, str(src),
           str(PKG / "csrc" / "rtx_policy.hip"), str(PKG / "csrc" / "rtx_anim.hip"),
           str(PKG / "csrc" / "rtx_anim_host.hip"), str(PKG / "csrc" / "rtx_group.cpp"), "-o", str(out)]
    print(" ".join(cmd[-4:]), flush=True)
    return subprocess.call(cmd)


if __name__ == "__main__":
    sys.exit(main())
